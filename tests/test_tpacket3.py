"""AF_PACKET TPACKET_V3 block walk (pv_tpacket3_block_records, afpacket.cpp:72-86) on blocks laid
out as the kernel fills them (linux/if_packet.h): packets in order, each with the block's
ts_last_pkt and its snap length (the reference's RawPacket), malformed blocks refused."""
import os
import struct

import pytest

import pktvisor_amd as pa
from tests.pcapng_util import pcap_packets

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def block(pkts, ts_last=(1700000000, 123456789), size=1 << 16):
    """tpacket_block_desc (version, offset_to_priv, hdr_v1) then tpacket3_hdr + frame per packet"""
    first = 64
    body = b""
    offs = []
    for k, data in enumerate(pkts):
        mac = 48 + 18  # header + sockaddr_ll-ish gap, then the frame (tp_mac)
        ln = (mac + len(data) + 15) & ~15
        nxt = ln if k + 1 < len(pkts) else 0
        hdr = struct.pack("<IIIIIIHH", nxt, 1, 2, len(data), len(data) + 100, 1, mac, 0)
        rec = hdr + b"\0" * (mac - len(hdr)) + data
        body += rec + b"\0" * (ln - len(rec))
    # hdr_v1: block_status, num_pkts, offset_to_first_pkt, blk_len, seq_num (u64),
    # ts_first_pkt (sec, nsec), ts_last_pkt (sec, nsec)
    h1 = struct.pack("<IIIIQIIII", 1, len(pkts), first, first + len(body), 7, 1, 0, *ts_last)
    head = struct.pack("<II", 3, 0) + h1
    raw = head + b"\0" * (first - len(head)) + body
    return raw + b"\0" * max(0, size - len(raw))


def test_blocks_to_records():
    pcap = open(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), "rb").read()
    _, pk = pcap_packets(pcap)
    frames = [p[4] for p in pk]
    recs = pa.tpacket3_records([block(frames[:10]), block(frames[10:], ts_last=(1700000001, 5))])
    p, got = 0, []
    while p < len(recs):
        s, ns, cl, ol = struct.unpack_from("<IIII", recs, p)
        got.append((s, ns, cl, ol, recs[p + 16:p + 16 + cl]))
        p += 16 + cl
    assert [g[4] for g in got] == frames
    assert all(g[2] == g[3] == len(g[4]) for g in got)
    assert all((g[0], g[1]) == (1700000000, 123456789) for g in got[:10])
    assert all((g[0], g[1]) == (1700000001, 5) for g in got[10:])


def test_malformed_block():
    b = bytearray(block([b"x" * 60, b"y" * 60]))
    struct.pack_into("<I", b, 64, 0)  # first packet's tp_next_offset = 0 with a second to come
    with pytest.raises(pa.PvError):
        pa.tpacket3_records([bytes(b)])
    with pytest.raises(pa.PvError):
        pa.tpacket3_records([b"\0" * 8])
