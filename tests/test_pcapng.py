"""pcapng input (pv_pcapng_records): a reference pcap fixture written as pcapng in several block
and option shapes must come back as the same records (host conversion, no GPU)."""
import os
import struct

import pytest

import pktvisor_amd as pa
from tests.pcapng_util import pcap_packets, to_pcapng

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def records(recs):
    p, out = 0, []
    while p + 16 <= len(recs):
        s, ns, cl, ol = struct.unpack_from("<IIII", recs, p)
        out.append((s, ns, cl, ol, recs[p + 16:p + 16 + cl]))
        p += 16 + cl
    return out


@pytest.mark.parametrize("kw", [{}, {"tsresol": 9}, {"tsresol": 6, "be": True}, {"sections": 3},
                                {"tsresol": 0x80 | 30}, {"options": False}])
def test_pcapng_records_equal_pcap(kw):
    pcap = open(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), "rb").read()
    lt, pk = pcap_packets(pcap)
    lt2, recs = pa.pcapng_records(to_pcapng(pcap, **kw))
    assert lt2 == lt
    got = records(recs)
    assert len(got) == len(pk)
    for a, b in zip(got, pk):
        if kw.get("tsresol", 0) & 0x80:
            assert a[0] == b[0] and abs(a[1] - b[1]) <= 1 and a[2:] == b[2:]
        else:
            assert a == b


def test_pcapng_simple_packets():
    pcap = open(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), "rb").read()
    _, pk = pcap_packets(pcap)
    _, recs = pa.pcapng_records(to_pcapng(pcap, simple=True))
    got = records(recs)
    assert [(g[2], g[3], g[4]) for g in got] == [(p[2], p[3], p[4]) for p in pk]
    assert all(g[0] == 0 and g[1] == 0 for g in got)


def test_pcapng_errors(tmp_path):
    with pytest.raises(pa.PvError):
        pa.pcapng_records(struct.pack("<III", 0x0A0D0D0A, 28, 0x11223344) + b"\0" * 16)
    pcap = open(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), "rb").read()
    ng = to_pcapng(pcap)
    # truncated final block: the packets before it
    _, recs = pa.pcapng_records(ng[:-7])
    assert len(records(recs)) == len(pcap_packets(pcap)[1]) - 1
    p = tmp_path / "x.pcapng"
    p.write_bytes(ng)
    lt, nano, recs = pa.read_pcap(str(p))
    assert nano == 1 and len(records(recs)) == len(pcap_packets(pcap)[1])


@pytest.mark.parametrize("tsresol", [20, 29, 73, 127])
def test_pcapng_decimal_resolution_out_of_range(tsresol):
    """if_tsresol 10^-k with k > 19 does not fit 64-bit timestamp arithmetic: refused as a
    format error (no SIGFPE, no wrapped timestamps)"""
    pcap = open(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), "rb").read()
    lt, pk = pcap_packets(pcap)
    ng = to_pcapng(pcap[:24] + pcap[24:24 + 16 + pk[0][2]])  # one packet, default 10^-6
    # rewrite the IDB with the resolution option
    from tests.pcapng_util import _blk, _opt
    shb_len, = struct.unpack_from("<I", ng, 4)
    idb = _blk(1, struct.pack("<HHI", lt, 0, 262144) + _opt(9, bytes([tsresol])) + _opt(0, b""))
    rest = ng[shb_len:]
    old_idb_len, = struct.unpack_from("<I", rest, 4)
    with pytest.raises(pa.PvError):
        pa.pcapng_records(ng[:shb_len] + idb + rest[old_idb_len:])
