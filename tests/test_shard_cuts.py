"""pv_shard_cuts (CPU): a sharded run's record cuts keep every DNS-over-TCP connection inside
one shard and stay near the equal split when the capture allows it."""
import struct

import numpy as np

import pktvisor_amd as pa
from pktvisor_amd import synth

DNS_PORTS = {53, 5353, 5355, 53000}


def tcp_flow_keys(pcap):
    """per record: an order-free 4-tuple of a TCP packet with a DNS port (Ethernet + IPv4/IPv6), else None"""
    keys = []
    for _, _, r in synth.records_of(pcap):
        f = r[16:]
        k = None
        et = struct.unpack_from(">H", f, 12)[0] if len(f) >= 14 else 0
        if et == 0x0800 and len(f) >= 34 and f[23] == 6:
            hl = (f[14] & 15) * 4
            sp, dp = struct.unpack_from(">HH", f, 14 + hl)
            if sp in DNS_PORTS or dp in DNS_PORTS:
                k = frozenset([(bytes(f[26:30]), sp), (bytes(f[30:34]), dp)])
        elif et == 0x86DD and len(f) >= 58 and f[20] == 6:
            sp, dp = struct.unpack_from(">HH", f, 54)
            if sp in DNS_PORTS or dp in DNS_PORTS:
                k = frozenset([(bytes(f[22:38]), sp), (bytes(f[38:54]), dp)])
        keys.append(k)
    return keys


def cuts_of(pcap, world):
    lt, tn, recs = 1, 0, pcap[24:]
    idx = pa.RecordIndex(recs, tn)
    return pa.shard_cuts(recs, idx, lt, tn, world), idx.n


def test_cuts_keep_tcp_flows_whole():
    pcap = synth.merged_pcap(synth.pcap_bytes(4, 20000, ts_step_us=5000),
                             synth.tcp_dns_pcap(seed=5, flows=150, duration_s=90.0))
    keys = tcp_flow_keys(pcap)
    spans = {}
    for i, k in enumerate(keys):
        if k is not None:
            a, b = spans.get(k, (i, i))
            spans[k] = (min(a, i), max(b, i))
    n = len(keys)
    ok = [not any(a < c <= b for a, b in spans.values()) for c in range(n + 1)]
    for world in (2, 3, 8):
        cuts, n2 = cuts_of(pcap, world)
        assert n2 == n and cuts[0] == 0 and cuts[-1] == n and cuts == sorted(cuts)
        per = (n + world - 1) // world
        for r in range(1, world):
            c = cuts[r]
            assert ok[c], (world, c)
            # the allowed boundary nearest the equal split (not before the previous cut)
            ideal = max(cuts[r - 1], min(n, r * per))
            d = abs(c - ideal)
            assert not any(ok[x] for x in range(max(cuts[r - 1], ideal - d + 1), min(n, ideal + d - 1) + 1)), (world, c)


def test_cuts_equal_split_without_tcp():
    pcap = synth.pcap_bytes(4, 10000)
    for world in (1, 2, 7):
        cuts, n = cuts_of(pcap, world)
        per = (n + world - 1) // world
        assert cuts == [min(n, r * per) for r in range(world)] + [n]


def test_cut_moves_past_a_long_connection():
    """one connection across the whole capture: every cut lands after its last packet"""
    pcap = synth.tcp_dns_pcap(seed=2, flows=1, duration_s=5.0, udp_share=2.0, noise_share=2.0)
    keys = tcp_flow_keys(pcap)
    last = max(i for i, k in enumerate(keys) if k is not None)
    first = min(i for i, k in enumerate(keys) if k is not None)
    cuts, n = cuts_of(pcap, 4)
    for c in cuts[1:-1]:
        assert c <= first or c > last
