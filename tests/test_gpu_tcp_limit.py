"""PcapInputStream's tcp_packet_reassembly_cache_limit (src/inputs/pcap/PcapInputStream.cpp:97-99,
254-283,449-465) on the device: a dry run of the TCP stage records each segment's LRU events,
the host replays the LRU list (pv_host.cpp tcp_lru_replay) and the stage closes the connections
it evicts. Against the oracle's sequential restatement (every TCP connection in the list, the
reference's put / erase / overflow order), bit-exact; the reference KAT (DNS v2 "TCP tests with
limit", test_dns_layer.cpp:131-162) runs in test_gpu_kat.py."""
import os

import numpy as np
import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.test_gpu_parity import GOLD, diff

pytestmark = pytest.mark.gpu
HOST = "10.0.0.0/8,2001:db8::/32"


def both(oracle, pcap, tmp_path, host, periods, limit, **kw):
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host or None, periods=periods, tcp_packet_reassembly_cache_limit=limit,
                             **kw)
    okw = {}
    if "dns2_config" in kw:
        okw["dns2_groups"] = 0x3ff
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods,
                           tcp_packet_reassembly_cache_limit=limit, **okw)
    return gpu, ref


@pytest.mark.parametrize("limit", [1, 2, 5, 10, 40, 100000])
@pytest.mark.parametrize("fixture,host", [("dns_ipv4_tcp.pcap", ""), ("dns_ipv6_tcp.pcap", ""),
                                          ("dns_udp_tcp_random.pcap", "192.168.0.0/24")])
def test_limit_fixture_parity(oracle, tmp_path, fixture, host, limit):
    gpu, ref = both(oracle, open(os.path.join(GOLD, fixture), "rb").read(), tmp_path, host, 1, limit)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("limit", [3, 10])
def test_limit_v2(oracle, tmp_path, limit):
    pcap = open(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), "rb").read()
    gpu, ref = both(oracle, pcap, tmp_path, "192.168.0.0/24", 5, limit,
                    dns2_config={"enable": ["top_size", "top_ports", "top_ecs", "xact_times"]})
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("limit", [4, 16, 64])
@pytest.mark.parametrize("periods", [1, 5])
def test_limit_synthetic(oracle, tmp_path, limit, periods):
    """connections cut at random bytes, out of order, lost SYNs, FIN / RST, non-DNS TCP (443) in
    the same list, idle connections past the 30 s timeout"""
    pcap = synth.tcp_dns_pcap(7, flows=120, duration_s=150, pauses=10)
    gpu, ref = both(oracle, pcap, tmp_path, HOST, periods, limit)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("limit", [2, 3])
def test_limit_reput_crafted(oracle, tmp_path, limit):
    """closing an evicted connection flushes its held fragment, whose put evicts the next tail
    (synth.tcp_reput_pcap: at 2 no TCP query survives, at 3 one does; the oracle's counts are
    pinned by test_synth_oracle.py::test_tcp_reput_crafted)"""
    gpu, ref = both(oracle, synth.tcp_reput_pcap(), tmp_path, "", 1, limit)
    assert diff(gpu, ref) is None, diff(gpu, ref)
    assert gpu["1m"]["dns"]["wire_packets"]["tcp"] == (0 if limit == 2 else 1)


@pytest.mark.parametrize("limit", [2, 3, 5, 8])
@pytest.mark.parametrize("seed", [1, 2])
def test_limit_held_evict(oracle, tmp_path, seed, limit):
    """connections evicted while they hold out-of-order fragments (synth.tcp_held_evict_pcap:
    seed 1 at limit 3 has 17 such closes whose flush evicts another connection)"""
    gpu, ref = both(oracle, synth.tcp_held_evict_pcap(seed), tmp_path, HOST, 1, limit)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("limit,kind", [(3, "dns"), (12, "dns"), (3, "held")])
def test_limit_across_batches(oracle, limit, kind):
    """many small batches: the LRU list, and evictions of connections with no segment in their
    batch (closed ahead of their next segment), carried from batch to batch; "held": the
    connections holding fragments, carried too"""
    pcap = synth.tcp_dns_pcap(5, flows=80, duration_s=100, pauses=6) if kind == "dns" else synth.tcp_held_evict_pcap(3)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    offs = list(idx.offsets) + [len(recs)]
    o = np.asarray(idx.offsets, dtype=np.int64)
    secs = np.frombuffer(recs, dtype=np.uint8)[o[:, None] + np.arange(4)].copy().view("<u4")[:, 0].astype(np.int64)
    rng = np.random.default_rng(limit)
    h = pa.PvHandlers(host_spec=HOST, num_periods=1, max_records=512, tcp_packet_reassembly_cache_limit=limit)
    try:
        i = 0
        while i < idx.n:
            j = min(idx.n, i + int(rng.integers(1, 200)))
            h.process_host(recs[offs[i]:offs[j]])
            i = j
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        gpu = {"1m": h.window_json(0, merged=False)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec=HOST, num_periods=1, window=1, tcp_packet_reassembly_cache_limit=limit)
    assert diff(gpu, ref) is None, diff(gpu, ref)
    assert secs.size == idx.n


def test_limit_set_before_first_batch(tmp_path):
    h = pa.PvHandlers(num_periods=1, max_records=64)
    try:
        pcap = open(os.path.join(GOLD, "dns_ipv4_tcp.pcap"), "rb").read()
        h.process_host(pcap[24:])
        with pytest.raises(pa.PvError, match="before the first batch"):
            h._check(h.lib.pv_set_tcp_reassembly_limit(h.ctx, 10), "pv_set_tcp_reassembly_limit")
    finally:
        h.close()
