"""DNS over TCP on the device (pv_tcp.hip + pv_dns_tcp) against the oracle's restatement of
PcapPlusPlus TcpReassembly + DnsTcpSessionData (oracle/pv_oracle.cpp), bit-exact.

The reference's own TCP fixtures are pinned in test_gpu_kat.py / test_gpu_parity.py; these
cases use synth.tcp_dns_pcap: segments cut at random byte boundaries, out-of-order and
retransmitted segments, lost SYNs, invalid framing, FIN / RST closes, port reuse, idle
connections past the 30 s timeout, messages carried across batch edges."""
import os

import numpy as np
import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.test_gpu_parity import diff, run_both

pytestmark = pytest.mark.gpu
HOST = "10.0.0.0/8,2001:db8::/32"


@pytest.mark.parametrize("periods", [1, 5])
@pytest.mark.parametrize("seed", range(6))
def test_tcp_reassembly_parity(oracle, tmp_path, seed, periods):
    gpu, ref = run_both(oracle, synth.tcp_dns_pcap(seed), HOST, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("periods", [2, 5])
def test_tcp_timeouts_and_period_shifts(oracle, tmp_path, periods):
    """150 s of traffic: connections idle 35 s time out, and DNS period shifts may fall on a
    TCP message (its stamp is the connection's end time)"""
    gpu, ref = run_both(oracle, synth.tcp_dns_pcap(11, flows=120, duration_s=150, pauses=12), HOST, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("dns_filters", [{"only_rcode": [3]}, {"only_qname": ["nonexistent.example.com"]},
                                         {"only_queries": True}, {"only_qname_suffix": ["example.net"]}])
def test_tcp_filters(oracle, tmp_path, dns_filters):
    """a TCP message meets only_rcode / only_qname as ordinary filters (no input predicate)"""
    pcap = synth.tcp_dns_pcap(3)
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=HOST, periods=1, net_config={}, dns_config=dns_filters)
    ocfg = {}
    if "only_rcode" in dns_filters:
        ocfg["only_rcode_mask"] = sum(1 << r for r in dns_filters["only_rcode"])
    if "only_qname" in dns_filters:
        ocfg["only_qname"] = ",".join(dns_filters["only_qname"])
    if "only_queries" in dns_filters:
        ocfg["only_queries"] = 1
    if "only_qname_suffix" in dns_filters:
        ocfg["only_qname_suffix"] = ",".join(dns_filters["only_qname_suffix"])
    ref = oracle.run_bytes(pcap, host_spec=HOST, num_periods=1, window=1, **ocfg)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("periods", [1, 5])
def test_tcp_across_batches(oracle, periods):
    """the same capture as many small batches: connection state, held message bytes and
    out-of-order fragments carried from batch to batch"""
    pcap = synth.tcp_dns_pcap(5, flows=80, duration_s=100, pauses=6)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    offs = list(idx.offsets) + [len(recs)]
    o = np.asarray(idx.offsets, dtype=np.int64)
    secs = np.frombuffer(recs, dtype=np.uint8)[o[:, None] + np.arange(4)].copy().view("<u4")[:, 0].astype(np.int64)

    def bad(j):  # no batch edge inside a second at which a period may shift
        return 0 < j < idx.n and secs[j] == secs[j - 1] and secs[j] != secs[0] and (secs[j] - secs[0]) % 60 == 0

    rng = np.random.default_rng(periods)
    h = pa.PvHandlers(host_spec=HOST, num_periods=periods, max_records=512)
    try:
        i = 0
        while i < idx.n:
            j = min(idx.n, i + int(rng.integers(1, 200)))
            while bad(j) and j > i + 1:
                j -= 1
            while bad(j):
                j += 1
            h.process_host(recs[offs[i]:offs[j]])
            i = j
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        key = f"{1 if periods == 1 else periods}m"
        gpu = {key: h.window_json(0 if periods == 1 else periods, merged=periods != 1)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec=HOST, num_periods=periods, window=periods)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("seed", range(6))
def test_tcp_exact_lru_parity(oracle, tmp_path, seed):
    """the exact LRU mode (pv_set_tcp_exact_lru): PcapInputStream's LRU list of every TCP
    connection replayed per packet; the same windows as the restatement"""
    pcap = synth.tcp_dns_pcap(seed)
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=HOST, periods=5, tcp_exact_lru=True)
    ref = oracle.run_bytes(pcap, host_spec=HOST, num_periods=5, window=5)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_tcp_exact_lru_without_handshakes(oracle, tmp_path):
    """The reference's TCP fixture read through a BPF program that drops the small packets (every
    handshake, ACK and FIN segment; VERDICT r4: the default mode reported 1 413 more TCP
    responses here). Each connection's first packet then carries data, so its LRU entry holds
    the zero endTime and PcapInputStream closes it as soon as it reaches the list's tail; its
    response is a packet of a closed flow. The exact LRU mode reproduces that."""
    from tests import bpf_progs
    pcap = open(os.path.join(os.path.dirname(__file__), "golden", "dns_udp_tcp_random.pcap"), "rb").read()
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    insns = bpf_progs.ARITH
    gpu = pa.pktvisor_reader(str(p), host_spec="192.168.0.0/24", periods=1, bpf=insns, tcp_exact_lru=True)
    kept = pcap[:24] + bpf_progs.filter_records(pcap[24:], insns)
    ref = oracle.run_bytes(kept, host_spec="192.168.0.0/24", num_periods=1, window=1)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("lost_syn", [False, True])
def test_tcp_exact_lru_across_batches(oracle, lost_syn):
    """the exact mode over small batches: the LRU list carried on the host, connections closed in
    a batch that holds none of their packets (close-only segments)"""
    pcap = synth.tcp_dns_pcap(7, flows=80, duration_s=100, pauses=6)
    if lost_syn:
        # drop every SYN: first packets carry data (zero endTime entries)
        keep = []
        for _, _, r in synth.records_of(pcap):
            f = r[16:]
            if len(f) > 47 and f[12:14] == b"\x08\x00" and f[23] == 6 and f[14 + (f[14] & 15) * 4 + 13] & 2:
                continue
            keep.append(r)
        pcap = pa.pcap_file_bytes(b"".join(keep))
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    offs = list(idx.offsets) + [len(recs)]
    rng = np.random.default_rng(3)
    h = pa.PvHandlers(host_spec=HOST, num_periods=1, max_records=512, tcp_exact_lru=True)
    try:
        i = 0
        while i < idx.n:
            j = min(idx.n, i + int(rng.integers(1, 200)))
            h.process_host(recs[offs[i]:offs[j]])
            i = j
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        gpu = {"1m": h.window_json(0)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec=HOST, num_periods=1, window=1)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def _batches(h, recs, idx, rng, eoc=True):
    offs = list(idx.offsets) + [len(recs)]
    i = 0
    while i < idx.n:
        j = min(idx.n, i + int(rng.integers(1, 200)))
        if j == idx.n and eoc:
            h.set_end_of_capture()
        h.process_host(recs[offs[i]:offs[j]])
        i = j


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("periods", [1, 5])
@pytest.mark.parametrize("seed", range(3))
def test_tcp_end_of_capture_flush(oracle, tmp_path, seed, periods, exact):
    """connections that lost a segment for good and never close: the segments after the hole are
    held until the file ends, when PcapInputStream closes every connection
    (PcapInputStream.cpp:522, TcpReassembly::closeAllConnections) and their out-of-order data is
    delivered (pv_set_end_of_capture, pv_tcp_eoc)"""
    pcap = synth.tcp_dns_pcap(seed, flows=80, open_tails=16)
    gpu, ref = run_both(oracle, pcap, HOST, periods, tmp_path, tcp_exact_lru=exact)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("exact", [False, True])
def test_tcp_end_of_capture_across_batches(oracle, exact):
    """the flush armed before the last of many small batches; without it the held data is lost,
    (the control run must differ, so the capture really leaves data for the flush: most held data
    follows a "[N bytes missing]" text and frames nothing, but in this capture one connection's
    flushed bytes complete a message whose question parses)"""
    pcap = synth.tcp_dns_pcap(0, flows=80, open_tails=16)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    ref = oracle.run_bytes(pcap, host_spec=HOST, num_periods=1, window=1)
    got = []
    for eoc in (True, False):
        h = pa.PvHandlers(host_spec=HOST, num_periods=1, max_records=512, tcp_exact_lru=exact)
        try:
            _batches(h, recs, idx, np.random.default_rng(9), eoc)
            h.set_end_tstamp(*pa.last_record_ts(recs, idx))
            got.append({"1m": h.window_json(0)})
        finally:
            h.close()
    assert diff(got[0], ref) is None, diff(got[0], ref)
    if not exact:  # (the exact LRU list closes that connection before the end: a lost SYN)
        assert diff(got[1], ref) is not None


def test_tcp_end_of_capture_device_batch(oracle):
    """the flush after a batch resident in HBM (pv_process_device, the bench's entry point)"""
    import torch
    pcap = synth.tcp_dns_pcap(6, flows=120, duration_s=40, open_tails=24)
    recs = pcap[24:]
    buf = np.zeros(len(recs) + 256, dtype=np.uint8)
    buf[:len(recs)] = np.frombuffer(recs, dtype=np.uint8)
    idx = pa.RecordIndex(recs)
    d_recs = torch.from_numpy(buf).cuda()
    d_offs = torch.from_numpy(idx.offsets).cuda()
    torch.cuda.synchronize()
    h = pa.PvHandlers(host_spec=HOST, num_periods=5, max_records=idx.n)
    try:
        h.set_end_of_capture()
        h.process_device(d_recs.data_ptr(), d_offs.data_ptr(), idx)
        h.synchronize()
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        gpu = {"5m": h.window_json(5, merged=True)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec=HOST, num_periods=5, window=5)
    assert diff(gpu, ref) is None, diff(gpu, ref)
