"""DNS over TCP on the device (pv_tcp.hip + pv_dns_tcp) against the oracle's restatement of
PcapPlusPlus TcpReassembly + DnsTcpSessionData (oracle/pv_oracle.cpp), bit-exact.

The reference's own TCP fixtures are pinned in test_gpu_kat.py / test_gpu_parity.py; these
cases use synth.tcp_dns_pcap: segments cut at random byte boundaries, out-of-order and
retransmitted segments, lost SYNs, invalid framing, FIN / RST closes, port reuse, idle
connections past the 30 s timeout, messages carried across batch edges."""
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
