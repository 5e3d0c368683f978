"""DNS v2 ("dns", src/handlers/dns/v2) on the device against the oracle's restatement
(oracle/pv_oracle.cpp dns2_event / dns2_json), bit-exact: per-direction transaction maps in
the sorted event keys, accounting on the response in pv_xact_resolve (dns2_xact).

The reference's own v2 KATs (test_dns_layer.cpp v2 :57-302) run through the GPU path in
test_gpu_kat.py; these cases cover every fixture (UDP and TCP), synthetic query/response
mixes with all rcodes, every group (top_ecs: the query's subnet carried with its event), period shifts with time-outs,
per-direction p90 slow tops, and transactions carried across many small batches."""
import os

import numpy as np
import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.test_gpu_parity import FIXTURES, GOLD, diff

pytestmark = pytest.mark.gpu
ALL = 0x3ff  # every v2 group
ALL_NAMES = ["cardinality", "counters", "quantiles", "top_ecs", "top_qtypes", "top_rcodes", "top_size", "top_qnames",
             "top_ports", "xact_times"]
DEFAULT = 1 | 2 | 4 | 16 | 32 | 128


def run_both(oracle, pcap, host, periods, tmp_path, groups=ALL, dns2_config=None):
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    if dns2_config is None:
        dns2_config = {"enable": ALL_NAMES} if groups == ALL else {}
    gpu = pa.pktvisor_reader(str(p), host_spec=host or None, periods=periods, dns2_config=dns2_config)
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods, dns2_groups=groups)
    return gpu, ref


@pytest.mark.parametrize("periods", [1, 5])
@pytest.mark.parametrize("fixture,host", FIXTURES, ids=[f[0] for f in FIXTURES])
def test_dns2_fixture_parity(oracle, tmp_path, fixture, host, periods):
    pcap = open(os.path.join(GOLD, fixture), "rb").read()
    gpu, ref = run_both(oracle, pcap, host, periods, tmp_path)
    assert all("observed_packets" in w["dns"] for w in gpu.values())
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_dns2_default_groups(oracle, tmp_path):
    pcap = open(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), "rb").read()
    gpu, ref = run_both(oracle, pcap, "192.168.0.0/24", 1, tmp_path, DEFAULT, {})
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("cfg,n", [(1, 1000), (4, 60000)])
@pytest.mark.parametrize("periods", [1, 5])
def test_dns2_synthetic_parity(oracle, tmp_path, cfg, n, periods):
    gpu, ref = run_both(oracle, synth.pcap_bytes(cfg, n), synth.HOST_SPEC, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("periods", [2, 5])
def test_dns2_period_shifts(oracle, tmp_path, periods):
    """shifts inside the batch: purge time-outs per direction, p90 slow thresholds per direction"""
    pcap = synth.pcap_bytes(4, 200000, ts_step_us=900)
    gpu, ref = run_both(oracle, pcap, synth.HOST_SPEC, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_dns2_sparse_boundaries(oracle, tmp_path):
    """DNS shifts seconds after the Net shifts (no DNS traffic around the 60 s marks)"""
    gpu, ref = run_both(oracle, synth.sparse_dns_pcap(), synth.HOST_SPEC, 5, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_dns2_small_batches(oracle):
    """open queries carried across many small batches (per-direction keys in the carried list)"""
    pcap = synth.pcap_bytes(1, 1000)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    offs = list(idx.offsets) + [len(recs)]
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=1, max_records=512, dns2_config={"enable": ALL_NAMES})
    try:
        rng = np.random.default_rng(4)
        i = 0
        while i < idx.n:
            j = min(idx.n, i + int(rng.integers(1, 60)))
            h.process_host(recs[offs[i]:offs[j]])
            i = j
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        gpu = h.window_json(0)
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=1, window=1, dns2_groups=ALL)
    assert diff(gpu["dns"], ref["1m"]["dns"]) is None, diff(gpu["dns"], ref["1m"]["dns"])


@pytest.mark.parametrize("most", [1, 3])
def test_dns2_ecs_carried(oracle, most):
    """top_ecs with the queries in earlier batches than their responses: the subnet rides in the
    carried list (pv_xact_defer / pv_xact_carry) to the response's resolve"""
    pcap = open(os.path.join(GOLD, "ecs.pcap"), "rb").read()
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    offs = list(idx.offsets) + [len(recs)]
    h = pa.PvHandlers(num_periods=1, max_records=64, dns2_config={"enable": ALL_NAMES})
    try:
        rng = np.random.default_rng(most)
        i = 0
        while i < idx.n:
            j = min(idx.n, i + int(rng.integers(1, most + 1)))
            h.process_host(recs[offs[i]:offs[j]])
            i = j
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        gpu = h.window_json(0)
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec="", num_periods=1, window=1, dns2_groups=ALL)
    assert gpu["dns"]["unknown"]["ecs_xacts"] == 2
    assert diff(gpu["dns"], ref["1m"]["dns"]) is None, diff(gpu["dns"], ref["1m"]["dns"])


def test_dns2_tcp_parity(oracle, tmp_path):
    """DNS over TCP messages as v2 transactions (reassembly as in test_gpu_tcp.py)"""
    gpu, ref = run_both(oracle, synth.tcp_dns_pcap(2), "10.0.0.0/8,2001:db8::/32", 1, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


# ---- DNS v2 filters (dns/v2/DnsStreamHandler.cpp:61-170,484-609; process_filtered :1147-1174)
def oracle2_kw(f):
    """the oracle's v2 filter keys: the v1 typed keys plus only_xact_directions' disabled bits"""
    from tests.test_gpu_filters import oracle_kw
    kw = oracle_kw({k: v for k, v in f.items() if k != "only_xact_directions"})
    if "only_xact_directions" in f:
        kw["xact_dirs_disabled"] = 7 & ~sum({"in": 1, "out": 2, "unknown": 4}[d] for d in f["only_xact_directions"])
    return kw


V2_FILTERS = [{"exclude_noerror": True}, {"only_rcode": ["nxdomain", "refused"]}, {"only_rcode": 0, "answer_count": 0},
              {"only_qtype": ["AAAA", "TXT"]}, {"only_xact_directions": ["in"]}, {"only_xact_directions": ["out", "unknown"]},
              {"only_qname_suffix": ["test.com"]}, {"only_qname": ["nonexistent.google.com"]},
              {"only_dnssec_response": True, "only_xact_directions": ["unknown", "in"]}]


@pytest.mark.parametrize("periods", [1, 5])
@pytest.mark.parametrize("f", V2_FILTERS, ids=[",".join(f) for f in V2_FILTERS])
@pytest.mark.parametrize("fixture,host", [("dns_udp_tcp_random.pcap", "192.168.0.0/24"),
                                          ("dns_udp_mixed_rcode.pcap", "192.168.0.0/26")])
def test_dns2_filters_parity(oracle, tmp_path, fixture, host, periods, f):
    """filtered messages are events and `filtered_packets`, and still open / end transactions:
    a response to a filtered query counts as filtered, a filtered response to a valid query twice"""
    pcap = open(os.path.join(GOLD, fixture), "rb").read()
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host, periods=periods, dns2_config={"enable": ALL_NAMES, **f})
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods, dns2_groups=ALL, **oracle2_kw(f))
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("f", [{"exclude_noerror": True}, {"only_xact_directions": ["out"]}, {"only_qtype": ["A"]}],
                         ids=["noerror", "dir_out", "qtype"])
def test_dns2_filters_synthetic_shifts(oracle, tmp_path, f):
    """C4 traffic over several 60 s marks, periods 5: filtered queries purged at shifts count as
    time-outs, responses to them as filtered, across batches (carried transactions)"""
    pcap = synth.pcap_bytes(4, 120000, ts_step_us=2500)
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=synth.HOST_SPEC, periods=5, dns2_config={"enable": ALL_NAMES, **f})
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5, dns2_groups=ALL, **oracle2_kw(f))
    assert diff(gpu, ref) is None, diff(gpu, ref)
