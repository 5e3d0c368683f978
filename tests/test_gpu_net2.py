"""Net v2 ("net", src/handlers/net/v2) on the device (pv_net2_kernel) against the oracle's
restatement (oracle/pv_oracle.cpp net2_packet / net2_json), bit-exact, next to v1.

The reference's own v2 KATs (test_net_layer.cpp:15-181,358-440) run through the GPU path in
test_gpu_kat.py; these cases cover every fixture, the synthetic shapes (both directions,
IPv6, the edge mix of VLAN / extension headers / fragments / tunnels), group subsets,
merged multi-period windows and many small batches."""
import os

import numpy as np
import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.test_gpu_parity import FIXTURES, GOLD, diff

pytestmark = pytest.mark.gpu
ALL = 31


def run_both(oracle, pcap, host, periods, tmp_path, net2_config=None, groups=ALL):
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host or None, periods=periods, net2_config=net2_config or {})
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods, net2_groups=groups)
    return gpu, ref


@pytest.mark.parametrize("periods", [1, 5])
@pytest.mark.parametrize("fixture,host", FIXTURES, ids=[f[0] for f in FIXTURES])
def test_net2_fixture_parity(oracle, tmp_path, fixture, host, periods):
    pcap = open(os.path.join(GOLD, fixture), "rb").read()
    gpu, ref = run_both(oracle, pcap, host, periods, tmp_path)
    assert all("net" in w for w in gpu.values())
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("cfg,n,host", [(2, 60000, synth.HOST_SPEC), (4, 60000, synth.HOST_SPEC),
                                        (9, 40000, "10.0.0.0/8,2000::/3,192.168.0.0/16")])
@pytest.mark.parametrize("periods", [1, 5])
def test_net2_synthetic_parity(oracle, tmp_path, cfg, n, host, periods):
    gpu, ref = run_both(oracle, synth.pcap_bytes(cfg, n), host, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_net2_multi_period(oracle, tmp_path):
    """period shifts inside the batch: counters, payload histograms and CPC per period"""
    pcap = synth.pcap_bytes(4, 200000, ts_step_us=900)
    gpu, ref = run_both(oracle, pcap, synth.HOST_SPEC, 5, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("disable,groups", [(["cardinality", "counters"], 4 | 8 | 16), (["top_ips", "top_geo"], 1 | 2 | 4),
                                            (["quantiles"], 1 | 2 | 8 | 16)])
def test_net2_groups(oracle, tmp_path, disable, groups):
    pcap = open(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), "rb").read()
    gpu, ref = run_both(oracle, pcap, "192.168.0.0/24", 1, tmp_path, {"disable": disable}, groups)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_net2_small_batches(oracle):
    """many small batches: the LDS histogram and key cache are per workgroup and batch"""
    pcap = synth.pcap_bytes(4, 30000)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    offs = list(idx.offsets) + [len(recs)]
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=1, max_records=4096, net2_config={})
    try:
        rng = np.random.default_rng(2)
        i = 0
        while i < idx.n:
            j = min(idx.n, i + int(rng.integers(1, 3000)))
            h.process_host(recs[offs[i]:offs[j]])
            i = j
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        gpu = {"1m": h.window_json(0)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=1, window=1, net2_groups=ALL)
    assert diff(gpu["1m"]["net"], ref["1m"]["net"]) is None, diff(gpu["1m"]["net"], ref["1m"]["net"])
