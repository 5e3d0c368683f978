"""deep_sample_rate < 100 on the GPU path against the oracle's restatement (jsf32 draws per
manager in stream order; not-deep events count in the counters only; a not-deep response
pairs but feeds no quantile, ratio or slow top): reference fixtures and a synthetic C4 capture
over many ingest batches; DNS filters (a filtered event draws nothing and counts the manager's
last flag, process_filtered) and DNS over TCP (messages draw in stream order among the UDP
events), and the v2 handlers (Net v2's draws equal v1's; a DNS v2 response's draw decides
new_dns_transaction's deep part; v2 filters draw nothing). Geo filters with sampling fail loudly."""
import os

import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.test_gpu_parity import GOLD, diff

pytestmark = pytest.mark.gpu


def both(oracle, pcap, tmp_path, host, periods, rate, f=None, **kw):
    from tests.test_gpu_filters import oracle_kw
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host or None, periods=periods, deep_sample_rate=rate, dns_filters=f, **kw)
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods, deep_sample_rate=rate,
                           **(oracle_kw(f) if f else {}))
    return gpu, ref


@pytest.mark.parametrize("fixture,host", [("dns_ipv4_udp.pcap", ""), ("dns_ipv6_udp.pcap", ""),
                                          ("dns_udp_mixed_rcode.pcap", "")])
@pytest.mark.parametrize("rate", [1, 50, 99])
@pytest.mark.parametrize("periods", [1, 5])
def test_fixture_sampled_parity(oracle, tmp_path, fixture, host, rate, periods):
    gpu, ref = both(oracle, open(os.path.join(GOLD, fixture), "rb").read(), tmp_path, host, periods, rate)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("rate", [33, 80])
def test_synthetic_sampled_parity_many_batches(oracle, tmp_path, monkeypatch, rate):
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "1")
    pcap = synth.pcap_bytes(4, 60000, ts_step_us=1500)
    gpu, ref = both(oracle, pcap, tmp_path, synth.HOST_SPEC, 5, rate)
    assert diff(gpu, ref) is None, diff(gpu, ref)


SAMPLED_FILTERS = [None, {"only_qtype": ["AAAA", "TXT"]}, {"exclude_noerror": True}, {"only_queries": True},
                   {"only_rcode": ["noerror"]}, {"only_qname_suffix": ["test.com"]}, {"answer_count": 0}]


@pytest.mark.parametrize("rate", [1, 50, 99])
@pytest.mark.parametrize("f", SAMPLED_FILTERS, ids=["none"] + [",".join(f) for f in SAMPLED_FILTERS[1:]])
@pytest.mark.parametrize("periods", [1, 5])
def test_sampled_filters_udp_tcp(oracle, tmp_path, rate, f, periods):
    """the reference's mixed UDP / TCP capture with DNS filters at rates 1 / 50 / 99"""
    pcap = open(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), "rb").read()
    gpu, ref = both(oracle, pcap, tmp_path, "192.168.0.0/24", periods, rate, f)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("rate", [20, 70])
def test_sampled_tcp_synthetic(oracle, tmp_path, rate):
    """DNS-over-TCP connections (out-of-order, retransmitted, cut at random bytes) among UDP DNS"""
    pcap = synth.tcp_dns_pcap(seed=4, flows=80, duration_s=150.0)
    gpu, ref = both(oracle, pcap, tmp_path, "10.0.0.0/8", 5, rate, {"only_qtype": ["A", "AAAA", "MX"]})
    assert diff(gpu, ref) is None, diff(gpu, ref)


# ---- the v2 handlers (net/v2 ...cpp:494-500,756-762; dns/v2 ...cpp:1006-1008,1092-1174)
V2_ALL = ["cardinality", "counters", "quantiles", "top_ecs", "top_qtypes", "top_rcodes", "top_size", "top_qnames",
          "top_ports", "xact_times"]


@pytest.mark.parametrize("rate", [1, 50, 99])
@pytest.mark.parametrize("periods", [1, 5])
@pytest.mark.parametrize("fixture,host", [("dns_udp_tcp_random.pcap", "192.168.0.0/24"),
                                          ("dns_udp_mixed_rcode.pcap", "192.168.0.0/26"), ("dns_ipv6_udp.pcap", "")])
def test_v2_sampled_parity(oracle, tmp_path, fixture, host, rate, periods):
    """Net v2 next to v1 and DNS v2, every v2 group, UDP and TCP DNS"""
    pcap = open(os.path.join(GOLD, fixture), "rb").read()
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host or None, periods=periods, deep_sample_rate=rate, net2_config={},
                             dns2_config={"enable": V2_ALL})
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods, deep_sample_rate=rate,
                           net2_groups=0x1f, dns2_groups=0x3ff)
    assert diff(gpu, ref) is None, diff(gpu, ref)


V2_SAMPLED_FILTERS = [{"exclude_noerror": True}, {"only_qtype": ["AAAA", "TXT"]}, {"only_xact_directions": ["in"]},
                      {"only_qname_suffix": ["test.com"]}]


@pytest.mark.parametrize("rate", [1, 50, 99])
@pytest.mark.parametrize("f", V2_SAMPLED_FILTERS, ids=[",".join(f) for f in V2_SAMPLED_FILTERS])
def test_v2_sampled_filters(oracle, tmp_path, rate, f):
    """DNS v2 filters with sampling: a filtered message draws nothing and counts the last flag"""
    from tests.test_gpu_dns2 import oracle2_kw
    pcap = open(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), "rb").read()
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec="192.168.0.0/24", periods=5, deep_sample_rate=rate,
                             dns2_config={"enable": V2_ALL, **f})
    ref = oracle.run_bytes(pcap, host_spec="192.168.0.0/24", num_periods=5, window=5, deep_sample_rate=rate,
                           dns2_groups=0x3ff, **oracle2_kw(f))
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("rate", [30, 90])
def test_v2_sampled_synthetic_shifts(oracle, tmp_path, monkeypatch, rate):
    """C4 traffic over several 60 s marks in 1 MiB ingest batches, Net v2 + DNS v2"""
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "1")
    pcap = synth.pcap_bytes(4, 80000, ts_step_us=2500)
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=synth.HOST_SPEC, periods=5, deep_sample_rate=rate, net2_config={},
                             dns2_config={"enable": V2_ALL})
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5, deep_sample_rate=rate,
                           net2_groups=0x1f, dns2_groups=0x3ff)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_sampling_refusals(tmp_path):
    with pytest.raises(pa.PvError, match="geo filters"):
        pa.PvHandlers(deep_sample_rate=50, net_config={"geoloc_notfound": True})
