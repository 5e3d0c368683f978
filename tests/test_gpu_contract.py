"""The output contract on the GPU path, against the oracle and the reference's own checks:
metric groups (enable / disable, including histograms, top_ecs, top_qnames_details), window
keys (topn_count, topn_percentile_threshold), the geo filters without a geo database, the
reference's window schemas, and the ECS known answers (test_dns_layer.cpp:711-757)."""
import json
import os

import pytest

import pktvisor_amd as pa
from pktvisor_amd import config as pvcfg
from pktvisor_amd import synth
from tests.schema_check import errors
from tests.test_gpu_filters import oracle_kw
from tests.test_gpu_parity import diff

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

CONFIGS = [
    ({}, {}),
    ({}, {"enable": ["top_ecs", "top_qnames_details", "histograms"]}),
    ({}, {"disable": ["cardinality", "counters"], "enable": ["histograms"]}),
    ({}, {"disable": ["top_qnames", "dns_transaction"]}),
    ({}, {"disable": ["quantiles"], "enable": ["histograms", "top_ecs"]}),
    ({"disable": ["all"]}, {"disable": ["all"]}),
    ({"disable": ["top_ips"]}, {"enable": ["all"]}),
    ({"disable": ["cardinality", "counters"]}, {"disable": ["top_ports"], "topn_count": 3}),
    ({"topn_percentile_threshold": 50}, {"topn_percentile_threshold": 50, "enable": ["top_qnames_details"]}),
    ({"asn_notfound": True}, {"geoloc_notfound": True}),
    ({}, {"xact_ttl_ms": 30, "only_queries": True, "enable": ["histograms"]}),
]
IDS = ["defaults", "ecs_details_hist", "no_card_ctr_hist", "no_qnames_xact", "hist_not_quant", "all_off", "all_on",
       "net_no_card_ctr_top3", "pct50", "geo_filters", "ttl30_queries"]


def oracle_config(net_cfg, dns_cfg, periods):
    """the oracle's keys for a pair of handler configs (the same typed result the GPU gets)"""
    win = pvcfg.window_config([net_cfg, dns_cfg])
    n, d = pvcfg.net_start(dict(net_cfg)), pvcfg.dns_start(dict(dns_cfg))
    kw = dict(num_periods=periods, window=periods, net_groups=n["groups"] & 0xff, dns_groups=d["groups"] & 0xfff,
              topn_count=win.get("topn_count", 10), topn_pct=win.get("topn_percentile_threshold", 0))
    if n["filter_all"]:
        kw["net_filter_all"] = 1
    if d["filters"]["filter_all"]:
        kw["filter_all"] = 1
    if d["xact_ttl_ms"] is not None:
        kw["xact_ttl_ms"] = d["xact_ttl_ms"]
    f = {k: dns_cfg[k] for k in pa.DNS_FILTER_KEYS if k in dns_cfg}
    kw.update(oracle_kw(f) if f else {})
    return kw


def run_both(oracle, pcap: bytes, host: str, periods: int, tmp_path, net_cfg, dns_cfg):
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host or None, periods=periods, net_config=net_cfg, dns_config=dns_cfg)
    ref = oracle.run_bytes(pcap, host_spec=host, **oracle_config(net_cfg, dns_cfg, periods))
    return gpu, ref


@pytest.mark.parametrize("cfgs", CONFIGS, ids=IDS)
@pytest.mark.parametrize("src", ["dns_udp_tcp_random", "ecs", "c4"])
def test_groups_parity(oracle, tmp_path, cfgs, src):
    if src == "c4":
        pcap, host = synth.pcap_bytes(4, 60000, ts_step_us=1500), synth.HOST_SPEC
    else:
        pcap, host = open(os.path.join(GOLD, f"{src}.pcap"), "rb").read(), "192.168.0.0/24"
    for periods in (1, 5):
        gpu, ref = run_both(oracle, pcap, host, periods, tmp_path, *cfgs)
        assert diff(gpu, ref) is None, (periods, diff(gpu, ref))


def test_window_schemas():
    """the reference's schema tests' configs (dns/v1/tests/test_json_schema.cpp:24-39,
    net/v1/tests/test_json_schema.cpp) on the GPU path"""
    path = os.path.join(GOLD, "dns_udp_tcp_random.pcap")
    out = pa.pktvisor_reader(path, host_spec="192.168.0.0/24", periods=5, net_config={},
                             dns_config={"recorded_stream": True, "enable": ["top_ecs", "top_ports", "top_qnames_details"]})
    dns_s = json.load(open(os.path.join(GOLD, "dns_v1_window-schema.json")))
    net_s = json.load(open(os.path.join(GOLD, "net_v1_window-schema.json")))
    assert errors(dns_s, {"dns": out["5m"]["dns"]}) == []
    assert errors(net_s, {"packets": out["5m"]["packets"]}) == []


def test_ecs_reference_kat():
    """test_dns_layer.cpp:711-757 on ecs.pcap (its UDP share: the ECS queries are UDP)"""
    d = pa.pktvisor_reader(os.path.join(GOLD, "ecs.pcap"), host_spec="192.168.0.0/24", periods=1, net_config={},
                           dns_config={"enable": ["top_ecs"]})["1m"]["dns"]
    assert d["wire_packets"]["query_ecs"] == 5
    assert d["cardinality"]["qname"] == 9
    assert d["top_query_ecs"] == [{"name": "2001:470:1f0b:1600::", "estimate": 5}]
    # no geo database is enabled (the KAT enables the MaxMind test databases)
    assert d["top_geoLoc_ecs"] == [] and d["top_asn_ecs"] == []


def test_topn_custom_size():
    """test_dns_layer.cpp:412-444: topn_count 3 lists three qtypes"""
    d = pa.pktvisor_reader(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), host_spec="192.168.0.0/24", periods=1,
                           net_config={}, dns_config={"topn_count": 3})["1m"]["dns"]
    assert len(d["top_qtype"]) == 3 and len(d["top_qname2"]) <= 3
