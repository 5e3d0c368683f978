"""Prometheus and OpenTelemetry output of the v2 handlers (DnsMetricsBucket::to_prometheus,
dns/v2/DnsStreamHandler.cpp:759-842; NetworkMetricsBucket::to_prometheus,
net/v2/NetStreamHandler.cpp:333-383): every sample of the text equals the value the same
bucket's JSON holds, per direction label. No reference fixture holds v2 Prometheus text, so the
names and labels follow the metric definitions (DnsStreamHandler.h / NetStreamHandler.h) and the
values are pinned to the JSON, itself pinned to the oracle in test_gpu_dns2.py / test_gpu_net2.py."""
import os
import re

import pytest

import pktvisor_amd as pa
from tests.test_gpu_dns2 import ALL_NAMES
from tests.test_gpu_parity import GOLD

pytestmark = pytest.mark.gpu

LINE = re.compile(r'^([a-z0-9_]+)\{(.*)\} (\S+)$')


def samples(txt):
    out = {}
    for ln in txt.splitlines():
        if ln.startswith("#") or not ln:
            continue
        m = LINE.match(ln)
        assert m, ln
        labels = dict(re.findall(r'(\w+)="([^"]*)"', m.group(2)))
        labels.pop("instance", None)  # a static label another test may have added (process-wide)
        out[(m.group(1), tuple(sorted(labels.items())))] = float(m.group(3))
    return out


def get(s, name, **labels):
    return s[(name, tuple(sorted(labels.items())))]


@pytest.mark.parametrize("fixture,host", [("dns_udp_mixed_rcode.pcap", "192.168.0.0/24"),
                                          ("dns_udp_tcp_random.pcap", "192.168.0.0/24")])
def test_v2_prometheus_matches_json(fixture, host):
    recs_path = os.path.join(GOLD, fixture)
    lt, tn, recs = pa.read_pcap(recs_path)
    h = pa.PvHandlers(host_spec=host, num_periods=1, linktype=lt, ts_nano=tn, max_records=1 << 16,
                      net2_config={}, dns2_config={"enable": ALL_NAMES})
    try:
        h.process_host(recs)
        j = h.window_json(0)
        s = samples(h.window_prometheus(0, labels={"policy": "p"}))
        otlp = h.window_opentelemetry(0, labels={"policy": "p"})
    finally:
        h.close()
    d, n = j["dns"], j["net"]
    assert get(s, "dns_observed_packets", policy="p") == d["observed_packets"]
    assert get(s, "dns_filtered_packets", policy="p") == d["filtered_packets"]
    assert get(s, "net_observed_packets", policy="p") == n["observed_packets"]
    dirs = [x for x in ("in", "out", "unknown") if x in d]
    assert dirs
    for x in dirs:
        jd = d[x]
        for k in ("xacts", "udp_xacts", "tcp_xacts", "ipv4_xacts", "nxdomain_xacts", "noerror_xacts", "timeout_queries",
                  "orphan_responses", "checking_disabled_xacts"):
            assert get(s, f"dns_{k}", policy="p", direction=x) == jd[k], (x, k)
        assert get(s, "dns_cardinality_qname", policy="p", direction=x) == jd["cardinality"]["qname"]
        for e in jd["top_qname2_xacts"]:
            assert get(s, "dns_top_qname2_xacts", policy="p", direction=x, qname=e["name"]) == e["estimate"]
        for e in jd["top_rcode_xacts"]:
            assert get(s, "dns_top_rcode_xacts", policy="p", direction=x, rcode=e["name"]) == e["estimate"]
        if "xact_time_us" in jd:
            q = jd["xact_time_us"]
            assert get(s, "dns_xact_time_us", policy="p", direction=x, quantile="0.5") == q["p50"]
            assert get(s, "dns_xact_time_us", policy="p", direction=x, quantile="0.99") == q["p99"]
            assert get(s, "dns_xact_histogram_us_bucket", policy="p", direction=x, le="+Inf") == jd["xact_histogram_us"]["buckets"]["+Inf"]
    for x in ("in", "out", "unknown"):
        if x not in n:
            continue
        for k in ("udp_packets", "tcp_packets", "ipv4_packets", "ipv6_packets", "total_packets"):
            assert get(s, f"net_{k}", policy="p", direction=x) == n[x][k], (x, k)
        for e in n[x]["top_ipv4_packets"]:
            assert get(s, "net_top_ipv4_packets", policy="p", direction=x, ipv4=e["name"]) == e["estimate"]
    # OpenTelemetry: the same metric names as ScopeMetrics entries, with the direction attribute
    for name in (b"dns_xacts", b"dns_observed_packets", b"net_udp_packets", b"direction"):
        assert name in otlp
