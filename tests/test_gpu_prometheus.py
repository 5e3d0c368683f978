"""window_prometheus on the GPU path (pv_window_prometheus).

The text format is the reference primitives' (pinned line by line by
src/tests/test_metrics.cpp:160-170,219-239,285-307,421-465,525-535: "# HELP", "# TYPE",
static labels then the added ones, each set in key order, quantile / le / item labels);
the metric order, names and HELP texts are the handlers' (net/v1
NetStreamHandler.cpp:332-388 + .h:81-127, dns/v1 DnsStreamHandler.cpp:1139-1238 +
.h:116-171). The values are checked against the same bucket's window JSON, which the
oracle pins bit-exactly elsewhere; `_sum` (the sketch's max item) and `_count` are
checked against the JSON's own counts where it has them.
"""
import os
import re

import pytest

import pktvisor_amd as pa

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SAMPLE = re.compile(r'^([a-z0-9_]+)\{(.*)\} (\S+)$')


def run(path, host_spec, dns_config=None):
    linktype, ts_nano, recs = pa.read_pcap(path)
    idx = pa.RecordIndex(recs, ts_nano)
    h = pa.PvHandlers(host_spec=host_spec, num_periods=1, linktype=linktype, ts_nano=ts_nano,
                      max_records=max(1, idx.n), dns_config=dns_config or {})
    try:
        h.process_host(recs)
        h.set_end_tstamp(*pa.last_record_ts(recs, idx, ts_nano))
        return h.window_json(0), h.window_prometheus(0, {"policy": "default"})
    finally:
        h.close()


def parse(txt):
    """[(name, labels dict, value str)] plus the HELP/TYPE header of every metric, checked"""
    out, heads = [], {}
    lines = txt.splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i]
        if ln.startswith("# HELP "):
            name = ln.split(" ")[2]
            t = lines[i + 1].split(" ")
            assert t[:3] == ["#", "TYPE", name], (ln, lines[i + 1])
            heads[name] = t[3]
            i += 2
            continue
        m = SAMPLE.match(ln)
        assert m, ln
        labels = dict(re.findall(r'([a-z0-9_]+)="([^"]*)"', m.group(2)))
        out.append((m.group(1), labels, m.group(3), m.group(2)))
        i += 1
    return out, heads


@pytest.fixture(scope="module", autouse=True)
def static_label():
    pa.add_static_label("instance", "test instance")


def tops(samples, name, key):
    return [(lb[key], int(v)) for n, lb, v, _ in samples if n == name]


def json_tops(arr):
    return [(e["name"], e["estimate"]) for e in arr]


def test_prometheus_matches_window_json():
    j, txt = run(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), "192.168.0.0/24")
    s, heads = parse(txt)
    val = {n: v for n, lb, v, _ in s if not ({"quantile", "ipv4", "ipv6", "qname", "port", "rcode", "qtype", "le"} & set(lb))}
    p, d = j["packets"], j["dns"]
    # label text: static labels first, then the added ones in key order
    assert all(raw.startswith('instance="test instance",') for _, _, _, raw in s)
    assert f'packets_udp{{instance="test instance",policy="default"}} {p["udp"]}' in txt.splitlines()
    for k in ("udp", "tcp", "other_l4", "ipv4", "ipv6", "in", "out", "unknown_dir", "total", "filtered", "events",
              "deep_samples"):
        assert int(val["packets_" + k]) == p[k], k
    assert int(val["packets_protocol_tcp_syn"]) == p["protocol"]["tcp"]["syn"]
    assert int(val["packets_cardinality_src_ips_in"]) == p["cardinality"]["src_ips_in"]
    assert int(val["packets_cardinality_dst_ips_out"]) == p["cardinality"]["dst_ips_out"]
    assert tops(s, "packets_top_ipv4", "ipv4") == json_tops(p["top_ipv4"])
    q = {lb["quantile"]: int(v) for n, lb, v, _ in s if n == "packets_payload_size"}
    assert q == {"0.5": p["payload_size"]["p50"], "0.9": p["payload_size"]["p90"], "0.95": p["payload_size"]["p95"],
                 "0.99": p["payload_size"]["p99"]}
    assert heads["packets_payload_size"] == "summary"
    assert int(val["packets_payload_size_count"]) == p["deep_samples"]
    assert int(val["packets_payload_size_sum"]) >= p["payload_size"]["p99"]  # the max item
    w = d["wire_packets"]
    for k in ("queries", "replies", "tcp", "udp", "ipv4", "ipv6", "nxdomain", "refused", "srvfail", "noerror", "nodata",
              "total", "filtered", "events", "deep_samples"):
        assert int(val["dns_wire_packets_" + k]) == w[k], k
    assert int(val["dns_cardinality_qname"]) == d["cardinality"]["qname"]
    assert int(val["dns_xact_counts_total"]) == d["xact"]["counts"]["total"]
    assert int(val["dns_xact_in_total"]) == d["xact"]["in"]["total"]
    assert int(val["dns_xact_out_total"]) == d["xact"]["out"]["total"]
    for side in ("in", "out"):
        if "quantiles_us" in d["xact"][side]:
            qq = {lb["quantile"]: int(v) for n, lb, v, _ in s if n == f"dns_xact_{side}_quantiles_us"}
            ref = d["xact"][side]["quantiles_us"]
            assert qq == {"0.5": ref["p50"], "0.9": ref["p90"], "0.95": ref["p95"], "0.99": ref["p99"]}
    assert tops(s, "dns_top_udp_ports", "port") == [(int(a), b) for a, b in json_tops(d["top_udp_ports"])] or \
        tops(s, "dns_top_udp_ports", "port") == json_tops(d["top_udp_ports"])
    for m in ("qname2", "qname3", "nxdomain", "refused", "srvfail", "nodata"):
        assert tops(s, "dns_top_" + m, "qname") == json_tops(d["top_" + m]), m
    assert tops(s, "dns_top_rcode", "rcode") == json_tops(d["top_rcode"])
    assert tops(s, "dns_top_qtype", "qtype") == json_tops(d["top_qtype"])
    # the handlers' metric order
    order = [n for n in dict.fromkeys(n for n, _, _, _ in s)]
    assert order.index("packets_events") < order.index("packets_udp") < order.index("packets_payload_size")
    assert order.index("dns_wire_packets_events") < order.index("dns_wire_packets_queries") < order.index("dns_top_qtype")
    assert heads["dns_top_qname2"] == "gauge"
    assert "# HELP dns_top_qname2 Top QNAMES, aggregated at a depth of two labels" in txt


def test_prometheus_histograms_and_ratio():
    j, txt = run(os.path.join(GOLD, "dns_ipv4_udp.pcap"), "192.168.0.0/24",
                 dns_config={"enable": ["histograms"]})
    s, heads = parse(txt)
    d = j["dns"]["xact"]
    for side in ("in", "out"):
        if "histogram_us" not in d[side]:
            continue
        name = f"dns_xact_{side}_histogram_us"
        assert heads[name] == "histogram"
        b = {lb["le"]: float(v) for n, lb, v, _ in s if n == name + "_bucket"}
        assert b == {k: float(v) for k, v in d[side]["histogram_us"]["buckets"].items()}
        cnt = [int(v) for n, _, v, _ in s if n == name + "_count"]
        assert cnt == [int(d[side]["histogram_us"]["buckets"]["+Inf"])]
        # le sorts between instance and policy
        assert any(re.search(r'\{instance="test instance",le="[^"]+",policy="default"\}', raw and "{" + raw + "}")
                   for n, _, _, raw in s if n == name + "_bucket")
    if "ratio" in d:
        qq = {lb["quantile"]: float(v) for n, lb, v, _ in s if n == "dns_xact_ratio_quantiles"}
        ref = d["ratio"]["quantiles"]
        for k, jk in (("0.5", "p50"), ("0.9", "p90"), ("0.95", "p95"), ("0.99", "p99")):
            assert qq[k] == pytest.approx(ref[jk], rel=1e-5)  # ostream precision 6, as the reference prints


def test_prometheus_groups_and_errors():
    path = os.path.join(GOLD, "dns_ipv4_udp.pcap")
    _, txt = run(path, "192.168.0.0/24", dns_config={"disable": ["all"]})
    assert "dns_" not in txt and "packets_udp" in txt  # a handler with no group enabled writes nothing
    linktype, ts_nano, recs = pa.read_pcap(path)
    h = pa.PvHandlers(host_spec="192.168.0.0/24", num_periods=2, linktype=linktype, ts_nano=ts_nano, max_records=1024)
    try:
        h.process_host(recs)
        with pytest.raises(pa.PvError, match=r"invalid metrics period, specify \[0, 1\]"):
            h.window_prometheus(2)
    finally:
        h.close()


def test_prometheus_per_handler():
    """each plugin alias renders only its own schema key (one StreamHandler per alias)"""
    path = os.path.join(GOLD, "dns_ipv4_udp.pcap")
    linktype, ts_nano, recs = pa.read_pcap(path)
    h = pa.PvHandlers(host_spec="192.168.0.0/24", num_periods=1, linktype=linktype, ts_nano=ts_nano, max_records=1024)
    try:
        h.process_host(recs)
        both = h.window_prometheus(0, {"policy": "p"})
        net = h.window_prometheus(0, {"policy": "p"}, handlers="net")
        dns = h.window_prometheus(0, {"policy": "p"}, handlers="dns")
        assert net and dns and net + dns == both
        def names(txt):
            return [ln.split(" ")[2] if ln.startswith("#") else ln.split("{")[0] for ln in txt.splitlines()]
        assert names(net) and all(x.startswith("packets_") for x in names(net))
        assert names(dns) and all(x.startswith("dns_") for x in names(dns))
    finally:
        h.close()
