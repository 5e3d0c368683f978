"""window_opentelemetry on the GPU path (pv_window_opentelemetry).

The library returns the protobuf wire bytes of the ScopeMetrics `metrics` (field 2) the
reference's primitives add (src/Metrics.cpp:22-36,82-96; src/Metrics.h:289-327,450-481,
523-533,693-769) in the handlers' order (the same order as window_prometheus). The
opentelemetry-proto package is not in this image, so the bytes are decoded here with a
plain protobuf wire-format reader against the metrics/v1 field numbers (restated; parity
unpinned beyond the reference's own calls: the reference's test_metrics.cpp only checks
names and data-point kinds, :172-179,241-248,309-320,437-448,537-545).
"""
import os
import struct

import pytest

import pktvisor_amd as pa

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def varint(b, i):
    v = s = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return v, i


def fields(b):
    out, i = [], 0
    while i < len(b):
        k, i = varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = varint(b, i)
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 2:
            n, i = varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise AssertionError(f"wire type {wt}")
        out.append((f, wt, v))
    return out


def attrs(items, field):
    out = []
    for f, _, v in items:
        if f != field:
            continue
        kv = dict((ff, vv) for ff, _, vv in fields(v))
        anyv = dict((ff, vv) for ff, _, vv in fields(kv[2]))
        out.append((kv[1].decode(), anyv.get(1, b"").decode()))
    return out


def u64(v):
    return struct.unpack("<Q", v)[0]


def f64(v):
    return struct.unpack("<d", v)[0]


def decode(buf):
    """[(name, desc, kind, points)]"""
    ms = []
    for f, wt, v in fields(buf):
        assert f == 2 and wt == 2  # ScopeMetrics.metrics
        m = fields(v)
        assert [x[0] for x in m] == sorted(x[0] for x in m)  # protobuf writes fields in number order
        md = {ff: vv for ff, _, vv in m}
        name, desc = md[1].decode(), md[2].decode()
        if 5 in md:
            pts = []
            for ff, _, dp in fields(md[5]):
                d = fields(dp)
                dd = {a: b for a, _, b in d}
                pts.append({"start": u64(dd.get(2, b"\0" * 8)), "time": u64(dd[3]), "int": struct.unpack("<q", dd[6])[0],
                            "attrs": attrs(d, 7)})
            ms.append((name, desc, "gauge", pts))
        elif 11 in md:
            (ff, _, dp), = fields(md[11])
            d = fields(dp)
            q = []
            for a, _, b in d:
                if a == 6:
                    qq = {x: f64(y) for x, _, y in fields(b)}
                    q.append((qq.get(1, 0.0), qq.get(2, 0.0)))
            assert 4 not in {a for a, _, _ in d} and 5 not in {a for a, _, _ in d}  # no count / sum
            ms.append((name, desc, "summary", {"q": q, "attrs": attrs(d, 7)}))
        elif 9 in md:
            h = fields(md[9])
            assert h[-1][0] == 2 and h[-1][2] == 2  # AGGREGATION_TEMPORALITY_CUMULATIVE
            d = fields(h[0][2])
            dd = {a: b for a, _, b in d}
            cnt = [u64(dd[6][k:k + 8]) for k in range(0, len(dd[6]), 8)]
            bnd = [f64(dd[7][k:k + 8]) for k in range(0, len(dd[7]), 8)]
            ms.append((name, desc, "histogram", {"n": u64(dd[4]), "counts": cnt, "bounds": bnd, "attrs": attrs(d, 9)}))
        else:
            ms.append((name, desc, "none", None))
    return ms


def run(path, host_spec, dns_config=None):
    linktype, ts_nano, recs = pa.read_pcap(path)
    idx = pa.RecordIndex(recs, ts_nano)
    h = pa.PvHandlers(host_spec=host_spec, num_periods=1, linktype=linktype, ts_nano=ts_nano,
                      max_records=max(1, idx.n), dns_config=dns_config or {})
    try:
        h.process_host(recs)
        h.set_end_tstamp(*pa.last_record_ts(recs, idx, ts_nano))
        return (h.window_json(0), h.window_prometheus(0, {"policy": "default"}),
                h.window_opentelemetry(0, {"policy": "default"}))
    finally:
        h.close()


def prom_metrics(txt):
    """[(name, help)] in order, from the Prometheus text of the same bucket"""
    return [(ln.split(" ")[2], ln.split(" ", 3)[3]) for ln in txt.splitlines() if ln.startswith("# HELP ")]


def test_otlp_matches_prometheus_and_json():
    j, prom, otlp = run(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), "192.168.0.0/24")
    ms = decode(otlp)
    assert [(n, d) for n, d, _, _ in ms] == prom_metrics(prom)
    byname = {n: (k, p) for n, _, k, p in ms}
    p, d = j["packets"], j["dns"]
    kind, pts = byname["packets_udp"]
    assert kind == "gauge" and len(pts) == 1 and pts[0]["int"] == p["udp"]
    assert pts[0]["attrs"] == [("policy", "default")]  # added labels only, no static labels
    assert pts[0]["start"] // 10**9 == p["period"]["start_ts"] and pts[0]["time"] >= pts[0]["start"]
    assert byname["dns_wire_packets_queries"][1][0]["int"] == d["wire_packets"]["queries"]
    assert byname["dns_cardinality_qname"][1][0]["int"] == d["cardinality"]["qname"]
    top = byname["dns_top_qname2"][1]
    assert [(dict(x["attrs"])["qname"], x["int"]) for x in top] == [(e["name"], e["estimate"]) for e in d["top_qname2"]]
    assert all([k for k, _ in x["attrs"]] == sorted(k for k, _ in x["attrs"]) for x in top)
    ipv4 = byname["packets_top_ipv4"][1]
    assert [(dict(x["attrs"])["ipv4"], x["int"]) for x in ipv4] == [(e["name"], e["estimate"]) for e in p["top_ipv4"]]
    kind, s = byname["packets_payload_size"]
    assert kind == "summary"
    assert s["q"] == [(0.5, p["payload_size"]["p50"]), (0.9, p["payload_size"]["p90"]), (0.95, p["payload_size"]["p95"]),
                      (0.99, p["payload_size"]["p99"])]


def test_otlp_histogram_quirk():
    """bucket_counts = static_cast<uint64_t>(CDF) * n (src/Metrics.h:312-314): n where the CDF
    reached 1, else 0; no +Inf bucket"""
    j, _, otlp = run(os.path.join(GOLD, "dns_ipv4_udp.pcap"), "192.168.0.0/24", dns_config={"enable": ["histograms"]})
    ms = {n: (k, p) for n, _, k, p in decode(otlp)}
    for side in ("in", "out"):
        hj = j["dns"]["xact"][side].get("histogram_us")
        if not hj:
            continue
        kind, h = ms[f"dns_xact_{side}_histogram_us"]
        assert kind == "histogram"
        n = int(hj["buckets"]["+Inf"])
        assert h["n"] == n
        pts = [k for k in hj["buckets"] if k != "+Inf"]
        assert h["bounds"] == [float(k) for k in pts]
        assert h["counts"] == [n if int(hj["buckets"][k]) == n else 0 for k in pts]


def test_otlp_per_handler():
    path = os.path.join(GOLD, "dns_ipv4_udp.pcap")
    linktype, ts_nano, recs = pa.read_pcap(path)
    h = pa.PvHandlers(host_spec="192.168.0.0/24", num_periods=1, linktype=linktype, ts_nano=ts_nano, max_records=1024)
    try:
        h.process_host(recs)
        h.set_end_tstamp(*pa.last_record_ts(recs, pa.RecordIndex(recs, ts_nano), ts_nano))
        both = h.window_opentelemetry(0)
        net = h.window_opentelemetry(0, handlers="net")
        dns = h.window_opentelemetry(0, handlers="dns")
        names = lambda b: [(n, d, k) for n, d, k, _ in decode(b)]  # noqa: E731
        assert names(net) + names(dns) == names(both)
        assert all(n.startswith("packets_") for n, _, _, _ in decode(net))
        assert all(n.startswith("dns_") for n, _, _, _ in decode(dns))
    finally:
        h.close()
