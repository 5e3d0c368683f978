"""The handler surface beyond window_json(period, merged) (StreamMetricsHandler,
src/StreamHandler.h:221-269), on the GPU path against the oracle's restatement:

- heartbeats: pv_check_period_shift, the input's heartbeat_signal -> check_period_shift in both
  handlers (src/AbstractMetricsManager.h:462-470; net/v1/NetStreamHandler.cpp:99-102,
  dns/v1/DnsStreamHandler.cpp:219-222), DNS on_period_shift purge and slow thresholds included
  (dns/v1/DnsStreamHandler.h:252-267);
- external buckets: pv_bucket_merge / pv_bucket_json, a policy folding like handlers across taps
  (Policy::_get_merged_buckets, src/Policies.cpp:420-446; simple_merge / multiple_merge with
  Aggregate::SUM, src/AbstractMetricsManager.h:649-706, src/Metrics.h:356-372);
- window_prometheus's period choice (period 1 once a manager holds more than one bucket)."""
import os
import struct

import pytest

import pktvisor_amd as pa
from tests.test_gpu_parity import diff

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
HOST = "192.168.0.0/24"


def records(pcap: bytes):
    p, out = 24, []
    while p + 16 <= len(pcap):
        s, us, cl, ol = struct.unpack_from("<IIII", pcap, p)
        out.append([s, us, cl, ol, pcap[p + 16:p + 16 + cl]])
        p += 16 + cl
    return out


def rec_bytes(rs):
    return b"".join(struct.pack("<IIII", s, us, cl, ol) + d for s, us, cl, ol, d in rs)


def shifted(rs, dsec, drop_every=0):
    """records moved by dsec seconds; drop_every: every k-th DNS response removed (open queries)"""
    out = []
    for k, (s, us, cl, ol, d) in enumerate(rs):
        if drop_every and k % drop_every == 0 and len(d) > 44 and d[23] == 17 and d[34:36] == b"\x00\x35":
            continue  # a response from port 53
        out.append([s + dsec, us, cl, ol, d])
    return out


def heartbeat_case():
    pcap = open(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), "rb").read()
    hdr, rs = pcap[:24], records(pcap)
    t0 = rs[0][0]
    a, b, c = rs, shifted(rs, 100, drop_every=3), shifted(rs, 250)
    return hdr, t0, a, b, c


def run_gpu(hdr, parts, beats, periods=5, **kw):
    h = pa.PvHandlers(host_spec=HOST, num_periods=periods, max_records=1 << 16, **kw)
    try:
        last = None
        for recs, beat in zip(parts, beats):
            h.process_host(rec_bytes(recs))
            last = recs[-1]
            for t in beat:
                h.check_period_shift(t, 0)
        h.set_end_tstamp(last[0], last[1] * 1000)
        out = {"5m": h.window_json(5, merged=True)}
        for k in range(5):
            try:
                out[f"p{k}"] = h.window_json(k)
            except pa.PvError as e:  # fewer periods than the window holds
                assert "not yet accumulated" in str(e)
                break
        return out
    finally:
        h.close()


def test_heartbeat_rotates_both_windows(oracle):
    hdr, t0, a, b, c = heartbeat_case()
    beats = [t0 + 70, t0 + 200]
    gpu = run_gpu(hdr, [a, b, c], [[beats[0]], [beats[1]], []])
    full = hdr + rec_bytes(a + b + c)
    hb = ",".join(str(x) for x in beats)
    ref = oracle.run_bytes(full, host_spec=HOST, num_periods=5, window=5, heartbeats=hb)
    assert diff(gpu["5m"], ref["5m"]) is None, diff(gpu["5m"], ref["5m"])
    for k in range(5):
        r = oracle.run_bytes(full, host_spec=HOST, num_periods=5, window=5, heartbeats=hb, single=k)
        assert diff(gpu[f"p{k}"], r[f"p{k}"]) is None, (k, diff(gpu[f"p{k}"], r[f"p{k}"]))
    # five buckets: [t0, +70) closed by the first heartbeat, a data-driven shift in capture B
    # (+131), the second heartbeat (+200), a data-driven shift in capture C (+265); the second
    # heartbeat timed capture B's unanswered queries out into the bucket it opened
    starts = [gpu[f"p{k}"]["packets"]["period"]["start_ts"] - t0 for k in range(5)]
    assert starts == [265, 200, 131, 70, 0], starts
    assert gpu["p1"]["dns"]["xact"]["counts"]["timed_out"] > 0
    # without the heartbeats the windows differ (the shifts then come from the packets alone)
    plain = run_gpu(hdr, [a, b, c], [[], [], []])
    assert [plain[f"p{k}"]["packets"]["period"]["start_ts"] - t0 for k in range(5) if f"p{k}" in plain] != starts


def test_heartbeat_before_next_shift_and_before_start(oracle):
    hdr, t0, a, b, c = heartbeat_case()
    h = pa.PvHandlers(host_spec=HOST, num_periods=5, max_records=1 << 16)
    try:
        h.check_period_shift(t0 + 1000)  # no record yet: ignored
        h.process_host(rec_bytes(a))
        h.check_period_shift(t0 + 59)   # next shift is t0 + 60
        with pytest.raises(pa.PvError, match="requested metrics period has not yet accumulated"):
            h.window_json(1)
        h.check_period_shift(t0 + 60)
        assert h.window_json(0)["packets"]["period"]["start_ts"] == t0 + 60
    finally:
        h.close()
    h1 = pa.PvHandlers(host_spec=HOST, num_periods=1, max_records=1 << 16)
    try:
        h1.process_host(rec_bytes(a))
        h1.check_period_shift(t0 + 1000)  # num_periods 1: no shifting
        assert h1.window_json(0)["packets"]["period"]["start_ts"] == t0
    finally:
        h1.close()


def _ctx(recs, periods=5, beats=()):
    h = pa.PvHandlers(host_spec=HOST, num_periods=periods, max_records=1 << 16)
    h.process_host(rec_bytes(recs))
    for t in beats:
        h.check_period_shift(t)
    h.set_end_tstamp(recs[-1][0], recs[-1][1] * 1000)
    return h


CAPS = ["dns_udp_mixed_rcode.pcap", "dns_udp_tcp_random.pcap", "dns_ipv4_udp.pcap"]


@pytest.mark.parametrize("period,merged,prometheus", [(0, False, False), (2, True, False), (0, False, True),
                                                      (1, False, False)])
def test_policy_bucket_merge(oracle, period, merged, prometheus):
    """two or three handlers' buckets folded through pv_bucket_merge == the oracle's policy merge"""
    pcaps = [open(os.path.join(GOLD, f), "rb").read() for f in CAPS]
    # the first capture crosses a period mark (two buckets), the others stay in one
    parts = [records(p) for p in pcaps]
    parts[0] = parts[0] + shifted(parts[0], 70)
    files = [pcaps[0][:24] + rec_bytes(parts[0])] + pcaps[1:]
    ctxs = [_ctx(r) for r in parts]
    try:
        if period >= 1 and not merged and not prometheus:
            # bucket 1 exists only in the first context: the others raise the reference's PeriodException
            b = ctxs[0].merge("dns", None, period)
            with pytest.raises(pa.PvError, match="requested metrics period has not yet accumulated"):
                ctxs[1].merge("dns", b, period)
            return
        for handler, key in (("net", "packets"), ("dns", "dns")):
            b = None
            for h in ctxs:
                b = h.merge(handler, b, period, prometheus=prometheus, merged=merged)
            got = ctxs[0].bucket_json(b)
            ref = oracle.run_policy(files, period=period, merged=merged, prometheus=prometheus, host_spec=HOST,
                                    num_periods=5)
            assert diff(got[key], ref[key]) is None, (handler, diff(got[key], ref[key]))
            # a Prometheus / OpenTelemetry rendering of the same bucket
            txt = ctxs[0].bucket_prometheus(b, {"policy": "p", "handler": key + "_merged"})
            assert txt and ('handler="' + key + '_merged"') in txt
            assert len(ctxs[0].bucket_opentelemetry(b, {"policy": "p"})) > 0
            b.free()
    finally:
        for h in ctxs:
            h.close()


V2_ALL = ["cardinality", "counters", "quantiles", "top_ecs", "top_qtypes", "top_rcodes", "top_size", "top_qnames",
          "top_ports", "xact_times"]


def _ctx2(recs, periods=5):
    h = pa.PvHandlers(host_spec=HOST, num_periods=periods, max_records=1 << 16, net2_config={},
                      dns2_config={"enable": V2_ALL})
    h.process_host(rec_bytes(recs))
    h.set_end_tstamp(recs[-1][0], recs[-1][1] * 1000)
    return h


@pytest.mark.parametrize("period,merged,prometheus", [(0, False, False), (2, True, False), (0, False, True)])
def test_policy_bucket_merge_v2(oracle, period, merged, prometheus):
    """the v2 handlers' buckets (Net v2 "net", DNS v2 "dns") folded through pv_bucket_merge == the
    oracle's policy merge (net/v2 ...cpp:286-331, dns/v2 ...cpp:619-676: per direction, quantiles
    by the SUM rule, the xact time histogram merging)"""
    pcaps = [open(os.path.join(GOLD, f), "rb").read() for f in CAPS]
    parts = [records(p) for p in pcaps]
    parts[0] = parts[0] + shifted(parts[0], 70)
    files = [pcaps[0][:24] + rec_bytes(parts[0])] + pcaps[1:]
    ctxs = [_ctx2(r) for r in parts]
    try:
        ref = oracle.run_policy(files, period=period, merged=merged, prometheus=prometheus, host_spec=HOST,
                                num_periods=5, net2_groups=31, dns2_groups=0x3ff)
        for handler, key in (("net", "net"), ("dns", "dns")):
            b = None
            for h in ctxs:
                b = h.merge(handler, b, period, prometheus=prometheus, merged=merged)
            got = ctxs[0].bucket_json(b)
            assert diff(got[key], ref[key]) is None, (handler, diff(got[key], ref[key]))
            txt = ctxs[0].bucket_prometheus(b, {"policy": "p"})
            assert txt and ("net_" if key == "net" else "dns_xacts") in txt
            assert len(ctxs[0].bucket_opentelemetry(b, {"policy": "p"})) > 0
            b.free()
    finally:
        for h in ctxs:
            h.close()


def test_bucket_merge_quantile_sum(oracle):
    """Aggregate::SUM: quantiles of a merged bucket are the p-wise sums (Quantile::merge)"""
    pcaps = [open(os.path.join(GOLD, f), "rb").read() for f in CAPS[:2]]
    ctxs = [_ctx(records(p)) for p in pcaps]
    try:
        singles = [h.window_json(0) for h in ctxs]
        b = None
        for h in ctxs:
            b = h.merge("dns", b, 0)
        got = ctxs[0].bucket_json(b)["dns"]["xact"]
        for side in ("in", "out"):
            q = [s["dns"]["xact"][side].get("quantiles_us") for s in singles]
            if q[0] and q[1]:
                assert got[side]["quantiles_us"] == {k: q[0][k] + q[1][k] for k in q[0]}
        b.free()
    finally:
        for h in ctxs:
            h.close()


def test_prometheus_period_auto():
    """window_prometheus reads bucket 1 once the manager holds more than one (StreamHandler.h:226-233)"""
    hdr, t0, a, b, c = heartbeat_case()
    h = pa.PvHandlers(host_spec=HOST, num_periods=5, max_records=1 << 16)
    try:
        h.process_host(rec_bytes(a))
        assert h.window_prometheus(pa.PV_PERIOD_AUTO) == h.window_prometheus(0)
        h.check_period_shift(t0 + 70)
        h.process_host(rec_bytes(b))
        auto = h.window_prometheus(pa.PV_PERIOD_AUTO)
        assert auto == h.window_prometheus(1) and auto != h.window_prometheus(0)
        assert h.window_opentelemetry(pa.PV_PERIOD_AUTO) == h.window_opentelemetry(1)
    finally:
        h.close()
