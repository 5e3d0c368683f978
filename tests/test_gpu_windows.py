"""Independent Net and DNS windows (each manager shifts on the first of its own events at or
after its next_shift, src/AbstractMetricsManager.h:318-333) on the GPU path against the
oracle, bit-exact: sparse DNS around the 60 s marks, input predicates that make most DNS
packets non-events, more shifts in one batch than a device span holds, small batches, and
contiguous shards merged across ranks under the global period plan."""
import json

import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.dist_launch import run_ranks
from tests.test_gpu_filters import oracle_kw
from tests.test_gpu_parity import diff

pytestmark = pytest.mark.gpu


def run_both(oracle, pcap, periods, tmp_path, f=None, host=synth.HOST_SPEC):
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host, periods=periods, dns_filters=f)
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods, **(oracle_kw(f) if f else {}))
    return gpu, ref


def dns_start(j, key):
    return j[key]["dns"]["period"]["start_ts"], j[key]["packets"]["period"]["start_ts"]


@pytest.mark.parametrize("periods", [2, 5])
@pytest.mark.parametrize("f", [None, {"only_rcode": ["nxdomain", "refused"]}, {"only_queries": True},
                               {"only_qtype": ["AAAA"]}], ids=["plain", "rcode_pred", "only_queries", "qtype"])
def test_sparse_dns_boundaries(oracle, tmp_path, periods, f):
    pcap = synth.sparse_dns_pcap()
    gpu, ref = run_both(oracle, pcap, periods, tmp_path, f)
    assert diff(gpu, ref) is None, diff(gpu, ref)
    key = f"{periods}m"
    d, n = dns_start(ref, key)
    assert d != n, "the DNS window must start at its own boundary in this capture"


def test_only_qname_predicate_boundaries(oracle, tmp_path):
    """only_qname's predicate: a DNS packet with another name is no event and never shifts"""
    pcap = synth.sparse_dns_pcap(quiet=(50, 5))
    full = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=1, window=1)["1m"]["dns"]
    names = [e["name"] for e in full["top_nxdomain"][:3]]
    gpu, ref = run_both(oracle, pcap, 5, tmp_path, {"only_qname": names})
    assert ref["5m"]["dns"]["wire_packets"]["total"] > 0
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("periods", [5, 10])
def test_more_shifts_than_a_span(oracle, tmp_path, periods):
    """60k records x 12 ms = 720 s: 11 shifts of each manager in one batch (device spans of 6)"""
    pcap = synth.pcap_bytes(4, 60000, ts_step_us=12000)
    gpu, ref = run_both(oracle, pcap, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_sparse_dns_small_chunks(oracle, tmp_path, monkeypatch):
    """the host-memory pipeline over 1 MiB chunks: DNS shifts decided in chunks that hold no
    Net shift, and Net shifts in chunks without DNS"""
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "1")
    pcap = synth.sparse_dns_pcap(n=80000, ts_step_us=4000)
    gpu, ref = run_both(oracle, pcap, 5, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_dns_event_seconds_host():
    """pv_dns_event_seconds_host lists exactly the seconds holding a UDP DNS packet"""
    pcap = synth.sparse_dns_pcap(n=20000, ts_step_us=5000)
    want = []
    for s, _, r in synth.records_of(pcap):
        if synth.is_udp_dns(r) and (not want or want[-1] != s):
            want.append(s)
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=5, max_records=1 << 16)
    try:
        assert h.dns_event_seconds_host(pcap[24:]) == want
    finally:
        h.close()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", ["c4_300s", "sparse_dns"])
def test_sharded_multi_period_merge(oracle, tmp_path, world, case):
    """W ranks, contiguous shards of a capture spanning several 60 s marks, periods=5: rank 0's
    merged 5m window equals the oracle's single pass"""
    pcap = synth.pcap_bytes(4, 120000, ts_step_us=2500) if case == "c4_300s" else synth.sparse_dns_pcap()
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    out = tmp_path / "out.json"
    run_ranks(world, ["gpu", str(p), str(out), synth.HOST_SPEC, "5"])
    gpu = json.load(open(out))
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5)
    # top_slow included: the ranks' candidates are judged against the whole stream's p90 of the
    # bucket that closed at each DNS shift (pv_slow_finish)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_sharded_world8_c4_tcp(oracle, tmp_path):
    """8 ranks (sharing the GPU) over C4 traffic mixed with DNS-over-TCP connections, 300 s,
    periods=5: shard cuts no TCP flow spans (pv_shard_cuts), UDP transactions crossing every
    shard edge carried rank by rank (pv_edge_carry), top_slow against the whole stream's p90s,
    TCP messages in the global DNS period plan; rank 0's merged window equals the oracle's
    single pass, every key included"""
    pcap = synth.c4_tcp_pcap()
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    out = tmp_path / "out.json"
    run_ranks(8, ["gpu", str(p), str(out), synth.HOST_SPEC, "5"], timeout=400)
    gpu = json.load(open(out))
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5)
    d = ref["5m"]["dns"]
    assert d["wire_packets"]["tcp"] > 0 and d["xact"]["counts"]["total"] > 0
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("rate,f", [(40, None), (75, {"only_qtype": ["A", "AAAA"]})], ids=["plain", "qtype"])
def test_sharded_deep_sampling(oracle, tmp_path, rate, f):
    """3 ranks, deep_sample_rate < 100, C4 traffic with DNS over TCP: each rank steps its
    managers' generators past the earlier shards' draws (pv_sample_skip; the DNS draws counted
    by the planning prescan, filtered events excluded), so the merged window equals the single pass"""
    from tests.test_gpu_filters import oracle_kw
    pcap = synth.c4_tcp_pcap(n=60000, ts_step_us=2500, flows=150)
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    out = tmp_path / "out.json"
    run_ranks(3, ["gpu", str(p), str(out), synth.HOST_SPEC, "5", str(rate)] + ([json.dumps(f)] if f else []))
    gpu = json.load(open(out))
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5, deep_sample_rate=rate,
                           **(oracle_kw(f) if f else {}))
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("budget_mb", [None, "1"], ids=["grow", "drain"])
def test_value_buffer_small_batches(oracle, tmp_path, monkeypatch, budget_mb):
    """Many small batches of query/response pairs across DNS period shifts: the transaction value
    buffer keeps two values of room per record of a batch (growing in HBM, or draining to the host
    when PV_XV_BUDGET_MB caps it) and the shift thresholds select over it; windows equal the
    oracle's (a response-heavy batch must never run past the buffer)"""
    if budget_mb:
        monkeypatch.setenv("PV_XV_BUDGET_MB", budget_mb)
    pcap = synth.pcap_bytes(4, 40000, ts_step_us=5000)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=5, max_records=1024)
    try:
        h.process_host(recs)
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        got = {"5m": h.window_json(5, merged=True)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5)
    assert diff(got, ref) is None, diff(got, ref)


def _jittered(pcap, frac=0.1, back=3, seed=5):
    """the capture with a fraction of its records stamped up to `back` seconds earlier (timestamps
    out of order around every minute mark, as real captures have them)"""
    import struct
    import numpy as np
    rng = np.random.default_rng(seed)
    out = []
    for s, u, r in synth.records_of(pcap):
        if rng.random() < frac:
            r = struct.pack("<I", s - int(rng.integers(1, back + 1))) + r[4:]
        out.append(r)
    return pa.pcap_file_bytes(b"".join(out))


@pytest.mark.parametrize("periods", [2, 5])
def test_non_monotone_timestamps_across_shifts(oracle, tmp_path, periods):
    """period shifts inside batches whose timestamps go back: each manager shifts on the first event
    (in stream order) at or past its next shift second, and every later event belongs to the new
    period whatever its stamp (AbstractMetricsManager::new_event); was refused before round 5"""
    pcap = _jittered(synth.pcap_bytes(4, 60000, ts_step_us=5000))
    gpu, ref = run_both(oracle, pcap, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_non_monotone_small_chunks(oracle, tmp_path, monkeypatch):
    """the same over 1 MiB ingest batches, with DNS over TCP in the stream"""
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "1")
    pcap = _jittered(synth.c4_tcp_pcap(n=60000, ts_step_us=5000, flows=100), frac=0.05)
    gpu, ref = run_both(oracle, pcap, 5, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)
