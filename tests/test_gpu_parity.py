"""GPU parity: the HIP path (through the C-ABI) against the oracle on the same inputs.

Bit-exact for everything emitted: counters, dense tables, top-N (exact counts,
ties ordered by name), CPC estimates (exact HIP/ICON replay), quantiles (exact
KLL rank rule). Rates are not emitted by either side (wall-clock driven)."""
import json
import os

import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

FIXTURES = [("dns_ipv4_udp.pcap", ""), ("dns_ipv6_udp.pcap", ""), ("dns_udp_tcp_random.pcap", "192.168.0.0/24"),
            ("dns_udp_mixed_rcode.pcap", "192.168.0.0/24"), ("dnssec.pcap", ""), ("ecs.pcap", ""),
            ("dns_ipv4_tcp.pcap", ""), ("dns_ipv6_tcp.pcap", "")]


def diff(a, b, path=""):
    """first differing path between two JSON values (for readable failures)"""
    if type(a) != type(b):
        return f"{path}: {a!r} != {b!r}"
    if isinstance(a, dict):
        for k in sorted(set(a) | set(b)):
            if k not in a or k not in b:
                return f"{path}.{k}: missing on {'gpu' if k not in a else 'oracle'}"
            d = diff(a[k], b[k], f"{path}.{k}")
            if d:
                return d
        return None
    if isinstance(a, list):
        if len(a) != len(b):
            return f"{path}: len {len(a)} != {len(b)}: {json.dumps(a)[:300]} vs {json.dumps(b)[:300]}"
        for i, (x, y) in enumerate(zip(a, b)):
            d = diff(x, y, f"{path}[{i}]")
            if d:
                return d
        return None
    return None if a == b else f"{path}: {a!r} != {b!r}"


def run_both(oracle, pcap: bytes, host: str, periods: int, tmp_path, **kw):
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host or None, periods=periods, **kw)
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods)
    return gpu, ref


@pytest.mark.parametrize("periods", [1, 5])
@pytest.mark.parametrize("fixture,host", FIXTURES, ids=[f[0] for f in FIXTURES])
def test_fixture_parity(oracle, tmp_path, fixture, host, periods):
    pcap = open(os.path.join(GOLD, fixture), "rb").read()
    gpu, ref = run_both(oracle, pcap, host, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("cfg,n,host", [(1, 1000, synth.HOST_SPEC), (2, 60000, synth.HOST_SPEC),
                                        (3, 60000, synth.HOST_SPEC), (4, 60000, synth.HOST_SPEC),
                                        (9, 60000, "10.0.0.0/8,2000::/3,192.168.0.0/16")])
@pytest.mark.parametrize("periods", [1, 5])
def test_synthetic_parity(oracle, tmp_path, cfg, n, host, periods):
    gpu, ref = run_both(oracle, synth.pcap_bytes(cfg, n), host, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("periods", [2, 3, 5])
def test_multi_period_parity(oracle, tmp_path, periods):
    # 120k records x 1.5 ms = 180 s: three period shifts inside one batch
    gpu, ref = run_both(oracle, synth.pcap_bytes(4, 120000, ts_step_us=1500), synth.HOST_SPEC, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_edge_mix_many_seeds(oracle, tmp_path):
    for seed in range(5):
        gpu, ref = run_both(oracle, synth.pcap_bytes(9, 20000, seed=1000 + seed), "10.0.0.0/8,2000::/3", 1, tmp_path)
        assert diff(gpu, ref) is None, (seed, diff(gpu, ref))


def test_large_c4_against_oracle(oracle, tmp_path):
    gpu, ref = run_both(oracle, synth.pcap_bytes(4, 1_000_000), synth.HOST_SPEC, 5, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("periods", [1, 5])
def test_chunked_ingest_parity(oracle, tmp_path, monkeypatch, periods):
    """pv_process_host's pipeline over 1 MiB chunks (many chunks, a period shift and DNS
    transactions straddling chunk edges) against the oracle's single pass."""
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "1")
    monkeypatch.setenv("PV_HOST_THREADS", "7")
    gpu, ref = run_both(oracle, synth.pcap_bytes(4, 60000, ts_step_us=1500), synth.HOST_SPEC, periods, tmp_path)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_registered_host_buffer_same_result(tmp_path, monkeypatch):
    """A page-locked source (pv_host_register: H2D straight from the caller's buffer)
    gives the same windows as pageable staging."""
    import numpy as np
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "2")
    recs = np.frombuffer(synth.pcap_bytes(4, 40000)[24:], dtype=np.uint8).copy()
    out = []
    for reg in (False, True):
        h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=1, max_records=len(recs) // 16)
        lib = pa.load_library()
        if reg:
            assert lib.pv_host_register(recs.ctypes.data, recs.nbytes) == 0
        try:
            h.process_host(recs)
            out.append(h.window_json(0, merged=False))
        finally:
            if reg:
                lib.pv_host_unregister(recs.ctypes.data)
            h.close()
    assert diff(out[1], out[0]) is None, diff(out[1], out[0])


@pytest.mark.parametrize("cfg,n,step_us,xv_budget", [(1, 1000, 1, None), (4, 20000, 9000, None), (4, 20000, 9000, "0")])
def test_many_small_batches_parity(oracle, monkeypatch, cfg, n, step_us, xv_budget):
    """The same capture submitted as many small batches (1..60 records each): DNS queries
    carried across batch edges (query-only batches defer pairing, later batches pair them;
    with 9 ms steps also TTL purges at period shifts) must give the single-pass result. The
    transaction values outgrow the 2 x max_records device buffer: it doubles in HBM, or with
    PV_XV_BUDGET_MB=0 drains to the host copy."""
    import numpy as np
    if xv_budget is not None:
        monkeypatch.setenv("PV_XV_BUDGET_MB", xv_budget)
    pcap = synth.pcap_bytes(cfg, n, ts_step_us=step_us)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    offs = list(idx.offsets) + [len(recs)]
    rng = np.random.default_rng(cfg)
    # batch edges anywhere, except inside a second at which a period shifts (a window
    # shift at S0 + 60 k; pv_process_host's chunks end at second boundaries for this)
    o = np.asarray(idx.offsets, dtype=np.int64)
    secs = np.frombuffer(recs, dtype=np.uint8)[o[:, None] + np.arange(4)].copy().view("<u4")[:, 0].astype(np.int64)

    def bad(j):
        return 0 < j < idx.n and secs[j] == secs[j - 1] and secs[j] != secs[0] and (secs[j] - secs[0]) % 60 == 0

    for periods in (1, 5):
        h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=periods, max_records=256)
        try:
            i = 0
            while i < idx.n:
                j = min(idx.n, i + int(rng.integers(1, 61)))
                while bad(j) and j > i + 1:
                    j -= 1
                while bad(j):
                    j += 1
                assert j - i <= 256
                h.process_host(recs[offs[i]:offs[j]])
                i = j
            h.set_end_tstamp(*pa.last_record_ts(recs, idx))
            key = f"{1 if periods == 1 else periods}m"
            gpu = {key: h.window_json(0 if periods == 1 else periods, merged=periods != 1)}
        finally:
            h.close()
        ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=periods, window=periods)
        assert diff(gpu, ref) is None, (periods, diff(gpu, ref))
