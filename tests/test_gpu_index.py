"""The record index on the device (pv_index.hip) against the sequential walk
(pv_index_records, the PcapInputStream::_open_pcap record loop,
src/inputs/pcap/PcapInputStream.cpp:471-527), on the blobs built to defeat start guesses
(tests/test_index_parallel.py), the fixtures and the bench shapes; and the host-memory
ingest with the device index against the host walk, end to end."""
import os

import numpy as np
import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.test_gpu_parity import GOLD, diff
from tests.test_index_parallel import blob

pytestmark = pytest.mark.gpu


def check(h, b, max_records=None):
    a = pa.RecordIndex(b, max_records=max_records) if max_records else pa.RecordIndex(b)
    offs, sci, scs, info = h.index_device(b, max_records=max_records)
    for f in ("n_records", "bytes_used", "first_sec", "first_nsec", "last_sec", "last_nsec", "monotone",
              "n_sec_changes"):
        assert getattr(a.info, f) == getattr(info, f), f
    assert np.array_equal(a.offsets, offs)
    k = a.info.n_sec_changes
    assert np.array_equal(a.sc_idx[:k], sci[:k]) and np.array_equal(a.sc_sec[:k], scs[:k])


@pytest.fixture(scope="module")
def handler():
    # the chunk (and so the largest block) is sized when the ingest staging is first used
    old = os.environ.get("PV_INGEST_CHUNK_MB")
    os.environ["PV_INGEST_CHUNK_MB"] = "256"
    h = pa.PvHandlers(num_periods=1, max_records=1 << 24)
    h.index_device(b"")  # sizes the staging now
    if old is None:
        del os.environ["PV_INGEST_CHUNK_MB"]
    else:
        os.environ["PV_INGEST_CHUNK_MB"] = old
    yield h
    h.close()


@pytest.mark.parametrize("kind,n", [("small", 120_000), ("mixed", 4_000), ("adv", 1_500)])
def test_device_index_matches_sequential(handler, kind, n):
    rng = np.random.default_rng(hash(kind) & 0xffff)
    b = blob(rng, n, kind)
    check(handler, b)
    check(handler, b[: len(b) - 7])      # truncated tail record
    check(handler, b, max_records=n // 3)  # record cap


@pytest.mark.parametrize("fixture", ["dns_udp_tcp_random.pcap", "dns_ipv6_tcp.pcap", "ecs.pcap"])
def test_device_index_fixtures(handler, fixture):
    check(handler, open(os.path.join(GOLD, fixture), "rb").read()[24:])


@pytest.mark.parametrize("cfg,n", [(2, 1_000_000), (3, 300_000), (4, 200_000)])
def test_device_index_bench_shapes(handler, cfg, n):
    check(handler, synth.pcap_bytes(cfg, n)[24:])


@pytest.mark.parametrize("chunk_mb,ring", [("1", "4"), ("3", "4"), ("1", "3"), ("1", "8")])
def test_ingest_device_index_parity(oracle, monkeypatch, chunk_mb, ring):
    """pv_process_host with the device index (small chunks: many cuts at ts_sec boundaries;
    ring depths 3..8: the producer 1..6 pieces ahead) equals the oracle's single pass"""
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", chunk_mb)
    monkeypatch.setenv("PV_INGEST_RING", ring)
    pcap = synth.pcap_bytes(4, 300_000, ts_step_us=700)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=5, max_records=1 << 20)
    try:
        h.process_host(recs)
        h.set_end_tstamp(*pa.last_record_ts(recs, idx))
        gpu = {"5m": h.window_json(5, merged=True)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_ingest_reset_reuses_ring(oracle, monkeypatch):
    """One context, pv_reset between two passes of the same stream (bench --config 5's steps): the
    ingest ring, index state and device tables carry over, the window restarts; both passes equal
    the oracle's single pass"""
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "1")
    monkeypatch.setenv("PV_INGEST_RING", "6")
    pcap = synth.pcap_bytes(4, 200_000, ts_step_us=700)
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5)
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=5, max_records=1 << 20)
    try:
        for _ in range(2):
            h.reset()
            h.process_host(recs)
            h.set_end_tstamp(*pa.last_record_ts(recs, idx))
            gpu = {"5m": h.window_json(5, merged=True)}
            assert diff(gpu, ref) is None, diff(gpu, ref)
    finally:
        h.close()
