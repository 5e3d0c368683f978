"""b5: reads of a handler while its input thread writes it.

The reference's HTTP threads read buckets under shared locks while the input thread's
packet signals write them (src/AbstractMetricsManager.h:480-504: window_json / merge take
`std::shared_lock` on the manager's bucket mutex; process_* take the unique lock). The C-ABI
serialises each entry point on the context mutex (pv_host.cpp `pv_ctx::mu`), so a read issued
while pv_process_host runs sees the handler at a batch boundary.

The test streams one capture in batches from a producer thread while a reader thread loops
pv_window_json and pv_bucket_merge / pv_bucket_json; every read must equal the window after
some batch boundary (the snapshots of a sequential run, which are pinned to the oracle on the
same record prefixes), and the reads must move forward through the batches."""
import os
import threading

import pytest

import pktvisor_amd as pa
from tests.test_gpu_boundary import rec_bytes, records
from tests.test_gpu_parity import diff

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
HOST = "192.168.0.0/24"


def strip_period(doc):
    """the window without its period stamps (a read may land between a batch and the
    producer's set_end_tstamp)"""
    return {k: {f: v for f, v in d.items() if f != "period"} for k, d in doc.items()}


def batches(rs, k):
    step = (len(rs) + k - 1) // k
    return [rs[i:i + step] for i in range(0, len(rs), step)]


@pytest.mark.parametrize("name", ["dns_udp_tcp_random.pcap", "dns_ipv4_udp.pcap"])
def test_reads_during_process_host(oracle, name):
    pcap = open(os.path.join(GOLD, name), "rb").read()
    hdr, rs = pcap[:24], records(pcap)
    parts = batches(rs, 12)
    mk = lambda: pa.PvHandlers(host_spec=HOST, num_periods=1, max_records=1 << 16)

    # sequential run: the window after every batch (before and after the producer's
    # set_end_tstamp), the latter pinned to the oracle on the record prefix
    snaps, net_snaps = [], []
    h = mk()
    try:
        done = 0
        for part in parts:
            h.process_host(rec_bytes(part))
            done += len(part)
            snaps.append(strip_period(h.window_json(0)))
            b = h.merge("net", None, 0)
            net_snaps.append(strip_period(h.bucket_json(b)))
            b.free()
            h.set_end_tstamp(part[-1][0], part[-1][1] * 1000)
            w = h.window_json(0)
            ref = oracle.run_bytes(hdr + rec_bytes(rs[:done]), host_spec=HOST, num_periods=1, window=1)["1m"]
            assert w == ref, f"batch boundary {len(snaps)}: GPU window differs from the oracle prefix"
            snaps.append(strip_period(w))
            b = h.merge("net", None, 0)
            net_snaps.append(strip_period(h.bucket_json(b)))
            b.free()
    finally:
        h.close()

    # concurrent run: one producer, one reader
    h = mk()
    errors, reads, bucket_reads = [], [], []
    first = threading.Event()
    stop = threading.Event()

    def producer():
        try:
            for j, part in enumerate(parts):
                h.process_host(rec_bytes(part))
                h.set_end_tstamp(part[-1][0], part[-1][1] * 1000)
                if j == 0:
                    first.set()
        except Exception as e:  # noqa: BLE001 - reported by the main thread
            errors.append(("producer", repr(e)))
        finally:
            first.set()
            stop.set()

    def reader():
        first.wait()
        try:
            k = 0
            while not stop.is_set() or k < 3:
                reads.append(strip_period(h.window_json(0)))
                if k % 2 == 0:
                    b = h.merge("net", None, 0)
                    bucket_reads.append(strip_period(h.bucket_json(b)))
                    b.free()
                k += 1
        except Exception as e:  # noqa: BLE001
            errors.append(("reader", repr(e)))

    try:
        ts = [threading.Thread(target=producer), threading.Thread(target=reader)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in ts), "producer or reader hung"
        assert not errors, errors
        assert h.window_json(0) == oracle.run_bytes(pcap, host_spec=HOST, num_periods=1, window=1)["1m"]
    finally:
        h.close()

    assert len(reads) >= 3
    last = 0
    for r in reads:
        hits = [j for j, s in enumerate(snaps) if s == r]
        if not hits:
            for j, sn in enumerate(snaps):
                print("snapshot", j, (diff(sn, r) or "")[:160])
        assert hits, "a concurrent window_json read matches no batch boundary"
        assert max(hits) >= last, "reads went back in the stream"
        last = min(j for j in hits if j >= last)
    last = 0
    for r in bucket_reads:
        hits = [j for j, s in enumerate(net_snaps) if s == r]
        assert hits, "a concurrent bucket merge matches no batch boundary"
        assert max(hits) >= last
        last = min(j for j in hits if j >= last)


def test_read_latency_inside_one_host_block(monkeypatch):
    """a read issued while ONE pv_process_host call works through a large block
    waits for the batch in flight, not for the block: the ingest loop takes the context mutex per
    batch (pv_process_device), so a reader thread sees several intermediate batch boundaries
    inside the call, each read returning within a few batch times"""
    import time
    from pktvisor_amd import synth
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "4")
    pcap = synth.pcap_bytes(4, 400000)
    recs = pcap[24:]
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=1, max_records=1 << 20)
    try:
        t = threading.Thread(target=lambda: h.process_host(recs))
        lat, seen = [], []
        t.start()
        while t.is_alive():
            a = time.perf_counter()
            try:
                w = h.window_json(0)
            except pa.PvError:
                time.sleep(0.002)
                continue  # before the first batch: no data yet
            lat.append(time.perf_counter() - a)
            seen.append(w["packets"]["events"])
            time.sleep(0.002)  # an HTTP poller's pace, not a spin on the context mutex
        t.join()
        final = h.window_json(0)["packets"]["events"]
    finally:
        h.close()
    assert final == 400000
    inside = sorted(set(e for e in seen if 0 < e < final))
    assert len(inside) >= 3, f"reads saw {inside}: no batch boundaries inside the block"
    assert seen == sorted(seen), "reads must move forward through the batches"
    assert max(lat) < 1.0, f"a read waited {max(lat):.3f} s"
