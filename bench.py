#!/usr/bin/env python3
"""Device-resident Mpkt/s of pktvisor's Net+DNS handler path on MI355X.

python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4] [--records R]

One step = one pass of the fused Net v1 + DNS v1 hot path over one batch of
synthetic pcap records already resident in HBM, added to the live window: the parse
kernels (pv_net_kernel, pv_dns_kernel, the top-N merge kernels), DNS transaction pairing
when the batch has DNS, the status read-back. Each rank processes its own shard of R
records per step (weak scaling). For N > 1 the window is read once after the K steps,
inside the timed region, as pktvisord merges its handlers at read time
(src/Policies.cpp:420-446, src/AbstractMetricsManager.h:177-195): merge_window (windows
checked aligned, DNS shard edges, RCCL SUM / MIN all-reduce of the buckets over xGMI,
top-N entries to their region owners) and finalize_window (leading entries + names, exact
distributed quantile selection), reported as `merge`. Rank 0 prints one JSON line. The default workload is BASELINE.json configs[1] (C2: 10M x 64 B
UDP, host_spec 10.0.0.0/8) with both handlers attached, the config the
north-star roofline target is quoted on.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
TIMING_EVERY = 4  # timed steps per stamped Net-pass launch (roofline kernel_ms sample)
NET_WINDOW = 80  # bytes of a record the Net pass reads: 16-B pcap header + 64 B of frame headers
WORKLOADS = {
    2: "C2: Net+DNS handlers, 64 B UDP (Eth+IPv4+UDP+22 B), Zipf IPs, host_spec 10.0.0.0/8",
    3: "C3: Net+DNS handlers, UDP/53 queries, single label L~U[51,63] + EDNS0, mean 128 B",
    4: "C4: Net+DNS handlers, IMIX 70% {64,576,1500} + 30% DNS query/response pairs",
    5: "C5: 100M-record C4-shape stream (1 us/record: crosses 60 s period marks), contiguous shard per rank from "
       "host memory, global period plan, Net+DNS, merge_window (RCCL all-reduce + exchanges)",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(WORKLOADS))
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--stream-records", type=int, default=100_000_000, help="--config 5: records of the whole stream")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--net-groups", type=int, default=0, help="pv_net_group bits (0 = reference defaults)")
    ap.add_argument("--dns-groups", type=int, default=0, help="pv_dns_group bits (0 = reference defaults)")
    ap.add_argument("--read-ceiling", action="store_true", help="also time a plain read of the blob (HBM ceiling)")
    ap.add_argument("--reset-each-step", action="store_true",
                    help="reset the window before every step (rounds 1-5's step; N = 1 only)")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false",
                    help="skip timing the host-memory path (record blob in host RAM -> index -> H2D -> kernels)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.reset_each_step and world > 1:
        raise SystemExit("bench: --reset-each-step is a single-GPU step (the read merges the accumulated window)")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    import pktvisor_amd as pa
    from pktvisor_amd import dist as pvdist
    from pktvisor_amd import synth

    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    if args.config == 5:
        return bench_stream(args, world, rank, local, device)

    # ---- synthetic shard for this rank, then resident in HBM
    n = args.records
    seed = synth.SEEDS[args.config] + 7919 * rank
    buf, offs, used = synth.records(args.config, n, seed=seed, with_offsets=False)
    idx = pa.RecordIndex(buf[:used], max_records=n)
    assert idx.n == n
    d_recs = torch.from_numpy(buf).to(device)  # includes 256 B zero padding
    d_offs = torch.from_numpy(idx.offsets).to(device)
    torch.cuda.synchronize(device)
    algo_bytes = used  # sum over records of (16 + caplen): the step's algorithmic bytes
    # the Net pass's own: the first NET_WINDOW bytes of each record (pcap header + the frame's
    # L2-L4 headers). Payload past them is no part of the Net handler's algorithm (C4's IMIX
    # payloads are read by nothing; a DNS message's by the DNS pass, whose bytes the step counts)
    rec_len = np.diff(np.append(idx.offsets[:n].astype(np.int64), used))
    net_bytes = int(np.minimum(rec_len, NET_WINDOW).sum())

    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=5, max_records=n, device=local,
                      net_groups=args.net_groups, dns_groups=args.dns_groups)
    h.set_global_base(rank * n)
    if world > 1:
        # the library's own RCCL communicator: the merge runs device to device (pv_comm_*)
        uid = [pa.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        h.comm_init(uid[0], world, rank)

    def step():
        # one batch into the live window (no reset: the window accumulates the steps' batches,
        # as a capture's stream does)
        if args.reset_each_step:
            h.reset()
        h.process_device(d_recs.data_ptr(), d_offs.data_ptr(), idx)
        h.synchronize()

    def read():
        # the merged read view of every rank's window, once per read (dist.merge_window with
        # finalize): state merge, then the read view
        tm = time.perf_counter()
        pvdist.merge_window(h, device, comm="pv", finalize=False)
        h.synchronize()
        tf = time.perf_counter()
        pvdist.finalize_window(h, comm="pv")
        h.synchronize()
        return (tf - tm) * 1e3, (time.perf_counter() - tf) * 1e3

    for _ in range(args.warmup):
        h.reset()
        step()
    if world > 1 and args.warmup:
        read()  # the merge's own buffers and RCCL channels come up outside the timed region
    h.reset()
    # the Net pass's dispatch stamps on every TIMING_EVERY-th timed step (a stamped dispatch
    # leaves the device idle ~14 us around it; the others run as a deployment would)
    h.set_kernel_timing(TIMING_EVERY)
    h.kernel_timing(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    step_ms = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        step()  # ends with a device synchronisation
        step_ms.append((time.perf_counter() - ts) * 1e3)
    h.synchronize()
    tr = time.perf_counter()
    merge_ms = read() if world > 1 else (0.0, 0.0)
    steps_s = tr - t0
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    # the Net pass's HIP events (its own stream), summed inside the library over the K steps
    kms, launches = h.kernel_timing(reset=True)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed, kms / max(launches, 1), steps_s, merge_ms[0], merge_ms[1]], dtype=torch.float64,
                         device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms, steps_s = float(t[0]), float(t[1]), float(t[2])
        merge_ms = (float(t[3]), float(t[4]))
    else:
        kernel_ms = kms / max(launches, 1)

    # sanity on the final state (not timed): every step's batch of every rank is in the window
    # (for N > 1 the merged window every rank now holds)
    out = h.window_json(0, merged=False)
    events = out["packets"]["events"]
    if args.reset_each_step:
        expect = n
    else:
        expect = n * world * args.steps
    if events != expect:
        if not os.environ.get("PVGPU_LIB"):
            raise SystemExit(f"bench: bucket holds {events} events, expected {expect}")
        # a tuning variant (lean levels) skips work on purpose
        print(f"bench: tuning variant: bucket holds {events} events, expected {expect}",
              file=sys.stderr)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = n * world * args.steps / elapsed / 1e6
        achieved = net_bytes / (kernel_ms * 1e-3) / 1e9
        step_achieved = algo_bytes / (ms_per_step * 1e-3) / 1e9
        prof = profile_traffic(args.config, n)
        line = {
            "metric": "Mpkt/s device-resident (Net+DNS handler parse)",
            "value": round(value, 2),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "ms_per_step_median": round(float(np.median(step_ms)), 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": WORKLOADS[args.config], "records_per_gpu": n,
                       "bytes_per_record": round(algo_bytes / n, 2), "handlers": "net v1 + dns v1 (default groups)",
                       "parallelism": f"dp{world} (record shards; one read-time merge of the window after the "
                                      "steps: RCCL bucket all-reduce + top-N owner exchange)" if world > 1 else "dp1"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": prof.get("hbm_bytes_per_launch"),
                         "kernel": h.net_kernel_name(), "kernel_ms": round(kernel_ms, 4),
                         "kernel_ms_sample": f"mean of {launches} dispatch-stamped launches (every {TIMING_EVERY}th "
                                             f"of the {args.steps} timed steps)",
                         "bytes_per_launch": net_bytes,
                         "bytes_rule": f"sum over records of min(16 + caplen, {NET_WINDOW}): the bytes the Net pass's "
                                       "algorithm reads (pcap header + L2-L4 headers); step_* use sum(16 + caplen)",
                         # the whole device-resident step against the same algorithmic bytes, and the
                         # step's HBM bytes summed over its kernels (committed rocprofv3 PMC pass)
                         "step_achieved": round(step_achieved, 1), "step_frac": round(step_achieved / HBM_PEAK_GBS, 4),
                         "step_traffic": prof.get("hbm_bytes_per_step"),
                         "traffic_source": prof.get("source")},
        }
        tr = prof.get("hbm_bytes_per_launch")
        if tr:
            # the Net pass's counter bandwidth next to the algorithmic one (its PMC HBM bytes include
            # its writes: the IP log, the DNS work list)
            ca = tr / (kernel_ms * 1e-3) / 1e9
            line["roofline"]["counter_achieved"] = round(ca, 1)
            line["roofline"]["counter_frac"] = round(ca / HBM_PEAK_GBS, 4)
        if args.read_ceiling:
            line["read_ceiling_gbs"] = read_ceiling(d_recs, used)
        if args.e2e and world == 1:
            line["e2e"] = end_to_end(h, buf[:used], n, max(3, args.steps // 4))
        if args.net_groups or args.dns_groups:
            line["groups"] = {"net": args.net_groups, "dns": args.dns_groups}
        if world > 1:
            line["merge"] = {"state_merge_ms": round(merge_ms[0], 3), "finalize_ms": round(merge_ms[1], 3),
                             "steps_ms": round(steps_s * 1e3, 3),
                             "what": "once per read, inside the timed region after the K steps (max over ranks): "
                                     "merge_window = pv_comm_allgather window check, DNS shard edges, "
                                     "pv_comm_allreduce_window (SUM/MIN), pv_comm_merge_topn (top-N entries to region "
                                     "owners over RCCL, merged on the device); finalize_window = leading entries + "
                                     "names, exact distributed quantile selection"}
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    h.close()
    if world > 1:
        dist.destroy_process_group()


def bench_stream(args, world: int, rank: int, local: int, device):
    """--config 5 (BASELINE configs[4]): one stream of --stream-records C4-shape records at
    1 us each, rank r holding the contiguous shard r (generated in host memory). Timed: the
    shard's processing from host memory (global period plan, index, H2D, kernels) and then
    dist.merge_window, reported separately; value = stream records / (max-over-ranks parse +
    merge). One step processes the whole stream once."""
    import torch
    import torch.distributed as dist
    import pktvisor_amd as pa
    from pktvisor_amd import dist as pvdist
    from pktvisor_amd import synth
    total = args.stream_records
    lo, hi = pvdist.shard_range(total, world, rank)
    last = [0.0]

    def progress(k):
        if time.time() - last[0] > 20:
            last[0] = time.time()
            print(f"rank {rank}: generated {k} of {hi - lo} records", file=sys.stderr, flush=True)
    buf, used = synth.stream_shard(4, lo, hi, synth.SEEDS[5] + rank, progress=progress)
    recs = buf[:used]
    # the shard stands for a capture already in page-locked host memory (an AF_PACKET ring's
    # staging, a pinned pcap read buffer): registered once, outside the timed region, so the feed is
    # the DMA rate of the copy streams and not a pageable staging copy
    lib = pa.load_library()
    registered = lib.pv_host_register(buf.ctypes.data, used) == 0
    idx = None
    if world > 1:
        # the global period plan needs the shard's record seconds (u32 record offsets: < 4 GiB)
        if used >= 1 << 32:
            raise SystemExit(f"bench --config 5: a {used} B shard exceeds the 4 GiB record index; use more GPUs")
        idx = pa.RecordIndex(recs, max_records=hi - lo, threads=16)
    start_sec = synth.T0_US // 1000000
    times = []
    # one context for every step, reset between them outside the timed region (as C2-C4 steps are):
    # its device buffers, ingest ring and index state are allocated once, by the first step
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=5, max_records=min(hi - lo, 16_000_000) or 1,
                      device=local)
    h.set_kernel_timing(1)  # every chunk's Net pass (summed per step; the host link bounds C5)
    if world > 1:
        uid = [pa.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        h.comm_init(uid[0], world, rank)
    for it in range(args.warmup + args.steps):
        h.reset()
        h.set_global_base(lo)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        if world > 1:
            pvdist.process_shard(h, recs, idx, start_sec)
        else:
            h.set_start_tstamp(start_sec, 0)
            h.process_host(recs)
        h.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            pvdist.merge_window(h, device, comm="pv")
        h.synchronize()
        t2 = time.perf_counter()
        kms, launches = h.kernel_timing()
        ing = h.ingest_timing(reset=True)
        if it >= args.warmup:
            times.append((t1 - t0, t2 - t1, kms, ing))
        events = h.window_json(5, merged=True)["packets"]["events"] if it == args.warmup + args.steps - 1 else None
    h.close()
    if registered:
        lib.pv_host_unregister(buf.ctypes.data)
    parse = float(np.median([t[0] for t in times]))
    merge = float(np.median([t[1] for t in times]))
    kernel_ms = float(np.median([t[2] for t in times]))
    if world > 1:
        t = torch.tensor([parse, merge, kernel_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        parse, merge, kernel_ms = float(t[0]), float(t[1]), float(t[2])
    if rank == 0:
        per_rec = used / max(hi - lo, 1)
        achieved = used / (kernel_ms * 1e-3) / 1e9 if kernel_ms else 0.0  # shard bytes / summed Net-pass time
        line = {
            "metric": "Mpkt/s end-to-end (host-memory stream shard per GPU, Net+DNS handler parse + merge_window)",
            "value": round(total / (parse + merge) / 1e6, 2),
            "unit": "Mpkt/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round((parse + merge) * 1e3, 2), "parse_ms": round(parse * 1e3, 2),
            "merge_window_ms": round(merge * 1e3, 2), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": WORKLOADS[5], "stream_records": total, "records_per_gpu": hi - lo,
                       "bytes_per_record": round(per_rec, 2), "window_events_5m": events,
                       "host_memory": "page-locked (pv_host_register)" if registered else "pageable",
                       "parallelism": f"dp{world} (contiguous shards, global period plan, merge_window)"},
            # pv_process_host's own split, ms (rank 0, last step): waiting for a piece's index (H2D
            # landed + device index), the batches' device work with their status read-backs
            "ingest_ms": {"index_wait": round(times[-1][3][1], 1), "device": round(times[-1][3][3], 1),
                          "staging_copy": round(times[-1][3][0], 1), "h2d_issue": round(times[-1][3][2], 1)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": "pv_net_kernel",
                         "kernel_ms_total": round(kernel_ms, 3), "note": "Net-pass time summed over the shard's chunks"},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def read_ceiling(d_recs, used: int) -> float:
    """GB/s of a plain full read of the same blob (torch reduction), for reference."""
    import torch
    v = d_recs[: used // 8 * 8].view(torch.int64)
    for _ in range(3):
        v.sum()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        v.sum()
    torch.cuda.synchronize()
    return round(used * 10 / (time.perf_counter() - t0) / 1e9, 1)


def end_to_end(h, blob, n: int, steps: int) -> dict:
    """Mpkt/s of the path that starts in host memory (pv_process_host: parallel copy into
    pinned staging, parallel record index, H2D on a copy stream overlapping the previous
    chunk's kernels, status read-back), from pageable memory and from a page-locked
    (pv_host_register) buffer, with the host-side time split."""
    import numpy as np
    import pktvisor_amd as pa
    lib = pa.load_library()
    buf = np.frombuffer(blob, dtype=np.uint8).copy()
    out = {"unit": "Mpkt/s", "steps": steps, "chunk_mb": int(os.environ.get("PV_INGEST_CHUNK_MB", "128")),
           "path": ("record blob in host RAM -> (pageable only) parallel copy to pinned staging -> H2D of fixed "
                    "chunks on two copy streams into a device ring (PV_INGEST_RING slots, default 4) -> record index on the device "
                    "(pv_index.hip) -> kernels")}
    for mode in ("pageable", "registered"):
        if mode == "registered" and lib.pv_host_register(buf.ctypes.data, buf.nbytes) != 0:
            out[mode] = None
            continue
        try:
            h.reset()
            h.process_host(buf)
            h.synchronize()
            h.ingest_timing(reset=True)
            t0 = time.perf_counter()
            for _ in range(steps):
                h.reset()
                h.process_host(buf)
                h.synchronize()
            dt = (time.perf_counter() - t0) / steps
            t = [round(x / steps, 3) for x in h.ingest_timing(reset=True)]
            out[mode] = {"value": round(n / dt / 1e6, 2), "ms_per_step": round(dt * 1e3, 3),
                         "staging_copy_ms": t[0], "wait_index_ms": t[1], "device_ms": t[3]}
        finally:
            if mode == "registered":
                lib.pv_host_unregister(buf.ctypes.data)
    out["value"] = out["pageable"]["value"]
    return out


def profile_traffic(cfg: int, n: int) -> dict:
    """HBM bytes from the committed rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
    MI355X_MICROARCH.md HBM section) of this workload, if present: the Net pass per launch and
    the whole step (every pv_* kernel of one step; tools/pmc_bench.py)."""
    p = os.path.join(ROOT, "profiles", f"pmc_c{cfg}_{n}.json")
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except Exception:
            return {}
    return {}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg: int, seconds: float):
    """The oracle (CPU restatement of the reference handlers, oracle/pv_oracle.cpp) on a
    bounded sample of the same workload, timed on this host: one thread, then one
    independent oracle instance per core this process may run on (`nproc`, as SURVEY.md §8(d)
    and BASELINE.md ask, bounded by the affinity mask and the cgroup's CPU quota: the GPU box
    shows 256 CPUs to a job with a 16-CPU quota, where 256 threads measured 49 against ~100
    Mpkt/s on C2 for 16, the quota throttling them), each over the same in-memory pcap, as the
    reference's per-input handler threads would run on separate captures (ctypes releases the
    GIL for the call). The all-core rate is `value`; the one-thread rate is `single_thread`,
    and `nproc_estimate` scales it to every CPU the host has (linear, an upper bound)."""
    import threading
    from pktvisor_amd import synth
    from tests.oracle_ctypes import load
    orc = load()
    cfgs = dict(host_spec=synth.HOST_SPEC, num_periods=5, window=5)
    probe_n = 100_000
    pcap = synth.pcap_bytes(cfg, probe_n)
    t0 = time.perf_counter()
    orc.run_bytes(pcap, **cfgs)
    rate = probe_n / (time.perf_counter() - t0)
    n = int(min(2_000_000, max(probe_n, rate * seconds / 4)))
    pcap = synth.pcap_bytes(cfg, n)
    reps = max(1, int(round(seconds / 2 / (n / rate))))
    t0 = time.perf_counter()
    for _ in range(reps):
        orc.run_bytes(pcap, **cfgs)
    dt1 = time.perf_counter() - t0
    rate1 = n * reps / dt1
    nproc = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = nproc
    quota = cgroup_cpus()
    threads = max(1, min(nproc, avail, int(quota) if quota else nproc))
    # the all-core leg: about 2 x seconds of CPU work over the threads (one independent pass of
    # the sample per repetition), so it stays a bounded sample on any core count
    per_thread_s = 2.0 * seconds / threads
    n_t = int(max(10_000, min(n, rate1 * per_thread_s)))
    if n_t != n:
        pcap = synth.pcap_bytes(cfg, n_t)
    reps_t = max(1, int(round(per_thread_s * rate1 / n_t)))

    def work():
        for _ in range(reps_t):
            orc.run_bytes(pcap, **cfgs)
    ts = [threading.Thread(target=work) for _ in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dtn = time.perf_counter() - t0
    raten = n_t * reps_t * threads / dtn
    return {"value": round(raten / 1e6, 4), "unit": "Mpkt/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "single_thread": round(rate1 / 1e6, 4), "nproc": nproc, "affinity_cpus": avail,
            "cgroup_cpu_quota": quota, "nproc_estimate": round(rate1 * nproc / 1e6, 2),
            "sample": (f"the same synthetic workload as in-memory pcaps, oracle/pv_oracle.cpp: {threads} threads "
                       f"(the CPUs this job may use of nproc {nproc}) x {n_t} records x {reps_t} passes in {dtn:.1f} s; one thread {n} "
                       f"records x {reps} passes in {dt1:.1f} s ({rate1 / 1e6:.3f} Mpkt/s)")}


def cgroup_cpus():
    """the CPU quota of this process's cgroup in cores (cpu.max), or None when unlimited"""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


if __name__ == "__main__":
    main()
