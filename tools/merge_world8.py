"""merge_window cost at world 8, measured with ranks that share one GPU.

Without RANK in the environment this starts WORLD (default 8) rank processes of itself on
127.0.0.1 (gloo: RCCL needs one GPU per rank, so the exchange here is host blobs and gloo
all-reduces; on an 8-GPU node the same steps run on the library's RCCL communicator). Each rank
generates its contiguous shard of a C5-shape stream (--records in total, C4 records at 1 us; --config 2:
C2 records, the bench's N > 1 shape),
processes it under the global period plan (dist.process_shard), and then times, separately:
  state merge    dist.merge_window(finalize=False): edges, slow tops, bucket all-reduce, top-N
                 entries to their region owners (what bench.py --gpus N runs every step);
  finalize       dist.finalize_window: top-N candidates + names, quantiles by distributed
                 selection.
The bytes each rank contributes to the gathers and all-reduces are counted. Rank 0 prints one
JSON line (times are the max over ranks)."""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def launch(args):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    for p in procs:
        rc |= p.wait()
    return rc


def rank_main(args):
    import numpy as np
    import torch
    import torch.distributed as dist
    import pktvisor_amd as pa
    from pktvisor_amd import dist as pvdist
    from pktvisor_amd import synth
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = pvdist.shard_range(args.records, world, rank)
    t = time.time()
    buf, used = synth.stream_shard(args.config, lo, hi, synth.SEEDS[5] + rank)
    recs = buf[:used]
    idx = pa.RecordIndex(recs, max_records=hi - lo, threads=2)
    if rank == 0:
        print(f"generated and indexed {hi - lo} records per rank in {time.time() - t:.1f} s", file=sys.stderr, flush=True)
    sent = {"gather": 0, "allreduce": 0}
    orig_gather = pvdist._allgather

    def counting_gather(handlers, blob, group=None, comm=None):
        sent["gather"] += len(blob)
        return orig_gather(handlers, blob, group, comm)
    pvdist._allgather = counting_gather
    orig_ar = pvdist._torch_allreduce

    def counting_ar(group=None, device=None):
        f = orig_ar(group, device)

        def ar(a, op):
            sent["allreduce"] += a.nbytes
            f(a, op)
        return ar
    pvdist._torch_allreduce = counting_ar
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=5, max_records=min(hi - lo, 16_000_000), device=0)
    try:
        h.set_global_base(lo)
        dist.barrier()
        t0 = time.perf_counter()
        pvdist.process_shard(h, recs, idx, synth.T0_US // 1000000)
        h.synchronize()
        t1 = time.perf_counter()
        # the bucket all-reduce's regions (torch tensors over gloo): their bytes
        sums, mins = pvdist.bucket_views(h, dev)
        region_bytes = sum(x.numel() * x.element_size() for x in sums + mins)
        dist.barrier()
        t2 = time.perf_counter()
        # merge_window(finalize=False), step by step
        part = {}

        def step(name, f):
            a, g0 = time.perf_counter(), sent["gather"]
            f()
            h.synchronize()
            part[name] = {"ms": round((time.perf_counter() - a) * 1e3, 1), "gathered_bytes": sent["gather"] - g0}
        h.synchronize()
        counts = []
        step("check_aligned", lambda: counts.append(pvdist.check_aligned(h)))
        step("edges", lambda: pvdist.merge_edges(h, hints=counts[0]))
        step("slow", lambda: pvdist.merge_slow(h))
        step("buckets", lambda: pvdist.reduce_handlers(h, dev))
        step("topn_owner", lambda: pvdist.merge_topn(h))
        t3 = time.perf_counter()
        state = dict(sent)
        dist.barrier()
        t4 = time.perf_counter()
        step("finalize_topn", lambda: pvdist.finalize_topn(h))
        step("finalize_values", lambda: pvdist.merge_values(h))
        t5 = time.perf_counter()
        fin = {k: sent[k] - state[k] for k in sent}
        events = h.window_json(5, merged=True)["packets"]["events"]
        v = torch.tensor([t1 - t0, t3 - t2, t5 - t4, state["gather"], state["allreduce"], fin["gather"], fin["allreduce"]],
                         dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        if rank == 0:
            print(json.dumps({
                "tool": "merge_world8", "world": world, "config": args.config, "records": args.records, "records_per_rank": hi - lo,
                "transport": "gloo, ranks sharing one GPU (host blobs + gloo all-reduce)",
                "process_shard_s_max": round(float(v[0]), 3),
                "state_merge_ms_max": round(float(v[1]) * 1e3, 1), "finalize_ms_max": round(float(v[2]) * 1e3, 1),
                "state_merge_bytes_per_rank_max": {"gathered": int(v[3]), "allreduced": int(v[4]),
                                                   "bucket_regions": int(region_bytes)},
                "finalize_bytes_per_rank_max": {"gathered": int(v[5]), "allreduced": int(v[6])},
                "rank0_steps_ms": part, "window_events_5m": events}), flush=True)
    finally:
        h.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--records", type=int, default=100_000_000)
    ap.add_argument("--config", type=int, default=4, help="record shape: 4 = C4 / C5 stream (default), 2 = C2 (the bench's N > 1 step)")
    a = ap.parse_args()
    if "RANK" in os.environ:
        rank_main(a)
    else:
        sys.exit(launch(a))
