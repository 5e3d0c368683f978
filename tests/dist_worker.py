"""Rank process of the multi-rank parity tests (test_dist_gloo.py, test_gpu_dist.py).

GPU mode: rank r processes the contiguous shard r of a pcap on its GPU (all ranks may
share cuda:0 under gloo), the ranks merge with pktvisor_amd.dist.merge_window, and
rank 0 writes the merged window JSON. CPU mode ("cpu"): exercises the collective
helpers of pktvisor_amd.dist alone and writes what each rank saw.

usage: python -m tests.dist_worker gpu PCAP OUT HOST_SPEC PERIODS [DEEP_SAMPLE_RATE [DNS_FILTERS_JSON [DNS2_CONFIG_JSON]]]
       (DNS_FILTERS_JSON "null": none)
       python -m tests.dist_worker cpu OUT
(RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the environment)"""
import json
import os
import struct
import sys


def cpu_main(out):
    import torch
    import torch.distributed as dist
    from pktvisor_amd import dist as pvdist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # u64 counters as int64 (two's complement wrap), CPC first-occurrence minima
    big = (1 << 63) - 5
    s = torch.tensor([rank + 1, big if rank == 0 else 10, 7], dtype=torch.int64)
    m = torch.tensor([100 + rank, 5 - rank, (1 << 62) if rank else 3], dtype=torch.int64)
    pvdist.reduce_regions([s], [m])
    ranges = [pvdist.shard_range(10, world, r) for r in range(world)]
    got = [None] * world
    dist.all_gather_object(got, {"rank": rank, "blob": bytes([rank]) * (rank + 1)})
    # a sharded run in the exact TCP LRU mode is refused before it touches the handlers
    class ExactLru:
        tcp_exact = True
    try:
        pvdist.process_shard(ExactLru(), b"", None, 0)
        refused = ""
    except ValueError as e:
        refused = str(e)
    json.dump({"sum": [int(x) for x in s], "min": [int(x) for x in m], "ranges": ranges,
               "gathered": [(g["rank"], g["blob"].hex()) for g in got], "exact_lru_refused": refused},
              open(f"{out}.{rank}", "w"))
    dist.destroy_process_group()


def gpu_main(pcap_path, out, host, periods, rate=100, filters=None, dns2_config=None):
    import torch
    import torch.distributed as dist
    import pktvisor_amd as pa
    from pktvisor_amd import dist as pvdist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # torch's HIP runtime before the library's (the other order leaves torch without a device)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ndev)
    torch.cuda.set_device(dev)
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    linktype, ts_nano, recs = pa.read_pcap(pcap_path)
    idx = pa.RecordIndex(recs, ts_nano)
    cuts = pa.shard_cuts(recs, idx, linktype, ts_nano, world)
    lo, hi = cuts[rank], cuts[rank + 1]
    offs = [int(x) for x in idx.offsets] + [len(recs)]
    h = pa.PvHandlers(host_spec=host or None, num_periods=periods, linktype=linktype, ts_nano=ts_nano,
                      max_records=max(1, hi - lo), device=dev.index, deep_sample_rate=rate, dns_filters=filters,
                      dns2_config=dns2_config, table_log2=int(os.environ.get("PV_TEST_TABLE_LOG2", "0")))
    try:
        h.set_global_base(lo)
        sec, frac = struct.unpack_from("<II", recs, offs[0])
        shard = recs[offs[lo]:offs[hi]]
        sidx = pa.RecordIndex(shard, ts_nano) if hi > lo else None
        # the capture's start_tstamp on every rank, the global period plan, the shard
        pvdist.process_shard(h, shard, sidx, sec, frac if ts_nano else frac * 1000)
        h.set_end_tstamp(*pa.last_record_ts(recs, idx, ts_nano))
        pvdist.merge_window(h, dev)
        if rank == 0:
            key = f"{1 if periods == 1 else periods}m"
            json.dump({key: h.window_json(0 if periods == 1 else periods, merged=periods != 1)}, open(out, "w"))
    finally:
        h.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    if sys.argv[1] == "cpu":
        cpu_main(sys.argv[2])
    else:
        gpu_main(sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), int(sys.argv[6]) if len(sys.argv) > 6 else 100,
                 json.loads(sys.argv[7]) if len(sys.argv) > 7 else None, json.loads(sys.argv[8]) if len(sys.argv) > 8 else None)
