"""Multi-GPU reduce of per-shard metric buckets (one process per GPU).

Period boundaries are global: the ranks exchange each shard's record seconds and DNS-event
seconds, compute both managers' shifts once (plan_windows), and each rank applies the
shifts owned by other shards as window operations, so every rank's windows hold the same
periods in the same slots (a contiguous split of a capture that crosses 60 s marks merges).

Packets shard trivially: each rank processes a contiguous record range and its
own buckets; one collective round then merges them, the analog of
AbstractMetricsBucket::merge (src/AbstractMetricsManager.h:177-195) and
Policy::_get_merged_buckets (src/Policies.cpp:420-446):

  * SUM region (uint64 counters, payload histogram, port/qtype/rcode tables):
    all-reduce SUM over RCCL (xGMI on one node);
  * MIN region (int64 CPC first-occurrence global record index per coupon):
    all-reduce MIN, which yields the exact global coupon order, so the
    HIP/ICON estimate equals a single-GPU run over the whole stream;
  * top-N tables: exact per-rank counts exchanged and summed by key;
  * DNS transactions across shard edges: every rank's stubs (queries open at its
    end, responses that are the first event of their (flow, txid) in it, its period
    shifts) are all-gathered; each rank pairs its own stub responses with what the
    earlier shards leave open, before the SUM round (pv_edge_merge);
  * quantile inputs of the live window: all-gathered and appended (pv_values_*);
  * top_slow: a slow transaction is judged against the p90 of the bucket that closed at the last
    DNS shift, a bucket spread over several shards; each rank keeps its candidates with their
    response records (pv_set_slow_defer) and, once every rank's transaction times per period
    are gathered, counts the ones above the whole stream's thresholds (pv_slow_finish).

merge_window() runs the whole sequence; reduce_handlers() is the device part alone
(the per-step collective of the bench).

Only the slots of the live window are reduced (a few MB), so the round is
latency-bound on xGMI next to the parse.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist


class _DevArray:
    """Zero-copy view of library-owned device memory for torch (CUDA array interface)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 3}


def device_view(ptr: int, n: int, dtype: torch.dtype, device) -> torch.Tensor:
    typestr = {torch.int64: "<i8", torch.int32: "<i4", torch.uint8: "|u1"}[dtype]
    return torch.as_tensor(_DevArray(ptr, n, typestr), device=device)


def shard_range(total: int, world: int, rank: int):
    """Contiguous record range [lo, hi) of `rank` (per-flow time order kept inside a shard)."""
    per = (total + world - 1) // world
    lo = min(total, rank * per)
    return lo, min(total, lo + per)


def reduce_regions(sum_parts, min_parts, group=None):
    """All-reduce SUM the uint64 parts (as int64: two's-complement sums are identical)
    and MIN the int64 CPC parts, in place. RCCL reduces device memory directly; gloo
    (CPU tests, or several ranks sharing one GPU) goes through host copies."""
    staged = dist.get_backend(group) == "gloo"
    for parts, op in ((sum_parts, dist.ReduceOp.SUM), (min_parts, dist.ReduceOp.MIN)):
        for t in parts:
            if staged and t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, op=op, group=group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=op, group=group)


def bucket_views(handlers, device):
    """Tensors over the live windows' device regions (pv_window_regions): the Net slots' net
    parts and the DNS slots' dns parts, split by reduce op."""
    from pktvisor_amd import PV_REDUCE_SUM
    sums, mins = [], []
    for ptr, words, op in handlers.window_regions():
        (sums if op == PV_REDUCE_SUM else mins).append(device_view(ptr, words, torch.int64, device))
    return sums, mins


def reduce_handlers(handlers, device, group=None):
    """Merge every rank's buckets into every rank's handlers (device-resident)."""
    handlers.synchronize()
    sums, mins = bucket_views(handlers, device)
    reduce_regions(sums, mins, group)
    torch.cuda.synchronize(device)


# ---- the global period table: every rank's windows must hold the same periods
def shifts_of(start_sec: int, per_rank_secs):
    """One manager's shifts over a stream cut into contiguous shards: per_rank_secs[r] lists,
    in stream order, the seconds in which shard r holds an event of that manager. The manager
    shifts on the first event with ts_sec >= next_shift, then next_shift = that second + 60
    (AbstractMetricsManager::new_event / _period_shift, src/AbstractMetricsManager.h:276-333).
    Returns [(threshold second, owner rank)], the owner being the shard holding that event."""
    out, nxt = [], start_sec + 60
    for r, secs in enumerate(per_rank_secs):
        for s in secs:
            if s >= nxt:
                out.append((int(s), r))
                nxt = int(s) + 60
    return out


def plan_windows(handlers, start_sec: int, rec_secs, dns_secs, group=None, draws=(0, 0)):
    """All-gather each rank's record seconds (Net events) and DNS-event seconds, compute both
    managers' global shifts, and return this rank's part of the plan:
    {"net": (leading, trailing), "dns": (leading, trailing), "skip": (net, dns)} — the shifts
    owned by earlier and by later ranks, which this rank applies as window operations
    (pv_advance_windows), and the deep-sampling draws of the earlier ranks (pv_sample_skip)."""
    world, me = dist.get_world_size(group), dist.get_rank(group)
    allv = [None] * world
    dist.all_gather_object(allv, ([int(x) for x in rec_secs], [int(x) for x in dns_secs], [int(d) for d in draws]),
                           group=group)
    plan = {}
    for key, k in (("net", 0), ("dns", 1)):
        sh = shifts_of(start_sec, [v[k] for v in allv])
        plan[key] = ([t for t, r in sh if r < me], [t for t, r in sh if r > me])
    plan["skip"] = (sum(v[2][0] for v in allv[:me]), sum(v[2][1] for v in allv[:me]))
    return plan


def apply_plan(handlers, plan, which: int):
    """which = 0: the leading shifts (before the shard's first batch), 1: the trailing ones"""
    from pktvisor_amd import PART_DNS, PART_NET
    handlers.advance_windows(PART_NET, plan["net"][which])
    handlers.advance_windows(PART_DNS, plan["dns"][which])


def record_seconds(index):
    """distinct record seconds of a RecordIndex, in stream order"""
    return [int(x) for x in index.sc_sec[: index.info.n_sec_changes]]


def process_shard(handlers, recs, index, start_sec: int, start_nsec: int = 0, group=None):
    """A rank's whole shard of a capture held in host memory: the capture's start_tstamp,
    the global period plan, the shard's batches, the later ranks' shifts. Afterwards every
    rank's windows hold the same periods in the same slots."""
    if getattr(handlers, "tcp_exact", False) and _world(group) > 1:
        # the exact LRU mode replays PcapInputStream's one list of TCP connections over the whole
        # capture (PcapInputStream.cpp:449-459: time-outs of connections of earlier records, at
        # most MAX_TCP_CLEANUPS per packet, evictions past the cache limit); a shard's list starts
        # empty, so a sharded run could close connections differently: refused, not approximated
        raise ValueError("sharded runs do not carry the exact TCP LRU list across shards "
                         "(tcp_exact_lru / tcp_packet_reassembly_cache_limit): process the capture on one rank")
    handlers.set_start_tstamp(start_sec, start_nsec)
    if not getattr(handlers, "slow_defer", False):
        try:
            handlers.set_slow_defer(True)
        except Exception:  # DNS v2: its slow tops keep the rank's own thresholds
            handlers.slow_defer = False
    dns = handlers.dns_event_seconds_host(recs) if len(recs) else []
    draws = (index.n if index is not None else 0, handlers.plan_dns_draws() if len(recs) else 0)
    plan = plan_windows(handlers, start_sec, record_seconds(index) if index is not None and index.n else [], dns, group,
                        draws)
    handlers.sample_skip(*plan["skip"])
    apply_plan(handlers, plan, 0)
    if len(recs):
        handlers.process_host(recs)
    apply_plan(handlers, plan, 1)
    return plan


def _world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _allgather(handlers, blob, group=None, comm=None):
    """every rank's host blob, in rank order: the library's RCCL communicator (comm="pv",
    pv_comm_allgather) or torch.distributed"""
    if comm == "pv":
        return handlers.comm_allgather(blob)
    allv = [None] * dist.get_world_size(group)
    dist.all_gather_object(allv, blob, group=group)
    return allv


def _rank(handlers, group=None, comm=None):
    return handlers.comm_rank if comm == "pv" else dist.get_rank(group)


def check_aligned(handlers, group=None, comm=None):
    """The bucket merge pairs slots by id: every rank's windows must hold the same periods
    (slot, start second) — what the global plan guarantees; checked before the merge. The same
    gather carries each rank's merge hints (pv_merge_hints: DNS queries open at its shard's end,
    DNS transaction values), which merge_edges and the selections use; returns them in rank
    order."""
    import json
    from pktvisor_amd import PART_DNS, PART_NET
    wins = [handlers.window_periods(PART_NET), handlers.window_periods(PART_DNS)]
    mine = json.dumps([wins, list(handlers.merge_hints())]).encode()
    allv = [json.loads(v) for v in _allgather(handlers, mine, group, comm)]
    if any(v[0] != allv[0][0] for v in allv):
        raise RuntimeError(f"shard windows differ across ranks: {[v[0] for v in allv]}")
    hints = [tuple(int(x) for x in v[1]) for v in allv]
    handlers._merge_hints = hints  # (merge_values, in finalize_window, reads the value counts)
    return hints


def merge_edges(handlers, group=None, comm=None, hints=None):
    """DNS transactions across shard edges. Deferred runs carry the open queries rank by rank
    (pv_edge_carry: rank r computes its carry in round r from rank r-1's), so a query meets the
    first event of its key in ANY later shard, after that shard's purges; otherwise every rank's
    stubs are gathered once and paired with the previous shards'. hints (every rank's
    pv_merge_hints, from check_aligned): a rank before the first that leaves a query open
    receives nothing, so the chain starts there, and with no open query anywhere nothing crosses
    an edge and no round runs (a stream without DNS transactions). The last rank's carry is
    nobody's input: it is computed, not gathered."""
    if hints is None:
        hints = check_aligned(handlers, group, comm)
    open_counts = [h[0] for h in hints]
    if not any(open_counts):
        return
    first = next(r for r, k in enumerate(open_counts) if k)
    me = _rank(handlers, group, comm)
    world = len(open_counts)
    if getattr(handlers, "slow_defer", False):
        carried = b""
        for r in range(first, world):
            mine = handlers.edge_carry(carried) if r == me else b""
            if r == world - 1:
                break
            got = _allgather(handlers, mine, group, comm)
            carried = got[r]
        return
    handlers.edge_merge(_allgather(handlers, handlers.edge_export(), group, comm), me)


def _no_values(handlers):
    """every rank reported no DNS transaction value at check_aligned (nothing to select)"""
    hints = getattr(handlers, "_merge_hints", None)
    return hints is not None and not any(h[1] for h in hints)


def merge_slow(handlers, group=None, comm=None):
    """top_slow over the whole stream: each DNS period's p90 over every rank's transaction times
    by distributed selection (no values shipped), then each rank's deferred candidates (after the
    edge merge, before the top-N exchange); skipped when no rank holds a transaction value"""
    if getattr(handlers, "slow_defer", False) and not _no_values(handlers):
        if comm == "pv":
            handlers.comm_slow_finish()
        else:
            handlers.slow_x_finish(_torch_allreduce(group, _handlers_device(handlers)))


def _torch_allreduce(group=None, device=None):
    """an all-reduce of a host uint64 array through torch.distributed (int64: two's-complement
    sums are identical; the values summed and maxed here are below 2^63). On RCCL the array
    travels through `device` (the handlers' GPU), not torch's current device, so ranks that
    never called torch.cuda.set_device still reduce on their own GPU."""
    def ar(a, op):
        t = torch.from_numpy(a.view(np.int64))
        if dist.get_backend(group) != "gloo":
            d = t.to(device if device is not None else torch.device("cuda", torch.cuda.current_device()))
            dist.all_reduce(d, op=dist.ReduceOp.MAX if op else dist.ReduceOp.SUM, group=group)
            t.copy_(d.cpu())
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MAX if op else dist.ReduceOp.SUM, group=group)
    return ar


def _handlers_device(handlers):
    """the torch device of the handlers' GPU (None: torch's current device)"""
    d = getattr(handlers, "device", -1)
    return torch.device("cuda", d) if isinstance(d, int) and d >= 0 else None


def merge_values(handlers, group=None, comm=None):
    """quantile inputs across shards: exact distributed selection (pv_values_x_select), eight
    rounds of group histograms summed over the ranks instead of every rank's values"""
    if (handlers.comm_ranks if comm == "pv" else dist.get_world_size(group)) == 1 or _no_values(handlers):
        return
    if comm == "pv":
        handlers.comm_values_select()
    else:
        handlers.values_x_select(_torch_allreduce(group, _handlers_device(handlers)))


def merge_window(handlers, device, group=None, comm=None, finalize=True):
    """Full merge of every rank's shard into every rank's handlers (read path). comm="pv"
    runs every collective on the library's own RCCL communicator (pv_comm_init first).
    The state merge (edges, slow tops, bucket all-reduce, top-N to the region owners) is the
    device part; finalize=True then assembles the read view (the top-N lists with names, the
    quantiles by distributed selection), which finalize_window also does on its own."""
    handlers.synchronize()
    hints = check_aligned(handlers, group, comm)
    merge_edges(handlers, group, comm, hints)
    merge_slow(handlers, group, comm)
    if comm == "pv":
        handlers.comm_allreduce_window()
    else:
        reduce_handlers(handlers, device, group)
    merge_topn(handlers, group, comm)
    if finalize:
        finalize_window(handlers, group, comm)


def finalize_window(handlers, group=None, comm=None):
    """the merged read view: top-N lists (every owner's leading entries, names from any rank) and
    the quantile inputs (exact distributed selection)"""
    finalize_topn(handlers, group, comm)
    merge_values(handlers, group, comm)


def merge_topn(handlers, group=None, comm=None):
    """Top-N across shards on the device: every table's regions are split over the ranks, each
    rank ships the live entries of the regions others own to their owners (RCCL point-to-point
    with comm="pv", else host blobs over torch.distributed), and the owners merge them into their
    regions (pv_topn_merge). Names stay where they are until finalize_topn."""
    world = handlers.comm_ranks if comm == "pv" else dist.get_world_size(group)
    if world == 1:
        return
    me = _rank(handlers, group, comm)
    if comm == "pv":
        handlers.comm_merge_topn()
    else:
        handlers.topn_x_import(world, me, _allgather(handlers, handlers.topn_x_export(world, me), group, comm))


def finalize_topn(handlers, group=None, comm=None):
    """the merged top-N lists: every owner's leading entries per metric (topn_count and the ties
    of the last), the names of those that lack one from the rank that holds it"""
    world = handlers.comm_ranks if comm == "pv" else dist.get_world_size(group)
    if world == 1:
        return
    cands = _allgather(handlers, handlers.topn_x_candidates(), group, comm)
    names = _allgather(handlers, handlers.topn_x_names(cands), group, comm)
    handlers.topn_x_view(cands, names)
