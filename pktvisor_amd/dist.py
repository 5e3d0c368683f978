"""Multi-GPU reduce of per-shard metric buckets (one process per GPU).

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
  * quantile inputs of the live window: all-gathered and appended (pv_values_*).

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
    """Tensors over the live-window slots of a PvHandlers' SUM and MIN regions."""
    sum_ptr, _, min_ptr, _ = handlers.state_regions()
    slots, sw, mw = handlers.window_slots()
    sums = [device_view(sum_ptr + s * sw * 8, sw, torch.int64, device) for s in slots]
    mins = [device_view(min_ptr + s * mw * 8, mw, torch.int64, device) for s in slots]
    return sums, mins


def reduce_handlers(handlers, device, group=None):
    """Merge every rank's buckets into every rank's handlers (device-resident)."""
    handlers.synchronize()
    sums, mins = bucket_views(handlers, device)
    reduce_regions(sums, mins, group)
    torch.cuda.synchronize(device)


def check_aligned(handlers, group=None):
    """The bucket merge pairs slots by id: every rank's live window must hold the same
    periods (slot, start second). Ranks start their windows at the global first second
    (pv_set_start_tstamp); a shard that ends in a different period is refused."""
    mine = handlers.window_periods()
    allv = [None] * dist.get_world_size(group)
    dist.all_gather_object(allv, mine, group=group)
    if any(v != allv[0] for v in allv):
        raise RuntimeError(f"shard windows differ across ranks: {allv}")


def merge_edges(handlers, group=None):
    exports = [None] * dist.get_world_size(group)
    dist.all_gather_object(exports, handlers.edge_export(), group=group)
    handlers.edge_merge(exports, dist.get_rank(group))


def merge_values(handlers, group=None):
    world = dist.get_world_size(group)
    allv = [None] * world
    dist.all_gather_object(allv, handlers.values_export(), group=group)
    me = dist.get_rank(group)
    for r, data in enumerate(allv):
        if r != me and data:
            handlers.values_merge(data)


def merge_window(handlers, device, group=None):
    """Full merge of every rank's shard into every rank's handlers (read path)."""
    handlers.synchronize()
    check_aligned(handlers, group)
    merge_edges(handlers, group)
    merge_values(handlers, group)
    reduce_handlers(handlers, device, group)
    merge_topn(handlers, group)


def merge_topn(handlers, group=None):
    """Exchange exact per-rank top-N counts (host records) and add the other ranks' into this view."""
    mine = handlers.export_topn()
    world = dist.get_world_size(group)
    allv = [None] * world
    dist.all_gather_object(allv, mine, group=group)
    me = dist.get_rank(group)
    for r, data in enumerate(allv):
        if r != me and data:
            handlers.merge_topn(data)
