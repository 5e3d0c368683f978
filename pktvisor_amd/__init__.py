"""pktvisor_amd — MI355X-native Net v1 + DNS v1 per-packet path of pktvisor.

Python mirror of the reference's handler surface over the C-ABI in
include/pvgpu.h (libpvgpu.so, built in-tree by pktvisor_amd/Makefile):

  * ``PvHandlers`` ~ a NetStreamHandler + DnsStreamHandler pair attached to one
    PcapInputStream (src/handlers/net/v1/NetStreamHandler.cpp:31-130,
    src/handlers/dns/v1/DnsStreamHandler.cpp:30-232), with ``window_json``
    (src/StreamHandler.h:71-77) and the window config keys of
    AbstractMetricsManager (src/AbstractMetricsManager.h:351-389).
  * ``read_pcap`` / ``index_records`` ~ PcapInputStream::_open_pcap's record walk
    (src/inputs/pcap/PcapInputStream.cpp:471-527).
  * ``pktvisor_reader`` ~ cmd/pktvisor-reader/main.cpp:86-258 for net + dns.

There is no CPU fallback: if the HIP library cannot be loaded or no GPU is
present, constructing a handler raises.
"""
from __future__ import annotations

import ctypes
import json
import os
import struct
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpvgpu.so")

PV_NET_COUNTERS, PV_NET_CARDINALITY, PV_NET_TOP_GEO, PV_NET_TOP_IPS = 1, 2, 4, 8
DNS_GROUPS = {"cardinality": 1 << 0, "counters": 1 << 1, "quantiles": 1 << 2, "histograms": 1 << 3,
              "dns_transaction": 1 << 4, "top_ecs": 1 << 5, "top_qnames": 1 << 6, "top_qnames_details": 1 << 7,
              "top_ports": 1 << 8}
NET_GROUPS = {"counters": 1, "cardinality": 2, "top_geo": 4, "top_ips": 8}
DNS_DEFAULT = sum(DNS_GROUPS[g] for g in ("cardinality", "counters", "quantiles", "dns_transaction", "top_qnames",
                                          "top_ports"))
NET_DEFAULT = 15


from pktvisor_amd.config import PvError  # noqa: E402  (base of every error this package raises)


class pv_config(ctypes.Structure):
    _fields_ = [("host_spec", ctypes.c_char_p), ("num_periods", ctypes.c_uint32), ("topn_count", ctypes.c_uint32),
                ("xact_ttl_ms", ctypes.c_uint32), ("net_groups", ctypes.c_uint32), ("dns_groups", ctypes.c_uint32),
                ("linktype", ctypes.c_uint32), ("ts_nano", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("table_log2", ctypes.c_uint32), ("max_records", ctypes.c_uint64),
                ("topn_percentile_threshold", ctypes.c_uint32), ("net_filter_all", ctypes.c_uint32),
                ("net2_groups", ctypes.c_uint32), ("dns2_groups", ctypes.c_uint32),
                ("deep_sample_rate", ctypes.c_uint32)]


class pv_dns_filters(ctypes.Structure):
    _fields_ = [("exclude_noerror", ctypes.c_uint32), ("only_rcode_mask", ctypes.c_uint32),
                ("answer_count", ctypes.c_int32), ("only_queries", ctypes.c_uint32), ("only_responses", ctypes.c_uint32),
                ("n_qtypes", ctypes.c_uint32), ("qtypes", ctypes.c_uint16 * 16), ("n_qnames", ctypes.c_uint32),
                ("qnames", ctypes.POINTER(ctypes.c_char_p)), ("n_qname_suffixes", ctypes.c_uint32),
                ("qname_suffixes", ctypes.POINTER(ctypes.c_char_p)), ("only_dnssec_response", ctypes.c_uint32),
                ("filter_all", ctypes.c_uint32), ("public_suffix_list", ctypes.c_uint32), ("v2", ctypes.c_uint32),
                ("xact_dirs_disabled", ctypes.c_uint32)]


from pktvisor_amd.config import ConfigException as ConfigError  # noqa: E402  (the reference's texts)
from pktvisor_amd.config import StreamHandlerException  # noqa: E402,F401


DNS_FILTER_KEYS = ("exclude_noerror", "only_rcode", "answer_count", "only_queries", "only_responses", "only_qtype",
                   "only_qname", "only_qname_suffix", "only_dnssec_response", "public_suffix_list")
DNS_FILTER_NOT_BUILT = ("geoloc_notfound", "asn_notfound", "dnstap_msg_type")


def _dns_code(kind: int, name: str):
    v = ctypes.c_uint32()
    return int(v.value) if load_library().pv_dns_code(kind, str(name).encode(), ctypes.byref(v)) == 0 else None


def dns_filter_config(cfg: dict, v2: bool = False) -> dict:
    """DnsStreamHandler::start's filter setup (src/handlers/dns/v1/DnsStreamHandler.cpp:60-150):
    typed values in, the pv_dns_filters fields out; ConfigError with the reference's text."""
    out = dict(exclude_noerror=0, only_rcode_mask=0, answer_count=-1, only_queries=0, only_responses=0, only_qtype=[],
               only_qname=[], only_qname_suffix=[], only_dnssec_response=0, filter_all=0,
               public_suffix_list=0)
    for k in cfg:
        if k in DNS_FILTER_NOT_BUILT:
            raise ConfigError(f"DnsStreamHandler: filter {k} is not supported by the GPU handler")
        if k not in DNS_FILTER_KEYS:
            raise ConfigError(f"{k} is an invalid/unsupported config or filter. The valid configs/filters are: "
                              + ", ".join(DNS_FILTER_KEYS))
    # Configurable::config_get<T> (src/Configurable.h:101-112): a value of another type throws
    for k in ("exclude_noerror", "only_queries", "only_responses", "only_dnssec_response", "public_suffix_list"):
        if k in cfg and not isinstance(cfg[k], bool):
            raise ConfigError(f"wrong type for key: {k}")
    for k in ("only_qtype", "only_qname", "only_qname_suffix"):
        if k in cfg and (not isinstance(cfg[k], (list, tuple)) or not all(isinstance(x, str) for x in cfg[k])):
            raise ConfigError(f"wrong type for key: {k}")
    if cfg.get("exclude_noerror"):
        out["exclude_noerror"] = 1
    elif "only_rcode" in cfg:
        v = cfg["only_rcode"]
        if isinstance(v, bool) or not isinstance(v, (int, list, tuple)):
            raise ConfigError("DnsStreamHandler: wrong value type for only_rcode filter. It should be an integer or an array")
        if isinstance(v, int):
            if _dns_code(0, str(v)) is None:
                raise ConfigError("DnsStreamHandler: only_rcode filter contained an invalid/unsupported rcode")
            codes = [v]
        else:
            codes = []
            for r in v:
                c = _dns_code(0, r)
                if c is None:
                    raise ConfigError(f"DnsStreamHandler: only_rcode filter contained an invalid/unsupported rcode: {r}")
                codes.append(c)
        for c in codes:
            if c > 15:  # a DNS header carries a 4-bit rcode; the reference accepts these but never matches them
                raise ConfigError("DnsStreamHandler: only_rcode filter contained an invalid/unsupported rcode")
            out["only_rcode_mask"] |= 1 << c
    if cfg.get("only_queries"):
        out["only_queries"] = 1
    if cfg.get("only_responses"):
        out["only_responses"] = 1
    if cfg.get("only_dnssec_response"):
        out["only_dnssec_response"] = 1
    # public_suffix_list (:187-189, applied in _configs :648-657): a config, ignored while
    # only_qname_suffix is set
    if cfg.get("public_suffix_list"):
        out["public_suffix_list"] = 1
    if "answer_count" in cfg:
        v = cfg["answer_count"]
        if isinstance(v, bool) or not isinstance(v, int):
            raise ConfigError("DnsStreamHandler: wrong value type for answer_count filter. It should be an integer")
        out["answer_count"] = v
    for q in cfg.get("only_qtype", []):
        c = _dns_code(1, q)
        if c is None:
            raise ConfigError(f"DnsStreamHandler: only_qtype filter contained an invalid/unsupported qtype: {q}")
        out["only_qtype"].append(c)
    # only_qname (:151-160): lower-cased; an input predicate, as only_rcode is
    out["only_qname"] = [str(q).lower() for q in cfg.get("only_qname", [])]
    if out["only_qname"] and out["only_rcode_mask"] and not v2:
        raise ConfigError("DnsStreamHandler: only_qname and only_rcode both install an input predicate: use one")
    if len(out["only_qname"]) > 8 or any(not q or len(q) > 255 for q in out["only_qname"]):
        raise ConfigError("DnsStreamHandler: only_qname: 1..8 names of 1..255 characters")
    # only_qname_suffix (:161-169): lower-cased, first match wins
    out["only_qname_suffix"] = [str(q).lower() for q in cfg.get("only_qname_suffix", [])]
    if len(out["only_qname_suffix"]) > 4:
        raise ConfigError("DnsStreamHandler: only_qname_suffix: at most 4 suffixes")
    if len(out["only_qtype"]) > 16:
        raise ConfigError("DnsStreamHandler: only_qtype: at most 16 qtypes")
    return out


class pv_index_info(ctypes.Structure):
    _fields_ = [("n_records", ctypes.c_uint64), ("bytes_used", ctypes.c_uint64), ("first_sec", ctypes.c_int64),
                ("first_nsec", ctypes.c_int64), ("last_sec", ctypes.c_int64), ("last_nsec", ctypes.c_int64),
                ("monotone", ctypes.c_uint32), ("n_sec_changes", ctypes.c_uint32)]


# every symbol include/pvgpu.h declares (checked by tests/test_abi.py)
EXPORTS = ["pv_version", "pv_device_count", "pv_create", "pv_destroy", "pv_last_error", "pv_index_records",
           "pv_index_records_device",
           "pv_process_device", "pv_process_host", "pv_set_start_tstamp", "pv_set_end_tstamp", "pv_synchronize",
           "pv_reset", "pv_window_json", "pv_free", "pv_state_regions", "pv_set_global_base", "pv_export_topn",
           "pv_merge_topn", "pv_kernel_timing", "pv_set_kernel_timing", "pv_window_regions", "pv_index_records_mt", "pv_host_register",
           "pv_host_unregister", "pv_ingest_timing", "pv_edge_export", "pv_edge_merge", "pv_values_export",
           "pv_values_merge", "pv_window_periods", "pv_set_dns_filters", "pv_dns_code", "pv_advance_windows",
           "pv_dns_event_seconds", "pv_dns_event_seconds_host", "pv_comm_unique_id", "pv_comm_init",
           "pv_comm_allreduce_window", "pv_comm_allgather", "pv_comm_destroy", "pv_process_dnstap", "pv_dnstap_count",
           "pv_pcapng_records", "pv_tpacket3_block_records", "pv_window_prometheus", "pv_add_static_label",
           "pv_window_opentelemetry", "pv_check_period_shift", "pv_bucket_merge", "pv_bucket_json",
           "pv_bucket_prometheus", "pv_bucket_opentelemetry", "pv_bucket_free", "pv_set_slow_defer",
           "pv_slow_values_export", "pv_slow_finish", "pv_edge_carry", "pv_merge_hints", "pv_set_end_of_capture", "pv_shard_cuts", "pv_net_kernel_name",
           "pv_plan_dns_draws", "pv_sample_skip", "pv_set_tcp_reassembly_limit", "pv_set_tcp_exact_lru", "pv_set_dnstap_only_hosts",
           "pv_afpacket_open", "pv_afpacket_attach", "pv_afpacket_run", "pv_afpacket_start", "pv_afpacket_stop",
           "pv_afpacket_stats", "pv_afpacket_close", "pv_afpacket_last_error", "pv_set_bpf", "pv_bpf_validate",
           "pv_bpf_run", "pv_bpf_filter_records", "pv_comm_merge_topn", "pv_topn_x_export", "pv_topn_x_import",
           "pv_topn_x_candidates", "pv_topn_x_names", "pv_topn_x_view", "pv_values_x_select", "pv_comm_values_select",
           "pv_slow_x_finish", "pv_comm_slow_finish"]
# pv_allreduce_fn: (uint64_t *buf, size_t n, int op, void *user) -> int
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p)
PV_HANDLER_NET, PV_HANDLER_DNS = 1, 2
PV_PERIOD_AUTO = 0xFFFFFFFF
PART_NET, PART_DNS = 0, 1
PV_REDUCE_SUM, PV_REDUCE_MIN = 0, 1


class pv_bpf_insn(ctypes.Structure):
    """struct sock_filter (linux/filter.h): one classic-BPF instruction"""
    _fields_ = [("code", ctypes.c_uint16), ("jt", ctypes.c_uint8), ("jf", ctypes.c_uint8), ("k", ctypes.c_uint32)]


def bpf_program(insns):
    """a ctypes array of pv_bpf_insn from (code, jt, jf, k) tuples (`tcpdump -dd EXPR` output)"""
    arr = (pv_bpf_insn * max(1, len(insns)))()
    for i, (c, jt, jf, k) in enumerate(insns):
        arr[i] = pv_bpf_insn(c, jt, jf, k & 0xFFFFFFFF)
    return arr


def bpf_filter(recs: bytes, insns) -> bytes:
    """the classic-pcap records of `recs` the program keeps (pv_bpf_filter_records, host only)"""
    lib = load_library()
    prog = bpf_program(insns)
    src = np.frombuffer(recs, dtype=np.uint8)
    out = np.empty(max(1, len(recs)), dtype=np.uint8)
    nb = ctypes.c_size_t()
    rc = lib.pv_bpf_filter_records(prog, len(insns), src.ctypes.data if len(recs) else None, len(recs), out.ctypes.data,
                                   ctypes.byref(nb), None)
    if rc:
        raise PvError(f"pv_bpf_filter_records failed ({rc}): invalid BPF program")
    return out[:nb.value].tobytes()


class pv_afpacket_config(ctypes.Structure):
    _fields_ = [("interface", ctypes.c_char_p), ("fanout_group_id", ctypes.c_int), ("block_size", ctypes.c_uint32),
                ("frame_size", ctypes.c_uint32), ("num_blocks", ctypes.c_uint32), ("bpf_insns", ctypes.c_void_p),
                ("bpf_len", ctypes.c_uint32), ("batch_bytes", ctypes.c_uint32), ("flush_ms", ctypes.c_uint32)]


class pv_afpacket_counters(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in ("blocks", "packets", "batches", "bytes", "kernel_packets", "kernel_drops",
                                              "kernel_freezes")]


AFPACKET_SINK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64)


class pv_region(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("words", ctypes.c_uint64), ("op", ctypes.c_uint32), ("pad", ctypes.c_uint32)]

_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libpvgpu.so (raises if it was not built: there is no fallback).
    PVGPU_LIB overrides the path (kernel tuning variants built in-tree)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("PVGPU_LIB", path)
    if not os.path.exists(path):
        raise PvError(f"{path} missing: run `make -C pktvisor_amd` (or __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    P, U32, U64, I64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64
    lib.pv_version.restype = ctypes.c_char_p
    lib.pv_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    lib.pv_create.argtypes = [ctypes.POINTER(pv_config), ctypes.POINTER(P)]
    lib.pv_destroy.argtypes = [P]
    lib.pv_destroy.restype = None
    lib.pv_last_error.argtypes = [P]
    lib.pv_last_error.restype = ctypes.c_char_p
    lib.pv_index_records.argtypes = [P, ctypes.c_size_t, U32, P, U64, P, P, U32, ctypes.POINTER(pv_index_info)]
    lib.pv_index_records_device.argtypes = [P, P, ctypes.c_size_t, P, U64, P, P, U32, ctypes.POINTER(pv_index_info)]
    lib.pv_process_device.argtypes = [P, P, P, ctypes.POINTER(pv_index_info), P, P, P]
    lib.pv_index_records_mt.argtypes = [P, ctypes.c_size_t, U32, P, U64, P, P, U32, ctypes.POINTER(pv_index_info),
                                        U32]
    lib.pv_process_host.argtypes = [P, P, ctypes.c_size_t]
    lib.pv_host_register.argtypes = [P, ctypes.c_size_t]
    lib.pv_host_unregister.argtypes = [P]
    lib.pv_ingest_timing.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    lib.pv_set_start_tstamp.argtypes = [P, I64, I64]
    lib.pv_set_end_tstamp.argtypes = [P, I64, I64]
    lib.pv_synchronize.argtypes = [P]
    lib.pv_reset.argtypes = [P]
    lib.pv_window_json.argtypes = [P, U32, ctypes.c_int, ctypes.POINTER(P)]
    lib.pv_window_prometheus.argtypes = [P, U32, U32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                         U32, ctypes.POINTER(P)]
    lib.pv_add_static_label.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.pv_window_opentelemetry.argtypes = [P, U32, U32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                            U32, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_free.argtypes = [P]
    lib.pv_free.restype = None
    lib.pv_check_period_shift.argtypes = [P, I64, I64]
    lib.pv_bucket_merge.argtypes = [P, U32, ctypes.POINTER(P), U32, ctypes.c_int, ctypes.c_int]
    lib.pv_bucket_json.argtypes = [P, P, ctypes.POINTER(P)]
    lib.pv_bucket_prometheus.argtypes = [P, P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p), U32,
                                         ctypes.POINTER(P)]
    lib.pv_bucket_opentelemetry.argtypes = [P, P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                            U32, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_bucket_free.argtypes = [P]
    lib.pv_bucket_free.restype = None
    lib.pv_state_regions.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(P),
                                     ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_set_global_base.argtypes = [P, U64]
    lib.pv_export_topn.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_merge_topn.argtypes = [P, P, ctypes.c_size_t]
    lib.pv_window_regions.argtypes = [P, P, U32, ctypes.POINTER(U32)]
    lib.pv_advance_windows.argtypes = [P, ctypes.c_int, P, U32]
    lib.pv_dns_event_seconds.argtypes = [P, P, P, ctypes.POINTER(pv_index_info), P, P, P, U32, ctypes.POINTER(U32)]
    lib.pv_dns_event_seconds_host.argtypes = [P, P, ctypes.c_size_t, P, U32, ctypes.POINTER(U32)]
    lib.pv_kernel_timing.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64), ctypes.c_int]
    lib.pv_set_kernel_timing.argtypes = [P, ctypes.c_uint32]
    lib.pv_edge_export.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_edge_merge.argtypes = [P, P, P, U32, U32]
    lib.pv_set_slow_defer.argtypes = [P, ctypes.c_int]
    lib.pv_plan_dns_draws.argtypes = [P, ctypes.POINTER(ctypes.c_uint64)]
    lib.pv_sample_skip.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64]
    lib.pv_net_kernel_name.argtypes = [P]
    lib.pv_net_kernel_name.restype = ctypes.c_char_p
    lib.pv_shard_cuts.argtypes = [P, ctypes.c_size_t, P, ctypes.c_uint64, U32, U32, U32, P]
    lib.pv_edge_carry.argtypes = [P, P, ctypes.c_size_t, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_merge_hints.argtypes = [P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.pv_set_end_of_capture.argtypes = [P, ctypes.c_int]
    lib.pv_slow_values_export.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_slow_finish.argtypes = [P, P, P, U32]
    lib.pv_values_export.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_values_merge.argtypes = [P, P, ctypes.c_size_t]
    lib.pv_window_periods.argtypes = [P, ctypes.c_int, P, P, U32, ctypes.POINTER(U32)]
    lib.pv_set_dns_filters.argtypes = [P, ctypes.POINTER(pv_dns_filters)]
    lib.pv_set_tcp_reassembly_limit.argtypes = [P, ctypes.c_uint64]
    lib.pv_set_tcp_exact_lru.argtypes = [P, ctypes.c_int]
    lib.pv_set_bpf.argtypes = [P, P, U32]
    lib.pv_bpf_validate.argtypes = [P, U32]
    lib.pv_bpf_run.argtypes = [P, P, U32, U32]
    lib.pv_bpf_run.restype = ctypes.c_uint32
    lib.pv_bpf_filter_records.argtypes = [P, U32, P, ctypes.c_size_t, P, ctypes.POINTER(ctypes.c_size_t), P]
    lib.pv_set_dnstap_only_hosts.argtypes = [P, ctypes.c_char_p]
    lib.pv_dns_code.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(U32)]
    lib.pv_comm_unique_id.argtypes = [P]
    lib.pv_comm_init.argtypes = [P, P, ctypes.c_int, ctypes.c_int]
    lib.pv_comm_allreduce_window.argtypes = [P]
    lib.pv_comm_allgather.argtypes = [P, P, ctypes.c_size_t, ctypes.POINTER(P), P]
    lib.pv_comm_destroy.argtypes = [P]
    lib.pv_comm_merge_topn.argtypes = [P]
    lib.pv_topn_x_export.argtypes = [P, U32, U32, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_topn_x_import.argtypes = [P, U32, U32, P, P]
    lib.pv_topn_x_candidates.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_topn_x_names.argtypes = [P, P, P, U32, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.pv_topn_x_view.argtypes = [P, P, P, P, P, U32]
    lib.pv_values_x_select.argtypes = [P, ALLREDUCE_FN, P]
    lib.pv_comm_values_select.argtypes = [P]
    lib.pv_slow_x_finish.argtypes = [P, ALLREDUCE_FN, P]
    lib.pv_comm_slow_finish.argtypes = [P]
    lib.pv_process_dnstap.argtypes = [P, P, ctypes.c_size_t, U32]
    lib.pv_tpacket3_block_records.argtypes = [P, ctypes.c_size_t, P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                              ctypes.POINTER(U64)]
    lib.pv_pcapng_records.argtypes = [P, ctypes.c_size_t, P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.POINTER(U32), ctypes.POINTER(U64)]
    lib.pv_dnstap_count.argtypes = [P, ctypes.c_size_t, ctypes.POINTER(U32), ctypes.POINTER(U32)]
    lib.pv_afpacket_open.argtypes = [ctypes.POINTER(pv_afpacket_config), ctypes.POINTER(P)]
    lib.pv_afpacket_attach.argtypes = [P, U32, U32, ctypes.c_int, ctypes.POINTER(pv_afpacket_config), ctypes.POINTER(P)]
    lib.pv_afpacket_run.argtypes = [P, AFPACKET_SINK, P]
    lib.pv_afpacket_start.argtypes = [P, P]
    lib.pv_afpacket_stop.argtypes = [P]
    lib.pv_afpacket_stats.argtypes = [P, ctypes.POINTER(pv_afpacket_counters)]
    lib.pv_afpacket_close.argtypes = [P]
    lib.pv_afpacket_close.restype = None
    lib.pv_afpacket_last_error.restype = ctypes.c_char_p
    _lib = lib
    return lib


def comm_unique_id() -> bytes:
    """ncclGetUniqueId bytes for pv_comm_init (one rank creates, every rank receives)"""
    buf = ctypes.create_string_buffer(128)
    if load_library().pv_comm_unique_id(buf) != 0:
        raise PvError("pv_comm_unique_id failed")
    return buf.raw


def device_count() -> int:
    n = ctypes.c_int(0)
    load_library().pv_device_count(ctypes.byref(n))
    return n.value


def pcapng_records(data: bytes):
    """pcapng bytes -> (linktype, classic pcap records with nanosecond fractions) (pv_pcapng_records)."""
    lib = load_library()
    buf = np.frombuffer(data, dtype=np.uint8)
    nb, lt, nr = ctypes.c_size_t(0), ctypes.c_uint32(0), ctypes.c_uint64(0)
    rc = lib.pv_pcapng_records(buf.ctypes.data, buf.nbytes, None, 0, ctypes.byref(nb), ctypes.byref(lt), ctypes.byref(nr))
    if rc:
        raise PvError("Cannot open pcap/pcapng file" + (" (interfaces with different linktypes)" if rc == -7 else ""))
    out = np.empty(nb.value, dtype=np.uint8)
    rc = lib.pv_pcapng_records(buf.ctypes.data, buf.nbytes, out.ctypes.data, out.nbytes, ctypes.byref(nb),
                               ctypes.byref(lt), ctypes.byref(nr))
    if rc:
        raise PvError(f"pv_pcapng_records failed ({rc})")
    return lt.value, out.tobytes()


def read_pcap(path: str):
    """pcap or pcapng file -> (linktype, ts_nano, record bytes): classic pcap records after the
    24-byte global header, or a pcapng file's packets as records with ns fractions (ts_nano 1)."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) >= 12 and struct.unpack_from("<I", data, 0)[0] == 0x0A0D0D0A:
        lt, recs = pcapng_records(data)
        return lt, 1, recs
    if len(data) < 24:
        raise PvError("Cannot open pcap/pcapng file")
    magic = struct.unpack_from("<I", data, 0)[0]
    if magic not in (0xA1B2C3D4, 0xA1B23C4D):
        raise PvError("Cannot open pcap/pcapng file (only little-endian classic pcap is supported)")
    linktype = struct.unpack_from("<I", data, 20)[0]
    return linktype, int(magic == 0xA1B23C4D), data[24:]


def tpacket3_records(blocks, out_cap: int = 1 << 26) -> bytes:
    """TPACKET_V3 ring blocks (bytes each) -> pcap records with ns fractions (pv_tpacket3_block_records)."""
    lib = load_library()
    out = np.empty(out_cap, dtype=np.uint8)
    used, n = ctypes.c_size_t(0), ctypes.c_uint64(0)
    for b in blocks:
        buf = np.frombuffer(b, dtype=np.uint8)
        rc = lib.pv_tpacket3_block_records(buf.ctypes.data, buf.nbytes, out.ctypes.data, out.nbytes, ctypes.byref(used),
                                           ctypes.byref(n))
        if rc:
            raise PvError(f"pv_tpacket3_block_records failed ({rc})")
    return out[: used.value].tobytes()


def dnstap_count(frames: bytes):
    """(data frames, dnstap MESSAGE events) of a Frame Streams file (host decode only)."""
    nf, ne = ctypes.c_uint32(0), ctypes.c_uint32(0)
    buf = np.frombuffer(frames, dtype=np.uint8)
    load_library().pv_dnstap_count(buf.ctypes.data, buf.nbytes, ctypes.byref(nf), ctypes.byref(ne))
    return nf.value, ne.value


def dnstap_reader(path: str, periods: int = 1, only_hosts: Optional[list] = None, **kw) -> dict:
    """A dnstap file (DnstapInputStream "dnstap_file") through the Net v1 ("packets") and DNS v1
    ("dns") handlers: {"<periods>m": window}. only_hosts: the input proxy's filter config."""
    with open(path, "rb") as f:
        frames = f.read()
    h = PvHandlers(num_periods=periods, **kw)
    try:
        if only_hosts is not None:
            h._check(h.lib.pv_set_dnstap_only_hosts(h.ctx, ",".join(only_hosts).encode()), "pv_set_dnstap_only_hosts")
        h.process_dnstap(frames)
        key = f"{1 if periods == 1 else periods}m"
        return {key: h.window_json(0 if periods == 1 else periods, merged=periods != 1)}
    finally:
        h.close()


def pcap_file_bytes(records: bytes, linktype: int = 1, ts_nano: int = 0) -> bytes:
    magic = 0xA1B23C4D if ts_nano else 0xA1B2C3D4
    return struct.pack("<IHHiIII", magic, 2, 4, 0, 0, 262144, linktype) + records


class Bucket:
    """A pv_bucket: one handler's metrics bucket taken out of a context (StreamHandler::merge)."""

    def __init__(self, lib, ptr: int, handler: str):
        self.lib, self.ptr, self.handler = lib, ptr, handler

    def free(self):
        if self.ptr:
            self.lib.pv_bucket_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class RecordIndex:
    """Host-side index of a run of pcap records (offsets + second-change points)."""

    def __init__(self, recs, ts_nano: int = 0, max_records: Optional[int] = None, max_changes: int = 1 << 20,
                 threads: int = 1):
        """threads > 1: the parallel walk (pv_index_records_mt), identical results."""
        lib = load_library()
        buf = np.frombuffer(recs, dtype=np.uint8) if not isinstance(recs, np.ndarray) else recs
        if max_records is None:
            max_records = max(1, len(buf) // 16)
        self.offsets = np.empty(max_records, dtype=np.uint32)
        self.sc_idx = np.empty(max_changes, dtype=np.uint32)
        self.sc_sec = np.empty(max_changes, dtype=np.uint32)
        self.info = pv_index_info()
        args = (buf.ctypes.data, len(buf), ts_nano, self.offsets.ctypes.data, max_records, self.sc_idx.ctypes.data,
                self.sc_sec.ctypes.data, max_changes, ctypes.byref(self.info))
        rc = lib.pv_index_records_mt(*args, threads) if threads != 1 else lib.pv_index_records(*args)
        self.rc = rc
        if rc:
            raise PvError(f"pv_index_records failed ({rc})")
        self.offsets = self.offsets[: self.info.n_records]
        self.n = int(self.info.n_records)


def shard_cuts(recs, index: RecordIndex, linktype: int, ts_nano: int, world: int):
    """world + 1 record cuts of a capture for a sharded run (pv_shard_cuts): about equal shards,
    no DNS-over-TCP flow across a cut"""
    buf = np.frombuffer(recs, dtype=np.uint8) if not isinstance(recs, np.ndarray) else recs
    offs = np.ascontiguousarray(index.offsets, dtype=np.uint32)
    cuts = np.zeros(world + 1, dtype=np.uint64)
    rc = load_library().pv_shard_cuts(buf.ctypes.data, len(buf), offs.ctypes.data, index.n, linktype, ts_nano, world,
                                      cuts.ctypes.data)
    if rc:
        raise PvError(f"pv_shard_cuts failed ({rc})")
    return [int(x) for x in cuts]


def add_static_label(key: str, value: str) -> None:
    """Metric::add_static_label: a label on every Prometheus sample of every handler."""
    if load_library().pv_add_static_label(key.encode(), value.encode()):
        raise PvError(f"pv_add_static_label({key!r}) failed")


class AfPacket:
    """The AF_PACKET TPACKET_V3 capture loop (pv_afpacket_*, AFPacket in
    src/inputs/pcap/afpacket.cpp): AfPacket.open(interface, ...) binds a raw socket and its ring
    (CAP_NET_RAW); AfPacket.attach(ring, block_size, num_blocks, wake_fd) runs the same loop over a
    ring the caller maps. start(handlers) feeds pv_process_host on a capture thread (handlers made
    with linktype 1, ts_nano 1); run(fn) captures on the calling thread into fn(records_bytes,
    n_records) until stop() is called from another thread."""

    def __init__(self, ptr, keep=None):
        self.lib = load_library()
        self.ptr = ptr
        self._keep = keep

    @staticmethod
    def _cfg(**kw):
        c = pv_afpacket_config()
        c.interface = kw.get("interface", "any").encode()
        c.fanout_group_id = kw.get("fanout_group_id", -1)
        for k in ("block_size", "frame_size", "num_blocks", "batch_bytes", "flush_ms"):
            setattr(c, k, int(kw.get(k, 0)))
        bpf = kw.get("bpf")  # bytes of struct sock_filter[] (8 B each)
        if bpf:
            buf = ctypes.create_string_buffer(bytes(bpf), len(bpf))
            c.bpf_insns = ctypes.cast(buf, ctypes.c_void_p)
            c.bpf_len = len(bpf) // 8
            c._buf = buf
        return c

    @classmethod
    def open(cls, interface: str = "any", **kw) -> "AfPacket":
        lib = load_library()
        cfg = cls._cfg(interface=interface, **kw)
        p = ctypes.c_void_p()
        rc = lib.pv_afpacket_open(ctypes.byref(cfg), ctypes.byref(p))
        if rc != 0:
            raise PvError(f"pv_afpacket_open failed ({rc}): {lib.pv_afpacket_last_error().decode()}")
        return cls(p.value, cfg)

    @classmethod
    def attach(cls, ring_addr: int, block_size: int, num_blocks: int, wake_fd: int = -1, **kw) -> "AfPacket":
        lib = load_library()
        cfg = cls._cfg(**kw)
        p = ctypes.c_void_p()
        rc = lib.pv_afpacket_attach(ring_addr, block_size, num_blocks, wake_fd, ctypes.byref(cfg), ctypes.byref(p))
        if rc != 0:
            raise PvError(f"pv_afpacket_attach failed ({rc}): {lib.pv_afpacket_last_error().decode()}")
        return cls(p.value, cfg)

    def run(self, fn) -> int:
        def sink(user, recs, nbytes, n):
            try:
                return int(fn(ctypes.string_at(recs, nbytes), n) or 0)
            except Exception:  # noqa: BLE001 - a failing sink stops the capture
                return -1
        cb = AFPACKET_SINK(sink)
        self._cb = cb
        return self.lib.pv_afpacket_run(self.ptr, cb, None)

    def start(self, handlers: "PvHandlers"):
        rc = self.lib.pv_afpacket_start(self.ptr, handlers.ctx)
        if rc != 0:
            raise PvError(f"pv_afpacket_start failed ({rc})")

    def stop(self) -> int:
        return self.lib.pv_afpacket_stop(self.ptr)

    def stats(self) -> dict:
        c = pv_afpacket_counters()
        self.lib.pv_afpacket_stats(self.ptr, ctypes.byref(c))
        return {k: getattr(c, k) for k, _ in c._fields_}

    def close(self):
        if self.ptr:
            self.lib.pv_afpacket_close(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class PvHandlers:
    """Net v1 ("packets") + DNS v1 ("dns") handlers on one MI355X.

    net_config / dns_config: the handlers' own config maps with the reference's keys and
    validation (enable / disable groups, filters, xact_ttl_*, window keys; see
    pktvisor_amd.config), raising the reference's StreamHandlerException / ConfigException
    texts. The older keyword form (net_groups / dns_groups bits, dns_filters) stays."""

    def __init__(self, host_spec: Optional[str] = None, num_periods: int = 5, topn_count: int = 10,
                 xact_ttl_ms: int = 5000, linktype: int = 1, ts_nano: int = 0, device: int = -1,
                 table_log2: int = 0, max_records: int = 1 << 20, net_groups: int = 0, dns_groups: int = 0,
                 dns_filters: Optional[dict] = None, net_config: Optional[dict] = None,
                 dns_config: Optional[dict] = None, topn_percentile_threshold: int = 0,
                 net2_config: Optional[dict] = None, dns2_config: Optional[dict] = None,
                 deep_sample_rate: int = 100, tcp_packet_reassembly_cache_limit: int = 0, bpf=None,
                 tcp_exact_lru: bool = False):
        from pktvisor_amd import config as pvcfg
        self.lib = load_library()
        filt = dns_filter_config(dns_filters) if dns_filters else None
        net_filter_all = 0
        self.dnstap_mask = 0
        net2_groups = 0
        if net2_config is not None:
            # the Net v2 handler ("net") attached next to v1 ("packets")
            net2_groups = pvcfg.net2_start(dict(net2_config))
        dns2_groups = 0
        if dns2_config is not None:
            # the DNS v2 handler in place of v1 (both use the "dns" schema key)
            if dns_config:
                raise PvError("dns_config and dns2_config are exclusive: one DNS handler version")
            d2 = pvcfg.dns2_start(dict(dns2_config))
            dns2_groups = d2["groups"]
            filt = d2["filters"]
            self.dnstap_mask = d2["dnstap_mask"]
            if d2["xact_ttl_ms"] is not None:
                xact_ttl_ms = d2["xact_ttl_ms"]
        if net_config is not None or dns_config is not None or net2_config is not None or dns2_config is not None:
            ncfg, dcfg = dict(net_config or {}), dict(dns_config or {})
            win = pvcfg.window_config([ncfg, dcfg, dict(net2_config or {}), dict(dns2_config or {})])
            deep_sample_rate = win.get("deep_sample_rate", deep_sample_rate)
            num_periods = win.get("num_periods", num_periods)
            topn_count = win.get("topn_count", topn_count)
            topn_percentile_threshold = win.get("topn_percentile_threshold", topn_percentile_threshold)
            n, d = pvcfg.net_start(ncfg), pvcfg.dns_start(dcfg)
            net_groups, dns_groups, net_filter_all = n["groups"], d["groups"], int(n["filter_all"])
            if dns2_config is None:
                filt = d["filters"]
            if dns2_config is None:
                self.dnstap_mask = d["dnstap_mask"]
            if d["xact_ttl_ms"] is not None and dns2_config is None:
                xact_ttl_ms = d["xact_ttl_ms"]
        self._host = host_spec.encode() if host_spec else None
        cfg = pv_config(self._host, num_periods, topn_count, xact_ttl_ms, net_groups, dns_groups, linktype, ts_nano,
                        device, table_log2, max_records, topn_percentile_threshold, net_filter_all, net2_groups,
                        dns2_groups, deep_sample_rate)
        self.num_periods = num_periods
        self.device = device  # HIP device ordinal (-1: the caller's current device at pv_create)
        self.ctx = ctypes.c_void_p()
        rc = self.lib.pv_create(ctypes.byref(cfg), ctypes.byref(self.ctx))
        if rc:
            msg = self.lib.pv_last_error(self.ctx).decode() if self.ctx else "pv_create"
            self.lib.pv_destroy(self.ctx)
            self.ctx = None
            raise PvError(f"pv_create failed ({rc}): {msg}")
        if filt:
            f = pv_dns_filters(filt["exclude_noerror"], filt["only_rcode_mask"], filt["answer_count"],
                               filt["only_queries"], filt["only_responses"], len(filt["only_qtype"]))
            for k, q in enumerate(filt["only_qtype"]):
                f.qtypes[k] = q
            f.only_dnssec_response = filt["only_dnssec_response"]
            f.filter_all = filt.get("filter_all", 0)
            f.public_suffix_list = filt.get("public_suffix_list", 0)
            f.v2 = filt.get("v2", 0)
            f.xact_dirs_disabled = filt.get("xact_dirs_disabled", 0)
            if filt["only_qname"]:
                self._qnames = (ctypes.c_char_p * len(filt["only_qname"]))(*[q.encode() for q in filt["only_qname"]])
                f.n_qnames = len(filt["only_qname"])
                f.qnames = ctypes.cast(self._qnames, ctypes.POINTER(ctypes.c_char_p))
            if filt["only_qname_suffix"]:
                sx = filt["only_qname_suffix"]
                self._qsfx = (ctypes.c_char_p * len(sx))(*[q.encode() for q in sx])
                f.n_qname_suffixes = len(sx)
                f.qname_suffixes = ctypes.cast(self._qsfx, ctypes.POINTER(ctypes.c_char_p))
            self._check(self.lib.pv_set_dns_filters(self.ctx, ctypes.byref(f)), "pv_set_dns_filters")
        # PcapInputStream's LRU of TCP connections replayed per packet (a cache limit implies it)
        self.tcp_exact = bool(tcp_exact_lru or tcp_packet_reassembly_cache_limit)
        if tcp_packet_reassembly_cache_limit:
            # the pcap input's config (PcapInputStream.cpp:97-99)
            self._check(self.lib.pv_set_tcp_reassembly_limit(self.ctx, int(tcp_packet_reassembly_cache_limit)),
                        "pv_set_tcp_reassembly_limit")
        if tcp_exact_lru:
            # PcapInputStream's LRU of TCP connections replayed exactly (pv_set_tcp_exact_lru)
            self._check(self.lib.pv_set_tcp_exact_lru(self.ctx, 1), "pv_set_tcp_exact_lru")
        if bpf:
            self.set_bpf(bpf)

    def set_bpf(self, insns):
        """the pcap input's "bpf" filter as its compiled classic-BPF program (pv_set_bpf): records it
        rejects never reach the handlers; [] removes it"""
        self._bpf = bpf_program(insns or [])
        self._check(self.lib.pv_set_bpf(self.ctx, self._bpf, len(insns or [])), "pv_set_bpf")

    def _check(self, rc, what):
        if rc:
            raise PvError(f"{what} failed ({rc}): {self.lib.pv_last_error(self.ctx).decode()}")

    def close(self):
        if self.ctx:
            self.lib.pv_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process_host(self, recs):
        buf = recs if isinstance(recs, np.ndarray) else np.frombuffer(recs, dtype=np.uint8)
        self._check(self.lib.pv_process_host(self.ctx, buf.ctypes.data, buf.nbytes), "pv_process_host")

    def set_end_of_capture(self, on: bool = True):
        """the next process_host / process_device call ends the capture: TCP connections still open
        after its last record are closed (pv_set_end_of_capture, TcpReassembly::closeAllConnections)"""
        self._check(self.lib.pv_set_end_of_capture(self.ctx, int(on)), "pv_set_end_of_capture")

    def process_dnstap(self, frames):
        """pv_process_dnstap: a dnstap Frame Streams file's events through both handlers (the
        DNS handler's dnstap_msg_type from dns_config)."""
        buf = frames if isinstance(frames, np.ndarray) else np.frombuffer(frames, dtype=np.uint8)
        self._check(self.lib.pv_process_dnstap(self.ctx, buf.ctypes.data, buf.nbytes, self.dnstap_mask),
                    "pv_process_dnstap")

    def index_device(self, recs, max_records: Optional[int] = None, max_changes: int = 1 << 16):
        """pv_index_records_device: the record index of one block computed on the device;
        returns (offsets, sc_idx, sc_sec, pv_index_info) as RecordIndex holds them."""
        buf = np.frombuffer(recs, dtype=np.uint8) if not isinstance(recs, np.ndarray) else recs
        if max_records is None:
            max_records = max(1, len(buf) // 16)
        offs = np.empty(max_records, dtype=np.uint32)
        sci = np.empty(max_changes, dtype=np.uint32)
        scs = np.empty(max_changes, dtype=np.uint32)
        info = pv_index_info()
        self._check(self.lib.pv_index_records_device(self.ctx, buf.ctypes.data, len(buf), offs.ctypes.data, max_records,
                                                     sci.ctypes.data, scs.ctypes.data, max_changes, ctypes.byref(info)),
                    "pv_index_records_device")
        return offs[: info.n_records], sci, scs, info

    def ingest_timing(self, reset: bool = False):
        """ms spent by pv_process_host: copy + index (pageable), index (pinned), H2D enqueue, device."""
        v = (ctypes.c_double * 4)()
        self.lib.pv_ingest_timing(self.ctx, v, int(reset))
        return list(v)

    def process_device(self, d_recs: int, d_offs: int, index: RecordIndex, stream: Optional[int] = None):
        self._check(self.lib.pv_process_device(self.ctx, d_recs, d_offs, ctypes.byref(index.info),
                                               index.sc_idx.ctypes.data, index.sc_sec.ctypes.data, stream),
                    "pv_process_device")

    def set_end_tstamp(self, sec: int, nsec: int):
        self._check(self.lib.pv_set_end_tstamp(self.ctx, sec, nsec), "pv_set_end_tstamp")

    def set_start_tstamp(self, sec: int, nsec: int):
        self._check(self.lib.pv_set_start_tstamp(self.ctx, sec, nsec), "pv_set_start_tstamp")

    def check_period_shift(self, sec: int, nsec: int = 0):
        """heartbeat_signal -> check_period_shift in both handlers (pv_check_period_shift)."""
        self._check(self.lib.pv_check_period_shift(self.ctx, sec, nsec), "pv_check_period_shift")

    def merge(self, handler: str, bucket: Optional["Bucket"], period: int, prometheus: bool = False,
              merged: bool = False) -> "Bucket":
        """StreamHandler::merge(bucket, period, prometheus, merged) of handler "net" or "dns":
        a new Bucket when bucket is None, else this handler's bucket folded into it with
        Aggregate::SUM (the same Bucket is returned)."""
        h = {"net": PV_HANDLER_NET, "dns": PV_HANDLER_DNS}[handler]
        ptr = ctypes.c_void_p(bucket.ptr if bucket is not None else None)
        self._check(self.lib.pv_bucket_merge(self.ctx, h, ctypes.byref(ptr), period, int(prometheus), int(merged)),
                    "pv_bucket_merge")
        if bucket is not None:
            return bucket
        return Bucket(self.lib, ptr.value, handler)

    def bucket_json(self, bucket: "Bucket") -> dict:
        """window_json(j, bucket): {"packets": {...}} or {"dns": {...}}."""
        out = ctypes.c_void_p()
        self._check(self.lib.pv_bucket_json(self.ctx, bucket.ptr, ctypes.byref(out)), "pv_bucket_json")
        txt = ctypes.string_at(out.value).decode()
        self.lib.pv_free(out)
        return json.loads(txt)

    def bucket_prometheus(self, bucket: "Bucket", labels: Optional[dict] = None) -> str:
        labels = labels or {}
        keys = (ctypes.c_char_p * max(1, len(labels)))(*[k.encode() for k in labels])
        vals = (ctypes.c_char_p * max(1, len(labels)))(*[str(v).encode() for v in labels.values()])
        out = ctypes.c_void_p()
        self._check(self.lib.pv_bucket_prometheus(self.ctx, bucket.ptr, keys, vals, len(labels), ctypes.byref(out)),
                    "pv_bucket_prometheus")
        txt = ctypes.string_at(out.value).decode()
        self.lib.pv_free(out)
        return txt

    def bucket_opentelemetry(self, bucket: "Bucket", labels: Optional[dict] = None) -> bytes:
        labels = labels or {}
        keys = (ctypes.c_char_p * max(1, len(labels)))(*[k.encode() for k in labels])
        vals = (ctypes.c_char_p * max(1, len(labels)))(*[str(v).encode() for v in labels.values()])
        out, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(self.lib.pv_bucket_opentelemetry(self.ctx, bucket.ptr, keys, vals, len(labels), ctypes.byref(out),
                                                     ctypes.byref(n)), "pv_bucket_opentelemetry")
        data = ctypes.string_at(out.value, n.value)
        self.lib.pv_free(out)
        return data

    def set_global_base(self, base: int):
        self._check(self.lib.pv_set_global_base(self.ctx, base), "pv_set_global_base")

    def synchronize(self):
        self._check(self.lib.pv_synchronize(self.ctx), "pv_synchronize")

    def reset(self):
        self._merge_hints = None  # (dist.check_aligned's, for this window only)
        self._check(self.lib.pv_reset(self.ctx), "pv_reset")

    def window_json(self, period: int = 0, merged: bool = False) -> dict:
        out = ctypes.c_void_p()
        self._check(self.lib.pv_window_json(self.ctx, period, 1 if merged else 0, ctypes.byref(out)),
                    "pv_window_json")
        txt = ctypes.string_at(out.value).decode()
        self.lib.pv_free(out)
        return json.loads(txt)

    def window_prometheus(self, period: int = 0, labels: Optional[dict] = None, handlers: str = "net,dns") -> str:
        """StreamHandler::window_prometheus (src/AbstractMetricsManager.h:506-531): the
        Prometheus text of bucket `period` of the named handlers ("net", "dns"), with
        `labels` added to every sample."""
        hmask = sum({"net": 1, "dns": 2}[x] for x in handlers.split(","))
        labels = labels or {}
        keys = (ctypes.c_char_p * max(1, len(labels)))(*[k.encode() for k in labels])
        vals = (ctypes.c_char_p * max(1, len(labels)))(*[str(v).encode() for v in labels.values()])
        out = ctypes.c_void_p()
        self._check(self.lib.pv_window_prometheus(self.ctx, period, hmask, keys, vals, len(labels), ctypes.byref(out)),
                    "pv_window_prometheus")
        txt = ctypes.string_at(out.value).decode()
        self.lib.pv_free(out)
        return txt

    def window_opentelemetry(self, period: int = 0, labels: Optional[dict] = None, handlers: str = "net,dns") -> bytes:
        """StreamHandler::window_opentelemetry (src/AbstractMetricsManager.h:533-575): the
        protobuf bytes of the ScopeMetrics `metrics` the named handlers add for bucket
        `period`, with `labels` as attributes."""
        labels = labels or {}
        hmask = sum({"net": 1, "dns": 2}[x] for x in handlers.split(","))
        keys = (ctypes.c_char_p * max(1, len(labels)))(*[k.encode() for k in labels])
        vals = (ctypes.c_char_p * max(1, len(labels)))(*[str(v).encode() for v in labels.values()])
        out, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(self.lib.pv_window_opentelemetry(self.ctx, period, hmask, keys, vals, len(labels), ctypes.byref(out),
                                                     ctypes.byref(n)), "pv_window_opentelemetry")
        data = ctypes.string_at(out.value, n.value)
        self.lib.pv_free(out)
        return data

    def state_regions(self):
        sp, mp = ctypes.c_void_p(), ctypes.c_void_p()
        sb, mb = ctypes.c_size_t(), ctypes.c_size_t()
        self._check(self.lib.pv_state_regions(self.ctx, ctypes.byref(sp), ctypes.byref(sb), ctypes.byref(mp),
                                              ctypes.byref(mb)), "pv_state_regions")
        return sp.value, sb.value, mp.value, mb.value

    def set_kernel_timing(self, every: int):
        """stamp the Net pass of every `every`-th batch for kernel_timing (0: none, the default;
        a stamped dispatch costs ~14 us of device idle, pv_set_kernel_timing)"""
        self._check(self.lib.pv_set_kernel_timing(self.ctx, int(every)), "pv_set_kernel_timing")

    def kernel_timing(self, reset: bool = False):
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        self._check(self.lib.pv_kernel_timing(self.ctx, ctypes.byref(ms), ctypes.byref(n), int(reset)),
                    "pv_kernel_timing")
        return ms.value, n.value

    # ---- RCCL communicator in the library (pv_comm_*): a C++ host needs no torch
    def comm_init(self, uid: bytes, nranks: int, rank: int):
        b = ctypes.create_string_buffer(bytes(uid), 128)
        self._check(self.lib.pv_comm_init(self.ctx, b, nranks, rank), "pv_comm_init")
        self.comm_ranks, self.comm_rank = nranks, rank

    def comm_allreduce_window(self):
        self._check(self.lib.pv_comm_allreduce_window(self.ctx), "pv_comm_allreduce_window")

    def comm_allgather(self, blob: bytes):
        """every rank's blob, in rank order"""
        out = ctypes.c_void_p()
        sizes = (ctypes.c_uint64 * self.comm_ranks)()
        src = ctypes.create_string_buffer(bytes(blob), max(1, len(blob)))
        self._check(self.lib.pv_comm_allgather(self.ctx, src, len(blob), ctypes.byref(out), sizes), "pv_comm_allgather")
        try:
            data = ctypes.string_at(out.value, sum(sizes)) if sum(sizes) else b""
        finally:
            self.lib.pv_free(out)
        res, at = [], 0
        for n in sizes:
            res.append(data[at:at + n])
            at += n
        return res

    def comm_destroy(self):
        self._check(self.lib.pv_comm_destroy(self.ctx), "pv_comm_destroy")

    def window_regions(self):
        """[(device ptr, 64-bit words, PV_REDUCE_SUM | PV_REDUCE_MIN)] of both live windows, in the
        order every rank with the same windows lists them (pv_window_regions)"""
        regs = (pv_region * 256)()
        n = ctypes.c_uint32()
        self._check(self.lib.pv_window_regions(self.ctx, regs, 256, ctypes.byref(n)), "pv_window_regions")
        return [(int(r.ptr), int(r.words), int(r.op)) for r in regs[: n.value]]

    def advance_windows(self, part: int, thresholds):
        """apply shifts whose shifting event lies in another shard (pv_advance_windows)"""
        t = np.asarray(list(thresholds), dtype=np.int64)
        if len(t):
            self._check(self.lib.pv_advance_windows(self.ctx, part, t.ctypes.data, len(t)), "pv_advance_windows")

    def dns_event_seconds_host(self, recs, max_n: int = 1 << 22):
        """seconds (stream order) in which the records hold a DNS event (pv_dns_event_seconds_host)"""
        buf = recs if isinstance(recs, np.ndarray) else np.frombuffer(recs, dtype=np.uint8)
        out = np.zeros(max_n, dtype=np.int64)
        n = ctypes.c_uint32()
        self._check(self.lib.pv_dns_event_seconds_host(self.ctx, buf.ctypes.data, buf.nbytes, out.ctypes.data, max_n,
                                                       ctypes.byref(n)), "pv_dns_event_seconds_host")
        return [int(x) for x in out[: n.value]]

    def dns_event_seconds(self, d_recs: int, d_offs: int, index: "RecordIndex", max_n: int = 1 << 22):
        out = np.zeros(max_n, dtype=np.int64)
        n = ctypes.c_uint32()
        self._check(self.lib.pv_dns_event_seconds(self.ctx, d_recs, d_offs, ctypes.byref(index.info),
                                                  index.sc_idx.ctypes.data, index.sc_sec.ctypes.data, out.ctypes.data,
                                                  max_n, ctypes.byref(n)), "pv_dns_event_seconds")
        return [int(x) for x in out[: n.value]]

    def export_topn(self) -> bytes:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(self.lib.pv_export_topn(self.ctx, ctypes.byref(p), ctypes.byref(n)), "pv_export_topn")
        data = ctypes.string_at(p.value, n.value) if n.value else b""
        self.lib.pv_free(p)
        return data

    def merge_topn(self, data: bytes):
        buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, dtype=np.uint8)
        self._check(self.lib.pv_merge_topn(self.ctx, buf.ctypes.data, len(data)), "pv_merge_topn")

    # ---- multi-GPU top-N merge on the device (pv_topn_x_*, pv_comm_merge_topn)
    @staticmethod
    def _blob_arrays(blobs):
        keep = [np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, dtype=np.uint8) for b in blobs]
        ptrs = (ctypes.c_void_p * max(1, len(blobs)))(*[k.ctypes.data for k in keep])
        sizes = (ctypes.c_size_t * max(1, len(blobs)))(*[len(b) for b in blobs])
        return keep, ptrs, sizes

    def comm_merge_topn(self):
        self._check(self.lib.pv_comm_merge_topn(self.ctx), "pv_comm_merge_topn")

    def topn_x_export(self, ranks: int, rank: int) -> bytes:
        return self._export(lambda c, p, n: self.lib.pv_topn_x_export(c, ranks, rank, p, n), "pv_topn_x_export")

    def topn_x_import(self, ranks: int, rank: int, blobs):
        keep, ptrs, sizes = self._blob_arrays(blobs)
        self._check(self.lib.pv_topn_x_import(self.ctx, ranks, rank, ptrs, sizes), "pv_topn_x_import")

    def topn_x_candidates(self) -> bytes:
        return self._export(self.lib.pv_topn_x_candidates, "pv_topn_x_candidates")

    def topn_x_names(self, cands) -> bytes:
        keep, ptrs, sizes = self._blob_arrays(cands)
        return self._export(lambda c, p, n: self.lib.pv_topn_x_names(c, ptrs, sizes, len(cands), p, n), "pv_topn_x_names")

    def topn_x_view(self, cands, names):
        kc, pc, sc = self._blob_arrays(cands)
        kn, pn, sn = self._blob_arrays(names)
        self._check(self.lib.pv_topn_x_view(self.ctx, pc, sc, pn, sn, len(cands)), "pv_topn_x_view")

    def values_x_select(self, allreduce):
        """allreduce(np.ndarray uint64, op) sums (op 0) or maxes (op 1) the array over the ranks in place"""
        err = []

        def cb(buf, n, op, user):
            try:
                a = np.ctypeslib.as_array(buf, shape=(n,))
                allreduce(a, op)
                return 0
            except Exception as e:  # surfaced after the call
                err.append(e)
                return 1
        fn = ALLREDUCE_FN(cb)
        rc = self.lib.pv_values_x_select(self.ctx, fn, None)
        if err:
            raise err[0]
        self._check(rc, "pv_values_x_select")

    def _with_allreduce(self, fn, what, allreduce):
        err = []

        def cb(buf, n, op, user):
            try:
                allreduce(np.ctypeslib.as_array(buf, shape=(n,)), op)
                return 0
            except Exception as e:  # surfaced after the call
                err.append(e)
                return 1
        cfn = ALLREDUCE_FN(cb)
        rc = fn(self.ctx, cfn, None)
        if err:
            raise err[0]
        self._check(rc, what)

    def slow_x_finish(self, allreduce):
        self._with_allreduce(self.lib.pv_slow_x_finish, "pv_slow_x_finish", allreduce)

    def comm_slow_finish(self):
        self._check(self.lib.pv_comm_slow_finish(self.ctx), "pv_comm_slow_finish")

    def comm_values_select(self):
        self._check(self.lib.pv_comm_values_select(self.ctx), "pv_comm_values_select")

    def _export(self, fn, what) -> bytes:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(fn(self.ctx, ctypes.byref(p), ctypes.byref(n)), what)
        data = ctypes.string_at(p.value, n.value) if n.value else b""
        self.lib.pv_free(p)
        return data

    def edge_export(self) -> bytes:
        """shard-edge DNS transaction stubs of this shard (pv_edge_export)"""
        return self._export(self.lib.pv_edge_export, "pv_edge_export")

    def edge_merge(self, exports, rank: int):
        """pair this shard's stub responses with queries the earlier shards leave open"""
        bufs = [np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, dtype=np.uint8) for b in exports]
        ptrs = (ctypes.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
        sizes = (ctypes.c_size_t * len(bufs))(*[len(b) for b in exports])
        self._check(self.lib.pv_edge_merge(self.ctx, ptrs, sizes, len(bufs), rank), "pv_edge_merge")

    def plan_dns_draws(self) -> int:
        """DNS draws the last dns_event_seconds_host call counted (pv_plan_dns_draws)"""
        v = ctypes.c_uint64()
        self._check(self.lib.pv_plan_dns_draws(self.ctx, ctypes.byref(v)), "pv_plan_dns_draws")
        return int(v.value)

    def sample_skip(self, net_draws: int, dns_draws: int):
        """step the generators past the earlier shards' draws (pv_sample_skip)"""
        self._check(self.lib.pv_sample_skip(self.ctx, net_draws, dns_draws), "pv_sample_skip")

    def net_kernel_name(self) -> str:
        """the Net-pass kernel the last span launched (pv_net_kernel_name)"""
        return self.lib.pv_net_kernel_name(self.ctx).decode()

    def edge_carry(self, open_in: bytes) -> bytes:
        """sharded runs in rank order (pv_edge_carry): account the queries the earlier shards leave
        open against this shard's events; returns the queries still open at this shard's end"""
        buf = np.frombuffer(open_in, dtype=np.uint8) if open_in else np.zeros(1, dtype=np.uint8)
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(self.lib.pv_edge_carry(self.ctx, buf.ctypes.data, len(open_in), ctypes.byref(p), ctypes.byref(n)),
                    "pv_edge_carry")
        data = ctypes.string_at(p.value, n.value) if n.value else b""
        self.lib.pv_free(p)
        return data

    def merge_hints(self):
        """(DNS queries this shard leaves open at its end (an upper bound), its DNS transaction
        values) before a merge (pv_merge_hints)"""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.pv_merge_hints(self.ctx, ctypes.byref(a), ctypes.byref(b)), "pv_merge_hints")
        return int(a.value), int(b.value)

    def values_export(self) -> bytes:
        return self._export(self.lib.pv_values_export, "pv_values_export")

    def set_slow_defer(self, on: bool = True):
        """sharded top_slow: keep the slow candidates for pv_slow_finish (before the first batch)"""
        self._check(self.lib.pv_set_slow_defer(self.ctx, int(on)), "pv_set_slow_defer")
        self.slow_defer = on

    def slow_values_export(self) -> bytes:
        return self._export(self.lib.pv_slow_values_export, "pv_slow_values_export")

    def slow_finish(self, exports):
        """every rank's slow_values_export (rank order): the window's slow thresholds over the
        whole stream, then this rank's deferred candidates into the top_slow tables"""
        bufs = [np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, dtype=np.uint8) for b in exports]
        ptrs = (ctypes.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
        sizes = (ctypes.c_size_t * len(bufs))(*[len(b) for b in exports])
        self._check(self.lib.pv_slow_finish(self.ctx, ptrs, sizes, len(bufs)), "pv_slow_finish")

    def values_merge(self, data: bytes):
        buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, dtype=np.uint8)
        self._check(self.lib.pv_values_merge(self.ctx, buf.ctypes.data, len(data)), "pv_values_merge")

    def window_periods(self, part: int = PART_NET):
        """[(slot, bucket start second)] of one manager's live window, newest first"""
        slots = np.zeros(32, dtype=np.uint32)
        starts = np.zeros(32, dtype=np.int64)
        n = ctypes.c_uint32()
        self._check(self.lib.pv_window_periods(self.ctx, part, slots.ctypes.data, starts.ctypes.data, 32,
                                               ctypes.byref(n)), "pv_window_periods")
        return [(int(a), int(b)) for a, b in zip(slots[: n.value], starts[: n.value])]

    def set_start_tstamp(self, sec: int, nsec: int = 0):
        self._check(self.lib.pv_set_start_tstamp(self.ctx, sec, nsec), "pv_set_start_tstamp")


def last_record_ts(recs: bytes, index: RecordIndex, ts_nano: int = 0):
    off = int(index.offsets[-1])
    sec, frac = struct.unpack_from("<II", recs, off)
    return sec, (frac if ts_nano else frac * 1000)


def pktvisor_reader(path: str, host_spec: Optional[str] = None, periods: int = 5, **kw) -> dict:
    """GPU equivalent of `pktvisor-reader [-H host_spec] --periods N FILE` for net + dns."""
    linktype, ts_nano, recs = read_pcap(path)
    bpf = kw.pop("bpf", None)
    if bpf:
        # the reader delivers only the records the filter keeps (their last one ends the capture);
        # the context then gets no program of its own (the records are filtered once)
        recs = bpf_filter(recs, bpf)
    idx = RecordIndex(recs, ts_nano)
    h = PvHandlers(host_spec=host_spec, num_periods=periods, linktype=linktype, ts_nano=ts_nano,
                   max_records=max(1, idx.n), **kw)
    try:
        # the file's end closes the connections still open (PcapInputStream.cpp:522)
        h.set_end_of_capture()
        h.process_host(recs)
        if idx.n:
            h.set_end_tstamp(*last_record_ts(recs, idx, ts_nano))
        key = f"{1 if periods == 1 else periods}m"
        return {key: h.window_json(0 if periods == 1 else periods, merged=periods != 1)}
    finally:
        h.close()
