"""Handler configuration with the reference's validation and error texts.

Mirrors what StreamMetricsHandler::start does before any packet flows
(src/StreamHandler.h:94-152) for the two handlers on the path:

  * validate_configs: every key of the handler config must be one of the handler's
    _config_defs, a window config key, "enable" or "disable"
    (NetStreamHandler.h:204-209, DnsStreamHandler.h:381-397);
  * process_groups: the handler's default groups, then "disable", then "enable", each
    list stopping at "all" (src/StreamHandler.h:111-133; defaults
    NetStreamHandler.cpp:53-56, DnsStreamHandler.cpp:52-57);
  * the DNS filters and configs (DnsStreamHandler::start, :60-201).

The result is the typed pv_config / pv_dns_filters content the C-ABI takes; the GPU
path never sees a config it does not implement (unbuilt keys raise, never ignored).
"""
from __future__ import annotations


class PvError(RuntimeError):
    """Base of every error pktvisor_amd raises."""


class StreamHandlerException(PvError):
    """visor::StreamHandlerException (src/StreamHandler.h)"""


class ConfigException(PvError):
    """visor::ConfigException (src/Configurable.h)"""


WINDOW_CONFIG_DEFS = ("deep_sample_rate", "num_periods", "topn_count", "topn_percentile_threshold")
NET_CONFIG_DEFS = ("geoloc_notfound", "asn_notfound", "only_geoloc_prefix", "only_asn_number", "recorded_stream")
DNS_CONFIG_DEFS = ("exclude_noerror", "only_rcode", "only_queries", "only_responses", "only_dnssec_response",
                   "answer_count", "only_qtype", "only_qname", "only_qname_suffix", "geoloc_notfound", "asn_notfound",
                   "dnstap_msg_type", "public_suffix_list", "recorded_stream", "xact_ttl_secs", "xact_ttl_ms")
# group name -> pv_net_group / pv_dns_group bit (include/pvgpu.h); listed sorted, as std::map iterates
NET_GROUP_DEFS = {"cardinality": 1 << 1, "counters": 1 << 0, "top_geo": 1 << 2, "top_ips": 1 << 3}
DNS_GROUP_DEFS = {"cardinality": 1 << 0, "counters": 1 << 1, "dns_transaction": 1 << 4, "histograms": 1 << 3,
                  "quantiles": 1 << 2, "top_ecs": 1 << 5, "top_ports": 1 << 8, "top_qnames": 1 << 6,
                  "top_qnames_details": 1 << 7}
NET_DEFAULT_GROUPS = ("counters", "cardinality", "top_geo", "top_ips")
DNS_DEFAULT_GROUPS = ("cardinality", "counters", "quantiles", "dns_transaction", "top_qnames", "top_ports")
DNSTAP_MSG_TYPES = ("auth", "client", "forwarder", "resolver", "stub", "tool", "update")
# dnstap Message.Type numbers of each dnstap_msg_type (DnsStreamHandler.h:340-347; dnstap.proto:160-227)
DNSTAP_TYPE_PAIRS = {"auth": (1, 2), "resolver": (3, 4), "client": (5, 6), "forwarder": (7, 8), "stub": (9, 10),
                     "tool": (11, 12), "update": (13, 14)}
GROUPS_SET = 0x80000000  # PV_GROUPS_SET


def validate_configs(cfg: dict, defs) -> None:
    """StreamMetricsHandler::validate_configs (src/StreamHandler.h:135-152)"""
    for key in cfg:
        if key in WINDOW_CONFIG_DEFS or key in defs or key in ("enable", "disable", "_internal_tap_name"):
            continue
        raise StreamHandlerException(f"{key} is an invalid/unsupported config or filter. The valid configs/filters are: "
                                     f"{', '.join(defs)}, {', '.join(WINDOW_CONFIG_DEFS)}")


def _string_list(cfg: dict, key: str) -> list:
    v = cfg[key]
    if not isinstance(v, (list, tuple)) or not all(isinstance(x, str) for x in v):
        raise ConfigException(f"wrong type for key: {key}")  # Configurable::config_get (src/Configurable.h:110)
    return list(v)


def process_groups(cfg: dict, group_defs: dict, defaults) -> int:
    """StreamMetricsHandler::process_groups (src/StreamHandler.h:94-133): the enabled group bits"""
    bits = 0
    for g in defaults:
        bits |= group_defs[g]

    def one(g):
        if g not in group_defs:
            raise StreamHandlerException(f"{g} is an invalid/unsupported metric group. The valid groups are: all, "
                                         + ", ".join(sorted(group_defs)))
        return group_defs[g]

    if "disable" in cfg:
        for g in _string_list(cfg, "disable"):
            if g == "all":
                bits = 0
                break
            bits &= ~one(g)
    if "enable" in cfg:
        for g in _string_list(cfg, "enable"):
            if g == "all":
                for v in group_defs.values():
                    bits |= v
                break
            bits |= one(g)
    return bits


def _bool(cfg: dict, key: str) -> bool:
    v = cfg.get(key, False)
    if not isinstance(v, bool):
        raise ConfigException(f"wrong type for key: {key}")
    return v


def _uint(cfg: dict, key: str) -> int:
    v = cfg[key]
    if isinstance(v, bool) or not isinstance(v, int) or v < 0:
        raise ConfigException(f"wrong type for key: {key}")
    return v


def window_config(cfgs) -> dict:
    """The window config keys (AbstractMetricsManager::AbstractMetricsManager,
    src/AbstractMetricsManager.h:351-389): num_periods 1..10, deep_sample_rate 1..100, topn_count,
    topn_percentile_threshold 0..99 — one value shared by both handlers here."""
    out = {}
    for cfg in cfgs:
        for k in WINDOW_CONFIG_DEFS:
            if k in cfg:
                v = _uint(cfg, k)
                if k in out and out[k] != v:
                    raise ConfigException(f"{k} differs between the net and dns handler configs")
                out[k] = v
    np = out.get("num_periods", 5)
    if not 1 <= np <= 10:
        raise ConfigException("num_periods must be between 1 and 10")
    if "deep_sample_rate" in out:
        # clamped, not refused (AbstractMetricsManager.h:357-365)
        out["deep_sample_rate"] = max(1, min(100, out["deep_sample_rate"]))
    if out.get("topn_percentile_threshold", 0) > 99:
        raise ConfigException("topn_percentile_threshold must be between 0 and 99")
    return out


def net_start(cfg: dict) -> dict:
    """NetStreamHandler::start (src/handlers/net/v1/NetStreamHandler.cpp:45-130) up to the
    signal wiring: {"groups": bits | GROUPS_SET, "filter_all": bool}"""
    validate_configs(cfg, NET_CONFIG_DEFS)
    groups = process_groups(cfg, NET_GROUP_DEFS, NET_DEFAULT_GROUPS)
    out = {"groups": groups | GROUPS_SET, "filter_all": False}
    # the geo / ASN filters match a MaxMind lookup; with no database enabled every packet is
    # filtered (_filtering :223-283: !city->enabled() => will_filter)
    if _bool(cfg, "geoloc_notfound") or _bool(cfg, "asn_notfound"):
        out["filter_all"] = True
    if "only_geoloc_prefix" in cfg:
        _string_list(cfg, "only_geoloc_prefix")
        out["filter_all"] = True
    if "only_asn_number" in cfg:
        for number in _string_list(cfg, "only_asn_number"):
            if not number.isdigit():
                raise ConfigException(f"NetStreamHandler: only_asn_number filter contained an invalid/unsupported value: {number}")
        out["filter_all"] = True
    return out


# Net v2 (src/handlers/net/v2/NetStreamHandler.h:25-31,262-267; defaults :47-52)
NET2_GROUP_DEFS = {"cardinality": 1 << 1, "counters": 1 << 0, "quantiles": 1 << 2, "top_geo": 1 << 3, "top_ips": 1 << 4}
NET2_DEFAULT_GROUPS = ("counters", "cardinality", "quantiles", "top_geo", "top_ips")


def net2_start(cfg: dict) -> int:
    """NetStreamHandler v2 start (src/handlers/net/v2/NetStreamHandler.cpp:45-95) up to the
    signal wiring: the enabled group bits | GROUPS_SET. Its geo / ASN filters need a MaxMind
    database and are not built for v2."""
    validate_configs(cfg, NET_CONFIG_DEFS)
    groups = process_groups(cfg, NET2_GROUP_DEFS, NET2_DEFAULT_GROUPS)
    for k in ("geoloc_notfound", "asn_notfound", "only_geoloc_prefix", "only_asn_number"):
        if k in cfg:
            raise ConfigException(f"{k} is not supported by the GPU Net v2 handler")
    return groups | GROUPS_SET


# DNS v2 (src/handlers/dns/v2/DnsStreamHandler.h:40-52,549-575; defaults .cpp:51-57)
DNS2_GROUP_DEFS = {"cardinality": 1 << 0, "counters": 1 << 1, "quantiles": 1 << 2, "top_ecs": 1 << 3,
                   "top_qtypes": 1 << 4, "top_rcodes": 1 << 5, "top_size": 1 << 6, "top_qnames": 1 << 7,
                   "top_ports": 1 << 8, "xact_times": 1 << 9}
DNS2_DEFAULT_GROUPS = ("cardinality", "counters", "quantiles", "top_qnames", "top_rcodes", "top_qtypes")
DNS2_CONFIG_DEFS = ("exclude_noerror", "only_rcode", "only_dnssec_response", "only_xact_directions", "answer_count",
                    "only_qtype", "only_qname", "only_qname_suffix", "geoloc_notfound", "asn_notfound", "dnstap_msg_type",
                    "public_suffix_list", "recorded_stream", "xact_ttl_secs", "xact_ttl_ms")
DNS2_FILTER_KEYS = ("exclude_noerror", "only_rcode", "only_dnssec_response", "answer_count", "only_qtype", "only_qname",
                    "only_qname_suffix")


def dns2_start(cfg: dict) -> dict:
    """DnsStreamHandler v2 start (src/handlers/dns/v2/DnsStreamHandler.cpp:43-236) up to the
    signal wiring: {"groups": bits | GROUPS_SET, "filters": pv_dns_filters fields (v2) or None,
    "xact_ttl_ms": int|None}. The geo / ASN filters (no MaxMind database) are not built for the
    GPU v2 handler; top_ecs keeps
    its geo / ASN tops empty (no MaxMind database)."""
    from pktvisor_amd import dns_filter_config
    validate_configs(cfg, DNS2_CONFIG_DEFS)
    groups = process_groups(cfg, DNS2_GROUP_DEFS, DNS2_DEFAULT_GROUPS)
    for k in ("geoloc_notfound", "asn_notfound"):
        if k in cfg:
            raise ConfigException(f"{k} is not supported by the GPU DNS v2 handler")
    # dnstap_msg_type (dns/v2/DnsStreamHandler.cpp:176-190): as v1's
    if "dnstap_msg_type" in cfg and cfg["dnstap_msg_type"] not in DNSTAP_MSG_TYPES:
        raise ConfigException("DnsStreamHandler: dnstap_msg_type contained an invalid/unsupported type. Valid types: "
                              + ", ".join(DNSTAP_MSG_TYPES))
    mask = 0
    if "dnstap_msg_type" in cfg:
        q, r = DNSTAP_TYPE_PAIRS[cfg["dnstap_msg_type"]]
        mask = (1 << q) | (1 << r)
    filters = None
    psl = _bool(cfg, "public_suffix_list")  # _configs (dns/v2/DnsStreamHandler.cpp:192-194,612-619)
    if any(k in cfg for k in DNS2_FILTER_KEYS) or "only_xact_directions" in cfg or psl:
        filters = dns_filter_config({k: cfg[k] for k in DNS2_FILTER_KEYS if k in cfg}, v2=True)
        filters["v2"] = 1
        filters["public_suffix_list"] = 1 if psl else 0
        # only_xact_directions (:107-122): every direction filtered but the listed ones
        if "only_xact_directions" in cfg:
            dis = 7
            for d in _string_list(cfg, "only_xact_directions"):
                if d not in ("in", "out", "unknown"):
                    raise ConfigException("DnsStreamHandler: only_xact_directions filter contained an invalid/unsupported "
                                          f"direction: {d}")
                dis &= ~{"in": 1, "out": 2, "unknown": 4}[d]
            filters["xact_dirs_disabled"] = dis
    ttl = None
    if "xact_ttl_ms" in cfg:
        ttl = _uint(cfg, "xact_ttl_ms")
    elif "xact_ttl_secs" in cfg:
        ttl = _uint(cfg, "xact_ttl_secs") * 1000
    return {"groups": groups | GROUPS_SET, "filters": filters, "xact_ttl_ms": ttl, "dnstap_mask": mask}


def dns_start(cfg: dict) -> dict:
    """DnsStreamHandler::start (src/handlers/dns/v1/DnsStreamHandler.cpp:43-201) up to the signal
    wiring: {"groups": bits | GROUPS_SET, "filters": pv_dns_filters fields, "xact_ttl_ms": int|None}"""
    from pktvisor_amd import dns_filter_config
    validate_configs(cfg, DNS_CONFIG_DEFS)
    groups = process_groups(cfg, DNS_GROUP_DEFS, DNS_DEFAULT_GROUPS)
    fkeys = ("exclude_noerror", "only_rcode", "answer_count", "only_queries", "only_responses", "only_qtype",
             "only_qname", "only_qname_suffix", "only_dnssec_response")
    filters = dns_filter_config({k: cfg[k] for k in fkeys if k in cfg})
    # with no geo database enabled, geoloc_notfound / asn_notfound filter every packet (:619-642)
    filters["filter_all"] = 1 if (_bool(cfg, "geoloc_notfound") or _bool(cfg, "asn_notfound")) else 0
    if "dnstap_msg_type" in cfg and cfg["dnstap_msg_type"] not in DNSTAP_MSG_TYPES:
        raise ConfigException("DnsStreamHandler: dnstap_msg_type contained an invalid/unsupported type. Valid types: "
                              + ", ".join(DNSTAP_MSG_TYPES))
    # public_suffix_list (_configs, dns/v1/DnsStreamHandler.cpp:187-189,648-657): a config the DNS
    # pass applies (pv_dns_filters.public_suffix_list)
    filters["public_suffix_list"] = 1 if _bool(cfg, "public_suffix_list") else 0
    ttl = None
    if "xact_ttl_ms" in cfg:
        ttl = _uint(cfg, "xact_ttl_ms")
    elif "xact_ttl_secs" in cfg:
        ttl = _uint(cfg, "xact_ttl_secs") * 1000
    mask = 0
    if "dnstap_msg_type" in cfg:
        q, r = DNSTAP_TYPE_PAIRS[cfg["dnstap_msg_type"]]
        mask = (1 << q) | (1 << r)
    return {"groups": groups | GROUPS_SET, "filters": filters, "xact_ttl_ms": ttl, "dnstap_mask": mask}
