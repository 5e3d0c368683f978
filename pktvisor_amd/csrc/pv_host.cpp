// SPDX-License-Identifier: MPL-2.0
//
// pv_host.cpp — host runtime behind include/pvgpu.h.
//
// Owns the device state of one Net v1 + DNS v1 handler pair on one GPU:
// bucket slots (ring of PV_SLOTS), the window of the last num_periods buckets,
// period-shift bookkeeping (AbstractMetricsManager::new_event/_period_shift,
// src/AbstractMetricsManager.h:276-333), the transaction pairing pass, and the
// finalisation of device buckets into the reference's JSON shape
// (NetworkMetricsBucket::to_json net/v1 ...cpp:447-505, DnsMetricsBucket::to_json
// dns/v1 ...cpp:735-836, window_merged_json AbstractMetricsManager.h:601-647).
//
// Sketch outputs: counters and dense tables are exact; top-N estimates are
// exact counts (inside the FI sketch's stated error bound, which allows
// [true, true + 3.5/2^13 * N]); quantiles are exact under the KLL rank rule
// (identical to KLL while n <= 200, within its rank error beyond); CPC is the
// reference estimator replayed exactly from per-coupon first-occurrence indices
// (HIP for a single bucket, ICON after a union), bit-identical to datasketches.
#include "pv_host.h"

namespace {

int parse_host_spec(pv_ctx *c, const char *spec)
{
    if (!spec) return 0;
    std::string s = spec;
    size_t pos = 0;
    while (pos < s.size()) {
        size_t e = s.find(',', pos);
        std::string host = s.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
        pos = e == std::string::npos ? s.size() : e + 1;
        if (host.empty()) continue;
        // libs/visor_utils/utils.cpp:128-164 (same error strings)
        size_t d = host.find('/');
        if (d == std::string::npos) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
        std::string ip = host.substr(0, d), cs = host.substr(d + 1);
        if (cs.empty() || !std::all_of(cs.begin(), cs.end(), ::isdigit)) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
        int cidr = atoi(cs.c_str());
        if (ip.find(':') != std::string::npos) {
            if (cidr < 0 || cidr > 128) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
            if (c->nets.n6 >= PV_MAX_SUBNETS) return c->fail(PV_EINVAL, "too many host subnets");
            uint8_t a[16];
            if (inet_pton(AF_INET6, ip.c_str(), a) != 1) return c->fail(PV_EINVAL, "invalid IPv6 address: %s", ip.c_str());
            memcpy(c->nets.v6_addr[c->nets.n6], a, 16);
            c->nets.v6_cidr[c->nets.n6++] = (uint32_t)cidr;
        } else {
            if (cidr < 0 || cidr > 32) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
            if (c->nets.n4 >= PV_MAX_SUBNETS) return c->fail(PV_EINVAL, "too many host subnets");
            in_addr a;
            if (inet_pton(AF_INET, ip.c_str(), &a) != 1) return c->fail(PV_EINVAL, "invalid IPv4 address: %s", ip.c_str());
            uint32_t i = c->nets.n4++;
            c->nets.v4_addr[i] = a.s_addr;
            c->nets.v4_all[i] = cidr == 0;
            c->nets.v4_mask[i] = cidr == 0 ? 0 : htonl(0xFFFFFFFFu << (32 - cidr));
        }
    }
    return 0;
}

// Device fills are queued and launched together by flush_fills (one kernel instead of
// one per region); every path that launches kernels or reads device state flushes first.
} // namespace
namespace pvh {
void flush_fills(pv_ctx *c)
{
    if (!c->fills.n) return;
    hipSetDevice(c->device);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((c->fills_max + 255) / 256, 4096);
    hipLaunchKernelGGL(pv_fill_multi, dim3(blocks), dim3(256), 0, c->stream, c->fills);
    c->fills.n = 0;
    c->fills_max = 0;
}
} // namespace pvh
namespace {
void queue_fill(pv_ctx *c, void *p, uint64_t n, uint64_t v, uint32_t w32)
{
    if (!n) return;
    if (c->fills.n == PV_FILL_SEGS) flush_fills(c);
    c->fills.s[c->fills.n++] = PvFillSeg{p, n, v, w32, 0};
    c->fills_max = std::max(c->fills_max, n);
}
int launch_fill64(pv_ctx *c, uint64_t *p, uint64_t n, uint64_t v)
{
    queue_fill(c, p, n, v, 0);
    return 0;
}
} // namespace
namespace pvh {
int launch_fill32(pv_ctx *c, uint32_t *p, uint64_t n, uint32_t v)
{
    queue_fill(c, p, n, v, 1);
    return 0;
}
} // namespace pvh
namespace {

// Clear one handler's part of a slot on the device (enqueued on the context stream):
// its SUM and MIN words and its top-N table. A part that is still clean is skipped.
} // namespace
namespace pvh {
void clear_part(pv_ctx *c, int part, uint32_t s)
{
    Window &w = part == PART_NET ? c->net : c->dns;
    if (part == PART_DNS) {
        // quantile inputs of the slot's previous bucket no longer match (bounded host memory)
        c->gen[s] = (c->gen[s] + 1) & 0xffffff;
        // (a sharded run keeps them: the merge computes every period's slow thresholds)
        if (!c->slow_defer)
            c->xvals_host.erase(std::remove_if(c->xvals_host.begin(), c->xvals_host.end(),
                                               [s](const PvXValue &v) { return (v.slot & 0xff) == s; }),
                                c->xvals_host.end());
    }
    const uint32_t t = s + (part == PART_DNS ? PV_SLOTS : 0);
    c->remote_topn.erase(t);
    c->x_view.clear(); // (its slot sets name slots)
    w.meta[s] = SlotMeta();
    if (w.clean[s]) return;
    const uint64_t tcap = 1ull << c->tcap_log2;
    uint64_t *sum = c->d_sum + (uint64_t)s * PV_SUM_WORDS;
    uint64_t *cpc = (uint64_t *)c->d_cpc + (uint64_t)s * PV_MIN_WORDS;
    if (part == PART_NET) {
        launch_fill64(c, sum, PV_SUM_NET_WORDS, 0);
        launch_fill64(c, cpc, PV_MIN_NET_WORDS, (uint64_t)PV_CPC_EMPTY);
    } else {
        launch_fill64(c, sum + PV_OFF_DNS, PV_SUM_WORDS - PV_OFF_DNS, 0);
        launch_fill64(c, cpc + PV_MIN_NET_WORDS, PV_MIN_WORDS - PV_MIN_NET_WORDS, (uint64_t)PV_CPC_EMPTY);
    }
    // keys only: a count or name word is read only behind a non-zero key, and whoever
    // claims an entry overwrites its name word and adds net of the stale count (global_add,
    // pv_topn_merge)
    launch_fill64(c, c->d_tkeys + t * tcap, tcap, 0);
    launch_fill64(c, c->d_arena_top + (uint64_t)t * PV_ARENA_PARTS, PV_ARENA_PARTS, 0);
    launch_fill32(c, c->d_tab_live + t, 1, 0);
    c->roff[t].clear();
    w.clean[s] = true;
}
} // namespace pvh
namespace {

// _period_shift (src/AbstractMetricsManager.h:276-305) on the host mirror of one window: the
// live bucket becomes read-only at T, the next ordinal's slot (reserved and cleared before
// the batch that shifts) becomes live, the oldest beyond num_periods drops out.
} // namespace
namespace pvh {
void win_shift(pv_ctx *c, Window &w, int64_t T, int64_t Tns)
{
    w.meta[w.slots.front()].set_read_only(T, Tns);
    w.ordinal++;
    const uint32_t s = w.slot_at(0);
    w.meta[s] = SlotMeta();
    w.meta[s].start_sec = T;
    w.meta[s].start_nsec = Tns;
    w.slots.push_front(s);
    if (w.slots.size() > c->cfg.num_periods) w.slots.pop_back();
    w.next_shift_sec = T + 60;
    if (&w == &c->dns) c->sg_ord[s | (c->gen[s] << 8)] = w.ordinal;
}
} // namespace pvh
namespace {

int ensure_started(pv_ctx *c, int64_t sec, int64_t nsec)
{
    if (c->started) return 0;
    // set_start_tstamp on both managers (AbstractMetricsManager.h:423-431)
    for (int part : {PART_NET, PART_DNS}) {
        Window &w = part == PART_NET ? c->net : c->dns;
        w.ordinal = 0;
        clear_part(c, part, 0);
        w.meta[0].start_sec = sec;
        w.meta[0].start_nsec = nsec;
        w.slots.assign(1, 0);
        w.next_shift_sec = sec + 60;
    }
    c->sg_ord[0 | (c->gen[0] << 8)] = 0;
    c->started = true;
    return 0;
}

} // namespace
namespace pvh {
uint64_t quantile_at(std::vector<uint64_t> v, double r)
{
    // the element of rank ceil(r n) - 1 of the sorted values: a selection, not a sort (a period
    // shift's thresholds select over every transaction of the bucket that closed)
    uint64_t w = (uint64_t)std::ceil(r * (double)v.size());
    size_t idx = w == 0 ? 0 : (size_t)(w - 1);
    if (idx >= v.size()) idx = v.size() - 1;
    std::nth_element(v.begin(), v.begin() + idx, v.end());
    return v[idx];
}
} // namespace pvh
namespace {

// copy the transaction values appended on the device since the last sync
} // namespace
namespace pvh {
int sync_xvals(pv_ctx *c)
{
    flush_fills(c);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return c->hipfail(e, "synchronize");
    uint32_t status[ST_WORDS], nv = 0;
    if (!hip_ok(e = hipMemcpy(status, c->d_status, sizeof status, hipMemcpyDeviceToHost)) ||
        !hip_ok(e = hipMemcpy(&nv, c->d_nvals, 4, hipMemcpyDeviceToHost)))
        return c->hipfail(e, "status");
    if (status[ST_FLAGS] & PVF_VALUES_FULL || nv > c->xv_cap)
        return c->fail(PV_ECAPACITY, "transaction value buffer full");
    if (nv > c->xvals_synced) {
        size_t old = c->xvals_host.size(), add = nv - c->xvals_synced;
        c->xvals_host.resize(old + add);
        if (!hip_ok(e = hipMemcpy(&c->xvals_host[old], c->d_xvals + c->xvals_synced, add * sizeof(PvXValue),
                                  hipMemcpyDeviceToHost)))
            return c->hipfail(e, "transaction values");
        c->xvals_synced = nv;
    }
    return 0;
}
} // namespace pvh
namespace pvh {

int window_slots(pv_ctx *c, const Window &w, uint32_t period, bool merged, std::vector<uint32_t> &out)
{
    out.clear();
    if (!merged) {
        if (period >= c->cfg.num_periods)
            return c->fail(PV_EINVAL, "invalid metrics period, specify [0, %u]", c->cfg.num_periods - 1);
        if (period >= w.slots.size())
            return c->fail(PV_EINVAL, "requested metrics period has not yet accumulated, current range is [0, %zu]",
                           w.slots.size() - 1);
        out.push_back(w.slots[period]);
        return 0;
    }
    if (period <= 1 || period > c->cfg.num_periods)
        return c->fail(PV_EINVAL, "invalid metrics period, specify [2, %u]", c->cfg.num_periods);
    for (size_t i = 0; i < w.slots.size() && i < period; i++) out.push_back(w.slots[i]);
    return 0;
}

} // namespace

// the merge entry points rewrite the window with other shards' data (note at pv_ctx::merged)
namespace pvh {
void mark_merged(pv_ctx *c, const char *by)
{
    if (!c) return;
    c->merged = true;
    if (!c->merged_by) c->merged_by = by;
}
} // namespace pvh
static int merged_refuse(pv_ctx *c)
{
    if (!c->merged) return 0;
    return c->fail(PV_EINVAL, "the window was merged across ranks (%s): a merged window is read-only until pv_reset",
                   c->merged_by ? c->merged_by : "merge");
}

// ====================================================================== C ABI
extern "C" {

const char *pv_version(void) { return "pvgpu 0.1 (gfx950)"; }

int pv_device_count(int *count)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return 0;
}

const char *pv_last_error(const pv_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void pv_free(void *p) { free(p); }

int pv_dns_code(int kind, const char *name, uint32_t *value)
{
    if (!name || !value || (kind != 0 && kind != 1)) return PV_EINVAL;
    const auto &m = kind == 0 ? rcode_names() : qtype_names();
    std::string n(name);
    if (n.empty()) return PV_EINVAL;
    if (std::all_of(n.begin(), n.end(), [](unsigned char ch) { return std::isdigit(ch); })) {
        if (n.size() > 6) return PV_EINVAL;
        const unsigned long v = std::stoul(n);
        if (!m.count((uint16_t)v) || v > 65535) return PV_EINVAL;
        *value = (uint32_t)v;
        return 0;
    }
    std::transform(n.begin(), n.end(), n.begin(), [](unsigned char ch) { return (char)std::toupper(ch); });
    for (const auto &kv : m)
        if (n == kv.second) { *value = kv.first; return 0; }
    return PV_EINVAL;
}

int pv_set_tcp_reassembly_limit(pv_ctx *c, uint64_t limit)
{
    if (!c) return PV_EINVAL;
    if (c->records_seen) return c->fail(PV_EINVAL, "tcp_packet_reassembly_cache_limit must be set before the first batch");
    c->tcp_limit = limit;
    return 0;
}

int pv_set_tcp_exact_lru(pv_ctx *c, int on)
{
    if (!c) return PV_EINVAL;
    if (c->records_seen) return c->fail(PV_EINVAL, "the exact TCP LRU mode must be set before the first batch");
    c->tcp_exact = on != 0;
    return 0;
}

// the public_suffix_list table on the device and the per-record suffix sizes (v1 and v2)
static int psl_setup(pv_ctx *c)
{
    hipError_t e = hipSuccess;
    if (!c->d_psl) {
        const std::vector<uint32_t> blob = pvname::psl_blob();
        if (!hip_ok(e = hipSetDevice(c->device)) || !hip_ok(e = hipMalloc(&c->d_psl, blob.size() * 4)) ||
            !hip_ok(e = hipMemcpy(c->d_psl, blob.data(), blob.size() * 4, hipMemcpyHostToDevice)))
            return c->hipfail(e, "public_suffix_list table");
    }
    if (!c->d_sfx && (!hip_ok(e = hipSetDevice(c->device)) || !hip_ok(e = hipMalloc(&c->d_sfx, c->max_records + 64))))
        return c->hipfail(e, "public_suffix_list record buffer");
    return 0;
}

int pv_set_dns_filters(pv_ctx *c, const pv_dns_filters *f)
{
    if (!c) return PV_EINVAL;
    if (c->records_seen) return c->fail(PV_EINVAL, "DNS filters must be set before the first batch");
    if (!f) { c->f_flags = c->f_rcode_mask = c->f_ancount = c->f_nq = c->f_nqn = c->f_nsx = 0; return 0; }
    uint32_t fl = 0;
    if (f->v2) {
        // DnsStreamHandler v2 start (dns/v2/DnsStreamHandler.cpp:61-170): one rcode mask for
        // exclude_noerror (every rcode but NOERROR) or only_rcode, tested on responses only
        if (!c->dns2_groups) return c->fail(PV_EINVAL, "v2 DNS filters without the DNS v2 handler");
        if (f->only_queries || f->only_responses || f->filter_all)
            return c->fail(PV_EUNSUPPORTED, "only_queries / only_responses / geo filters are not DNS v2 filters here");
        fl |= PVDF_V2;
        uint32_t mask = 0;
        if (f->exclude_noerror) mask = 0xfffeu;
        else if (f->only_rcode_mask) {
            for (uint32_t r = 0; r < 32; r++)
                if ((f->only_rcode_mask >> r) & 1 && (r > 15 || !rcode_names().count((uint16_t)r)))
                    return c->fail(PV_EINVAL, "DnsStreamHandler: only_rcode filter contained an invalid/unsupported rcode");
            mask = f->only_rcode_mask;
        }
        if (mask) fl |= PVDF2_RCODE;
        if (f->answer_count >= 0) fl |= PVDF_ANSWER_COUNT;
        if (f->only_dnssec_response) fl |= PVDF_ONLY_DNSSEC;
        if (f->xact_dirs_disabled & 1) fl |= PVDF2_NOIN;
        if (f->xact_dirs_disabled & 2) fl |= PVDF2_NOOUT;
        if (f->xact_dirs_disabled & 4) fl |= PVDF2_NOUNK;
        if (f->n_qtypes > PV_MAX_QTYPES) return c->fail(PV_EINVAL, "only_qtype: at most %d qtypes", PV_MAX_QTYPES);
        for (uint32_t k = 0; k < f->n_qtypes; k++)
            if (!qtype_names().count(f->qtypes[k]))
                return c->fail(PV_EINVAL, "DnsStreamHandler: only_qtype filter contained an invalid/unsupported qtype: %u",
                               (unsigned)f->qtypes[k]);
        if (f->n_qtypes) fl |= PVDF_ONLY_QTYPE;
        if (f->n_qnames > PV_MAX_QNAMES) return c->fail(PV_EINVAL, "only_qname: at most %d names", PV_MAX_QNAMES);
        for (uint32_t k = 0; k < f->n_qnames; k++) {
            const char *q = f->qnames ? f->qnames[k] : nullptr;
            if (!q || !*q || strlen(q) > 255) return c->fail(PV_EINVAL, "only_qname: empty or over-long name");
            c->f_qn[k] = pvname::name_fp(q, strlen(q));
        }
        c->f_nqn = f->n_qnames;
        if (f->n_qnames) fl |= PVDF2_QNAME;
        if (f->n_qname_suffixes > PV_MAX_SUFFIXES)
            return c->fail(PV_EINVAL, "only_qname_suffix: at most %d suffixes", PV_MAX_SUFFIXES);
        for (uint32_t k = 0; k < f->n_qname_suffixes; k++) {
            const char *q = f->qname_suffixes ? f->qname_suffixes[k] : nullptr;
            if (!q || strlen(q) > 254) return c->fail(PV_EINVAL, "only_qname_suffix: missing or over-long suffix");
            c->f_sxl[k] = (uint32_t)strlen(q);
            c->f_sxh[k] = pvname::name_ph(q, strlen(q));
        }
        c->f_nsx = f->n_qname_suffixes;
        if (f->n_qname_suffixes) {
            fl |= PVDF_ONLY_QSUFFIX;
            hipError_t e;
            if (!c->d_sfx && (!hip_ok(e = hipSetDevice(c->device)) || !hip_ok(e = hipMalloc(&c->d_sfx, c->max_records + 64))))
                return c->hipfail(e, "only_qname_suffix record buffer");
        }
        // public_suffix_list (_configs, dns/v2/DnsStreamHandler.cpp:192-194,612-619): only while
        // only_qname_suffix is off; a response's own size aggregates its transaction's names
        if (f->public_suffix_list && !f->n_qname_suffixes) {
            if (int rc = psl_setup(c)) return rc;
            fl |= PVDF_PSL;
        }
        c->f_flags = fl;
        c->f_rcode_mask = mask;
        c->f_ancount = f->answer_count >= 0 ? (uint32_t)f->answer_count : 0;
        c->f_nq = f->n_qtypes;
        for (uint32_t k = 0; k < f->n_qtypes; k++) c->f_qt[k] = f->qtypes[k];
        return 0;
    }
    if (f->exclude_noerror) fl |= PVDF_EXCLUDE_NOERROR;
    else if (f->only_rcode_mask) {
        for (uint32_t r = 0; r < 32; r++)
            if ((f->only_rcode_mask >> r) & 1 && (r > 15 || !rcode_names().count((uint16_t)r)))
                // a DNS header carries a 4-bit rcode: extended rcodes can never match
                return c->fail(PV_EINVAL, "DnsStreamHandler: only_rcode filter contained an invalid/unsupported rcode");
        fl |= PVDF_ONLY_RCODE;
    }
    if (f->answer_count >= 0) fl |= PVDF_ANSWER_COUNT;
    if (f->only_queries) fl |= PVDF_ONLY_QUERIES;
    if (f->only_responses) fl |= PVDF_ONLY_RESPONSES;
    if (f->only_dnssec_response) fl |= PVDF_ONLY_DNSSEC;
    if (f->filter_all) fl |= PVDF_FILTER_ALL;
    if (f->n_qtypes > PV_MAX_QTYPES) return c->fail(PV_EINVAL, "only_qtype: at most %d qtypes", PV_MAX_QTYPES);
    for (uint32_t k = 0; k < f->n_qtypes; k++)
        if (!qtype_names().count(f->qtypes[k]))
            return c->fail(PV_EINVAL, "DnsStreamHandler: only_qtype filter contained an invalid/unsupported qtype: %u",
                           (unsigned)f->qtypes[k]);
    if (f->n_qtypes) fl |= PVDF_ONLY_QTYPE;
    if (f->n_qnames > PV_MAX_QNAMES) return c->fail(PV_EINVAL, "only_qname: at most %d names", PV_MAX_QNAMES);
    if (f->n_qnames && (fl & PVDF_ONLY_RCODE))
        return c->fail(PV_EINVAL, "only_qname and only_rcode both install an input predicate: use one");
    for (uint32_t k = 0; k < f->n_qnames; k++) {
        const char *q = f->qnames ? f->qnames[k] : nullptr;
        if (!q || !*q || strlen(q) > 255) return c->fail(PV_EINVAL, "only_qname: empty or over-long name");
        c->f_qn[k] = pvname::name_fp(q, strlen(q)); // NameStats lower-cases, as only_qname's qname_ci (:151-160)
    }
    c->f_nqn = f->n_qnames;
    if (f->n_qnames) fl |= PVDF_ONLY_QNAME;
    if (f->n_qname_suffixes > PV_MAX_SUFFIXES)
        return c->fail(PV_EINVAL, "only_qname_suffix: at most %d suffixes", PV_MAX_SUFFIXES);
    for (uint32_t k = 0; k < f->n_qname_suffixes; k++) {
        const char *q = f->qname_suffixes ? f->qname_suffixes[k] : nullptr;
        if (!q || strlen(q) > 254) return c->fail(PV_EINVAL, "only_qname_suffix: missing or over-long suffix");
        c->f_sxl[k] = (uint32_t)strlen(q);
        c->f_sxh[k] = pvname::name_ph(q, strlen(q));
    }
    c->f_nsx = f->n_qname_suffixes;
    // public_suffix_list (DnsStreamHandler::_configs, dns/v1/DnsStreamHandler.cpp:648-657,
    // v2 :612-619): a config, not a filter, and only while only_qname_suffix is off. v2 applies
    // the size of a response's own first query name to its transaction's top_qname2/3
    // (new_dns_transaction :1067-1072)
    if (f->public_suffix_list && !f->n_qname_suffixes) {
        if (int rc = psl_setup(c)) return rc;
        fl |= PVDF_PSL;
    }
    if (f->n_qname_suffixes) {
        fl |= PVDF_ONLY_QSUFFIX;
        hipError_t e;
        if (!c->d_sfx && (!hip_ok(e = hipSetDevice(c->device)) || !hip_ok(e = hipMalloc(&c->d_sfx, c->max_records + 64))))
            return c->hipfail(e, "only_qname_suffix record buffer");
    }
    c->f_flags = fl;
    c->f_rcode_mask = (fl & PVDF_ONLY_RCODE) ? f->only_rcode_mask : 0;
    c->f_ancount = f->answer_count >= 0 ? (uint32_t)f->answer_count : 0;
    c->f_nq = f->n_qtypes;
    for (uint32_t k = 0; k < f->n_qtypes; k++) c->f_qt[k] = f->qtypes[k];
    return 0;
}

int pv_create(const pv_config *cfg, pv_ctx **out)
{
    *out = nullptr;
    if (!cfg) return PV_EINVAL;
    pv_ctx *c = new pv_ctx();
    c->cfg = *cfg;
    if (c->cfg.num_periods == 0) c->cfg.num_periods = 5;
    c->cfg.num_periods = std::max(1u, std::min(c->cfg.num_periods, 10u));
    if (c->cfg.topn_count == 0) c->cfg.topn_count = 10;
    if (c->cfg.xact_ttl_ms == 0) c->cfg.xact_ttl_ms = 5000;
    if (c->cfg.linktype == 0) c->cfg.linktype = 1;
    // group bits, 0 = the handler's defaults; PV_GROUPS_SET marks an explicit set (which may be empty)
    if (c->cfg.net_groups) c->net_groups = c->cfg.net_groups & ~PV_GROUPS_SET;
    if (c->cfg.dns_groups) c->dns_groups = c->cfg.dns_groups & ~PV_GROUPS_SET;
    if (c->cfg.net2_groups)
        c->net2_groups = PV_N2G_ON | ((c->cfg.net2_groups & PV_GROUPS_SET) ? (c->cfg.net2_groups & PV_NET2_DEFAULT_GROUPS)
                                                                           : PV_NET2_DEFAULT_GROUPS);
    if (c->cfg.dns2_groups) {
        c->dns2_groups = PV_N2G_ON | ((c->cfg.dns2_groups & PV_GROUPS_SET) ? (c->cfg.dns2_groups & 0x3ffu)
                                                                           : PV_DNS2_DEFAULT_GROUPS);
        // v1's DNS pass runs for the events (and their counts) only
        c->dns_groups = PV_DNS_TRANSACTIONS;
    }
    if (c->cfg.table_log2) c->tcap_log2 = c->cfg.table_log2;
    if (c->tcap_log2 < 8 || c->tcap_log2 > PV_REGION_LOG2 + PV_MAX_REGIONS_LOG2) {
        *out = c;
        return c->fail(PV_EINVAL, "table_log2 %u out of range [8, %d]", c->tcap_log2, PV_REGION_LOG2 + PV_MAX_REGIONS_LOG2);
    }
    c->reg_log2 = c->tcap_log2 > PV_REGION_LOG2 ? c->tcap_log2 - PV_REGION_LOG2 : 0;
    c->nn_cap = (uint32_t)std::min<uint64_t>(1ull << c->tcap_log2, 1ull << 22);
    if (c->cfg.max_records == 0) c->cfg.max_records = 1 << 20;
    c->max_records = c->cfg.max_records;
    c->ovf_cap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(2 * c->max_records, 1u << 16), 1ull << 28);
    // deep_sample_rate (AbstractMetricsManager::configure, src/AbstractMetricsManager.h:357-365: > 100 -> 100, < 1 -> 1)
    c->sample_rate = c->cfg.deep_sample_rate == 0 ? 100u : std::max(1u, std::min(c->cfg.deep_sample_rate, 100u));
    if (c->sample_rate < 100 && c->cfg.net_filter_all) {
        *out = c;
        return c->fail(PV_EUNSUPPORTED, "deep_sample_rate below 100 with geo filters is not built");
    }
    // TransactionManager(ttl_ms) split (TransactionManager.h:60-68)
    if (c->cfg.xact_ttl_ms > 1000) { c->ttl_s = c->cfg.xact_ttl_ms / 1000; c->ttl_ms = c->cfg.xact_ttl_ms - c->ttl_s * 1000; }
    else c->ttl_ms = c->cfg.xact_ttl_ms;
    int rc = parse_host_spec(c, cfg->host_spec);
    if (rc) { *out = c; return rc; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { *out = c; return c->fail(PV_ENODEV, "no HIP device"); }
    if (cfg->device >= 0) {
        if (cfg->device >= ndev) { *out = c; return c->fail(PV_EINVAL, "device %d out of range", cfg->device); }
        c->device = cfg->device;
    } else {
        hipGetDevice(&c->device);
    }
    hipSetDevice(c->device);
    hipError_t e;
    uint64_t tcap = 1ull << c->tcap_log2;
    uint64_t mr = c->max_records;
    hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device);
    {
        // the grid's partition of a batch (DNS pass, combine, merge and the general Net passes):
        // three workgroups per CU; the register-window Net pass walks it with one workgroup per
        // CU (reg_wg_per_cu). PV_NET_WGCU / PV_REG_WGCU override them for A/B runs
        c->wg_per_cu = 3;
        if (const char *w = getenv("PV_NET_WGCU")) { c->wg_per_cu = std::max(1, atoi(w)); c->wg_forced = true; }
        if (const char *w = getenv("PV_REG_WGCU")) c->reg_wg_per_cu = std::max(1, atoi(w));
        {
            int nb = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(pv_dns_kernel), 64 * PV_DNS_WAVES, 0) == hipSuccess &&
                nb > 0)
                c->dns_wg_per_cu = nb;
        }
        if (const char *w = getenv("PV_DNS_WGCU")) c->dns_wg_per_cu = std::max(1, atoi(w));
    }
    // event / DNS work-list regions: main workgroups own wt_per_block * 64 slots each (the
    // last may overhang the batch by < wt_per_block tiles), boundary workgroups 64 each
    // (the last workgroup's region may overhang the batch by < wt_per_block tiles)
    // DNS over TCP messages of one batch (pv_dns_tcp appends their events behind the UDP
    // regions: one more region of slack)
    c->tmsg_cap = (uint32_t)std::min<uint64_t>(mr + 65536, 0x7fffffffull);
    c->tseg_cap = (uint32_t)std::min<uint64_t>(mr + 64, 0xffffffffull);
    const uint64_t region_max = mr / ((uint64_t)c->wg_per_cu * c->cus) + 64 * 64;
    const uint64_t ev_cap = mr + region_max + 64 * 64 + 16 * 256 + c->tmsg_cap + 2 * region_max;
    c->pend_cap = 2 * mr; // open queries carried between batches
    c->ev_store_cap = std::max<uint64_t>(ev_cap, c->pend_cap + mr);
    c->key_cap = mr + c->tmsg_cap + c->pend_cap;
    const size_t esc = (size_t)c->ev_store_cap, kc = (size_t)c->key_cap;
    c->orph_cap = (uint32_t)std::min<uint64_t>(2 * mr, 1u << 30);
    if (!hip_ok(e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) ||
        !hip_ok(e = hipMalloc(&c->d_sum, (size_t)PV_SLOTS * PV_SUM_WORDS * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_cpc, (size_t)PV_SLOTS * PV_MIN_WORDS * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tkeys, (size_t)PV_TABLES * tcap * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tcnt, (size_t)PV_TABLES * tcap * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_taux, (size_t)PV_TABLES * tcap * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_arena, (size_t)PV_TABLES * c->arena_cap)) ||
        !hip_ok(e = hipMalloc(&c->d_arena_top, PV_TABLES * PV_ARENA_PARTS * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_dbits, (size_t)(mr / 64 + 2) * 8)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_dbits, (size_t)(mr / 64 + 2) * 8, hipHostMallocDefault)) ||
        !hip_ok(e = hipMalloc(&c->d_events, esc * sizeof(PvXEvent))) ||
        !hip_ok(e = hipMalloc(&c->d_ekeys, (size_t)ev_cap * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_mq_cnt, 65536 * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_dq, (size_t)ev_cap * 32)) ||
        !hip_ok(e = hipMalloc(&c->d_dq_cnt, 65536 * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_stamps, 65536 * 4 * 8 * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_blk_events, 65536 * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_orph, (size_t)c->orph_cap * sizeof(PvXEvent))) ||
        !hip_ok(e = hipMalloc(&c->d_pend[0], esc * sizeof(PvXEvent))) ||
        !hip_ok(e = hipMalloc(&c->d_pend[1], esc * sizeof(PvXEvent))) ||
        !hip_ok(e = hipMalloc(&c->d_pkeys[0], kc * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_pkeys[1], kc * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_pvals[0], kc * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_pvals[1], kc * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_skeys, kc * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_skeys2, kc * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_svals, kc * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_svals2, kc * 4)) ||
        !hip_ok(e = (c->xv_cap = (uint64_t)mr * 2, hipMalloc(&c->d_xvals, (size_t)mr * 2 * sizeof(PvXValue)))) ||
        !hip_ok(e = hipMalloc(&c->d_valid, (size_t)mr * sizeof(PvXValid))) ||
        !hip_ok(e = hipMalloc(&c->d_nvals, 16)) ||
        // one read-back block: the status words, the tables' live counts, the two overflow
        // words (a batch reads them back with one copy)
        !hip_ok(e = hipMalloc(&c->d_status, ST_RB_WORDS * 4)) ||
        !hip_ok(e = (c->d_tab_live = c->d_status + ST_ALLOC, c->d_ovf_cnt = c->d_tab_live + PV_TABLES, hipSuccess)) ||
        !hip_ok(e = hipMemsetAsync(c->d_status, 0, ST_RB_WORDS * 4, c->stream)) ||
        !hip_ok(e = hipMalloc(&c->d_theta, ((size_t)1 << c->reg_log2) * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_ovf, (size_t)c->ovf_cap * sizeof(PvOvf))) ||
        ((c->dns2_groups & PV_DNS2_TOP_ECS) &&
         (!hip_ok(e = hipMalloc(&c->d_eecs, esc * 8)) ||
          !hip_ok(e = hipMalloc(&c->d_pecs[0], esc * 8)) ||
          !hip_ok(e = hipMalloc(&c->d_pecs[1], esc * 8)))) ||
        !hip_ok(e = hipMalloc(&c->d_ovf2, (size_t)c->ovf_cap * sizeof(PvOvf))) ||

        !hip_ok(e = hipMalloc(&c->d_nn, (size_t)c->nn_cap * sizeof(PvNewName))) ||
        !hip_ok(e = hipMalloc(&c->d_iplog, (size_t)(mr + 64) * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_iplog32, (size_t)(mr + 64) * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_ipx_rep, (size_t)(mr + 64) * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_ipdir, (size_t)(mr / 64 + 2) * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_ipx_cnt, (size_t)PV_MAX_GRID * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_trash, (size_t)PV_TRASH_WAVES * 2048)) ||
        !hip_ok(e = hipMalloc(&c->d_cb_cnt, 65536 * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_params, 2 * sizeof(PvParams))) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_params, 2 * sizeof(PvParams), hipHostMallocDefault)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_xparams, sizeof(PvXactParams), hipHostMallocDefault)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_status, ST_RB_WORDS * 4, hipHostMallocDefault)) ||
        !hip_ok(e = (c->h_tab_live = c->h_status + ST_ALLOC, c->h_ovf = c->h_tab_live + PV_TABLES, hipSuccess)) ||
        !hip_ok(e = hipMalloc(&c->d_tseg, (size_t)c->tseg_cap * sizeof(PvTcpSeg))) ||
        !hip_ok(e = hipMalloc(&c->d_tmask, (size_t)(mr / 64 + 2) * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tpm, (size_t)(mr / 64 + 2) * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_tcpcnt, (PVT_WORDS + 1) * 4)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_tcpcnt, (PVT_WORDS + 1) * 4, hipHostMallocDefault)) ||
        !hip_ok(e = hipMalloc(&c->d_tparams, sizeof(PvTcpParams))) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_tparams, sizeof(PvTcpParams), hipHostMallocDefault)) ||
        !hip_ok(e = hipMalloc(&c->d_xparams, sizeof(PvXactParams))) || !hip_ok(e = hipEventCreate(&c->ev_start)) ||
        !hip_ok(e = hipEventCreate(&c->ev_stop))) {
        *out = c;
        return c->hipfail(e, "device allocation");
    }
    size_t tmp = 0;
    pv_radix_sort_pairs(nullptr, &tmp, c->d_skeys, c->d_skeys2, c->d_svals, c->d_svals2, kc, c->stream);
    c->sort_tmp_bytes = std::max<size_t>(tmp, 256);
    if (!hip_ok(e = hipMalloc(&c->d_sort_tmp, c->sort_tmp_bytes))) { *out = c; return c->hipfail(e, "sort scratch"); }
    *out = c;
    return pv_reset(c);
}

void pv_destroy(pv_ctx *c)
{
    if (c && c->hprof_on)
        fprintf(stderr, "pv_hostprof ms: wait=%.1f index=%.1f cut=%.1f shifts=%.1f kernels=%.1f tcp=%.1f pairs=%.1f tail=%.1f sync=%.1f loop=%.1f | launch=%.1f pend_in=%.1f sort=%.1f resolve=%.1f nv_sync=%.1f | X=%.1f memset=%.1f upload=%.1f launch=%.1f xsync=%.1f\n",
                c->hprof[0], c->hprof[1], c->hprof[2], c->hprof[3], c->hprof[4], c->hprof[5], c->hprof[6], c->hprof[7],
                c->hprof[8], c->hprof[9], c->hprof[14], c->hprof[10], c->hprof[11], c->hprof[12], c->hprof[13], c->hprof[15], c->hprof[16], c->hprof[17], c->hprof[18], c->hprof[19]);
    if (!c) return;
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    if (c->stream) { hipSetDevice(c->device); hipStreamSynchronize(c->stream); }
    void *ptrs[] = {c->d_sum, c->d_cpc, c->d_tkeys, c->d_tcnt, c->d_taux, c->d_arena, c->d_arena_top, c->d_events,
                    c->d_xvh, c->d_skeys, c->d_skeys2, c->d_svals, c->d_svals2, c->d_sort_tmp, c->d_xvals, c->d_status,
                    c->d_valid, c->d_nvals, c->d_params, c->d_xparams, c->d_ekeys, c->d_blk_events, c->d_mq, c->d_tpbuf, c->d_cb, c->d_cb_cnt, c->d_cb_h, c->d_nn, c->d_iplog, c->d_trash, c->d_mq_cnt, c->d_stamps, c->d_dq, c->d_dq_cnt,
                    c->stage[0].d_recs, c->stage[0].d_offs, c->stage[1].d_recs, c->stage[1].d_offs,
                    c->d_pend[0], c->d_pend[1], c->d_pkeys[0], c->d_pkeys[1], c->d_pvals[0], c->d_pvals[1], c->d_orph, c->d_orph_ord, c->d_sfx, c->d_psl,
                    c->d_tseg, c->d_tmask, c->d_tpm, c->d_tcpcnt, c->d_tparams, c->d_tkey[0], c->d_tkey[1], c->d_tval[0],
                    c->d_tval[1], c->d_run_flow, c->d_tsort_tmp, c->d_flows, c->d_carry[0], c->d_carry[1], c->d_clist[0],
                    c->d_clist[1], c->d_frags, c->d_marena, c->d_moffs, c->d_tmq, c->d_tsfx,
                    c->d_theta, c->d_ctmp, c->d_ctop, c->d_ovf, c->d_ovf2, c->d_iplog32,
                    c->d_ipx_rep, c->d_ipdir, c->d_ipx_cnt, c->d_slow, c->d_ecs, c->d_eecs, c->d_pecs[0], c->d_pecs[1], c->d_lru_ev, c->d_fclose,
                    c->d_xcnt, c->d_xrhdr, c->d_xtot, c->d_xsend, c->d_xrecv, c->d_xp, c->d_bpf, c->d_fwork, c->d_frecs,
                    c->d_foffs, c->d_fsc, c->d_fscan, c->d_eoc, c->d_eoc_cnt};
    for (void *p : ptrs) if (p) hipFree(p);
    if (c->d_dbits) hipFree(c->d_dbits);
    for (void *hp : {(void *)c->h_params, (void *)c->h_xparams, (void *)c->h_status, (void *)c->h_dbits, (void *)c->h_tcpcnt,
                     (void *)c->h_tparams})
        if (hp) hipHostFree(hp);
    for (auto &st : c->stage) {
        if (st.d_ix) hipFree(st.d_ix);
        if (st.h_ix) hipHostFree(st.h_ix);
        if (st.h_recs) hipHostFree(st.h_recs);
        if (st.h_offs) hipHostFree(st.h_offs);
        if (st.copied) hipEventDestroy(st.copied);
    }
    for (auto &r : c->ring) {
        if (r.d_buf) hipFree(r.d_buf);
        if (r.d_offs) hipFree(r.d_offs);
        if (r.h_stage) hipHostFree(r.h_stage);
        if (r.landed) hipEventDestroy(r.landed);
    }
    if (c->copy_stream) hipStreamDestroy(c->copy_stream);
    if (c->copy_stream2) hipStreamDestroy(c->copy_stream2);
    if (c->d_ndeep) hipFree(c->d_ndeep);
    if (c->h_ndeep) hipHostFree(c->h_ndeep);
    for (void *p : {(void *)c->d_fbits, (void *)c->d_tfbits, (void *)c->d_ntcp}) if (p) hipFree(p);
    for (void *p : {(void *)c->h_fbits, (void *)c->h_tfbits, (void *)c->h_ntcp}) if (p) hipHostFree(p);
    c->pool.reset();
    if (c->ev_start) hipEventDestroy(c->ev_start);
    if (c->ev_stop) hipEventDestroy(c->ev_stop);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

// TCP: no connection, no carried bytes, no TCP record seen
static void tcp_reset(pv_ctx *c)
{
    launch_fill32(c, c->d_tcpcnt + PVT_WORDS, 1, 0);
    if (c->d_flows) launch_fill32(c, (uint32_t *)c->d_flows, ((uint64_t)sizeof(PvTcpFlow) / 4) << c->flow_cap_log2, 0);
    c->n_clist = 0;
    c->carry_used = 0;
    c->tcp_active = false;
    c->lru.clear();
    c->lru_at.clear();
    c->lru_hold.clear();
}

int pv_reset(pv_ctx *c)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    // device state stays as it is: which slot parts are clean carries over
    for (Window *w : {&c->net, &c->dns}) {
        bool cl[PV_SLOTS];
        memcpy(cl, w->clean, sizeof cl);
        *w = Window();
        memcpy(w->clean, cl, sizeof cl);
    }
    c->started = c->ended = false;
    c->records_seen = 0;
    c->draws_net.reset(Jsf32());
    c->draws_dns.reset(Jsf32());
    c->dns_deep_now = true;
    c->xvals_host.clear();
    c->xvals_synced = 0;
    c->from90 = c->to90 = 0.0f;
    c->p90_2[0] = c->p90_2[1] = c->p90_2[2] = 0.0f;
    c->remote_topn.clear();
    c->x_ranks = c->x_rank = 0;
    c->x_view_on = false;
    c->merged = false;
    c->merged_by = nullptr;
    c->x_view.clear();
    c->xq_on = false;
    c->xq.clear();
    c->n_pend = 0;
    c->pend_hi = 0;
    c->pend_base = -1;
    c->dns_shifts.clear();
    c->sg_ord.clear();
    c->sstore.clear();
    c->scands.clear();
    c->sorph.clear();
    c->orph_done = 0;
    c->xv_local_end = SIZE_MAX;
    c->slow_xv.clear();
    c->stubs.clear();
    c->edge_h = 0;
    c->dns_shift_ord.clear();
    launch_fill32(c, c->d_nvals, 4, 0); // with the next batch's slot clears
    tcp_reset(c);
    return 0;
}

int pv_set_global_base(pv_ctx *c, uint64_t base)
{
    c->global_base = base;
    return 0;
}

int pv_index_records(const uint8_t *recs, size_t bytes, uint32_t ts_nano, uint32_t *offsets, uint64_t max_records,
                     uint32_t *sc_idx, uint32_t *sc_sec, uint32_t max_changes, pv_index_info *info)
{
    (void)ts_nano;
    memset(info, 0, sizeof *info);
    info->monotone = 1;
    size_t pos = 0;
    uint64_t n = 0;
    uint32_t nc = 0;
    int64_t prev_sec = -1;
    while (pos + 16 <= bytes && n < max_records) {
        uint32_t h[4];
        memcpy(h, recs + pos, 16);
        if (pos + 16 + h[2] > bytes) break;
        if (pos > 0xffffffffull) return PV_EINVAL; // offsets are 32-bit: split larger runs
        offsets[n] = (uint32_t)pos;
        int64_t sec = h[0];
        int64_t nsec = ts_nano ? h[1] : (int64_t)h[1] * 1000;
        if (n == 0) { info->first_sec = sec; info->first_nsec = nsec; }
        info->last_sec = sec; info->last_nsec = nsec;
        if (sec != prev_sec) {
            if (sec < prev_sec) info->monotone = 0;
            if (nc < max_changes) { sc_idx[nc] = (uint32_t)n; sc_sec[nc] = (uint32_t)sec; }
            nc++;
            prev_sec = sec;
        }
        pos += 16 + h[2];
        n++;
    }
    info->n_records = n;
    info->bytes_used = pos;
    info->n_sec_changes = nc;
    if (nc > max_changes) return PV_ECAPACITY;
    return 0;
}

namespace {

// A period shift inside a batch: its threshold second (the shifting event's ts_sec) and the
// batch record index of that event (AbstractMetricsManager::new_event, src/AbstractMetricsManager.h:318-333)
struct Shift {
    int64_t sec;
    uint64_t idx;
    uint64_t ord; // DNS shifts: position of the shifting event (record * 4, + sub for a TCP message)
};

// The Net manager's shifts: every packet is a Net event, so the first record with
// ts_sec >= next_shift shifts, then next_shift = its second + 60, repeatedly.
void net_shifts_of(int64_t T, const pv_index_info *info, const uint32_t *sc_idx, const uint32_t *sc_sec,
                   std::vector<Shift> &out)
{
    for (uint32_t k = 0; k < info->n_sec_changes; k++)
        if ((int64_t)sc_sec[k] >= T) {
            out.push_back({(int64_t)sc_sec[k], sc_idx[k], (uint64_t)sc_idx[k] * 4});
            T = (int64_t)sc_sec[k] + 60;
        }
}

uint64_t next_bit(const uint64_t *bits, uint64_t from, uint64_t n)
{
    for (uint64_t w = from >> 6; (w << 6) < n; w++) {
        uint64_t v = bits[w];
        if (w == (from >> 6)) v &= ~0ull << (from & 63);
        if (v) {
            const uint64_t i = (w << 6) + (uint64_t)__builtin_ctzll(v);
            return i < n ? i : n;
        }
    }
    return n;
}

// The DNS manager's shifts: the first DNS event (in stream order) with ts_sec >= next_shift, then
// next_shift = its second + 60, repeatedly (AbstractMetricsManager::new_event, per event: the
// batch's timestamps need not be monotone). DNS events: the UDP datagrams of pv_dns_prescan's
// bits, and the TCP messages (ord, stamp second) of the batch's TCP stage, whose stamps (a
// connection's end time) may lag their position.
void dns_shifts_of(int64_t T, const uint64_t *bits, uint64_t n, const pv_index_info *info, const uint32_t *sc_idx,
                   const uint32_t *sc_sec, const std::vector<std::pair<uint64_t, int64_t>> &tcp, std::vector<Shift> &out)
{
    const uint32_t nsc = info->n_sec_changes;
    uint32_t k = 0;     // the second-run holding record `after / 4`
    size_t t = 0;
    uint64_t after = 0; // events at ord >= after are still candidates
    for (;;) {
        // UDP: the first event at or past `after` whose record's second is >= T, run by run of
        // equal seconds (sc_idx / sc_sec: the batch's change points, in record order)
        const uint64_t from = (after + 3) / 4;
        while (k + 1 < nsc && sc_idx[k + 1] <= from) k++;
        uint64_t ui = n, uord = ~0ull;
        int64_t usec = 0;
        for (uint32_t kk = k; kk < nsc; kk++) {
            if ((int64_t)sc_sec[kk] < T) continue;
            const uint64_t lo = std::max<uint64_t>(sc_idx[kk], from), hi = kk + 1 < nsc ? sc_idx[kk + 1] : n;
            if (lo >= hi) continue;
            const uint64_t i = next_bit(bits, lo, hi);
            if (i < hi) {
                ui = i;
                usec = (int64_t)sc_sec[kk];
                uord = ui * 4;
                break;
            }
        }
        // TCP: the first message after the last shift whose stamp second is >= T
        while (t < tcp.size() && tcp[t].first < after) t++;
        size_t tt = t;
        while (tt < tcp.size() && tcp[tt].second < T && tcp[tt].first < uord) tt++;
        const bool tcp_first = tt < tcp.size() && tcp[tt].second >= T && tcp[tt].first < uord;
        if (tcp_first) {
            out.push_back({tcp[tt].second, tcp[tt].first / 4, tcp[tt].first});
            T = tcp[tt].second + 60;
            after = tcp[tt].first + 1;
            t = tt + 1;
            continue;
        }
        if (uord == ~0ull) return;
        out.push_back({usec, ui, uord});
        T = usec + 60;
        after = uord + 1;
    }
}

// parameter fields every kernel reads: record access, parse configuration, DNS filters
// A parameter block to device memory through pv_store_blob's kernel arguments (blocks up to
// 2 KiB; larger ones by copy)
static hipError_t upload_params(void *dst, const void *src, size_t bytes, hipStream_t st)
{
    if (bytes > sizeof(PvBlob) || ((uintptr_t)dst & 15)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    PvBlob b;
    memcpy(b.w, src, bytes);
    const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
    hipLaunchKernelGGL(pv_store_blob, dim3(1), dim3(PV_BLOB_WORDS), 0, st, b, (uint4 *)dst, n16);
    return hipGetLastError();
}

// The queued fills and a parameter block in one launch (pv_fill_store) when both fit; else the
// fills, then upload_params
static hipError_t fill_and_upload(pv_ctx *c, void *dst, const void *src, size_t bytes, hipStream_t st)
{
    static const char *nofuse = getenv("PV_FILL_FUSE"); // (=0: separate launches, A/B runs)
    if (!c->fills.n || st != c->stream || bytes > sizeof(PvBlob) || ((uintptr_t)dst & 15) || (nofuse && !strcmp(nofuse, "0"))) {
        flush_fills(c);
        return upload_params(dst, src, bytes, st);
    }
    PvBlob b;
    memcpy(b.w, src, bytes);
    const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
    hipSetDevice(c->device);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((c->fills_max + 255) / 256, 4096);
    static_assert(PV_BLOB_WORDS <= 256, "the blob's words in the first workgroup");
    hipLaunchKernelGGL(pv_fill_store, dim3(blocks), dim3(256), 0, c->stream, c->fills, b, (uint4 *)dst, n16);
    c->fills.n = 0;
    c->fills_max = 0;
    return hipGetLastError();
}

} // namespace
namespace pvh {
void params_common(pv_ctx *c, PvParams &P, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n)
{
    memset(&P, 0, sizeof P);
    P.recs = d_recs;
    P.offs = d_offs;
    P.n = n;
    P.linktype = c->cfg.linktype;
    P.ts_nano = c->cfg.ts_nano;
    P.net_groups = c->net_groups;
    P.dns_groups = c->dns_groups;
    P.net2_groups = c->net2_groups;
    P.dns2_groups = c->dns2_groups;
    P.net_filter_all = c->cfg.net_filter_all ? 1u : 0u;
    P.nets = c->nets;
    P.f_flags = c->f_flags;
    P.f_rcode_mask = c->f_rcode_mask;
    P.f_ancount = c->f_ancount;
    P.f_nq = c->f_nq;
    for (uint32_t k = 0; k < c->f_nq; k++) P.f_qt[k] = c->f_qt[k];
    P.f_nqn = c->f_nqn;
    for (uint32_t k = 0; k < c->f_nqn; k++) P.f_qn[k] = c->f_qn[k];
    P.f_nsx = c->f_nsx;
    P.sfx_of = c->d_sfx;
    P.psl = c->d_psl;
    for (uint32_t k = 0; k < c->f_nsx; k++) { P.f_sxl[k] = c->f_sxl[k]; P.f_sxh[k] = c->f_sxh[k]; }
    P.dbits = c->d_dbits;
    P.tseg = c->d_tseg;
    P.tseg_cap = c->tseg_cap;
    P.tseg_cnt = c->d_status + ST_TSEG;
    P.tmask = c->d_tmask;
}
} // namespace pvh
namespace {

// pv_dns_prescan over a batch, its bits copied to c->h_dbits (synchronises); with tcp_emit
// also the batch's TCP segments and tile masks (their counts into tseg[2])
int dns_prescan(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n, hipStream_t st, bool tcp_emit,
                uint32_t *tseg, bool fbits = false)
{
    launch_fill32(c, c->d_status + ST_TSEG, 2, 0);
    flush_fills(c);
    PvParams P;
    params_common(c, P, d_recs, d_offs, n);
    // 2: every TCP connection, 4: every TCP packet (the exact LRU mode: the LRU holds every
    // connection and runs its cleanup after every TCP packet)
    P.tcp_emit = tcp_emit ? (c->tcp_exact_on() ? 7u : 1u) : 0u;
    if (fbits) P.fbits = c->d_fbits;
    hipError_t e;
    *c->h_params = P;
    if (!hip_ok(e = upload_params(c->d_params, c->h_params, sizeof P, st)))
        return c->hipfail(e, "parameter upload");
    const uint64_t tiles = (n + 63) / 64;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((tiles + 3) / 4, (uint64_t)c->cus * 8);
    hipLaunchKernelGGL(pv_dns_prescan, dim3(grid), dim3(256), 0, st, (const PvParams *)c->d_params);
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_dns_prescan");
    if (!hip_ok(e = hipMemcpyAsync(c->h_dbits, c->d_dbits, tiles * 8, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(c->h_status + ST_TSEG, c->d_status + ST_TSEG, 8, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "DNS prescan");
    tseg[0] = c->h_status[ST_TSEG];
    tseg[1] = c->h_status[ST_TSEG_BYTES];
    if (fbits && (!hip_ok(e = hipMemcpyAsync(c->h_fbits, c->d_fbits, tiles * 8, hipMemcpyDeviceToHost, st)) ||
                  !hip_ok(e = hipStreamSynchronize(st))))
        return c->hipfail(e, "DNS filter prescan");
    return 0;
}

// ---- DNS over TCP (pv_tcp.hip)
int grow_bytes(pv_ctx *c, void **p, uint64_t &cap, uint64_t need, size_t elem, const char *what)
{
    if (need <= cap && *p) return 0;
    if (*p) hipFree(*p);
    *p = nullptr;
    cap = 0;
    const uint64_t n = std::max<uint64_t>(need + need / 2, 1u << 16);
    hipError_t e;
    if (!hip_ok(e = hipMalloc(p, n * elem))) return c->hipfail(e, what);
    cap = n;
    return 0;
}
#define PV_GROW(c, p, cap, need, what) grow_bytes(c, (void **)&(p), cap, need, sizeof(*(p)), what)

// the stage's fixed buffers, on the first batch that holds a DNS-port TCP segment
int tcp_alloc(pv_ctx *c)
{
    if (c->tcp_alloced) return 0;
    hipError_t e;
    const uint64_t ns = c->tseg_cap, fc = 1ull << c->flow_cap_log2;
    if (!hip_ok(e = hipMalloc(&c->d_tkey[0], ns * 8)) || !hip_ok(e = hipMalloc(&c->d_tkey[1], ns * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tval[0], ns * 4)) || !hip_ok(e = hipMalloc(&c->d_tval[1], ns * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_run_flow, ns * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_flows, fc * sizeof(PvTcpFlow))) ||
        !hip_ok(e = hipMemsetAsync(c->d_flows, 0, fc * sizeof(PvTcpFlow), c->stream)) ||
        !hip_ok(e = hipMalloc(&c->d_clist[0], fc * 4)) || !hip_ok(e = hipMalloc(&c->d_clist[1], fc * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_moffs, (size_t)c->tmsg_cap * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_tmq, (size_t)c->tmsg_cap * 32)) ||
        !hip_ok(e = hipMalloc(&c->d_tsfx, (size_t)c->tmsg_cap)))
        return c->hipfail(e, "TCP stage allocation");
    size_t tmp = 0;
    pv_tcp_sort(nullptr, &tmp, c->d_tkey[0], c->d_tkey[1], c->d_tval[0], c->d_tval[1], ns, c->stream);
    c->tsort_tmp_bytes = std::max<size_t>(tmp, 256);
    if (!hip_ok(e = hipMalloc(&c->d_tsort_tmp, c->tsort_tmp_bytes))) return c->hipfail(e, "TCP sort scratch");
    c->tcp_alloced = true;
    return 0;
}

// PcapInputStream's LRU list in the exact LRU mode (PcapInputStream.cpp:97-99,254-283,429-465),
// replayed over the batch's segments (every TCP packet) in capture order from the dry run's events
// (skey: sorted fkey << 32 | record index; sval: segment index per sorted key; ev per sorted key:
// flags | dir << 8, second, LRU time of the segment's last put). Per packet, as the reference: the
// reassembly's puts (a connection start with its start second, a message delivery with endTime,
// which is 0 until the connection's second packet) move the connection to the head and, past the
// limit, evict the tail; a FIN/RST close erases it; then at most MAX_TCP_CLEANUPS (100) connections
// leave from the tail while the tail's time + 30 s <= the packet's second, then the evicted ones
// close. Every connection closed this way is closed after that record (closeConnection): fclose
// (per segment index) at its first sorted segment when it has packets in the batch (its later
// packets are then Ignore_PacketOfClosedFlow, and their events are skipped here), else a
// close-only segment appended to `extra` with its fclose in `extra_fc`. A connection whose close
// flushes held fragments is put into the list once more by that delivery before its end erases
// it (PcapInputStream.cpp:254-263,276-283): an evicted one can evict the next tail that way,
// which the same overflow loop then closes.
void tcp_lru_replay(pv_ctx *c, const std::vector<uint64_t> &skey, const std::vector<uint32_t> &sval,
                    const std::vector<uint32_t> &ev, std::vector<uint32_t> &fclose, std::vector<PvTcpSeg> &extra,
                    std::vector<uint32_t> &extra_fc)
{
    static constexpr int MAX_TCP_CLEANUPS = 100; // PcapInputStream.h:98
    const size_t n = skey.size();
    std::vector<uint32_t> order(n);
    std::unordered_map<uint32_t, uint32_t> first; // flow -> its first sorted segment
    for (size_t k = 0; k < n; k++) {
        order[k] = (uint32_t)k;
        if (!k || (skey[k] >> 32) != (skey[k - 1] >> 32)) first[(uint32_t)(skey[k] >> 32)] = (uint32_t)k;
    }
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return (uint32_t)skey[a] < (uint32_t)skey[b]; });
    auto erase = [&](uint32_t f) {
        auto it = c->lru_at.find(f);
        if (it == c->lru_at.end()) return;
        c->lru.erase(it->second);
        c->lru_at.erase(it);
    };
    std::unordered_map<uint32_t, bool> closed; // closed by the replay in this batch
    std::vector<uint32_t> overflow;
    auto put = [&](uint32_t f, uint32_t t) {
        erase(f);
        c->lru.emplace_front(f, t);
        c->lru_at[f] = c->lru.begin();
        if (c->tcp_limit && c->lru_at.size() > c->tcp_limit) {
            const uint32_t v = c->lru.back().first;
            c->lru_at.erase(v);
            c->lru.pop_back();
            overflow.push_back(v);
        }
    };
    auto close_after = [&](uint32_t v, uint32_t idx, uint32_t sec, uint32_t dir) {
        if (closed.count(v)) { erase(v); return; }
        closed[v] = true;
        // the flush's put (its time is moot: the connection's end erases it next)
        if (c->lru_hold.erase(v)) put(v, 0);
        erase(v);
        auto it = first.find(v);
        if (it != first.end()) {
            uint32_t *w = &fclose[3 * (size_t)sval[it->second]];
            w[0] = idx; w[1] = sec; w[2] = dir;
            return;
        }
        PvTcpSeg g;
        memset(&g, 0, sizeof g);
        g.idx = idx;
        g.fkey = v;
        g.sec = sec;
        g.flags = PV_TF_CLOSE;
        g.dirv6 = (uint8_t)dir;
        extra.push_back(g);
        extra_fc.insert(extra_fc.end(), {idx, sec, dir});
    };
    for (uint32_t k : order) {
        const uint32_t f = (uint32_t)(skey[k] >> 32), idx = (uint32_t)skey[k];
        const uint32_t fl = ev[3 * k] & 0xff, dir = (ev[3 * k] >> 8) & 3, sec = ev[3 * k + 1], pt = ev[3 * k + 2];
        if (!closed.count(f)) {
            if (fl & PVT_EV_NEW) put(f, sec);
            if (fl & PVT_EV_PUT) put(f, pt);
            if (fl & PVT_EV_CLOSE) erase(f);
            if (fl & PVT_EV_HOLD) c->lru_hold.insert(f);
            else c->lru_hold.erase(f);
        }
        for (int q = 0; q < MAX_TCP_CLEANUPS && !c->lru.empty(); q++) {
            const auto back = c->lru.back();
            if ((uint64_t)sec < (uint64_t)back.second + PV_TCP_TIMEOUT) break;
            close_after(back.first, idx, sec, dir);
        }
        // indexed: a close's put may append the next eviction
        for (size_t q = 0; q < overflow.size(); q++) close_after(overflow[q], idx, sec, dir);
        overflow.clear();
    }
}

// The segment arrays of the TCP stage for `need` segments (the end of a capture adds one per open
// connection to a batch's own), the first `keep` segments kept
int tcp_grow_segs(pv_ctx *c, uint64_t need, uint32_t keep, hipStream_t st)
{
    if (need <= c->tseg_cap) return 0;
    if (need > 0xffffffffull) return c->fail(PV_ECAPACITY, "TCP segments");
    hipError_t e;
    PvTcpSeg *seg = nullptr;
    if (!hip_ok(e = hipMalloc(&seg, need * sizeof(PvTcpSeg))) ||
        (keep && !hip_ok(e = hipMemcpyAsync(seg, c->d_tseg, (size_t)keep * sizeof(PvTcpSeg), hipMemcpyDeviceToDevice, st))) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "TCP segments");
    hipFree(c->d_tseg);
    c->d_tseg = seg;
    for (int k = 0; k < 2; k++) {
        hipFree(c->d_tkey[k]);
        hipFree(c->d_tval[k]);
        c->d_tkey[k] = nullptr;
        c->d_tval[k] = nullptr;
    }
    hipFree(c->d_run_flow);
    hipFree(c->d_tsort_tmp);
    c->d_run_flow = nullptr;
    c->d_tsort_tmp = nullptr;
    if (!hip_ok(e = hipMalloc(&c->d_tkey[0], need * 8)) || !hip_ok(e = hipMalloc(&c->d_tkey[1], need * 8)) ||
        !hip_ok(e = hipMalloc(&c->d_tval[0], need * 4)) || !hip_ok(e = hipMalloc(&c->d_tval[1], need * 4)) ||
        !hip_ok(e = hipMalloc(&c->d_run_flow, need * 4)))
        return c->hipfail(e, "TCP segments");
    size_t tmp = 0;
    pv_tcp_sort(nullptr, &tmp, c->d_tkey[0], c->d_tkey[1], c->d_tval[0], c->d_tval[1], need, st);
    c->tsort_tmp_bytes = std::max<size_t>(tmp, 256);
    if (!hip_ok(e = hipMalloc(&c->d_tsort_tmp, c->tsort_tmp_bytes))) return c->hipfail(e, "TCP sort scratch");
    c->tseg_cap = (uint32_t)need;
    return 0;
}

// The TCP stage of a batch: its segments (n_seg, seg_bytes payload) through reassembly and
// framing into message records. d_offs / n: the whole batch. With want_ords the messages'
// (ord, second) pairs come back for the DNS shift plan.
int tcp_stage(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n, uint32_t n_seg, uint64_t seg_bytes,
              uint32_t now_sec, bool want_ords, hipStream_t st)
{
    c->tcp_nmsg = 0;
    c->tcp_ords.clear();
    if (n_seg > c->tseg_cap)
        return c->fail(PV_ECAPACITY, "%u DNS-over-TCP segments in one batch exceed the capacity %u (max_records)", n_seg,
                       c->tseg_cap);
    const bool eoc = c->eoc_stage && n > 0;
    c->eoc_stage = false;
    if (n_seg == 0 && !c->tcp_active) return 0;
    if (int rc = tcp_alloc(c)) return rc;
    hipError_t e;
    // bounds of this stage's output: every byte a flow can deliver (payloads, carried bytes,
    // missing-data texts) lands in at most one message record, reserved at most three times
    const uint64_t B = seg_bytes + c->carry_used + 32ull * (n_seg + c->carry_used / 8);
    if (int rc = PV_GROW(c, c->d_marena, c->marena_cap, 3 * B + 44 * (B / 17 + 2ull * n_seg) + 4096 + PV_RECS_PAD, "TCP message arena"))
        return rc;
    uint64_t fcap = c->frag_cap;
    if (int rc = PV_GROW(c, c->d_frags, fcap, n_seg + c->carry_used / 8 + 64, "TCP fragment pool")) return rc;
    c->frag_cap = (uint32_t)std::min<uint64_t>(fcap, 0xffffffffull);
    const uint32_t out = c->carry_cur ^ 1;
    if (int rc = PV_GROW(c, c->d_carry[out], c->carry_cap[out], 2 * B + 8 * (n_seg + c->carry_used / 8) + 4096, "TCP carry arena"))
        return rc;
    if (!c->d_carry[c->carry_cur]) {
        if (int rc = PV_GROW(c, c->d_carry[c->carry_cur], c->carry_cap[c->carry_cur], 4096, "TCP carry arena")) return rc;
    }
    c->tcp_stage++;
    PvTcpParams &T = *c->h_tparams;
    memset(&T, 0, sizeof T);
    T.seg = c->d_tseg;
    T.skey = c->d_tkey[1];
    T.sval = c->d_tval[1];
    T.n_seg = n_seg;
    T.stage = c->tcp_stage;
    T.now_sec = now_sec;
    T.flow_cap_log2 = c->flow_cap_log2;
    T.flows = c->d_flows;
    T.run_flow = c->d_run_flow;
    T.tmask = c->d_tmask;
    T.tpm = c->d_tpm;
    T.lt_carry = c->d_tcpcnt + PVT_WORDS;
    T.recs = d_recs;
    T.offs = d_offs;
    T.n_tiles = (uint32_t)((n + 63) / 64);
    T.ts_nano = c->cfg.ts_nano;
    T.carry_in = c->d_carry[c->carry_cur];
    T.carry_out = c->d_carry[out];
    T.carry_cap = c->carry_cap[out];
    T.clist_in = c->d_clist[c->carry_cur];
    T.n_clist_in = c->n_clist;
    T.clist_out = c->d_clist[out];
    T.frags = c->d_frags;
    T.frag_cap = c->frag_cap;
    T.marena = c->d_marena;
    T.marena_cap = c->marena_cap;
    T.moffs = c->d_moffs;
    T.mq = c->d_tmq;
    T.mq_cap = c->tmsg_cap;
    T.cnt = c->d_tcpcnt;
    flush_fills(c);
    const PvTcpParams *dT = c->d_tparams;
    uint32_t blocks = (n_seg + 255) / 256;
    // one run of the stage's kernels (dry: the exact LRU replay's recording run)
    auto run = [&](bool dry) -> int {
        T.dry = dry ? 1u : 0u;
        if (!hip_ok(e = hipMemsetAsync(c->d_tcpcnt, 0, PVT_WORDS * 4, st)) ||
            !hip_ok(e = upload_params(c->d_tparams, c->h_tparams, sizeof T, st)))
            return c->hipfail(e, "TCP stage upload");
        hipLaunchKernelGGL(pv_tcp_scan, dim3(1), dim3(1024), 0, st, dT);
        if (n_seg) {
            {
                hipLaunchKernelGGL(pv_tcp_keys, dim3(blocks), dim3(256), 0, st, (const PvTcpSeg *)c->d_tseg, n_seg, c->d_tkey[0],
                                   c->d_tval[0]);
                size_t tmp = c->tsort_tmp_bytes;
                if (!hip_ok(e = pv_tcp_sort(c->d_tsort_tmp, &tmp, c->d_tkey[0], c->d_tkey[1], c->d_tval[0], c->d_tval[1], n_seg, st)))
                    return c->hipfail(e, "TCP segment sort");
            }
            hipLaunchKernelGGL(pv_tcp_lookup, dim3(blocks), dim3(256), 0, st, dT);
            hipLaunchKernelGGL(pv_tcp_insert, dim3(blocks), dim3(256), 0, st, dT);
            hipLaunchKernelGGL(pv_tcp_flow, dim3(blocks), dim3(256), 0, st, dT);
            if (c->n_clist && !dry) hipLaunchKernelGGL(pv_tcp_migrate, dim3((c->n_clist + 255) / 256), dim3(256), 0, st, dT);
        }
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch TCP stage");
        return 0;
    };
    T.exact = c->tcp_exact_on() ? 1u : 0u;
    if (T.exact && n_seg) {
        // the exact LRU mode: record the segments' LRU events, replay the LRU list on the host,
        // then run the stage with the closes it found (close-only segments behind the batch's)
        if (int rc = PV_GROW(c, c->d_lru_ev, c->lru_ev_cap, 3ull * n_seg, "TCP LRU events")) return rc;
        T.lru_ev = c->d_lru_ev;
        T.fclose = nullptr;
        if (int rc = run(true)) return rc;
        std::vector<uint64_t> skey(n_seg);
        std::vector<uint32_t> sval(n_seg), ev(3ull * n_seg);
        if (!hip_ok(e = hipMemcpyAsync(skey.data(), c->d_tkey[1], (size_t)n_seg * 8, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipMemcpyAsync(sval.data(), c->d_tval[1], (size_t)n_seg * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipMemcpyAsync(ev.data(), c->d_lru_ev, ev.size() * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "TCP LRU events");
        std::vector<uint32_t> fclose(3ull * n_seg, PVT_FCLOSE_NONE), extra_fc;
        std::vector<PvTcpSeg> extra;
        tcp_lru_replay(c, skey, sval, ev, fclose, extra, extra_fc);
        if (!extra.empty()) {
            if (n_seg + extra.size() > c->tseg_cap)
                return c->fail(PV_ECAPACITY, "%u TCP segments and %zu LRU closes in one batch exceed the capacity %u (max_records)",
                               n_seg, extra.size(), c->tseg_cap);
            fclose.insert(fclose.end(), extra_fc.begin(), extra_fc.end());
            if (!hip_ok(e = hipMemcpyAsync(c->d_tseg + n_seg, extra.data(), extra.size() * sizeof(PvTcpSeg), hipMemcpyHostToDevice, st)))
                return c->hipfail(e, "TCP LRU closes");
            n_seg += (uint32_t)extra.size();
            T.n_seg = n_seg;
            blocks = (n_seg + 255) / 256;
        }
        if (int rc = PV_GROW(c, c->d_fclose, c->fclose_cap, 3ull * n_seg, "TCP LRU closes")) return rc;
        if (!hip_ok(e = hipMemcpyAsync(c->d_fclose, fclose.data(), fclose.size() * 4, hipMemcpyHostToDevice, st)))
            return c->hipfail(e, "TCP LRU closes");
        c->tcp_stage++;
        T.stage = c->tcp_stage;
        T.lru_ev = nullptr;
        T.fclose = c->d_fclose;
        if (!hip_ok(e = hipStreamSynchronize(st))) return c->hipfail(e, "TCP LRU closes");
    }
    if (eoc) {
        // TcpReassembly::closeAllConnections after the capture's last record (PcapInputStream.cpp:522,
        // :244 on stop): a close segment for every open connection, with the last record's time and
        // the direction the input cached for it (_packet_dir_cache, :399-416)
        const uint32_t ncap = 1u << c->flow_cap_log2;
        const uint64_t ncand = (uint64_t)ncap + n_seg;
        uint32_t set_log2 = 4;
        while ((1ull << set_log2) < 2 * ncand) set_log2++;
        if (ncand > c->eoc_cap) {
            if (c->d_eoc) (void)hipFree(c->d_eoc);
            c->d_eoc = nullptr;
            c->eoc_cap = 0;
            if (!hip_ok(e = hipMalloc(&c->d_eoc, (size_t)ncand * sizeof(PvTcpSeg)))) return c->hipfail(e, "TCP end-of-capture segments");
            c->eoc_cap = ncand;
        }
        if (!c->d_eoc_cnt && !hip_ok(e = hipMalloc(&c->d_eoc_cnt, 4))) return c->hipfail(e, "TCP end-of-capture segments");
        uint64_t *d_set = nullptr;
        struct SetFree {
            uint64_t *&p;
            ~SetFree() { if (p) (void)hipFree(p); }
        } set_free{d_set};
        if (!hip_ok(e = hipMalloc((void **)&d_set, (size_t)8 << set_log2)) ||
            !hip_ok(e = hipMemsetAsync(d_set, 0, (size_t)8 << set_log2, st)))
            return c->hipfail(e, "TCP end-of-capture key set");
        uint32_t lo = 0;
        uint8_t rec[16 + 512];
        memset(rec, 0, sizeof rec);
        if (!hip_ok(e = hipMemcpyAsync(&lo, d_offs + (n - 1), 4, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)) ||
            !hip_ok(e = hipMemcpyAsync(rec, d_recs + lo, 16, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "last record");
        uint32_t hdr[4];
        memcpy(hdr, rec, 16);
        const uint32_t cap = std::min<uint32_t>(hdr[2], 512);
        if (cap && (!hip_ok(e = hipMemcpyAsync(rec + 16, d_recs + lo + 16, cap, hipMemcpyDeviceToHost, st)) ||
                    !hip_ok(e = hipStreamSynchronize(st))))
            return c->hipfail(e, "last record");
        PvParams P;
        params_common(c, P, d_recs, d_offs, n);
        pvname::Parsed o;
        pvname::parse_record(pvname::HostRecs{rec, 16 + (size_t)cap}, pvname::parse_cfg(P), P, 0, o);
        const uint32_t usec = c->cfg.ts_nano ? hdr[1] / 1000u : hdr[1];
        if (!hip_ok(e = hipMemsetAsync(c->d_eoc_cnt, 0, 4, st)) || !hip_ok(e = upload_params(c->d_tparams, c->h_tparams, sizeof T, st)))
            return c->hipfail(e, "TCP end of capture");
        hipLaunchKernelGGL(pv_tcp_eoc, dim3((uint32_t)((ncand + 255) / 256)), dim3(256), 0, st, dT, (const PvTcpSeg *)c->d_tseg, n_seg,
                           d_set, (uint32_t)((1ull << set_log2) - 1), c->d_eoc, c->d_eoc_cnt, (uint32_t)(n - 1), hdr[0], usec,
                           (uint32_t)o.dir);
        uint32_t ne = 0;
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(&ne, c->d_eoc_cnt, 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "TCP end of capture");
        if (ne) {
            if (int rc = tcp_grow_segs(c, (uint64_t)n_seg + ne, n_seg, st)) return rc;
            if (!hip_ok(e = hipMemcpyAsync(c->d_tseg + n_seg, c->d_eoc, (size_t)ne * sizeof(PvTcpSeg), hipMemcpyDeviceToDevice, st)))
                return c->hipfail(e, "TCP end of capture");
            if (T.fclose) {
                // (the exact LRU mode's closes are per segment: none for these)
                std::vector<uint32_t> none(3ull * ne, PVT_FCLOSE_NONE);
                if (int rc = PV_GROW(c, c->d_fclose, c->fclose_cap, 3ull * (n_seg + ne), "TCP LRU closes")) return rc;
                if (!hip_ok(e = hipMemcpyAsync(c->d_fclose + 3ull * n_seg, none.data(), none.size() * 4, hipMemcpyHostToDevice, st)) ||
                    !hip_ok(e = hipStreamSynchronize(st)))
                    return c->hipfail(e, "TCP end of capture");
                T.fclose = c->d_fclose;
            }
            n_seg += ne;
            T.n_seg = n_seg;
            T.seg = c->d_tseg;
            T.skey = c->d_tkey[1];
            T.sval = c->d_tval[1];
            T.run_flow = c->d_run_flow;
            blocks = (n_seg + 255) / 256;
        }
    }
    if (int rc = run(false)) return rc;
    if (!hip_ok(e = hipMemcpyAsync(c->h_tcpcnt, c->d_tcpcnt, PVT_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "TCP stage");
    c->tcp_active = true;
    if (!n_seg) return 0; // the TCP record seconds advanced; no flow moved
    const uint32_t *k = c->h_tcpcnt;
    if (k[PVT_FLAGS] & PVT_F_TABLE)
        return c->fail(PV_ECAPACITY, "TCP flow table full (%u entries)", 1u << c->flow_cap_log2);
    if (k[PVT_FLAGS] & PVT_F_MSGS)
        return c->fail(PV_ECAPACITY, "more than %u DNS-over-TCP messages in one batch", c->tmsg_cap);
    if (k[PVT_FLAGS] & (PVT_F_ARENA | PVT_F_CARRY | PVT_F_FRAGS))
        return c->fail(PV_ECAPACITY, "TCP stage buffer overflow (flags 0x%x)", k[PVT_FLAGS]);
    c->tcp_nmsg = k[PVT_NMSG];
    c->n_clist = k[PVT_NCARRY];
    c->carry_used = k[PVT_CARRY];
    c->carry_cur = out;
    if (const char *dp = getenv("PV_TCP_DUMP")) {
        // debug: the batch's messages as "record sub length txid stamp_sec stamp_nsec"
        std::vector<uint32_t> items((size_t)c->tcp_nmsg * 8);
        std::vector<uint8_t> arena(k[PVT_ARENA]);
        if (c->tcp_nmsg) hipMemcpy(items.data(), c->d_tmq, items.size() * 4, hipMemcpyDeviceToHost);
        if (!arena.empty()) hipMemcpy(arena.data(), c->d_marena, arena.size(), hipMemcpyDeviceToHost);
        if (FILE *f = fopen(dp, "a")) {
            for (uint32_t q = 0; q < c->tcp_nmsg; q++) {
                const uint32_t *it = &items[(size_t)q * 8];
                const uint32_t mo = it[1];
                fprintf(f, "%llu %u %u %u %u %u\n", (unsigned long long)(c->records_seen + it[7] / 4), it[7] & 3, it[2] & 0xffff,
                        mo + 1 < arena.size() ? (arena[mo] << 8 | arena[mo + 1]) : 0u, it[5], it[6]);
            }
            fclose(f);
        }
    }
    if (want_ords && c->tcp_nmsg) {
        std::vector<uint32_t> items((size_t)c->tcp_nmsg * 8);
        if (!hip_ok(e = hipMemcpy(items.data(), c->d_tmq, items.size() * 4, hipMemcpyDeviceToHost)))
            return c->hipfail(e, "TCP message order");
        c->tcp_ords.resize(c->tcp_nmsg);
        for (uint32_t q = 0; q < c->tcp_nmsg; q++) c->tcp_ords[q] = {items[(size_t)q * 8 + 7], (int64_t)items[(size_t)q * 8 + 5]};
        std::sort(c->tcp_ords.begin(), c->tcp_ords.end());
        c->tcp_items.resize(c->tcp_nmsg);
        for (uint32_t q = 0; q < c->tcp_nmsg; q++) c->tcp_items[q] = {items[(size_t)q * 8 + 7], q};
        std::sort(c->tcp_items.begin(), c->tcp_items.end());
    }
    return 0;
}

// The TCP DNS pass of a span: the batch's messages with ord in [4 * a, 4 * b), events in
// the workgroup regions behind the span's grid; returns the workgroups it used
uint32_t tcp_pass(pv_ctx *c, const PvParams &P, uint64_t a, uint64_t b, hipStream_t st, PvParams *d_slot)
{
    if (!c->tcp_nmsg) return 0;
    PvParams Q = P;
    Q.recs = c->d_marena;
    Q.offs = c->d_moffs;
    Q.linktype = 101;
    Q.dq = c->d_tmq;
    Q.sfx_of = c->d_tsfx;
    Q.tcp_pass = 1;
    Q.ndeep_dns = c->sample_rate < 100 ? c->d_ntcp : nullptr; // per message item (pv_dns_tcp)
    Q.tcp_emit = 0;
    Q.tcp_nmsg = c->tcp_nmsg;
    Q.ord_lo = (uint32_t)(a * 4);
    Q.ord_hi = (uint32_t)std::min<uint64_t>(b * 4, 0xffffffffull);
    Q.ord_base = (uint32_t)(a * 4);
    const uint64_t region = (uint64_t)P.wt_per_block * 64;
    const uint32_t gt = (uint32_t)((c->tcp_nmsg + region - 1) / region);
    *d_slot = Q; // pinned host staging of the second parameter block
    hipMemcpyAsync(c->d_params + 1, d_slot, sizeof Q, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(pv_dns_tcp, dim3(gt), dim3(256), 0, st, (const PvParams *)(c->d_params + 1));
    return gt;
}

// One device batch with at most PV_MAX_SHIFTS shifts of each manager. nsh / dsh: the Net and
// DNS shifts inside it (record indices relative to d_offs).
// Bounded top-N (the frequent-items sketch's purge as TopN uses it, src/Metrics.h:488-503):
// a table holding more than half its capacity after a batch has each region purged at its
// median count (pv_topn_purge); the thetas become the estimate offsets read_topn adds. The
// name arena of a purged table is compacted once its fullest partition is half used. The
// live counts are the ones read back with the batch status (names added by the transaction
// pass afterwards are counted at the next batch).
int purge_table(pv_ctx *c, uint32_t t, hipStream_t st, const PvParams *dP = nullptr);
int purge_tables(pv_ctx *c, hipStream_t st)
{
    const uint64_t tcap = 1ull << c->tcap_log2;
    for (uint32_t t = 0; t < PV_TABLES; t++) {
        if (c->h_tab_live[t] <= tcap / 2) continue;
        if (int rc = purge_table(c, t, st)) return rc;
    }
    return 0;
}

// Updates full regions could not take in this batch (PvOvf list): purge each table they belong
// to, as the sketch purges when its map is full, and insert them again, until none is left.
// Each round at least halves the live entries of every region it purges, so the rounds end.
// known: c->h_ovf already holds the words (read back with the batch status).
} // namespace
namespace pvh {
int drain_overflow(pv_ctx *c, hipStream_t st, bool known, bool *drained, const PvParams *dP)
{
    if (!dP) dP = c->d_params;
    hipError_t e;
    for (int round = 0;; round++) {
        uint32_t oc[2];
        if (!(known && round == 0) &&
            (!hip_ok(e = hipMemcpyAsync(c->h_ovf, c->d_ovf_cnt, 8, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st))))
            return c->hipfail(e, "top-N overflow");
        memcpy(oc, c->h_ovf, 8);
        if (!oc[0]) return 0;
        if (drained) *drained = true;
        if (oc[0] > c->ovf_cap) return c->fail(PV_ECAPACITY, "top-N overflow list full (%u updates)", oc[0]);
        if (round >= 64) return c->fail(PV_ECAPACITY, "top-N overflow not drained after %d purge rounds", round);
        for (uint32_t t = 0; t < PV_TABLES; t++)
            if ((oc[1] >> t) & 1)
                if (int rc = purge_table(c, t, st, dP)) return rc;
        if (!hip_ok(e = hipMemcpyAsync(c->d_ovf2, c->d_ovf, (size_t)oc[0] * sizeof(PvOvf), hipMemcpyDeviceToDevice, st)) ||
            !hip_ok(e = hipMemsetAsync(c->d_ovf_cnt, 0, 8, st)))
            return c->hipfail(e, "top-N overflow");
        hipLaunchKernelGGL(pv_topn_retry, dim3((oc[0] + 255) / 256), dim3(256), 0, st, dP, c->d_ovf2, oc[0]);
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_topn_retry");
        c->ovf_rounds++;
    }
}
} // namespace pvh
namespace {

int purge_table(pv_ctx *c, uint32_t t, hipStream_t st, const PvParams *dP)
{
    if (!dP) dP = c->d_params;
    const uint32_t nreg = 1u << c->reg_log2;
    hipError_t e;
    {
        c->h_tab_live[t] = 0; // stale until the next batch reads the device count back
        hipLaunchKernelGGL(pv_topn_purge, dim3(nreg), dim3(1024), 0, st, dP, t, c->d_theta);
        std::vector<uint32_t> th(nreg);
        uint64_t tops[PV_ARENA_PARTS];
        if (!hip_ok(e = hipGetLastError()) ||
            !hip_ok(e = hipMemcpyAsync(th.data(), c->d_theta, nreg * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipMemcpyAsync(tops, c->d_arena_top + (uint64_t)t * PV_ARENA_PARTS, sizeof tops, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "top-N purge");
        std::vector<uint64_t> &ro = c->roff[t];
        ro.resize(nreg, 0);
        for (uint32_t r = 0; r < nreg; r++) ro[r] += th[r];
        c->purges++;
        const uint64_t pcap = c->arena_cap / PV_ARENA_PARTS;
        uint64_t most = 0;
        for (uint64_t u : tops) most = std::max(most, u);
        if (most <= pcap / 2) return 0;
        if (!c->d_ctmp) {
            if (!hip_ok(e = hipMalloc(&c->d_ctmp, c->arena_cap)) || !hip_ok(e = hipMalloc(&c->d_ctop, PV_ARENA_PARTS * 8)))
                return c->hipfail(e, "arena compaction scratch");
        }
        uint8_t *arena = c->d_arena + (uint64_t)t * c->arena_cap;
        if (!hip_ok(e = hipMemsetAsync(c->d_ctop, 0, PV_ARENA_PARTS * 8, st))) return c->hipfail(e, "arena compaction");
        hipLaunchKernelGGL(pv_topn_compact, dim3((uint32_t)c->cus * 8), dim3(256), 0, st, dP, t, c->d_ctmp, c->d_ctop);
        if (!hip_ok(e = hipGetLastError()) ||
            !hip_ok(e = hipMemcpyAsync(arena, c->d_ctmp, c->arena_cap, hipMemcpyDeviceToDevice, st)) ||
            !hip_ok(e = hipMemcpyAsync(c->d_arena_top + (uint64_t)t * PV_ARENA_PARTS, c->d_ctop, PV_ARENA_PARTS * 8,
                                       hipMemcpyDeviceToDevice, st)))
            return c->hipfail(e, "arena compaction");
    }
    return 0;
}

// Records of `n` batch indices (d_idx[i * stride], PV_TCP_IDX: the TCP message arena) appended
// to the context's slow store; offs_out[i] = each record's offset there
int gather_records(pv_ctx *c, const PvParams &P, const uint32_t *d_idx, uint32_t stride, uint32_t n,
                   std::vector<uint32_t> &offs_out, hipStream_t st)
{
    offs_out.assign(n, 0);
    if (!n) return 0;
    hipError_t e;
    uint32_t *d_sz = nullptr, *d_off = nullptr;
    uint8_t *d_out = nullptr;
    struct Free { void *p[3]; ~Free() { for (void *q : p) if (q) hipFree(q); } } fr{{nullptr, nullptr, nullptr}};
    if (!hip_ok(e = hipMalloc(&d_sz, (size_t)n * 4)) || !hip_ok(e = hipMalloc(&d_off, (size_t)n * 4)))
        return c->hipfail(e, "slow store scratch");
    fr.p[0] = d_sz; fr.p[1] = d_off;
    hipLaunchKernelGGL(pv_rec_sizes, dim3((n + 255) / 256), dim3(256), 0, st, P.recs, P.offs, c->d_marena, c->d_moffs, d_idx, stride,
                       n, d_sz);
    std::vector<uint32_t> sz(n);
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(sz.data(), d_sz, (size_t)n * 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "slow store sizes");
    uint64_t tot = 0;
    std::vector<uint32_t> rel(n);
    for (uint32_t i = 0; i < n; i++) { rel[i] = (uint32_t)tot; tot += sz[i]; }
    if (c->sstore.size() + tot > 0xfffffff0ull) return c->fail(PV_ECAPACITY, "deferred slow-transaction records exceed 4 GiB");
    if (!hip_ok(e = hipMalloc(&d_out, tot ? tot : 4))) return c->hipfail(e, "slow store scratch");
    fr.p[2] = d_out;
    if (!hip_ok(e = hipMemcpyAsync(d_off, rel.data(), (size_t)n * 4, hipMemcpyHostToDevice, st))) return c->hipfail(e, "slow store");
    hipLaunchKernelGGL(pv_rec_gather, dim3((n + 3) / 4), dim3(256), 0, st, P.recs, P.offs, c->d_marena, c->d_moffs, d_idx, stride, n,
                       d_off, d_out);
    const size_t base = c->sstore.size();
    c->sstore.resize(base + tot);
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(c->sstore.data() + base, d_out, tot, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "slow store");
    for (uint32_t i = 0; i < n; i++) offs_out[i] = (uint32_t)(base + rel[i]);
    return 0;
}

// Sharded top_slow (pv_set_slow_defer): the batch's slow-transaction candidates (every valid,
// deep transaction of known direction: the resolve was given no threshold) and its new orphan
// stubs are kept with their response records; pv_slow_finish checks them against the
// thresholds of the whole stream (DnsMetricsManager::on_period_shift, dns/v1/DnsStreamHandler.h:
// 252-267) once the ranks' values are merged.
int defer_slow(pv_ctx *c, const PvParams &P, hipStream_t st)
{
    hipError_t e;
    uint32_t nv[4];
    if (!hip_ok(e = hipMemcpyAsync(nv, c->d_nvals, 16, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "deferred candidates");
    // period k of the span: the k-th DNS shift after the live one (the window bookkeeping of
    // this span's shifts runs after the transaction stage, so the slots' ordinals are not
    // recorded yet)
    (void)P;
    auto ord_of = [&](uint32_t period) -> uint64_t { return c->dns.ordinal + period; };
    if (nv[1]) {
        std::vector<PvXValid> v(nv[1]);
        std::vector<uint32_t> offs;
        if (!hip_ok(e = hipMemcpy(v.data(), c->d_valid, v.size() * sizeof(PvXValid), hipMemcpyDeviceToHost)))
            return c->hipfail(e, "deferred candidates");
        if (int rc = gather_records(c, P, reinterpret_cast<const uint32_t *>(c->d_valid), sizeof(PvXValid) / 4, nv[1], offs, st))
            return rc;
        for (uint32_t i = 0; i < nv[1]; i++)
            if (v[i].dir < 2 || v[i].dir >= 4) // v1 directions, DNS v2's 4 + transaction direction
                c->scands.push_back(pv_ctx::SlowCand{ord_of(v[i].period), v[i].us, offs[i], v[i].dir, (uint8_t)((v[i].idx & PV_TCP_IDX) != 0)});
        const uint32_t zero = 0;
        if (!hip_ok(e = hipMemcpyAsync(c->d_nvals + 1, &zero, 4, hipMemcpyHostToDevice, st))) return c->hipfail(e, "deferred candidates");
    }
    const uint32_t no = std::min(nv[3], c->orph_cap);
    if (nv[3] > c->orph_cap) return c->fail(PV_ECAPACITY, "%u shard-edge stubs exceed the stub capacity", nv[3]);
    if (no > c->orph_done) {
        const uint32_t k = no - c->orph_done;
        std::vector<PvXEvent> o(k);
        std::vector<int64_t> oo(k, 0);
        if (!hip_ok(e = hipMemcpy(o.data(), c->d_orph + c->orph_done, (size_t)k * sizeof(PvXEvent), hipMemcpyDeviceToHost)) ||
            (c->d_orph_ord && !hip_ok(e = hipMemcpy(oo.data(), c->d_orph_ord + c->orph_done, (size_t)k * 8, hipMemcpyDeviceToHost))))
            return c->hipfail(e, "orphan stubs");
        // the records of the responses (an edge pair's top_slow candidate needs its name)
        std::vector<uint32_t> ridx;
        for (auto &x : o)
            if (x.qr) ridx.push_back(x.idx);
        std::vector<uint32_t> offs;
        if (!ridx.empty()) {
            uint32_t *d_idx = nullptr;
            if (!hip_ok(e = hipMalloc(&d_idx, ridx.size() * 4)) ||
                !hip_ok(e = hipMemcpy(d_idx, ridx.data(), ridx.size() * 4, hipMemcpyHostToDevice)))
                return c->hipfail(e, "orphan stubs");
            const int rc = gather_records(c, P, d_idx, 1, (uint32_t)ridx.size(), offs, st);
            hipFree(d_idx);
            if (rc) return rc;
        }
        size_t r = 0;
        for (uint32_t i = 0; i < k; i++) {
            const uint64_t ord = ord_of(o[i].period & 0x3f); // DNS v2 stubs: the kept flag in bit 7
            int64_t cand = -1;
            if (o[i].qr) {
                cand = (int64_t)c->sorph.size();
                c->sorph.push_back(pv_ctx::SlowCand{ord, 0, offs[r++], o[i].dir, (uint8_t)((o[i].idx & PV_TCP_IDX) != 0)});
            }
            c->stubs.push_back(pv_ctx::EdgeStub{o[i], ord, cand, oo[i]});
        }
        c->orph_done = no;
    }
    return hip_ok(e = hipStreamSynchronize(st)) ? 0 : c->hipfail(e, "deferred candidates");
}

// The DNS transaction stage of a batch (TransactionManager state across batches): a batch with
// responses or a DNS period shift pairs (sort + resolve) its nev_b events together with the
// queries carried in; a batch of queries only just appends them to the carried list. Also the
// heartbeat's DNS shift (nev_b = 0, one shift): the carried queries the shift purges time out
// in the new live bucket, the rest carry on.
// The rank values quantile_at(values, r) gives for each kind of PvXvSel among the transaction
// values of slot sg: the device buffer's by radix selection there (pv_xv_hist, eight passes), and
// those a drain already moved to the host (xvals_host ahead of the current device buffer's copy)
// counted into the same histograms. have[k] = the kind has values. Synchronises.
int xv_select(pv_ctx *c, uint32_t sg, double r, bool have[PV_XV_SEL], uint64_t out[PV_XV_SEL])
{
    hipError_t e;
    if (!c->d_xvh && (!hip_ok(e = hipMalloc(&c->d_xvh, PV_XV_SEL * 256 * 4)) ||
                      !hip_ok(e = hipHostMalloc((void **)&c->h_xvh, PV_XV_SEL * 256 * 4, hipHostMallocDefault))))
        return c->hipfail(e, "threshold selection");
    auto kind_of = [](uint32_t kind) {
        return kind == XV_FROM_US ? 0 : kind == XV_TO_US ? 1 : (kind >= XV2_TIME && kind < XV2_TIME + 3) ? 2 + (int)(kind - XV2_TIME) : -1;
    };
    {
        // a value buffer that overflowed holds a truncated value set: fail as sync_xvals does
        uint32_t flags = 0, nv = 0;
        if (!hip_ok(e = hipStreamSynchronize(c->stream)) ||
            !hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost)) ||
            !hip_ok(e = hipMemcpy(&nv, c->d_nvals, 4, hipMemcpyDeviceToHost)))
            return c->hipfail(e, "threshold selection");
        if ((flags & PVF_VALUES_FULL) || nv > c->xv_cap) return c->fail(PV_ECAPACITY, "transaction value buffer full");
    }
    std::vector<uint64_t> hv[PV_XV_SEL];
    const size_t host_only = c->xvals_host.size() - c->xvals_synced;
    for (size_t i = 0; i < host_only; i++) {
        const PvXValue &v = c->xvals_host[i];
        const int k = v.slot == sg ? kind_of(v.kind) : -1;
        if (k >= 0) hv[k].push_back(v.bits);
    }
    PvXvSel sel;
    memset(&sel, 0, sizeof sel);
    uint64_t rank[PV_XV_SEL] = {0};
    for (int pass = 0; pass < 8; pass++) {
        const uint32_t shift = 56 - 8 * pass;
        if (!hip_ok(e = hipMemsetAsync(c->d_xvh, 0, PV_XV_SEL * 256 * 4, c->stream))) return c->hipfail(e, "threshold selection");
        hipLaunchKernelGGL(pv_xv_hist, dim3(std::max<uint32_t>(1u, (uint32_t)c->cus * 2)), dim3(256), 0, c->stream, c->d_xvals, c->d_nvals,
                           (uint32_t)c->xv_cap, sg, shift, sel, c->d_xvh);
        if (!hip_ok(e = hipGetLastError()) ||
            !hip_ok(e = hipMemcpyAsync(c->h_xvh, c->d_xvh, PV_XV_SEL * 256 * 4, hipMemcpyDeviceToHost, c->stream)) ||
            !hip_ok(e = hipStreamSynchronize(c->stream)))
            return c->hipfail(e, "threshold selection");
        const uint64_t hm = shift >= 56 ? 0ull : ~0ull << (shift + 8);
        for (int k = 0; k < PV_XV_SEL; k++) {
            uint64_t h[256];
            for (int b = 0; b < 256; b++) h[b] = c->h_xvh[k * 256 + b];
            for (uint64_t x : hv[k])
                if ((x & hm) == (sel.prefix[k] & hm)) h[(x >> shift) & 255]++;
            if (pass == 0) {
                uint64_t total = 0;
                for (int b = 0; b < 256; b++) total += h[b];
                have[k] = total > 0;
                const uint64_t w = (uint64_t)std::ceil(r * (double)total);
                rank[k] = w == 0 ? 0 : std::min(w - 1, total ? total - 1 : 0);
            }
            if (!have[k]) continue;
            uint64_t cum = 0;
            int b = 0;
            while (b < 255 && cum + h[b] <= rank[k]) cum += h[b++];
            rank[k] -= cum;
            sel.prefix[k] |= (uint64_t)b << shift;
        }
    }
    for (int k = 0; k < PV_XV_SEL; k++) out[k] = sel.prefix[k];
    return 0;
}

int pair_stage(pv_ctx *c, const PvParams &P, uint32_t nev_b, uint32_t nkeys, uint32_t nresp, uint64_t n, hipStream_t st,
               uint64_t ev_hi)
{
    hipError_t e;
    c->ovf_known = false;
    const bool dns_here = nev_b > 0;
    bool pair =(dns_here && (nresp > 0 || P.n_dshift > 0)) || (!dns_here && P.n_dshift > 0 && c->n_pend > 0);
    if (dns_here && !pair && (c->n_pend + nev_b > c->pend_cap || (c->n_pend && c->pend_hi + nev_b > c->ev_store_cap)))
        pair = true; // compact the carried list
    if (dns_here && !pair) {
        const uint32_t cur = c->pend_cur;
        if (c->n_pend == 0 && nkeys == nev_b) {
            // nothing carried: the batch's event store, sorted-key inputs and ECS words become the
            // carried list as they lie (pointer exchange; the next batch writes the other buffers)
            std::swap(c->d_events, c->d_pend[cur]);
            std::swap(c->d_skeys, c->d_pkeys[cur]);
            std::swap(c->d_svals, c->d_pvals[cur]);
            if (c->d_eecs) std::swap(c->d_eecs, c->d_pecs[cur]);
            c->pend_hi = ev_hi;
        } else {
            // (the key list's sentinel slots, messages without an event, are left out)
            if (!hip_ok(e = hipMemsetAsync(c->d_nvals + 2, 0, 4, st))) return c->hipfail(e, "defer counter");
            hipLaunchKernelGGL(pv_xact_defer, dim3((nkeys + 255) / 256), dim3(256), 0, st, c->d_skeys, c->d_svals,
                               c->d_events, nkeys, c->d_pend[cur], c->d_pkeys[cur], c->d_pvals[cur], (uint32_t)c->n_pend,
                               (uint32_t)c->pend_hi, c->d_eecs, c->d_pecs[cur], c->d_nvals + 2);
            if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_xact_defer");
            c->pend_hi += nev_b;
        }
        c->n_pend += nev_b;
    }
    if (pair) {
        const uint32_t np_in = (uint32_t)c->n_pend;
        if (np_in) {
            hipLaunchKernelGGL(pv_xact_pend_in, dim3((np_in + 255) / 256), dim3(256), 0, st, c->d_skeys, c->d_svals,
                               c->d_pkeys[c->pend_cur], c->d_pvals[c->pend_cur], np_in, nkeys);
            if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_xact_pend_in");
        }
        HP(10);
        // sorted: this batch's events and the carried queries first, the sentinel slots behind
        const uint32_t nev = nev_b + np_in;
        uint32_t threads = 256, blocks = (nev + threads - 1) / threads;
        size_t tmp = c->sort_tmp_bytes;
        if (!hip_ok(e = pv_radix_sort_pairs(c->d_sort_tmp, &tmp, c->d_skeys, c->d_skeys2, c->d_svals, c->d_svals2,
                                             (size_t)nkeys + np_in, st)))
            return c->hipfail(e, "radix sort");
        HP(11);
        PvXactParams X;
        memset(&X, 0, sizeof X);
        X.P = P;
        X.events = c->d_events;
        X.skeys = c->d_skeys2;
        X.svals = c->d_svals2;
        X.n = nev;
        X.ttl_s = c->ttl_s;
        X.ttl_ms = c->ttl_ms;
        X.quantiles = ((c->dns_groups & PV_DNS_QUANTILES) ? 1u : 0u) | ((c->dns_groups & PV_DNS_HISTOGRAMS) ? 2u : 0u);
        for (uint32_t k = 0; k <= P.n_dshift; k++) {
            X.slot_gen[k] = P.dslot_of[k] | (c->gen[P.dslot_of[k]] << 8);
            X.thr_from[k] = k == 0 && !c->slow_defer ? c->from90 : -1.0f;
            X.thr_to[k] = k == 0 && !c->slow_defer ? c->to90 : -1.0f;
            for (uint32_t d = 0; d < 3; d++) X.thr2[k][d] = k == 0 && !c->slow_defer ? c->p90_2[d] : -1.0f;
        }
        X.vals = c->d_xvals;
        X.n_vals = c->d_nvals;
        X.vals_cap = (uint32_t)c->xv_cap;
        X.valid = c->d_valid;
        X.n_valid = c->d_nvals + 1;
        X.pend = c->d_pend[c->pend_cur];
        X.pend_out = c->d_pend[c->pend_cur ^ 1];
        X.pecs = c->d_pecs[c->pend_cur];
        X.pecs_out = c->d_pecs[c->pend_cur ^ 1];
        X.pkeys_out = c->d_pkeys[c->pend_cur ^ 1];
        X.pvals_out = c->d_pvals[c->pend_cur ^ 1];
        X.n_pend_out = c->d_nvals + 2;
        X.orph = c->d_orph;
        X.n_orph = c->d_nvals + 3;
        X.orph_cap = c->orph_cap;
        X.trecs = c->d_marena;
        X.toffs = c->d_moffs;
        X.tsfx = c->d_tsfx;
        X.edge_h = c->slow_defer ? c->edge_h : 0;
        X.orph_ord = c->slow_defer && c->dns2_groups ? c->d_orph_ord : nullptr; // DNS v2 stubs
        HP(15);
        if (!hip_ok(e = hipMemsetAsync(c->d_nvals + 2, 0, 4, st))) return c->hipfail(e, "parameter upload");
        HP(16);
        if (!hip_ok(e = (*c->h_xparams = X, upload_params(c->d_xparams, c->h_xparams, sizeof X, st))))
            return c->hipfail(e, "parameter upload");
        HP(17);
        // the v1 resolve (36 VGPRs) would hold eight workgroups a CU; its scattered event reads
        // run best at three (C4: 190 us at eight, 162 at four, 157 at three, 162 at two, 233 at
        // one; profiles/r6/resolve/), which 30 KiB of dynamic LDS beside its 18 KiB XState sets
        const uint32_t rpad = P.dns2_groups ? 0u : PV_RESOLVE_PAD;
        hipLaunchKernelGGL(P.dns2_groups ? pv_xact_resolve2 : pv_xact_resolve, dim3(blocks), dim3(threads), rpad, st,
                           (const PvXactParams *)c->d_xparams);
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_xact_resolve");
        HP(18);
        // (the resolve kernel also moves the queries still open to the carried list: pv_xact_carry's work)
        // the DNS v1 resolve lists the slow transactions of periods with a threshold for
        // pv_xact_slow_dev instead of naming them itself
        const bool listed_slow = !P.dns2_groups && (X.thr_from[0] > 0.0f || X.thr_to[0] > 0.0f);
        const bool shift_thr = P.n_dshift > 0 && ((c->dns_groups & PV_DNS_QUANTILES) || (c->dns2_groups & PV_DNS2_XACT_TIMES));
        if (c->slow_defer) {
            if (int rc = defer_slow(c, P, st)) return rc;
        } else if (shift_thr || listed_slow) {
            // on_period_shift: slow thresholds = p90 of the bucket that just closed
            // (dns/v1/DnsStreamHandler.h:259-266); kept when that bucket had none
            HP(19);
            for (uint32_t k = 1; shift_thr && k <= P.n_dshift; k++) {
                const uint32_t sg = P.dslot_of[k - 1] | (c->gen[P.dslot_of[k - 1]] << 8);
                bool have[PV_XV_SEL];
                uint64_t q[PV_XV_SEL];
                if (int rc = xv_select(c, sg, 0.90, have, q)) return rc;
                if (have[0]) c->from90 = (float)q[0];
                if (have[1]) c->to90 = (float)q[1];
                X.thr_from[k] = c->from90;
                X.thr_to[k] = c->to90;
                // DNS v2: per direction (dns/v2/DnsStreamHandler.h:440-453)
                for (uint32_t d = 0; d < 3; d++) {
                    if (have[2 + d]) c->p90_2[d] = (float)q[2 + d];
                    X.thr2[k][d] = c->p90_2[d];
                }
            }
            // (xv_select synchronised the stream: the parameter block is free to rewrite)
            if (shift_thr && !hip_ok(e = (*c->h_xparams = X, upload_params(c->d_xparams, c->h_xparams, sizeof X, st))))
                return c->hipfail(e, "parameter upload");
            // the listed transactions, their count read on the device
            hipLaunchKernelGGL(pv_xact_slow_dev, dim3((uint32_t)c->cus), dim3(256), 0, st, (const PvXactParams *)c->d_xparams);
            if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemsetAsync(c->d_nvals + 1, 0, 4, st)))
                return c->hipfail(e, "launch pv_xact_slow_dev");
        }
        HP(12);
        // one read-back: the value / carried counts, the flags and the overflow words (the
        // caller's top_slow drain then needs no read of its own)
        uint32_t nv3[3] = {0, 0, 0};
        if (!hip_ok(e = hipMemcpyAsync(nv3, c->d_nvals, 12, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipMemcpyAsync(c->h_status, c->d_status, ST_RB_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "carried queries");
        c->ovf_known = true;
        const uint32_t npo = nv3[2];
        const uint32_t vflags = c->h_status[ST_FLAGS];
        if ((vflags & PVF_VALUES_FULL) || nv3[0] > c->xv_cap) return c->fail(PV_ECAPACITY, "transaction value buffer full");
        // a batch pushes at most two values per response (time + ratio), so keep 2 x max_records free
        if (c->xv_cap - nv3[0] < 2ull * c->max_records) {
            // less than that room: the device value buffer doubles while it stays
            // within PV_XV_BUDGET_MB (HBM is plentiful; a copy inside HBM instead of a read-back
            // of every value inside the stream), else it drains to the host copy and every batch
            // then has the whole capacity (at most two values per response)
            const uint64_t grow = c->xv_cap * 2;
            const char *bv = getenv("PV_XV_BUDGET_MB");
            const uint64_t budget = (bv ? strtoull(bv, nullptr, 10) : 4096ull) << 20;
            PvXValue *nb = nullptr;
            if (grow <= 0xffffffffull && grow * sizeof(PvXValue) <= budget && hip_ok(hipMalloc(&nb, grow * sizeof(PvXValue)))) {
                if (!hip_ok(e = hipMemcpyAsync(nb, c->d_xvals, (size_t)nv3[0] * sizeof(PvXValue), hipMemcpyDeviceToDevice, st)) ||
                    !hip_ok(e = hipStreamSynchronize(st)))
                    return c->hipfail(e, "value buffer growth");
                hipFree(c->d_xvals);
                c->d_xvals = nb;
                c->xv_cap = grow;
            } else {
                if (int rc = sync_xvals(c)) return rc;
                c->xvals_synced = 0;
                if (!hip_ok(e = hipMemsetAsync(c->d_nvals, 0, 4, st))) return c->hipfail(e, "value buffer drain");
            }
        }
        if (npo > c->pend_cap) return c->fail(PV_ECAPACITY, "%u open DNS queries exceed the carried-list capacity", npo);
        c->n_pend = npo;
        c->pend_hi = npo;
        c->pend_cur ^= 1;
        c->pend_base = (int64_t)(c->records_seen + n) - 1;
        HP(13);
    }

    return 0;
}

// the per-message bitmaps of deep sampling (filtered, not deep), for nmsg messages
int tcp_bits_alloc(pv_ctx *c, uint32_t nmsg)
{
    if (nmsg + 64 <= c->tmsg_bits_cap) return 0;
    for (void *p : {(void *)c->d_tfbits, (void *)c->d_ntcp}) if (p) hipFree(p);
    for (void *p : {(void *)c->h_tfbits, (void *)c->h_ntcp}) if (p) hipHostFree(p);
    c->d_tfbits = c->h_tfbits = nullptr;
    c->d_ntcp = c->h_ntcp = nullptr;
    c->tmsg_bits_cap = 0;
    const uint64_t cap = (uint64_t)nmsg + 4096;
    hipError_t e;
    if (!hip_ok(e = hipMalloc(&c->d_tfbits, (cap / 64 + 2) * 8)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_tfbits, (cap / 64 + 2) * 8, hipHostMallocDefault)) ||
        !hip_ok(e = hipMalloc(&c->d_ntcp, (cap / 32 + 64) * 4)) ||
        !hip_ok(e = hipHostMalloc((void **)&c->h_ntcp, (cap / 32 + 64) * 4, hipHostMallocDefault)))
        return c->hipfail(e, "deep sampling message bitmaps");
    c->tmsg_bits_cap = cap;
    return 0;
}

// which of the batch's DNS-over-TCP messages _filtering rejects (pv_dns_tcp_filter) into
// c->h_tfbits (synchronises)
int tcp_filter_bits(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, uint64_t n, hipStream_t st)
{
    const uint32_t nmsg = c->tcp_nmsg;
    if (!nmsg) return 0;
    if (int rc = tcp_bits_alloc(c, nmsg)) return rc;
    PvParams Q;
    params_common(c, Q, d_recs, d_offs, n);
    Q.recs = c->d_marena;
    Q.offs = c->d_moffs;
    Q.linktype = 101;
    Q.dq = c->d_tmq;
    Q.tcp_nmsg = nmsg;
    Q.fbits = c->d_tfbits;
    c->h_params[1] = Q;
    hipError_t e;
    if (!hip_ok(e = upload_params(c->d_params + 1, c->h_params + 1, sizeof Q, st)))
        return c->hipfail(e, "parameter upload");
    const uint32_t tiles = (nmsg + 63) / 64;
    hipLaunchKernelGGL(pv_dns_tcp_filter, dim3(std::min<uint32_t>((tiles + 3) / 4, (uint32_t)c->cus * 8)), dim3(256), 0, st,
                       (const PvParams *)(c->d_params + 1));
    if (!hip_ok(e = hipGetLastError()) ||
        !hip_ok(e = hipMemcpyAsync(c->h_tfbits, c->d_tfbits, (size_t)tiles * 8, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "DNS-over-TCP filter prescan");
    return 0;
}

int process_span(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_boffs, uint64_t a, uint64_t n, uint64_t rec_bytes,
                 const std::vector<Shift> &nsh, const std::vector<Shift> &dsh, uint32_t first_sec, hipStream_t st)
{
    const uint32_t np = c->cfg.num_periods;
    const uint32_t *d_offs = d_boffs + a;
    PvParams P;
    params_common(c, P, d_recs, d_offs, n);
    // a batch with no TCP stage ahead of it is one span: its Net pass emits the TCP segments
    // and the tile masks of its TCP records (zeroed here; the pass stores non-zero masks only)
    P.tcp_emit = c->tcp_pre ? 0u : (c->tcp_exact_on() ? 7u : 1u);
    if (P.tcp_emit) launch_fill64(c, c->d_tmask, (n + 63) / 64, 0);
    P.gbase = c->global_base + c->records_seen;
    if (c->slow_defer && !c->edge_h) c->edge_h = (int64_t)first_sec + c->ttl_s + 61;
    if (c->sample_rate < 100) {
        // AbstractMetricsManager::new_event (:318-333): one draw per event of each manager, in
        // stream order. Net events are the records. DNS events are the DNS-port UDP records the
        // input predicates pass and the DNS-over-TCP messages (their order: record * 4 + the
        // message's rank); an event _filtering rejects is process_filtered, new_event(stamp,
        // false): no draw, the manager's last flag (dns/v1/DnsStreamHandler.cpp:1341-1375)
        const uint64_t words = n / 32 + 64; // padded: inactive lanes of the last tile read in bounds
        hipError_t e;
        if (words > c->ndeep_words) {
            if (c->d_ndeep) hipFree(c->d_ndeep);
            if (c->h_ndeep) hipHostFree(c->h_ndeep);
            c->d_ndeep = nullptr;
            c->h_ndeep = nullptr;
            c->ndeep_words = 0;
            if (!hip_ok(e = hipMalloc(&c->d_ndeep, words * 8)) || !hip_ok(e = hipHostMalloc((void **)&c->h_ndeep, words * 8, hipHostMallocDefault)))
                return c->hipfail(e, "deep sampling bitmaps");
            c->ndeep_words = words;
        }
        const bool filt = c->f_flags != 0;
        if (filt && !c->d_fbits) {
            const size_t fw = (size_t)(c->max_records / 64 + 2);
            if (!hip_ok(e = hipMalloc(&c->d_fbits, fw * 8)) || !hip_ok(e = hipHostMalloc((void **)&c->h_fbits, fw * 8, hipHostMallocDefault)))
                return c->hipfail(e, "deep sampling filter bits");
        }
        uint32_t tseg[2];
        if (int rc = dns_prescan(c, d_recs, d_offs, n, st, false, tseg, filt)) return rc;
        // the span's messages (ord in [4a, 4(a + n))), and which of them are filtered
        const uint32_t nmsg = c->tcp_nmsg;
        if (nmsg) {
            if (int rc = tcp_bits_alloc(c, nmsg)) return rc;
            if (filt)
                if (int rc = tcp_filter_bits(c, d_recs, d_offs, n, st)) return rc;
            memset(c->h_ntcp, 0, ((size_t)nmsg / 32 + 1) * 4);
        }
        uint32_t *hn = c->h_ndeep, *hd = c->h_ndeep + words;
        memset(hn, 0, words * 8);
        auto dns_draw = [&](bool filtered) {
            if (!filtered) c->dns_deep_now = c->draws_dns.next(c->sample_rate);
            return c->dns_deep_now;
        };
        const uint64_t olo = a * 4, ohi = (a + n) * 4;
        auto it = std::lower_bound(c->tcp_items.begin(), c->tcp_items.end(), std::make_pair(olo, 0u));
        c->draws_net.take_not_deep(c->sample_rate, hn, n);
        // the DNS events in stream order: each DNS-port UDP record, then the messages a TCP
        // record completes (ord (a + i) * 4 + sub) after the records before it
        auto tcp_upto = [&](uint64_t rec_end) {
            for (; it != c->tcp_items.end() && it->first < ohi && (it->first >> 2) < a + rec_end; ++it) {
                const uint32_t q = it->second;
                const bool f = filt && ((c->h_tfbits[q >> 6] >> (q & 63)) & 1);
                if (!dns_draw(f)) c->h_ntcp[q >> 5] |= 1u << (q & 31);
            }
        };
        for (uint64_t w = 0; w < (n + 63) / 64; w++) {
            uint64_t m = c->h_dbits[w];
            if (w == (n - 1) / 64 && n % 64) m &= (1ull << (n % 64)) - 1;
            while (m) {
                const uint64_t i = w * 64 + __builtin_ctzll(m);
                m &= m - 1;
                tcp_upto(i);
                const bool f = filt && ((c->h_fbits[i >> 6] >> (i & 63)) & 1);
                if (!dns_draw(f)) hd[i >> 5] |= 1u << (i & 31);
            }
        }
        tcp_upto(n);
        if (!hip_ok(e = hipMemcpyAsync(c->d_ndeep, c->h_ndeep, words * 8, hipMemcpyHostToDevice, st)) ||
            (nmsg && !hip_ok(e = hipMemcpyAsync(c->d_ntcp, c->h_ntcp, ((size_t)nmsg / 32 + 1) * 4, hipMemcpyHostToDevice, st))))
            return c->hipfail(e, "deep sampling bitmaps");
        P.ndeep_net = c->d_ndeep;
        P.ndeep_dns = c->d_ndeep + words;
    }
    // Net periods and slots: period 0 -> the live bucket, each shift -> the next ordinal's slot
    P.n_shift = (uint32_t)nsh.size();
    for (size_t k = 0; k < nsh.size(); k++) { P.thresh[k] = nsh[k].sec; P.pstart[k] = nsh[k].idx; }
    P.skip_before = P.n_shift + 1 > np ? P.n_shift + 1 - np : 0;
    for (uint32_t k = 0; k <= P.n_shift; k++) {
        P.slot_of[k] = c->net.slot_at(k);
        if (k) clear_part(c, PART_NET, P.slot_of[k]);
    }
    // DNS periods and slots, from the DNS manager's own shifts
    P.n_dshift = (uint32_t)dsh.size();
    for (size_t k = 0; k < dsh.size(); k++) { P.dthresh[k] = dsh[k].sec; P.dpos[k] = (uint32_t)dsh[k].ord; }
    P.dskip_before = P.n_dshift + 1 > np ? P.n_dshift + 1 - np : 0;
    for (uint32_t k = 0; k <= P.n_dshift; k++) {
        P.dslot_of[k] = c->dns.slot_at(k);
        if (k) clear_part(c, PART_DNS, P.dslot_of[k]);
    }
    P.sum = c->d_sum;
    P.cpc = c->d_cpc;
    P.tkeys = c->d_tkeys;
    P.tcnt = c->d_tcnt;
    P.taux = c->d_taux;
    P.tcap_log2 = c->tcap_log2;
    P.arena = c->d_arena;
    P.arena_top = c->d_arena_top;
    P.arena_cap = c->arena_cap;
    P.tab_live = c->d_tab_live; // global_add counts the entries it creates
    P.events = c->d_events;
    P.eecs = c->d_eecs;
    P.ekeys = c->d_ekeys;
    P.blk_events = c->d_blk_events;
    P.skeys = c->d_skeys;
    P.svals = c->d_svals;
    P.n_events = c->d_status + ST_NEV; // [0] events, [1] responses (ST_NRESP)
    P.n_keys = c->d_status + ST_NKEYS;
    P.n_dns = c->d_status + ST_NDNS;
    P.n_slow = c->d_status + ST_NSLOW;
    P.n_ecs = c->d_status + ST_NECS;
    P.want_events = ((c->dns_groups & PV_DNS_TRANSACTIONS) || c->dns2_groups) ? 1 : 0;
    // sort ranks: carried queries 0, this batch's records from records_seen - pend_base on
    if (c->n_pend == 0) c->pend_base = (int64_t)c->records_seen - 1;
    if ((uint64_t)((int64_t)(c->records_seen + n) - c->pend_base) >= 0x3fffffffull)
        return c->fail(PV_ECAPACITY, "open DNS queries carried over more than 2^30 records without a response");
    P.ekey_base = (uint32_t)((int64_t)c->records_seen - c->pend_base);
    P.flags = c->d_status + ST_FLAGS;
    launch_fill32(c, c->d_status, ST_ALLOC, 0);
    hipError_t e;
    const uint64_t tiles = (n + 63) / 64; // 64-record wave tiles
    // persistent grid: exactly the workgroups that are resident at once (LDS/VGPR
    // occupancy), each owning a contiguous run of wave tiles
    // (a batch after one that was mostly DNS messages takes four ranges per CU: the DNS pass,
    // combine and merge of such batches gain from the finer partition, C3 2.16 -> 2.11 ms, while
    // Net-heavy batches lose, C2 0.450 -> 0.465; profiles/r5/experiments/r5oo)
    const int wgcu = !c->wg_forced && c->dns_heavy ? std::max(c->wg_per_cu, 4) : c->wg_per_cu;
    uint32_t grid = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(tiles, (uint64_t)c->cus * wgcu), PV_MAX_GRID);
    P.wt_per_block = (uint32_t)((tiles + grid - 1) / grid);
    P.rec_bytes = rec_bytes;
    {
        static const char *dbg = getenv("PV_DEBUG_STAGES");
        P.dbg = dbg ? (uint32_t)atoi(dbg) : 0;
    }
    grid = (uint32_t)((tiles + P.wt_per_block - 1) / P.wt_per_block);
    P.grid_main = grid;
    // per workgroup: at most 6 hashed updates per record, plus one cache flush per pass
    // (Net v2: two more updates per record and one more cache flush)
    P.mq_cap = P.wt_per_block * 64u * (PV_MQ_PER_REC + (c->net2_groups ? 2u : 0u)) + PV_CACHE_MAX * (c->net2_groups ? 3u : 2u);
    {
        const size_t need = (size_t)grid * P.mq_cap * 16;
        if (need > c->mq_bytes) {
            if (c->d_mq) hipFree(c->d_mq);
            if (c->d_tpbuf) hipFree(c->d_tpbuf);

            if (c->d_cb) hipFree(c->d_cb);
            c->d_mq = c->d_tpbuf = c->d_cb = nullptr;
            c->mq_bytes = 0;
            if (!hip_ok(e = hipMalloc(&c->d_mq, need)) || !hip_ok(e = hipMalloc(&c->d_tpbuf, need)) ||

                !hip_ok(e = hipMalloc(&c->d_cb, need)))
                return c->hipfail(e, "top-N update log");
            c->mq_bytes = need;
        }
    }
    if (grid > PV_MAX_GRID) return c->fail(PV_ECAPACITY, "grid of %u workgroups exceeds %d", grid, PV_MAX_GRID);
    if (P.mq_cap >= (1u << 24)) return c->fail(PV_ECAPACITY, "batch too large: %u update-log entries per workgroup", P.mq_cap);
    if (grid > c->cb_h_grid) {
        if (c->d_cb_h) hipFree(c->d_cb_h);
        c->d_cb_h = nullptr;
        c->cb_h_grid = 0;
        // run table: (2 << PV_MAX_REGIONS_LOG2) run keys x the grid padded to a multiple of 8
        if (!hip_ok(e = hipMalloc(&c->d_cb_h, (size_t)((grid + 7) & ~7u) << (PV_MAX_REGIONS_LOG2 + 4))))
            return c->hipfail(e, "region runs");
        c->cb_h_grid = grid;
    }
    P.mq = c->d_mq;
    P.mq_cnt = c->d_mq_cnt;
    P.reg_log2 = c->reg_log2;
    P.tab_live = c->d_tab_live;
    P.ovf = c->d_ovf;
    P.ovf_cnt = c->d_ovf_cnt;
    P.ovf_cap = c->ovf_cap;
    P.cb_run = (uint64_t *)c->d_cb_h;
    P.tp_hands = c->d_status + ST_HANDS;
    P.tp_buf = c->d_tpbuf;
    P.nn_cnt = c->d_status + ST_NNEW;
    P.nn = c->d_nn;
    P.nn_cap = c->nn_cap;
    P.iplog = c->d_iplog;
    P.iplog32 = c->d_iplog32;
    P.ipdir = c->d_ipdir;
    P.ipx_cnt = c->d_ipx_cnt;
    P.ipx_rep = c->d_ipx_rep;
    P.trash = c->d_trash;
    if ((uint64_t)grid * 4 > PV_TRASH_WAVES) return c->fail(PV_ECAPACITY, "grid of %u workgroups exceeds the trash area", grid);
    P.cb = c->d_cb;
    P.cb_cnt = c->d_cb_cnt;
    P.cb_hm = c->d_cb_cnt + 32768;
    {
        // grid ranges per combine workgroup (PV_CB_FAN, A/B runs): fewer, larger tables
        static const char *fan = getenv("PV_CB_FAN");
        P.cb_fan = fan ? std::max(1u, std::min(8u, (uint32_t)atoi(fan))) : c->cb_fan;
        while (P.cb_fan > 1 && (uint64_t)P.cb_fan * P.mq_cap >= (1u << 24)) P.cb_fan--; // run starts are 24-bit
        P.cb_grid = (grid + P.cb_fan - 1) / P.cb_fan;
    }
    P.stamps = c->d_stamps;
    P.dq = c->d_dq;
    P.dq_cnt = c->d_dq_cnt;
    // the specialised passes when nothing in the batch needs the general one: the lean pass
    // (one Net period, Ethernet, at most two IPv4 host subnets, a wave's tiles below 2^16 for
    // its packed lane counters), else the shift-free general pass. PV_NET_KERNEL=ns|general
    // forces one for A/B runs.
    static const char *force = getenv("PV_NET_KERNEL");
    // (every TCP packet for the exact LRU replay: the general pass emits them)
    const bool general = P.n_shift || P.net_filter_all || P.dbg || P.ndeep_net || c->tcp_exact_on() ||
                         (force && !strcmp(force, "general"));
    const uint32_t reg_grid = std::min<uint32_t>(grid, (uint32_t)(c->cus * c->reg_wg_per_cu));
    const uint64_t per_wave = ((uint64_t)P.wt_per_block / 4 + 1) * ((grid + reg_grid - 1) / reg_grid); // packed lane counters
    const bool lean = !general && P.linktype == 1 && P.nets.n4 <= 2 && P.skip_before == 0 && per_wave < 65535 &&
                      !(force && !strcmp(force, "ns"));
    // lean: the register-window pass (pv_net_kernel_reg, its top-IPs specialisation _tc), which
    // writes the compact IP log (4 B + a direction bit per record)
    P.ip_compact = lean ? 1u : 0u;
    P.ip_base = ((uint64_t)P.slot_of[0] << 60) | ((uint64_t)TM_IPV4 << 56) |
                ((uint64_t)((c->net_groups & PV_NET_CARDINALITY) ? 1 : 0) << 33);
    const bool tc = (c->net_groups & PV_NET_TOP_IPS) != 0;
    // PV_NET_KERNEL=span: the span-load pass (top-IPs groups), kept for A/B runs
    const bool span = lean && tc && force && !strcmp(force, "span");
    // both lean passes defer general-path records to pv_net_slow_list
    if (lean) {
        if (c->slow_cap < P.n) {
            if (c->d_slow) hipFree(c->d_slow);
            c->d_slow = nullptr;
            c->slow_cap = 0;
            if (!hip_ok(e = hipMalloc(&c->d_slow, (size_t)(P.n + PV_MAX_GRID) * 4))) return c->hipfail(e, "deferred record list");
            c->slow_cap = P.n;
        }
        P.slow_list = c->d_slow;
        P.slow_cnt = c->d_slow + c->slow_cap; // written for every range by the lean passes
    }
    // top_ecs: the UDP DNS pass lists its updates (at most one per record) for pv_dns_ecs
    if (c->dns_groups & PV_DNS_TOP_ECS) {
        if (c->ecs_cap < P.n) {
            if (c->d_ecs) hipFree(c->d_ecs);
            c->d_ecs = nullptr;
            c->ecs_cap = 0;
            if (!hip_ok(e = hipMalloc(&c->d_ecs, (size_t)P.n * sizeof(uint4)))) return c->hipfail(e, "top_ecs list");
            c->ecs_cap = P.n;
        }
        P.ecs_list = reinterpret_cast<uint32_t *>(c->d_ecs);
        P.ecs_cap = (uint32_t)c->ecs_cap;
    }
    *c->h_params = P;
    if (!hip_ok(e = fill_and_upload(c, c->d_params, c->h_params, sizeof P, st)))
        return c->hipfail(e, "parameter upload");
    c->net_kernel = general ? "pv_net_kernel"
                            : (lean ? (span ? "pv_net_kernel_span" : (tc ? "pv_net_kernel_reg_tc" : "pv_net_kernel_reg"))
                                    : "pv_net_kernel_ns");
    // pv_kernel_timing (bench roofline): the record-parse kernel alone, timed by the start and
    // end stamps of its own dispatch packet (hipExtLaunchKernelGGL), so no event marker packets
    // sit in the stream between the step's kernels
    const PvParams *dp = (const PvParams *)c->d_params;
    // (stamping a dispatch costs ~14 us of idle around it: only the batches pv_set_kernel_timing
    // asks for are stamped)
    const bool timed = c->timing_every && (c->timing_ctr++ % c->timing_every) == 0;
    hipEvent_t e0 = timed ? c->ev_start : nullptr, e1 = timed ? c->ev_stop : nullptr;
    if (general) hipExtLaunchKernelGGL(pv_net_kernel, dim3(grid), dim3(PV_NET_THREADS), 0, st, e0, e1, 0, dp);
    else if (lean) {
        // the lean pass, then its deferred general-path records (the dispatch stamps span both)
        if (span) hipExtLaunchKernelGGL(pv_net_kernel_span, dim3(reg_grid), dim3(PV_NET_THREADS), 0, st, e0, (hipEvent_t) nullptr, 0, dp);
        else if (tc) hipExtLaunchKernelGGL(pv_net_kernel_reg_tc, dim3(reg_grid), dim3(PV_NET_THREADS), 0, st, e0, (hipEvent_t) nullptr, 0, dp);
        else hipExtLaunchKernelGGL(pv_net_kernel_reg, dim3(reg_grid), dim3(PV_NET_THREADS), 0, st, e0, (hipEvent_t) nullptr, 0, dp);
        hipExtLaunchKernelGGL(pv_net_slow_list, dim3(c->cus * 2), dim3(256), 0, st, (hipEvent_t) nullptr, e1, 0, dp);
    }
    else hipExtLaunchKernelGGL(pv_net_kernel_ns, dim3(grid), dim3(PV_NET_THREADS), 0, st, e0, e1, 0, dp);
    e = hipGetLastError();
    if (e != hipSuccess) return c->hipfail(e, "launch pv_net_kernel");
    if (P.f_flags & (PVDF_ONLY_QSUFFIX | PVDF_PSL))
        hipLaunchKernelGGL(pv_dns_suffix, dim3(grid), dim3(256), 0, st, (const PvParams *)c->d_params);
    // the DNS pass walks the logical grid's ranges with its resident grid
    const uint32_t dns_grid = std::min<uint32_t>(grid, (uint32_t)(c->cus * c->dns_wg_per_cu));
    if (P.f_flags & (PVDF_ONLY_QSUFFIX | PVDF_PSL))
        hipLaunchKernelGGL(pv_dns_kernel_sfx, dim3(dns_grid), dim3(64 * PV_DNS_WAVES), 0, st, (const PvParams *)c->d_params);
    else if (P.f_flags)
        hipLaunchKernelGGL(pv_dns_kernel_f, dim3(dns_grid), dim3(64 * PV_DNS_WAVES), 0, st, (const PvParams *)c->d_params);
    else
        hipLaunchKernelGGL(pv_dns_kernel, dim3(dns_grid), dim3(64 * PV_DNS_WAVES), 0, st, (const PvParams *)c->d_params);
    if (c->dns_groups & PV_DNS_TOP_ECS)
        hipLaunchKernelGGL(pv_dns_ecs, dim3((uint32_t)c->cus * 2), dim3(256), 0, st, (const PvParams *)c->d_params);
    if (c->net2_groups) hipLaunchKernelGGL(pv_net2_kernel, dim3(grid), dim3(256), 0, st, (const PvParams *)c->d_params);
    // top-N: combine each workgroup's updates into a list sorted by table region, merge
    // each region's runs in LDS, decode the names of new entries
    static int cb_threads = 0; // the kernel's own launch bound (tuning builds change it)
    if (!cb_threads) {
        hipFuncAttributes fa{};
        cb_threads = hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(pv_topn_combine)) == hipSuccess ? fa.maxThreadsPerBlock
                                                                                                             : PV_CB_THREADS;
    }
    hipLaunchKernelGGL(c->reg_log2 <= 10 ? pv_topn_combine : pv_topn_combine_r12, dim3(P.cb_grid), dim3(cb_threads), 0, st,
                       (const PvParams *)c->d_params);
    hipLaunchKernelGGL(pv_topn_merge, dim3(2u << c->reg_log2), dim3(pv_topn_merge_threads()), 0, st, (const PvParams *)c->d_params);
    // names: as many workgroups as are resident (LDS: two per CU), each pipelining its entries
    hipLaunchKernelGGL((P.f_flags & (PVDF_ONLY_QSUFFIX | PVDF_PSL)) ? pv_topn_names_sfx : pv_topn_names, dim3((uint32_t)c->cus * 2),
                       dim3(256), 0, st, (const PvParams *)c->d_params);
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch");

    // ---- transactions: pair responses with queries (sort by key, then record index)
    uint32_t status[ST_WORDS];
    HP(14);
    if (!hip_ok(e = hipMemcpyAsync(c->h_status, c->d_status, ST_RB_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "kernel execution");
    memcpy(status, c->h_status, sizeof status);
    c->dns_heavy = (uint64_t)status[ST_NDNS] * 2 > n;
    if (status[ST_FLAGS] & PVF_NAMES_PENDING) {
        // more created entries than the new-name list holds: their names, before anything reads
        // or purges the tables
        for (uint32_t t = 0; t < PV_TABLES; t++)
            hipLaunchKernelGGL(pv_topn_name_fix, dim3((uint32_t)c->cus * 4), dim3(256), 0, st, (const PvParams *)c->d_params, t);
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipStreamSynchronize(st))) return c->hipfail(e, "pending names");
        if (getenv("PV_NAMEFIX_TRACE")) fprintf(stderr, "pv: pending top-N names written (pv_topn_name_fix)\n");
    }
    HP(4);
    {
        float ms = 0;
        if (timed && hipEventElapsedTime(&ms, c->ev_start, c->ev_stop) == hipSuccess) { c->kernel_ms += ms; c->kernel_launches++; }
    }
    // the parts this batch wrote are no longer clean
    // ---- DNS over TCP: the stage of a one-span batch (its segments came from the Net pass),
    // then this span's messages through the DNS pass, their events behind the UDP ones
    if (!c->tcp_pre) {
        if (int rc = tcp_stage(c, d_recs, d_offs, n, status[ST_TSEG], status[ST_TSEG_BYTES], first_sec, false, st)) return rc;
    }
    const uint32_t gt = tcp_pass(c, P, a, a + n, st, c->h_params + 1);
    if (gt) {
        // the TCP messages' events behind the UDP pass's key list
        if (P.want_events)
            hipLaunchKernelGGL(pv_xact_compact, dim3(gt), dim3(256), 0, st, (const PvParams *)c->d_params, grid,
                               status[ST_NKEYS]);
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_dns_tcp");
        if (!hip_ok(e = hipMemcpyAsync(c->h_status, c->d_status, ST_RB_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "TCP DNS pass");
        memcpy(status, c->h_status, sizeof status);
    }
    for (uint32_t k = 0; k <= P.n_shift; k++) c->net.clean[P.slot_of[k]] = false;
    if (status[ST_NDNS] || gt)
        for (uint32_t k = 0; k <= P.n_dshift; k++) c->dns.clean[P.dslot_of[k]] = false;
    bool drained = false;
    if (int rc = drain_overflow(c, st, true, &drained)) return rc;
    uint32_t flags = status[ST_FLAGS];
    if (drained && !hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
    if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "top-N table full: raise table_log2");
    if (flags & PVF_ARENA_FULL) return c->fail(PV_ECAPACITY, "top-N name arena full");
    if (getenv("PV_TSTAMPS")) {
        // -DPV_TSTAMPS builds: mean cycles per workgroup of the top-N combine / merge phases
        std::vector<uint64_t> tv(65536 + (2u << c->reg_log2) * 8);
        if (hip_ok(hipMemcpy(tv.data(), c->d_stamps + (1u << 20), tv.size() * 8, hipMemcpyDeviceToHost))) {
            double cs[8] = {0}, ms[8] = {0};
            uint64_t nm = 0;
            for (uint32_t w = 0; w < grid; w++)
                for (int k = 0; k < 8; k++) cs[k] += (double)tv[w * 8 + k];
            for (uint32_t w = 0; w < (2u << c->reg_log2); w++) {
                const uint64_t *m = &tv[65536 + w * 8];
                if (!m[0] && !m[1]) continue;
                nm++;
                for (int k = 0; k < 8; k++) ms[k] += (double)m[k];
            }
            fprintf(stderr, "pv_tstamps combine (%u wg): init=%.0f insert=%.0f count=%.0f scan=%.0f out=%.0f | merge (%lu wg): "
                            "runs=%.0f load=%.0f insert=%.0f wb=%.0f names=%.0f\n",
                    grid, cs[0] / grid, cs[1] / grid, cs[2] / grid, cs[3] / grid, cs[4] / grid, (unsigned long)nm,
                    ms[0] / std::max<uint64_t>(nm, 1), ms[1] / std::max<uint64_t>(nm, 1), ms[2] / std::max<uint64_t>(nm, 1),
                    ms[3] / std::max<uint64_t>(nm, 1), ms[4] / std::max<uint64_t>(nm, 1));
            hipMemset(c->d_stamps + (1u << 20), 0, tv.size() * 8);
        }
    }
    if (getenv("PV_STAMPS")) {
        std::vector<uint64_t> stv((size_t)grid * 4 * 8);
        if (hip_ok(hipMemcpy(stv.data(), c->d_stamps, stv.size() * 8, hipMemcpyDeviceToHost))) {
            double sum[8] = {0};
            for (size_t w = 0; w < (size_t)grid * 4; w++)
                for (int k = 0; k < 8; k++) sum[k] += (double)stv[w * 8 + k];
            fprintf(stderr, "pv_stamps (mean cycles per wave, %u wave tiles/wg):", P.wt_per_block);
            static const char *nm[8] = {"slot", "commit", "barA", "issue", "parse", "lane", "barB", "flush"};
            for (int k = 0; k < 8; k++) fprintf(stderr, " %s=%.0f", nm[k], sum[k] / (grid * 4.0));
            fprintf(stderr, "\n");
        }
    }
    HP(5);
    if (int rc = pair_stage(c, P, status[ST_NEV], status[ST_NKEYS], status[ST_NRESP], n, st,
                            (uint64_t)(grid + gt) * P.wt_per_block * 64u))
        return rc;
    HP(6);
    // top_slow updates of the transaction stage (only when it ran; its read-back after the
    // resolve holds the overflow words)
    const bool ovf_known = c->ovf_known;
    c->ovf_known = false;
    if ((status[ST_NEV] || c->n_pend) && P.want_events)
        if (int rc = drain_overflow(c, st, ovf_known)) return rc;

    // ---- window bookkeeping (host mirror of each manager's _period_shift)
    for (const Shift &sh : nsh) win_shift(c, c->net, sh.sec);
    for (const Shift &sh : dsh) {
        win_shift(c, c->dns, sh.sec);
        c->dns_shifts.emplace_back(sh.sec, c->dns.slot_at(0));
        c->dns_shift_ord.emplace_back(sh.sec, c->dns.ordinal);
    }
    c->records_seen += n;
    const int prc = purge_tables(c, st);
    HP(7);
    return prc;
}

// Both managers' shifts of a batch (Net from the record seconds, DNS from the prescan bits
// and the TCP messages). A batch that may shift DNS windows, or that the Net shifts split
// into spans, runs its TCP stage here, ahead of the spans (the prescan emits the segments);
// any other batch runs it inside its one span, behind the Net pass (c->tcp_pre).
int batch_shifts(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                 const uint32_t *sc_idx, const uint32_t *sc_sec, hipStream_t st, std::vector<Shift> &nsh,
                 std::vector<Shift> &dsh)
{
    c->tcp_pre = false;
    c->tcp_nmsg = 0;
    c->tcp_ords.clear();
    c->tcp_items.clear();
    // the batch's latest second (its last record's, unless the timestamps go back somewhere)
    int64_t top = info->last_sec;
    if (!info->monotone)
        for (uint32_t k = 0; k < info->n_sec_changes; k++) top = std::max<int64_t>(top, (int64_t)sc_sec[k]);
    if (c->sample_rate < 100) {
        // deep sampling draws per DNS event in stream order, DNS-over-TCP messages among them:
        // the TCP stage runs ahead of the spans so their order is known first
        c->tcp_pre = true;
        uint32_t tseg[2] = {0, 0};
        if (int rc = dns_prescan(c, d_recs, d_offs, info->n_records, st, true, tseg)) return rc;
        const bool dns_may = c->cfg.num_periods > 1 && top >= c->dns.next_shift_sec;
        c->eoc_stage = c->eoc_batch;
        if (int rc = tcp_stage(c, d_recs, d_offs, info->n_records, tseg[0], tseg[1], (uint32_t)info->first_sec, true, st))
            return rc;
        if (c->cfg.num_periods <= 1) return 0;
        const bool net_may = top >= c->net.next_shift_sec;
        if (!net_may && !dns_may) return 0;
        if (net_may) net_shifts_of(c->net.next_shift_sec, info, sc_idx, sc_sec, nsh);
        if (dns_may) dns_shifts_of(c->dns.next_shift_sec, c->h_dbits, info->n_records, info, sc_idx, sc_sec, c->tcp_ords, dsh);
        return 0;
    }
    if (c->cfg.num_periods <= 1) return 0;
    const bool net_may = top >= c->net.next_shift_sec, dns_may = top >= c->dns.next_shift_sec;
    if (!net_may && !dns_may) return 0;
    if (net_may) net_shifts_of(c->net.next_shift_sec, info, sc_idx, sc_sec, nsh);
    c->tcp_pre = dns_may || nsh.size() > PV_MAX_SHIFTS;
    if (c->tcp_pre) {
        uint32_t tseg[2] = {0, 0};
        if (int rc = dns_prescan(c, d_recs, d_offs, info->n_records, st, true, tseg)) return rc;
        c->eoc_stage = c->eoc_batch;
        if (int rc = tcp_stage(c, d_recs, d_offs, info->n_records, tseg[0], tseg[1], (uint32_t)info->first_sec, dns_may, st))
            return rc;
    }
    if (dns_may) dns_shifts_of(c->dns.next_shift_sec, c->h_dbits, info->n_records, info, sc_idx, sc_sec, c->tcp_ords, dsh);
    return 0;
}

} // namespace

int x_grow_dev(pv_ctx *c, void **p, size_t &have, size_t need, const char *what)
{
    if (need <= have) return 0;
    hipError_t e;
    if (*p) hipFree(*p);
    *p = nullptr;
    have = 0;
    if (!hip_ok(e = hipMalloc(p, std::max<size_t>(need, 256)))) return c->hipfail(e, what);
    have = std::max<size_t>(need, 256);
    return 0;
}
// The BPF filter on a device batch: keep flags and sizes (pv_bpf_keep), their exclusive scans (byte
// offsets, ranks), the kept records compacted into d_frecs / d_foffs (pv_bpf_gather), and the
// kept run's index info and ts_sec change points (pv_bpf_secs). The caller holds c->mu.
int bpf_filter_device(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info, hipStream_t st,
                      pv_index_info &out, std::vector<uint32_t> &sci, std::vector<uint32_t> &scs)
{
    hipError_t e;
    const uint32_t n = (uint32_t)info->n_records;
    memset(&out, 0, sizeof out);
    if (c->bpf_dirty || !c->d_bpf) {
        if (c->d_bpf) hipFree(c->d_bpf);
        c->d_bpf = nullptr;
        if (!hip_ok(e = hipMalloc(&c->d_bpf, c->bpf.size() * sizeof(pv_bpf_insn))) ||
            !hip_ok(e = hipMemcpy(c->d_bpf, c->bpf.data(), c->bpf.size() * sizeof(pv_bpf_insn), hipMemcpyHostToDevice)))
            return c->hipfail(e, "BPF program");
        c->d_bpf_n = c->bpf.size();
        c->bpf_dirty = false;
    }
    if (n > c->fwork_n) {
        for (void *p : {(void *)c->d_fwork, (void *)c->d_foffs, (void *)c->d_fsc}) if (p) hipFree(p);
        c->d_fwork = c->d_foffs = c->d_fsc = nullptr;
        c->fwork_n = 0;
        if (!hip_ok(e = hipMalloc(&c->d_fwork, (size_t)n * 16)) || !hip_ok(e = hipMalloc(&c->d_foffs, (size_t)n * 4)) ||
            !hip_ok(e = hipMalloc(&c->d_fsc, (size_t)n * 8 + 64)))
            return c->hipfail(e, "BPF filter buffers");
        c->fwork_n = n;
    }
    if (info->bytes_used + PV_RECS_PAD > c->frecs_bytes) {
        if (c->d_frecs) hipFree(c->d_frecs);
        c->d_frecs = nullptr;
        c->frecs_bytes = 0;
        if (!hip_ok(e = hipMalloc(&c->d_frecs, info->bytes_used + PV_RECS_PAD)) ||
            !hip_ok(e = hipMemsetAsync(c->d_frecs, 0, info->bytes_used + PV_RECS_PAD, st)))
            return c->hipfail(e, "BPF filter buffers");
        c->frecs_bytes = info->bytes_used + PV_RECS_PAD;
    }
    size_t tb = 0;
    if (!hip_ok(e = pv_exclusive_scan_u32(nullptr, &tb, nullptr, nullptr, n, st))) return c->hipfail(e, "scan size");
    if (int rc = x_grow_dev(c, &c->d_fscan, c->fscan_bytes, tb, "BPF scan")) return rc;
    uint32_t *sz = c->d_fwork, *kf = sz + n, *boff = kf + n, *rank = boff + n;
    const uint32_t grid = (n + 255) / 256;
    hipLaunchKernelGGL(pv_bpf_keep, dim3(grid), dim3(256), 0, st, d_recs, d_offs, n, (const PvBpfIns *)c->d_bpf,
                       (uint32_t)c->d_bpf_n, sz, kf);
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_bpf_keep");
    tb = c->fscan_bytes;
    if (!hip_ok(e = pv_exclusive_scan_u32(c->d_fscan, &tb, sz, boff, n, st))) return c->hipfail(e, "scan");
    tb = c->fscan_bytes;
    if (!hip_ok(e = pv_exclusive_scan_u32(c->d_fscan, &tb, kf, rank, n, st))) return c->hipfail(e, "scan");
    uint32_t tail[4];
    if (!hip_ok(e = hipMemcpyAsync(&tail[0], boff + n - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&tail[1], sz + n - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&tail[2], rank + n - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&tail[3], kf + n - 1, 4, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)))
        return c->hipfail(e, "BPF filter");
    const uint64_t bytes = (uint64_t)tail[0] + tail[1];
    const uint32_t nk = tail[2] + tail[3];
    if (!nk) return 0;
    hipLaunchKernelGGL(pv_bpf_gather, dim3(grid), dim3(256), 0, st, d_recs, d_offs, n, (const uint32_t *)sz, (const uint32_t *)boff,
                       (const uint32_t *)rank, c->d_frecs, c->d_foffs);
    // the kept run's change points (sz / kf / boff reused: flags, seconds, positions)
    uint32_t *flag = sz, *sec = kf, *pos = boff, *down = c->d_fsc + 2 * (size_t)n;
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemsetAsync(down, 0, 4, st))) return c->hipfail(e, "BPF filter");
    hipLaunchKernelGGL(pv_bpf_secs, dim3((nk + 255) / 256), dim3(256), 0, st, (const uint8_t *)c->d_frecs, (const uint32_t *)c->d_foffs,
                       nk, flag, sec, down);
    tb = c->fscan_bytes;
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = pv_exclusive_scan_u32(c->d_fscan, &tb, flag, pos, nk, st)))
        return c->hipfail(e, "BPF filter");
    hipLaunchKernelGGL(pv_bpf_secs_compact, dim3((nk + 255) / 256), dim3(256), 0, st, (const uint32_t *)flag, (const uint32_t *)pos,
                       (const uint32_t *)sec, nk, n, c->d_fsc, c->d_fsc + n);
    uint32_t w[4], lo = 0, hi_off = 0;
    uint32_t h0[4], h1[4];
    if (!hip_ok(e = hipGetLastError()) ||
        !hip_ok(e = hipMemcpyAsync(&w[0], pos + nk - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&w[1], flag + nk - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&w[2], down, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(&hi_off, c->d_foffs + nk - 1, 4, hipMemcpyDeviceToHost, st)) ||
        !hip_ok(e = hipMemcpyAsync(h0, c->d_frecs, 16, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)) ||
        !hip_ok(e = hipMemcpy(h1, c->d_frecs + hi_off, 16, hipMemcpyDeviceToHost)))
        return c->hipfail(e, "BPF filter");
    (void)lo;
    const uint32_t nch = w[0] + w[1];
    sci.resize(nch);
    scs.resize(nch);
    if (nch && (!hip_ok(e = hipMemcpy(sci.data(), c->d_fsc, (size_t)nch * 4, hipMemcpyDeviceToHost)) ||
                !hip_ok(e = hipMemcpy(scs.data(), c->d_fsc + n, (size_t)nch * 4, hipMemcpyDeviceToHost))))
        return c->hipfail(e, "BPF filter");
    out.n_records = nk;
    out.bytes_used = bytes;
    out.first_sec = h0[0];
    out.first_nsec = c->cfg.ts_nano ? (int64_t)h0[1] : (int64_t)h0[1] * 1000;
    out.last_sec = h1[0];
    out.last_nsec = c->cfg.ts_nano ? (int64_t)h1[1] : (int64_t)h1[1] * 1000;
    out.monotone = w[2] == 0;
    out.n_sec_changes = nch;
    return 0;
}

int pv_process_device(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                      const uint32_t *sc_idx, const uint32_t *sc_sec, void *stream)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (int rc = merged_refuse(c)) return rc;
    hipSetDevice(c->device);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    hipStream_t saved = c->stream;
    c->stream = st;
    struct Restore { pv_ctx *c; hipStream_t s; ~Restore() { c->stream = s; } } restore{c, saved};
    // the end of the capture (pv_set_end_of_capture): a direct call is the capture's final batch;
    // pv_process_host's ingest loops mark their final batch themselves
    if (!c->in_host) c->eoc_batch = c->eoc_armed;
    struct EocDone {
        pv_ctx *c;
        ~EocDone()
        {
            c->eoc_stage = false;
            if (!c->in_host) c->eoc_armed = c->eoc_batch = false;
        }
    } eoc_done{c};
    if (info->n_records == 0) return 0;
    if (info->n_records > c->max_records) return c->fail(PV_ECAPACITY, "batch of %llu records exceeds max_records %llu",
                                           (unsigned long long)info->n_records, (unsigned long long)c->max_records);
    pv_index_info finfo;
    std::vector<uint32_t> fsci, fscs;
    if (!c->bpf.empty()) {
        // the pcap input's BPF filter (PcapInputStream.cpp:485-488) over the batch in HBM: the kept
        // records become the batch
        if (int rc = bpf_filter_device(c, d_recs, d_offs, info, st, finfo, fsci, fscs)) return rc;
        if (finfo.n_records == 0) return 0;
        d_recs = c->d_frecs;
        d_offs = c->d_foffs;
        info = &finfo;
        sc_idx = fsci.data();
        sc_sec = fscs.data();
    }
    const uint64_t n = info->n_records;
    ensure_started(c, info->first_sec, info->first_nsec);
    std::vector<Shift> nsh, dsh;
    if (int rc = batch_shifts(c, d_recs, d_offs, info, sc_idx, sc_sec, st, nsh, dsh)) return rc;
    HP(3);
    // spans of at most PV_MAX_SHIFTS shifts of each manager, cut at the shifting record
    uint64_t a = 0;
    size_t ni = 0, di = 0;
    while (a < n) {
        uint64_t b = n;
        if (nsh.size() - ni > PV_MAX_SHIFTS) b = std::min<uint64_t>(b, nsh[ni + PV_MAX_SHIFTS].idx);
        if (dsh.size() - di > PV_MAX_SHIFTS) b = std::min<uint64_t>(b, dsh[di + PV_MAX_SHIFTS].idx);
        std::vector<Shift> ns, ds;
        for (; ni < nsh.size() && nsh[ni].idx < b; ni++) ns.push_back({nsh[ni].sec, nsh[ni].idx - a, 0});
        for (; di < dsh.size() && dsh[di].idx < b; di++) ds.push_back({dsh[di].sec, dsh[di].idx - a, dsh[di].ord - 4 * a});
        uint64_t rec_bytes = info->bytes_used;
        if (b < n) {
            uint32_t ob = 0;
            hipError_t e;
            if (!hip_ok(e = hipMemcpyAsync(&ob, d_offs + b, 4, hipMemcpyDeviceToHost, st)) || !hip_ok(e = hipStreamSynchronize(st)))
                return c->hipfail(e, "span end");
            rec_bytes = ob;
        }
        // (a batch with a TCP stage ahead of its spans ran it in batch_shifts)
        c->eoc_stage = c->eoc_batch && b == n && !c->tcp_pre;
        if (int rc = process_span(c, d_recs, d_offs, a, b - a, rec_bytes, ns, ds, (uint32_t)info->first_sec, st)) return rc;
        a = b;
    }
    c->last_sec = info->last_sec;
    c->last_nsec = info->last_nsec;
    return 0;
}

int pv_synchronize(pv_ctx *c)
{
    flush_fills(c);
    hipSetDevice(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return c->hipfail(e, "synchronize");
    return 0;
}

namespace {

int ingest_setup(pv_ctx *c)
{
    if (c->copy_stream) return 0;
    hipError_t e;
    // 128 MiB pieces: the top-N merge's cost per batch is per region, not per entry, so larger
    // pieces amortise it (C5 100M: 172.5 / 184.2 / 184.9 Mpkt/s at 64 / 128 / 256 MiB,
    // profiles/r5/c5_chunk*.log)
    size_t chunk = 128ull << 20;
    if (const char *v = getenv("PV_INGEST_CHUNK_MB")) chunk = std::max<size_t>(1, strtoull(v, nullptr, 10)) << 20;
    c->stage_recs = std::min<uint64_t>(c->max_records, chunk / 16 + 1);
    c->stage_bytes = chunk;
    if (const char *v = getenv("PV_INGEST_RING")) c->ring_n = (uint32_t)std::min<unsigned long>(8, std::max<unsigned long>(3, strtoul(v, nullptr, 10)));
    c->pool.reset(new pvi::Pool(pvi::default_threads()));
    if (!hip_ok(e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking))) return c->hipfail(e, "copy stream");
    for (auto &st : c->stage) {
        if (!hip_ok(e = hipHostMalloc((void **)&st.h_recs, chunk + PV_RECS_PAD, hipHostMallocDefault)) ||
            !hip_ok(e = hipHostMalloc((void **)&st.h_offs, c->stage_recs * 4, hipHostMallocDefault)) ||
            !hip_ok(e = hipMalloc(&st.d_recs, chunk + PV_RECS_PAD)) || !hip_ok(e = hipMalloc(&st.d_offs, c->stage_recs * 4)) ||
            !hip_ok(e = hipEventCreateWithFlags(&st.copied, hipEventDisableTiming)))
            return c->hipfail(e, "ingest staging");
        st.sci.resize(1 << 16);
        st.scs.resize(1 << 16);
        // device record index state for a chunk of up to `chunk` bytes
        const uint32_t nseg = (uint32_t)((2 * chunk + PV_IX_SEG - 1) / PV_IX_SEG); // a ring run: tail + chunk
        const size_t bytes = 256 + (size_t)nseg * 8 * 3 + (size_t)(nseg + 1) * 4 * 2 + 64 + st.sci.size() * 8 + 1024;
        if (!hip_ok(e = hipMalloc(&st.d_ix, bytes)) ||
            !hip_ok(e = hipHostMalloc((void **)&st.h_ix, 256 + 64 + st.sci.size() * 8 + 1024, hipHostMallocDefault)))
            return c->hipfail(e, "device index state");
        st.ix_nseg = nseg;
    }
    if (const char *v = getenv("PV_INGEST_INDEX")) c->device_index = strcmp(v, "host") != 0;
    return 0;
}

// The record index of the records at [first, end) of d_base (256-B aligned, first < 256),
// already on the device, on the device (pv_index.hip): offsets (relative to d_base) into
// d_offs, the ts_sec change points into st.sci / st.scs (sorted), st.info as pv_index_records
// fills it (bytes_used relative to d_base), *capped when more complete records follow the
// first stage_recs. `hfirst` is byte `first` in host memory (headers of the first and last
// records). Returns 1 when the validation passes do not settle (adversarial bytes: the caller
// walks the block on the host), < 0 on an error.
int device_index(pv_ctx *c, pv_ctx::Stage &st, const uint8_t *d_base, uint32_t first, const uint8_t *hfirst, size_t L,
                 uint32_t *d_offs, hipStream_t s, bool *capped)
{
    const uint32_t nseg = (uint32_t)((L + PV_IX_SEG - 1) / PV_IX_SEG);
    if (nseg > st.ix_nseg) return c->fail(PV_ECAPACITY, "index block of %zu bytes exceeds the index state", L);
    *capped = false;
    uint8_t *d = st.d_ix;
    PvIxParams X;
    memset(&X, 0, sizeof X);
    size_t at = 256;
    auto take = [&](size_t b) { uint8_t *q = d + at; at += (b + 63) & ~(size_t)63; return q; };
    X.recs = d_base;
    X.bytes = L;
    X.first = first;
    X.nseg = nseg;
    X.frac_lim = c->cfg.ts_nano ? 1000000000u : 1000000u;
    memcpy(&X.sec0, hfirst, 4);
    X.start = (uint64_t *)take((size_t)nseg * 8);
    X.exit[0] = (uint64_t *)take((size_t)nseg * 8);
    X.exit[1] = (uint64_t *)take((size_t)nseg * 8);
    X.cnt = (uint32_t *)take((size_t)nseg * 4);
    X.base = (uint32_t *)take((size_t)(nseg + 1) * 4);
    X.status = (uint32_t *)take(32);
    X.sci = (uint32_t *)take(st.sci.size() * 4);
    X.scs = (uint32_t *)take(st.sci.size() * 4);
    X.offs = d_offs;
    X.max_records = c->stage_recs;
    X.max_changes = (uint32_t)st.sci.size();
    uint32_t *h = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(st.h_ix) + 256); // read-back words
    *st.h_ix = X;
    const PvIxParams *dX = reinterpret_cast<const PvIxParams *>(d);
    const dim3 g((nseg + 255) / 256), b(256);
    hipError_t e;
    if (!hip_ok(e = hipMemcpyAsync(d, st.h_ix, sizeof X, hipMemcpyHostToDevice, s)) ||
        !hip_ok(e = hipMemsetAsync(X.status, 0, 32, s)))
        return c->hipfail(e, "device index");
    hipLaunchKernelGGL(pv_ix_guess, dim3((nseg + 3) / 4), dim3(256), 0, s, dX); // a wave per segment
    // one validation pass, then the scan, the offsets, the change points and the last change's
    // neighbours, read back under one synchronisation: a pass that changed nothing (the guesses
    // were right) settles the chain. Otherwise the passes run on, one read-back each, until they
    // settle, and the rest runs again (its first run only wrote offsets of valid walks).
    const uint32_t pre = 1024; // change points read back with the status; more in a second copy
    const uint32_t secs_grid = (uint32_t)std::min<uint64_t>((c->stage_recs + 255) / 256, (uint64_t)c->cus * 8);
    uint32_t src = 0;
    auto fix_pass = [&]() {
        hipMemsetAsync(X.status, 0, 4, s);
        hipLaunchKernelGGL(pv_ix_fix, g, b, 0, s, dX, src);
        src ^= 1;
    };
    auto rest = [&]() -> hipError_t {
        hipLaunchKernelGGL(pv_ix_scan, dim3(1), dim3(1024), 0, s, dX);
        hipMemsetAsync(X.status + 1, 0, 28, s);
        hipLaunchKernelGGL(pv_ix_write, g, b, 0, s, dX);
        hipLaunchKernelGGL(pv_ix_secs, dim3(std::max(1u, secs_grid)), dim3(256), 0, s, dX, (uint32_t)c->stage_recs);
        hipLaunchKernelGGL(pv_ix_cut, dim3(1), dim3(64), 0, s, dX);
        hipError_t e2 = hipGetLastError();
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h, X.status, 32, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h + 8, X.base + nseg, 4, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h + 10, X.exit[src] + nseg - 1, 8, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h + 16, X.sci, pre * 4, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipMemcpyAsync(h + 16 + st.sci.size(), X.scs, pre * 4, hipMemcpyDeviceToHost, s);
        if (e2 == hipSuccess) e2 = hipStreamSynchronize(s);
        return e2;
    };
    fix_pass();
    if (!hip_ok(e = rest())) return c->hipfail(e, "device index");
    if (h[0] != 0) {
        bool settled = false;
        for (int pass = 1; pass < 64 && !settled; pass++) {
            fix_pass();
            if (!hip_ok(e = hipMemcpyAsync(h, X.status, 4, hipMemcpyDeviceToHost, s)) || !hip_ok(e = hipStreamSynchronize(s)))
                return c->hipfail(e, "device index pass");
            settled = h[0] == 0;
        }
        if (!settled) return 1;
        if (!hip_ok(e = rest())) return c->hipfail(e, "device index");
    }
    const uint64_t total = h[8];
    uint64_t chain_end = 0;
    memcpy(&chain_end, h + 10, 8);
    const uint64_t n = std::min<uint64_t>(total, c->stage_recs);
    pv_index_info &info = st.info;
    memset(&info, 0, sizeof info);
    info.monotone = 1;
    info.n_records = n;
    info.bytes_used = chain_end & ~PV_IX_STOP;
    if (n == 0) return 0;
    const uint32_t nc = h[1];
    const uint32_t last_off = h[3];
    st.cut_o[0] = h[5];
    st.cut_o[1] = h[6];
    if (nc > st.sci.size()) return c->fail(PV_ECAPACITY, "more than %zu ts_sec changes in one ingest chunk", st.sci.size());
    if (nc > pre &&
        (!hip_ok(e = hipMemcpyAsync(h + 16, X.sci, (size_t)nc * 4, hipMemcpyDeviceToHost, s)) ||
         !hip_ok(e = hipMemcpyAsync(h + 16 + st.sci.size(), X.scs, (size_t)nc * 4, hipMemcpyDeviceToHost, s)) ||
         !hip_ok(e = hipStreamSynchronize(s))))
        return c->hipfail(e, "device index change points");
    std::vector<std::pair<uint32_t, uint32_t>> ch(nc);
    for (uint32_t k = 0; k < nc; k++) ch[k] = {h[16 + k], h[16 + st.sci.size() + k]};
    std::sort(ch.begin(), ch.end());
    for (uint32_t k = 0; k < nc; k++) { st.sci[k] = ch[k].first; st.scs[k] = ch[k].second; }
    info.n_sec_changes = nc;
    info.monotone = h[2] ? 0 : 1;
    uint32_t h0[4], h1[4];
    memcpy(h0, hfirst, 16);
    memcpy(h1, hfirst + (last_off - first), 16);
    if (n < total) {
        info.bytes_used = (uint64_t)last_off + 16 + h1[2];
        *capped = true;
    }
    info.first_sec = h0[0];
    info.first_nsec = c->cfg.ts_nano ? (int64_t)h0[1] : (int64_t)h0[1] * 1000;
    info.last_sec = h1[0];
    info.last_nsec = c->cfg.ts_nano ? (int64_t)h1[1] : (int64_t)h1[1] * 1000;
    return 0;
}

// device_index's fallback: the host walk of the block, its offsets copied to d_offs
int host_index_run(pv_ctx *c, pv_ctx::Stage &st, const uint8_t *d_base, uint32_t first, const uint8_t *hfirst, size_t end,
                   uint32_t *d_offs, bool *capped)
{
    (void)d_base;
    pv_index_info &info = st.info;
    if (int rc = pv_index_records(hfirst, end - first, c->cfg.ts_nano, st.h_offs, c->stage_recs, st.sci.data(), st.scs.data(),
                                  (uint32_t)st.sci.size(), &info))
        return c->fail(rc, "record index failed");
    const uint64_t n = info.n_records;
    *capped = false;
    if (n == c->stage_recs && info.bytes_used + 16 <= end - first) {
        uint32_t cl;
        memcpy(&cl, hfirst + info.bytes_used + 8, 4);
        *capped = info.bytes_used + 16 + (uint64_t)cl <= end - first;
    }
    for (uint64_t i = 0; i < n; i++) st.h_offs[i] += first;
    info.bytes_used += first;
    if (info.n_sec_changes > 1 && info.n_sec_changes <= st.sci.size()) {
        const uint32_t cut = st.sci[info.n_sec_changes - 1];
        st.cut_o[0] = st.h_offs[cut - 1];
        st.cut_o[1] = st.h_offs[cut];
    }
    hipError_t e;
    if (n && (!hip_ok(e = hipMemcpyAsync(d_offs, st.h_offs, n * 4, hipMemcpyHostToDevice, c->stream)) ||
              !hip_ok(e = hipStreamSynchronize(c->stream))))
        return c->hipfail(e, "H2D offsets");
    return 0;
}

bool host_pinned(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}


double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

} // namespace

// pv_dns_event_seconds over records in host memory, through the ingest staging (chunked).
static int dns_event_seconds_batch(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                                   const uint32_t *sc_idx, const uint32_t *sc_sec, int64_t *secs, uint32_t max, uint32_t *n);
int pv_dns_event_seconds_host(pv_ctx *c, const uint8_t *recs, size_t bytes, int64_t *secs, uint32_t max, uint32_t *n)
{
    hipSetDevice(c->device);
    *n = 0;
    c->plan_draws = 0;
    if (c->tcp_active) return c->fail(PV_EINVAL, "pv_dns_event_seconds_host after DNS-over-TCP state (call it before the first batch)");
    struct TcpClean { pv_ctx *c; ~TcpClean() { std::lock_guard<std::mutex> g(c->mu); tcp_reset(c); } } clean{c};
    if (int rc = ingest_setup(c)) return rc;
    pv_ctx::Stage &st = c->stage[0];
    size_t pos = 0;
    uint32_t k = 0;
    while (pos < bytes) {
        const size_t L = std::min(c->stage_bytes, bytes - pos);
        int rc = pvi::index_records_parallel(*c->pool, recs + pos, L, c->cfg.ts_nano, st.h_offs, c->stage_recs,
                                             st.sci.data(), st.scs.data(), (uint32_t)st.sci.size(), &st.info, st.h_recs);
        if (rc) return c->fail(rc, "record index failed");
        if (st.info.n_records == 0) return c->fail(PV_ECAPACITY, "record larger than the ingest chunk");
        const size_t used = st.info.bytes_used;
        hipError_t e;
        if (!hip_ok(e = hipMemcpyAsync(st.d_recs, st.h_recs, used, hipMemcpyHostToDevice, c->stream)) ||
            !hip_ok(e = hipMemsetAsync(st.d_recs + used, 0, PV_RECS_PAD, c->stream)) ||
            !hip_ok(e = hipMemcpyAsync(st.d_offs, st.h_offs, st.info.n_records * 4, hipMemcpyHostToDevice, c->stream)))
            return c->hipfail(e, "H2D");
        std::vector<int64_t> part(st.info.n_records + 1);
        uint32_t m = 0;
        {
            std::lock_guard<std::mutex> g(c->mu);
            if ((rc = dns_event_seconds_batch(c, st.d_recs, st.d_offs, &st.info, st.sci.data(), st.scs.data(), part.data(),
                                              (uint32_t)part.size(), &m)))
                return rc;
        }
        for (uint32_t j = 0; j < m; j++) {
            if (k && secs[k - 1] == part[j]) continue; // a second split across chunks
            if (k >= max) return c->fail(PV_ECAPACITY, "more than %u DNS seconds", max);
            secs[k++] = part[j];
        }
        pos += used;
    }
    *n = k;
    return 0;
}

// dnstap input (DnstapInputStream, src/inputs/dnstap/DnstapInputStream.cpp:33-92) into the Net
// and DNS handlers' process_dnstap paths (net/v1 NetStreamHandler.cpp:549-620,832-843;
// dns/v1 DnsStreamHandler.cpp:260-266,839-909,1376-1412). The host decodes the Frame Streams
// file (pv_dnstap.cpp) and lays each event out as a PvDtEv plus a linktype-101 record (IP
// header with the query / response addresses, UDP header, the DNS message); the managers'
// period shifts are applied between spans of events; pv_dnstap_kernel does the accounting.
int dns_period_shift(pv_ctx *c, int64_t sec, int64_t nsec);
// lib::utils::match_subnet(IPv4subnetList &, IPv6subnetList &, const std::string &) as the
// dnstap proxy calls it (libs/visor_utils/utils.cpp:26-80): the std::string is the message's raw
// address bytes, which pcpp::IPv4Address / IPv6Address parse as TEXT (inet_pton on the string up
// to its first NUL; an unparsable one is the unspecified address, which isValid() rejects), so a
// 4- or 16-byte binary address practically never matches
static bool dt_match_subnet(const pv_ctx *c, const std::vector<uint8_t> &raw)
{
    const std::string txt(raw.begin(), std::find(raw.begin(), raw.end(), (uint8_t)0));
    in_addr a4{};
    if (inet_pton(AF_INET, txt.c_str(), &a4) == 1 && a4.s_addr != 0) {
        for (auto &n : c->dt_v4) {
            if (n.second == 0) return true;
            const uint32_t mask = htonl(0xFFFFFFFFu << (32 - n.second));
            if (((a4.s_addr ^ n.first) & mask) == 0) return true;
        }
        return false;
    }
    uint8_t a6[16] = {0};
    static const uint8_t zero[16] = {0};
    if (inet_pton(AF_INET6, txt.c_str(), a6) == 1 && memcmp(a6, zero, 16) != 0) {
        for (auto &n : c->dt_v6) {
            const uint32_t bytes = n.second / 8, bits = n.second % 8;
            bool r = false;
            if (bytes > 0) r = memcmp(n.first.data(), a6, bytes) == 0;
            if ((r || n.second < 8) && bits > 0) r = (n.first[bytes] >> (8 - bits)) == (a6[bytes] >> (8 - bits));
            if (r) return true;
        }
    }
    return false;
}

int pv_set_dnstap_only_hosts(pv_ctx *c, const char *hosts)
{
    if (!c) return PV_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (!hosts) {
        c->dt_v4.clear();
        c->dt_v6.clear();
        c->dt_only_hosts = false;
        return 0;
    }
    // parse_host_specs (libs/visor_utils/utils.cpp:128-164), its error texts. The lists are
    // parsed into locals and committed together with the flag only when every spec parses: a
    // failing call leaves the previous filter as it was (the reference throws from the input
    // proxy's constructor, so no half-applied filter ever exists)
    decltype(c->dt_v4) v4;
    decltype(c->dt_v6) v6;
    const std::string s = hosts;
    size_t pos = 0;
    while (pos < s.size()) {
        const size_t e = s.find(',', pos);
        const std::string host = s.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
        pos = e == std::string::npos ? s.size() : e + 1;
        if (host.empty()) continue;
        const size_t d = host.find('/');
        if (d == std::string::npos) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
        const std::string ip = host.substr(0, d), cs = host.substr(d + 1);
        if (cs.empty() || !std::all_of(cs.begin(), cs.end(), ::isdigit)) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
        const int cidr = atoi(cs.c_str());
        if (ip.find(':') != std::string::npos) {
            std::array<uint8_t, 16> a{};
            if (cidr < 0 || cidr > 128) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
            if (inet_pton(AF_INET6, ip.c_str(), a.data()) != 1) return c->fail(PV_EINVAL, "invalid IPv6 address: %s", ip.c_str());
            v6.push_back({a, (uint32_t)cidr});
        } else {
            in_addr a{};
            if (cidr < 0 || cidr > 32) return c->fail(PV_EINVAL, "invalid CIDR: %s", host.c_str());
            if (inet_pton(AF_INET, ip.c_str(), &a) != 1) return c->fail(PV_EINVAL, "invalid IPv4 address: %s", ip.c_str());
            v4.push_back({a.s_addr, (uint32_t)cidr});
        }
    }
    c->dt_v4 = std::move(v4);
    c->dt_v6 = std::move(v6);
    c->dt_only_hosts = true;
    return 0;
}

int pv_process_dnstap(pv_ctx *c, const uint8_t *buf, size_t bytes, uint32_t msg_type_mask)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (int rc = merged_refuse(c)) return rc;
    hipSetDevice(c->device);
    std::vector<pvi::DtMessage> msgs;
    uint32_t frames = 0;
    pvi::dnstap_decode(buf, bytes, msgs, &frames);
    if (c->dt_only_hosts) {
        // DnstapInputEventProxy::dnstap_cb's only_hosts block, in its branch order: both addresses
        // and neither matches, one address that does not match, and (its final else) every
        // other message: filtered before any handler sees it
        std::vector<pvi::DtMessage> kept;
        for (auto &m : msgs) {
            bool filt;
            if (m.has_qaddr && m.has_raddr) filt = !dt_match_subnet(c, m.qaddr) && !dt_match_subnet(c, m.raddr);
            else if (m.has_qaddr && !dt_match_subnet(c, m.qaddr)) filt = true;
            else if (m.has_raddr && !dt_match_subnet(c, m.raddr)) filt = true;
            else filt = true;
            if (!filt) kept.push_back(std::move(m));
        }
        msgs.swap(kept);
    }
    const size_t n = msgs.size();
    if (n == 0) return 0;
    if (n > 0x3fffffffull) return c->fail(PV_ECAPACITY, "too many dnstap events in one call");
    std::vector<PvDtEv> ev(n);
    std::vector<uint32_t> offs(n);
    std::vector<int64_t> ssec(n), snsec(n);
    std::vector<uint8_t> arena;
    arena.reserve(n * 96 + bytes);
    timespec now{};
    for (size_t j = 0; j < n; j++) {
        const pvi::DtMessage &m = msgs[j];
        PvDtEv &e = ev[j];
        memset(&e, 0, sizeof e);
        const uint32_t t = m.type;
        // the event's timestamp (DnsMetricsManager::process_dnstap :1379-1402): the response
        // time for CLIENT/AUTH/RESOLVER responses, the query time for their queries, else now
        // (also when that time is absent, where the reference leaves the stamp unset)
        int64_t sec = -1, nsec = 0;
        if ((t == 6 || t == 2 || t == 4) && m.has_rsec) { sec = (int64_t)m.rsec; nsec = m.rnsec; }
        else if ((t == 5 || t == 1 || t == 3) && m.has_qsec) { sec = (int64_t)m.qsec; nsec = m.qnsec; }
        if (sec < 0) {
            if (!now.tv_sec) timespec_get(&now, TIME_UTC);
            sec = now.tv_sec;
            nsec = now.tv_nsec;
        }
        ssec[j] = sec;
        snsec[j] = nsec;
        e.sec = (uint32_t)sec;
        e.nsec = (uint32_t)nsec;
        e.size = m.frame_len;
        // Net direction by message type (net/v1 :578-597)
        switch (t) {
        case 5: case 10: case 4: case 1: case 8: case 13: case 12: e.dir = 0; break;
        case 9: case 6: case 3: case 2: case 7: case 14: case 11: e.dir = 1; break;
        default: e.dir = 2;
        }
        e.side = (t >= 1 && t <= 14 && (t & 1) == 0) ? 1 : 0; // responses have even type numbers
        e.l3 = m.has_family ? (m.family == 2 ? 6 : (m.family == 1 ? 4 : 0)) : 0;
        e.l4 = m.has_protocol ? (m.protocol == 1 ? 17 : (m.protocol == 2 ? 6 : 0)) : 0;
        e.qport = m.has_qport ? (uint16_t)m.qport : 0;
        e.filtered = (msg_type_mask && !(t < 32 && ((msg_type_mask >> t) & 1))) ? 1 : 0; // a type past the mask's bits never matches
        // deep sampling: each manager draws per dnstap event in stream order (new_event:
        // net/v1 ...cpp:840, dns/v1 ...cpp:1409); a dnstap_msg_type-filtered event is the DNS
        // manager's process_filtered, new_event(stamp, false): no draw, the last flag.
        // pad[0]: bit 0 not deep for the Net manager, bit 1 for the DNS manager
        if (c->sample_rate < 100) {
            const bool net_deep = c->draws_net.next(c->sample_rate);
            if (!e.filtered) c->dns_deep_now = c->draws_dns.next(c->sample_rate);
            e.pad[0] = (uint8_t)((net_deep ? 0u : 1u) | (c->dns_deep_now ? 0u : 2u));
        }
        const uint8_t *msg = nullptr;
        size_t mlen = 0;
        if (c->dns2_groups) {
            // DNS v2 (dns/v2 ...cpp:1176-1270): the transaction direction by message type, a
            // response with its message ends a transaction, else a query message starts one.
            // pad[1]: direction | response << 2 | a message << 3 | socket protocol << 4
            const uint32_t xd = (t == 5 || t == 6 || t == 1 || t == 2 || t == 13 || t == 14) ? 0u
                              : ((t >= 3 && t <= 4) || (t >= 7 && t <= 12)) ? 1u : 2u;
            uint32_t v2 = xd;
            if (e.side == 1 && m.has_rmsg) { v2 |= 4u | 8u; msg = m.rmsg; mlen = m.rmsg_len; }
            else if (m.has_qmsg) { v2 |= 8u; msg = m.qmsg; mlen = m.qmsg_len; }
            if (m.has_protocol && m.protocol >= 1 && m.protocol <= 7) v2 |= (uint32_t)m.protocol << 4;
            e.pad[1] = (uint8_t)v2;
            e.dns_mode = msg ? PV_DT_MESSAGE : PV_DT_EVENT_ONLY;
        } else if (!m.has_qmsg && !m.has_rmsg) e.dns_mode = PV_DT_SIDE;
        else if (e.side == 0 && m.has_qmsg) { e.dns_mode = PV_DT_MESSAGE; msg = m.qmsg; mlen = m.qmsg_len; }
        else if (e.side == 1 && m.has_rmsg) { e.dns_mode = PV_DT_MESSAGE; msg = m.rmsg; mlen = m.rmsg_len; }
        else e.dns_mode = PV_DT_EVENT_ONLY;
        if (mlen > 65535 - 48) mlen = 65535 - 48; // a DNS message fits 16 bits (TCP framing)
        e.qlen = m.has_qaddr ? (uint8_t)std::min<size_t>(m.qaddr.size(), 255) : 0;
        e.rlen = m.has_raddr ? (uint8_t)std::min<size_t>(m.raddr.size(), 255) : 0;
        if (e.qlen == 4 || e.qlen == 16) memcpy(e.qaddr, m.qaddr.data(), e.qlen);
        if (e.rlen == 4 || e.rlen == 16) memcpy(e.raddr, m.raddr.data(), e.rlen);
        // the record: pcap header, IPv4 (or IPv6) header, UDP header, message
        const bool v6 = e.l3 == 6;
        const uint32_t iph = v6 ? 40 : 20;
        const uint32_t incl = iph + 8 + (uint32_t)mlen;
        const size_t r = arena.size();
        arena.resize(r + ((16 + incl + 3) & ~3u), 0);
        uint8_t *h = arena.data() + r;
        const uint32_t hw[4] = {(uint32_t)sec, c->cfg.ts_nano ? (uint32_t)nsec : (uint32_t)(nsec / 1000), incl, incl};
        memcpy(h, hw, 16);
        uint8_t *ip = h + 16;
        const uint32_t udp_len = 8 + (uint32_t)mlen;
        if (v6) {
            ip[0] = 0x60;
            ip[4] = (uint8_t)(udp_len >> 8); ip[5] = (uint8_t)udp_len;
            ip[6] = 17; ip[7] = 64;
            if (e.qlen == 16) memcpy(ip + 8, e.qaddr, 16);
            if (e.rlen == 16) memcpy(ip + 24, e.raddr, 16);
        } else {
            const uint32_t tot = 20 + udp_len;
            ip[0] = 0x45;
            if (tot <= 65535) { ip[2] = (uint8_t)(tot >> 8); ip[3] = (uint8_t)tot; }
            ip[8] = 64; ip[9] = 17;
            if (e.qlen == 4) memcpy(ip + 12, e.qaddr, 4);
            if (e.rlen == 4) memcpy(ip + 16, e.raddr, 4);
        }
        uint8_t *u = ip + iph;
        u[0] = (uint8_t)(e.qport >> 8); u[1] = (uint8_t)e.qport;
        u[2] = 0; u[3] = 53;
        u[4] = (uint8_t)(udp_len >> 8); u[5] = (uint8_t)udp_len;
        if (mlen) memcpy(u + 8, msg, mlen);
        offs[j] = (uint32_t)r;
        e.rec = (uint32_t)r;
        e.moff = (uint32_t)(r + 16 + iph + 8);
        e.mlen = (uint32_t)mlen;
        if (arena.size() > 0xfffff000ull) return c->fail(PV_ECAPACITY, "dnstap events exceed 4 GiB of records");
    }
    arena.resize(arena.size() + PV_RECS_PAD, 0);
    hipError_t e;
    uint8_t *d_arena = nullptr;
    uint32_t *d_offs = nullptr;
    PvDtEv *d_ev = nullptr;
    struct Free {
        void *p[3];
        ~Free() { for (void *q : p) if (q) hipFree(q); }
    } fr{{nullptr, nullptr, nullptr}};
    if (!hip_ok(e = hipMalloc(&d_arena, arena.size())) || !hip_ok(e = hipMalloc(&d_offs, n * 4)) ||
        !hip_ok(e = hipMalloc(&d_ev, n * sizeof(PvDtEv))))
        return c->hipfail(e, "dnstap buffers");
    fr.p[0] = d_arena; fr.p[1] = d_offs; fr.p[2] = d_ev;
    hipStream_t st = c->stream;
    if (!hip_ok(e = hipMemcpyAsync(d_arena, arena.data(), arena.size(), hipMemcpyHostToDevice, st)) ||
        !hip_ok(e = hipMemcpyAsync(d_offs, offs.data(), n * 4, hipMemcpyHostToDevice, st)) ||
        !hip_ok(e = hipMemcpyAsync(d_ev, ev.data(), n * sizeof(PvDtEv), hipMemcpyHostToDevice, st)))
        return c->hipfail(e, "dnstap H2D");
    ensure_started(c, ssec[0], snsec[0]);
    const uint32_t np = c->cfg.num_periods;
    auto span = [&](size_t a, size_t b) -> int {
        if (b <= a) return 0;
        PvParams P;
        params_common(c, P, d_arena, d_offs + a, b - a);
        P.linktype = 101;
        P.tap = 1;
        P.f_flags = 0; // the DNS filters do not apply to dnstap events (only dnstap_msg_type)
        P.dq = reinterpret_cast<uint64_t *>(d_ev + a);
        P.gbase = c->global_base + c->records_seen;
        P.slot_of[0] = c->net.slot_at(0);
        P.dslot_of[0] = c->dns.slot_at(0);
        P.sum = c->d_sum;
        P.cpc = c->d_cpc;
        P.tkeys = c->d_tkeys;
        P.tcnt = c->d_tcnt;
        P.taux = c->d_taux;
        P.tcap_log2 = c->tcap_log2;
        P.reg_log2 = c->reg_log2;
        P.arena = c->d_arena;
        P.arena_top = c->d_arena_top;
        P.arena_cap = c->arena_cap;
        P.flags = c->d_status + ST_FLAGS;
        P.tab_live = c->d_tab_live;
        P.ovf = c->d_ovf;
        P.ovf_cnt = c->d_ovf_cnt;
        P.ovf_cap = c->ovf_cap;
        const uint32_t blocks = (uint32_t)((b - a + 255) / 256);
        // DNS v2: transaction events, one 256-event region per block (pv_xact_compact), paired by
        // the transaction stage as a pcap batch's are
        P.want_events = c->dns2_groups ? 1u : 0u;
        if (P.want_events) {
            if (b - a > c->max_records) return c->fail(PV_ECAPACITY, "a dnstap period span exceeds max_records events");
            P.events = c->d_events;
            P.eecs = c->d_eecs;
            P.ekeys = c->d_ekeys;
            P.blk_events = c->d_blk_events;
            P.skeys = c->d_skeys;
            P.svals = c->d_svals;
            P.n_events = c->d_status + ST_NEV;
            P.n_keys = c->d_status + ST_NKEYS;
            P.wt_per_block = 4; // 64-record tiles: 256 events per block
            P.grid_main = blocks;
            if (c->n_pend == 0) c->pend_base = (int64_t)c->records_seen - 1;
            P.ekey_base = (uint32_t)((int64_t)c->records_seen - c->pend_base);
            launch_fill32(c, c->d_status, ST_ALLOC, 0);
        }
        launch_fill32(c, c->d_status + ST_FLAGS, 1, 0);
        flush_fills(c);
        *c->h_params = P;
        if (!hip_ok(e = upload_params(c->d_params, c->h_params, sizeof P, st)))
            return c->hipfail(e, "parameter upload");
        hipLaunchKernelGGL(pv_dnstap_kernel, dim3(blocks), dim3(256), 0, st, (const PvParams *)c->d_params);
        if (P.want_events) hipLaunchKernelGGL(pv_xact_compact, dim3(blocks), dim3(256), 0, st, (const PvParams *)c->d_params, 0u, 0u);
        if (!hip_ok(e = hipGetLastError()) ||
            !hip_ok(e = hipMemcpyAsync(c->h_status, c->d_status, ST_RB_WORDS * 4, hipMemcpyDeviceToHost, st)) ||
            !hip_ok(e = hipStreamSynchronize(st)))
            return c->hipfail(e, "pv_dnstap_kernel");
        if (P.want_events) {
            const uint32_t nev = c->h_status[ST_NEV], nresp = c->h_status[ST_NRESP];
            if (int rc = pair_stage(c, P, nev, c->h_status[ST_NKEYS], nresp, b - a, st, (uint64_t)blocks * P.wt_per_block * 64u))
                return rc;
        }
        if (int rc = drain_overflow(c, st)) return rc;
        uint32_t flags = 0;
        if (!hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
        if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "top-N table full: raise table_log2");
        if (flags & PVF_ARENA_FULL) return c->fail(PV_ECAPACITY, "top-N name arena full");
        c->net.clean[P.slot_of[0]] = false;
        c->dns.clean[P.dslot_of[0]] = false;
        c->records_seen += b - a;
        return purge_tables(c, st);
    };
    size_t a = 0;
    for (size_t j = 0; j < n; j++) {
        // each manager shifts on the first of its events at or after its next shift
        // (AbstractMetricsManager::new_event, src/AbstractMetricsManager.h:318-333)
        const bool ns = np > 1 && ssec[j] >= c->net.next_shift_sec;
        const bool ds = np > 1 && ssec[j] >= c->dns.next_shift_sec;
        if (!ns && !ds) continue;
        if (int rc = span(a, j)) return rc;
        if (ns) { clear_part(c, PART_NET, c->net.slot_at(1)); win_shift(c, c->net, ssec[j]); }
        if (ds && c->dns2_groups) {
            // DNS v2's on_period_shift purge of the open transactions (as a heartbeat shift)
            if (int rc = dns_period_shift(c, ssec[j], snsec[j])) return rc;
        } else if (ds) { clear_part(c, PART_DNS, c->dns.slot_at(1)); win_shift(c, c->dns, ssec[j]); }
        a = j;
    }
    if (int rc = span(a, n)) return rc;
    c->last_sec = ssec[n - 1];
    c->last_nsec = snsec[n - 1];
    return 0;
}

// pcapng -> classic pcap records with nanosecond fractions (pv_pcapng.cpp). out == NULL (or too
// small): only *out_bytes / *n_records are set (PV_ECAPACITY when out is too small).
int pv_pcapng_records(const uint8_t *buf, size_t bytes, uint8_t *out, size_t out_cap, size_t *out_bytes,
                      uint32_t *linktype, uint64_t *n_records)
{
    std::vector<uint8_t> v;
    const int rc = pvi::pcapng_to_records(buf, bytes, &v, linktype, n_records);
    if (rc == pvi::PVNG_ELINKTYPES) return PV_EUNSUPPORTED;
    if (rc) return PV_EINVAL;
    *out_bytes = v.size();
    if (!out) return 0;
    if (out_cap < v.size()) return PV_ECAPACITY;
    memcpy(out, v.data(), v.size());
    return 0;
}

// One TPACKET_V3 ring block (AFPacket::walk_block, src/inputs/pcap/afpacket.cpp:72-86) ->
// classic pcap records with nanosecond fractions, appended at out + *out_bytes. As the
// reference hands them on, every packet takes the block's ts_last_pkt (not its own tp_sec /
// tp_nsec) and its snap length as both lengths (RawPacket(data, tp_snaplen, ...)).
int pv_tpacket3_block_records(const uint8_t *block, size_t block_size, uint8_t *out, size_t out_cap, size_t *out_bytes,
                              uint64_t *n_records)
{
    if (block_size < sizeof(tpacket_block_desc)) return PV_EINVAL;
    const tpacket_block_desc *bd = reinterpret_cast<const tpacket_block_desc *>(block);
    const tpacket_hdr_v1 &h = bd->hdr.bh1;
    const uint32_t ts_sec = h.ts_last_pkt.ts_sec, ts_nsec = h.ts_last_pkt.ts_nsec;
    size_t o = *out_bytes;
    uint64_t n = 0;
    size_t p = h.offset_to_first_pkt;
    for (uint32_t i = 0; i < h.num_pkts; i++) {
        if (p + sizeof(tpacket3_hdr) > block_size) return PV_EINVAL;
        tpacket3_hdr ph;
        memcpy(&ph, block + p, sizeof ph);
        const size_t d = p + ph.tp_mac;
        if (d + ph.tp_snaplen > block_size) return PV_EINVAL;
        if (o + 16 + ph.tp_snaplen > out_cap) return PV_ECAPACITY;
        const uint32_t rh[4] = {ts_sec, ts_nsec, ph.tp_snaplen, ph.tp_snaplen};
        memcpy(out + o, rh, 16);
        memcpy(out + o + 16, block + d, ph.tp_snaplen);
        o += 16 + ph.tp_snaplen;
        n++;
        if (i + 1 < h.num_pkts && ph.tp_next_offset == 0) return PV_EINVAL;
        p += ph.tp_next_offset;
    }
    *out_bytes = o;
    if (n_records) *n_records += n;
    return 0;
}

// Frame Streams decode only (tests): data frames read and dnstap MESSAGE events found.
int pv_dnstap_count(const uint8_t *buf, size_t bytes, uint32_t *frames, uint32_t *events)
{
    std::vector<pvi::DtMessage> msgs;
    pvi::dnstap_decode(buf, bytes, msgs, frames);
    *events = (uint32_t)msgs.size();
    return 0;
}

// Host-memory path with the record index on the device. The blob is cut into fixed
// chunk-sized pieces in host order, so their H2D copies stream back to back (a producer
// thread, two copy streams, a ring of ring_n device buffers of two chunks each) without
// waiting on any index. The calling thread, per piece: moves the previous batch's tail (the
// records after its last ts_sec cut) in front of the piece on the device, indexes the joined
// run there (pv_index.hip), cuts it at its last ts_sec boundary and runs the batch. The host
// reads a few header words only. Batches are cut as pv_process_host's host-index path cuts
// them (at most stage_recs records, ending at a ts_sec boundary unless the data ends).
int process_host_ring(pv_ctx *c, const uint8_t *recs, size_t bytes)
{
    const size_t L = c->stage_bytes; // a multiple of 256: runs start 256-B aligned (+ first)
    hipError_t e;
    const uint32_t NR = c->ring_n;
    for (uint32_t q = 0; q < NR; q++) {
        pv_ctx::Ring &r = c->ring[q];
        if (r.d_buf) continue;
        if (!hip_ok(e = hipMalloc(&r.d_buf, 2 * L + PV_RECS_PAD)) || !hip_ok(e = hipMalloc(&r.d_offs, c->stage_recs * 4)) ||
            !hip_ok(e = hipEventCreateWithFlags(&r.landed, hipEventDisableTiming)) ||
            // on the context's stream: a null-stream memset is not ordered with the
            // non-blocking copy streams and could land after a piece's copy
            !hip_ok(e = hipMemsetAsync(r.d_buf, 0, 2 * L + PV_RECS_PAD, c->stream)) ||
            !hip_ok(e = hipStreamSynchronize(c->stream)))
            return c->hipfail(e, "ingest ring");
    }
    if (!c->copy_stream2 && !hip_ok(e = hipStreamCreateWithFlags(&c->copy_stream2, hipStreamNonBlocking)))
        return c->hipfail(e, "copy stream");
    const bool pinned = host_pinned(recs);
    if (!pinned)
        for (uint32_t q = 0; q < NR; q++)
            if (!c->ring[q].h_stage && !hip_ok(e = hipHostMalloc((void **)&c->ring[q].h_stage, L, hipHostMallocDefault)))
                return c->hipfail(e, "ingest staging");
    const uint64_t npieces = (bytes + L - 1) / L;
    // producer: piece p's copy into ring slot p % NR at offset L. Slot p % NR last held run
    // p - NR, whose batches are done and whose tail run p - NR + 1 has moved out: issued once the
    // consumer has finished run p - NR + 1 (freed > p - NR), so up to NR - 2 pieces ahead of it. The consumer synchronises its stream
    // after each run, so the host-side order is the device-side order.
    std::mutex mu;
    std::condition_variable cv;
    uint64_t issued = 0, freed = 0;
    bool abort = false;
    int prod_rc = 0;
    std::string prod_err;
    auto producer = [&] {
        for (uint64_t k = 0; k < npieces; k++) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return abort || k < freed + NR; });
                if (abort) return;
            }
            pv_ctx::Ring &r = c->ring[k % NR];
            const size_t len = std::min(L, bytes - k * L);
            const uint8_t *src = recs + k * L;
            if (!pinned) {
                auto t1 = std::chrono::steady_clock::now();
                pvi::copy_parallel(*c->pool, r.h_stage, src, len);
                src = r.h_stage;
                c->ingest_ms[0] += ms_since(t1);
            }
            hipStream_t cs = (k & 1) ? c->copy_stream2 : c->copy_stream;
            const auto ti = std::chrono::steady_clock::now();
            const bool ok = hip_ok(e = hipMemcpyAsync(r.d_buf + L, src, len, hipMemcpyHostToDevice, cs)) &&
                            hip_ok(e = hipEventRecord(r.landed, cs));
            c->ingest_ms[2] += ms_since(ti); // host time the copy's issue takes (a blocking copy shows here)
            if (!ok) {
                std::lock_guard<std::mutex> g(mu);
                prod_rc = PV_EHIP;
                prod_err = std::string("H2D: ") + hipGetErrorString(e);
                abort = true;
                cv.notify_all();
                return;
            }
            std::lock_guard<std::mutex> g(mu);
            issued = k + 1;
            cv.notify_all();
        }
    };
    std::thread th(producer);
    pv_ctx::Stage &st = c->stage[0]; // index state, change lists, host offsets (fallback)
    int rc = 0;
    size_t tail = 0;
    const uint8_t *tail_src = nullptr;
    for (uint64_t k = 0; k < npieces && !rc; k++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return abort || issued > k; });
            if (abort) break;
        }
        HP(0);
        pv_ctx::Ring &r = c->ring[k % NR];
        const size_t len = std::min(L, bytes - k * L);
        const bool last_piece = k + 1 == npieces;
        // the run: the tail at [L - tail, L), the piece at [L, L + len); b is 256-B aligned and
        // the first record at b + first; hf is that record in host memory
        uint8_t *b = r.d_buf + ((L - tail) & ~(size_t)255);
        uint32_t first = (uint32_t)((L - tail) & 255);
        const uint8_t *hf = recs + k * L - tail;
        size_t end = first + tail + len;
        auto t0 = std::chrono::steady_clock::now();
        if (!hip_ok(e = hipStreamWaitEvent(c->stream, r.landed, 0)) ||
            (tail && !hip_ok(e = hipMemcpyAsync(b + first, tail_src, tail, hipMemcpyDeviceToDevice, c->stream)))) {
            rc = c->hipfail(e, "ingest run");
            break;
        }
        tail = 0;
        for (;;) {
            bool capped = false;
            int ix = device_index(c, st, b, first, hf, end, r.d_offs, c->stream, &capped);
            if (ix < 0) { rc = ix; break; }
            if (ix > 0 && (rc = host_index_run(c, st, b, first, hf, end, r.d_offs, &capped))) break;
            pv_index_info info = st.info;
            c->ingest_ms[1] += ms_since(t0);
            HP(1);
            const bool more = !last_piece || capped; // records follow this batch
            if (info.n_records == 0) {
                if (!last_piece && end - first >= L) { rc = c->fail(PV_ECAPACITY, "record larger than the ingest chunk"); break; }
                if (!last_piece) { tail = end - first; tail_src = b + first; }
                break;
            }
            // a batch that more records follow ends at its last ts_sec boundary when it spans
            // more than one second, so a period shift and the DNS records of its first second
            // reach the device in the same batch
            if (more && info.n_sec_changes > 1 && info.n_sec_changes <= st.sci.size()) {
                const uint32_t cut = st.sci[info.n_sec_changes - 1];
                const uint32_t o[2] = {st.cut_o[0], st.cut_o[1]}; // the offsets either side of the cut
                info.n_records = cut;
                info.bytes_used = o[1];
                info.n_sec_changes -= 1;
                uint32_t h[2];
                memcpy(h, hf + (o[0] - first), 8);
                info.last_sec = h[0];
                info.last_nsec = c->cfg.ts_nano ? (int64_t)h[1] : (int64_t)h[1] * 1000;
                capped = true;
            }
            auto t2 = std::chrono::steady_clock::now();
            HP(2);
            c->eoc_batch = c->eoc_armed && !capped && last_piece; // the data ends with this batch
            rc = pv_process_device(c, b, r.d_offs, &info, st.sci.data(), st.scs.data(), nullptr);
            if (!rc) rc = pv_synchronize(c);
            HP(8);
            c->ingest_ms[3] += ms_since(t2);
            if (rc) break;
            t0 = std::chrono::steady_clock::now();
            const size_t used = info.bytes_used;
            const size_t rest = end - used;
            if (!capped && last_piece) break;          // the data ends (at most a partial record)
            if (!last_piece && (!capped || rest <= L)) {
                if (rest > L) { rc = c->fail(PV_ECAPACITY, "record larger than the ingest chunk"); break; }
                tail = rest;
                tail_src = b + used;
                break;
            }
            // more batches from this run, in place
            hf += used - first;
            b += used & ~(size_t)255;
            first = (uint32_t)(used & 255);
            end -= used & ~(size_t)255;
        }
        {
            std::lock_guard<std::mutex> g(mu);
            freed = k; // slot (k - 1) % NR is free: its tail has moved into this run
            cv.notify_all();
        }
        HP(9);
    }
    {
        std::lock_guard<std::mutex> g(mu);
        if (rc) abort = true;
        freed = npieces + NR;
        cv.notify_all();
    }
    th.join();
    hipStreamSynchronize(c->copy_stream);
    hipStreamSynchronize(c->copy_stream2);
    if (rc) return rc;
    if (prod_rc) return c->fail(prod_rc, "%s", prod_err.c_str());
    return 0;
}

// Host-memory path, pipelined over chunks of the record blob: a producer thread stages
// chunk k + 1 (parallel copy into pinned memory unless the caller's buffer is already
// pinned, parallel record index, H2D on the copy stream) while the calling thread runs
// chunk k's kernels. Results equal one pv_process_device per chunk, in order.
int pv_set_bpf(pv_ctx *c, const pv_bpf_insn *prog, uint32_t n)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (n == 0) { c->bpf.clear(); return 0; }
    if (pv_bpf_validate(prog, n)) return c->fail(PV_EINVAL, "invalid BPF program (classic-BPF checker)");
    c->bpf.assign(prog, prog + n);
    c->bpf_dirty = true;
    return 0;
}

namespace {
int process_host_block(pv_ctx *c, const uint8_t *recs, size_t bytes);
}

int pv_process_host(pv_ctx *c, const uint8_t *recs, size_t bytes)
{
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (int rc = merged_refuse(c)) return rc;
        c->in_host = true;
    }
    // (the pcap input's BPF filter, PcapInputStream.cpp:485-488, runs on the device on each batch:
    // pv_process_device)
    const int rc = process_host_block(c, recs, bytes);
    std::lock_guard<std::mutex> g(c->mu);
    c->in_host = false;
    c->eoc_armed = c->eoc_batch = c->eoc_stage = false;
    return rc;
}

namespace {
int process_host_block(pv_ctx *c, const uint8_t *recs, size_t bytes)
{
    hipSetDevice(c->device);
    if (int rc = ingest_setup(c)) return rc;
    if (c->device_index && bytes >= 4096) return process_host_ring(c, recs, bytes);
    const bool pinned = host_pinned(recs);
    std::mutex mu;
    std::condition_variable cv;
    int state[2] = {0, 0};        // 0 free, 1 ready
    bool prod_done = false, abort = false;
    uint64_t nchunks = 0;
    int prod_rc = 0;
    std::string prod_err;
    auto producer = [&] {
        size_t pos = 0;
        uint64_t k = 0;
        int rc = 0;
        while (pos < bytes) {
            pv_ctx::Stage &st = c->stage[k & 1];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return state[k & 1] == 0 || abort; });
                if (abort) break;
            }
            const size_t L = std::min(c->stage_bytes, bytes - pos);
            const uint8_t *src = recs + pos;
            auto t1 = std::chrono::steady_clock::now();
            // pageable source: copied into pinned staging by the threads that index it
            rc = pvi::index_records_parallel(*c->pool, src, L, c->cfg.ts_nano, st.h_offs, c->stage_recs, st.sci.data(),
                                             st.scs.data(), (uint32_t)st.sci.size(), &st.info, pinned ? nullptr : st.h_recs);
            if (rc) { prod_err = "record index failed"; break; }
            const uint8_t *base = pinned ? src : st.h_recs;
            c->ingest_ms[pinned ? 1 : 0] += ms_since(t1);
            if (st.info.n_records == 0) {
                if (L == c->stage_bytes && pos + L < bytes) { rc = PV_ECAPACITY; prod_err = "record larger than the ingest chunk"; }
                break;
            }
            // a chunk that is not the last ends at a ts_sec boundary when it spans more than
            // one second, so a period shift and the DNS records of its first second reach
            // the device in the same batch
            if (pos + st.info.bytes_used < bytes && st.info.n_sec_changes > 1 &&
                st.info.n_sec_changes <= st.sci.size()) {
                const uint32_t last = st.sci[st.info.n_sec_changes - 1];
                st.info.n_records = last;
                st.info.bytes_used = st.h_offs[last];
                st.info.n_sec_changes -= 1;
                const uint32_t prev = st.h_offs[last - 1];
                uint32_t h[2];
                memcpy(h, base + prev, 8);
                st.info.last_sec = h[0];
                st.info.last_nsec = c->cfg.ts_nano ? (int64_t)h[1] : (int64_t)h[1] * 1000;
            }
            auto t2 = std::chrono::steady_clock::now();
            const size_t used = st.info.bytes_used;
            hipError_t e = hipSuccess;
            const bool ok = hip_ok(e = hipMemcpyAsync(st.d_recs, base, used, hipMemcpyHostToDevice, c->copy_stream)) &&
                             hip_ok(e = hipMemsetAsync(st.d_recs + used, 0, PV_RECS_PAD, c->copy_stream)) &&
                             hip_ok(e = hipMemcpyAsync(st.d_offs, st.h_offs, st.info.n_records * 4, hipMemcpyHostToDevice,
                                                       c->copy_stream));
            if (!ok || !hip_ok(e = hipEventRecord(st.copied, c->copy_stream))) {
                rc = PV_EHIP;
                prod_err = std::string("H2D: ") + hipGetErrorString(e);
                break;
            }
            c->ingest_ms[2] += ms_since(t2);
            pos += used;
            // the final batch: no complete record follows (at most a partial one)
            {
                const size_t rest = bytes - pos;
                uint32_t cl = 0;
                if (rest >= 16) memcpy(&cl, recs + pos + 8, 4);
                st.last = rest < 16 || 16 + (size_t)cl > rest;
            }
            std::lock_guard<std::mutex> g(mu);
            state[k & 1] = 1;
            k++;
            cv.notify_all();
        }
        std::lock_guard<std::mutex> g(mu);
        prod_rc = rc;
        prod_done = true;
        nchunks = k;
        cv.notify_all();
    };
    std::thread th(producer);
    int rc = 0;
    for (uint64_t k = 0;; k++) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return state[k & 1] == 1 || (prod_done && k >= nchunks); });
            if (state[k & 1] != 1) break;
        }
        pv_ctx::Stage &st = c->stage[k & 1];
        auto t0 = std::chrono::steady_clock::now();
        hipError_t e = hipStreamWaitEvent(c->stream, st.copied, 0);
        if (!hip_ok(e)) rc = c->hipfail(e, "stream wait");
        c->eoc_batch = c->eoc_armed && st.last;
        if (!rc) rc = pv_process_device(c, st.d_recs, st.d_offs, &st.info, st.sci.data(), st.scs.data(), nullptr);
        if (!rc) rc = pv_synchronize(c);
        c->ingest_ms[3] += ms_since(t0);
        std::lock_guard<std::mutex> g(mu);
        state[k & 1] = 0;
        if (rc) abort = true;
        cv.notify_all();
        if (rc) break;
    }
    th.join();
    hipStreamSynchronize(c->copy_stream);
    if (rc) return rc;
    if (prod_rc) return c->fail(prod_rc, "%s", prod_err.c_str());
    return 0;
}
} // namespace

// The device record index (pv_index.hip) of one block in host memory, filled as
// pv_index_records fills its outputs (a block of at most one ingest chunk).
int pv_index_records_device(pv_ctx *c, const uint8_t *recs, size_t bytes, uint32_t *offsets, uint64_t max_records,
                            uint32_t *sc_idx, uint32_t *sc_sec, uint32_t max_changes, pv_index_info *info)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (int rc = ingest_setup(c)) return rc;
    if (bytes > c->stage_bytes) return c->fail(PV_EINVAL, "block of %zu bytes exceeds the ingest chunk", bytes);
    if (bytes < 16) { // no complete record header
        memset(info, 0, sizeof *info);
        info->monotone = 1;
        return 0;
    }
    pv_ctx::Stage &st = c->stage[0];
    hipError_t e;
    if (!hip_ok(e = hipMemcpyAsync(st.d_recs, recs, bytes, hipMemcpyHostToDevice, c->copy_stream)) ||
        !hip_ok(e = hipMemsetAsync(st.d_recs + bytes, 0, PV_RECS_PAD, c->copy_stream)))
        return c->hipfail(e, "H2D");
    bool capped = false;
    hipStreamSynchronize(c->copy_stream);
    int rc = device_index(c, st, st.d_recs, 0, recs, bytes, st.d_offs, c->stream, &capped);
    if (rc < 0) return rc;
    if (rc > 0 && (rc = host_index_run(c, st, st.d_recs, 0, recs, bytes, st.d_offs, &capped))) return rc;
    const uint64_t n = std::min<uint64_t>(st.info.n_records, max_records);
    if (n && (!hip_ok(e = hipMemcpyAsync(offsets, st.d_offs, n * 4, hipMemcpyDeviceToHost, c->copy_stream)) ||
              !hip_ok(e = hipStreamSynchronize(c->copy_stream))))
        return c->hipfail(e, "D2H offsets");
    *info = st.info;
    info->n_records = n;
    uint32_t nch = (uint32_t)st.info.n_sec_changes;
    if (n && n < st.info.n_records) {
        // capped at max_records: the walk as pv_index_records stops it there
        uint32_t hl[4];
        memcpy(hl, recs + offsets[n - 1], 16);
        info->bytes_used = offsets[n - 1] + 16 + (uint64_t)hl[2];
        info->last_sec = hl[0];
        info->last_nsec = c->cfg.ts_nano ? (int64_t)hl[1] : (int64_t)hl[1] * 1000;
        while (nch && st.sci[nch - 1] >= n) nch--;
        info->n_sec_changes = nch;
        // monotonicity of the first n records
        info->monotone = 1;
        for (uint32_t k = 1; k < nch; k++)
            if (st.scs[k] < st.scs[k - 1]) info->monotone = 0;
    }
    const uint32_t nc = std::min<uint32_t>(nch, max_changes);
    for (uint32_t k = 0; k < nc; k++) { sc_idx[k] = st.sci[k]; sc_sec[k] = st.scs[k]; }
    return nch > max_changes ? PV_ECAPACITY : 0;
}

int pv_ingest_timing(pv_ctx *c, double *ms4, int reset)
{
    for (int i = 0; i < 4; i++) ms4[i] = c->ingest_ms[i];
    if (reset) for (double &v : c->ingest_ms) v = 0;
    return 0;
}

int pv_host_register(void *p, size_t bytes)
{
    return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? 0 : PV_EHIP;
}

int pv_host_unregister(void *p)
{
    return hipHostUnregister(p) == hipSuccess ? 0 : PV_EHIP;
}

int pv_index_records_mt(const uint8_t *recs, size_t bytes, uint32_t ts_nano, uint32_t *offsets, uint64_t max_records,
                        uint32_t *sc_idx, uint32_t *sc_sec, uint32_t max_changes, pv_index_info *info,
                        uint32_t nthreads)
{
    pvi::Pool pool(nthreads ? nthreads : pvi::default_threads());
    return pvi::index_records_parallel(pool, recs, bytes, ts_nano, offsets, max_records, sc_idx, sc_sec, max_changes,
                                       info);
}

int pv_set_start_tstamp(pv_ctx *c, int64_t sec, int64_t nsec)
{
    std::lock_guard<std::mutex> g(c->mu);
    return ensure_started(c, sec, nsec);
}

int pv_set_end_tstamp(pv_ctx *c, int64_t sec, int64_t nsec)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->started) return 0;
    // end_tstamp_signal: the live bucket of each manager becomes read-only
    c->net.meta[c->net.slots.front()].set_read_only(sec, nsec);
    c->dns.meta[c->dns.slots.front()].set_read_only(sec, nsec);
    c->ended = true;
    return 0;
}

// heartbeat_signal -> StreamMetricsHandler::check_period_shift in both handlers
// (src/AbstractMetricsManager.h:462-470; net/v1/NetStreamHandler.cpp:99-102,
// dns/v1/DnsStreamHandler.cpp:219-222): each manager shifts its window at `stamp` when
// num_periods > 1 and stamp.sec has reached its next shift, with no event. The DNS manager's
// on_period_shift (dns/v1/DnsStreamHandler.h:252-267; v2 .h:440-453) then purges the open
// transactions the stamp expires (timed out in the new live bucket) and takes the slow
// thresholds from the bucket just closed.
int pv_check_period_shift(pv_ctx *c, int64_t sec, int64_t nsec)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (int rc = merged_refuse(c)) return rc;
    hipSetDevice(c->device);
    if (!c->started || c->cfg.num_periods <= 1) return 0;
    if (sec >= c->net.next_shift_sec) {
        clear_part(c, PART_NET, c->net.slot_at(1));
        c->net.clean[c->net.slot_at(1)] = false;
        win_shift(c, c->net, sec, nsec);
    }
    if (sec < c->dns.next_shift_sec) return 0;
    return dns_period_shift(c, sec, nsec);
}

// The DNS manager's shift at `sec` with no event (a heartbeat, or a dnstap span boundary): the
// new live bucket, DnsMetricsManager::on_period_shift's purge of the open transactions through
// the pairing stage, the slow thresholds of the bucket just closed
int dns_period_shift(pv_ctx *c, int64_t sec, int64_t nsec)
{
    hipStream_t st = c->stream;
    const uint32_t s0 = c->dns.slot_at(0), s1 = c->dns.slot_at(1);
    clear_part(c, PART_DNS, s1);
    c->dns.clean[s1] = false;
    const bool xacts = (c->dns_groups & PV_DNS_TRANSACTIONS) || c->dns2_groups;
    if (xacts && c->n_pend > 0) {
        // the carried queries through the pairing stage with one shift at the stamp and no
        // events: purge_period() times out those with stamp.sec >= ttl_s + start.sec
        PvParams P;
        params_common(c, P, nullptr, nullptr, 0);
        P.n_dshift = 1;
        P.dthresh[0] = sec;
        P.dskip_before = 0;
        P.dslot_of[0] = s0;
        P.dslot_of[1] = s1;
        P.slot_of[0] = c->net.slot_at(0);
        P.sum = c->d_sum;
        P.cpc = c->d_cpc;
        P.tkeys = c->d_tkeys;
        P.tcnt = c->d_tcnt;
        P.taux = c->d_taux;
        P.tcap_log2 = c->tcap_log2;
        P.reg_log2 = c->reg_log2;
        P.arena = c->d_arena;
        P.arena_top = c->d_arena_top;
        P.arena_cap = c->arena_cap;
        P.tab_live = c->d_tab_live; // global_add counts the entries it creates
        P.events = c->d_events;
        P.eecs = c->d_eecs;
        P.gbase = c->global_base + c->records_seen;
        P.ekey_base = (uint32_t)((int64_t)c->records_seen - c->pend_base);
        P.flags = c->d_status + ST_FLAGS;
        flush_fills(c);
        if (int rc = pair_stage(c, P, 0, 0, 0, 0, st, 0)) return rc;
    } else if (xacts && ((c->dns_groups & PV_DNS_QUANTILES) || (c->dns2_groups & PV_DNS2_XACT_TIMES))) {
        // nothing open: only the slow thresholds of the closed bucket (kept when it had none)
        if (int rc = sync_xvals(c)) return rc;
        const uint32_t sg = s0 | (c->gen[s0] << 8);
        std::vector<uint64_t> fr, to, t2[3];
        for (auto &v : c->xvals_host) {
            if (v.slot != sg) continue;
            if (v.kind == XV_FROM_US) fr.push_back(v.bits);
            else if (v.kind == XV_TO_US) to.push_back(v.bits);
            else if (v.kind >= XV2_TIME && v.kind < XV2_TIME + 3) t2[v.kind - XV2_TIME].push_back(v.bits);
        }
        if (!fr.empty()) c->from90 = (float)quantile_at(fr, 0.90);
        if (!to.empty()) c->to90 = (float)quantile_at(to, 0.90);
        for (uint32_t d = 0; d < 3; d++)
            if (!t2[d].empty()) c->p90_2[d] = (float)quantile_at(t2[d], 0.90);
    }
    win_shift(c, c->dns, sec, nsec);
    c->dns_shifts.emplace_back(sec, c->dns.slot_at(0));
    c->dns_shift_ord.emplace_back(sec, c->dns.ordinal);
    flush_fills(c);
    hipError_t e = hipStreamSynchronize(st);
    return hip_ok(e) ? 0 : c->hipfail(e, "heartbeat period shift");
}

} // extern "C"
extern "C" {

int pv_state_regions(pv_ctx *c, void **sum_ptr, size_t *sum_bytes, void **min_ptr, size_t *min_bytes)
{
    flush_fills(c);
    *sum_ptr = c->d_sum;
    *sum_bytes = (size_t)PV_SLOTS * PV_SUM_WORDS * 8;
    *min_ptr = c->d_cpc;
    *min_bytes = (size_t)PV_SLOTS * PV_MIN_WORDS * 8;
    return 0;
}

// record: u32 table, u64 key, u64 count, u16 name_len, name bytes
int pv_export_topn(pv_ctx *c, uint8_t **buf, size_t *bytes)
{
    flush_fills(c);
    std::vector<uint8_t> o;
    std::vector<uint32_t> live; // the tables of both windows
    for (auto s : c->net.slots) live.push_back(s);
    for (auto s : c->dns.slots) live.push_back(s + PV_SLOTS);
    for (uint32_t s : live) {
        std::vector<TopRec> recs;
        int rc = read_topn(c, s, recs);
        if (rc) return rc;
        for (auto &r : recs) {
            uint16_t l = (uint16_t)std::min<size_t>(r.name.size(), 65535);
            size_t p = o.size();
            o.resize(p + 4 + 8 + 8 + 2 + l);
            memcpy(&o[p], &s, 4);
            memcpy(&o[p + 4], &r.key, 8);
            memcpy(&o[p + 12], &r.count, 8);
            memcpy(&o[p + 20], &l, 2);
            memcpy(&o[p + 22], r.name.data(), l);
        }
    }
    *bytes = o.size();
    *buf = (uint8_t *)malloc(o.size() ? o.size() : 1);
    if (!o.empty()) memcpy(*buf, o.data(), o.size());
    return 0;
}

int pv_merge_topn(pv_ctx *c, const uint8_t *buf, size_t bytes)
{
    mark_merged(c, "pv_merge_topn");
    size_t p = 0;
    while (p + 22 <= bytes) {
        uint32_t s; uint64_t key, cnt; uint16_t l;
        memcpy(&s, buf + p, 4); memcpy(&key, buf + p + 4, 8); memcpy(&cnt, buf + p + 12, 8); memcpy(&l, buf + p + 20, 2);
        if (p + 22 + l > bytes || s >= PV_TABLES) return c->fail(PV_EINVAL, "malformed top-N buffer");
        auto &e = c->remote_topn[s][key];
        e.first += cnt;
        e.second.assign((const char *)buf + p + 22, l);
        p += 22 + l;
    }
    return 0;
}

static int dns_event_seconds_batch(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                                   const uint32_t *sc_idx, const uint32_t *sc_sec, int64_t *secs, uint32_t max, uint32_t *n)
{
    *n = 0;
    const uint64_t nr = info->n_records;
    if (!nr) return 0;
    if (nr > c->max_records) return c->fail(PV_ECAPACITY, "batch exceeds max_records");
    uint32_t tseg[2];
    const bool filt = c->sample_rate < 100 && c->f_flags;
    if (filt && !c->d_fbits) {
        hipError_t e;
        const size_t fw = (size_t)(c->max_records / 64 + 2);
        if (!hip_ok(e = hipMalloc(&c->d_fbits, fw * 8)) || !hip_ok(e = hipHostMalloc((void **)&c->h_fbits, fw * 8, hipHostMallocDefault)))
            return c->hipfail(e, "deep sampling filter bits");
    }
    if (int rc = dns_prescan(c, d_recs, d_offs, nr, c->stream, true, tseg, filt)) return rc;
    if (int rc = tcp_stage(c, d_recs, d_offs, nr, tseg[0], tseg[1], (uint32_t)info->first_sec, true, c->stream)) return rc;
    if (c->sample_rate < 100) {
        // the DNS manager's draws in this batch: its unfiltered events (a sharded run steps
        // each rank's generator past the earlier shards' draws, pv_sample_skip)
        uint64_t d = 0;
        for (uint64_t t = 0; t < (nr + 63) / 64; t++) d += __builtin_popcountll(c->h_dbits[t] & ~(filt ? c->h_fbits[t] : 0ull));
        uint64_t dt = c->tcp_nmsg;
        if (filt && c->tcp_nmsg) {
            if (int rc = tcp_filter_bits(c, d_recs, d_offs, nr, c->stream)) return rc;
            for (uint64_t t = 0; t < ((uint64_t)c->tcp_nmsg + 63) / 64; t++) {
                uint64_t w = c->h_tfbits[t];
                if (t == (c->tcp_nmsg - 1) / 64 && (c->tcp_nmsg & 63)) w &= (1ull << (c->tcp_nmsg & 63)) - 1;
                dt -= __builtin_popcountll(w);
            }
        }
        c->plan_draws += d + dt;
    }
    // (ord, second) of every DNS event in stream order: a second's first UDP event, the messages
    std::vector<std::pair<uint64_t, int64_t>> ev;
    for (uint32_t j = 0; j < info->n_sec_changes; j++) {
        const uint64_t lo = sc_idx[j], hi = j + 1 < info->n_sec_changes ? sc_idx[j + 1] : nr;
        const uint64_t b = next_bit(c->h_dbits, lo, nr);
        if (b < hi) ev.push_back({b * 4, (int64_t)sc_sec[j]});
    }
    const size_t nu = ev.size();
    ev.insert(ev.end(), c->tcp_ords.begin(), c->tcp_ords.end());
    std::inplace_merge(ev.begin(), ev.begin() + nu, ev.end());
    c->tcp_ords.clear();
    c->tcp_nmsg = 0;
    uint32_t k = 0;
    for (auto &x : ev) {
        if (k && secs[k - 1] == x.second) continue;
        if (k >= max) return c->fail(PV_ECAPACITY, "more than %u DNS seconds", max);
        secs[k++] = x.second;
    }
    *n = k;
    return 0;
}

int pv_dns_event_seconds(pv_ctx *c, const uint8_t *d_recs, const uint32_t *d_offs, const pv_index_info *info,
                         const uint32_t *sc_idx, const uint32_t *sc_sec, int64_t *secs, uint32_t max, uint32_t *n)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    *n = 0;
    if (c->tcp_active) return c->fail(PV_EINVAL, "pv_dns_event_seconds after DNS-over-TCP state (call it before the first batch)");
    const int rc = dns_event_seconds_batch(c, d_recs, d_offs, info, sc_idx, sc_sec, secs, max, n);
    tcp_reset(c);
    return rc;
}

} // extern "C"

// Shard cuts of a capture for a sharded run: world contiguous record ranges of about equal
// size, each cut moved to the nearest record boundary that no DNS-over-TCP flow spans (every
// flow key seen before the cut has its last packet before it), so each shard's TCP stage
// starts from the empty state a single pass holds for those flows there. A capture with a
// flow across a whole shard moves the cut past it (shards grow, some may be empty).
int pv_shard_cuts(const uint8_t *recs, size_t bytes, const uint32_t *offs, uint64_t n, uint32_t linktype, uint32_t ts_nano,
                  uint32_t world, uint64_t *cuts)
{
    if (!world) return PV_EINVAL;
    PvParams P;
    memset(&P, 0, sizeof P);
    P.linktype = linktype;
    P.ts_nano = ts_nano;
    const pvname::HostRecs R{recs, bytes};
    std::vector<uint32_t> key(n);
    std::vector<uint8_t> tcp(n, 0);
    std::unordered_map<uint32_t, uint64_t> last;
    for (uint64_t i = 0; i < n; i++) {
        if (offs[i] + 16ull > bytes) return PV_EINVAL;
        if (pvname::tcp_dns_flow(R, P, offs[i], &key[i])) {
            tcp[i] = 1;
            last[key[i]] = i;
        }
    }
    // ok[c]: no flow has packets on both sides of record boundary c
    std::vector<uint8_t> ok(n + 1, 1);
    int64_t reach = -1;
    for (uint64_t i = 0; i < n; i++) {
        if (tcp[i]) reach = std::max<int64_t>(reach, (int64_t)last[key[i]]);
        ok[i + 1] = reach <= (int64_t)i;
    }
    const uint64_t per = (n + world - 1) / world;
    cuts[0] = 0;
    for (uint32_t r = 1; r < world; r++) {
        const uint64_t lo = cuts[r - 1], ideal = std::max(lo, std::min<uint64_t>(n, (uint64_t)r * per));
        uint64_t best = n;
        for (uint64_t d = 0;; d++) {
            const bool up = ideal + d <= n, down = ideal >= lo + d;
            if (!up && !down) break;
            if (up && ok[ideal + d]) { best = ideal + d; break; }
            if (down && ok[ideal - d]) { best = ideal - d; break; }
        }
        cuts[r] = best;
    }
    cuts[world] = n;
    return 0;
}

// the Net-pass kernel the context's last span launched (the symbol rocprofv3 reports)
const char *pv_net_kernel_name(pv_ctx *c)
{
    return c ? c->net_kernel : "none";
}

// Deep sampling over a sharded stream: each manager's generator stepped past the draws the
// earlier shards make (net_draws: their records, dns_draws: their unfiltered DNS events, as
// pv_dns_event_seconds_host counts them in pv_plan_dns_draws), so every rank draws what the
// single pass draws for its events (AbstractMetricsManager::new_event, :318-323); the DNS
// manager's flag is the last of those draws (a filtered event at the shard start counts it).
// Cost: O(net_draws + dns_draws) generator steps on the calling thread (jsf32 has no jump-ahead),
// about 1 ns each; a rank calls it once, before its first batch.
int pv_sample_skip(pv_ctx *c, uint64_t net_draws, uint64_t dns_draws)
{
    if (!c) return PV_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->records_seen) return c->fail(PV_EINVAL, "pv_sample_skip after the first batch");
    if (c->sample_rate >= 100) return 0;
    Jsf32 rn, rd;
    for (uint64_t k = 0; k < net_draws; k++) rn.next();
    for (uint64_t k = 1; k < dns_draws; k++) rd.next();
    if (dns_draws) c->dns_deep_now = rd.next() % 100u < c->sample_rate; // the manager's last flag
    c->draws_net.reset(rn);
    c->draws_dns.reset(rd);
    return 0;
}

int pv_plan_dns_draws(pv_ctx *c, uint64_t *draws)
{
    *draws = c->plan_draws;
    return 0;
}
