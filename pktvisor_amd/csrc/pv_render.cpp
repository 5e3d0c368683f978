// SPDX-License-Identifier: MPL-2.0
//
// pv_render.cpp — the output half of the host runtime behind include/pvgpu.h: a window's device
// buckets read into host buckets (HostBucket: counters, top-N lists with their names, CPC replay,
// exact quantiles) and rendered as the reference renders them: JSON (NetworkMetricsBucket::to_json
// net/v1 ...cpp:447-505, DnsMetricsBucket::to_json dns/v1 ...cpp:735-836, window_merged_json
// AbstractMetricsManager.h:601-647), Prometheus (window_single_prometheus :506-531) and
// OpenTelemetry (window_single_opentelemetry :533-575); external buckets for a policy's merge
// (StreamHandler::merge, src/StreamHandler.h:259-269).
#include "pv_host.h"

namespace pvh {

// Device-side top-N records of one table: (key, count, name)

int read_topn(pv_ctx *c, uint32_t s, std::vector<TopRec> &out) // s: table (PV_TSLOT)
{
    flush_fills(c);
    uint64_t tcap = 1ull << c->tcap_log2;
    std::vector<uint64_t> keys(tcap), cnt(tcap);
    std::vector<uint32_t> aux(tcap);
    uint64_t tops[PV_ARENA_PARTS];
    hipError_t e;
    if (!hip_ok(e = hipMemcpyAsync(keys.data(), c->d_tkeys + s * tcap, tcap * 8, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipMemcpyAsync(cnt.data(), c->d_tcnt + s * tcap, tcap * 8, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipMemcpyAsync(aux.data(), c->d_taux + s * tcap, tcap * 4, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipMemcpyAsync(tops, c->d_arena_top + (uint64_t)s * PV_ARENA_PARTS, sizeof tops, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "read top-N table");
    const uint64_t pcap = c->arena_cap / PV_ARENA_PARTS;
    std::vector<std::vector<uint8_t>> parts(PV_ARENA_PARTS);
    for (uint32_t p = 0; p < PV_ARENA_PARTS; p++) {
        uint64_t used = std::min<uint64_t>(tops[p], pcap);
        parts[p].resize(used);
        if (used && !hip_ok(e = hipMemcpy(parts[p].data(), c->d_arena + s * c->arena_cap + p * pcap, used, hipMemcpyDeviceToHost)))
            return c->hipfail(e, "read name arena");
    }
    const std::vector<uint64_t> &roff = c->roff[s];
    // after a multi-GPU exchange (before pv_topn_x_view), this rank's regions only
    uint64_t i0 = 0, i1 = tcap;
    if (c->x_ranks > 1) {
        const uint32_t nreg = 1u << c->reg_log2, rsl = c->tcap_log2 - c->reg_log2;
        i0 = (uint64_t)(((uint64_t)c->x_rank * nreg + c->x_ranks - 1) / c->x_ranks) << rsl;
        i1 = (uint64_t)(((uint64_t)(c->x_rank + 1) * nreg + c->x_ranks - 1) / c->x_ranks) << rsl;
    }
    for (uint64_t i = i0; i < i1; i++) {
        if (!keys[i]) continue;
        // a purged region's survivors report count + the thetas its purges subtracted (the
        // frequent-items estimate, exact for a key no purge dropped)
        const uint64_t off = roff.empty() ? 0 : roff[(i >> (c->tcap_log2 - c->reg_log2))];
        TopRec r{keys[i], cnt[i] + off, std::string()};
        uint32_t m = PV_KEY_METRIC(keys[i]);
        if (m == TM_IPV4) {
            uint32_t ip = (uint32_t)keys[i];
            char b[20];
            snprintf(b, sizeof b, "%u.%u.%u.%u", ip & 0xff, (ip >> 8) & 0xff, (ip >> 16) & 0xff, ip >> 24);
            r.name = b;
        } else if (aux[i] && (aux[i] - 1) % pcap + 2 <= parts[(aux[i] - 1) / pcap].size()) {
            const std::vector<uint8_t> &arena = parts[(aux[i] - 1) / pcap];
            const uint64_t top = arena.size();
            uint64_t p = (aux[i] - 1) % pcap;
            uint32_t len = arena[p] | (arena[p + 1] << 8);
            if (p + 2 + len <= top) {
                if (m == TM_IPV6) {
                    char b[64];
                    inet_ntop(AF_INET6, &arena[p + 2], b, sizeof b);
                    r.name = b;
                } else if (m == TM_ECS && len == 17) {
                    // ECS client subnet text (inet_ntop, DnsAdditionalRecord.h:86,95)
                    char b[64];
                    inet_ntop(arena[p + 2] == 1 ? AF_INET : AF_INET6, &arena[p + 3], b, sizeof b);
                    r.name = b;
                } else {
                    r.name.assign((const char *)&arena[p + 2], len);
                }
            }
        }
        out.push_back(std::move(r));
    }
    auto it = c->remote_topn.find(s);
    if (it != c->remote_topn.end())
        for (auto &kv : it->second) out.push_back(TopRec{kv.first, kv.second.first, kv.second.second});
    return 0;
}

// Host-side metric of a top-N entry: its key's metric, or for Net v2 keys a metric per
// direction (TMH_V2_IP4 + dir, TMH_V2_IP6 + dir)
enum { TMH_V2_IP4 = 32, TMH_V2_IP6 = 36, TMH_V2_DNS = 64 }; // DNS v2: 64 + 4 * metric + dir
uint32_t host_metric(const pv_ctx *c, uint64_t key)
{
    if (PV_IS_V2_IP4(key)) return TMH_V2_IP4 + (uint32_t)((key >> 34) & 3);
    if (PV_IS_V2_IP6(key)) return TMH_V2_IP6 + (uint32_t)((key >> 53) & 3);
    // (v1 name keys carry a full 56-bit fingerprint: only a DNS v2 context holds v2 name keys)
    if (c->dns2_groups && PV_IS_V2_DKEY(key)) return TMH_V2_DNS + 4 * PV_KEY_METRIC(key) + (uint32_t)((key >> 53) & 3);
    return PV_KEY_METRIC(key);
}

// A finalised bucket (possibly the merge of several slots) on the host.
struct HostBucket {
    int64_t start_sec = 0;
    uint64_t period_length = 0;
    std::vector<uint64_t> sum;                           // PV_SUM_WORDS
    std::vector<int64_t> cpc;                            // PV_MIN_WORDS (min-merged)
    std::map<uint32_t, std::map<std::string, uint64_t>> tops; // metric -> name -> count
    std::vector<uint64_t> from_us, to_us;
    std::vector<double> ratio;
    std::vector<uint64_t> time2[3]; // DNS v2 per direction
    std::vector<double> ratio2[3];
    bool merged = false;
    // an exported bucket (pv_bucket) after an Aggregate::SUM merge: Quantile::_quantiles_sum
    // (src/Metrics.h:338-372), which the output prefers to the sketch's own quantiles, and the
    // Histogram values, which keep merging while the quantile sketches do not
    std::vector<uint64_t> qs_payload, qs_from, qs_to;
    std::vector<double> qs_ratio;
    bool hist_sep = false;
    std::vector<uint64_t> hfrom_us, hto_us;
    int64_t start_nsec = 0, end_sec = 0, end_nsec = 0;
    const std::vector<uint64_t> &hist_from() const { return hist_sep ? hfrom_us : from_us; }
    const std::vector<uint64_t> &hist_to() const { return hist_sep ? hto_us : to_us; }
    // the same for the v2 handlers, per direction: payload sizes (Net v2), transaction times and
    // size ratios (DNS v2) after a SUM merge, and the xact time histograms that keep merging
    std::vector<uint64_t> qs_payload2[3], qs_time2[3];
    std::vector<double> qs_ratio2[3];
    bool hist2_sep = false;
    std::vector<uint64_t> htime2[3];
    const std::vector<uint64_t> &hist_time2(uint32_t x) const { return hist2_sep ? htime2[x] : time2[x]; }
};

template <typename T>
std::vector<T> quantiles(std::vector<T> v)
{
    std::sort(v.begin(), v.end());
    std::vector<T> out;
    for (double r : {0.50, 0.90, 0.95, 0.99}) {
        uint64_t w = (uint64_t)std::ceil(r * (double)v.size());
        size_t idx = w == 0 ? 0 : (size_t)(w - 1);
        if (idx >= v.size()) idx = v.size() - 1;
        out.push_back(v[idx]);
    }
    return out;
}

// exact quantiles of the payload-size histogram with the KLL inclusive rank rule
std::vector<uint64_t> hist_quantiles(const uint64_t *h, size_t bins, uint64_t &n)
{
    n = 0;
    for (size_t i = 0; i < bins; i++) n += h[i];
    std::vector<uint64_t> out;
    if (!n) return out;
    for (double r : {0.50, 0.90, 0.95, 0.99}) {
        uint64_t w = (uint64_t)std::ceil(r * (double)n);
        if (w == 0) w = 1;
        uint64_t acc = 0;
        size_t i = 0;
        for (; i < bins; i++) { acc += h[i]; if (acc >= w) break; }
        out.push_back(std::min(i, bins - 1));
    }
    return out;
}

double cpc_estimate(const int64_t *t, bool merged)
{
    if (merged) {
        uint32_t c = 0;
        for (uint32_t i = 0; i < PV_CPC_COUPONS; i++) c += t[i] != PV_CPC_EMPTY;
        return icon11(c);
    }
    std::vector<std::pair<int64_t, uint32_t>> f;
    for (uint32_t i = 0; i < PV_CPC_COUPONS; i++)
        if (t[i] != PV_CPC_EMPTY) f.push_back({t[i], i});
    return cpc_hip(f);
}

// One handler's bucket over `slots` (merged: window_merged_json's fold, AbstractMetricsManager.h:601-647)
// The merged view's values of a set of DNS slots (pv_values_x_select; mask: bit per slot): per kind a stand-in list of the
// group's count whose histogram-point counts and maximum are the merged ones (each value at the
// point that bounds it, the largest replaced by the maximum), its quantiles set as overrides.
void x_values_standin(pv_ctx *c, uint32_t mask, HostBucket &b)
{
    const std::vector<uint64_t> &pts = hist_points();
    for (auto &kv : c->xq) {
        if (kv.first.first != mask) continue;
        const uint32_t kind = kv.first.second;
        const XQuant &x = kv.second;
        std::vector<uint64_t> v;
        v.reserve(x.n);
        if (!x.cdf.empty()) {
            uint64_t prev = 0;
            for (size_t k = 0; k < pts.size(); k++) {
                for (uint64_t i = prev; i < x.cdf[k]; i++) v.push_back(pts[k]);
                prev = std::max(prev, x.cdf[k]);
            }
        }
        while (v.size() < x.n) v.push_back(x.max);
        if (!v.empty()) v.back() = x.max;
        auto dbl = [](const std::vector<uint64_t> &u) {
            std::vector<double> d(u.size());
            for (size_t i = 0; i < u.size(); i++) memcpy(&d[i], &u[i], 8);
            return d;
        };
        if (kind == XV_FROM_US) { b.from_us.insert(b.from_us.end(), v.begin(), v.end()); b.qs_from = x.q; }
        else if (kind == XV_TO_US) { b.to_us.insert(b.to_us.end(), v.begin(), v.end()); b.qs_to = x.q; }
        else if (kind == XV_RATIO) { auto d = dbl(v); b.ratio.insert(b.ratio.end(), d.begin(), d.end()); b.qs_ratio = dbl(x.q); }
        else if (kind >= XV2_TIME && kind < XV2_TIME + 3) { auto &t = b.time2[kind - XV2_TIME]; t.insert(t.end(), v.begin(), v.end()); b.qs_time2[kind - XV2_TIME] = x.q; }
        else if (kind >= XV2_RATIO && kind < XV2_RATIO + 3) {
            auto d = dbl(v);
            auto &t = b.ratio2[kind - XV2_RATIO];
            t.insert(t.end(), d.begin(), d.end());
            b.qs_ratio2[kind - XV2_RATIO] = dbl(x.q);
        }
    }
}

int load_bucket(pv_ctx *c, const std::vector<uint32_t> &slots, bool merged, int part, HostBucket &b)
{
    flush_fills(c);
    const Window &win = part == PART_NET ? c->net : c->dns;
    b.sum.assign(PV_SUM_WORDS, 0);
    b.cpc.assign(PV_MIN_WORDS, PV_CPC_EMPTY);
    b.merged = merged;
    // this handler's part of the slot's SUM and MIN words
    const size_t s0 = part == PART_NET ? 0 : PV_OFF_DNS, s1 = part == PART_NET ? PV_SUM_NET_WORDS : PV_SUM_WORDS;
    const size_t m0 = part == PART_NET ? 0 : PV_MIN_NET_WORDS, m1 = part == PART_NET ? PV_MIN_NET_WORDS : PV_MIN_WORDS;
    std::vector<uint64_t> sum(PV_SUM_WORDS);
    std::vector<int64_t> cpc(PV_MIN_WORDS);
    bool first = true;
    for (uint32_t s : slots) {
        hipError_t e;
        if (!hip_ok(e = hipMemcpyAsync(sum.data() + s0, c->d_sum + (uint64_t)s * PV_SUM_WORDS + s0, (s1 - s0) * 8,
                                       hipMemcpyDeviceToHost, c->stream)) ||
            !hip_ok(e = hipMemcpyAsync(cpc.data() + m0, c->d_cpc + (uint64_t)s * PV_MIN_WORDS + m0, (m1 - m0) * 8,
                                       hipMemcpyDeviceToHost, c->stream)) ||
            !hip_ok(e = hipStreamSynchronize(c->stream)))
            return c->hipfail(e, "read bucket");
        for (size_t i = s0; i < s1; i++) b.sum[i] += sum[i];
        // CPC union: a coupon is present if present in any bucket; for a single
        // bucket the first-occurrence order is kept for the HIP replay
        for (size_t i = m0; i < m1; i++) b.cpc[i] = std::min(b.cpc[i], cpc[i]);
        const SlotMeta &m = win.meta[s];
        b.period_length += m.read_only ? m.period_length : 0;
        if (first || m.start_sec < b.start_sec) { b.start_sec = m.start_sec; b.start_nsec = m.start_nsec; }
        if (m.end_sec > b.end_sec) { b.end_sec = m.end_sec; b.end_nsec = m.end_nsec; }
        first = false;
        if (!(c->x_ranks > 1 && c->x_view_on)) {
            std::vector<TopRec> recs;
            int rc = read_topn(c, s + (part == PART_DNS ? PV_SLOTS : 0), recs);
            if (rc) return rc;
            for (auto &r : recs) b.tops[host_metric(c, r.key)][r.name] += r.count;
        }
        if (part != PART_DNS) continue;
        const uint32_t sg = s | (c->gen[s] << 8);
        if (c->xq_on) continue; // (the merged view's values: after the loop, for the slot set)
        for (auto &v : c->xvals_host) {
            if (v.slot != sg) continue;
            if (v.kind == XV_FROM_US) b.from_us.push_back(v.bits);
            else if (v.kind == XV_TO_US) b.to_us.push_back(v.bits);
            else if (v.kind == XV_RATIO) { double d; memcpy(&d, &v.bits, 8); b.ratio.push_back(d); }
            else if (v.kind >= XV2_TIME && v.kind < XV2_TIME + 3) b.time2[v.kind - XV2_TIME].push_back(v.bits);
            else if (v.kind >= XV2_RATIO && v.kind < XV2_RATIO + 3) {
                double d;
                memcpy(&d, &v.bits, 8);
                b.ratio2[v.kind - XV2_RATIO].push_back(d);
            }
        }
    }
    uint32_t mask = 0;
    for (uint32_t sl : slots) mask |= 1u << sl;
    if (c->x_ranks > 1 && c->x_view_on) {
        // a multi-GPU merged view (pv_topn_x_view): every owner's leading entries of this slot set
        auto it = c->x_view.find(((uint32_t)part << 16) | mask);
        if (it != c->x_view.end())
            for (auto &kv : it->second) b.tops[host_metric(c, kv.first)][kv.second.second] += kv.second.first;
    }
    if (part == PART_DNS && c->xq_on) x_values_standin(c, mask, b);
    return 0;
}

// TopN::to_json (src/Metrics.h:577-590): the first topn_count items by estimate, cut at the
// first one below the topn_percentile_threshold quantile of those estimates (_get_threshold,
// :510-521, the KLL inclusive rank rule on them)
void top_json(Json &j, const char *key, const std::vector<std::pair<std::string, uint64_t>> &v0, size_t n, uint32_t pct)
{
    auto v = v0;
    std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) {
        if (a.second != b.second) return a.second > b.second;
        return a.first < b.first;
    });
    const size_t k = std::min(n, v.size());
    uint64_t thr = 0;
    if (k) {
        std::vector<uint64_t> est;
        for (size_t i = 0; i < k; i++) est.push_back(v[i].second);
        std::sort(est.begin(), est.end());
        const uint64_t w = (uint64_t)std::ceil((double)pct / 100.0 * (double)k);
        thr = est[w == 0 ? 0 : std::min<size_t>(w - 1, k - 1)];
    }
    j.key(key);
    j.arr();
    for (size_t i = 0; i < k && v[i].second >= thr; i++) {
        j.obj();
        j.key("name").str(v[i].first);
        j.key("estimate").u(v[i].second);
        j.end_obj();
    }
    j.end_arr();
}
std::vector<std::pair<std::string, uint64_t>> tops_of(const HostBucket &b, uint32_t metric)
{
    std::vector<std::pair<std::string, uint64_t>> v;
    auto it = b.tops.find(metric);
    if (it != b.tops.end())
        for (auto &kv : it->second) v.push_back(kv);
    return v;
}
std::vector<std::pair<std::string, uint64_t>> dense_tops(const uint64_t *t, size_t bins, int kind)
{
    std::vector<std::pair<std::string, uint64_t>> v;
    for (size_t i = 0; i < bins; i++) {
        if (!t[i]) continue;
        std::string name;
        if (kind == 0) name = std::to_string(i);
        else {
            auto &m = kind == 1 ? qtype_names() : rcode_names();
            auto it = m.find((uint16_t)i);
            name = it != m.end() ? it->second : std::to_string(i);
        }
        v.push_back({name, t[i]});
    }
    return v;
}

// Histogram::to_json (src/Metrics.h:193-262) over exact values: split points are the distinct
// uint64 values of 10^(b/18) * 10^e, e in [-9, 18), b in [0, 18); a point is listed when the
// inclusive PMF interval that ends at it holds a value, with the inclusive CDF times n (a
// double, as KLL's normalized rank times get_n()); "+Inf" closes with n
const std::vector<uint64_t> &hist_points()
{
    static const std::vector<uint64_t> pts = [] {
        std::vector<uint64_t> p;
        for (int e = -9; e < 18; e++)
            for (int k = 0; k < 18; k++) {
                const uint64_t x = static_cast<uint64_t>(std::pow(10.0, static_cast<float>(k) / 18) * std::pow(10.0, e));
                if (p.empty() || p.back() != x) p.push_back(x);
            }
        return p;
    }();
    return pts;
}
void hist_json(Json &j, const char *key, std::vector<uint64_t> v)
{
    if (v.empty()) return;
    const std::vector<uint64_t> &pts = hist_points();
    std::sort(v.begin(), v.end());
    const double n = (double)v.size();
    j.key(key).obj();
    j.key("buckets").obj();
    uint64_t prev = 0;
    for (uint64_t x : pts) {
        const uint64_t c = (uint64_t)(std::upper_bound(v.begin(), v.end(), x) - v.begin());
        if (c != prev) j.key(std::to_string(x)).d(((double)c / n) * n);
        prev = c;
    }
    j.key("+Inf").d(1.0 * n);
    j.end_obj();
    j.end_obj();
}

template <typename T>
void quant_json(Json &j, const char *key, const std::vector<T> &v, const std::vector<T> *qsum = nullptr)
{
    if (v.empty()) return;
    auto q = qsum && !qsum->empty() ? *qsum : quantiles(v);
    const char *names[4] = {"p50", "p90", "p95", "p99"};
    j.key(key);
    j.obj();
    for (int i = 0; i < 4; i++) {
        j.key(names[i]);
        if constexpr (std::is_floating_point<T>::value) j.d(q[i]);
        else j.u((uint64_t)q[i]);
    }
    j.end_obj();
}

void net_json(pv_ctx *c, Json &j, const HostBucket &b)
{
    const uint64_t *n = &b.sum[PV_OFF_NET];
    size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    j.key("period").obj();
    j.key("start_ts").i(b.start_sec);
    j.key("length").u(b.period_length);
    j.end_obj();
    j.key("events").u(n[NC_EVENTS]);
    j.key("deep_samples").u(n[NC_SAMPLES]);
    if (c->net_groups & PV_NET_COUNTERS) {
        j.key("udp").u(n[NC_UDP]);
        j.key("tcp").u(n[NC_TCP]);
        j.key("protocol").obj(); j.key("tcp").obj(); j.key("syn").u(n[NC_SYN]); j.end_obj(); j.end_obj();
        j.key("other_l4").u(n[NC_OTHER]);
        j.key("ipv4").u(n[NC_V4]);
        j.key("ipv6").u(n[NC_V6]);
        j.key("in").u(n[NC_IN]);
        j.key("out").u(n[NC_OUT]);
        j.key("unknown_dir").u(n[NC_UNK]);
        j.key("total").u(n[NC_TOTAL]);
        j.key("filtered").u(n[NC_FILTERED]);
    }
    if (c->net_groups & PV_NET_CARDINALITY) {
        j.key("cardinality").obj();
        j.key("src_ips_in").i(lround(cpc_estimate(&b.cpc[CPC_SRC * PV_CPC_COUPONS], b.merged)));
        j.key("dst_ips_out").i(lround(cpc_estimate(&b.cpc[CPC_DST * PV_CPC_COUPONS], b.merged)));
        j.end_obj();
    }
    if (c->net_groups & PV_NET_TOP_IPS) {
        top_json(j, "top_ipv4", tops_of(b, TM_IPV4), topn, pct);
        top_json(j, "top_ipv6", tops_of(b, TM_IPV6), topn, pct);
    }
    if (c->net_groups & PV_NET_TOP_GEO) {
        j.key("top_geoLoc").arr(); j.end_arr();
        j.key("top_ASN").arr(); j.end_arr();
    }
    uint64_t cnt;
    auto q = hist_quantiles(&b.sum[PV_OFF_PAYLOAD], PV_PAYLOAD_BINS, cnt);
    if (!b.qs_payload.empty()) q = b.qs_payload;
    if (cnt) {
        j.key("payload_size").obj();
        j.key("p50").u(q[0]); j.key("p90").u(q[1]); j.key("p95").u(q[2]); j.key("p99").u(q[3]);
        j.end_obj();
    }
}

// NetworkMetricsBucket::to_json, Net v2 (src/handlers/net/v2/NetStreamHandler.cpp:436-484):
// base event counts, `filtered_packets`, then one object per direction the bucket has seen
// (the reference creates a direction's entry on its first packet)
void net2_json(pv_ctx *c, Json &j, const HostBucket &b)
{
    const uint64_t *n = &b.sum[PV_OFF_NET2];
    const uint32_t g = c->net2_groups;
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    j.key("period").obj();
    j.key("start_ts").i(b.start_sec);
    j.key("length").u(b.period_length);
    j.end_obj();
    j.key("observed_packets").u(n[N2_EVENTS]);
    j.key("deep_sampled_packets").u(n[N2_SAMPLES]);
    if (g & PV_N2G_COUNTERS) j.key("filtered_packets").u(n[N2_FILTERED]);
    static const char *dirs[3] = {"in", "out", "unknown"};
    for (uint32_t d = 0; d < 3; d++) {
        const uint64_t *dc = n + N2_DIR + 8 * d;
        if (!dc[N2_TOTAL]) continue;
        j.key(dirs[d]).obj();
        if (g & PV_N2G_COUNTERS) {
            j.key("udp_packets").u(dc[N2_UDP]);
            j.key("tcp_packets").u(dc[N2_TCP]);
            j.key("other_l4_packets").u(dc[N2_OTHER]);
            j.key("ipv4_packets").u(dc[N2_V4]);
            j.key("ipv6_packets").u(dc[N2_V6]);
            j.key("tcp").obj(); j.key("syn_packets").u(dc[N2_SYN]); j.end_obj();
            j.key("total_packets").u(dc[N2_TOTAL]);
        }
        if (g & PV_N2G_CARDINALITY) {
            j.key("cardinality").obj();
            j.key("ips").i(lround(cpc_estimate(&b.cpc[(CPC_V2 + d) * PV_CPC_COUPONS], b.merged)));
            j.end_obj();
        }
        if (g & PV_N2G_TOP_IPS) {
            top_json(j, "top_ipv4_packets", tops_of(b, TMH_V2_IP4 + d), topn, pct);
            top_json(j, "top_ipv6_packets", tops_of(b, TMH_V2_IP6 + d), topn, pct);
        }
        if (g & PV_N2G_TOP_GEO) {
            j.key("top_geo_loc_packets").arr(); j.end_arr();
            j.key("top_asn_packets").arr(); j.end_arr();
        }
        if (g & PV_N2G_QUANTILES) {
            uint64_t cnt;
            auto q = hist_quantiles(&b.sum[PV_OFF_PAYLOAD2 + d * PV_PAYLOAD_BINS], PV_PAYLOAD_BINS, cnt);
            if (cnt && !b.qs_payload2[d].empty()) q = b.qs_payload2[d];
            if (cnt) {
                j.key("payload_size_bytes").obj();
                j.key("p50").u(q[0]); j.key("p90").u(q[1]); j.key("p95").u(q[2]); j.key("p99").u(q[3]);
                j.end_obj();
            }
        }
        j.end_obj();
    }
}

// DnsMetricsBucket::to_json, DNS v2 (src/handlers/dns/v2/DnsStreamHandler.cpp:678-757): base
// event counts (the DNS pass's event counters), `filtered_packets`, then per transaction
// direction the bucket has set up: counters, qname cardinality and the top / quantile groups
void dns2_json(pv_ctx *c, Json &j, const HostBucket &b)
{
    const uint64_t *d = &b.sum[PV_OFF_DNS];
    const uint32_t g = c->dns2_groups;
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    j.key("period").obj();
    j.key("start_ts").i(b.start_sec);
    j.key("length").u(b.period_length);
    j.end_obj();
    j.key("observed_packets").u(d[DC_EVENTS]);
    j.key("deep_sampled_packets").u(d[DC_SAMPLES]);
    if (g & PV_DNS2_COUNTERS) j.key("filtered_packets").u(d[DC_FILTERED]);
    static const char *dirs[3] = {"in", "out", "unknown"};
    for (uint32_t x = 0; x < 3; x++) {
        const uint64_t *c2 = &b.sum[PV_OFF_DNS2 + x * PV_DNS2_CTRS];
        if (!c2[D2_SEEN]) continue;
        auto tops = [&](uint32_t metric) { return tops_of(b, TMH_V2_DNS + 4 * metric + x); };
        j.key(dirs[x]).obj();
        if (g & PV_DNS2_COUNTERS) {
            const std::pair<const char *, uint64_t> ctr[] = {
                {"xacts", c2[D2_XACTS]}, {"udp_xacts", c2[D2_UDP]}, {"tcp_xacts", c2[D2_TCP]}, {"dot_xacts", c2[D2_DOT]},
                {"doh_xacts", c2[D2_DOH]}, {"dnscrypt_udp_xacts", c2[D2_CRYPT_UDP]}, {"dnscrypt_tcp_xacts", c2[D2_CRYPT_TCP]},
                {"doq_xacts", c2[D2_DOQ]},
                {"ipv4_xacts", c2[D2_V4]}, {"ipv6_xacts", c2[D2_V6]}, {"nxdomain_xacts", c2[D2_NX]}, {"ecs_xacts", c2[D2_ECS]},
                {"refused_xacts", c2[D2_REFUSED]}, {"srvfail_xacts", c2[D2_SRVFAIL]}, {"noerror_xacts", c2[D2_NOERROR]},
                {"nodata_xacts", c2[D2_NODATA]}, {"authenticated_data_xacts", c2[D2_AD]},
                {"authoritative_answer_xacts", c2[D2_AA]}, {"checking_disabled_xacts", c2[D2_CD]},
                {"timeout_queries", c2[D2_TIMEOUT]}, {"orphan_responses", c2[D2_ORPHAN]}};
            for (auto &kv : ctr) j.key(kv.first).u(kv.second);
        }
        if (g & PV_DNS2_CARDINALITY) {
            j.key("cardinality").obj();
            j.key("qname").i(lround(cpc_estimate(&b.cpc[(CPC_QNAME2 + x) * PV_CPC_COUPONS], b.merged)));
            j.end_obj();
        }
        if (g & PV_DNS2_TOP_PORTS)
            top_json(j, "top_udp_ports_xacts", dense_tops(&b.sum[PV_OFF_PORT2 + x * PV_PORT_BINS], PV_PORT_BINS, 0), topn, pct);
        if (g & PV_DNS2_TOP_ECS) {
            // geo / ASN of the subnet need a MaxMind database; none is enabled (HandlerModulePlugin::city/asn)
            j.key("top_geo_loc_ecs_xacts").arr(); j.end_arr();
            j.key("top_asn_ecs_xacts").arr(); j.end_arr();
            top_json(j, "top_ecs_xacts", tops(TM_ECS), topn, pct);
        }
        if (g & PV_DNS2_TOP_RCODES) {
            top_json(j, "top_nxdomain_xacts", tops(TM_NX), topn, pct);
            top_json(j, "top_refused_xacts", tops(TM_REFUSED), topn, pct);
            top_json(j, "top_srvfail_xacts", tops(TM_SRVFAIL), topn, pct);
            top_json(j, "top_nodata_xacts", tops(TM_NODATA), topn, pct);
            top_json(j, "top_noerror_xacts", tops(TM_NOERROR), topn, pct);
            top_json(j, "top_rcode_xacts", dense_tops(&b.sum[PV_OFF_RCODE2 + x * PV_RCODE_BINS], PV_RCODE_BINS, 2), topn, pct);
        }
        if (g & PV_DNS2_TOP_QNAMES) {
            top_json(j, "top_qname2_xacts", tops(TM_QNAME2), topn, pct);
            top_json(j, "top_qname3_xacts", tops(TM_QNAME3), topn, pct);
        }
        if (g & PV_DNS2_TOP_SIZE) {
            top_json(j, "top_response_bytes", tops(TM_SIZED), topn, pct);
            quant_json(j, "response_query_size_ratio", b.ratio2[x], &b.qs_ratio2[x]);
        }
        if (g & PV_DNS2_TOP_QTYPES)
            top_json(j, "top_qtype_xacts", dense_tops(&b.sum[PV_OFF_QTYPE2 + x * PV_QTYPE_BINS], PV_QTYPE_BINS, 1), topn, pct);
        if (g & PV_DNS2_XACT_TIMES) {
            quant_json(j, "xact_time_us", b.time2[x], &b.qs_time2[x]);
            hist_json(j, "xact_histogram_us", b.hist_time2(x));
            top_json(j, "top_slow_xacts", tops(TM_SLOW_OUT), topn, pct);
        }
        j.end_obj();
    }
}

void dns_json(pv_ctx *c, Json &j, const HostBucket &b)
{
    const uint64_t *d = &b.sum[PV_OFF_DNS];
    size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    uint32_t g = c->dns_groups;
    j.key("period").obj();
    j.key("start_ts").i(b.start_sec);
    j.key("length").u(b.period_length);
    j.end_obj();
    j.key("wire_packets").obj();
    j.key("events").u(d[DC_EVENTS]);
    j.key("deep_samples").u(d[DC_SAMPLES]);
    if (g & PV_DNS_COUNTERS) {
        j.key("queries").u(d[DC_QUERIES]);
        j.key("replies").u(d[DC_REPLIES]);
        j.key("tcp").u(d[DC_TCP]);
        j.key("udp").u(d[DC_UDP]);
        j.key("ipv4").u(d[DC_V4]);
        j.key("ipv6").u(d[DC_V6]);
        j.key("nxdomain").u(d[DC_NX]);
        j.key("refused").u(d[DC_REFUSED]);
        j.key("srvfail").u(d[DC_SRVFAIL]);
        j.key("noerror").u(d[DC_NOERROR]);
        j.key("nodata").u(d[DC_NODATA]);
        j.key("total").u(d[DC_TOTAL]);
        j.key("filtered").u(d[DC_FILTERED]);
        if (g & PV_DNS_TOP_ECS) j.key("query_ecs").u(d[DC_QECS]);
    }
    j.end_obj();
    if (g & PV_DNS_CARDINALITY) {
        j.key("cardinality").obj();
        j.key("qname").i(lround(cpc_estimate(&b.cpc[CPC_QNAME * PV_CPC_COUPONS], b.merged)));
        j.end_obj();
    }
    if (g & PV_DNS_TRANSACTIONS) {
        j.key("xact").obj();
        j.key("counts").obj(); j.key("total").u(d[DC_XTOTAL]); j.key("timed_out").u(d[DC_XTIMEOUT]); j.end_obj();
        j.key("in").obj();
        j.key("total").u(d[DC_XIN]);
        top_json(j, "top_slow", tops_of(b, TM_SLOW_IN), topn, pct);
        if (g & PV_DNS_QUANTILES) quant_json(j, "quantiles_us", b.to_us, &b.qs_to);
        if (g & PV_DNS_HISTOGRAMS) hist_json(j, "histogram_us", b.hist_to());
        j.end_obj();
        j.key("out").obj();
        j.key("total").u(d[DC_XOUT]);
        top_json(j, "top_slow", tops_of(b, TM_SLOW_OUT), topn, pct);
        if (g & PV_DNS_QUANTILES) quant_json(j, "quantiles_us", b.from_us, &b.qs_from);
        if (g & PV_DNS_HISTOGRAMS) hist_json(j, "histogram_us", b.hist_from());
        j.end_obj();
        if ((g & PV_DNS_QUANTILES) && !b.ratio.empty()) { j.key("ratio").obj(); quant_json(j, "quantiles", b.ratio, &b.qs_ratio); j.end_obj(); }
        j.end_obj();
    }
    if (g & PV_DNS_TOP_PORTS) top_json(j, "top_udp_ports", dense_tops(&b.sum[PV_OFF_PORT], PV_PORT_BINS, 0), topn, pct);
    if (g & PV_DNS_TOP_ECS) {
        // geo / ASN of the subnet need a MaxMind database; none is enabled (HandlerModulePlugin::city/asn)
        j.key("top_geoLoc_ecs").arr(); j.end_arr();
        j.key("top_asn_ecs").arr(); j.end_arr();
        top_json(j, "top_query_ecs", tops_of(b, TM_ECS), topn, pct);
    }
    if (g & PV_DNS_TOP_QNAMES) {
        top_json(j, "top_qname2", tops_of(b, TM_QNAME2), topn, pct);
        top_json(j, "top_qname3", tops_of(b, TM_QNAME3), topn, pct);
        top_json(j, "top_nxdomain", tops_of(b, TM_NX), topn, pct);
        top_json(j, "top_refused", tops_of(b, TM_REFUSED), topn, pct);
        top_json(j, "top_srvfail", tops_of(b, TM_SRVFAIL), topn, pct);
        top_json(j, "top_nodata", tops_of(b, TM_NODATA), topn, pct);
        if (g & PV_DNS_TOP_QNAMES_DETAILS) {
            top_json(j, "top_qname_by_resp_bytes", tops_of(b, TM_SIZED), topn, pct);
            top_json(j, "top_noerror", tops_of(b, TM_NOERROR), topn, pct);
        }
    }
    top_json(j, "top_rcode", dense_tops(&b.sum[PV_OFF_RCODE], PV_RCODE_BINS, 2), topn, pct);
    top_json(j, "top_qtype", dense_tops(&b.sum[PV_OFF_QTYPE], PV_QTYPE_BINS, 1), topn, pct);
}

// ---- Prometheus exposition (window_single_prometheus, src/AbstractMetricsManager.h:506-531)
// Metric text as the reference's primitives write it (src/Metrics.cpp:15-20,75-80,120-155;
// src/Metrics.h:264-289,416-448,614-691): "# HELP <schema>_<names> <desc>", "# TYPE ...", then
// samples named <schema>_<names>[_suffix]{static labels, then the added labels, each set in key
// order}. Numbers go through an ostream, as the reference's do (doubles with precision 6).
// Rates are timer-driven and not kept by this handler: an empty Rate writes nothing.
using PromLabels = std::map<std::string, std::string>;
std::mutex g_static_mu;
PromLabels g_static_labels; // Metric::_static_labels (Metric::add_static_label)

struct Prom {
    std::ostringstream o;
    PromLabels add;
    std::string lbl(const PromLabels &a) const
    {
        std::string t = "{";
        {
            std::lock_guard<std::mutex> g(g_static_mu);
            for (auto &kv : g_static_labels) t += kv.first + "=\"" + kv.second + "\",";
        }
        for (auto &kv : a) t += kv.first + "=\"" + kv.second + "\",";
        if (t.back() == ',') t.pop_back();
        return t + "}";
    }
    void head(const std::string &name, const char *desc, const char *type)
    {
        o << "# HELP " << name << ' ' << desc << '\n' << "# TYPE " << name << ' ' << type << '\n';
    }
    template <typename V>
    void gauge(const std::string &name, const char *desc, V v)
    {
        head(name, desc, "gauge");
        o << name << lbl(add) << ' ' << v << '\n';
    }
    // Quantile::to_prometheus: p50..p99, _sum = the sketch's max item, _count = n
    template <typename T>
    void summary(const std::string &name, const char *desc, const std::vector<T> &q, T max_item, uint64_t n)
    {
        if (q.empty()) return;
        head(name, desc, "summary");
        static const char *qs[4] = {"0.5", "0.9", "0.95", "0.99"};
        for (int i = 0; i < 4; i++) {
            PromLabels l(add);
            l["quantile"] = qs[i];
            o << name << lbl(l) << ' ' << q[i] << '\n';
        }
        o << name << "_sum" << lbl(add) << ' ' << max_item << '\n';
        o << name << "_count" << lbl(add) << ' ' << n << '\n';
    }
    // TopN::to_prometheus: the to_json selection, one sample per item labelled item_key=name
    void topn(const std::string &name, const char *item_key, const char *desc,
              const std::vector<std::pair<std::string, uint64_t>> &v0, size_t n, uint32_t pct)
    {
        auto v = v0;
        std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) {
            if (a.second != b.second) return a.second > b.second;
            return a.first < b.first;
        });
        const size_t k = std::min(n, v.size());
        if (!k) return;
        std::vector<uint64_t> est;
        for (size_t i = 0; i < k; i++) est.push_back(v[i].second);
        std::sort(est.begin(), est.end());
        const uint64_t w = (uint64_t)std::ceil((double)pct / 100.0 * (double)k);
        const uint64_t thr = est[w == 0 ? 0 : std::min<size_t>(w - 1, k - 1)];
        head(name, desc, "gauge");
        PromLabels l(add);
        for (size_t i = 0; i < k && v[i].second >= thr; i++) {
            l[item_key] = v[i].first;
            o << name << lbl(l) << ' ' << v[i].second << '\n';
        }
    }
    // Histogram::to_prometheus over exact values (the split points of hist_json)
    void histogram(const std::string &name, const char *desc, std::vector<uint64_t> v)
    {
        if (v.empty()) return;
        std::sort(v.begin(), v.end());
        head(name, desc, "histogram");
        const double n = (double)v.size();
        uint64_t prev = 0;
        for (uint64_t x : hist_points()) {
            const uint64_t c = (uint64_t)(std::upper_bound(v.begin(), v.end(), x) - v.begin());
            if (c != prev) {
                PromLabels l(add);
                l["le"] = std::to_string(x);
                o << name << "_bucket" << lbl(l) << ' ' << ((double)c / n) * n << '\n';
            }
            prev = c;
        }
        PromLabels l(add);
        l["le"] = "+Inf";
        o << name << "_bucket" << lbl(l) << ' ' << 1.0 * n << '\n';
        o << name << "_count" << lbl(add) << ' ' << v.size() << '\n';
    }
};

// ---- OpenTelemetry (window_single_opentelemetry, src/AbstractMetricsManager.h:533-575): the
// metrics the reference's primitives add to a ScopeMetrics (src/Metrics.cpp:22-36,82-96;
// src/Metrics.h:289-327,450-481,523-533,693-769), as protobuf wire bytes of the ScopeMetrics
// fields they fill (repeated `metrics`, field 2), serialized as protobuf does: fields in
// number order, proto3 defaults omitted, oneof members always written, packed repeated
// scalars. Messages of opentelemetry-proto metrics/v1 (the reference links
// opentelemetry-cpp 1.17.0's opentelemetry_proto; not vendored, field numbers restated):
// Metric{name 1, description 2, gauge 5, histogram 9, summary 11}; Gauge/Summary/Histogram
// {data_points 1; Histogram.aggregation_temporality 2}; NumberDataPoint{start 2, time 3,
// as_int 6, attributes 7}; SummaryDataPoint{start 2, time 3, quantile_values 6, attributes 7};
// ValueAtQuantile{quantile 1, value 2}; HistogramDataPoint{start 2, time 3, count 4,
// bucket_counts 6, explicit_bounds 7, attributes 9}; KeyValue{key 1, value 2};
// AnyValue{string_value 1}. Attributes are the added labels only (no static labels).
struct Pb {
    std::string s;
    void varint(uint64_t v)
    {
        while (v >= 0x80) { s.push_back((char)(uint8_t)(v | 0x80)); v >>= 7; }
        s.push_back((char)(uint8_t)v);
    }
    void tag(uint32_t f, uint32_t wt) { varint((uint64_t)f << 3 | wt); }
    void bytes(uint32_t f, const std::string &v) { tag(f, 2); varint(v.size()); s += v; }
    void str(uint32_t f, const std::string &v) { if (!v.empty()) bytes(f, v); }
    void fx64(uint32_t f, uint64_t v, bool always = false)
    {
        if (!v && !always) return;
        tag(f, 1);
        s.append(reinterpret_cast<const char *>(&v), 8);
    }
    void dbl(uint32_t f, double v)
    {
        uint64_t u;
        memcpy(&u, &v, 8);
        fx64(f, u);
    }
    void enm(uint32_t f, uint32_t v) { if (v) { tag(f, 0); varint(v); } }
};
struct Otlp {
    Pb out; // ScopeMetrics fields
    PromLabels add;
    uint64_t t0 = 0, t1 = 0;
    std::string attrs(uint32_t f, const PromLabels &l) const
    {
        Pb p;
        for (auto &kv : l) {
            Pb any, kvm;
            any.bytes(1, kv.second); // oneof string_value: written even when empty
            kvm.str(1, kv.first);
            kvm.bytes(2, any.s);
            p.bytes(f, kvm.s);
        }
        return p.s;
    }
    std::string number_point(const PromLabels &l, int64_t v) const
    {
        Pb d;
        d.fx64(2, t0);
        d.fx64(3, t1);
        d.fx64(6, (uint64_t)v, true); // oneof as_int
        d.s += attrs(7, l);
        return d.s;
    }
    void metric(const std::string &name, const char *desc, uint32_t field, const std::string &data, bool has_data = true)
    {
        Pb m;
        m.str(1, name);
        m.str(2, desc);
        if (has_data) m.bytes(field, data);
        out.bytes(2, m.s);
    }
    // Counter / Cardinality: a gauge of one int point
    template <typename V>
    void gauge(const std::string &name, const char *desc, V v)
    {
        Pb g;
        g.bytes(1, number_point(add, (int64_t)v));
        metric(name, desc, 5, g.s);
    }
    // Quantile: a summary point with the four quantiles (no count / sum, as the reference)
    template <typename T>
    void summary(const std::string &name, const char *desc, const std::vector<T> &q, T, uint64_t)
    {
        if (q.empty()) return;
        static const double fr[4] = {0.50, 0.90, 0.95, 0.99};
        Pb d;
        d.fx64(2, t0);
        d.fx64(3, t1);
        for (int i = 0; i < 4; i++) {
            Pb qv;
            qv.dbl(1, fr[i]);
            qv.dbl(2, (double)q[i]);
            d.bytes(6, qv.s);
        }
        d.s += attrs(7, add);
        Pb sm;
        sm.bytes(1, d.s);
        metric(name, desc, 11, sm.s);
    }
    // TopN: one gauge point per reported item (items with an empty name are skipped)
    void topn(const std::string &name, const char *item_key, const char *desc,
              const std::vector<std::pair<std::string, uint64_t>> &v0, size_t n, uint32_t pct)
    {
        auto v = v0;
        std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) {
            if (a.second != b.second) return a.second > b.second;
            return a.first < b.first;
        });
        const size_t k = std::min(n, v.size());
        if (!k) return;
        std::vector<uint64_t> est;
        for (size_t i = 0; i < k; i++) est.push_back(v[i].second);
        std::sort(est.begin(), est.end());
        const uint64_t w = (uint64_t)std::ceil((double)pct / 100.0 * (double)k);
        const uint64_t thr = est[w == 0 ? 0 : std::min<size_t>(w - 1, k - 1)];
        PromLabels l(add);
        Pb g;
        bool any = false;
        for (size_t i = 0; i < k && v[i].second >= thr; i++) {
            if (v[i].first.empty()) continue;
            l[item_key] = v[i].first;
            g.bytes(1, number_point(l, (int64_t)v[i].second));
            any = true;
        }
        metric(name, desc, 5, g.s, any);
    }
    // Histogram: bounds at the listed split points, bucket_counts as the reference computes
    // them (static_cast<uint64_t>(cdf) * n: n where the CDF reached 1, else 0)
    void histogram(const std::string &name, const char *desc, std::vector<uint64_t> v)
    {
        if (v.empty()) return;
        std::sort(v.begin(), v.end());
        const uint64_t n = v.size();
        std::vector<uint64_t> cnt;
        std::vector<double> bnd;
        uint64_t prev = 0;
        for (uint64_t x : hist_points()) {
            const uint64_t c = (uint64_t)(std::upper_bound(v.begin(), v.end(), x) - v.begin());
            if (c != prev) {
                bnd.push_back((double)x);
                cnt.push_back(static_cast<uint64_t>((double)c / (double)n) * n);
            }
            prev = c;
        }
        Pb d;
        d.fx64(2, t0);
        d.fx64(3, t1);
        d.fx64(4, n);
        d.tag(6, 2);
        d.varint(cnt.size() * 8);
        d.s.append(reinterpret_cast<const char *>(cnt.data()), cnt.size() * 8);
        d.tag(7, 2);
        d.varint(bnd.size() * 8);
        d.s.append(reinterpret_cast<const char *>(bnd.data()), bnd.size() * 8);
        d.s += attrs(9, add);
        Pb h;
        h.bytes(1, d.s);
        h.enm(2, 2); // AGGREGATION_TEMPORALITY_CUMULATIVE
        metric(name, desc, 9, h.s);
    }
};

// NetworkMetricsBucket::to_prometheus (src/handlers/net/v1/NetStreamHandler.cpp:332-388);
// names and descriptions from NetStreamHandler.h:81-127
template <class Sink>
void net_metrics(pv_ctx *c, Sink &p, const HostBucket &b)
{
    const uint64_t *n = &b.sum[PV_OFF_NET];
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    p.gauge("packets_events", "Total packets events generated", n[NC_EVENTS]);
    p.gauge("packets_deep_samples", "Total packets that were sampled for deep inspection", n[NC_SAMPLES]);
    if (c->net_groups & PV_NET_COUNTERS) {
        p.gauge("packets_udp", "Count of UDP packets", n[NC_UDP]);
        p.gauge("packets_tcp", "Count of TCP packets", n[NC_TCP]);
        p.gauge("packets_protocol_tcp_syn", "Count of TCP SYN packets", n[NC_SYN]);
        p.gauge("packets_other_l4", "Count of packets which are not UDP or TCP", n[NC_OTHER]);
        p.gauge("packets_ipv4", "Count of IPv4 packets", n[NC_V4]);
        p.gauge("packets_ipv6", "Count of IPv6 packets", n[NC_V6]);
        p.gauge("packets_in", "Count of total ingress packets", n[NC_IN]);
        p.gauge("packets_out", "Count of total egress packets", n[NC_OUT]);
        p.gauge("packets_unknown_dir", "Count of total unknown direction packets", n[NC_UNK]);
        p.gauge("packets_total", "Count of total packets matching the configured filter(s)", n[NC_TOTAL]);
        p.gauge("packets_filtered", "Count of total packets that did not match the configured filter(s) (if any)", n[NC_FILTERED]);
    }
    if (c->net_groups & PV_NET_CARDINALITY) {
        p.gauge("packets_cardinality_src_ips_in", "Source IP cardinality", lround(cpc_estimate(&b.cpc[CPC_SRC * PV_CPC_COUPONS], b.merged)));
        p.gauge("packets_cardinality_dst_ips_out", "Destination IP cardinality", lround(cpc_estimate(&b.cpc[CPC_DST * PV_CPC_COUPONS], b.merged)));
    }
    if (c->net_groups & PV_NET_TOP_IPS) {
        p.topn("packets_top_ipv4", "ipv4", "Top IPv4 IP addresses", tops_of(b, TM_IPV4), topn, pct);
        p.topn("packets_top_ipv6", "ipv6", "Top IPv6 IP addresses", tops_of(b, TM_IPV6), topn, pct);
    }
    // top_geo: no MaxMind database, the TopNs stay empty and write nothing
    uint64_t cnt;
    const uint64_t *h = &b.sum[PV_OFF_PAYLOAD];
    auto q = hist_quantiles(h, PV_PAYLOAD_BINS, cnt);
    if (!b.qs_payload.empty() && cnt) q = b.qs_payload;
    uint64_t mx = 0;
    for (size_t i = 0; i < PV_PAYLOAD_BINS; i++)
        if (h[i]) mx = i;
    p.template summary<uint64_t>("packets_payload_size", "Quantiles of payload sizes, in bytes", q, mx, cnt);
}

// DnsMetricsBucket::to_prometheus (src/handlers/dns/v1/DnsStreamHandler.cpp:1139-1238);
// names and descriptions from DnsStreamHandler.h:116-171
template <class Sink>
void dns_metrics(pv_ctx *c, Sink &p, const HostBucket &b)
{
    const uint64_t *d = &b.sum[PV_OFF_DNS];
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    const uint32_t g = c->dns_groups;
    p.gauge("dns_wire_packets_events", "Total DNS wire packets events", d[DC_EVENTS]);
    p.gauge("dns_wire_packets_deep_samples", "Total DNS wire packets that were sampled for deep inspection", d[DC_SAMPLES]);
    if (g & PV_DNS_COUNTERS) {
        p.gauge("dns_wire_packets_queries", "Total DNS wire packets flagged as query (ingress and egress)", d[DC_QUERIES]);
        p.gauge("dns_wire_packets_replies", "Total DNS wire packets flagged as reply (ingress and egress)", d[DC_REPLIES]);
        p.gauge("dns_wire_packets_tcp", "Total DNS wire packets received over TCP (ingress and egress)", d[DC_TCP]);
        p.gauge("dns_wire_packets_udp", "Total DNS wire packets received over UDP (ingress and egress)", d[DC_UDP]);
        p.gauge("dns_wire_packets_ipv4", "Total DNS wire packets received over IPv4 (ingress and egress)", d[DC_V4]);
        p.gauge("dns_wire_packets_ipv6", "Total DNS wire packets received over IPv6 (ingress and egress)", d[DC_V6]);
        p.gauge("dns_wire_packets_nxdomain", "Total DNS wire packets flagged as reply with response code NXDOMAIN (ingress and egress)", d[DC_NX]);
        p.gauge("dns_wire_packets_refused", "Total DNS wire packets flagged as reply with response code REFUSED (ingress and egress)", d[DC_REFUSED]);
        p.gauge("dns_wire_packets_srvfail", "Total DNS wire packets flagged as reply with response code SRVFAIL (ingress and egress)", d[DC_SRVFAIL]);
        p.gauge("dns_wire_packets_noerror", "Total DNS wire packets flagged as reply with response code NOERROR (ingress and egress)", d[DC_NOERROR]);
        p.gauge("dns_wire_packets_nodata", "Total DNS wire packets flagged as reply with response code NOERROR and no answer section data (ingress and egress)", d[DC_NODATA]);
        p.gauge("dns_wire_packets_total", "Total DNS wire packets matching the configured filter(s)", d[DC_TOTAL]);
        p.gauge("dns_wire_packets_filtered", "Total DNS wire packets seen that did not match the configured filter(s) (if any)", d[DC_FILTERED]);
    }
    if (g & PV_DNS_CARDINALITY)
        p.gauge("dns_cardinality_qname", "Cardinality of unique QNAMES, both ingress and egress", lround(cpc_estimate(&b.cpc[CPC_QNAME * PV_CPC_COUPONS], b.merged)));
    auto vmax = [](const auto &v) { return v.empty() ? 0 : *std::max_element(v.begin(), v.end()); };
    if (g & PV_DNS_TRANSACTIONS) {
        p.gauge("dns_xact_counts_total", "Total DNS transactions (query/reply pairs)", d[DC_XTOTAL]);
        p.gauge("dns_xact_counts_timed_out", "Total number of DNS transactions that timed out", d[DC_XTIMEOUT]);
        p.gauge("dns_xact_in_total", "Total ingress DNS transactions (host is server)", d[DC_XIN]);
        p.topn("dns_xact_in_top_slow", "qname", "Top QNAMES in transactions where host is the server and transaction speed is slower than p90",
               tops_of(b, TM_SLOW_IN), topn, pct);
        if (g & PV_DNS_QUANTILES) {
            if (!b.from_us.empty())
                p.template summary<uint64_t>("dns_xact_out_quantiles_us", "Quantiles of transaction timing (query/reply pairs) when host is client, in microseconds",
                                    b.qs_from.empty() ? quantiles(b.from_us) : b.qs_from, vmax(b.from_us), b.from_us.size());
            if (!b.to_us.empty())
                p.template summary<uint64_t>("dns_xact_in_quantiles_us", "Quantiles of transaction timing (query/reply pairs) when host is server, in microseconds",
                                    b.qs_to.empty() ? quantiles(b.to_us) : b.qs_to, vmax(b.to_us), b.to_us.size());
            if (!b.ratio.empty())
                p.template summary<double>("dns_xact_ratio_quantiles", "Quantiles of ratio of packet sizes in a DNS transaction (reply/query)",
                                  b.qs_ratio.empty() ? quantiles(b.ratio) : b.qs_ratio, vmax(b.ratio), b.ratio.size());
        }
        if (g & PV_DNS_HISTOGRAMS) {
            p.histogram("dns_xact_out_histogram_us", "Histogram of transaction timing (query/reply pairs) when host is client, in microseconds", b.hist_from());
            p.histogram("dns_xact_in_histogram_us", "Histogram of transaction timing (query/reply pairs) when host is server, in microseconds", b.hist_to());
        }
        p.gauge("dns_xact_out_total", "Total egress DNS transactions (host is client)", d[DC_XOUT]);
        p.topn("dns_xact_out_top_slow", "qname", "Top QNAMES in transactions where host is the client and transaction speed is slower than p90",
               tops_of(b, TM_SLOW_OUT), topn, pct);
    }
    if (g & PV_DNS_TOP_PORTS)
        p.topn("dns_top_udp_ports", "port", "Top UDP source port on the query side of a transaction", dense_tops(&b.sum[PV_OFF_PORT], PV_PORT_BINS, 0), topn, pct);
    if (g & PV_DNS_TOP_ECS) {
        if (g & PV_DNS_COUNTERS) p.gauge("dns_wire_packets_query_ecs", "Total queries that have EDNS Client Subnet (ECS) field set", d[DC_QECS]);
        // geo / ASN of the subnet: no MaxMind database, those TopNs write nothing
        p.topn("dns_top_query_ecs", "ecs", "Top EDNS Client Subnet (ECS) observed in DNS queries", tops_of(b, TM_ECS), topn, pct);
    }
    if (g & PV_DNS_TOP_QNAMES) {
        p.topn("dns_top_qname2", "qname", "Top QNAMES, aggregated at a depth of two labels", tops_of(b, TM_QNAME2), topn, pct);
        p.topn("dns_top_qname3", "qname", "Top QNAMES, aggregated at a depth of three labels", tops_of(b, TM_QNAME3), topn, pct);
        p.topn("dns_top_nxdomain", "qname", "Top QNAMES with result code NXDOMAIN", tops_of(b, TM_NX), topn, pct);
        p.topn("dns_top_refused", "qname", "Top QNAMES with result code REFUSED", tops_of(b, TM_REFUSED), topn, pct);
        p.topn("dns_top_srvfail", "qname", "Top QNAMES with result code SRVFAIL", tops_of(b, TM_SRVFAIL), topn, pct);
        p.topn("dns_top_nodata", "qname", "Top QNAMES with result code NOERROR and no answer section", tops_of(b, TM_NODATA), topn, pct);
        if (g & PV_DNS_TOP_QNAMES_DETAILS) {
            p.topn("dns_top_qname_by_resp_bytes", "qname", "Top QNAMES by response volume in bytes", tops_of(b, TM_SIZED), topn, pct);
            p.topn("dns_top_noerror", "qname", "Top QNAMES with result code NOERROR", tops_of(b, TM_NOERROR), topn, pct);
        }
    }
    p.topn("dns_top_rcode", "rcode", "Top result codes", dense_tops(&b.sum[PV_OFF_RCODE], PV_RCODE_BINS, 2), topn, pct);
    p.topn("dns_top_qtype", "qtype", "Top query types", dense_tops(&b.sum[PV_OFF_QTYPE], PV_QTYPE_BINS, 1), topn, pct);
}

// NetworkMetricsBucket::to_prometheus / to_opentelemetry, Net v2
// (src/handlers/net/v2/NetStreamHandler.cpp:333-383; names NetStreamHandler.h:72-181): the
// event counts, `filtered_packets`, then per direction the bucket has seen, labelled
// direction=in|out|unknown (rates are timer-driven and out of scope; geo / ASN TopNs empty)
template <class Sink>
void net2_metrics(pv_ctx *c, Sink &p, const HostBucket &b)
{
    const uint64_t *n = &b.sum[PV_OFF_NET2];
    const uint32_t g = c->net2_groups;
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    p.gauge("net_observed_packets", "Total packets events generated", n[N2_EVENTS]);
    p.gauge("net_deep_sampled_packets", "Total packets that were sampled for deep inspection", n[N2_SAMPLES]);
    if (g & PV_N2G_COUNTERS) p.gauge("net_filtered_packets", "Total packets seen that did not match the configured filter(s) (if any)", n[N2_FILTERED]);
    static const char *dirs[3] = {"in", "out", "unknown"};
    const PromLabels base = p.add;
    for (uint32_t d = 0; d < 3; d++) {
        const uint64_t *dc = n + N2_DIR + 8 * d;
        if (!dc[N2_TOTAL]) continue;
        p.add = base;
        p.add["direction"] = dirs[d];
        if (g & PV_N2G_COUNTERS) {
            p.gauge("net_udp_packets", "Count of UDP packets", dc[N2_UDP]);
            p.gauge("net_tcp_packets", "Count of TCP packets", dc[N2_TCP]);
            p.gauge("net_other_l4_packets", "Count of packets which are not UDP or TCP", dc[N2_OTHER]);
            p.gauge("net_ipv4_packets", "Count of IPv4 packets", dc[N2_V4]);
            p.gauge("net_ipv6_packets", "Count of IPv6 packets", dc[N2_V6]);
            p.gauge("net_tcp_syn_packets", "Count of TCP SYN packets", dc[N2_SYN]);
            p.gauge("net_total_packets", "Count of total packets matching the configured filter(s)", dc[N2_TOTAL]);
        }
        if (g & PV_N2G_CARDINALITY)
            p.gauge("net_cardinality_ips", "IP cardinality", lround(cpc_estimate(&b.cpc[(CPC_V2 + d) * PV_CPC_COUPONS], b.merged)));
        if (g & PV_N2G_TOP_IPS) {
            p.topn("net_top_ipv4_packets", "ipv4", "Top IPv4 addresses", tops_of(b, TMH_V2_IP4 + d), topn, pct);
            p.topn("net_top_ipv6_packets", "ipv6", "Top IPv6 addresses", tops_of(b, TMH_V2_IP6 + d), topn, pct);
        }
        if (g & PV_N2G_QUANTILES) {
            uint64_t cnt;
            const uint64_t *h = &b.sum[PV_OFF_PAYLOAD2 + d * PV_PAYLOAD_BINS];
            auto q = hist_quantiles(h, PV_PAYLOAD_BINS, cnt);
            if (cnt && !b.qs_payload2[d].empty()) q = b.qs_payload2[d];
            uint64_t mx = 0;
            for (size_t i = 0; i < PV_PAYLOAD_BINS; i++)
                if (h[i]) mx = i;
            if (cnt) p.template summary<uint64_t>("net_payload_size_bytes", "Quantiles of payload sizes, in bytes", q, mx, cnt);
        }
    }
    p.add = base;
}

// DnsMetricsBucket::to_prometheus / to_opentelemetry, DNS v2
// (src/handlers/dns/v2/DnsStreamHandler.cpp:759-842; names DnsStreamHandler.h:98-115,250-270):
// the event counts, `filtered_packets`, then per transaction direction the bucket has set up
template <class Sink>
void dns2_metrics(pv_ctx *c, Sink &p, const HostBucket &b)
{
    const uint64_t *d = &b.sum[PV_OFF_DNS];
    const uint32_t g = c->dns2_groups;
    const size_t topn = c->cfg.topn_count;
    const uint32_t pct = c->cfg.topn_percentile_threshold;
    p.gauge("dns_observed_packets", "Total DNS wire packets events", d[DC_EVENTS]);
    p.gauge("dns_deep_sampled_packets", "Total DNS wire packets that were sampled for deep inspection", d[DC_SAMPLES]);
    if (g & PV_DNS2_COUNTERS)
        p.gauge("dns_filtered_packets", "Total DNS wire packets seen that did not match the configured filter(s) (if any)", d[DC_FILTERED]);
    static const char *dirs[3] = {"in", "out", "unknown"};
    auto vmax = [](const auto &v) { return v.empty() ? 0 : *std::max_element(v.begin(), v.end()); };
    const PromLabels base = p.add;
    for (uint32_t x = 0; x < 3; x++) {
        const uint64_t *c2 = &b.sum[PV_OFF_DNS2 + x * PV_DNS2_CTRS];
        if (!c2[D2_SEEN]) continue;
        auto tops = [&](uint32_t metric) { return tops_of(b, TMH_V2_DNS + 4 * metric + x); };
        p.add = base;
        p.add["direction"] = dirs[x];
        if (g & PV_DNS2_COUNTERS) {
            p.gauge("dns_xacts", "Total DNS transactions (query/reply pairs)", c2[D2_XACTS]);
            p.gauge("dns_udp_xacts", "Total DNS transactions (query/reply pairs) received over UDP", c2[D2_UDP]);
            p.gauge("dns_tcp_xacts", "Total DNS transactions (query/reply pairs) received over TCP", c2[D2_TCP]);
            p.gauge("dns_dot_xacts", "Total DNS transactions (query/reply pairs) received over DNS over TLS", c2[D2_DOT]);
            p.gauge("dns_doh_xacts", "Total DNS transactions (query/reply pairs) received over DNS over HTTPS", c2[D2_DOH]);
            p.gauge("dns_dnscrypt_udp_xacts", "Total DNS transactions (query/reply pairs) received over DNSCrypt over UDP", c2[D2_CRYPT_UDP]);
            p.gauge("dns_dnscrypt_tcp_xacts", "Total DNS transactions (query/reply pairs) received over DNSCrypt over TCP", c2[D2_CRYPT_TCP]);
            p.gauge("dns_doq_xacts", "Total DNS transactions (query/reply pairs) received over DNS over QUIC", c2[D2_DOQ]);
            p.gauge("dns_ipv4_xacts", "Total DNS transactions (query/reply pairs) received over IPv4", c2[D2_V4]);
            p.gauge("dns_ipv6_xacts", "Total DNS transactions (query/reply pairs) received over IPv6", c2[D2_V6]);
            p.gauge("dns_nxdomain_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code NXDOMAIN", c2[D2_NX]);
            p.gauge("dns_ecs_xacts", "Total DNS transactions (query/reply pairs) with the EDNS Client Subnet option set", c2[D2_ECS]);
            p.gauge("dns_refused_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code REFUSED", c2[D2_REFUSED]);
            p.gauge("dns_srvfail_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code SRVFAIL", c2[D2_SRVFAIL]);
            p.gauge("dns_noerror_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code NOERROR", c2[D2_NOERROR]);
            p.gauge("dns_nodata_xacts", "Total DNS transactions (query/reply pairs) flagged as reply with response code NOERROR but with an empty answers section", c2[D2_NODATA]);
            p.gauge("dns_authenticated_data_xacts", "Total DNS transactions (query/reply pairs) with the AD flag set in the response", c2[D2_AD]);
            p.gauge("dns_authoritative_answer_xacts", "Total DNS transactions (query/reply pairs) with the AA flag set in the response", c2[D2_AA]);
            p.gauge("dns_checking_disabled_xacts", "Total DNS transactions (query/reply pairs) with the CD flag set in the query", c2[D2_CD]);
            p.gauge("dns_timeout_queries", "Total number of DNS queries that timed out", c2[D2_TIMEOUT]);
            p.gauge("dns_orphan_responses", "Total number of DNS responses that do not have a corresponding query", c2[D2_ORPHAN]);
        }
        if (g & PV_DNS2_CARDINALITY)
            p.gauge("dns_cardinality_qname", "Cardinality of unique QNAMES, both ingress and egress",
                    lround(cpc_estimate(&b.cpc[(CPC_QNAME2 + x) * PV_CPC_COUPONS], b.merged)));
        if (g & PV_DNS2_TOP_PORTS)
            p.topn("dns_top_udp_ports_xacts", "port", "Top UDP source port on the query side of a transaction",
                   dense_tops(&b.sum[PV_OFF_PORT2 + x * PV_PORT_BINS], PV_PORT_BINS, 0), topn, pct);
        if (g & PV_DNS2_TOP_ECS)
            // geo / ASN of the subnet: no MaxMind database, those TopNs write nothing
            p.topn("dns_top_ecs_xacts", "ecs", "Top EDNS Client Subnet (ECS) observed in DNS transaction", tops(TM_ECS), topn, pct);
        if (g & PV_DNS2_TOP_RCODES) {
            p.topn("dns_top_nxdomain_xacts", "qname", "Top QNAMES with result code NXDOMAIN", tops(TM_NX), topn, pct);
            p.topn("dns_top_refused_xacts", "qname", "Top QNAMES with result code REFUSED", tops(TM_REFUSED), topn, pct);
            p.topn("dns_top_srvfail_xacts", "qname", "Top QNAMES with result code SRVFAIL", tops(TM_SRVFAIL), topn, pct);
            p.topn("dns_top_nodata_xacts", "qname", "Top QNAMES with result code NOERROR and empty answer section", tops(TM_NODATA), topn, pct);
            p.topn("dns_top_noerror_xacts", "qname", "Top QNAMES with result code NOERROR", tops(TM_NOERROR), topn, pct);
            p.topn("dns_top_rcode_xacts", "rcode", "Top result codes", dense_tops(&b.sum[PV_OFF_RCODE2 + x * PV_RCODE_BINS], PV_RCODE_BINS, 2),
                   topn, pct);
        }
        if (g & PV_DNS2_TOP_QNAMES) {
            p.topn("dns_top_qname2_xacts", "qname", "Top QNAMES, aggregated at a depth of two labels", tops(TM_QNAME2), topn, pct);
            p.topn("dns_top_qname3_xacts", "qname", "Top QNAMES, aggregated at a depth of three labels", tops(TM_QNAME3), topn, pct);
        }
        if (g & PV_DNS2_TOP_SIZE) {
            p.topn("dns_top_response_bytes", "qname", "Top QNAMES by response volume in bytes", tops(TM_SIZED), topn, pct);
            const auto &r = b.ratio2[x];
            if (!r.empty())
                p.template summary<double>("dns_response_query_size_ratio", "Quantiles of ratio of packet sizes in a DNS transaction (reply/query)",
                                           b.qs_ratio2[x].empty() ? quantiles(r) : b.qs_ratio2[x], vmax(r), r.size());
        }
        if (g & PV_DNS2_TOP_QTYPES)
            p.topn("dns_top_qtype_xacts", "qtype", "Top query types", dense_tops(&b.sum[PV_OFF_QTYPE2 + x * PV_QTYPE_BINS], PV_QTYPE_BINS, 1),
                   topn, pct);
        if (g & PV_DNS2_XACT_TIMES) {
            const auto &t = b.time2[x];
            if (!t.empty())
                p.template summary<uint64_t>("dns_xact_time_us", "Quantiles of transaction timing (query/reply pairs) in microseconds",
                                             b.qs_time2[x].empty() ? quantiles(t) : b.qs_time2[x], vmax(t), t.size());
            p.histogram("dns_xact_histogram_us", "Histogram of transaction timing (query/reply pairs) in microseconds", b.hist_time2(x));
            p.topn("dns_top_slow_xacts", "qname", "Top QNAMES in transactions where host is the server and transaction speed is slower than p90",
                   tops(TM_SLOW_OUT), topn, pct);
        }
    }
    p.add = base;
}

// KLL inclusive rank rule on exact data
} // namespace pvh

extern "C" {

int pv_window_json(pv_ctx *c, uint32_t period, int merged, char **out)
{
    *out = nullptr;
    // the transaction values are drained under the lock: a batch the producer runs between
    // the drain and the read would otherwise show its counters without its values
    std::lock_guard<std::mutex> g(c->mu);
    int rc = sync_xvals(c);
    if (rc) return rc;
    flush_fills(c);
    if (!c->started) return c->fail(PV_EINVAL, "no data");
    Json j;
    j.obj();
    std::vector<uint32_t> slots;
    {
        if ((rc = window_slots(c, c->net, period, merged != 0, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, merged != 0, PART_NET, b))) return rc;
        j.key("packets").obj();
        net_json(c, j, b);
        j.end_obj();
        if (c->net2_groups) {
            j.key("net").obj();
            net2_json(c, j, b);
            j.end_obj();
        }
    }
    {
        if ((rc = window_slots(c, c->dns, period, merged != 0, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, merged != 0, PART_DNS, b))) return rc;
        j.key("dns").obj();
        if (c->dns2_groups) dns2_json(c, j, b);
        else dns_json(c, j, b);
        j.end_obj();
    }
    j.end_obj();
    *out = strdup(j.s.c_str());
    return 0;
}

// ---- external buckets: the bucket half of the handler object (StreamHandler::merge and the
// window_*(..., AbstractMetricsBucket *) overloads, src/StreamHandler.h:72-77,221-269), which
// a policy uses to fold like handlers across taps (Policy::_get_merged_buckets,
// src/Policies.cpp:420-446)

} // extern "C"

struct pv_bucket {
    int part;            // PART_NET / PART_DNS
    uint32_t handler;    // PV_HANDLER_NET / PV_HANDLER_DNS
    HostBucket b;
};
namespace {
// Quantile::merge(other, Aggregate::SUM) (src/Metrics.h:356-372) on exact values: the sketch of
// a non-empty bucket stays, the p-wise sum of the quantiles grows; an empty one merges
template <typename T>
void qsum_fold(std::vector<T> &dv, std::vector<T> &qs, const std::vector<T> &ov, const std::vector<T> &oqs)
{
    if (dv.empty()) { dv.insert(dv.end(), ov.begin(), ov.end()); return; }
    if (ov.empty()) return;
    const std::vector<T> oq = quantiles(ov);
    (void)oqs; // the other sketch's own quantiles (get_quantiles(other._quantile)), not its sums
    if (qs.empty()) qs = quantiles(dv);
    for (int i = 0; i < 4; i++) qs[i] += oq[i];
}
// AbstractMetricsBucket::merge(other, Aggregate::SUM) (src/AbstractMetricsManager.h:177-195) and
// the handlers' specialized_merge (net/v1/NetStreamHandler.cpp:285-330,
// dns/v1/DnsStreamHandler.cpp:658-733)
void bucket_fold_sum(HostBucket &d, const HostBucket &o, int part)
{
    d.period_length += o.period_length;
    if (o.start_sec < d.start_sec) { d.start_sec = o.start_sec; d.start_nsec = o.start_nsec; }
    if (o.end_sec > d.end_sec) { d.end_sec = o.end_sec; d.end_nsec = o.end_nsec; }
    // payload_size, a Quantile over a dense histogram: an empty one merges the other's sketch,
    // else the p-wise sums grow
    auto payload_fold = [&](size_t off, std::vector<uint64_t> &qs) {
        uint64_t dn = 0, on = 0;
        const auto dq = hist_quantiles(&d.sum[off], PV_PAYLOAD_BINS, dn);
        const auto oq = hist_quantiles(&o.sum[off], PV_PAYLOAD_BINS, on);
        if (!dn) {
            for (size_t i = 0; i < PV_PAYLOAD_BINS; i++) d.sum[off + i] += o.sum[off + i];
        } else if (on) {
            if (qs.empty()) qs = dq;
            for (int i = 0; i < 4; i++) qs[i] += oq[i];
        }
    };
    if (part == PART_NET) {
        // counters (v1, and v2's per direction); Net v2 specialized_merge
        // (net/v2/NetStreamHandler.cpp:286-331): per direction the same rules
        for (size_t i = 0; i < PV_SUM_NET_WORDS; i++)
            if ((i < PV_OFF_PAYLOAD || i >= PV_OFF_PAYLOAD + PV_PAYLOAD_BINS) && i < PV_OFF_PAYLOAD2) d.sum[i] += o.sum[i];
        payload_fold(PV_OFF_PAYLOAD, d.qs_payload);
        for (uint32_t x = 0; x < 3; x++) payload_fold(PV_OFF_PAYLOAD2 + x * PV_PAYLOAD_BINS, d.qs_payload2[x]);
    } else {
        for (size_t i = PV_OFF_DNS; i < PV_SUM_WORDS; i++) d.sum[i] += o.sum[i];
        // histograms merge their sketches; the quantiles follow the SUM rule
        if (!d.hist_sep) { d.hfrom_us = d.from_us; d.hto_us = d.to_us; d.hist_sep = true; }
        const auto &ohf = o.hist_from(), &oht = o.hist_to();
        d.hfrom_us.insert(d.hfrom_us.end(), ohf.begin(), ohf.end());
        d.hto_us.insert(d.hto_us.end(), oht.begin(), oht.end());
        qsum_fold(d.from_us, d.qs_from, o.from_us, o.qs_from);
        qsum_fold(d.to_us, d.qs_to, o.to_us, o.qs_to);
        qsum_fold(d.ratio, d.qs_ratio, o.ratio, o.qs_ratio);
        // DNS v2 specialized_merge (dns/v2/DnsStreamHandler.cpp:619-676), per direction:
        // dnsTimeUs and dnsRatio by the SUM rule, dnsHistTimeUs merging its sketch
        if (!d.hist2_sep) {
            for (uint32_t x = 0; x < 3; x++) d.htime2[x] = d.time2[x];
            d.hist2_sep = true;
        }
        for (uint32_t x = 0; x < 3; x++) {
            const auto &oh = o.hist_time2(x);
            d.htime2[x].insert(d.htime2[x].end(), oh.begin(), oh.end());
            qsum_fold(d.time2[x], d.qs_time2[x], o.time2[x], o.qs_time2[x]);
            qsum_fold(d.ratio2[x], d.qs_ratio2[x], o.ratio2[x], o.qs_ratio2[x]);
        }
    }
    for (size_t i = 0; i < PV_MIN_WORDS; i++) d.cpc[i] = std::min(d.cpc[i], o.cpc[i]); // CPC union (ICON)
    for (auto &m : o.tops)
        for (auto &kv : m.second) d.tops[m.first][kv.first] += kv.second;
}
} // namespace
extern "C" {

int pv_bucket_merge(pv_ctx *c, uint32_t handler, pv_bucket **bucket, uint32_t period, int prometheus, int merged)
{
    if (!bucket || (handler != PV_HANDLER_NET && handler != PV_HANDLER_DNS)) return c->fail(PV_EINVAL, "bucket merge: one handler");
    std::lock_guard<std::mutex> g(c->mu); // values drained under the lock (pv_window_json)
    int rc = sync_xvals(c);
    if (rc) return rc;
    flush_fills(c);
    if (!c->started) return c->fail(PV_EINVAL, "no data");
    const int part = handler == PV_HANDLER_NET ? PART_NET : PART_DNS;
    const Window &w = part == PART_NET ? c->net : c->dns;
    if (*bucket && (*bucket)->part != part) return c->fail(PV_EINVAL, "bucket merge: a bucket of another handler");
    // StreamMetricsHandler::merge: Prometheus output reads period 1 once the manager holds more
    // than one, never merged
    if (prometheus) { period = w.slots.size() > 1 ? 1 : 0; merged = 0; }
    std::vector<uint32_t> slots;
    if ((rc = window_slots(c, w, period, merged != 0, slots))) return rc;
    HostBucket b;
    // a fresh bucket merged from this handler's bucket(s): CPC through a union (ICON)
    if ((rc = load_bucket(c, slots, true, part, b))) return rc;
    if (!*bucket) {
        pv_bucket *nb = new (std::nothrow) pv_bucket;
        if (!nb) return c->fail(PV_ECAPACITY, "bucket merge: out of host memory");
        nb->part = part;
        nb->handler = handler;
        nb->b = std::move(b);
        *bucket = nb;
        return 0;
    }
    bucket_fold_sum((*bucket)->b, b, part);
    return 0;
}

void pv_bucket_free(pv_bucket *b) { delete b; }

int pv_bucket_json(pv_ctx *c, const pv_bucket *bk, char **out)
{
    *out = nullptr;
    if (!bk) return c->fail(PV_EINVAL, "bucket json: no bucket");
    std::lock_guard<std::mutex> g(c->mu);
    Json j;
    j.obj();
    // window_external_json: {"<schema key>": {period, metrics}} (AbstractMetricsManager.h:589-599)
    // (as pv_window_json: a Net bucket holds the v1 and v2 Net handlers' parts)
    if (bk->part == PART_NET) {
        if (c->net_groups) { j.key("packets").obj(); net_json(c, j, bk->b); j.end_obj(); }
        if (c->net2_groups) { j.key("net").obj(); net2_json(c, j, bk->b); j.end_obj(); }
    } else if (c->dns_groups) {
        j.key("dns").obj();
        if (c->dns2_groups) dns2_json(c, j, bk->b);
        else dns_json(c, j, bk->b);
        j.end_obj();
    }
    j.end_obj();
    *out = strdup(j.s.c_str());
    return 0;
}

int pv_bucket_prometheus(pv_ctx *c, const pv_bucket *bk, const char *const *label_keys, const char *const *label_values,
                         uint32_t n_labels, char **out)
{
    *out = nullptr;
    if (!bk) return c->fail(PV_EINVAL, "bucket prometheus: no bucket");
    std::lock_guard<std::mutex> g(c->mu);
    Prom p;
    for (uint32_t i = 0; i < n_labels; i++) {
        if (!label_keys || !label_values || !label_keys[i] || !label_values[i]) return c->fail(PV_EINVAL, "label %u missing", i);
        p.add[label_keys[i]] = label_values[i];
    }
    // window_external_prometheus (AbstractMetricsManager.h:580-587)
    if (bk->part == PART_NET && c->net_groups) {
        net_metrics(c, p, bk->b);
        if (c->net2_groups) net2_metrics(c, p, bk->b);
    }
    if (bk->part == PART_DNS && c->dns_groups) {
        if (c->dns2_groups) dns2_metrics(c, p, bk->b);
        else dns_metrics(c, p, bk->b);
    }
    *out = strdup(p.o.str().c_str());
    return 0;
}

int pv_bucket_opentelemetry(pv_ctx *c, const pv_bucket *bk, const char *const *label_keys, const char *const *label_values,
                            uint32_t n_labels, uint8_t **out, size_t *bytes)
{
    *out = nullptr;
    *bytes = 0;
    if (!bk) return c->fail(PV_EINVAL, "bucket opentelemetry: no bucket");
    std::lock_guard<std::mutex> g(c->mu);
    Otlp p;
    for (uint32_t i = 0; i < n_labels; i++) {
        if (!label_keys || !label_values || !label_keys[i] || !label_values[i]) return c->fail(PV_EINVAL, "label %u missing", i);
        p.add[label_keys[i]] = label_values[i];
    }
    // window_external_opentelemetry (AbstractMetricsManager.h:565-578): the bucket's stamps,
    // now for an end it does not have
    p.t0 = (uint64_t)bk->b.start_sec * 1000000000ull + (uint64_t)bk->b.start_nsec;
    if (bk->b.end_sec) p.t1 = (uint64_t)bk->b.end_sec * 1000000000ull + (uint64_t)bk->b.end_nsec;
    else {
        timespec now;
        timespec_get(&now, TIME_UTC);
        p.t1 = (uint64_t)now.tv_sec * 1000000000ull + (uint64_t)now.tv_nsec;
    }
    if (bk->part == PART_NET && c->net_groups) {
        net_metrics(c, p, bk->b);
        if (c->net2_groups) net2_metrics(c, p, bk->b);
    }
    if (bk->part == PART_DNS && c->dns_groups) {
        if (c->dns2_groups) dns2_metrics(c, p, bk->b);
        else dns_metrics(c, p, bk->b);
    }
    *out = (uint8_t *)malloc(p.out.s.size() ? p.out.s.size() : 1);
    if (!*out) return c->fail(PV_ECAPACITY, "bucket opentelemetry: out of host memory");
    memcpy(*out, p.out.s.data(), p.out.s.size());
    *bytes = p.out.s.size();
    return 0;
}

int pv_add_static_label(const char *key, const char *value)
{
    if (!key || !value || !*key) return PV_EINVAL;
    std::lock_guard<std::mutex> g(g_static_mu);
    g_static_labels[key] = value;
    return 0;
}

int pv_window_prometheus(pv_ctx *c, uint32_t period, uint32_t handlers, const char *const *label_keys,
                         const char *const *label_values, uint32_t n_labels, char **out)
{
    *out = nullptr;
    std::lock_guard<std::mutex> g(c->mu); // values drained under the lock (pv_window_json)
    int rc = sync_xvals(c);
    if (rc) return rc;
    flush_fills(c);
    if (!c->started) return c->fail(PV_EINVAL, "no data");
    if (period >= c->cfg.num_periods && period != PV_PERIOD_AUTO)
        return c->fail(PV_EINVAL, "invalid metrics period, specify [0, %u]", c->cfg.num_periods - 1);
    // StreamMetricsHandler::window_prometheus (src/StreamHandler.h:226-233): period 1 of a
    // manager holding more than one bucket, else 0 (each handler's own manager)
    auto per = [&](const Window &w) -> uint32_t { return period != PV_PERIOD_AUTO ? period : (w.slots.size() > 1 ? 1u : 0u); };
    Prom p;
    for (uint32_t i = 0; i < n_labels; i++) {
        if (!label_keys || !label_values || !label_keys[i] || !label_values[i]) return c->fail(PV_EINVAL, "label %u missing", i);
        p.add[label_keys[i]] = label_values[i];
    }
    std::vector<uint32_t> slots;
    // each handler's own window (its manager's window_single_prometheus); a handler with
    // every group disabled writes nothing (AbstractMetricsManager.h:522-524)
    if ((handlers & PV_HANDLER_NET) && c->net_groups) {
        if ((rc = window_slots(c, c->net, per(c->net), false, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, false, PART_NET, b))) return rc;
        net_metrics(c, p, b);
        if (c->net2_groups) net2_metrics(c, p, b);
    }
    if ((handlers & PV_HANDLER_DNS) && c->dns_groups) {
        if ((rc = window_slots(c, c->dns, per(c->dns), false, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, false, PART_DNS, b))) return rc;
        if (c->dns2_groups) dns2_metrics(c, p, b);
        else dns_metrics(c, p, b);
    }
    *out = strdup(p.o.str().c_str());
    return 0;
}

int pv_window_opentelemetry(pv_ctx *c, uint32_t period, uint32_t handlers, const char *const *label_keys,
                            const char *const *label_values, uint32_t n_labels, uint8_t **out, size_t *bytes)
{
    *out = nullptr;
    *bytes = 0;
    std::lock_guard<std::mutex> g(c->mu); // values drained under the lock (pv_window_json)
    int rc = sync_xvals(c);
    if (rc) return rc;
    flush_fills(c);
    if (!c->started) return c->fail(PV_EINVAL, "no data");
    if (period >= c->cfg.num_periods && period != PV_PERIOD_AUTO)
        return c->fail(PV_EINVAL, "invalid metrics period, specify [0, %u]", c->cfg.num_periods - 1);
    // StreamMetricsHandler::window_opentelemetry (src/StreamHandler.h:240-247)
    auto per = [&](const Window &w) -> uint32_t { return period != PV_PERIOD_AUTO ? period : (w.slots.size() > 1 ? 1u : 0u); };
    Otlp p;
    for (uint32_t i = 0; i < n_labels; i++) {
        if (!label_keys || !label_values || !label_keys[i] || !label_values[i]) return c->fail(PV_EINVAL, "label %u missing", i);
        p.add[label_keys[i]] = label_values[i];
    }
    std::vector<uint32_t> slots;
    // the bucket's start / end stamps (end unset: now, as window_single_opentelemetry does)
    auto stamps = [&](const Window &w, uint32_t slot) {
        const SlotMeta &m = w.meta[slot];
        p.t0 = (uint64_t)m.start_sec * 1000000000ull + (uint64_t)m.start_nsec;
        if (m.end_sec) p.t1 = (uint64_t)m.end_sec * 1000000000ull + (uint64_t)m.end_nsec;
        else {
            timespec now;
            timespec_get(&now, TIME_UTC);
            p.t1 = (uint64_t)now.tv_sec * 1000000000ull + (uint64_t)now.tv_nsec;
        }
    };
    if ((handlers & PV_HANDLER_NET) && c->net_groups) {
        if ((rc = window_slots(c, c->net, per(c->net), false, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, false, PART_NET, b))) return rc;
        stamps(c->net, slots[0]);
        net_metrics(c, p, b);
        if (c->net2_groups) net2_metrics(c, p, b);
    }
    if ((handlers & PV_HANDLER_DNS) && c->dns_groups) {
        if ((rc = window_slots(c, c->dns, per(c->dns), false, slots))) return rc;
        HostBucket b;
        if ((rc = load_bucket(c, slots, false, PART_DNS, b))) return rc;
        stamps(c->dns, slots[0]);
        if (c->dns2_groups) dns2_metrics(c, p, b);
        else dns_metrics(c, p, b);
    }
    *out = (uint8_t *)malloc(p.out.s.size() ? p.out.s.size() : 1);
    if (!*out) return c->fail(PV_ECAPACITY, "window_opentelemetry: out of host memory");
    memcpy(*out, p.out.s.data(), p.out.s.size());
    *bytes = p.out.s.size();
    return 0;
}

} // extern "C"
