// SPDX-License-Identifier: MPL-2.0
//
// pv_xshard.cpp — the multi-GPU half of the host runtime behind include/pvgpu.h: a sharded run's
// state merge and read view. Top-N entries to their region owners (pv_topn_x_*,
// pv_comm_merge_topn), the merged view's candidate lists and names, exact distributed quantile
// selection (pv_values_x_select), the RCCL communicator (pv_comm_*), DNS transactions across
// shard edges (pv_edge_*), top_slow against the whole stream's thresholds (pv_slow_*), value
// exports and the window alignment of the global period plan (pv_window_periods,
// pv_advance_windows). The analog of AbstractMetricsBucket::merge (src/AbstractMetricsManager.h:
// 177-195) and Policy::_get_merged_buckets (src/Policies.cpp:420-446) across GPUs.
#include "pv_host.h"

extern "C" {

int comm_allgather_locked(pv_ctx *c, const void *buf, size_t bytes, std::vector<uint8_t> &out);

// ------------------------------------------------------------------ multi-GPU top-N exchange
// (pv_topn_x_*, pv_comm_merge_topn; kernels pv_topn_x* in pv_kernels.hip). Every table's
// regions are split over the ranks in contiguous blocks; a rank ships the live entries of the
// regions others own to their owners (device lists, RCCL point-to-point or host blobs), and
// each owner merges them into its regions with pv_topn_merge. Afterwards a rank's top-N view is
// its own regions; pv_topn_x_candidates / _names / _view then assemble the merged lists from
// every owner's leading entries, names fetched from whichever rank holds them.
namespace {
const uint32_t X_MAGIC = 0x31585650u; // "PVX1"
// candidates per metric and owner: topn_count and the entries tied with the last; a tied group
// larger than this is cut by key order (the merged list's order among equal estimates can then
// differ from one stream's, which orders them by name)
const size_t PV_X_TIES = 8192;
struct XPrep {
    PvXTabs T;
    uint32_t nreg = 0, E = 0;
    std::vector<uint32_t> hdr;      // the header stream, (owner, handler, region, slot) order
    std::vector<uint64_t> dtot, dstart; // entries per owner, where its slice starts
};
uint32_t x_lo_h(uint32_t d, uint32_t nreg, uint32_t W) { return (uint32_t)(((uint64_t)d * nreg + W - 1) / W); }

void x_tables(pv_ctx *c, PvXTabs &T, uint32_t W, uint32_t me)
{
    memset(&T, 0, sizeof T);
    T.W = W;
    T.me = me;
    for (uint32_t s : c->net.slots) T.tb[T.n++] = s;
    for (uint32_t s : c->dns.slots) T.tb[T.n++] = PV_SLOTS + s;
}

// the parameter block the exchange kernels read (tables, geometry), uploaded to d_xp
int x_params(pv_ctx *c, PvParams &P)
{
    params_common(c, P, nullptr, nullptr, 0);
    P.tcap_log2 = c->tcap_log2;
    P.reg_log2 = c->reg_log2;
    P.tkeys = c->d_tkeys;
    P.tcnt = c->d_tcnt;
    P.taux = c->d_taux;
    P.tab_live = c->d_tab_live;
    P.flags = c->d_status + ST_FLAGS;
    P.cpc = c->d_cpc;
    P.sum = c->d_sum;
    hipError_t e;
    if (!c->d_xp && !hip_ok(e = hipMalloc(&c->d_xp, sizeof(PvParams)))) return c->hipfail(e, "exchange parameters");
    if (!hip_ok(e = hipMemcpyAsync(c->d_xp, &P, sizeof P, hipMemcpyHostToDevice, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "exchange parameters");
    return 0;
}

int x_grow(pv_ctx *c, void **p, size_t &have, size_t need, const char *what)
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

// the send list on the device (d_xsend) and its layout on the host
int x_prepare(pv_ctx *c, uint32_t W, uint32_t me, XPrep &X)
{
    hipSetDevice(c->device);
    flush_fills(c);
    x_tables(c, X.T, W, me);
    X.nreg = 1u << c->reg_log2;
    X.E = 2 * X.nreg * PV_SLOTS;
    PvParams P;
    if (int rc = x_params(c, P)) return rc;
    hipError_t e;
    size_t need = (size_t)X.E * 4;
    if (int rc = x_grow(c, (void **)&c->d_xcnt, c->xcnt_bytes, need * 3, "exchange counts")) return rc;
    uint32_t *d_cnt = c->d_xcnt, *d_off = c->d_xcnt + X.E, *d_hdr = c->d_xcnt + 2 * X.E;
    if (!hip_ok(e = hipMemsetAsync(d_cnt, 0, need, c->stream))) return c->hipfail(e, "exchange counts");
    if (X.T.n) {
        hipLaunchKernelGGL(pv_topn_xcount, dim3(X.T.n * X.nreg), dim3(256), 0, c->stream, (const PvParams *)c->d_xp, X.T, d_cnt);
        if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_topn_xcount");
    }
    hipLaunchKernelGGL(pv_topn_xscan, dim3(1), dim3(1024), 0, c->stream, c->reg_log2, W, (const uint32_t *)d_cnt, d_off, d_hdr);
    X.hdr.resize(X.E);
    if (!hip_ok(e = hipGetLastError()) ||
        !hip_ok(e = hipMemcpyAsync(X.hdr.data(), d_hdr, need, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "exchange scan");
    X.dtot.assign(W, 0);
    X.dstart.assign(W + 1, 0);
    for (uint32_t d = 0; d < W; d++) {
        const uint32_t lo = x_lo_h(d, X.nreg, W), hi = x_lo_h(d + 1, X.nreg, W);
        for (uint32_t p = 2 * PV_SLOTS * lo; p < 2 * PV_SLOTS * hi; p++) X.dtot[d] += X.hdr[p];
        X.dstart[d + 1] = X.dstart[d] + X.dtot[d];
    }
    if (int rc = x_grow(c, &c->d_xsend, c->xsend_bytes, (size_t)X.dstart[W] * 16, "exchange send list")) return rc;
    if (X.T.n && X.dstart[W]) {
        hipLaunchKernelGGL(pv_topn_xwrite, dim3(X.T.n * X.nreg), dim3(256), 0, c->stream, (const PvParams *)c->d_xp, X.T,
                           (const uint32_t *)d_off, (ulonglong2 *)c->d_xsend);
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipStreamSynchronize(c->stream))) return c->hipfail(e, "exchange list");
    }
    return 0;
}

// merge the received lists (device: d_xrecv, W slots of `stride` entries; headers d_xrhdr) into
// this rank's regions
int x_merge_recv(pv_ctx *c, uint32_t W, uint32_t me, const std::vector<uint64_t> &rtot, uint64_t stride)
{
    const uint32_t nreg = 1u << c->reg_log2;
    const uint32_t lo = x_lo_h(me, nreg, W), hi = x_lo_h(me + 1, nreg, W);
    if (stride >= (1u << 24)) return c->fail(PV_ECAPACITY, "multi-GPU top-N exchange: %lu entries from one rank exceed 2^24",
                                             (unsigned long)stride);
    uint64_t total = 0;
    for (uint64_t v : rtot) total += v;
    hipError_t e;
    // the run table ([run key][column] of W columns, pv_topn_merge's layout)
    if (W > c->cb_h_grid) {
        if (c->d_cb_h) hipFree(c->d_cb_h);
        c->d_cb_h = nullptr;
        c->cb_h_grid = 0;
        if (!hip_ok(e = hipMalloc(&c->d_cb_h, (size_t)((W + 7) & ~7u) << (PV_MAX_REGIONS_LOG2 + 4)))) return c->hipfail(e, "region runs");
        c->cb_h_grid = W;
    }
    if (!total) { c->x_ranks = W; c->x_rank = me; return 0; }
    hipLaunchKernelGGL(pv_topn_xruns, dim3(W), dim3(1024), 0, c->stream, c->reg_log2, W, me, (const uint32_t *)c->d_xrhdr,
                       2 * PV_SLOTS * (hi - lo), (uint64_t *)c->d_cb_h);
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "launch pv_topn_xruns");
    PvParams P;
    params_common(c, P, nullptr, nullptr, 0);
    P.tcap_log2 = c->tcap_log2;
    P.reg_log2 = c->reg_log2;
    P.tkeys = c->d_tkeys;
    P.tcnt = c->d_tcnt;
    P.taux = c->d_taux;
    P.tab_live = c->d_tab_live;
    P.flags = c->d_status + ST_FLAGS;
    P.cpc = c->d_cpc;
    P.xmerge = 1;
    P.x_lo = lo;
    P.x_hi = hi;
    // a full region's entries go to the overflow list; the table is purged (the frequent-items
    // merge's purge, src/Metrics.h:534-538) and they are inserted again (drain_overflow)
    P.ovf = c->d_ovf;
    P.ovf_cnt = c->d_ovf_cnt;
    P.ovf_cap = c->ovf_cap;
    P.arena = c->d_arena;
    P.arena_top = c->d_arena_top;
    P.arena_cap = c->arena_cap;
    P.cb = (uint64_t *)c->d_xrecv;
    P.cb_fan = 1;
    P.mq_cap = (uint32_t)stride;
    P.cb_grid = W;
    P.cb_run = (uint64_t *)c->d_cb_h;
    P.cb_hm = c->d_cb_cnt + 32768;
    P.tp_hands = c->d_cb_cnt + 32768 + 1024; // a word holding 3: both handlers
    P.slot_of[0] = c->net.slots.empty() ? 0 : c->net.slots.front();
    P.dslot_of[0] = c->dns.slots.empty() ? 0 : c->dns.slots.front();
    if (W + 1 > 1024 + 1) return c->fail(PV_EINVAL, "%u ranks", W);
    launch_fill32(c, c->d_cb_cnt + 32768, 1024 + 1, 3u);
    launch_fill32(c, c->d_status + ST_FLAGS, 1, 0u);
    flush_fills(c);
    if (!c->d_xp && !hip_ok(e = hipMalloc(&c->d_xp, sizeof(PvParams)))) return c->hipfail(e, "exchange parameters");
    if (!hip_ok(e = hipMemcpyAsync(c->d_xp, &P, sizeof P, hipMemcpyHostToDevice, c->stream))) return c->hipfail(e, "exchange parameters");
    hipLaunchKernelGGL(pv_topn_merge, dim3(2u << c->reg_log2), dim3(pv_topn_merge_threads()), 0, c->stream, (const PvParams *)c->d_xp);
    uint32_t flags = 0;
    if (!hip_ok(e = hipGetLastError())) return c->hipfail(e, "exchange merge");
    if (int rc = drain_overflow(c, c->stream, false, nullptr, c->d_xp)) return rc;
    if (!hip_ok(e = hipMemcpyAsync(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "exchange merge");
    if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "multi-GPU top-N merge: the overflow list is full (raise table_log2)");
    for (uint32_t s : c->net.slots) c->net.clean[s] = false;
    for (uint32_t s : c->dns.slots) c->dns.clean[s] = false;
    c->x_ranks = W;
    c->x_rank = me;
    return 0;
}

// the purge offsets (frequent-items thetas) of the live tables' regions, nreg u64 per table
void x_roff_pack(pv_ctx *c, const PvXTabs &T, uint32_t nreg, std::vector<uint64_t> &o)
{
    o.assign((size_t)T.n * nreg, 0);
    for (uint32_t t = 0; t < T.n; t++)
        if (!c->roff[T.tb[t]].empty())
            for (uint32_t r = 0; r < nreg; r++) o[(size_t)t * nreg + r] = c->roff[T.tb[t]][r];
}
// add another rank's offsets of this rank's regions
void x_roff_add(pv_ctx *c, const PvXTabs &T, uint32_t nreg, uint32_t lo, uint32_t hi, const uint64_t *o)
{
    for (uint32_t t = 0; t < T.n; t++) {
        bool any = false;
        for (uint32_t r = lo; r < hi && !any; r++) any = o[(size_t)t * nreg + r] != 0;
        if (!any) continue;
        std::vector<uint64_t> &ro = c->roff[T.tb[t]];
        if (ro.empty()) ro.assign(nreg, 0);
        for (uint32_t r = lo; r < hi; r++) ro[r] += o[(size_t)t * nreg + r];
    }
}
} // namespace

// blob: magic, W, rank, ntab, nreg | tb[ntab] | roff[ntab][nreg] | dtot[W] | hdr[E] | entries
int pv_topn_x_export(pv_ctx *c, uint32_t W, uint32_t me, uint8_t **blob, size_t *bytes)
{
    *blob = nullptr;
    *bytes = 0;
    if (W < 1 || me >= W || W > 1024) return c->fail(PV_EINVAL, "rank %u of %u", me, W);
    std::lock_guard<std::mutex> g(c->mu);
    XPrep X;
    if (int rc = x_prepare(c, W, me, X)) return rc;
    std::vector<uint64_t> ro;
    x_roff_pack(c, X.T, X.nreg, ro);
    const size_t head = 20 + 4 * (size_t)X.T.n;
    const size_t n = head + ro.size() * 8 + (size_t)W * 8 + (size_t)X.E * 4 + (size_t)X.dstart[W] * 16;
    uint8_t *o = (uint8_t *)malloc(n);
    if (!o) return c->fail(PV_ECAPACITY, "exchange blob");
    const uint32_t h[5] = {X_MAGIC, W, me, X.T.n, X.nreg};
    memcpy(o, h, 20);
    memcpy(o + 20, X.T.tb, 4 * (size_t)X.T.n);
    size_t at = head;
    memcpy(o + at, ro.data(), ro.size() * 8);
    at += ro.size() * 8;
    memcpy(o + at, X.dtot.data(), (size_t)W * 8);
    at += (size_t)W * 8;
    memcpy(o + at, X.hdr.data(), (size_t)X.E * 4);
    at += (size_t)X.E * 4;
    hipError_t e;
    if (X.dstart[W] && !hip_ok(e = hipMemcpy(o + at, c->d_xsend, (size_t)X.dstart[W] * 16, hipMemcpyDeviceToHost))) {
        free(o);
        return c->hipfail(e, "exchange download");
    }
    *blob = o;
    *bytes = n;
    return 0;
}

int pv_topn_x_import(pv_ctx *c, uint32_t W, uint32_t me, const uint8_t *const *blobs, const size_t *sizes)
{
    mark_merged(c, "pv_topn_x_import");
    if (W < 1 || me >= W || W > 1024) return c->fail(PV_EINVAL, "rank %u of %u", me, W);
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    PvXTabs T;
    x_tables(c, T, W, me);
    const uint32_t nreg = 1u << c->reg_log2, E = 2 * nreg * PV_SLOTS;
    const uint32_t lo = x_lo_h(me, nreg, W), hi = x_lo_h(me + 1, nreg, W);
    struct Src { const uint64_t *ro, *dtot; const uint32_t *hdr; const uint8_t *ent; };
    std::vector<Src> src(W);
    std::vector<uint64_t> rtot(W, 0);
    uint64_t stride = 0;
    for (uint32_t q = 0; q < W; q++) {
        const uint8_t *b = blobs[q];
        uint32_t h[5];
        if (!b || sizes[q] < 20) return c->fail(PV_EINVAL, "exchange blob %u missing", q);
        memcpy(h, b, 20);
        if (h[0] != X_MAGIC || h[1] != W || h[2] != q || h[3] != T.n || h[4] != nreg || memcmp(b + 20, T.tb, 4 * (size_t)T.n))
            return c->fail(PV_EINVAL, "exchange blob %u does not match this rank's windows", q);
        size_t at = 20 + 4 * (size_t)T.n;
        // the fixed sections (region offsets, per-owner totals, counts) must lie in the blob
        // before any of them is read
        if (at + (size_t)T.n * nreg * 8 + (size_t)W * 8 + (size_t)E * 4 > sizes[q])
            return c->fail(PV_EINVAL, "exchange blob %u truncated", q);
        src[q].ro = reinterpret_cast<const uint64_t *>(b + at);
        at += (size_t)T.n * nreg * 8;
        src[q].dtot = reinterpret_cast<const uint64_t *>(b + at);
        at += (size_t)W * 8;
        src[q].hdr = reinterpret_cast<const uint32_t *>(b + at);
        at += (size_t)E * 4;
        src[q].ent = b + at;
        uint64_t all = 0;
        for (uint32_t d = 0; d < W; d++) {
            if (src[q].dtot[d] > (uint64_t)1 << 40) return c->fail(PV_EINVAL, "exchange blob %u: bad entry total", q);
            all += src[q].dtot[d];
        }
        if (at + all * 16 > sizes[q]) return c->fail(PV_EINVAL, "exchange blob %u truncated", q);
        // the counts of this rank's slice (owner me: cells [2 * PV_SLOTS * lo, 2 * PV_SLOTS * hi))
        // index the receive list on the device (pv_topn_xruns / pv_topn_merge): they must add up to
        // what the source sends this rank
        uint64_t mine = 0;
        for (size_t k = (size_t)2 * PV_SLOTS * lo; k < (size_t)2 * PV_SLOTS * hi; k++) mine += src[q].hdr[k];
        if (mine != src[q].dtot[me]) return c->fail(PV_EINVAL, "exchange blob %u: counts do not match its total", q);
        rtot[q] = q == me ? 0 : src[q].dtot[me];
        stride = std::max(stride, rtot[q]);
    }
    hipError_t e;
    const size_t hlen = (size_t)2 * PV_SLOTS * (hi - lo);
    if (int rc = x_grow(c, (void **)&c->d_xrhdr, c->xrhdr_bytes, std::max<size_t>(1, W * hlen) * 4, "exchange headers")) return rc;
    if (int rc = x_grow(c, &c->d_xrecv, c->xrecv_bytes, std::max<size_t>(1, W * stride) * 16, "exchange receive list")) return rc;
    for (uint32_t q = 0; q < W; q++) {
        if (q == me) continue;
        uint64_t before = 0;
        for (uint32_t d = 0; d < me; d++) before += src[q].dtot[d];
        if (!hip_ok(e = hipMemcpyAsync(c->d_xrhdr + (size_t)q * hlen, src[q].hdr + (size_t)2 * PV_SLOTS * lo, hlen * 4,
                                       hipMemcpyHostToDevice, c->stream)) ||
            (rtot[q] && !hip_ok(e = hipMemcpyAsync((uint8_t *)c->d_xrecv + (size_t)q * stride * 16, src[q].ent + before * 16,
                                                   rtot[q] * 16, hipMemcpyHostToDevice, c->stream))))
            return c->hipfail(e, "exchange upload");
        x_roff_add(c, T, nreg, lo, hi, src[q].ro);
    }
    return x_merge_recv(c, W, me, rtot, stride);
}

int pv_comm_merge_topn(pv_ctx *c)
{
    mark_merged(c, "pv_comm_merge_topn");
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    const uint32_t W = (uint32_t)c->comm_ranks, me = (uint32_t)c->comm_rank;
    std::lock_guard<std::mutex> g(c->mu);
    XPrep X;
    if (int rc = x_prepare(c, W, me, X)) return rc;
    const uint32_t nreg = X.nreg, lo = x_lo_h(me, nreg, W), hi = x_lo_h(me + 1, nreg, W);
    hipError_t e;
    // entries per (source, this rank), and the purge offsets: one small all-to-all / all-gather
    if (int rc = x_grow(c, (void **)&c->d_xtot, c->xtot_bytes, (size_t)W * 16, "exchange counts")) return rc;
    if (!hip_ok(e = hipMemcpyAsync(c->d_xtot, X.dtot.data(), (size_t)W * 8, hipMemcpyHostToDevice, c->stream)))
        return c->hipfail(e, "exchange counts");
    ncclResult_t r = ncclGroupStart();
    for (uint32_t q = 0; q < W && r == ncclSuccess; q++) {
        if (q == me) continue;
        r = ncclSend(c->d_xtot + q, 1, ncclUint64, (int)q, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclRecv(c->d_xtot + W + q, 1, ncclUint64, (int)q, c->comm, c->stream);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) return c->fail(PV_EHIP, "exchange counts: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    std::vector<uint64_t> rtot(W, 0);
    if (!hip_ok(e = hipMemcpyAsync(rtot.data(), c->d_xtot + W, (size_t)W * 8, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "exchange counts");
    rtot[me] = 0;
    uint64_t stride = 0;
    for (uint64_t v : rtot) stride = std::max(stride, v);
    const size_t hlen = (size_t)2 * PV_SLOTS * (hi - lo);
    if (int rc = x_grow(c, (void **)&c->d_xrhdr, c->xrhdr_bytes, std::max<size_t>(1, W * hlen) * 4, "exchange headers")) return rc;
    if (int rc = x_grow(c, &c->d_xrecv, c->xrecv_bytes, std::max<size_t>(1, W * stride) * 16, "exchange receive list")) return rc;
    const uint32_t *d_hdr = c->d_xcnt + 2 * X.E;
    r = ncclGroupStart();
    for (uint32_t q = 0; q < W && r == ncclSuccess; q++) {
        if (q == me) continue;
        const uint32_t qlo = x_lo_h(q, nreg, W), qhi = x_lo_h(q + 1, nreg, W);
        r = ncclSend(d_hdr + (size_t)2 * PV_SLOTS * qlo, (size_t)2 * PV_SLOTS * (qhi - qlo), ncclUint32, (int)q, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclRecv(c->d_xrhdr + (size_t)q * hlen, hlen, ncclUint32, (int)q, c->comm, c->stream);
        if (r == ncclSuccess && X.dtot[q])
            r = ncclSend((const uint8_t *)c->d_xsend + X.dstart[q] * 16, X.dtot[q] * 2, ncclUint64, (int)q, c->comm, c->stream);
        if (r == ncclSuccess && rtot[q])
            r = ncclRecv((uint8_t *)c->d_xrecv + (size_t)q * stride * 16, rtot[q] * 2, ncclUint64, (int)q, c->comm, c->stream);
    }
    r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) return c->fail(PV_EHIP, "exchange lists: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    // purge offsets (host blobs, a few KB)
    {
        std::vector<uint64_t> ro;
        x_roff_pack(c, X.T, nreg, ro);
        bool any = false;
        for (uint64_t v : ro) any |= v != 0;
        uint8_t anyb = any ? 1 : 0;
        // (skipped when no rank purged: one byte each first)
        std::vector<uint8_t> flags;
        if (int rc = comm_allgather_locked(c, &anyb, 1, flags)) return rc;
        bool someone = false;
        for (uint8_t f : flags) someone |= f != 0;
        if (someone) {
            std::vector<uint8_t> all;
            if (int rc = comm_allgather_locked(c, ro.data(), ro.size() * 8, all)) return rc;
            for (uint32_t q = 0; q < W; q++)
                if (q != me) x_roff_add(c, X.T, nreg, lo, hi, reinterpret_cast<const uint64_t *>(all.data() + (size_t)q * ro.size() * 8));
        }
    }
    return x_merge_recv(c, W, me, rtot, stride);
}

// ---- the merged view's lists: every owner's leading entries per metric, names from any rank
namespace {
// the text of a table entry's name record (read_topn's rules)
void x_name_text(uint32_t metric, const uint8_t *rec, uint32_t len, std::string &out)
{
    char b[64];
    if (metric == TM_IPV6 && len == 16) out = inet_ntop(AF_INET6, rec, b, sizeof b) ? b : "";
    else if (metric == TM_ECS && len == 17) out = inet_ntop(rec[0] == 1 ? AF_INET : AF_INET6, rec + 1, b, sizeof b) ? b : "";
    else out.assign((const char *)rec, len);
}
// the texts of many name records at once (pv_xname_len / pv_xname_copy): ok[i] false where aux[i]
// is 0 (no record)
int x_read_names(pv_ctx *c, const std::vector<uint32_t> &tb, const std::vector<uint32_t> &aux, const std::vector<uint64_t> &key,
                 std::vector<std::string> &out, std::vector<bool> &ok)
{
    const size_t n = tb.size();
    out.assign(n, std::string());
    ok.assign(n, false);
    if (!n) return 0;
    hipError_t e;
    uint32_t *d_tb = nullptr, *d_aux = nullptr, *d_len = nullptr;
    uint64_t *d_off = nullptr;
    uint8_t *d_out = nullptr;
    struct Free { void *p[5]; ~Free() { for (void *q : p) if (q) hipFree(q); } } fr{{nullptr, nullptr, nullptr, nullptr, nullptr}};
    if (!hip_ok(e = hipMalloc(&d_tb, n * 4)) || !hip_ok(e = hipMalloc(&d_aux, n * 4)) || !hip_ok(e = hipMalloc(&d_len, n * 4)) ||
        !hip_ok(e = hipMalloc(&d_off, n * 8)))
        return c->hipfail(e, "name gather");
    fr.p[0] = d_tb; fr.p[1] = d_aux; fr.p[2] = d_len; fr.p[3] = d_off;
    std::vector<uint32_t> len(n);
    const uint32_t g = (uint32_t)((n + 255) / 256);
    if (!hip_ok(e = hipMemcpyAsync(d_tb, tb.data(), n * 4, hipMemcpyHostToDevice, c->stream)) ||
        !hip_ok(e = hipMemcpyAsync(d_aux, aux.data(), n * 4, hipMemcpyHostToDevice, c->stream)))
        return c->hipfail(e, "name gather");
    hipLaunchKernelGGL(pv_xname_len, dim3(g), dim3(256), 0, c->stream, c->d_arena, c->arena_cap, d_tb, d_aux, (uint32_t)n, d_len);
    if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(len.data(), d_len, n * 4, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "name gather");
    std::vector<uint64_t> off(n);
    uint64_t tot = 0;
    for (size_t i = 0; i < n; i++) { off[i] = tot; tot += len[i] == 0xffffffffu ? 0 : len[i]; }
    std::vector<uint8_t> bytes(tot);
    if (tot) {
        if (!hip_ok(e = hipMalloc(&d_out, tot))) return c->hipfail(e, "name gather");
        fr.p[4] = d_out;
        if (!hip_ok(e = hipMemcpyAsync(d_off, off.data(), n * 8, hipMemcpyHostToDevice, c->stream))) return c->hipfail(e, "name gather");
        hipLaunchKernelGGL(pv_xname_copy, dim3(g), dim3(256), 0, c->stream, c->d_arena, c->arena_cap, d_tb, d_aux, d_len, d_off,
                           (uint32_t)n, d_out);
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipMemcpyAsync(bytes.data(), d_out, tot, hipMemcpyDeviceToHost, c->stream)) ||
            !hip_ok(e = hipStreamSynchronize(c->stream)))
            return c->hipfail(e, "name gather");
    }
    for (size_t i = 0; i < n; i++) {
        if (len[i] == 0xffffffffu) continue;
        x_name_text(PV_KEY_METRIC(key[i]), bytes.data() + off[i], len[i], out[i]);
        ok[i] = true;
    }
    return 0;
}
void put_u32(std::vector<uint8_t> &o, uint32_t v) { const size_t p = o.size(); o.resize(p + 4); memcpy(&o[p], &v, 4); }
void put_u64(std::vector<uint8_t> &o, uint64_t v) { const size_t p = o.size(); o.resize(p + 8); memcpy(&o[p], &v, 8); }
void put_name(std::vector<uint8_t> &o, const std::string *s)
{
    const uint16_t l = s ? (uint16_t)std::min<size_t>(s->size(), 65534) : (uint16_t)0xffff;
    const size_t p = o.size();
    o.resize(p + 2 + (s ? l : 0));
    memcpy(&o[p], &l, 2);
    if (s && l) memcpy(&o[p + 2], s->data(), l);
}
} // namespace

// The slot sets a window read asks for, per part: each live slot alone and each run of the most
// recent slots (merged windows); a set id is part << 16 | slot mask.
void x_slot_sets(pv_ctx *c, int part, std::vector<uint32_t> &v)
{
    const Window &w = part == PART_NET ? c->net : c->dns;
    v.clear();
    uint32_t m = 0;
    for (size_t i = 0; i < w.slots.size(); i++) {
        v.push_back(((uint32_t)part << 16) | (1u << w.slots[i]));
        m |= 1u << w.slots[i];
        if (i) v.push_back(((uint32_t)part << 16) | m);
    }
}

// candidates: u32 set id | u64 key | u64 estimate | u16 name length (0xffff: unknown here) | name.
// Per slot set and metric, this rank's regions' leading entries by the estimate summed over the
// set's tables (the merged window's counts).
int pv_topn_x_candidates(pv_ctx *c, uint8_t **blob, size_t *bytes)
{
    *blob = nullptr;
    *bytes = 0;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->x_ranks < 1) return c->fail(PV_EINVAL, "no multi-GPU top-N merge on this context (pv_topn_x_import / pv_comm_merge_topn)");
    hipSetDevice(c->device);
    flush_fills(c);
    const uint32_t W = c->x_ranks, me = c->x_rank, nreg = 1u << c->reg_log2, rsl = c->tcap_log2 - c->reg_log2;
    const uint32_t lo = x_lo_h(me, nreg, W), hi = x_lo_h(me + 1, nreg, W);
    const size_t K = std::max<size_t>(c->cfg.topn_count, 1);
    const size_t n = (size_t)(hi - lo) << rsl;
    std::vector<uint8_t> o;
    hipError_t e;
    // each live table's regions, read once
    struct Slice { std::vector<uint64_t> keys, cnt; std::vector<uint32_t> aux; };
    std::map<uint32_t, Slice> sl;
    auto slice = [&](uint32_t tb) -> const Slice * {
        auto it = sl.find(tb);
        if (it != sl.end()) return &it->second;
        Slice &x = sl[tb];
        const size_t base = ((size_t)tb << c->tcap_log2) + ((size_t)lo << rsl);
        x.keys.resize(n); x.cnt.resize(n); x.aux.resize(n);
        if (n && (!hip_ok(e = hipMemcpy(x.keys.data(), c->d_tkeys + base, n * 8, hipMemcpyDeviceToHost)) ||
                  !hip_ok(e = hipMemcpy(x.cnt.data(), c->d_tcnt + base, n * 8, hipMemcpyDeviceToHost)) ||
                  !hip_ok(e = hipMemcpy(x.aux.data(), c->d_taux + base, n * 4, hipMemcpyDeviceToHost))))
            return nullptr;
        return &x;
    };
    // Per part: every live slot's entries of this rank's regions, sorted by key once; then per key
    // its estimate in each slot set (single slots and the merged runs) and, per (set, metric), the
    // topn_count leading entries with the ties of the last: a first walk finds each list's
    // threshold (a bounded heap of estimates), a second collects the entries at or above it.
    struct XE { uint64_t key, est; uint32_t tb, aux; uint32_t slot; };
    struct XOut { uint32_t set; uint64_t key, est; uint32_t tb, aux; };
    std::vector<XOut> out;
    for (int part = PART_NET; part <= PART_DNS; part++) {
        std::vector<uint32_t> sets;
        x_slot_sets(c, part, sets);
        if (sets.empty()) continue;
        const Window &w = part == PART_NET ? c->net : c->dns;
        std::vector<XE> ents;
        for (uint32_t s : w.slots) {
            const uint32_t tb = s + (part == PART_DNS ? PV_SLOTS : 0);
            const Slice *x = slice(tb);
            if (!x) return c->hipfail(e, "read top-N regions");
            const std::vector<uint64_t> &roff = c->roff[tb];
            for (size_t i = 0; i < n; i++)
                if (x->keys[i])
                    ents.push_back(XE{x->keys[i], x->cnt[i] + (roff.empty() ? 0 : roff[lo + (i >> rsl)]), tb, x->aux[i], s});
        }
        std::sort(ents.begin(), ents.end(), [](const XE &p1, const XE &p2) { return p1.key < p2.key; });
        const size_t NZ = sets.size();
        // per key group [g0, g1): the estimate in set z, and whether the set holds the key
        auto group_est = [&](size_t g0, size_t g1, size_t z, uint64_t &est) {
            bool in = false;
            est = 0;
            for (size_t j = g0; j < g1; j++)
                if ((sets[z] >> ents[j].slot) & 1) { est += ents[j].est; in = true; }
            return in;
        };
        // walk 1: thresholds (a min-heap of the K largest estimates per (set, metric))
        std::map<std::pair<uint32_t, uint32_t>, std::priority_queue<uint64_t, std::vector<uint64_t>, std::greater<uint64_t>>> heaps;
        for (size_t g0 = 0, g1; g0 < ents.size(); g0 = g1) {
            g1 = g0 + 1;
            while (g1 < ents.size() && ents[g1].key == ents[g0].key) g1++;
            const uint32_t hm = host_metric(c, ents[g0].key);
            for (size_t z = 0; z < NZ; z++) {
                uint64_t est;
                if (!group_est(g0, g1, z, est)) continue;
                auto &h = heaps[{(uint32_t)z, hm}];
                if (h.size() < K) h.push(est);
                else if (est > h.top()) { h.pop(); h.push(est); }
            }
        }
        std::map<std::pair<uint32_t, uint32_t>, uint64_t> thr;
        for (auto &kv : heaps) thr[kv.first] = kv.second.size() < K ? 0 : kv.second.top();
        // walk 2: entries at or above the threshold (est, key, name table, name aux)
        std::map<std::pair<uint32_t, uint32_t>, std::vector<std::tuple<uint64_t, uint64_t, uint32_t, uint32_t>>> got;
        for (size_t g0 = 0, g1; g0 < ents.size(); g0 = g1) {
            g1 = g0 + 1;
            while (g1 < ents.size() && ents[g1].key == ents[g0].key) g1++;
            const uint32_t hm = host_metric(c, ents[g0].key);
            for (size_t z = 0; z < NZ; z++) {
                uint64_t est;
                if (!group_est(g0, g1, z, est)) continue;
                if (est < thr[{(uint32_t)z, hm}]) continue;
                uint32_t ntb = 0, naux = 0;
                for (size_t j = g0; j < g1 && !naux; j++)
                    if (((sets[z] >> ents[j].slot) & 1) && ents[j].aux) { ntb = ents[j].tb; naux = ents[j].aux; }
                auto &v = got[{(uint32_t)z, hm}];
                v.emplace_back(est, ents[g0].key, ntb, naux);
                if (v.size() > 4 * (PV_X_TIES + K)) {
                    // a flat list: keep the leading ones by (estimate desc, key asc)
                    auto cmp = [](const auto &a1, const auto &b1) {
                        return std::get<0>(a1) != std::get<0>(b1) ? std::get<0>(a1) > std::get<0>(b1) : std::get<1>(a1) < std::get<1>(b1);
                    };
                    std::nth_element(v.begin(), v.begin() + (PV_X_TIES + K), v.end(), cmp);
                    v.resize(PV_X_TIES + K);
                }
            }
        }
        for (size_t z = 0; z < NZ; z++) {
            for (auto it = got.lower_bound({(uint32_t)z, 0u}); it != got.end() && it->first.first == z; ++it) {
                auto &v = it->second;
                std::sort(v.begin(), v.end(), [](const auto &a1, const auto &b1) {
                    return std::get<0>(a1) != std::get<0>(b1) ? std::get<0>(a1) > std::get<0>(b1) : std::get<1>(a1) < std::get<1>(b1);
                });
                // the topn_count leading entries and every entry tied with the last of them (the lists
                // order ties by name, which only the whole tied group decides; at most PV_X_TIES)
                size_t m = std::min(K, v.size());
                while (m < v.size() && m < PV_X_TIES && std::get<0>(v[m]) == std::get<0>(v[m - 1])) m++;
                for (size_t k = 0; k < m; k++) out.push_back(XOut{sets[z], std::get<1>(v[k]), std::get<0>(v[k]), std::get<2>(v[k]), std::get<3>(v[k])});
            }
        }
    }
    // the names: IPv4 from the key, the others gathered from the arena in one pass
    {
        std::vector<uint32_t> gtb, gaux;
        std::vector<uint64_t> gkey;
        std::vector<size_t> at;
        for (size_t i = 0; i < out.size(); i++)
            if (PV_KEY_METRIC(out[i].key) != TM_IPV4 && out[i].aux) {
                gtb.push_back(out[i].tb); gaux.push_back(out[i].aux); gkey.push_back(out[i].key); at.push_back(i);
            }
        std::vector<std::string> txt;
        std::vector<bool> okv;
        if (int rc = x_read_names(c, gtb, gaux, gkey, txt, okv)) return rc;
        std::vector<const std::string *> nmp(out.size(), nullptr);
        for (size_t j = 0; j < at.size(); j++) if (okv[j]) nmp[at[j]] = &txt[j];
        for (size_t i = 0; i < out.size(); i++) {
            const uint64_t key = out[i].key;
            put_u32(o, out[i].set);
            put_u64(o, key);
            put_u64(o, out[i].est);
            if (PV_KEY_METRIC(key) == TM_IPV4) {
                const uint32_t ip = (uint32_t)key;
                char bb[20];
                snprintf(bb, sizeof bb, "%u.%u.%u.%u", ip & 0xff, (ip >> 8) & 0xff, (ip >> 16) & 0xff, ip >> 24);
                const std::string nm = bb;
                put_name(o, &nm);
            } else {
                put_name(o, nmp[i]);
            }
        }
    }
    *blob = (uint8_t *)malloc(std::max<size_t>(o.size(), 1));
    if (!*blob) return c->fail(PV_ECAPACITY, "candidates");
    memcpy(*blob, o.data(), o.size());
    *bytes = o.size();
    return 0;
}

namespace {
struct XCand {
    uint32_t tb;
    uint64_t key, est;
    bool named;
    std::string name;
};
bool x_parse_cands(const uint8_t *b, size_t n, std::vector<XCand> &out)
{
    size_t p = 0;
    while (p < n) {
        if (p + 22 > n) return false;
        XCand x;
        uint16_t l;
        memcpy(&x.tb, b + p, 4);
        memcpy(&x.key, b + p + 4, 8);
        memcpy(&x.est, b + p + 12, 8);
        memcpy(&l, b + p + 20, 2);
        p += 22;
        x.named = l != 0xffff;
        if (x.named) {
            if (p + l > n) return false;
            x.name.assign((const char *)b + p, l);
            p += l;
        }
        out.push_back(std::move(x));
    }
    return true;
}
} // namespace

// answers: the names this rank holds for candidates (of every rank) that came without one:
// u32 tb | u64 key | u16 length | name
int pv_topn_x_names(pv_ctx *c, const uint8_t *const *cands, const size_t *sizes, uint32_t n, uint8_t **blob, size_t *bytes)
{
    *blob = nullptr;
    *bytes = 0;
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    std::vector<XCand> want;
    for (uint32_t q = 0; q < n; q++) {
        std::vector<XCand> v;
        if (!x_parse_cands(cands[q], sizes[q], v)) return c->fail(PV_EINVAL, "malformed candidate blob %u", q);
        for (auto &x : v)
            if (!x.named) want.push_back(x);
    }
    std::vector<uint8_t> o;
    // each wanted key against every live table of its set's part (a rank may hold it in any period)
    {
        std::vector<XCand> w2;
        for (auto &x : want) {
            const int part = (int)(x.tb >> 16);
            for (uint32_t s : (part == PART_DNS ? c->dns.slots : c->net.slots)) {
                XCand y = x;
                y.tb = s + (part == PART_DNS ? PV_SLOTS : 0);
                y.name = std::to_string(x.tb); // (the set id, for the answer)
                w2.push_back(y);
            }
        }
        want.swap(w2);
    }
    if (!want.empty()) {
        std::vector<uint64_t> keys;
        std::vector<uint32_t> tbs;
        for (auto &x : want) { keys.push_back(x.key); tbs.push_back(x.tb); }
        PvParams P;
        if (int rc = x_params(c, P)) return rc;
        uint64_t *d_k = nullptr;
        uint32_t *d_t = nullptr, *d_a = nullptr;
        hipError_t e;
        std::vector<uint32_t> aux(want.size());
        if (!hip_ok(e = hipMalloc(&d_k, keys.size() * 8)) || !hip_ok(e = hipMalloc(&d_t, keys.size() * 4)) ||
            !hip_ok(e = hipMalloc(&d_a, keys.size() * 4))) {
            hipFree(d_k); hipFree(d_t); hipFree(d_a);
            return c->hipfail(e, "name lookup");
        }
        bool ok = hip_ok(e = hipMemcpy(d_k, keys.data(), keys.size() * 8, hipMemcpyHostToDevice)) &&
                  hip_ok(e = hipMemcpy(d_t, tbs.data(), tbs.size() * 4, hipMemcpyHostToDevice));
        if (ok) {
            hipLaunchKernelGGL(pv_topn_xlookup, dim3((uint32_t)((keys.size() + 255) / 256)), dim3(256), 0, c->stream,
                               (const PvParams *)c->d_xp, (const uint64_t *)d_k, (const uint32_t *)d_t, (uint32_t)keys.size(), d_a);
            ok = hip_ok(e = hipGetLastError()) && hip_ok(e = hipStreamSynchronize(c->stream)) &&
                 hip_ok(e = hipMemcpy(aux.data(), d_a, aux.size() * 4, hipMemcpyDeviceToHost));
        }
        hipFree(d_k); hipFree(d_t); hipFree(d_a);
        if (!ok) return c->hipfail(e, "name lookup");
        std::vector<uint32_t> gtb, gaux;
        std::vector<uint64_t> gkey;
        for (size_t i = 0; i < want.size(); i++) { gtb.push_back(want[i].tb); gaux.push_back(aux[i]); gkey.push_back(want[i].key); }
        std::vector<std::string> txt;
        std::vector<bool> okv;
        if (int rc = x_read_names(c, gtb, gaux, gkey, txt, okv)) return rc;
        std::set<std::pair<uint32_t, uint64_t>> done;
        for (size_t i = 0; i < want.size(); i++) {
            const uint32_t set = (uint32_t)std::stoul(want[i].name);
            if (done.count({set, want[i].key}) || !okv[i]) continue;
            done.insert({set, want[i].key});
            put_u32(o, set);
            put_u64(o, want[i].key);
            put_name(o, &txt[i]);
        }
    }
    *blob = (uint8_t *)malloc(std::max<size_t>(o.size(), 1));
    if (!*blob) return c->fail(PV_ECAPACITY, "name answers");
    memcpy(*blob, o.data(), o.size());
    *bytes = o.size();
    return 0;
}

int pv_topn_x_view(pv_ctx *c, const uint8_t *const *cands, const size_t *csizes, const uint8_t *const *names,
                   const size_t *nsizes, uint32_t n)
{
    mark_merged(c, "pv_topn_x_view");
    std::lock_guard<std::mutex> g(c->mu);
    std::map<std::pair<uint32_t, uint64_t>, std::string> known;
    for (uint32_t q = 0; q < n; q++) {
        const uint8_t *b = names[q];
        size_t p = 0, m = nsizes[q];
        while (p + 14 <= m) {
            uint32_t tb; uint64_t key; uint16_t l;
            memcpy(&tb, b + p, 4); memcpy(&key, b + p + 4, 8); memcpy(&l, b + p + 12, 2);
            if (l == 0xffff || p + 14 + l > m) return c->fail(PV_EINVAL, "malformed name blob %u", q);
            known[{tb, key}].assign((const char *)b + p + 14, l);
            p += 14 + l;
        }
    }
    c->x_view.clear();
    for (uint32_t q = 0; q < n; q++) {
        std::vector<XCand> v;
        if (!x_parse_cands(cands[q], csizes[q], v)) return c->fail(PV_EINVAL, "malformed candidate blob %u", q);
        for (auto &x : v) {
            std::string nm = x.name;
            if (!x.named) {
                auto it = known.find({x.tb, x.key});
                if (it != known.end()) nm = it->second;
            }
            c->x_view[x.tb][x.key] = {x.est, nm};
        }
    }
    c->x_view_on = true;
    return 0;
}

// ---- quantile inputs across shards without shipping the values: exact radix selection whose
// per-pass group histograms (256 bins, one byte of the value) are summed over the ranks by a
// caller-supplied all-reduce (pv_values_x_select) or RCCL (pv_comm_values_select). Per live DNS
// slot and value kind: the count, p50/p90/p95/p99 and the maximum (the KLL inclusive rank rule
// of Quantile, src/Metrics.h:334-481, on the union of the shards' values: what one stream
// gives) and, for the time kinds, the count at or below each histogram point (Histogram,
// src/Metrics.h:189-327). The merged view then holds a stand-in value list per slot and kind
// with those counts, that maximum and those quantiles.
namespace {
int x_allreduce(pv_ctx *c, pv_allreduce_fn ar, void *user, std::vector<uint64_t> &buf, int op)
{
    if (buf.empty()) return 0;
    if (ar) return ar(buf.data(), buf.size(), op, user) ? c->fail(PV_EINVAL, "all-reduce callback failed") : 0;
    // RCCL on the context's communicator
    hipError_t e;
    uint64_t *d = nullptr;
    if (!hip_ok(e = hipMalloc(&d, buf.size() * 8))) return c->hipfail(e, "selection all-reduce");
    ncclResult_t r = ncclSuccess;
    const bool ok = hip_ok(e = hipMemcpyAsync(d, buf.data(), buf.size() * 8, hipMemcpyHostToDevice, c->stream)) &&
                    (r = ncclAllReduce(d, d, buf.size(), ncclUint64, op ? ncclMax : ncclSum, c->comm, c->stream)) == ncclSuccess &&
                    hip_ok(e = hipMemcpyAsync(buf.data(), d, buf.size() * 8, hipMemcpyDeviceToHost, c->stream)) &&
                    hip_ok(e = hipStreamSynchronize(c->stream));
    hipFree(d);
    if (r != ncclSuccess) return c->fail(PV_EHIP, "ncclAllReduce: %s", ncclGetErrorString(r));
    if (!ok) return c->hipfail(e, "selection all-reduce");
    return 0;
}
// rank of fraction p among n values (quantiles(): ceil(p n) - 1, clamped); p > 1: the maximum
uint64_t x_rank_of(double p, uint64_t n)
{
    if (p > 1.0) return n ? n - 1 : 0;
    const uint64_t w = (uint64_t)std::ceil(p * (double)n);
    uint64_t idx = w == 0 ? 0 : w - 1;
    return n && idx >= n ? n - 1 : idx;
}
// Exact distributed selection. gparts[g]: this rank's values of group g, as sorted parts (a
// value lies in one part); fr[g]: the fractions wanted. out[g][k]: the value at each fraction's
// rank over every rank's values (0 when the group is empty everywhere); n[g]: the group's count
// over every rank. Eight passes, one byte each from the top: per target the 256-bin histogram of
// the values whose higher bytes equal the target's prefix so far, all-reduced (one call per
// pass), then the bin holding the target's rank. The bins are counted by binary searches over the
// sorted parts (257 bin edges per part), so a pass costs O(targets x parts x 256 log n), not a
// scan of every value per target.
using XParts = std::vector<const std::vector<uint64_t> *>;
int x_select(pv_ctx *c, pv_allreduce_fn ar, void *user, const std::vector<XParts> &gparts,
             const std::vector<std::vector<double>> &fr, std::vector<uint64_t> &n, std::vector<std::vector<uint64_t>> &out)
{
    const size_t G = gparts.size();
    struct Tg { uint32_t g; double p; uint64_t rank, prefix; };
    std::vector<Tg> T;
    for (uint32_t g = 0; g < G; g++)
        for (double p : fr[g]) T.push_back(Tg{g, p, 0, 0});
    n.assign(G, 0);
    out.assign(G, {});
    // values <= x in a group's parts
    auto count_le = [&](const XParts &ps, uint64_t x) {
        uint64_t k = 0;
        for (const std::vector<uint64_t> *v : ps) k += (uint64_t)(std::upper_bound(v->begin(), v->end(), x) - v->begin());
        return k;
    };
    std::vector<uint64_t> h;
    for (int pass = 0; pass < 8; pass++) {
        const uint32_t shift = 56 - 8 * pass;
        h.assign(T.size() * 256, 0);
        std::map<std::pair<uint32_t, uint64_t>, size_t> done; // (group, range) -> target that counted it
        for (size_t t = 0; t < T.size(); t++) {
            const XParts &ps = gparts[T[t].g];
            // the target's range: its prefix above this byte, every value of the lower bytes
            const uint64_t base = pass == 0 ? 0ull : T[t].prefix & (~0ull << (shift + 8));
            auto it = done.find({T[t].g, base});
            if (it != done.end()) {
                std::copy(h.begin() + it->second * 256, h.begin() + it->second * 256 + 256, h.begin() + t * 256);
                continue;
            }
            done[{T[t].g, base}] = t;
            uint64_t below = base ? count_le(ps, base - 1) : 0;
            for (uint32_t bn = 0; bn < 256; bn++) {
                const uint64_t top = base + ((uint64_t)bn << shift) + ((1ull << shift) - 1);
                const uint64_t le = count_le(ps, top);
                h[t * 256 + bn] = le - below;
                below = le;
            }
        }
        if (int rc = x_allreduce(c, ar, user, h, 0)) return rc;
        for (size_t t = 0; t < T.size(); t++) {
            const uint64_t *hh = &h[t * 256];
            if (pass == 0) {
                uint64_t tot = 0;
                for (int b = 0; b < 256; b++) tot += hh[b];
                n[T[t].g] = tot;
                T[t].rank = x_rank_of(T[t].p, tot);
            }
            if (!n[T[t].g]) continue;
            uint64_t cum = 0;
            int b = 0;
            while (b < 255 && cum + hh[b] <= T[t].rank) cum += hh[b++];
            T[t].rank -= cum;
            T[t].prefix |= (uint64_t)b << shift;
        }
    }
    for (auto &t : T) out[t.g].push_back(n[t.g] ? t.prefix : 0);
    return 0;
}
const uint32_t X_KINDS[9] = {XV_FROM_US, XV_TO_US, XV_RATIO, XV2_TIME, XV2_TIME + 1, XV2_TIME + 2, XV2_RATIO, XV2_RATIO + 1, XV2_RATIO + 2};
bool x_time_kind(uint32_t k) { return k == XV_FROM_US || k == XV_TO_US || (k >= XV2_TIME && k < XV2_TIME + 3); }

int values_select(pv_ctx *c, pv_allreduce_fn ar, void *user)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (int rc = sync_xvals(c)) return rc;
    // groups: (slot set, kind), the sets a window read can ask for: each live DNS slot alone
    // (window_json of one period) and each run of the most recent slots (merged windows)
    std::vector<uint32_t> sets;
    for (uint32_t s : c->dns.slots) sets.push_back(1u << s);
    {
        uint32_t m = 0;
        for (size_t i = 0; i < c->dns.slots.size(); i++) {
            m |= 1u << c->dns.slots[i];
            if (i) sets.push_back(m);
        }
    }
    const size_t G = sets.size() * 9;
    std::vector<std::vector<double>> fr(G, std::vector<double>{0.50, 0.90, 0.95, 0.99, 2.0});
    // the values by (live slot, kind), each sorted once; a group (slot set, kind) is the parts of
    // its slots
    std::map<uint32_t, uint32_t> sg_idx; // live slot | gen << 8 -> its index among the live slots
    for (size_t i = 0; i < c->dns.slots.size(); i++) sg_idx[c->dns.slots[i] | (c->gen[c->dns.slots[i]] << 8)] = (uint32_t)i;
    const size_t NS = c->dns.slots.size();
    std::vector<std::vector<uint64_t>> part(NS * 9);
    for (const PvXValue &v : c->xvals_host) {
        auto it = sg_idx.find(v.slot);
        if (it == sg_idx.end()) continue;
        int k = 0;
        while (k < 9 && v.kind != X_KINDS[k]) k++;
        if (k == 9) continue;
        part[(size_t)it->second * 9 + k].push_back(v.bits);
    }
    for (auto &v : part) std::sort(v.begin(), v.end());
    std::vector<XParts> groups(G);
    for (size_t i = 0; i < sets.size(); i++)
        for (size_t si = 0; si < NS; si++)
            if (sets[i] & (1u << c->dns.slots[si]))
                for (int k = 0; k < 9; k++) groups[i * 9 + k].push_back(&part[si * 9 + k]);
    std::vector<uint64_t> n;
    std::vector<std::vector<uint64_t>> q;
    if (int rc = x_select(c, ar, user, groups, fr, n, q)) return rc;
    // counts at or below each histogram point, time kinds
    const std::vector<uint64_t> &pts = hist_points();
    std::vector<uint64_t> cdf(G * pts.size(), 0);
    for (size_t gi = 0; gi < G; gi++) {
        if (!x_time_kind(X_KINDS[gi % 9])) continue;
        for (size_t k = 0; k < pts.size(); k++)
            for (const std::vector<uint64_t> *v : groups[gi])
                cdf[gi * pts.size() + k] += (uint64_t)(std::upper_bound(v->begin(), v->end(), pts[k]) - v->begin());
    }
    if (int rc = x_allreduce(c, ar, user, cdf, 0)) return rc;
    c->xq.clear();
    for (size_t gi = 0; gi < G; gi++) {
        if (!n[gi]) continue;
        XQuant &x = c->xq[{sets[gi / 9], X_KINDS[gi % 9]}];
        x.n = n[gi];
        x.q.assign(q[gi].begin(), q[gi].begin() + 4);
        x.max = q[gi][4];
        if (x_time_kind(X_KINDS[gi % 9])) x.cdf.assign(cdf.begin() + gi * pts.size(), cdf.begin() + (gi + 1) * pts.size());
    }
    c->xq_on = true;
    return 0;
}
} // namespace

int pv_values_x_select(pv_ctx *c, pv_allreduce_fn ar, void *user)
{
    mark_merged(c, "pv_values_x_select");
    if (!ar) return c->fail(PV_EINVAL, "no all-reduce callback");
    return values_select(c, ar, user);
}

int pv_comm_values_select(pv_ctx *c)
{
    mark_merged(c, "pv_comm_values_select");
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    return values_select(c, nullptr, nullptr);
}

// The device regions of both live windows a multi-GPU reduce combines: each Net slot's
// net part and each DNS slot's dns part of the SUM (all-reduce SUM) and MIN (all-reduce MIN)
// words. The caller writes them, so they stop being clean.
int pv_window_regions(pv_ctx *c, pv_region *r, uint32_t max, uint32_t *n)
{
    mark_merged(c, "pv_window_regions");
    std::lock_guard<std::mutex> g(c->mu);
    flush_fills(c);
    std::vector<pv_region> v;
    // the parts of each slot the attached handler versions use (the others stay zero)
    auto sum = [&](uint32_t s, size_t a, size_t b) { v.push_back(pv_region{c->d_sum + (size_t)s * PV_SUM_WORDS + a, b - a, PV_REDUCE_SUM, 0}); };
    auto cpc = [&](uint32_t s, size_t k0, size_t k1) {
        v.push_back(pv_region{c->d_cpc + (size_t)s * PV_MIN_WORDS + k0 * PV_CPC_COUPONS, (k1 - k0) * PV_CPC_COUPONS,
                              PV_REDUCE_MIN, 0});
    };
    for (uint32_t s : c->net.slots) {
        sum(s, 0, PV_OFF_NET2);
        cpc(s, CPC_SRC, CPC_V2);
        if (c->net2_groups) { sum(s, PV_OFF_NET2, PV_SUM_NET_WORDS); cpc(s, CPC_V2, CPC_QNAME); }
        c->net.clean[s] = false;
    }
    for (uint32_t s : c->dns.slots) {
        if (c->dns2_groups) {
            sum(s, PV_OFF_DNS, PV_OFF_DNS + PV_DNS_CTRS);
            sum(s, PV_OFF_DNS2, PV_SUM_WORDS);
            cpc(s, CPC_QNAME2, CPC_QNAME2 + 3);
        } else {
            sum(s, PV_OFF_DNS, PV_OFF_DNS2);
            cpc(s, CPC_QNAME, CPC_QNAME + 1);
        }
        c->dns.clean[s] = false;
    }
    *n = (uint32_t)v.size();
    for (uint32_t i = 0; i < v.size() && i < max; i++) r[i] = v[i];
    return 0;
}

int pv_comm_unique_id(uint8_t id[PV_COMM_ID_BYTES])
{
    static_assert(sizeof(ncclUniqueId) == PV_COMM_ID_BYTES, "unique id size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return PV_EHIP;
    memcpy(id, &u, sizeof u);
    return 0;
}

int pv_comm_init(pv_ctx *c, const uint8_t id[PV_COMM_ID_BYTES], int nranks, int rank)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (c->comm) return c->fail(PV_EINVAL, "communicator already initialised");
    if (nranks < 1 || rank < 0 || rank >= nranks) return c->fail(PV_EINVAL, "rank %d of %d", rank, nranks);
    hipSetDevice(c->device);
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        return c->fail(PV_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    c->comm_ranks = nranks;
    c->comm_rank = rank;
    return 0;
}

int pv_comm_allreduce_window(pv_ctx *c)
{
    mark_merged(c, "pv_comm_allreduce_window");
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    std::vector<pv_region> v(8 * PV_SLOTS);
    uint32_t n = 0;
    if (int rc = pv_window_regions(c, v.data(), (uint32_t)v.size(), &n)) return rc;
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    flush_fills(c);
    ncclResult_t r = ncclGroupStart();
    for (uint32_t i = 0; i < n && r == ncclSuccess; i++)
        r = ncclAllReduce(v[i].ptr, v[i].ptr, v[i].words, v[i].op == PV_REDUCE_SUM ? ncclUint64 : ncclInt64,
                          v[i].op == PV_REDUCE_SUM ? ncclSum : ncclMin, c->comm, c->stream);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) return c->fail(PV_EHIP, "ncclAllReduce: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    hipError_t e;
    if (!hip_ok(e = hipStreamSynchronize(c->stream))) return c->hipfail(e, "window all-reduce");
    return 0;
}

// all-gather of one equal-sized host block per rank (the caller holds c->mu)
int comm_allgather_locked(pv_ctx *c, const void *buf, size_t bytes, std::vector<uint8_t> &out)
{
    const int R = c->comm_ranks;
    out.assign((size_t)R * bytes, 0);
    if (!bytes) return 0;
    hipError_t e;
    uint8_t *d = nullptr;
    if (!hip_ok(e = hipMalloc(&d, bytes * (R + 1)))) return c->hipfail(e, "all-gather buffers");
    ncclResult_t r = ncclSuccess;
    bool ok = hip_ok(e = hipMemcpyAsync(d + bytes * R, buf, bytes, hipMemcpyHostToDevice, c->stream)) &&
              (r = ncclAllGather(d + bytes * R, d, bytes, ncclUint8, c->comm, c->stream)) == ncclSuccess &&
              hip_ok(e = hipMemcpyAsync(out.data(), d, bytes * R, hipMemcpyDeviceToHost, c->stream)) &&
              hip_ok(e = hipStreamSynchronize(c->stream));
    hipFree(d);
    if (r != ncclSuccess) return c->fail(PV_EHIP, "ncclAllGather: %s", ncclGetErrorString(r));
    if (!ok) return c->hipfail(e, "all-gather");
    return 0;
}

int pv_comm_allgather(pv_ctx *c, const void *buf, size_t bytes, uint8_t **out, uint64_t *sizes)
{
    *out = nullptr;
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    const int R = c->comm_ranks;
    hipError_t e;
    uint64_t *d_sz = nullptr;
    uint8_t *d_in = nullptr, *d_all = nullptr;
    struct Free {
        void *a, *b, *c;
        ~Free() { for (void *p : {a, b, c}) if (p) hipFree(p); }
    } fr{nullptr, nullptr, nullptr};
    if (!hip_ok(e = hipMalloc(&d_sz, (size_t)R * 16))) return c->hipfail(e, "all-gather sizes");
    fr.a = d_sz;
    const uint64_t mine = bytes;
    if (!hip_ok(e = hipMemcpyAsync(d_sz + R, &mine, 8, hipMemcpyHostToDevice, c->stream))) return c->hipfail(e, "all-gather sizes");
    ncclResult_t r = ncclAllGather(d_sz + R, d_sz, 1, ncclUint64, c->comm, c->stream);
    if (r != ncclSuccess) return c->fail(PV_EHIP, "ncclAllGather: %s", ncclGetErrorString(r));
    if (!hip_ok(e = hipMemcpyAsync(sizes, d_sz, (size_t)R * 8, hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "all-gather sizes");
    uint64_t mx = 0, tot = 0;
    for (int k = 0; k < R; k++) { mx = std::max(mx, sizes[k]); tot += sizes[k]; }
    const size_t chunk = (size_t)std::max<uint64_t>(mx, 1);
    if (!hip_ok(e = hipMalloc(&d_in, chunk)) || !hip_ok(e = hipMalloc(&d_all, chunk * R))) return c->hipfail(e, "all-gather buffers");
    fr.b = d_in;
    fr.c = d_all;
    if (bytes && !hip_ok(e = hipMemcpyAsync(d_in, buf, bytes, hipMemcpyHostToDevice, c->stream))) return c->hipfail(e, "all-gather upload");
    r = ncclAllGather(d_in, d_all, chunk, ncclUint8, c->comm, c->stream);
    if (r != ncclSuccess) return c->fail(PV_EHIP, "ncclAllGather: %s", ncclGetErrorString(r));
    std::vector<uint8_t> all(chunk * R);
    if (!hip_ok(e = hipMemcpyAsync(all.data(), d_all, all.size(), hipMemcpyDeviceToHost, c->stream)) ||
        !hip_ok(e = hipStreamSynchronize(c->stream)))
        return c->hipfail(e, "all-gather download");
    uint8_t *o = (uint8_t *)malloc(std::max<uint64_t>(tot, 1));
    if (!o) return c->fail(PV_ECAPACITY, "all-gather result");
    uint64_t at = 0;
    for (int k = 0; k < R; k++) { memcpy(o + at, all.data() + (size_t)k * chunk, sizes[k]); at += sizes[k]; }
    *out = o;
    return 0;
}

int pv_comm_destroy(pv_ctx *c)
{
    if (!c->comm) return 0;
    ncclCommDestroy(c->comm);
    c->comm = nullptr;
    return 0;
}

int pv_set_kernel_timing(pv_ctx *c, uint32_t every)
{
    c->timing_every = every;
    c->timing_ctr = 0;
    return 0;
}

int pv_kernel_timing(pv_ctx *c, double *total_ms, uint64_t *launches, int reset)
{
    *total_ms = c->kernel_ms;
    *launches = c->kernel_launches;
    if (reset) { c->kernel_ms = 0; c->kernel_launches = 0; }
    return 0;
}

// ---- multi-GPU shard edges: DNS transactions across contiguous shards.
// Each rank exports its shard-edge stubs: the queries still open at the end of its
// stream (latest per (flow, txid)), its orphan responses (first event of their key in
// its stream) and its DNS period shifts. Every rank then replays the ranks before it:
// the open queries of shard j that shards j+1 .. r-1 neither answered nor purged reach
// shard r, where they pair with r's orphan responses (TransactionManager::
// maybe_end_transaction, libs/visor_transaction/TransactionManager.h:51-106) or time out
// at r's period shifts (DnsStreamHandler.h:252-267). Each rank counts only what happens
// in its own shard, into its own buckets, before the bucket all-reduce.
namespace {
struct EdgeHdr {
    uint32_t magic, n_open, n_orph, n_shift;
};
const uint32_t EDGE_MAGIC = 0x31455650u; // "PVE1"
struct EdgeView {
    std::vector<PvXEvent> open, orph;
    std::vector<std::pair<int64_t, uint32_t>> shifts;
};
bool edge_parse(const uint8_t *b, size_t n, EdgeView &v)
{
    EdgeHdr h;
    if (n < sizeof h) return false;
    memcpy(&h, b, sizeof h);
    const size_t need = sizeof h + ((size_t)h.n_open + h.n_orph) * sizeof(PvXEvent) + (size_t)h.n_shift * 12;
    if (h.magic != EDGE_MAGIC || n != need) return false;
    const uint8_t *p = b + sizeof h;
    v.open.resize(h.n_open);
    v.orph.resize(h.n_orph);
    if (h.n_open) memcpy(v.open.data(), p, h.n_open * sizeof(PvXEvent));
    p += h.n_open * sizeof(PvXEvent);
    if (h.n_orph) memcpy(v.orph.data(), p, h.n_orph * sizeof(PvXEvent));
    p += h.n_orph * sizeof(PvXEvent);
    v.shifts.resize(h.n_shift);
    for (uint32_t i = 0; i < h.n_shift; i++) {
        memcpy(&v.shifts[i].first, p + 12 * i, 8);
        memcpy(&v.shifts[i].second, p + 12 * i + 8, 4);
    }
    return true;
}
// first shift of `sh` at or after ttl + sec (the purge of a query started at sec), or -1
int purge_shift(const std::vector<std::pair<int64_t, uint32_t>> &sh, uint32_t ttl_s, int64_t sec)
{
    for (size_t i = 0; i < sh.size(); i++)
        if (sh[i].first >= (int64_t)ttl_s + sec) return (int)i;
    return -1;
}
int add_dns_words(pv_ctx *c, uint32_t slot, const uint64_t add[4])
{
    static const int w[4] = {DC_XTOTAL, DC_XOUT, DC_XIN, DC_XTIMEOUT};
    c->dns.clean[slot] = false;
    for (int k = 0; k < 4; k++) {
        if (!add[k]) continue;
        uint64_t *dp = c->d_sum + (size_t)slot * PV_SUM_WORDS + PV_OFF_DNS + w[k];
        uint64_t v = 0;
        hipError_t e;
        if (!hip_ok(e = hipMemcpy(&v, dp, 8, hipMemcpyDeviceToHost))) return c->hipfail(e, "edge counters");
        v += add[k];
        if (!hip_ok(e = hipMemcpy(dp, &v, 8, hipMemcpyHostToDevice))) return c->hipfail(e, "edge counters");
    }
    return 0;
}
bool in_dns_window(pv_ctx *c, uint32_t slot)
{
    return std::find(c->dns.slots.begin(), c->dns.slots.end(), slot) != c->dns.slots.end();
}
// the carried list on the host: each open query event (gathered from the event store by its
// index) with its sort key
int read_carried(pv_ctx *c, std::vector<PvXEvent> &pend, std::vector<uint64_t> &pk, std::vector<uint64_t> *ecs = nullptr)
{
    pend.clear();
    pk.assign(c->n_pend, 0);
    if (ecs) ecs->assign(c->n_pend, 0);
    if (!c->n_pend) return 0;
    std::vector<uint32_t> pv(c->n_pend);
    std::vector<PvXEvent> store(c->pend_hi);
    std::vector<uint64_t> estore(ecs && c->d_pecs[c->pend_cur] ? c->pend_hi : 0);
    hipError_t e;
    if (!hip_ok(e = hipMemcpy(pk.data(), c->d_pkeys[c->pend_cur], c->n_pend * 8, hipMemcpyDeviceToHost)) ||
        !hip_ok(e = hipMemcpy(pv.data(), c->d_pvals[c->pend_cur], c->n_pend * 4, hipMemcpyDeviceToHost)) ||
        !hip_ok(e = hipMemcpy(store.data(), c->d_pend[c->pend_cur], c->pend_hi * sizeof(PvXEvent), hipMemcpyDeviceToHost)) ||
        (!estore.empty() && !hip_ok(e = hipMemcpy(estore.data(), c->d_pecs[c->pend_cur], c->pend_hi * 8, hipMemcpyDeviceToHost))))
        return c->hipfail(e, "open queries");
    pend.resize(c->n_pend);
    for (size_t i = 0; i < pv.size(); i++) {
        if (pv[i] >= c->pend_hi) return c->fail(PV_EINVAL, "carried query %zu indexes past the event store", i);
        pend[i] = store[pv[i]];
        if (!estore.empty()) (*ecs)[i] = estore[pv[i]];
    }
    return 0;
}
// one SUM word of a slot += delta (host read-modify-write: the few counters an edge merge moves)
int add_sum_word(pv_ctx *c, uint32_t slot, uint32_t word, int64_t delta)
{
    if (!delta) return 0;
    c->dns.clean[slot] = false;
    uint64_t *dp = c->d_sum + (size_t)slot * PV_SUM_WORDS + word;
    uint64_t v = 0;
    hipError_t e;
    if (!hip_ok(e = hipMemcpy(&v, dp, 8, hipMemcpyDeviceToHost))) return c->hipfail(e, "edge counters");
    v += (uint64_t)delta;
    if (!hip_ok(e = hipMemcpy(dp, &v, 8, hipMemcpyHostToDevice))) return c->hipfail(e, "edge counters");
    return 0;
}

// pv_edge_carry for DNS v2 (one TransactionManager per transaction direction, the direction in
// the key; dns/v2/DnsStreamHandler.cpp:1100-1145, the manager's purge at its shifts .h:440-453):
// an open query meets the first event of its key in this shard as resolve_one2 would have met it
// in one stream. A response there, which this shard counted as an orphan, pairs instead: the
// orphan count is taken back and the transaction accounted on the response (pv_xact_edge2), or
// counted filtered / timed out. Purges are time-outs of the purging shift's bucket. The edge
// pairs' times feed the stream's thresholds (slow_xv) and their slow candidates (scands).
// Buffers: n x (PvXEvent [+ u64 ECS address with top_ecs]).
// The first stub (this shard's first event) of each incoming open query's key: a map over the
// incoming keys (usually few) and one scan of the stubs in first-occurrence order, instead of a map
// over every stub of the shard (millions in a shard the edge horizon covers whole: the map's build
// was most of each rank's turn in the edge chain).
static void edge_first_stubs(const pv_ctx *c, const uint8_t *in, size_t n, size_t esz, std::unordered_map<uint64_t, size_t> &first)
{
    first.reserve(n * 2);
    for (size_t k = 0; k < n; k++) {
        uint64_t key;
        memcpy(&key, in + k * esz + offsetof(PvXEvent, key), 8);
        first.emplace(key, SIZE_MAX);
    }
    if (first.empty()) return;
    size_t left = first.size();
    for (size_t i = 0; i < c->stubs.size() && left; i++) {
        auto it = first.find(c->stubs[i].e.key);
        if (it != first.end() && it->second == SIZE_MAX) { it->second = i; left--; }
    }
    for (auto it = first.begin(); it != first.end();) it = it->second == SIZE_MAX ? first.erase(it) : std::next(it);
}

int edge_carry2(pv_ctx *c, const uint8_t *in, size_t in_bytes, uint8_t **out, size_t *out_bytes)
{
    const bool ecs = c->d_pecs[0] != nullptr;
    const size_t esz = sizeof(PvXEvent) + (ecs ? 8 : 0);
    if (in_bytes % esz) return c->fail(PV_EINVAL, "malformed open-query buffer");
    std::unordered_map<uint64_t, size_t> first;
    edge_first_stubs(c, in, in_bytes / esz, esz, first);
    const uint64_t live = c->dns.ordinal;
    auto in_win = [&](uint64_t ord) { return ord <= live && ord + c->dns.slots.size() > live; };
    auto slot_of = [&](uint64_t ord) { return c->dns.slots[live - ord]; };
    const uint32_t g = c->dns2_groups;
    std::map<std::pair<uint32_t, uint32_t>, int64_t> add; // (slot, SUM word) -> delta
    std::vector<PvXEvent> keep;
    std::vector<uint64_t> keep_ecs;
    std::vector<PvEdgePair> pairs;
    std::vector<size_t> pair_stub;
    const size_t nin = in_bytes / esz;
    for (size_t k = 0; k < nin; k++) {
        PvXEvent qe;
        uint64_t qaddr = 0;
        memcpy(&qe, in + k * esz, sizeof qe);
        if (ecs) memcpy(&qaddr, in + k * esz + sizeof qe, 8);
        const uint32_t xd = (uint32_t)((qe.key >> 48) & 3) - 1;
        if (xd >= 3) return c->fail(PV_EINVAL, "open query %zu has no DNS v2 transaction direction", k);
        auto d2 = [&](uint32_t slot, uint32_t ctr, int64_t v) { add[{slot, PV_OFF_DNS2 + xd * PV_DNS2_CTRS + ctr}] += v; };
        int ps = -1;
        for (size_t i = 0; i < c->dns_shift_ord.size(); i++)
            if (c->dns_shift_ord[i].first >= (int64_t)c->ttl_s + qe.sec) { ps = (int)i; break; }
        auto purged = [&]() {
            const uint64_t o = c->dns_shift_ord[ps].second;
            if (in_win(o)) { d2(slot_of(o), D2_TIMEOUT, 1); d2(slot_of(o), D2_SEEN, 1); }
        };
        auto it = first.find(qe.key);
        if (it == first.end()) {
            if (ps >= 0) purged();
            else { keep.push_back(qe); keep_ecs.push_back(qaddr); }
            continue;
        }
        const pv_ctx::EdgeStub &st = c->stubs[it->second];
        if (ps >= 0 && st.ord >= c->dns_shift_ord[ps].second) { purged(); continue; } // purged before its key's next event
        if (!st.e.qr) continue;                                                          // overwritten by a new query
        const PvXEvent &r = st.e;
        const bool win = in_win(st.ord), kept = (r.period & 0x80) && win;
        const uint32_t slot = win ? slot_of(st.ord) : 0;
        const bool rf = r.pad & 4, qf = qe.pad & 4, rdeep = !(r.pad & 32);
        int64_t dsec = r.sec > qe.sec ? r.sec - qe.sec : qe.sec - r.sec;
        int64_t dnsec = (int64_t)r.nsec - (int64_t)qe.nsec;
        if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
        const bool timed_out = dsec > (int64_t)c->ttl_s || (dsec == (int64_t)c->ttl_s && ((double)dnsec / 1.0e6) >= (double)c->ttl_ms);
        if (kept && !rf) d2(slot, D2_ORPHAN, -1); // this shard counted it NotExist; it is Valid / TimedOut
        auto filtered = [&]() { if (kept && (g & PV_D2G_COUNTERS)) add[{slot, PV_OFF_DNS + DC_FILTERED}] += 1; };
        if (rf) { if (!timed_out && !qf) filtered(); continue; }
        if (qf) { filtered(); continue; }
        if (timed_out) { if (kept) d2(slot, D2_TIMEOUT, 1); continue; }
        const uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
        const PvXValue tv{us, 0, (uint32_t)XV2_TIME + xd};
        if (!(r.period & 0x80)) { // a period outside the window then: its time feeds the next p90 only
            if (g & PV_D2G_XACT_TIMES) c->slow_xv.push_back({st.ord, tv});
            continue;
        }
        if ((g & PV_D2G_XACT_TIMES) && rdeep) c->slow_xv.push_back({st.ord, tv});
        if (!win) continue; // its bucket has left the window since
        if ((g & PV_D2G_XACT_TIMES) && rdeep && st.cand >= 0) {
            pv_ctx::SlowCand sc = c->sorph[(size_t)st.cand];
            sc.us = us;
            sc.dir = (uint8_t)(4 + xd);
            c->scands.push_back(sc);
        }
        if (st.cand < 0) return c->fail(PV_EINVAL, "shard-edge response without its record");
        pairs.push_back(PvEdgePair{qe, r, qaddr, st.order, us});
        pair_stub.push_back(it->second);
    }
    for (auto &kv : add)
        if (int rc = add_sum_word(c, kv.first.first, kv.first.second, kv.second)) return rc;
    // the edge pairs on the device, by groups of at most PV_MAX_SHIFTS + 1 periods (the edge
    // run's period table)
    std::vector<uint64_t> ords;
    for (size_t i : pair_stub) ords.push_back(c->stubs[i].ord);
    std::sort(ords.begin(), ords.end());
    ords.erase(std::unique(ords.begin(), ords.end()), ords.end());
    hipError_t e;
    for (size_t g0 = 0; g0 < ords.size(); g0 += PV_MAX_SHIFTS + 1) {
        const size_t g1 = std::min(ords.size(), g0 + PV_MAX_SHIFTS + 1);
        std::vector<uint8_t> blob[2];
        std::vector<uint32_t> offs[2];
        std::vector<PvEdgePair> run;
        for (size_t i = 0; i < pairs.size(); i++) {
            const pv_ctx::EdgeStub &st = c->stubs[pair_stub[i]];
            auto itp = std::find(ords.begin() + g0, ords.begin() + g1, st.ord);
            if (itp == ords.begin() + g1) continue;
            const pv_ctx::SlowCand &sc = c->sorph[(size_t)st.cand];
            const uint8_t *rec = c->sstore.data() + sc.off;
            uint32_t cap;
            memcpy(&cap, rec + 8, 4);
            const uint32_t sz = (16 + cap + 3) & ~3u;
            offs[sc.tcp].push_back((uint32_t)blob[sc.tcp].size());
            blob[sc.tcp].insert(blob[sc.tcp].end(), rec, rec + sz);
            PvEdgePair pp = pairs[i];
            pp.r.idx = (uint32_t)(offs[sc.tcp].size() - 1) | (sc.tcp ? PV_TCP_IDX : 0u);
            pp.r.period = (uint8_t)(itp - (ords.begin() + g0));
            run.push_back(pp);
        }
        if (run.empty()) continue;
        for (int k = 0; k < 2; k++) blob[k].resize(blob[k].size() + PV_RECS_PAD, 0);
        void *d[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        struct Free { void **p; ~Free() { for (int i = 0; i < 7; i++) if (p[i]) hipFree(p[i]); } } fr{d};
        for (int k = 0; k < 2; k++) {
            if (!hip_ok(e = hipMalloc(&d[2 * k], blob[k].size())) || !hip_ok(e = hipMalloc(&d[2 * k + 1], (offs[k].size() + 1) * 4)) ||
                !hip_ok(e = hipMalloc(&d[4 + k], offs[k].size() + 1)) ||
                !hip_ok(e = hipMemcpy(d[2 * k], blob[k].data(), blob[k].size(), hipMemcpyHostToDevice)) ||
                (!offs[k].empty() && !hip_ok(e = hipMemcpy(d[2 * k + 1], offs[k].data(), offs[k].size() * 4, hipMemcpyHostToDevice))))
                return c->hipfail(e, "edge pairs");
        }
        if (!hip_ok(e = hipMalloc(&d[6], run.size() * sizeof(PvEdgePair))) ||
            !hip_ok(e = hipMemcpy(d[6], run.data(), run.size() * sizeof(PvEdgePair), hipMemcpyHostToDevice)))
            return c->hipfail(e, "edge pairs");
        PvParams P;
        params_common(c, P, (const uint8_t *)d[0], (const uint32_t *)d[1], offs[0].size());
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
        P.tab_live = c->d_tab_live;
        P.flags = c->d_status + ST_FLAGS;
        P.sfx_of = (uint8_t *)d[4];
        P.n_dshift = (uint32_t)(g1 - g0 - 1);
        PvXactParams X;
        memset(&X, 0, sizeof X); // thresholds 0: the slow candidates are the host's (scands)
        for (size_t j = g0; j < g1; j++) {
            const uint32_t k = (uint32_t)(j - g0), slot = slot_of(ords[j]);
            P.dslot_of[k] = slot;
            X.slot_gen[k] = slot | (c->gen[slot] << 8);
            c->dns.clean[slot] = false;
        }
        X.P = P;
        X.vals = c->d_xvals;
        X.n_vals = c->d_nvals;
        X.vals_cap = (uint32_t)c->xv_cap;
        X.valid = c->d_valid;
        X.n_valid = c->d_nvals + 1;
        X.trecs = (const uint8_t *)d[2];
        X.toffs = (const uint32_t *)d[3];
        X.tsfx = (const uint8_t *)d[5];
        flush_fills(c);
        *c->h_xparams = X;
        if (!hip_ok(e = hipMemcpyAsync(c->d_xparams, c->h_xparams, sizeof X, hipMemcpyHostToDevice, c->stream)))
            return c->hipfail(e, "edge pairs");
        hipLaunchKernelGGL(pv_xact_edge2, dim3((uint32_t)((run.size() + 255) / 256)), dim3(256), 0, c->stream,
                           (const PvXactParams *)c->d_xparams, (const PvEdgePair *)d[6], (uint32_t)run.size(), (uint8_t *)d[4],
                           (uint8_t *)d[5]);
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipStreamSynchronize(c->stream))) return c->hipfail(e, "pv_xact_edge2");
    }
    uint32_t flags = 0;
    if (!hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
    if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "top-N table full: raise table_log2");
    // this shard's own open queries (the carried list, latest event per key) with their ECS words
    if (c->n_pend) {
        std::vector<PvXEvent> pend;
        std::vector<uint64_t> pk, pe;
        if (int rc = read_carried(c, pend, pk, &pe)) return rc;
        std::unordered_map<uint64_t, size_t> last;
        last.reserve(pend.size() * 2);
        for (size_t i = 0; i < pend.size(); i++) {
            auto it = last.find(pend[i].key);
            if (it == last.end() || (uint32_t)pk[i] >= (uint32_t)pk[it->second]) last[pend[i].key] = i;
        }
        for (auto &kv : last) { keep.push_back(pend[kv.second]); keep_ecs.push_back(pe[kv.second]); }
    }
    *out_bytes = keep.size() * esz;
    *out = (uint8_t *)malloc(*out_bytes ? *out_bytes : 1);
    if (!*out) return c->fail(PV_ECAPACITY, "out of host memory");
    for (size_t i = 0; i < keep.size(); i++) {
        memcpy(*out + i * esz, &keep[i], sizeof(PvXEvent));
        if (ecs) memcpy(*out + i * esz + sizeof(PvXEvent), &keep_ecs[i], 8);
    }
    return 0;
}
} // namespace

int pv_edge_export(pv_ctx *c, uint8_t **buf, size_t *bytes)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return c->hipfail(e, "synchronize");
    uint32_t nv[4];
    if (!hip_ok(e = hipMemcpy(nv, c->d_nvals, 16, hipMemcpyDeviceToHost))) return c->hipfail(e, "edge counts");
    if (nv[3] > c->orph_cap) return c->fail(PV_ECAPACITY, "%u shard-edge responses exceed the stub capacity", nv[3]);
    // open queries: the carried list, latest event per key (rank order in the sort keys)
    std::vector<PvXEvent> pend, open;
    std::vector<uint64_t> pk;
    if (int rc = read_carried(c, pend, pk)) return rc;
    if (c->n_pend) {
        std::unordered_map<uint64_t, size_t> last;
        last.reserve(pend.size() * 2);
        for (size_t i = 0; i < pend.size(); i++) {
            auto it = last.find(pend[i].key);
            if (it == last.end() || (uint32_t)pk[i] >= (uint32_t)pk[it->second]) last[pend[i].key] = i;
        }
        open.reserve(last.size());
        for (auto &kv : last) open.push_back(pend[kv.second]);
    }
    std::vector<PvXEvent> orph(nv[3]);
    if (nv[3] && !hip_ok(e = hipMemcpy(orph.data(), c->d_orph, nv[3] * sizeof(PvXEvent), hipMemcpyDeviceToHost)))
        return c->hipfail(e, "edge responses");
    EdgeHdr h{EDGE_MAGIC, (uint32_t)open.size(), (uint32_t)orph.size(), (uint32_t)c->dns_shifts.size()};
    const size_t n = sizeof h + (open.size() + orph.size()) * sizeof(PvXEvent) + c->dns_shifts.size() * 12;
    uint8_t *o = (uint8_t *)malloc(n);
    if (!o) return c->fail(PV_ECAPACITY, "out of host memory");
    memcpy(o, &h, sizeof h);
    uint8_t *p = o + sizeof h;
    if (!open.empty()) memcpy(p, open.data(), open.size() * sizeof(PvXEvent));
    p += open.size() * sizeof(PvXEvent);
    if (!orph.empty()) memcpy(p, orph.data(), orph.size() * sizeof(PvXEvent));
    p += orph.size() * sizeof(PvXEvent);
    for (auto &sh : c->dns_shifts) {
        memcpy(p, &sh.first, 8);
        memcpy(p + 8, &sh.second, 4);
        p += 12;
    }
    *buf = o;
    *bytes = n;
    return 0;
}

int pv_edge_merge(pv_ctx *c, const uint8_t *const *bufs, const size_t *sizes, uint32_t nranks, uint32_t me)
{
    mark_merged(c, "pv_edge_merge");
    if (c->dns2_groups)
        return c->fail(PV_EUNSUPPORTED, "DNS v2 shard edges go rank by rank: pv_set_slow_defer, then pv_edge_carry");
    if (c->slow_defer) {
        // this rank's own transaction times end here (the edge pairs' follow)
        if (int rc = sync_xvals(c)) return rc;
        c->xv_local_end = c->xvals_host.size();
    }
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (me >= nranks) return c->fail(PV_EINVAL, "rank %u of %u", me, nranks);
    std::vector<EdgeView> v(nranks);
    for (uint32_t j = 0; j <= me; j++)
        if (!edge_parse(bufs[j], sizes[j], v[j])) return c->fail(PV_EINVAL, "malformed shard-edge buffer of rank %u", j);
    // queries open at the start of shard me, as the ranks before it leave them. A shift of shard j
    // purges every query with sec + ttl <= its second, so shard j purges the queries at or below
    // (its last shift - ttl): taken from a min-heap by second (entries a later query of the key or an
    // answer replaced are skipped by their sequence number), not by a walk over all of them per shard.
    std::unordered_map<uint64_t, std::pair<PvXEvent, uint64_t>> M; // key -> (query, sequence)
    using HE = std::tuple<int64_t, uint64_t, uint64_t>;              // second, sequence, key
    std::priority_queue<HE, std::vector<HE>, std::greater<HE>> H;
    uint64_t seqn = 0;
    for (uint32_t j = 0; j < me; j++) {
        for (auto &o : v[j].orph) M.erase(o.key); // answered (or found purged) in shard j
        if (!v[j].shifts.empty()) {
            int64_t last = v[j].shifts[0].first;
            for (auto &sh : v[j].shifts) last = std::max(last, sh.first);
            const int64_t lim = last - (int64_t)c->ttl_s;
            while (!H.empty() && std::get<0>(H.top()) <= lim) {
                const HE t = H.top();
                H.pop();
                auto it = M.find(std::get<2>(t));
                if (it != M.end() && it->second.second == std::get<1>(t)) M.erase(it);
            }
        }
        for (auto &q : v[j].open) {
            M[q.key] = {q, ++seqn};
            H.push(HE{(int64_t)q.sec, seqn, q.key});
        }
    }
    if (M.empty()) return 0;
    // the earliest orphan of each key (stubs are appended in stream order, one per key and batch)
    std::unordered_map<uint64_t, const PvXEvent *> orph;
    for (auto &o : v[me].orph) orph.emplace(o.key, &o);
    std::map<uint32_t, std::array<uint64_t, 4>> add; // slot -> total, out, in, timeout
    const bool quant = c->dns_groups & PV_DNS_QUANTILES;
    for (auto &kv : M) {
        const PvXEvent &qe = kv.second.first;
        const int ps = purge_shift(c->dns_shifts, c->ttl_s, qe.sec);
        auto it = orph.find(kv.first);
        if (it != orph.end() && (ps < 0 || it->second->sec < c->dns_shifts[ps].first)) {
            const PvXEvent &r = *it->second;
            const uint32_t slot = r.pad & 0x3f;
            const bool rdeep = !(r.pad & 0x40); // a response that is not deep: counts only
            const bool kept = (r.pad & 0x80) && in_dns_window(c, slot);
            // pv_xact_resolve's pairing arithmetic (timespec_diff, TransactionManager.h:24-37)
            int64_t dsec = r.sec > qe.sec ? r.sec - qe.sec : qe.sec - r.sec;
            int64_t dnsec = (int64_t)r.nsec - (int64_t)qe.nsec;
            if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
            const bool timed_out = dsec > (int64_t)c->ttl_s ||
                                   (dsec == (int64_t)c->ttl_s && ((double)dnsec / 1.0e6) >= (double)c->ttl_ms);
            auto &a = add[slot];
            if (timed_out) {
                if (kept) a[3]++;
                continue;
            }
            const uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
            if (kept) {
                a[0]++;
                if (r.dir == 0) a[1]++;
                else if (r.dir == 1) a[2]++;
            }
            // sharded top_slow: the edge pair is a candidate like any valid transaction (its
            // response record was kept with the stub)
            const size_t oi = (size_t)(it->second - v[me].orph.data());
            if (c->slow_defer && oi < c->sorph.size()) {
                pv_ctx::SlowCand sc = c->sorph[oi];
                if (quant && rdeep && r.dir < 2)
                    c->slow_xv.push_back({sc.ord, PvXValue{us, 0, r.dir == 0 ? (uint32_t)XV_FROM_US : (uint32_t)XV_TO_US}});
                if (kept && rdeep && r.dir < 2) {
                    sc.us = us;
                    sc.dir = r.dir;
                    c->scands.push_back(sc);
                }
            }
            if (quant && rdeep && in_dns_window(c, slot)) {
                const uint32_t sg = slot | (c->gen[slot] << 8);
                if (r.dir == 0) c->xvals_host.push_back(PvXValue{us, sg, XV_FROM_US});
                else if (r.dir == 1) c->xvals_host.push_back(PvXValue{us, sg, XV_TO_US});
                if (qe.len && kept) {
                    const double ratio = (double)r.len / (double)qe.len;
                    uint64_t bits;
                    memcpy(&bits, &ratio, 8);
                    c->xvals_host.push_back(PvXValue{bits, sg, XV_RATIO});
                }
            }
        } else if (ps >= 0) {
            const uint32_t slot = c->dns_shifts[ps].second;
            if (in_dns_window(c, slot)) add[slot][3]++;
        }
    }
    for (auto &kv : add) {
        const uint64_t a4[4] = {kv.second[0], kv.second[1], kv.second[2], kv.second[3]};
        if (int rc = add_dns_words(c, kv.first, a4)) return rc;
    }
    return 0;
}

// Sharded runs, in rank order (pv_set_slow_defer): `in` holds the DNS queries the earlier shards
// leave open at this shard's start (the previous rank's *out); each meets the first event of its
// key in this shard as TransactionManager would (libs/visor_transaction/TransactionManager.h:51-106):
// a response pairs with it (valid or timed out), a query overwrites it, a DNS shift of this shard
// at or after ttl + its start purges it first (a time-out there, DnsStreamHandler.h:252-267);
// the rest stay open. *out: those, and this shard's own queries open at its end (pv_free).
int pv_edge_carry(pv_ctx *c, const uint8_t *in, size_t in_bytes, uint8_t **out, size_t *out_bytes)
{
    mark_merged(c, "pv_edge_carry");
    *out = nullptr;
    *out_bytes = 0;
    if (!c->slow_defer) return c->fail(PV_EINVAL, "pv_edge_carry needs pv_set_slow_defer");
    if (!c->dns2_groups && in_bytes % sizeof(PvXEvent)) return c->fail(PV_EINVAL, "malformed open-query buffer");
    if (int rc = sync_xvals(c)) return rc;
    if (c->xv_local_end == SIZE_MAX) c->xv_local_end = c->xvals_host.size();
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return c->hipfail(e, "synchronize");
    if (c->dns2_groups) return edge_carry2(c, in, in_bytes, out, out_bytes);
    std::unordered_map<uint64_t, size_t> first;
    edge_first_stubs(c, in, in_bytes / sizeof(PvXEvent), sizeof(PvXEvent), first);
    const uint64_t live = c->dns.ordinal;
    auto in_win = [&](uint64_t ord) { return ord <= live && ord + c->dns.slots.size() > live; };
    const bool quant = c->dns_groups & PV_DNS_QUANTILES;
    std::map<uint32_t, std::array<uint64_t, 4>> add; // slot -> total, out, in, timeout
    std::vector<PvXEvent> keep;
    const size_t nin = in_bytes / sizeof(PvXEvent);
    for (size_t k = 0; k < nin; k++) {
        PvXEvent qe;
        memcpy(&qe, in + k * sizeof(PvXEvent), sizeof qe);
        int ps = -1;
        for (size_t i = 0; i < c->dns_shift_ord.size(); i++)
            if (c->dns_shift_ord[i].first >= (int64_t)c->ttl_s + qe.sec) { ps = (int)i; break; }
        auto purged = [&]() {
            const uint64_t o = c->dns_shift_ord[ps].second;
            if (in_win(o)) add[c->dns.slots[live - o]][3]++;
        };
        auto it = first.find(qe.key);
        if (it == first.end()) {
            if (ps >= 0) purged();
            else keep.push_back(qe);
            continue;
        }
        const pv_ctx::EdgeStub &st = c->stubs[it->second];
        if (ps >= 0 && st.ord >= c->dns_shift_ord[ps].second) { purged(); continue; } // purged before its key's next event
        if (!st.e.qr) continue;                                                          // overwritten by a new query
        const PvXEvent &r = st.e;
        const bool kept = (r.pad & 0x80) && in_win(st.ord);
        const uint32_t slot = r.pad & 0x3f;
        const bool rdeep = !(r.pad & 0x40); // a response that is not deep: counts only
        int64_t dsec = r.sec > qe.sec ? r.sec - qe.sec : qe.sec - r.sec;
        int64_t dnsec = (int64_t)r.nsec - (int64_t)qe.nsec;
        if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
        const bool timed_out = dsec > (int64_t)c->ttl_s || (dsec == (int64_t)c->ttl_s && ((double)dnsec / 1.0e6) >= (double)c->ttl_ms);
        if (timed_out) { if (kept) add[slot][3]++; continue; }
        const uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
        if (kept) {
            auto &a = add[slot];
            a[0]++;
            if (r.dir == 0) a[1]++;
            else if (r.dir == 1) a[2]++;
        }
        if (quant && rdeep && r.dir < 2) c->slow_xv.push_back({st.ord, PvXValue{us, 0, r.dir == 0 ? (uint32_t)XV_FROM_US : (uint32_t)XV_TO_US}});
        if (quant && rdeep && in_win(st.ord)) {
            const uint32_t sg = slot | (c->gen[slot] << 8);
            if (r.dir < 2) c->xvals_host.push_back(PvXValue{us, sg, r.dir == 0 ? (uint32_t)XV_FROM_US : (uint32_t)XV_TO_US});
            if (qe.len && kept) {
                const double ratio = (double)r.len / (double)qe.len;
                uint64_t bits;
                memcpy(&bits, &ratio, 8);
                c->xvals_host.push_back(PvXValue{bits, sg, XV_RATIO});
            }
        }
        if (kept && rdeep && r.dir < 2 && st.cand >= 0) {
            pv_ctx::SlowCand sc = c->sorph[(size_t)st.cand];
            sc.us = us;
            sc.dir = r.dir;
            c->scands.push_back(sc);
        }
    }
    for (auto &kv : add) {
        const uint64_t a4[4] = {kv.second[0], kv.second[1], kv.second[2], kv.second[3]};
        if (int rc = add_dns_words(c, kv.first, a4)) return rc;
    }
    // this shard's own open queries (the carried list, latest event per key)
    if (c->n_pend) {
        std::vector<PvXEvent> pend;
        std::vector<uint64_t> pk;
        if (int rc = read_carried(c, pend, pk)) return rc;
        std::unordered_map<uint64_t, size_t> last;
        last.reserve(pend.size() * 2);
        for (size_t i = 0; i < pend.size(); i++) {
            auto it = last.find(pend[i].key);
            if (it == last.end() || (uint32_t)pk[i] >= (uint32_t)pk[it->second]) last[pend[i].key] = i;
        }
        for (auto &kv : last) keep.push_back(pend[kv.second]);
    }
    *out_bytes = keep.size() * sizeof(PvXEvent);
    *out = (uint8_t *)malloc(*out_bytes ? *out_bytes : 1);
    if (!*out) return c->fail(PV_ECAPACITY, "out of host memory");
    if (!keep.empty()) memcpy(*out, keep.data(), *out_bytes);
    return 0;
}

int pv_set_end_of_capture(pv_ctx *c, int on)
{
    std::lock_guard<std::mutex> g(c->mu);
    c->eoc_armed = on != 0;
    return 0;
}

int pv_merge_hints(pv_ctx *c, uint64_t *open_queries, uint64_t *xact_values)
{
    if (int rc = sync_xvals(c)) return rc;
    std::lock_guard<std::mutex> g(c->mu);
    *open_queries = c->n_pend;
    *xact_values = c->xvals_host.size() + c->slow_xv.size() + c->scands.size();
    return 0;
}

int pv_set_slow_defer(pv_ctx *c, int defer)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (c->records_seen) return c->fail(PV_EINVAL, "set the slow-transaction mode before the first batch");
    if (defer && c->dns2_groups && !c->d_orph_ord) {
        // DNS v2 stubs carry their first-occurrence order (an edge pair's qname CPC order)
        hipSetDevice(c->device);
        hipError_t e;
        if (!hip_ok(e = hipMalloc(&c->d_orph_ord, (size_t)c->orph_cap * 8))) return c->hipfail(e, "stub orders");
    }
    c->slow_defer = defer != 0;
    return 0;
}

// This rank's own transaction times per DNS period ordinal: (ordinal u32, kind u32, value u64)
// records of kinds XV_FROM_US / XV_TO_US (DNS v2: XV2_TIME + transaction direction). Call before
// pv_values_merge (which appends the other ranks' values).
int pv_slow_values_export(pv_ctx *c, uint8_t **buf, size_t *bytes)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (int rc = sync_xvals(c)) return rc;
    std::vector<uint8_t> o;
    auto put = [&](uint32_t ord, const PvXValue &v) {
        const size_t p = o.size();
        o.resize(p + 16);
        memcpy(&o[p], &ord, 4);
        memcpy(&o[p + 4], &v.kind, 4);
        memcpy(&o[p + 8], &v.bits, 8);
    };
    const size_t nloc = std::min(c->xv_local_end, c->xvals_host.size());
    for (size_t i = 0; i < nloc; i++) {
        const PvXValue &v = c->xvals_host[i];
        if (v.kind != XV_FROM_US && v.kind != XV_TO_US && (v.kind < XV2_TIME || v.kind >= XV2_TIME + 3)) continue;
        auto it = c->sg_ord.find(v.slot);
        if (it != c->sg_ord.end()) put((uint32_t)it->second, v);
    }
    for (auto &ev : c->slow_xv) put((uint32_t)ev.first, ev.second);
    *bytes = o.size();
    *buf = (uint8_t *)malloc(o.size() ? o.size() : 1);
    if (!o.empty()) memcpy(*buf, o.data(), o.size());
    return 0;
}

// Every rank's pv_slow_values_export (bufs[0..nranks)): the slow thresholds of each period of
// the live DNS window over the whole stream (DnsMetricsManager::on_period_shift: at each shift
// the p90 of the bucket that closed, kept when it had no value; 0 before the first), then this
// rank's deferred candidates of those periods checked against them and counted into the
// periods' top_slow tables (DnsMetricsBucket::new_dns_transaction, dns/v1/DnsStreamHandler.cpp:
// 1121-1136). Call before the top-N exchange.
int slow_apply(pv_ctx *c, const std::vector<float> thr[5]);
int pv_slow_finish(pv_ctx *c, const uint8_t *const *bufs, const size_t *sizes, uint32_t nranks)
{
    mark_merged(c, "pv_slow_finish");
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (!c->slow_defer) return c->fail(PV_EINVAL, "pv_slow_finish without pv_set_slow_defer");
    // thresholds come from the quantile sketches: none without the quantiles group (v1) or the
    // transaction-times group (DNS v2, per transaction direction)
    const bool v2 = c->dns2_groups != 0;
    if (!c->started) return 0;
    if (v2 ? !(c->dns2_groups & PV_DNS2_XACT_TIMES)
           : (!(c->dns_groups & PV_DNS_QUANTILES) || !(c->dns_groups & PV_DNS_TRANSACTIONS)))
        return 0;
    // merged values per ordinal: [0] from, [1] to (v1); [2 + d] DNS v2 direction d
    constexpr int NK = 5;
    std::map<uint64_t, std::vector<uint64_t>> vals[NK];
    for (uint32_t r = 0; r < nranks; r++) {
        if (sizes[r] % 16) return c->fail(PV_EINVAL, "malformed slow-value buffer of rank %u", r);
        for (size_t p = 0; p < sizes[r]; p += 16) {
            uint32_t ord, kind;
            uint64_t bits;
            memcpy(&ord, bufs[r] + p, 4);
            memcpy(&kind, bufs[r] + p + 4, 4);
            memcpy(&bits, bufs[r] + p + 8, 8);
            if (kind == XV_FROM_US || kind == XV_TO_US) vals[kind == XV_TO_US][ord].push_back(bits);
            else if (kind >= XV2_TIME && kind < XV2_TIME + 3) vals[2 + kind - XV2_TIME][ord].push_back(bits);
        }
    }
    // thresholds of every ordinal up to the live one
    const uint64_t live = c->dns.ordinal;
    std::vector<float> thr[NK];
    for (int k = 0; k < NK; k++) {
        thr[k].assign(live + 1, 0.0f);
        float t = 0.0f;
        for (uint64_t o = 1; o <= live; o++) {
            auto it = vals[k].find(o - 1);
            if (it != vals[k].end() && !it->second.empty()) t = (float)quantile_at(it->second, 0.90);
            thr[k][o] = t;
        }
    }
    return slow_apply(c, thr);
}

// pv_slow_finish without shipping the values: each ordinal's p90 by the distributed selection
int slow_select(pv_ctx *c, pv_allreduce_fn ar, void *user)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (!c->slow_defer) return c->fail(PV_EINVAL, "pv_slow_finish without pv_set_slow_defer");
    const bool v2 = c->dns2_groups != 0;
    // (a collective: every rank takes part, even one with nothing to judge)
    const bool want = c->started && (v2 ? (c->dns2_groups & PV_DNS2_XACT_TIMES) != 0
                                        : ((c->dns_groups & PV_DNS_QUANTILES) && (c->dns_groups & PV_DNS_TRANSACTIONS)));
    if (int rc = sync_xvals(c)) return rc;
    constexpr int NK = 5;
    // the ordinals: every rank's windows hold the same (global period plan)
    const uint64_t live = c->dns.ordinal;
    std::vector<std::vector<uint64_t>> groups((size_t)NK * (live + 1));
    auto kind_of = [](uint32_t kind) {
        return kind == XV_FROM_US ? 0 : kind == XV_TO_US ? 1 : (kind >= XV2_TIME && kind < XV2_TIME + 3) ? 2 + (int)(kind - XV2_TIME) : -1;
    };
    auto put = [&](uint64_t ord, const PvXValue &v) {
        const int k = kind_of(v.kind);
        if (k >= 0 && ord <= live) groups[(size_t)k * (live + 1) + ord].push_back(v.bits);
    };
    const size_t nloc = std::min(c->xv_local_end, c->xvals_host.size());
    for (size_t i = 0; i < nloc; i++) {
        auto it = c->sg_ord.find(c->xvals_host[i].slot);
        if (it != c->sg_ord.end()) put(it->second, c->xvals_host[i]);
    }
    for (auto &ev : c->slow_xv) put(ev.first, ev.second);
    std::vector<std::vector<double>> fr(groups.size(), std::vector<double>{0.90});
    std::vector<XParts> gparts(groups.size());
    for (size_t i = 0; i < groups.size(); i++) {
        std::sort(groups[i].begin(), groups[i].end());
        gparts[i].push_back(&groups[i]);
    }
    std::vector<uint64_t> n;
    std::vector<std::vector<uint64_t>> q;
    if (int rc = x_select(c, ar, user, gparts, fr, n, q)) return rc;
    if (!want) return 0;
    std::vector<float> thr[NK];
    for (int k = 0; k < NK; k++) {
        thr[k].assign(live + 1, 0.0f);
        float t = 0.0f;
        for (uint64_t o = 1; o <= live; o++) {
            const size_t gi = (size_t)k * (live + 1) + (o - 1);
            if (n[gi]) t = (float)q[gi][0];
            thr[k][o] = t;
        }
    }
    return slow_apply(c, thr);
}

int pv_slow_x_finish(pv_ctx *c, pv_allreduce_fn ar, void *user)
{
    mark_merged(c, "pv_slow_x_finish");
    if (!ar) return c->fail(PV_EINVAL, "no all-reduce callback");
    return slow_select(c, ar, user);
}

int pv_comm_slow_finish(pv_ctx *c)
{
    mark_merged(c, "pv_comm_slow_finish");
    if (!c->comm) return c->fail(PV_EINVAL, "no communicator (pv_comm_init)");
    return slow_select(c, nullptr, nullptr);
}

// this rank's deferred slow candidates against the thresholds of every ordinal (thr[k][ord]:
// [0] from, [1] to (v1), [2 + d] DNS v2 direction d), counted into the periods' top_slow tables
// (the caller holds c->mu)
int slow_apply(pv_ctx *c, const std::vector<float> thr[5])
{
    const uint64_t live = c->dns.ordinal;
    // the window's periods: ordinal -> slot
    std::map<uint64_t, uint32_t> win;
    for (size_t i = 0; i < c->dns.slots.size(); i++) win[live - i] = c->dns.slots[i];
    std::vector<pv_ctx::SlowCand> sel;
    for (auto &sc : c->scands) {
        if (!win.count(sc.ord) || sc.ord > live) continue;
        // v1 dir 0 (toHost): from, 1 (fromHost): to; DNS v2 4 + transaction direction
        const float t = sc.dir >= 4 ? thr[2 + sc.dir - 4][sc.ord] : thr[sc.dir == 1][sc.ord];
        if (t > 0.0f && (float)sc.us >= t) sel.push_back(sc);
    }
    if (sel.empty()) return 0;
    // mini blobs (Ethernet records, TCP message records) and the valid list, by groups of at
    // most PV_MAX_SHIFTS + 1 periods (the resolve parameters' period arrays)
    std::vector<uint64_t> ords;
    for (auto &kv : win) ords.push_back(kv.first);
    for (size_t g0 = 0; g0 < ords.size(); g0 += PV_MAX_SHIFTS + 1) {
        const size_t g1 = std::min(ords.size(), g0 + PV_MAX_SHIFTS + 1);
        std::vector<uint8_t> blob[2];
        std::vector<uint32_t> offs[2];
        std::vector<PvXValid> valid;
        for (auto &sc : sel) {
            auto it = std::find(ords.begin() + g0, ords.begin() + g1, sc.ord);
            if (it == ords.begin() + g1) continue;
            const uint8_t *rec = c->sstore.data() + sc.off;
            uint32_t cap;
            memcpy(&cap, rec + 8, 4);
            const uint32_t sz = (16 + cap + 3) & ~3u;
            offs[sc.tcp].push_back((uint32_t)blob[sc.tcp].size());
            blob[sc.tcp].insert(blob[sc.tcp].end(), rec, rec + sz);
            PvXValid v{};
            v.idx = (uint32_t)(offs[sc.tcp].size() - 1) | (sc.tcp ? PV_TCP_IDX : 0u);
            v.period = (uint8_t)(it - (ords.begin() + g0));
            v.dir = sc.dir;
            v.us = sc.us;
            valid.push_back(v);
        }
        if (valid.empty()) continue;
        for (int k = 0; k < 2; k++) blob[k].resize(blob[k].size() + PV_RECS_PAD, 0);
        hipError_t e;
        uint8_t *d_blob[2] = {nullptr, nullptr};
        uint32_t *d_offs[2] = {nullptr, nullptr};
        PvXValid *d_valid = nullptr;
        struct Free { void *p[5]; ~Free() { for (void *q : p) if (q) hipFree(q); } } fr{{nullptr, nullptr, nullptr, nullptr, nullptr}};
        for (int k = 0; k < 2; k++) {
            if (!hip_ok(e = hipMalloc(&d_blob[k], blob[k].size())) || !hip_ok(e = hipMalloc(&d_offs[k], (offs[k].size() + 1) * 4)))
                return c->hipfail(e, "slow finish");
            fr.p[2 * k] = d_blob[k];
            fr.p[2 * k + 1] = d_offs[k];
            if (!hip_ok(e = hipMemcpy(d_blob[k], blob[k].data(), blob[k].size(), hipMemcpyHostToDevice)) ||
                (!offs[k].empty() && !hip_ok(e = hipMemcpy(d_offs[k], offs[k].data(), offs[k].size() * 4, hipMemcpyHostToDevice))))
                return c->hipfail(e, "slow finish");
        }
        if (!hip_ok(e = hipMalloc(&d_valid, valid.size() * sizeof(PvXValid))) ||
            !hip_ok(e = hipMemcpy(d_valid, valid.data(), valid.size() * sizeof(PvXValid), hipMemcpyHostToDevice)))
            return c->hipfail(e, "slow finish");
        fr.p[4] = d_valid;
        PvParams P;
        params_common(c, P, d_blob[0], d_offs[0], offs[0].size());
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
        P.flags = c->d_status + ST_FLAGS;
        PvXactParams X;
        memset(&X, 0, sizeof X);
        for (size_t j = g0; j < g1; j++) {
            const uint32_t k = (uint32_t)(j - g0);
            P.dslot_of[k] = win[ords[j]];
            X.thr_from[k] = thr[0][ords[j]];
            X.thr_to[k] = thr[1][ords[j]];
            for (int d = 0; d < 3; d++) X.thr2[k][d] = thr[2 + d][ords[j]];
            c->dns.clean[P.dslot_of[k]] = false;
        }
        X.P = P;
        X.valid = d_valid;
        X.trecs = d_blob[1];
        X.toffs = d_offs[1];
        flush_fills(c);
        *c->h_xparams = X;
        if (!hip_ok(e = hipMemcpyAsync(c->d_xparams, c->h_xparams, sizeof X, hipMemcpyHostToDevice, c->stream)))
            return c->hipfail(e, "slow finish");
        hipLaunchKernelGGL(pv_xact_slow, dim3((uint32_t)((valid.size() + 255) / 256)), dim3(256), 0, c->stream,
                           (const PvXactParams *)c->d_xparams, (uint32_t)valid.size());
        if (!hip_ok(e = hipGetLastError()) || !hip_ok(e = hipStreamSynchronize(c->stream))) return c->hipfail(e, "pv_xact_slow");
    }
    uint32_t flags = 0;
    hipError_t e;
    if (!hip_ok(e = hipMemcpy(&flags, c->d_status + ST_FLAGS, 4, hipMemcpyDeviceToHost))) return c->hipfail(e, "status");
    if (flags & PVF_TABLE_FULL) return c->fail(PV_ECAPACITY, "top-N table full: raise table_log2");
    return 0;
}

// Quantile inputs (transaction values) of the live window, exchanged so every rank's
// quantiles cover the whole stream: (slot, kind, bits) records.
int pv_values_export(pv_ctx *c, uint8_t **buf, size_t *bytes)
{
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    if (int rc = sync_xvals(c)) return rc;
    std::vector<uint8_t> o;
    for (auto &v : c->xvals_host) {
        const uint32_t slot = v.slot & 0xff;
        if (slot >= PV_SLOTS || (v.slot >> 8) != c->gen[slot] || !in_dns_window(c, slot)) continue;
        const size_t p = o.size();
        o.resize(p + 16);
        memcpy(&o[p], &v.bits, 8);
        memcpy(&o[p + 8], &slot, 4);
        memcpy(&o[p + 12], &v.kind, 4);
    }
    *bytes = o.size();
    *buf = (uint8_t *)malloc(o.size() ? o.size() : 1);
    if (!o.empty()) memcpy(*buf, o.data(), o.size());
    return 0;
}

int pv_values_merge(pv_ctx *c, const uint8_t *buf, size_t bytes)
{
    mark_merged(c, "pv_values_merge");
    std::lock_guard<std::mutex> g(c->mu);
    if (bytes % 16) return c->fail(PV_EINVAL, "malformed value buffer");
    if (int rc = sync_xvals(c)) return rc;
    for (size_t p = 0; p < bytes; p += 16) {
        PvXValue v;
        uint32_t slot;
        memcpy(&v.bits, buf + p, 8);
        memcpy(&slot, buf + p + 8, 4);
        memcpy(&v.kind, buf + p + 12, 4);
        if (slot >= PV_SLOTS) return c->fail(PV_EINVAL, "malformed value buffer");
        v.slot = slot | (c->gen[slot] << 8);
        c->xvals_host.push_back(v);
    }
    return 0;
}

// Window identity for the merge: (slot, start second) of every live bucket of one manager
// (part 0 = Net, 1 = DNS), newest first.
int pv_window_periods(pv_ctx *c, int part, uint32_t *slots, int64_t *start_sec, uint32_t max_n, uint32_t *n)
{
    std::lock_guard<std::mutex> g(c->mu);
    const Window &w = part == PART_NET ? c->net : c->dns;
    *n = (uint32_t)w.slots.size();
    for (uint32_t i = 0; i < w.slots.size() && i < max_n; i++) {
        slots[i] = w.slots[i];
        start_sec[i] = w.meta[w.slots[i]].start_sec;
    }
    return 0;
}

// Shifts of one manager that happen outside this context's stream (a sharded run: those
// whose shifting event lies in another rank's shard), applied in order as window operations
// only: a bucket opens at each threshold second (empty here), the oldest drops out, and
// next_shift moves on. No transaction purge is counted for them here (the shard that holds
// the shifting event counts its purges through pv_edge_merge).
int pv_advance_windows(pv_ctx *c, int part, const int64_t *thresh, uint32_t n)
{
    std::lock_guard<std::mutex> g(c->mu);
    if (part != PART_NET && part != PART_DNS) return c->fail(PV_EINVAL, "part %d", part);
    if (!c->started) return c->fail(PV_EINVAL, "pv_advance_windows before the start timestamp");
    if (c->cfg.num_periods <= 1) return 0;
    Window &w = part == PART_NET ? c->net : c->dns;
    for (uint32_t k = 0; k < n; k++) {
        if (thresh[k] < w.next_shift_sec)
            return c->fail(PV_EINVAL, "shift at %lld precedes the window's next shift %lld", (long long)thresh[k],
                           (long long)w.next_shift_sec);
        clear_part(c, part, w.slot_at(1));
        win_shift(c, w, thresh[k]);
    }
    return 0;
}

// The seconds (stream order, each once) in which a batch holds a DNS event, by pv_dns_prescan.
// A sharded run's ranks exchange these to compute the DNS manager's global shifts.
// One batch of pv_dns_event_seconds: the UDP events from the prescan bits, the DNS-over-TCP
// messages from a run of the TCP stage (which advances the TCP state: the callers reset it).
} // extern "C"
