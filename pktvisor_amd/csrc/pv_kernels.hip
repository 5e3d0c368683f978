// SPDX-License-Identifier: MPL-2.0
//
// pv_kernels.hip — CDNA4 (gfx950) kernels for pktvisor's Net v1 + DNS v1 per-packet path.
//
// One packet per lane. A persistent grid of 256-thread workgroups strides over
// tiles of 256 consecutive pcap records; each workgroup keeps its partial bucket
// in LDS (counters via wave ballot+popcount, a payload-size histogram, and a
// key->count cache that absorbs the hot top-N / dense-table keys) and flushes it
// to HBM with one atomic per distinct key when the bucket slot changes or the
// workgroup ends. CPC coupons go straight to a first-occurrence table with a
// read-before-atomicMin filter. No MFMA: this is byte-parallel parsing.
//
// Reference semantics implemented here (restated, not translated):
//   L2..L4 + direction ...... src/inputs/pcap/PcapInputStream.cpp:380-416 (+ PcapPlusPlus
//                             23.09 Packet(raw,TCP|UDP) parse rules)
//   hash5Tuple .............. PcapPlusPlus PacketUtils (FNV-1 over normalised 5-tuple)
//   Net v1 bucket ........... src/handlers/net/v1/NetStreamHandler.cpp:516-548,682-764
//   DNS entry + bucket ...... src/handlers/dns/v1/DnsStreamHandler.cpp:270-302,910-1049
//   decodeName .............. libs/visor_dns/DnsResource.cpp:53-148 (iterative form)
//   parseResources .......... libs/visor_dns/DnsLayer.cpp:119-209 (queryOnly)
//   aggregateDomain ......... libs/visor_dns/dns.cpp:9-43
//   CPC coupon .............. 3rd/datasketches/cpc/include/cpc_sketch_impl.hpp:124-193
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>
#include <stdint.h>

#include "pv_layout.h"

#define PV_BLOCK 256
#define PV_C __attribute__((address_space(4)))
#ifndef PV_CACHE_N
#define PV_CACHE_N 2048
#endif
#define PV_HIST_N 2048
// diagnostic build (-DPV_STAMPS): per-wave cycles spent in each phase of the tile loop
#ifdef PV_STAMPS
#define STAMP_DECL                                                                           \
    uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};                                          \
    uint64_t st_prev = __builtin_amdgcn_s_memtime();
#define STAMP(k)                                                                             \
    {                                                                                        \
        const uint64_t now = __builtin_amdgcn_s_memtime();                                   \
        st_acc[k] += now - st_prev;                                                          \
        st_prev = now;                                                                       \
    }
#define STAMP_FLUSH                                                                          \
    if ((threadIdx.x & 63) == 0)                                                             \
        for (int k_ = 0; k_ < 8; k_++) P.stamps[((uint64_t)blockIdx.x * 4 + threadIdx.x / 64) * 8 + k_] = st_acc[k_];
#else
#define STAMP_DECL
#define STAMP(k)
#define STAMP_FLUSH
#endif
static_assert(PV_CACHE_N <= PV_CACHE_MAX, "update log sized for PV_CACHE_MAX cache entries per flush");
#ifndef PV_WIN
#define PV_WIN 128 // bytes of each record staged into LDS (record header + frame start)
#endif
#ifndef PV_WPE
#define PV_WPE 2 // waves per SIMD the main kernel is register-budgeted for
#endif
#define PV_WINW (PV_WIN / 4)
#define PV_CPCF_N 512           // LDS filter of CPC coupons already submitted by this workgroup

// ------------------------------------------------------------------ byte access
// recs is 256-B aligned and padded by >= 256 bytes: two aligned dword loads and
// v_alignbyte give an unaligned little-endian u32.
__device__ __forceinline__ uint32_t pv_ld32(const uint8_t *base, uint64_t off)
{
    const uint32_t *p = reinterpret_cast<const uint32_t *>(base + (off & ~3ull));
    uint32_t lo = p[0], hi = p[1];
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}
__device__ __forceinline__ uint32_t pv_clz64(uint64_t x) { return (uint32_t)__clzll((long long)x); }
#define PV_FN __device__ __forceinline__
// kernel parameters are read through the constant address space (scalar loads)
#define PV_CREF(T) const PV_C T &
#include "pv_parse.h"

namespace {

// HBM accessor
struct GAcc {
    const uint8_t *R;
    PV_FN uint32_t u32(uint64_t off) const { return pv_ld32(R, off); }
    PV_FN uint32_t u8(uint64_t off) const { return R[off]; }
};

// LDS staging accessor. A tile's bytes sit in LDS in one of two layouts, chosen per
// tile (uniform):
//   packed  - the tile's whole contiguous record span, loaded with fully coalesced
//             16-B lane loads (small records): dword d of the span at stage[d];
//   window  - each lane's first PV_WIN bytes from the 16-B aligned start of its own
//             record (large records), dword-major: dword d of lane l at stage[d*256+l],
//             so per-lane reads at any offset are bank-conflict free.
// One multiply-add covers both (mul = 1/add = 0, or mul = 256/add = lane). Bytes
// outside the staged range come from HBM.
struct TAcc {
    const uint8_t *R;
    const uint32_t *L;
    uint64_t gbase;
    uint32_t lim, mul, add;
    PV_FN uint32_t u32(uint64_t off) const
    {
        uint64_t rel = off - gbase;
        if (rel < lim) {
            uint32_t r = (uint32_t)rel;
            uint32_t d = (r >> 2) * mul + add;
            return __builtin_amdgcn_alignbyte(L[d + mul], L[d], r & 3);
        }
        return pv_ld32(R, off);
    }
    PV_FN uint32_t u8(uint64_t off) const
    {
        uint64_t rel = off - gbase;
        if (rel < lim) {
            uint32_t r = (uint32_t)rel;
            return (L[(r >> 2) * mul + add] >> ((r & 3) * 8)) & 0xff;
        }
        return R[off];
    }
};

__device__ __forceinline__ uint64_t *slot_sum(PV_CREF(PvParams) P, uint32_t slot) { return P.sum + (uint64_t)slot * PV_SUM_WORDS; }

// Writes the name record for a newly created global top-N entry (arena: u16 len + bytes).
__device__ __noinline__ uint32_t write_name(PV_CREF(PvParams) P, uint32_t slot, uint32_t metric, uint32_t rep)
{
    Parsed o;
    const GAcc R{P.recs};
    parse_record(R, P, P.offs[rep], o);
    const uint32_t part = blockIdx.x & (PV_ARENA_PARTS - 1);
    const uint64_t pcap = P.arena_cap / PV_ARENA_PARTS;
    unsigned long long *top = (unsigned long long *)&P.arena_top[slot * PV_ARENA_PARTS + part];
    uint8_t *arena = P.arena + (uint64_t)slot * P.arena_cap;
    if (metric == TM_IPV6) {
        uint64_t a = (o.dir == 0) ? o.v6 + 8 : o.v6 + 24;
        uint64_t pos = atomicAdd(top, 18ull);
        if (pos + 18 > pcap) { atomicOr(P.flags, PVF_ARENA_FULL); return 0; }
        pos += part * pcap;
        arena[pos] = 16; arena[pos + 1] = 0;
        for (int i = 0; i < 16; i++) arena[pos + 2 + i] = (uint8_t)R.u8(a + i);
        return (uint32_t)pos + 1;
    }
    // DNS names: re-derive the first query name of the record
    uint64_t m = o.l4off + 8;
    uint32_t len = o.l4len - 8;
    NameStats st;
    st.init();
    uint32_t nl = name_len_l1(R, m, len, 12);
    if (nl > 0) name_emit(R, m, len, 12, st);
    int start = 0;
    uint32_t n = nl > 0 ? st.n : 0;
    if (metric == TM_QNAME2 || metric == TM_QNAME3) {
        int q2, q3; uint64_t h2, h3;
        if (nl > 0) agg_domain(st, q2, q3, h2, h3); else { q2 = 0; q3 = -1; }
        start = metric == TM_QNAME2 ? q2 : q3;
        if (start < 0) start = (int)n;
    }
    uint32_t slen = n - (uint32_t)start;
    uint64_t pos = atomicAdd(top, (unsigned long long)(slen + 2));
    if (pos + slen + 2 > pcap) { atomicOr(P.flags, PVF_ARENA_FULL); return 0; }
    pos += part * pcap;
    arena[pos] = (uint8_t)(slen & 0xff);
    arena[pos + 1] = (uint8_t)(slen >> 8);
    if (slen > 0 && nl > 0) {
        CopyEmit ce{arena + pos + 2, (uint32_t)start, 0, (metric == TM_SLOW_IN || metric == TM_SLOW_OUT) ? 1u : 0u};
        name_emit(R, m, len, 12, ce);
    }
    return (uint32_t)pos + 1;
}

__device__ __noinline__ void global_add(PV_CREF(PvParams) P, uint32_t slot, uint64_t key, uint64_t w, uint32_t rep)
{
    uint32_t metric = PV_KEY_METRIC(key);
    uint64_t *sum = slot_sum(P, slot);
    if (metric == TM_DENSE_PORT) { atomicAdd((unsigned long long *)&sum[PV_OFF_PORT + (key & 0xffff)], (unsigned long long)w); return; }
    if (metric == TM_DENSE_QTYPE) { atomicAdd((unsigned long long *)&sum[PV_OFF_QTYPE + (key & 0xffff)], (unsigned long long)w); return; }
    if (metric == TM_DENSE_RCODE) { atomicAdd((unsigned long long *)&sum[PV_OFF_RCODE + (key & 0xf)], (unsigned long long)w); return; }
    const uint64_t cap = 1ull << P.tcap_log2;
    const uint64_t base = (uint64_t)slot << P.tcap_log2;
    uint64_t h = fmix64(key ^ 0x5bd1e995ULL) & (cap - 1);
    // the probe loop only claims / finds the entry; a new entry's name record is
    // written once after it, so lanes never serialise on name decoding inside it
    int64_t created = -1;
    bool done = false;
    for (int probe = 0; probe < 128 && !done; probe++) {
        uint64_t *kp = &P.tkeys[base + h];
        uint64_t k = __atomic_load_n(kp, __ATOMIC_RELAXED);
        if (k == 0) {
            uint64_t prev = atomicCAS((unsigned long long *)kp, 0ull, (unsigned long long)key);
            if (prev == 0) created = (int64_t)h;
            k = prev == 0 ? key : prev;
        }
        if (k == key) {
            atomicAdd((unsigned long long *)&P.tcnt[base + h], (unsigned long long)w);
            done = true;
        } else {
            h = (h + 1) & (cap - 1);
        }
    }
    if (!done) atomicOr(P.flags, PVF_TABLE_FULL);
    if (created >= 0 && metric != TM_IPV4) P.taux[base + (uint64_t)created] = write_name(P, slot, metric, rep);
}

// ------------------------------------------------------------------ LDS workgroup state
struct BlockState {
    uint32_t stage[PV_WINW * PV_BLOCK]; // tile bytes (TAcc layouts), 32 KiB
    uint64_t ckey[PV_CACHE_N];       // key -> count cache for top-N and dense tables
    uint32_t ccnt[PV_CACHE_N];
    uint32_t crep[PV_CACHE_N];
    uint32_t hist[PV_HIST_N];        // payload-size histogram (caplen < PV_HIST_N)
    uint32_t cpcf[PV_CPCF_N];        // (sketch << 17 | coupon) + 1 submitted in an earlier tile
    uint32_t mq_n;                   // entries in this workgroup's top-N update log
    uint32_t nev;                    // DNS events appended to this block's region
    uint64_t ebase;                  // first event slot of this block's region
    uint32_t nresp;                  // of which responses
};

// LDS key cache: returns false when the probe window is full (caller goes global)
__device__ __forceinline__ bool cache_add(BlockState &S, uint64_t key, uint32_t w, uint32_t rep)
{
    uint32_t h = hash32(key) & (PV_CACHE_N - 1);
    for (int probe = 0; probe < 8; probe++) {
        uint64_t k = S.ckey[h];
        if (k == key) { atomicAdd(&S.ccnt[h], w); return true; }
        if (k == 0) {
            uint64_t prev = atomicCAS((unsigned long long *)&S.ckey[h], 0ull, (unsigned long long)key);
            if (prev == 0) { S.crep[h] = rep; atomicAdd(&S.ccnt[h], w); return true; }
            if (prev == key) { atomicAdd(&S.ccnt[h], w); return true; }
        }
        h = (h + 1) & (PV_CACHE_N - 1);
    }
    return false;
}

// Top-N updates that the LDS cache cannot absorb go to the workgroup's HBM update log
// (fire-and-forget stores; slot in the top 4 key bits, which hashed metrics leave free);
// pv_topn_insert applies the log to the global tables after the parse kernel, so no
// lane of the parse kernel ever waits on an HBM round trip for a table update.
__device__ __forceinline__ void log_put(PV_CREF(PvParams) P, BlockState &S, uint32_t slot, uint64_t key, uint32_t w,
                                        uint32_t rep)
{
    const uint32_t q = atomicAdd(&S.mq_n, 1u);
    PV_G uint64_t *e = P.mq + ((uint64_t)blockIdx.x * P.mq_cap + q) * 2;
    e[0] = key | ((uint64_t)slot << 60);
    e[1] = (uint64_t)w | ((uint64_t)rep << 32);
}
// dense tables (ports, qtypes, rcodes): plain HBM atomics, nothing waits on them
__device__ __forceinline__ void dense_add(PV_CREF(PvParams) P, uint32_t slot, uint64_t key, uint32_t w)
{
    PV_G uint64_t *sum = P.sum + (uint64_t)slot * PV_SUM_WORDS;
    const uint32_t metric = PV_KEY_METRIC(key);
    const uint32_t off = metric == TM_DENSE_PORT ? PV_OFF_PORT + (uint32_t)(key & 0xffff)
                       : metric == TM_DENSE_QTYPE ? PV_OFF_QTYPE + (uint32_t)(key & 0xffff)
                                                  : PV_OFF_RCODE + (uint32_t)(key & 0xf);
    __hip_atomic_fetch_add(sum + off, (uint64_t)w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// cached: LDS cache, then the update log; uncached (boundary kernel): the global table
__device__ __forceinline__ void top_add(PV_CREF(PvParams) P, BlockState &S, bool cached, uint32_t slot, uint64_t key,
                                        uint32_t w, uint32_t rep)
{
    if (cached) {
        if (cache_add(S, key, w, rep)) return;
        if (PV_KEY_METRIC(key) >= TM_DENSE_PORT) dense_add(P, slot, key, w);
        else log_put(P, S, slot, key, w, rep);
        return;
    }
    global_add(P, slot, key, w, rep);
}

// CPC first occurrence: atomicMin of the global record index into the coupon's slot.
// Records of a workgroup are visited in index order, so a coupon this workgroup already
// submitted in an EARLIER tile cannot lower the minimum: the LDS filter skips it. Keys
// seen in the current tile are inserted only after the tile's barrier (cpc_commit).
__device__ __forceinline__ uint32_t cpcf_slot(uint32_t key) { return (key * 0x9E3779B1u) >> (32 - 9); }
__device__ __forceinline__ void cpc_add(PV_CREF(PvParams) P, BlockState &S, bool cached, uint32_t slot, uint32_t sketch,
                                        uint32_t coupon, int64_t gidx, uint32_t &pending)
{
    const uint32_t key = ((sketch << 17) | coupon) + 1;
    if (cached && S.cpcf[cpcf_slot(key)] == key) return;
    int64_t *t = P.cpc + (uint64_t)slot * PV_MIN_WORDS + (uint64_t)sketch * PV_CPC_COUPONS + coupon;
    atomicMin((long long *)t, (long long)gidx); // no return value: nothing waits on it
    if (cached) pending = key;
}
__device__ __forceinline__ void cpc_commit(BlockState &S, uint32_t key)
{
    if (key) S.cpcf[cpcf_slot(key)] = key;
}
// workgroup barrier that orders LDS only (global loads in flight stay in flight)
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// per-lane counters of the current bucket slot, kept in registers
struct Ctr {
    uint32_t nev, nin, nout, nunk, n4, n6, nudp, ntcp, nsyn, noth;
    uint32_t dev, dq, dr, d4, d6, dnx, dref, dsrv, dnoerr, dnodata;
    PV_FN void zero()
    {
        nev = nin = nout = nunk = n4 = n6 = nudp = ntcp = nsyn = noth = 0;
        dev = dq = dr = d4 = d6 = dnx = dref = dsrv = dnoerr = dnodata = 0;
    }
};

// wave-reduce the register counters and add them to the slot's SUM region
__device__ void ctr_flush(PV_CREF(PvParams) P, uint32_t slot, Ctr &c)
{
    uint64_t *s = slot_sum(P, slot);
    const bool lead = (threadIdx.x & 63) == 0;
    const bool nc = P.net_groups & PV_NET_COUNTERS_BIT, dc = P.dns_groups & PV_DNS_COUNTERS_BIT;
#define PV_FL(field, word, on)                                                              \
    {                                                                                       \
        uint32_t v = wave_sum(c.field);                                                     \
        if (lead && v && (on)) atomicAdd((unsigned long long *)&s[word], (unsigned long long)v); \
    }
    PV_FL(nev, PV_OFF_NET + NC_EVENTS, true) PV_FL(nev, PV_OFF_NET + NC_SAMPLES, true)
    PV_FL(nev, PV_OFF_NET + NC_TOTAL, nc) PV_FL(nin, PV_OFF_NET + NC_IN, nc) PV_FL(nout, PV_OFF_NET + NC_OUT, nc)
    PV_FL(nunk, PV_OFF_NET + NC_UNK, nc) PV_FL(n4, PV_OFF_NET + NC_V4, nc) PV_FL(n6, PV_OFF_NET + NC_V6, nc)
    PV_FL(nudp, PV_OFF_NET + NC_UDP, nc) PV_FL(ntcp, PV_OFF_NET + NC_TCP, nc) PV_FL(nsyn, PV_OFF_NET + NC_SYN, nc)
    PV_FL(noth, PV_OFF_NET + NC_OTHER, nc)
    PV_FL(dev, PV_OFF_DNS + DC_EVENTS, true) PV_FL(dev, PV_OFF_DNS + DC_SAMPLES, true)
    PV_FL(dev, PV_OFF_DNS + DC_TOTAL, dc) PV_FL(dev, PV_OFF_DNS + DC_UDP, dc) PV_FL(dq, PV_OFF_DNS + DC_QUERIES, dc)
    PV_FL(dr, PV_OFF_DNS + DC_REPLIES, dc) PV_FL(d4, PV_OFF_DNS + DC_V4, dc) PV_FL(d6, PV_OFF_DNS + DC_V6, dc)
    PV_FL(dnx, PV_OFF_DNS + DC_NX, dc) PV_FL(dref, PV_OFF_DNS + DC_REFUSED, dc) PV_FL(dsrv, PV_OFF_DNS + DC_SRVFAIL, dc)
    PV_FL(dnoerr, PV_OFF_DNS + DC_NOERROR, dc) PV_FL(dnodata, PV_OFF_DNS + DC_NODATA, dc)
#undef PV_FL
    c.zero();
}

__device__ void block_clear(BlockState &S)
{
    for (uint32_t i = threadIdx.x; i < PV_CACHE_N; i += PV_BLOCK) { S.ckey[i] = 0; S.ccnt[i] = 0; }
    for (uint32_t i = threadIdx.x; i < PV_HIST_N; i += PV_BLOCK) S.hist[i] = 0;
    for (uint32_t i = threadIdx.x; i < PV_CPCF_N; i += PV_BLOCK) S.cpcf[i] = 0;
}

// Flush the LDS partial bucket of `slot` to HBM and clear it (all threads, block-uniform).
__device__ void block_flush(PV_CREF(PvParams) P, BlockState &S, uint32_t slot)
{
    __syncthreads();
    if (slot < PV_SLOTS) {
        uint64_t *sum = slot_sum(P, slot);
        for (uint32_t i = threadIdx.x; i < PV_CACHE_N; i += PV_BLOCK) {
            const uint64_t k = S.ckey[i];
            if (!k) continue;
            if (PV_KEY_METRIC(k) >= TM_DENSE_PORT) dense_add(P, slot, k, S.ccnt[i]);
            else log_put(P, S, slot, k, S.ccnt[i], S.crep[i]);
        }
        for (uint32_t i = threadIdx.x; i < PV_HIST_N; i += PV_BLOCK)
            if (S.hist[i]) atomicAdd((unsigned long long *)&sum[PV_OFF_PAYLOAD + i], (unsigned long long)S.hist[i]);
    }
    __syncthreads();
    block_clear(S);
    __syncthreads();
}

__device__ __forceinline__ uint32_t period_of(PV_CREF(PvParams) P, uint64_t i)
{
    uint32_t p = 0;
    while (p < P.n_shift && i >= P.pstart[p]) p++;
    return p;
}

// payload-size histogram: a per-lane run cache in front of the LDS histogram
__device__ __forceinline__ void hist_put(PV_CREF(PvParams) P, BlockState &S, bool cached, uint32_t slot, uint32_t v,
                                         uint32_t n)
{
    if (!n) return;
    if (cached && v < PV_HIST_N) atomicAdd(&S.hist[v], n);
    else atomicAdd((unsigned long long *)&slot_sum(P, slot)[PV_OFF_PAYLOAD + v], (unsigned long long)n);
}

// DNS v1 over UDP for one lane (DnsStreamHandler::process_udp_packet_cb, :270-302, and
// DnsMetricsBucket::process_dns_layer, :910-1049)
template <class A>
__device__ __forceinline__ void dns_lane(PV_CREF(PvParams) P, BlockState &S, const A &R, const Parsed &o, bool cached,
                                         bool upd, uint32_t slot, uint32_t period, uint64_t i, Ctr &c,
                                         uint32_t &pend_q)
{
    uint32_t pw = R.u32(o.l4off);
    uint32_t sport = ((pw & 0xff) << 8) | ((pw >> 8) & 0xff);
    uint32_t dport = ((pw >> 8) & 0xff00) | (pw >> 24);
    uint32_t metric_port = 0;
    if (dport == 53 || dport == 5353 || dport == 5355 || dport == 53000) metric_port = sport;
    else if (sport == 53 || sport == 5353 || sport == 5355 || sport == 53000) metric_port = dport;
    if (!metric_port) return;
    const uint64_t m = o.l4off + 8;
    const uint32_t dlen = o.l4len - 8;
    // header words; bytes past the capture read as 0 (the reference over-reads there)
    const uint64_t cap_end = o.frame + o.caplen;
    uint32_t w0, w1, w2;
    if (m + 12 <= cap_end) { w0 = R.u32(m); w1 = R.u32(m + 4); w2 = R.u32(m + 8); }
    else {
        w0 = w1 = w2 = 0;
        for (uint32_t b = 0; b < 12; b++) {
            uint32_t v = (m + b < cap_end) ? R.u8(m + b) : 0;
            if (b < 4) w0 |= v << (8 * b); else if (b < 8) w1 |= v << (8 * (b - 4)); else w2 |= v << (8 * (b - 8));
        }
    }
    const uint32_t txid = ((w0 & 0xff) << 8) | ((w0 >> 8) & 0xff);
    const uint32_t qr = (w0 >> 23) & 1;
    const uint32_t rcode = (w0 >> 24) & 15;
    const uint32_t qd = ((w1 & 0xff) << 8) | ((w1 >> 8) & 0xff);
    const uint32_t ancount = ((w1 >> 8) & 0xff00) | (w1 >> 24);
    const uint32_t ns = ((w2 & 0xff) << 8) | ((w2 >> 8) & 0xff);
    const uint32_t ar = ((w2 >> 8) & 0xff00) | (w2 >> 24);
    if (upd) {
        c.dev++;
        c.d4 += o.l3 == 4; c.d6 += o.l3 == 6;
        c.dq += !qr; c.dr += qr;
        c.dnoerr += qr && rcode == 0; c.dnodata += qr && rcode == 0 && ancount == 0;
        c.dsrv += qr && rcode == 2; c.dnx += qr && rcode == 3; c.dref += qr && rcode == 5;
        DnsInfo d;
        dns_parse(R, m, dlen, qd, ancount, ns, ar, d);
        if (P.dns_groups & PV_DNS_TOP_PORTS_BIT) top_add(P, S, cached, slot, PV_KEY(TM_DENSE_PORT, metric_port), 1, (uint32_t)i);
        if (d.ok) {
            if (qr) top_add(P, S, cached, slot, PV_KEY(TM_DENSE_RCODE, rcode), 1, (uint32_t)i);
            if (d.has_query) {
                NameStats st;
                st.init();
                if (d.name_len_enc > 0) name_emit(R, m, dlen, 12, st);
                uint64_t h1, h2;
                st.mm.finish(h1, h2);
                if (st.n > 0 && (P.dns_groups & PV_DNS_CARDINALITY_BIT))
                    cpc_add(P, S, cached, slot, CPC_QNAME, cpc_coupon(h1, h2), (int64_t)(P.gbase + i), pend_q);
                top_add(P, S, cached, slot, PV_KEY(TM_DENSE_QTYPE, d.qtype), 1, (uint32_t)i);
                if (P.dns_groups & PV_DNS_TOP_QNAMES_BIT) {
                    const uint64_t fp_full = fp56(st.ph, st.n, 0);
                    if (qr) {
                        if (rcode == 2) top_add(P, S, cached, slot, PV_KEY(TM_SRVFAIL, fp_full), 1, (uint32_t)i);
                        else if (rcode == 3) top_add(P, S, cached, slot, PV_KEY(TM_NX, fp_full), 1, (uint32_t)i);
                        else if (rcode == 5) top_add(P, S, cached, slot, PV_KEY(TM_REFUSED, fp_full), 1, (uint32_t)i);
                        else if (rcode == 0) {
                            if (P.dns_groups & PV_DNS_TOP_QNAMES_DETAILS_BIT)
                                top_add(P, S, cached, slot, PV_KEY(TM_NOERROR, fp_full), 1, (uint32_t)i);
                            if (!ancount) top_add(P, S, cached, slot, PV_KEY(TM_NODATA, fp_full), 1, (uint32_t)i);
                        }
                        if (P.dns_groups & PV_DNS_TOP_QNAMES_DETAILS_BIT)
                            top_add(P, S, cached, slot, PV_KEY(TM_SIZED, fp_full), dlen, (uint32_t)i);
                    }
                    int q2, q3;
                    uint64_t h2p, h3p;
                    agg_domain(st, q2, q3, h2p, h3p);
                    const uint64_t k2 = q2 == 0 ? st.ph : suffix_hash(st, q2, h2p);
                    top_add(P, S, cached, slot, PV_KEY(TM_QNAME2, fp56(k2, st.n - q2, 0)), 1, (uint32_t)i);
                    if (q3 >= 0 && (uint32_t)q3 < st.n) {
                        const uint64_t k3 = q3 == 0 ? st.ph : suffix_hash(st, q3, h3p);
                        top_add(P, S, cached, slot, PV_KEY(TM_QNAME3, fp56(k3, st.n - q3, 0)), 1, (uint32_t)i);
                    }
                }
            }
        }
    }
    if (P.want_events) {
        // append to this workgroup's event region (records are contiguous per workgroup,
        // so region order is record order); LDS counter, no global atomics
        uint32_t e = (uint32_t)S.ebase + atomicAdd(&S.nev, 1u);
        if (qr) atomicAdd(&S.nresp, 1u);
        PvXEvent ev;
        ev.key = ((uint64_t)flowkey(R, o) << 16) | txid;
        ev.idx = (uint32_t)i;
        ev.len = dlen;
        ev.sec = o.sec;
        ev.nsec = o.nsec;
        ev.qr = (uint8_t)qr;
        ev.dir = o.dir;
        ev.period = (uint8_t)period;
        ev.pad = 0;
        P.events[e] = ev;
        P.ekeys[e] = ((uint64_t)(hash32(ev.key) >> 1) << 32) | (uint32_t)i;
    }
    if (period > 0 && o.sec == P.thresh[period - 1]) P.dns_at_thresh[period] = 1;
}


// cardinality + top IPs of one record (NetworkMetricsBucket::process_net_layer :745-763)
template <class A>
__device__ __forceinline__ void net_ips(PV_CREF(PvParams) P, BlockState &S, const A &R, const Parsed &o, uint64_t i,
                                        bool cached, uint32_t slot, uint32_t &pend_n)
{
    const bool card = P.net_groups & PV_NET_CARDINALITY_BIT, tops = P.net_groups & PV_NET_TOP_IPS_BIT;
    if (o.dir == 2) return;
    if (o.has4) {
        const uint32_t ip = R.u32(o.dir == 0 ? o.v4 + 12 : o.v4 + 16);
        if (!ip) return;
        if (card) {
            uint64_t h1, h2;
            murmur_8((uint64_t)(int64_t)(int32_t)ip, h1, h2);
            cpc_add(P, S, cached, slot, o.dir == 0 ? CPC_SRC : CPC_DST, cpc_coupon(h1, h2), (int64_t)(P.gbase + i),
                    pend_n);
        }
        if (tops) top_add(P, S, cached, slot, PV_KEY(TM_IPV4, ip), 1, (uint32_t)i);
    } else if (o.has6) {
        const uint64_t a = o.dir == 0 ? o.v6 + 8 : o.v6 + 24;
        const uint64_t w0 = (uint64_t)R.u32(a) | ((uint64_t)R.u32(a + 4) << 32);
        const uint64_t w1 = (uint64_t)R.u32(a + 8) | ((uint64_t)R.u32(a + 12) << 32);
        if (!(w0 | w1)) return;
        uint64_t h1, h2;
        murmur_16(w0, w1, h1, h2);
        if (card)
            cpc_add(P, S, cached, slot, o.dir == 0 ? CPC_SRC : CPC_DST, cpc_coupon(h1, h2), (int64_t)(P.gbase + i),
                    pend_n);
        if (tops) top_add(P, S, cached, slot, PV_KEY(TM_IPV6, h1 ^ (h2 << 1)), 1, (uint32_t)i);
    }
}

// One record of a tile whose records all fall in period `period` -> bucket slot `slot`
// (both workgroup-uniform): counters in registers, tables through the LDS cache.
__device__ __forceinline__ void lane_hot(PV_CREF(PvParams) P, BlockState &S, const TAcc &R, const Parsed &o, uint64_t i,
                                         uint32_t period, uint32_t slot, Ctr &c, uint32_t &run_v,
                                         uint32_t &run_n, uint32_t &pend_n, uint32_t &pend_q)
{
    // Net v1 counters (NetworkMetricsBucket::process_net_layer)
    c.nev++;
    c.nin += o.dir == 0; c.nout += o.dir == 1; c.nunk += o.dir == 2;
    c.n4 += o.l3 == 4; c.n6 += o.l3 == 6;
    c.nudp += o.l4 == 17; c.ntcp += o.l4 == 6; c.nsyn += o.l4 == 6 && o.syn; c.noth += o.l4 == 0;
    uint32_t cl = o.caplen;
    if (cl > 65535) { atomicOr(P.flags, PVF_BIG_CAPLEN); cl = 65535; }
    if (cl == run_v) run_n++;
    else { hist_put(P, S, true, slot, run_v, run_n); run_v = cl; run_n = 1; }
    net_ips(P, S, R, o, i, true, slot, pend_n);
    if (o.l4 == 17 && !(P.dbg & 4)) dns_lane(P, S, R, o, true, true, slot, period, i, c, pend_q);
}

// One record of a boundary tile (a period shift inside the tile, or periods outside the
// kept window): the lane resolves its own period and updates HBM directly. Cold path.
template <class A>
__device__ __forceinline__ void lane_cold(PV_CREF(PvParams) P, BlockState &S, const A &R, const Parsed &o, uint64_t i)
{
    const uint32_t period = period_of(P, i);
    const uint32_t slot = P.slot_of[period];
    const bool upd = period >= P.skip_before;
    uint64_t *s = slot_sum(P, slot);
    uint32_t pend = 0;
    if (upd) {
        const bool nc = P.net_groups & PV_NET_COUNTERS_BIT;
        atomicAdd((unsigned long long *)&s[PV_OFF_NET + NC_EVENTS], 1ull);
        atomicAdd((unsigned long long *)&s[PV_OFF_NET + NC_SAMPLES], 1ull);
        if (nc) {
            atomicAdd((unsigned long long *)&s[PV_OFF_NET + NC_TOTAL], 1ull);
            atomicAdd((unsigned long long *)&s[PV_OFF_NET + (o.dir == 0 ? NC_IN : (o.dir == 1 ? NC_OUT : NC_UNK))], 1ull);
            if (o.l3) atomicAdd((unsigned long long *)&s[PV_OFF_NET + (o.l3 == 4 ? NC_V4 : NC_V6)], 1ull);
            atomicAdd((unsigned long long *)&s[PV_OFF_NET + (o.l4 == 17 ? NC_UDP : (o.l4 == 6 ? NC_TCP : NC_OTHER))], 1ull);
            if (o.l4 == 6 && o.syn) atomicAdd((unsigned long long *)&s[PV_OFF_NET + NC_SYN], 1ull);
        }
        const uint32_t cl = o.caplen > 65535 ? 65535 : o.caplen;
        if (o.caplen > 65535) atomicOr(P.flags, PVF_BIG_CAPLEN);
        atomicAdd((unsigned long long *)&s[PV_OFF_PAYLOAD + cl], 1ull);
        net_ips(P, S, R, o, i, false, slot, pend);
    }
    if (o.l4 == 17 && !(P.dbg & 4)) {
        Ctr one;
        one.zero();
        dns_lane(P, S, R, o, false, upd, slot, period, i, one, pend);
        if (upd && one.dev) {
            const bool dc = P.dns_groups & PV_DNS_COUNTERS_BIT;
            atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_EVENTS], 1ull);
            atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_SAMPLES], 1ull);
            if (dc) {
                atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_TOTAL], 1ull);
                atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_UDP], 1ull);
                if (one.d4) atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_V4], 1ull);
                if (one.d6) atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_V6], 1ull);
                atomicAdd((unsigned long long *)&s[PV_OFF_DNS + (one.dq ? DC_QUERIES : DC_REPLIES)], 1ull);
                if (one.dnoerr) atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_NOERROR], 1ull);
                if (one.dnodata) atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_NODATA], 1ull);
                if (one.dsrv) atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_SRVFAIL], 1ull);
                if (one.dnx) atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_NX], 1ull);
                if (one.dref) atomicAdd((unsigned long long *)&s[PV_OFF_DNS + DC_REFUSED], 1ull);
            }
        }
    }
}

} // namespace

// ------------------------------------------------------------------ the fused kernel
extern "C" __global__ void __launch_bounds__(PV_BLOCK, PV_WPE) pv_net_dns_kernel(const PvParams *__restrict__ Pp)
{
    // parameters live in device memory and are read-only for the launch: reading them
    // through the constant address space makes every uniform field a scalar load
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ BlockState S;
    block_clear(S);
    if (threadIdx.x == 0) {
        S.nev = 0; S.nresp = 0; S.mq_n = 0;
        S.ebase = (uint64_t)blockIdx.x * P.tiles_per_block * PV_BLOCK;
    }
    __syncthreads();
    uint32_t cur_slot = 0xffffffffu; // block-uniform: slot the LDS state and counters belong to
    Ctr c;
    c.zero();
    uint32_t run_v = 0, run_n = 0;   // payload-size run cache

    const uint64_t ntiles = (P.n + PV_BLOCK - 1) / PV_BLOCK;
    const uint32_t tid = threadIdx.x;
    // each workgroup owns a contiguous run of tiles (record order inside its event region)
    const uint64_t tbeg = (uint64_t)blockIdx.x * P.tiles_per_block;
    const uint64_t tend = tbeg + P.tiles_per_block < ntiles ? tbeg + P.tiles_per_block : ntiles;
    // software pipeline: while tile t is parsed, the staged bytes of tile t+1 are in
    // flight in registers, so HBM latency overlaps the parse instead of stalling each
    // tile. Everything the next issue needs (tile span bounds, window-tile lane offsets)
    // was loaded one tile earlier still, and cached lanes never wait on HBM mid-tile
    // (table misses are queued), so no wait inside the tile drains the prefetch.
    uint4 pf[PV_WIN / 16];
    auto tile_off = [&](uint64_t t) -> uint64_t {
        return t * PV_BLOCK < P.n ? (uint64_t)P.offs[t * PV_BLOCK] : P.rec_bytes;
    };
    auto lane_off = [&](uint64_t t) -> uint64_t {
        const uint64_t r = t * PV_BLOCK + tid;
        return (t < tend && r < P.n) ? (uint64_t)P.offs[r] : 0;
    };
    // issue the staging loads of tile t; b0/b1 = byte offsets of its first record and of
    // the next tile's first record (uniform), loff = the lane's record offset
    auto issue = [&](uint64_t t, uint64_t b0, uint64_t b1, uint64_t loff, uint32_t &chunks) {
        const uint64_t base = b0 & ~15ull;
        const uint64_t nch = (b1 - base + 15) >> 4;
        if (nch <= PV_WINW * PV_BLOCK / 4) {
            chunks = (uint32_t)nch;
            const uint4 *src = reinterpret_cast<const uint4 *>(P.recs + base);
#pragma unroll
            for (int j = 0; j < PV_WIN / 16; j++) {
                const uint32_t ch = j * PV_BLOCK + tid;
                pf[j] = ch < chunks ? src[ch] : make_uint4(0, 0, 0, 0);
            }
        } else {
            chunks = 0;
            const bool act = t * PV_BLOCK + tid < P.n;
            const uint4 *src = reinterpret_cast<const uint4 *>(P.recs + (loff & ~15ull));
#pragma unroll
            for (int j = 0; j < PV_WIN / 16; j++) pf[j] = act ? src[j] : make_uint4(0, 0, 0, 0);
        }
    };
    // ring: tile t's (b, lane offset) in use; t+1 and t+2 bounds, t+1 lane offsets loaded
    uint64_t b_cur = 0, b_n1 = 0, b_n2 = 0, off_cur = 0, off_n1 = 0;
    uint32_t chunks_cur = 0;
    if (tbeg < tend) {
        b_cur = tile_off(tbeg);
        b_n1 = tile_off(tbeg + 1);
        b_n2 = tile_off(tbeg + 2);
        off_cur = lane_off(tbeg);
        off_n1 = lane_off(tbeg + 1);
        issue(tbeg, b_cur, b_n1, off_cur, chunks_cur);
    }
    STAMP_DECL
    for (uint64_t tile_ = tbeg; tile_ < tend; tile_++) {
        // the tile index is workgroup-uniform: say so, or divergence analysis may keep it
        // (and every parameter load derived from it) in vector registers
        const uint64_t tile = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(tile_ >> 32)) << 32) |
                              __builtin_amdgcn_readfirstlane((uint32_t)tile_);
        const uint64_t t0 = tile * PV_BLOCK;
        const uint64_t t1 = (t0 + PV_BLOCK < P.n ? t0 + PV_BLOCK : P.n) - 1;
        // periods are contiguous index ranges (host-provided start indices): a tile is
        // uniform when its first and last record share a period
        const uint32_t p_lo = period_of(P, t0), p_hi = period_of(P, t1);
        const bool straddle = p_lo != p_hi; // pv_boundary_kernel's tile
        const bool uniform = !straddle && p_lo >= P.skip_before;
        if (uniform && P.slot_of[p_lo] != cur_slot) {
            if (cur_slot != 0xffffffffu) {
                hist_put(P, S, true, cur_slot, run_v, run_n);
                run_n = 0;
                ctr_flush(P, cur_slot, c);
                block_flush(P, S, cur_slot);
            }
            cur_slot = P.slot_of[p_lo];
        }
        const bool cached = uniform; // bucket slot cur_slot, period p_lo
        STAMP(0)

        const uint64_t i = t0 + tid;
        const bool active = i <= t1 && !straddle;
        const uint64_t off = off_cur;
        const uint64_t base = __builtin_amdgcn_readfirstlane((uint32_t)b_cur) & ~15u;
        const uint32_t chunks = __builtin_amdgcn_readfirstlane(chunks_cur);
        // commit tile t's staged bytes to LDS
        if (chunks) {
            uint4 *st4 = reinterpret_cast<uint4 *>(S.stage);
#pragma unroll
            for (int j = 0; j < PV_WIN / 16; j++) st4[j * PV_BLOCK + tid] = pf[j];
        } else {
#pragma unroll
            for (int j = 0; j < PV_WIN / 16; j++) {
                S.stage[(4 * j + 0) * PV_BLOCK + tid] = pf[j].x;
                S.stage[(4 * j + 1) * PV_BLOCK + tid] = pf[j].y;
                S.stage[(4 * j + 2) * PV_BLOCK + tid] = pf[j].z;
                S.stage[(4 * j + 3) * PV_BLOCK + tid] = pf[j].w;
            }
        }
        STAMP(1)
        lds_barrier(); // packed tiles: lanes read bytes other lanes staged
        STAMP(2)
        // issue tile t+1's staging loads; load tile t+3's bound and tile t+2's lane offsets
        if (tile + 1 < tend) {
            const uint64_t b0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b_n1 >> 32)) << 32) |
                                __builtin_amdgcn_readfirstlane((uint32_t)b_n1);
            const uint64_t b1 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b_n2 >> 32)) << 32) |
                                __builtin_amdgcn_readfirstlane((uint32_t)b_n2);
            issue(tile + 1, b0, b1, off_n1, chunks_cur);
            b_cur = b_n1;
            b_n1 = b_n2;
            b_n2 = tile_off(tile + 3);
            off_cur = off_n1;
            off_n1 = lane_off(tile + 2);
        }
        STAMP(3)
        uint32_t pend_n = 0, pend_q = 0; // CPC filter keys to commit after the tile barrier
        // (no `continue` in this loop: a divergent latch would make the tile loop
        // non-uniform and turn every uniform parameter load into a waiting vector load)
        if (P.dbg & 1) c.nev += active && (S.stage[tid] | 1);
        if (active && !(P.dbg & 1)) {
            const TAcc R = chunks ? TAcc{P.recs, S.stage, base, chunks * 16 - 4, 1u, 0u}
                                  : TAcc{P.recs, S.stage, off & ~15ull, PV_WIN - 4, (uint32_t)PV_BLOCK, tid};
            Parsed o;
            parse_record(R, P, off, o);
            STAMP(4)
            if (P.dbg & 2) { c.nev += 1; c.nin += o.dir == 0; c.nudp += o.l4 == 17; }
            else if (cached) lane_hot(P, S, R, o, i, p_lo, cur_slot, c, run_v, run_n, pend_n, pend_q);
            else if (o.l4 == 17) // a tile before the kept window: DNS transaction events only
                dns_lane(P, S, R, o, false, false, 0, p_lo, i, c, pend_q);
        }
        STAMP(5)
        // every lane's CPC filter probes of this tile precede the inserts
        lds_barrier();
        cpc_commit(S, pend_n);
        cpc_commit(S, pend_q);
        STAMP(6)
    }
    if (cur_slot != 0xffffffffu) {
        hist_put(P, S, true, cur_slot, run_v, run_n);
        ctr_flush(P, cur_slot, c);
        block_flush(P, S, cur_slot);
    }
    STAMP(7)
    STAMP_FLUSH
    __syncthreads();
    if (threadIdx.x == 0) {
        P.blk_events[blockIdx.x] = S.nev;
        P.mq_cnt[blockIdx.x] = S.mq_n;
        if (S.nresp) atomicAdd(P.n_events + 1, S.nresp);
    }
}

// Applies each workgroup's top-N update log (pv_net_dns_kernel) to the global tables:
// one entry per lane, so the insert round trips of many entries are in flight at once.
extern "C" __global__ void __launch_bounds__(PV_BLOCK) pv_topn_insert(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint32_t cnt = P.mq_cnt[blockIdx.x];
    const PV_G uint64_t *q = P.mq + (uint64_t)blockIdx.x * P.mq_cap * 2;
    for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) {
        const uint64_t e0 = q[2 * j], e1 = q[2 * j + 1];
        global_add(P, (uint32_t)(e0 >> 60), e0 & ((1ull << 60) - 1), (uint32_t)e1, (uint32_t)(e1 >> 32));
    }
}

// Tiles that hold a period shift: one workgroup per tile, each lane resolves its own
// period and updates HBM directly (no LDS bucket state). Runs after pv_net_dns_kernel
// on the same stream; its DNS events go to regions after the main kernel's.
extern "C" __global__ void __launch_bounds__(PV_BLOCK) pv_boundary_kernel(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ BlockState S;
    if (threadIdx.x == 0) {
        S.nev = 0; S.nresp = 0;
        S.ebase = ((uint64_t)P.grid_main * P.tiles_per_block + blockIdx.x) * PV_BLOCK;
    }
    __syncthreads();
    const uint64_t i = (uint64_t)P.btile[blockIdx.x] * PV_BLOCK + threadIdx.x;
    if (i < P.n) {
        const GAcc R{P.recs};
        Parsed o;
        const uint64_t off = P.offs[i];
        parse_record(R, P, off, o);
        lane_cold(P, S, R, o, i);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        P.blk_events[P.grid_main + blockIdx.x] = S.nev;
        if (S.nresp) atomicAdd(P.n_events + 1, S.nresp);
    }
}

// Packs the per-workgroup event regions into one dense run (workgroup order = record
// order) and writes the total to n_events[0].
extern "C" __global__ void pv_xact_compact(const PvParams *__restrict__ Pp, uint32_t nblk)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ uint32_t base;
    if (threadIdx.x == 0) {
        uint32_t b = 0;
        for (uint32_t j = 0; j < blockIdx.x; j++) b += P.blk_events[j];
        base = b;
        if (blockIdx.x == nblk - 1) P.n_events[0] = b + P.blk_events[blockIdx.x];
    }
    __syncthreads();
    const uint32_t cnt = P.blk_events[blockIdx.x];
    const uint64_t src = (blockIdx.x < P.grid_main ? (uint64_t)blockIdx.x * P.tiles_per_block
                                                   : (uint64_t)P.grid_main * P.tiles_per_block + (blockIdx.x - P.grid_main)) *
                         PV_BLOCK;
    for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) {
        P.skeys[base + j] = P.ekeys[src + j];
        P.svals[base + j] = (uint32_t)(src + j);
    }
}

// Zero a device region of 64-bit words (grid-stride).
extern "C" __global__ void pv_fill_u64(uint64_t *p, uint64_t n, uint64_t v)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = v;
}
extern "C" __global__ void pv_fill_u32(uint32_t *p, uint64_t n, uint32_t v)
{
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = v;
}

// ------------------------------------------------------------------ DNS transactions
// TransactionManager semantics (libs/visor_transaction/TransactionManager.h:51-106) over
// a whole batch at once: events sorted by (hash32(flow,txid), record index); a
// response pairs with the immediately preceding event of the same key iff that
// event is a query (start_transaction overwrites, maybe_end_transaction erases).
// Period shifts purge queries older than the TTL (DnsStreamHandler.h:252-267).
namespace {
// first shift k (1-based period index) after period `a` whose threshold purges a
// query started at `sec`; returns 0 if none inside this batch
__device__ __forceinline__ uint32_t purge_period(PV_CREF(PvParams) P, uint32_t ttl_s, uint32_t a, int64_t sec)
{
    for (uint32_t k = a + 1; k <= P.n_shift; k++)
        if (P.thresh[k - 1] >= (int64_t)ttl_s + sec) return k;
    return 0;
}
// Workgroup-local staging: transaction counters per period and the quantile / slow
// lists are gathered in LDS and reserved in global memory once per workgroup, so no
// global address sees more than one atomic per workgroup.
enum { XC_TOTAL, XC_OUT, XC_IN, XC_TIMEOUT, XC_N };
struct XState {
    uint32_t ctr[PV_MAX_SHIFTS + 1][XC_N];
    PvXValue val[PV_BLOCK * 3];
    PvXValid valid[PV_BLOCK];
    uint32_t nval, nvalid, vbase, dbase;
};
__device__ __forceinline__ void xctr(XState &T, uint32_t period, uint32_t c) { atomicAdd(&T.ctr[period][c], 1u); }
__device__ __forceinline__ void xval(PV_CREF(PvXactParams) X, XState &T, uint32_t period, uint32_t kind, uint64_t bits)
{
    T.val[atomicAdd(&T.nval, 1u)] = PvXValue{bits, X.slot_gen[period], kind};
}
// DnsMetricsBucket::new_dns_transaction slow branch (dns/v1 ...cpp:1126-1136): the
// response's first query name (getName(), case kept) into top_slow
__device__ void slow_check(PV_CREF(PvXactParams) X, uint32_t idx, uint32_t period, uint32_t dir, uint64_t us)
{
    const float thr = dir == 0 ? X.thr_from[period] : (dir == 1 ? X.thr_to[period] : 0.0f);
    if (!(thr > 0.0f && (float)us >= thr)) return;
    PV_CREF(PvParams) P = X.P;
    Parsed o;
    const GAcc R{P.recs};
    parse_record(R, P, P.offs[idx], o);
    uint64_t m = o.l4off + 8;
    uint32_t len = o.l4len - 8;
    DnsInfo d;
    dns_parse(R, m, len, be16(R, m + 4), be16(R, m + 6), be16(R, m + 8), be16(R, m + 10), d);
    if (!(d.ok && d.has_query)) return;
    RawName rn{0, 0};
    if (d.name_len_enc > 0) name_emit(R, m, len, 12, rn);
    const uint32_t metric = dir == 0 ? TM_SLOW_OUT : TM_SLOW_IN;
    global_add(P, P.slot_of[period], PV_KEY(metric, fp56(rn.ph, rn.n, 1)), 1, idx);
}
} // namespace

__device__ void resolve_one(PV_CREF(PvXactParams) X, XState &T, uint32_t p)
{
    PV_CREF(PvParams) P = X.P;
    const PvXEvent e = X.events[X.svals[p]];
    const uint32_t h = (uint32_t)(X.skeys[p] >> 32);
    if (e.qr) {
        // predecessor on the same (flow, txid)
        int q = (int)p - 1;
        for (; q >= 0 && (uint32_t)(X.skeys[q] >> 32) == h; q--)
            if (X.events[X.svals[q]].key == e.key) break;
        if (q < 0 || (uint32_t)(X.skeys[q] >> 32) != h) return; // NotExist
        const PvXEvent qe = X.events[X.svals[q]];
        if (qe.qr) return; // previous event was a response: erased => NotExist
        uint32_t kp = purge_period(P, X.ttl_s, qe.period, qe.sec);
        if (kp && kp <= e.period) return; // purged at a period shift before this response
        const bool kept = e.period >= P.skip_before;
        // timespec_diff(endTS, startTS) (TransactionManager.h:24-37)
        int64_t dsec = e.sec > qe.sec ? e.sec - qe.sec : qe.sec - e.sec;
        int64_t dnsec = (int64_t)e.nsec - (int64_t)qe.nsec;
        if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
        bool timed_out = dsec > (int64_t)X.ttl_s || (dsec == (int64_t)X.ttl_s && ((double)dnsec / 1.0e6) >= (double)X.ttl_ms);
        if (timed_out) { if (kept) xctr(T, e.period, XC_TIMEOUT); return; }
        // DnsMetricsBucket::new_dns_transaction (dns/v1 ...cpp:1093-1138)
        uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
        if (kept) {
            xctr(T, e.period, XC_TOTAL);
            if (e.dir == 0) xctr(T, e.period, XC_OUT);
            else if (e.dir == 1) xctr(T, e.period, XC_IN);
        }
        // quantile inputs of every period (skipped ones still feed the next period's p90)
        if (X.quantiles) {
            if (e.dir == 0) xval(X, T, e.period, XV_FROM_US, us);
            else if (e.dir == 1) xval(X, T, e.period, XV_TO_US, us);
            if (qe.len && kept) xval(X, T, e.period, XV_RATIO, (uint64_t)__double_as_longlong((double)e.len / (double)qe.len));
        }
        if (!kept || e.dir == 2) return;
        if (X.thr_from[e.period] < 0.0f) {
            T.valid[atomicAdd(&T.nvalid, 1u)] = PvXValid{e.idx, (uint8_t)e.period, (uint8_t)e.dir, 0, 0, us};
        } else {
            slow_check(X, e.idx, e.period, e.dir, us);
        }
    } else {
        // an open query purged at a later period shift counts as timed out there
        uint32_t kp = purge_period(P, X.ttl_s, e.period, e.sec);
        if (!kp) return;
        uint32_t q = p + 1;
        for (; q < X.n && (uint32_t)(X.skeys[q] >> 32) == h; q++)
            if (X.events[X.svals[q]].key == e.key) break;
        if (q < X.n && (uint32_t)(X.skeys[q] >> 32) == h && X.events[X.svals[q]].period < kp) return;
        if (kp < P.skip_before) return;
        xctr(T, kp, XC_TIMEOUT);
    }
}

extern "C" __global__ void __launch_bounds__(PV_BLOCK) pv_xact_resolve(const PvXactParams *__restrict__ Xp)
{
    PV_CREF(PvXactParams) X = *(const PV_C PvXactParams *)Xp;
    PV_CREF(PvParams) P = X.P;
    __shared__ XState T;
    for (uint32_t j = threadIdx.x; j < (PV_MAX_SHIFTS + 1) * XC_N; j += blockDim.x) (&T.ctr[0][0])[j] = 0;
    if (threadIdx.x == 0) { T.nval = 0; T.nvalid = 0; }
    __syncthreads();
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < X.n) resolve_one(X, T, p);
    __syncthreads();
    static const uint8_t dc[XC_N] = {DC_XTOTAL, DC_XOUT, DC_XIN, DC_XTIMEOUT};
    if (threadIdx.x < (PV_MAX_SHIFTS + 1) * XC_N) {
        const uint32_t per = threadIdx.x / XC_N, c = threadIdx.x % XC_N;
        const uint32_t v = T.ctr[per][c];
        if (v && per <= P.n_shift)
            atomicAdd((unsigned long long *)&P.sum[(uint64_t)P.slot_of[per] * PV_SUM_WORDS + PV_OFF_DNS + dc[c]],
                      (unsigned long long)v);
    }
    if (threadIdx.x == 0) {
        T.vbase = T.nval ? atomicAdd(X.n_vals, T.nval) : 0;
        T.dbase = T.nvalid ? atomicAdd(X.n_valid, T.nvalid) : 0;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < T.nval; j += blockDim.x) {
        const uint32_t q = T.vbase + j;
        if (q < X.vals_cap) X.vals[q] = T.val[j];
        else atomicOr(X.P.flags, PVF_VALUES_FULL);
    }
    for (uint32_t j = threadIdx.x; j < T.nvalid; j += blockDim.x) X.valid[T.dbase + j] = T.valid[j];
}

// top_slow for transactions of periods whose threshold became known after the resolve
extern "C" __global__ void pv_xact_slow(const PvXactParams *__restrict__ Xp, uint32_t n_valid)
{
    PV_CREF(PvXactParams) X = *(const PV_C PvXactParams *)Xp;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_valid) return;
    const PvXValid v = X.valid[i];
    slow_check(X, v.idx, v.period, v.dir, v.us);
}

// Stable LSD radix sort of (key, value) pairs over all 64 key bits (rocPRIM onesweep).
extern "C" hipError_t pv_radix_sort_pairs(void *tmp, size_t *tmp_bytes, uint64_t *kin, uint64_t *kout, uint32_t *vin,
                                          uint32_t *vout, size_t n, hipStream_t s)
{
    return rocprim::radix_sort_pairs(tmp, *tmp_bytes, kin, kout, vin, vout, n, 0, 64, s);
}
