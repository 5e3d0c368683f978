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
#define PV_CACHE_N 2048
#define PV_HIST_N 4096
#define PV_LDS_CTRS 64

namespace {

// ------------------------------------------------------------------ byte access
// recs is 256-B aligned and padded by >= 64 bytes: two aligned dword loads and
// v_alignbyte give an unaligned little-endian u32 without byte loops.
__device__ __forceinline__ uint32_t pv_ld32(const uint8_t *base, uint64_t off)
{
    const uint32_t *p = reinterpret_cast<const uint32_t *>(base + (off & ~3ull));
    uint32_t lo = p[0], hi = p[1];
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(off & 3));
}
__device__ __forceinline__ uint32_t pv_ld8(const uint8_t *base, uint64_t off) { return base[off]; }
__device__ __forceinline__ uint32_t pv_clz64(uint64_t x) { return (uint32_t)__clzll((long long)x); }
__device__ __forceinline__ uint64_t pv_umulhi(uint64_t a, uint64_t b) { return __umul64hi(a, b); }
#define PV_FN __device__ __forceinline__
} // namespace
#include "pv_parse.h"
namespace {

// ------------------------------------------------------------------ LDS workgroup state
struct BlockState {
    uint64_t ckey[PV_CACHE_N];
    uint32_t ccnt[PV_CACHE_N];
    uint32_t crep[PV_CACHE_N];
    uint32_t hist[PV_HIST_N];
    uint32_t ctr[PV_LDS_CTRS]; // [0,32) net, [32,64) dns
    uint32_t slot;             // bucket slot the LDS state accumulates for
    uint32_t tile_slot_lo, tile_slot_hi;
};

__device__ __forceinline__ uint64_t *slot_sum(const PvParams &P, uint32_t slot) { return P.sum + (uint64_t)slot * PV_SUM_WORDS; }

// Writes the name record for a newly created global top-N entry (arena: u16 len + bytes).
__device__ uint32_t write_name(const PvParams &P, uint32_t slot, uint32_t metric, uint32_t rep)
{
    Parsed o;
    parse_record(P, P.offs[rep], o);
    const uint8_t *R = P.recs;
    uint8_t *arena = P.arena + (uint64_t)slot * P.arena_cap;
    if (metric == TM_IPV6) {
        uint64_t a = (o.dir == 0) ? o.v6 + 8 : o.v6 + 24;
        uint64_t pos = atomicAdd((unsigned long long *)&P.arena_top[slot], 18ull);
        if (pos + 18 > P.arena_cap) { atomicOr(P.flags, PVF_ARENA_FULL); return 0; }
        arena[pos] = 16; arena[pos + 1] = 0;
        for (int i = 0; i < 16; i++) arena[pos + 2 + i] = (uint8_t)ld8(R, a + i);
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
    uint64_t pos = atomicAdd((unsigned long long *)&P.arena_top[slot], (unsigned long long)(slen + 2));
    if (pos + slen + 2 > P.arena_cap) { atomicOr(P.flags, PVF_ARENA_FULL); return 0; }
    arena[pos] = (uint8_t)(slen & 0xff);
    arena[pos + 1] = (uint8_t)(slen >> 8);
    if (slen > 0 && nl > 0) {
        CopyEmit ce{arena + pos + 2, (uint32_t)start, 0, (metric == TM_SLOW_IN || metric == TM_SLOW_OUT) ? 1u : 0u};
        name_emit(R, m, len, 12, ce);
    }
    return (uint32_t)pos + 1;
}

__device__ void global_add(const PvParams &P, uint32_t slot, uint64_t key, uint64_t w, uint32_t rep)
{
    uint32_t metric = PV_KEY_METRIC(key);
    uint64_t *sum = slot_sum(P, slot);
    if (metric == TM_DENSE_PORT) { atomicAdd((unsigned long long *)&sum[PV_OFF_PORT + (key & 0xffff)], (unsigned long long)w); return; }
    if (metric == TM_DENSE_QTYPE) { atomicAdd((unsigned long long *)&sum[PV_OFF_QTYPE + (key & 0xffff)], (unsigned long long)w); return; }
    if (metric == TM_DENSE_RCODE) { atomicAdd((unsigned long long *)&sum[PV_OFF_RCODE + (key & 0xf)], (unsigned long long)w); return; }
    uint64_t cap = 1ull << P.tcap_log2;
    uint64_t base = (uint64_t)slot << P.tcap_log2;
    uint64_t h = fmix64(key ^ 0x5bd1e995ULL) & (cap - 1);
    for (int probe = 0; probe < 128; probe++) {
        uint64_t *kp = &P.tkeys[base + h];
        uint64_t k = __atomic_load_n(kp, __ATOMIC_RELAXED);
        if (k == key) { atomicAdd((unsigned long long *)&P.tcnt[base + h], (unsigned long long)w); return; }
        if (k == 0) {
            uint64_t prev = atomicCAS((unsigned long long *)kp, 0ull, (unsigned long long)key);
            if (prev == 0) {
                atomicAdd((unsigned long long *)&P.tcnt[base + h], (unsigned long long)w);
                if (metric != TM_IPV4) P.taux[base + h] = write_name(P, slot, metric, rep);
                return;
            }
            if (prev == key) { atomicAdd((unsigned long long *)&P.tcnt[base + h], (unsigned long long)w); return; }
        }
        h = (h + 1) & (cap - 1);
    }
    atomicOr(P.flags, PVF_TABLE_FULL);
}

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

__device__ __forceinline__ void top_add(const PvParams &P, BlockState &S, bool cached, uint32_t slot, uint64_t key,
                                        uint32_t w, uint32_t rep)
{
    if (!(cached && cache_add(S, key, w, rep))) global_add(P, slot, key, w, rep);
}

__device__ void block_init(BlockState &S)
{
    for (uint32_t i = threadIdx.x; i < PV_CACHE_N; i += PV_BLOCK) { S.ckey[i] = 0; S.ccnt[i] = 0; }
    for (uint32_t i = threadIdx.x; i < PV_HIST_N; i += PV_BLOCK) S.hist[i] = 0;
    for (uint32_t i = threadIdx.x; i < PV_LDS_CTRS; i += PV_BLOCK) S.ctr[i] = 0;
}

// Flush the LDS partial bucket of S.slot to HBM and clear it (all threads).
__device__ void block_flush(const PvParams &P, BlockState &S)
{
    __syncthreads();
    uint32_t slot = S.slot;
    if (slot < PV_SLOTS) {
        uint64_t *sum = slot_sum(P, slot);
        for (uint32_t i = threadIdx.x; i < PV_CACHE_N; i += PV_BLOCK) {
            uint64_t k = S.ckey[i];
            if (k) global_add(P, slot, k, S.ccnt[i], S.crep[i]);
        }
        for (uint32_t i = threadIdx.x; i < PV_HIST_N; i += PV_BLOCK)
            if (S.hist[i]) atomicAdd((unsigned long long *)&sum[PV_OFF_PAYLOAD + i], (unsigned long long)S.hist[i]);
        for (uint32_t i = threadIdx.x; i < PV_LDS_CTRS; i += PV_BLOCK)
            if (S.ctr[i]) atomicAdd((unsigned long long *)&sum[(i < 32 ? PV_OFF_NET + i : PV_OFF_DNS + (i - 32))],
                                    (unsigned long long)S.ctr[i]);
    }
    __syncthreads();
    block_init(S);
    __syncthreads();
}

// wave-aggregated counter increment into LDS (lane-uniform slot) or HBM
__device__ __forceinline__ void ctr_add(const PvParams &P, BlockState &S, bool cached, uint32_t slot, uint32_t idx,
                                        bool flag)
{
    if (cached) {
        uint64_t b = __ballot(flag);
        if (b && (threadIdx.x & 63) == (uint32_t)(__ffsll((long long)b) - 1)) atomicAdd(&S.ctr[idx], (uint32_t)__popcll(b));
    } else if (flag) {
        uint64_t *sum = slot_sum(P, slot);
        atomicAdd((unsigned long long *)&sum[idx < 32 ? PV_OFF_NET + idx : PV_OFF_DNS + idx - 32], 1ull);
    }
}

__device__ __forceinline__ void cpc_add(const PvParams &P, uint32_t slot, uint32_t sketch, uint32_t coupon, int64_t gidx)
{
    int64_t *t = P.cpc + (uint64_t)slot * PV_MIN_WORDS + (uint64_t)sketch * PV_CPC_COUPONS + coupon;
    if (__atomic_load_n(t, __ATOMIC_RELAXED) > gidx) atomicMin((long long *)t, (long long)gidx);
}

} // namespace

// ------------------------------------------------------------------ the fused kernel
extern "C" __global__ void __launch_bounds__(PV_BLOCK) pv_net_dns_kernel(PvParams P)
{
    __shared__ BlockState S;
    block_init(S);
    if (threadIdx.x == 0) S.slot = 0xffffffffu;
    __syncthreads();

    const uint64_t ntiles = (P.n + PV_BLOCK - 1) / PV_BLOCK;
    const uint8_t *R = P.recs;
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t i = tile * PV_BLOCK + threadIdx.x;
        const bool active = i < P.n;
        Parsed o;
        uint32_t period = 0, slot = 0;
        bool in_window = false;
        if (active) {
            parse_record(P, P.offs[i], o);
            while (period < P.n_shift && o.sec >= P.thresh[period]) period++;
            slot = P.slot_of[period];
            in_window = period >= P.skip_before;
        }
        // tile slot uniformity (LDS reduce)
        if (threadIdx.x == 0) { S.tile_slot_lo = 0xffffffffu; S.tile_slot_hi = 0; }
        __syncthreads();
        if (active && in_window) { atomicMin(&S.tile_slot_lo, slot); atomicMax(&S.tile_slot_hi, slot); }
        __syncthreads();
        const uint32_t lo = S.tile_slot_lo, hi = S.tile_slot_hi;
        if (lo == hi && lo != S.slot) {
            block_flush(P, S);
            if (threadIdx.x == 0) S.slot = lo;
            __syncthreads();
        }
        const bool cached = (lo == hi) && (lo == S.slot);
        const bool upd = active && in_window;
        const int64_t rel = (int64_t)(P.gbase + i); // global record index (CPC first occurrence)
        uint64_t *sum = slot_sum(P, slot);

        // ---------------- Net v1 (NetworkMetricsBucket::process_net_layer)
        const bool net_ctr = upd && (P.net_groups & 1u);
        ctr_add(P, S, cached, slot, NC_EVENTS, upd);
        ctr_add(P, S, cached, slot, NC_SAMPLES, upd);
        ctr_add(P, S, cached, slot, NC_TOTAL, net_ctr);
        ctr_add(P, S, cached, slot, NC_IN, net_ctr && o.dir == 0);
        ctr_add(P, S, cached, slot, NC_OUT, net_ctr && o.dir == 1);
        ctr_add(P, S, cached, slot, NC_UNK, net_ctr && o.dir == 2);
        ctr_add(P, S, cached, slot, NC_V4, net_ctr && o.l3 == 4);
        ctr_add(P, S, cached, slot, NC_V6, net_ctr && o.l3 == 6);
        ctr_add(P, S, cached, slot, NC_UDP, net_ctr && o.l4 == 17);
        ctr_add(P, S, cached, slot, NC_TCP, net_ctr && o.l4 == 6);
        ctr_add(P, S, cached, slot, NC_SYN, net_ctr && o.l4 == 6 && o.syn);
        ctr_add(P, S, cached, slot, NC_OTHER, net_ctr && o.l4 == 0);
        if (upd) {
            uint32_t cl = o.caplen;
            if (cl > 65535) { atomicOr(P.flags, PVF_BIG_CAPLEN); cl = 65535; }
            if (cached && cl < PV_HIST_N) atomicAdd(&S.hist[cl], 1u);
            else atomicAdd((unsigned long long *)&sum[PV_OFF_PAYLOAD + cl], 1ull);

            const bool card = P.net_groups & 2u, tops = P.net_groups & 8u;
            if (o.has4 && o.dir != 2) {
                uint32_t ip = ld32(R, o.dir == 0 ? o.v4 + 12 : o.v4 + 16);
                if (ip) {
                    uint64_t h1, h2;
                    if (card) {
                        murmur_8((uint64_t)(int64_t)(int32_t)ip, h1, h2);
                        cpc_add(P, slot, o.dir == 0 ? CPC_SRC : CPC_DST, cpc_coupon(h1, h2), rel);
                    }
                    if (tops) top_add(P, S, cached, slot, PV_KEY(TM_IPV4, ip), 1, (uint32_t)i);
                }
            } else if (!o.has4 && o.has6 && o.dir != 2) {
                uint64_t a = o.dir == 0 ? o.v6 + 8 : o.v6 + 24;
                uint64_t w0 = (uint64_t)ld32(R, a) | ((uint64_t)ld32(R, a + 4) << 32);
                uint64_t w1 = (uint64_t)ld32(R, a + 8) | ((uint64_t)ld32(R, a + 12) << 32);
                if (w0 | w1) {
                    uint64_t h1, h2;
                    murmur_16(w0, w1, h1, h2);
                    if (card) cpc_add(P, slot, o.dir == 0 ? CPC_SRC : CPC_DST, cpc_coupon(h1, h2), rel);
                    if (tops) top_add(P, S, cached, slot, PV_KEY(TM_IPV6, h1 ^ (h2 << 1)), 1, (uint32_t)i);
                }
            }
        }

        // ---------------- DNS v1 over UDP (DnsStreamHandler::process_udp_packet_cb)
        bool dns = false;
        uint32_t metric_port = 0, dlen = 0, qr = 0, rcode = 0, ancount = 0, txid = 0;
        uint64_t m = 0;
        if (active && o.l4 == 17) {
            uint32_t pw = ld32(R, o.l4off);
            uint32_t sport = ((pw & 0xff) << 8) | ((pw >> 8) & 0xff);
            uint32_t dport = ((pw >> 8) & 0xff00) | (pw >> 24);
            auto isdns = [](uint32_t p) { return p == 53 || p == 5353 || p == 5355 || p == 53000; };
            if (isdns(dport)) metric_port = sport;
            else if (isdns(sport)) metric_port = dport;
            if (metric_port) {
                dns = true;
                m = o.l4off + 8;
                dlen = o.l4len - 8;
                // header bytes past the capture read as 0 (the reference over-reads)
                uint64_t cap_end = o.frame + o.caplen;
                uint32_t hb[12];
                for (int b = 0; b < 12; b++) hb[b] = (m + b < cap_end) ? ld8(R, m + b) : 0;
                txid = (hb[0] << 8) | hb[1];
                qr = hb[2] >> 7;
                rcode = hb[3] & 15;
                ancount = (hb[6] << 8) | hb[7];
                uint32_t qd = (hb[4] << 8) | hb[5], ns = (hb[8] << 8) | hb[9], ar = (hb[10] << 8) | hb[11];
                DnsInfo d;
                dns_parse(R, m, dlen, qd, ancount, ns, ar, d);
                if (upd) {
                    // deep path (DnsMetricsBucket::process_dns_layer :968-1023)
                    const bool qn = P.dns_groups & PV_DNS_TOP_QNAMES_BIT;
                    if (P.dns_groups & PV_DNS_TOP_PORTS_BIT) top_add(P, S, cached, slot, PV_KEY(TM_DENSE_PORT, metric_port), 1, (uint32_t)i);
                    if (d.ok) {
                        if (qr) top_add(P, S, cached, slot, PV_KEY(TM_DENSE_RCODE, rcode), 1, (uint32_t)i);
                        if (d.has_query) {
                            NameStats st;
                            st.init();
                            if (d.name_len_enc > 0) name_emit(R, m, dlen, 12, st);
                            uint64_t fp_full = fp56(st.ph, st.n, 0);
                            if (st.n > 0 && (P.dns_groups & PV_DNS_CARDINALITY_BIT)) {
                                uint64_t h1, h2;
                                st.mm.finish(h1, h2);
                                cpc_add(P, slot, CPC_QNAME, cpc_coupon(h1, h2), rel);
                            }
                            top_add(P, S, cached, slot, PV_KEY(TM_DENSE_QTYPE, d.qtype), 1, (uint32_t)i);
                            if (qn) {
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
                                uint64_t k2 = q2 == 0 ? st.ph : suffix_hash(st, q2, h2p);
                                top_add(P, S, cached, slot, PV_KEY(TM_QNAME2, fp56(k2, st.n - q2, 0)), 1, (uint32_t)i);
                                if (q3 >= 0 && (uint32_t)q3 < st.n) {
                                    uint64_t k3 = q3 == 0 ? st.ph : suffix_hash(st, q3, h3p);
                                    top_add(P, S, cached, slot, PV_KEY(TM_QNAME3, fp56(k3, st.n - q3, 0)), 1, (uint32_t)i);
                                }
                            }
                        }
                    }
                }
                if (P.want_events) {
                    uint32_t e = atomicAdd(P.n_events, 1u);
                    PvXEvent ev;
                    ev.key = ((uint64_t)flowkey(P, o) << 16) | txid;
                    ev.idx = (uint32_t)i;
                    ev.len = dlen;
                    ev.sec = o.sec;
                    ev.nsec = o.nsec;
                    ev.qr = (uint8_t)qr;
                    ev.dir = o.dir;
                    ev.period = (uint8_t)period;
                    ev.pad = 0;
                    P.events[e] = ev;
                }
                if (period > 0 && o.sec == P.thresh[period - 1]) P.dns_at_thresh[period] = 1;
            }
        }
        const bool dc = dns && upd && (P.dns_groups & PV_DNS_COUNTERS_BIT);
        ctr_add(P, S, cached, slot, 32 + DC_EVENTS, dns && upd);
        ctr_add(P, S, cached, slot, 32 + DC_SAMPLES, dns && upd);
        ctr_add(P, S, cached, slot, 32 + DC_TOTAL, dc);
        ctr_add(P, S, cached, slot, 32 + DC_UDP, dc);
        ctr_add(P, S, cached, slot, 32 + DC_V4, dc && o.l3 == 4);
        ctr_add(P, S, cached, slot, 32 + DC_V6, dc && o.l3 == 6);
        ctr_add(P, S, cached, slot, 32 + DC_QUERIES, dc && !qr);
        ctr_add(P, S, cached, slot, 32 + DC_REPLIES, dc && qr);
        ctr_add(P, S, cached, slot, 32 + DC_NOERROR, dc && qr && rcode == 0);
        ctr_add(P, S, cached, slot, 32 + DC_NODATA, dc && qr && rcode == 0 && ancount == 0);
        ctr_add(P, S, cached, slot, 32 + DC_SRVFAIL, dc && qr && rcode == 2);
        ctr_add(P, S, cached, slot, 32 + DC_NX, dc && qr && rcode == 3);
        ctr_add(P, S, cached, slot, 32 + DC_REFUSED, dc && qr && rcode == 5);
        __syncthreads();
    }
    block_flush(P, S);
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
extern "C" __global__ void pv_xact_keys(const PvXEvent *ev, uint32_t n, uint64_t *skeys, uint32_t *svals)
{
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    skeys[i] = ((uint64_t)hash32(ev[i].key) << 32) | ev[i].idx;
    svals[i] = i;
}

namespace {
// first shift k (1-based period index) after period `a` whose threshold purges a
// query started at `sec`; returns 0 if none inside this batch
__device__ __forceinline__ uint32_t purge_period(const PvParams &P, uint32_t ttl_s, uint32_t a, int64_t sec)
{
    for (uint32_t k = a + 1; k <= P.n_shift; k++)
        if (P.thresh[k - 1] >= (int64_t)ttl_s + sec) return k;
    return 0;
}
__device__ __forceinline__ void xctr(const PvParams &P, uint32_t slot, uint32_t c)
{
    atomicAdd((unsigned long long *)&P.sum[(uint64_t)slot * PV_SUM_WORDS + PV_OFF_DNS + c], 1ull);
}
__device__ __forceinline__ void xval(const PvXactParams &X, uint32_t period, uint32_t kind, uint64_t bits)
{
    uint32_t p = atomicAdd(X.n_vals, 1u);
    if (p >= X.vals_cap) { atomicOr(X.P.flags, PVF_VALUES_FULL); return; }
    X.vals[p] = PvXValue{bits, X.slot_gen[period], kind};
}
// DnsMetricsBucket::new_dns_transaction slow branch (dns/v1 ...cpp:1126-1136): the
// response's first query name (getName(), case kept) into top_slow
__device__ void slow_check(const PvXactParams &X, uint32_t idx, uint32_t period, uint32_t dir, uint64_t us)
{
    const float thr = dir == 0 ? X.thr_from[period] : (dir == 1 ? X.thr_to[period] : 0.0f);
    if (!(thr > 0.0f && (float)us >= thr)) return;
    const PvParams &P = X.P;
    Parsed o;
    parse_record(P, P.offs[idx], o);
    const uint8_t *R = P.recs;
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

extern "C" __global__ void pv_xact_resolve(PvXactParams X)
{
    uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= X.n) return;
    const PvParams &P = X.P;
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
        const uint32_t slot = P.slot_of[e.period];
        // timespec_diff(endTS, startTS) (TransactionManager.h:24-37)
        int64_t dsec = e.sec > qe.sec ? e.sec - qe.sec : qe.sec - e.sec;
        int64_t dnsec = (int64_t)e.nsec - (int64_t)qe.nsec;
        if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
        bool timed_out = dsec > (int64_t)X.ttl_s || (dsec == (int64_t)X.ttl_s && ((double)dnsec / 1.0e6) >= (double)X.ttl_ms);
        if (timed_out) { if (kept) xctr(P, slot, DC_XTIMEOUT); return; }
        // DnsMetricsBucket::new_dns_transaction (dns/v1 ...cpp:1093-1138)
        uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
        if (kept) {
            xctr(P, slot, DC_XTOTAL);
            if (e.dir == 0) xctr(P, slot, DC_XOUT);
            else if (e.dir == 1) xctr(P, slot, DC_XIN);
        }
        // quantile inputs of every period (skipped ones still feed the next period's p90)
        if (X.quantiles) {
            if (e.dir == 0) xval(X, e.period, XV_FROM_US, us);
            else if (e.dir == 1) xval(X, e.period, XV_TO_US, us);
            if (qe.len && kept) xval(X, e.period, XV_RATIO, (uint64_t)__double_as_longlong((double)e.len / (double)qe.len));
        }
        if (!kept || e.dir == 2) return;
        if (X.thr_from[e.period] < 0.0f) {
            uint32_t v = atomicAdd(X.n_valid, 1u);
            X.valid[v] = PvXValid{e.idx, e.period, e.dir, 0, 0, us};
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
        xctr(P, P.slot_of[kp], DC_XTIMEOUT);
    }
}

// top_slow for transactions of periods whose threshold became known after the resolve
extern "C" __global__ void pv_xact_slow(PvXactParams X, uint32_t n_valid)
{
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
