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
        for (int k_ = 0; k_ < 8; k_++) P.stamps[((uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 8 + k_] = st_acc[k_];
#else
#define STAMP_DECL
#define STAMP(k)
#define STAMP_FLUSH
#endif
// diagnostic build (-DPV_TSTAMPS): per-workgroup cycles of each top-N combine / merge phase
// (thread 0, after the phase's barrier), at stamps[1 << 20 ...]
#ifdef PV_TSTAMPS
#define TST_DECL uint64_t tst_prev = __builtin_amdgcn_s_memtime(), tst_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define TST(k)                                                                               \
    {                                                                                        \
        const uint64_t now = __builtin_amdgcn_s_memtime();                                   \
        tst_acc[k] += now - tst_prev;                                                        \
        tst_prev = now;                                                                      \
    }
#define TST_FLUSH(base)                                                                      \
    if (threadIdx.x == 0)                                                                    \
        for (int k_ = 0; k_ < 8; k_++) P.stamps[(1u << 20) + (base) + (uint64_t)blockIdx.x * 8 + k_] = tst_acc[k_];
#else
#define TST_DECL
#define TST(k)
#define TST_FLUSH(base)
#endif
#ifndef PV_WIN
#define PV_WIN 128 // bytes of each record staged into LDS (record header + frame start)
#endif
#ifndef PV_WPE
#define PV_WPE 4 // waves per SIMD the Net pass is register-budgeted for
#endif
#define PV_WINW (PV_WIN / 4)
#define PV_NWIN 192 // bytes of each record staged by pv_topn_names
#define PV_NOUT 6144 // bytes of name records a pv_topn_names wave packs in LDS before its copy-out

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
__device__ __forceinline__ uint32_t pv_alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) { return __builtin_amdgcn_alignbyte(hi, lo, sh); }
#define PV_FN __device__ __forceinline__
// kernel parameters are read through the constant address space (scalar loads)
#define PV_CREF(T) const PV_C T &
#include "pv_parse.h"
#include <type_traits>

namespace {

// HBM accessor
struct GAcc {
    const uint8_t *R;
    PV_FN uint32_t u32(uint64_t off) const { return pv_ld32(R, off); }
    PV_FN uint32_t u32a(uint64_t off) const { return *reinterpret_cast<const uint32_t *>(R + off); }
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
    PV_FN uint32_t u32a(uint64_t off) const // off 4-aligned
    {
        uint64_t rel = off - gbase;
        if (rel < lim) return L[(uint32_t)(rel >> 2) * mul + add];
        return *reinterpret_cast<const uint32_t *>(R + off);
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

// A lane's LDS window alone (TAcc without the HBM path), for messages the window holds whole:
// decoding them issues no vector-memory load, so it never waits on the loads in flight behind
// it (a load's vmcnt wait covers every load issued before it: TAcc's HBM path, even when no lane
// takes it, puts a vmcnt(0) after each access, draining the next tile's prefetch)
struct LAcc {
    const uint32_t *L;
    uint64_t gbase;
    uint32_t mul, add;
    PV_FN uint32_t u32(uint64_t off) const
    {
        const uint32_t r = (uint32_t)(off - gbase), d = (r >> 2) * mul + add;
        return __builtin_amdgcn_alignbyte(L[d + mul], L[d], r & 3);
    }
    PV_FN uint32_t u32a(uint64_t off) const { return L[((uint32_t)(off - gbase) >> 2) * mul + add]; }
    PV_FN uint32_t u8(uint64_t off) const
    {
        const uint32_t r = (uint32_t)(off - gbase);
        return (L[(r >> 2) * mul + add] >> ((r & 3) * 8)) & 0xff;
    }
};

// LAcc that records how far its reads went (the end of the highest dword read, in window
// bytes): a side-effect-free decode runs on it speculatively and is redone on TAcc when it read
// past the window
struct LAccT {
    const uint32_t *L;
    uint64_t gbase;
    uint32_t mul, add;
    uint32_t *hi;
    PV_FN uint32_t u32(uint64_t off) const
    {
        const uint32_t r = (uint32_t)(off - gbase), d = (r >> 2) * mul + add;
        *hi = max(*hi, ((r >> 2) + 2) * 4);
        return __builtin_amdgcn_alignbyte(L[d + mul], L[d], r & 3);
    }
    PV_FN uint32_t u32a(uint64_t off) const
    {
        const uint32_t r = (uint32_t)(off - gbase);
        *hi = max(*hi, ((r >> 2) + 1) * 4);
        return L[(r >> 2) * mul + add];
    }
    PV_FN uint32_t u8(uint64_t off) const
    {
        const uint32_t r = (uint32_t)(off - gbase);
        *hi = max(*hi, ((r >> 2) + 1) * 4);
        return (L[(r >> 2) * mul + add] >> ((r & 3) * 8)) & 0xff;
    }
};

__device__ __forceinline__ uint64_t *slot_sum(PV_CREF(PvParams) P, uint32_t slot) { return P.sum + (uint64_t)slot * PV_SUM_WORDS; }
// the DNS slot of a lane's period index as a select over the uniform table (a divergent index
// into the parameter block is a vector-memory load, whose wait drains the loads in flight)
__device__ __forceinline__ uint32_t dslot(PV_CREF(PvParams) P, uint32_t period)
{
    // readfirstlane keeps the table opaque (the optimiser would fold the chain back into a load)
    uint32_t s = __builtin_amdgcn_readfirstlane(P.dslot_of[0]);
#pragma unroll
    for (uint32_t k = 1; k <= PV_MAX_SHIFTS; k++) s = period == k ? __builtin_amdgcn_readfirstlane(P.dslot_of[k]) : s;
    return s;
}

// DnsStreamHandler::_filtering's only_qname_suffix (dns/v1/DnsStreamHandler.cpp:615-630): the
// length of the first listed suffix the lower-case first-query name ends with (the
// suffix_size aggregateDomain then uses), -1 if none. n / ph: the name's NameStats length
// and prefix hash, nl its encoded length. Out of line with by-value arguments, so the DNS
// pass keeps no stack frame and no extra registers for this filter-only path.
template <class A>
__device__ __noinline__ int qname_suffix(PV_CREF(PvParams) P, A R, uint64_t m, uint32_t len, uint32_t n, uint64_t ph,
                                         uint32_t nl)
{
    // one decode per listed suffix, a single capture each; the DNS pass records the result
    // per record (sfx_of) for the name writers, which never re-derive it
    for (uint32_t k = 0; k < P.f_nsx; k++) {
        const uint32_t L = P.f_sxl[k];
        if (L > n) continue;
        if (L == 0) return 0;
        SuffixCap sc{0, 0, 0, n - L};
        if (nl > 0) name_emit(R, m, len, 12, sc);
        if (ph_submul(ph, sc.cap, powb(L)) == P.f_sxh[k]) return (int)L;
    }
    return -1;
}

// match_public_suffix (libs/visor_dns/PublicSuffixList.h:226-250) of the lower-case first-query
// name (DnsStreamHandler::_configs, dns/v1/DnsStreamHandler.cpp:648-657): the last label picks
// a list; the first listed suffix the name ends with (byte compare, no label boundary) gives
// its size + 1, else the label's size + 1; 0 when the label is not listed. Exact compares
// against the table's strings, one decode into a private buffer.
template <class A>
__device__ __noinline__ uint32_t psl_match(PV_CREF(PvParams) P, A R, uint64_t m, uint32_t len)
{
    uint8_t nm[320];
    BufEmit be{nm, 0, 320};
    name_emit(R, m, len, 12, be);
    const uint32_t n = be.n;
    if (n == 0 || n > 320) return 0;
    int pos = (int)n - 1;
    while (pos >= 0 && nm[pos] != '.') pos--;
    if (pos < 0 || (uint32_t)pos + 1 == n) return 0;
    const uint32_t lab = (uint32_t)pos + 1, tl = n - lab;
    uint32_t h = 0x811C9DC5u;
    for (uint32_t k = lab; k < n; k++) h = (h ^ nm[k]) * 16777619u;
    const PV_G uint32_t *W = P.psl;
    const PV_G uint8_t *B = reinterpret_cast<const PV_G uint8_t *>(P.psl);
    for (uint32_t s = h & (PV_PSL_SLOTS - 1), probe = 0; probe < PV_PSL_SLOTS; s = (s + 1) & (PV_PSL_SLOTS - 1), probe++) {
        const uint32_t L = W[s * 4 + 2];
        if (L == 0) return 0;
        if (W[s * 4] != h || L != tl) continue;
        const uint32_t off = W[s * 4 + 1];
        bool eq = true;
        for (uint32_t k = 0; k < tl && eq; k++) eq = B[off + k] == nm[lab + k];
        if (!eq) continue;
        const uint32_t fc = W[s * 4 + 3], first = fc & 0xffff, cnt = fc >> 16;
        for (uint32_t j = first; j < first + cnt; j++) {
            const uint32_t so = W[PV_PSL_SFX_WORD + 2 * j], sl = W[PV_PSL_SFX_WORD + 2 * j + 1];
            if (sl > n) continue;
            bool e2 = true;
            for (uint32_t k = 1; k <= sl && e2; k++) e2 = B[so + sl - k] == nm[n - k];
            if (e2) return sl + 1;
        }
        return tl + 1;
    }
    return 0;
}

// only_qname_suffix result of one DNS message: the matched suffix size, 0xff if the
// message has no first query or no listed suffix matches; with public_suffix_list
// (PVDF_PSL) match_public_suffix's size, 0 without a first query
template <class A>
__device__ __forceinline__ uint32_t dns_suffix_of(PV_CREF(PvParams) P, const A &R, uint64_t m, uint32_t dlen,
                                                  uint32_t qd, uint32_t an, uint32_t ns, uint32_t ar)
{
    DnsInfo si;
    dns_parse(R, m, dlen, qd, an, ns, ar, si);
    if (P.f_flags & PVDF_PSL) return (si.ok && si.has_query && si.name_len_enc > 0) ? psl_match(P, R, m, dlen) : 0u;
    if (!si.ok || !si.has_query) return 0xffu;
    NameStats st;
    st.init();
    if (si.name_len_enc > 0) name_stats(R, m, dlen, 12, st);
    const int r = qname_suffix(P, R, m, dlen, st.n, st.ph, si.name_len_enc);
    return r < 0 ? 0xffu : (uint32_t)r;
}

// Writes the name record for a newly created global top-N entry (arena: u16 len + bytes).
// where a name is decoded from when it is not the batch's record `rep`: a TCP message record
// Net v2 IPv6 top-N key of the 16-byte address at a (PV_V2_IP6)
template <class A>
__device__ __forceinline__ uint64_t v2_ip6_key(const A &R, uint64_t a, uint32_t dir)
{
    const uint64_t w0 = (uint64_t)R.u32(a) | ((uint64_t)R.u32(a + 4) << 32);
    const uint64_t w1 = (uint64_t)R.u32(a + 8) | ((uint64_t)R.u32(a + 12) << 32);
    uint64_t h1, h2;
    murmur_16(w0, w1, h1, h2);
    return PV_V2_IP6(dir, h1 ^ (h2 << 1));
}
// the IPv6 address an IPv6 top-N entry names: v1 keys the address of the packet's
// direction (source to the host, else destination); a v2 key of the unknown direction
// may be either address, the one whose key it is
template <class A>
__device__ __forceinline__ uint64_t ip6_name_addr(const A &R, const Parsed &o, uint64_t key)
{
    if (!PV_IS_V2_IP6(key)) return o.dir == 0 ? o.v6 + 8 : o.v6 + 24;
    const uint32_t d = (uint32_t)(key >> 53) & 3;
    if (d != 2) return d == 0 ? o.v6 + 8 : o.v6 + 24;
    return v2_ip6_key(R, o.v6 + 8, 2) == key ? o.v6 + 8 : o.v6 + 24;
}
// the v1 top-N payload of a 16-byte address (net_ip_entry's IPv6 key)
template <class A>
__device__ __forceinline__ uint64_t v1_ip6_key(const A &R, uint64_t a)
{
    const uint64_t w0 = (uint64_t)R.u32(a) | ((uint64_t)R.u32(a + 4) << 32);
    const uint64_t w1 = (uint64_t)R.u32(a + 8) | ((uint64_t)R.u32(a + 12) << 32);
    uint64_t h1, h2;
    murmur_16(w0, w1, h1, h2);
    return (h1 ^ (h2 << 1)) & ((1ull << 55) - 1);
}
struct NameSrc {
    const PV_G uint8_t *recs;
    const PV_G uint32_t *offs;
    uint64_t ecs_addr; // an ECS name given directly (ecs_fam 1 / 2): no record to decode
    uint32_t ecs_fam;
    const PV_G uint8_t *sfx; // suffix sizes of these records (DNS v2 public_suffix_list)
};
// suffix_size of a record's top_qname2/3 aggregation (aggregateDomain): v1 only_qname_suffix or
// public_suffix_list (sfx_of, 0xff: none); v2 public_suffix_list only (v2 hands a response its
// own _configs size; only_qname_suffix is a query filter there), from the record's source
__device__ __forceinline__ uint32_t name_sfx(PV_CREF(PvParams) P, uint32_t rep, const PV_G uint8_t *v2src)
{
    if (P.f_flags & PVDF_V2) {
        if (!(P.f_flags & PVDF_PSL) || (P.f_flags & PVDF_ONLY_QSUFFIX) || !v2src) return 0;
        return v2src[rep];
    }
    if (!(P.f_flags & (PVDF_ONLY_QSUFFIX | PVDF_PSL))) return 0;
    const uint32_t r = P.sfx_of[rep];
    return r == 0xffu ? 0u : r;
}
__device__ __noinline__ uint32_t write_name(PV_CREF(PvParams) P, uint32_t slot, uint32_t metric, uint32_t rep,
                                            const NameSrc *ns = nullptr, uint64_t key = 0)
{
    const uint32_t part = (blockIdx.x * 7 + threadIdx.x / 64) & (PV_ARENA_PARTS - 1);
    const uint64_t pcap = P.arena_cap / PV_ARENA_PARTS;
    const uint32_t tab = PV_TSLOT(slot, metric);
    unsigned long long *top = (unsigned long long *)&P.arena_top[tab * PV_ARENA_PARTS + part];
    uint8_t *arena = P.arena + (uint64_t)tab * P.arena_cap;
    // an ECS address: family byte + 16 address bytes (the host formats it)
    auto ecs_name = [&](uint32_t fam, uint64_t addr) -> uint32_t {
        uint64_t pos = atomicAdd(top, 20ull);
        if (pos + 20 > pcap) { atomicOr(P.flags, PVF_ARENA_FULL); return 0; }
        pos += part * pcap;
        arena[pos] = 17; arena[pos + 1] = 0; arena[pos + 2] = (uint8_t)fam;
        for (int i = 0; i < 16; i++) arena[pos + 3 + i] = i < 8 ? (uint8_t)(addr >> (8 * i)) : 0;
        return (uint32_t)pos + 1;
    };
    if (ns && ns->ecs_fam) return ecs_name(ns->ecs_fam, ns->ecs_addr);
    Parsed o;
    const GAcc R{ns ? ns->recs : P.recs};
    if (ns) {
        ParseCfg C = parse_cfg(P);
        C.linktype = 101;
        parse_record(R, C, P, ns->offs[rep], o);
    } else {
        parse_record(R, P, P.offs[rep], o);
    }
    if (metric == TM_IPV6) {
        const uint64_t a = P.tap ? (v1_ip6_key(R, o.v6 + 8) == (key & ((1ull << 55) - 1)) ? o.v6 + 8 : o.v6 + 24)
                                 : ip6_name_addr(R, o, key);
        uint64_t pos = atomicAdd(top, 20ull); // records are 4-byte multiples (pv_topn_names copies dwords)
        if (pos + 20 > pcap) { atomicOr(P.flags, PVF_ARENA_FULL); return 0; }
        pos += part * pcap;
        arena[pos] = 16; arena[pos + 1] = 0;
        for (int i = 0; i < 16; i++) arena[pos + 2 + i] = (uint8_t)R.u8(a + i);
        return (uint32_t)pos + 1;
    }
    // DNS names: re-derive the first query name of the record
    uint64_t m = o.l4off + 8;
    uint32_t len = o.l4len - 8;
    if (metric == TM_ECS) {
        // the query's ECS address
        uint64_t addr = 0;
        const uint32_t fam = dns_ecs(R, m, len, be16(R, m + 4), be16(R, m + 6), be16(R, m + 8), be16(R, m + 10), addr);
        return ecs_name(fam, addr);
    }
    NameStats st;
    st.init();
    uint32_t nl = name_len_l1(R, m, len, 12);
    if (nl > 0) name_stats(R, m, len, 12, st);
    int start = 0;
    uint32_t n = nl > 0 ? st.n : 0;
    if (metric == TM_QNAME2 || metric == TM_QNAME3) {
        int q2, q3; uint64_t h2, h3;
        const uint32_t sfx = name_sfx(P, rep, ns ? ns->sfx : P.sfx_of);
        if (nl > 0) agg_domain_r(R, m, len, st, q2, q3, h2, h3, sfx); else { q2 = 0; q3 = -1; }
        start = metric == TM_QNAME2 ? q2 : q3;
        if (start < 0) start = (int)n;
    }
    uint32_t slen = n - (uint32_t)start;
    uint64_t pos = atomicAdd(top, (unsigned long long)((slen + 2 + 3) & ~3u));
    if (pos + slen + 2 > pcap) { atomicOr(P.flags, PVF_ARENA_FULL); return 0; }
    pos += part * pcap;
    arena[pos] = (uint8_t)(slen & 0xff);
    arena[pos + 1] = (uint8_t)(slen >> 8);
    if (slen > 0 && nl > 0) {
        CopyEmit ce{arena + pos + 2, (uint32_t)start, 0, ((metric == TM_SLOW_IN || metric == TM_SLOW_OUT) && !(P.dns2_groups && PV_IS_V2_DKEY(key))) ? 1u : 0u};
        name_emit(R, m, len, 12, ce);
    }
    return (uint32_t)pos + 1;
}

// Table position of a key: its region base (slot included) and start index in the region.
struct TPos {
    uint64_t rbase;
    uint32_t pos, rmask;
};
__device__ __forceinline__ uint64_t tkey_hash(uint64_t key) { return fmix64(key ^ 0x5bd1e995ULL); }
__device__ __forceinline__ uint32_t tregion(PV_CREF(PvParams) P, uint64_t h)
{
    return (uint32_t)(h >> 40) & ((1u << P.reg_log2) - 1);
}
__device__ __forceinline__ TPos tpos(PV_CREF(PvParams) P, uint32_t slot, uint64_t key)
{
    const uint32_t rsl = P.tcap_log2 - P.reg_log2;
    const uint64_t h = tkey_hash(key);
    TPos t;
    t.rmask = (1u << rsl) - 1;
    t.rbase = ((uint64_t)PV_TSLOT(slot, PV_KEY_METRIC(key)) << P.tcap_log2) + ((uint64_t)tregion(P, h) << rsl);
    t.pos = (uint32_t)h & t.rmask;
    return t;
}

// an update its full region could not take: kept for pv_topn_retry (after the host purges the
// table); past the list's capacity, or without a record to name the key from, the batch fails.
// A multi-GPU owner merge's entries carry no record (their names are fetched for the read view):
// they keep their 64-bit weight in (w, rep), marked by pad = 1.
__device__ __forceinline__ void table_overflow(PV_CREF(PvParams) P, uint32_t slot, uint64_t key, uint64_t w, uint32_t rep,
                                               bool named)
{
    const bool xm = P.xmerge != 0;
    if (!P.ovf || (!named && !xm)) { atomicOr(P.flags, PVF_TABLE_FULL); return; }
    const uint32_t k = atomicAdd(P.ovf_cnt, 1u);
    if (k >= P.ovf_cap) { atomicOr(P.flags, PVF_TABLE_FULL); return; }
    P.ovf[k] = xm ? PvOvf{key, (uint32_t)w, (uint32_t)(w >> 32), slot, 1u} : PvOvf{key, (uint32_t)w, rep, slot, 0};
    atomicOr(P.ovf_cnt + 1, 1u << PV_TSLOT(slot, PV_KEY_METRIC(key)));
}

// Direct insert into the global table (boundary tiles, slow transactions, regions with
// few updates in a batch): device-scope CAS / add, probing inside the key's region.
__device__ __noinline__ void global_add(PV_CREF(PvParams) P, uint32_t slot, uint64_t key, uint64_t w, uint32_t rep,
                                        const NameSrc *ns = nullptr)
{
    uint32_t metric = PV_KEY_METRIC(key);
    uint64_t *sum = slot_sum(P, slot);
    if (metric == TM_DENSE_PORT) { atomicAdd((unsigned long long *)&sum[PV_OFF_PORT + (key & 0xffff)], (unsigned long long)w); return; }
    if (metric == TM_DENSE_QTYPE) { atomicAdd((unsigned long long *)&sum[PV_OFF_QTYPE + (key & 0xffff)], (unsigned long long)w); return; }
    if (metric == TM_DENSE_RCODE) { atomicAdd((unsigned long long *)&sum[PV_OFF_RCODE + (key & 0xf)], (unsigned long long)w); return; }
    TPos t = tpos(P, slot, key);
    // the probe loop only claims / finds the entry; a new entry's name record is
    // written once after it, so lanes never serialise on name decoding inside it
    int64_t created = -1;
    bool done = false;
    for (int probe = 0; probe < PV_PROBES && !done; probe++) {
        uint64_t *kp = &P.tkeys[t.rbase + t.pos];
        uint64_t k = __atomic_load_n(kp, __ATOMIC_RELAXED);
        uint64_t add = w;
        if (k == 0) {
            // slot clears reset keys only: an empty entry's count word holds what its last
            // occupant left, and nobody adds to it before its key is claimed, so the claimer
            // reads it first (complete before the CAS issues) and adds its weight net of it
            const uint64_t stale = __atomic_load_n(&P.tcnt[t.rbase + t.pos], __ATOMIC_RELAXED);
            asm volatile("" ::"v"((uint32_t)stale), "v"((uint32_t)(stale >> 32)) : "memory");
            uint64_t prev = atomicCAS((unsigned long long *)kp, 0ull, (unsigned long long)key);
            if (prev == 0) { created = (int64_t)(t.rbase + t.pos); add = w - stale; }
            k = prev == 0 ? key : prev;
        }
        if (k == key) {
            atomicAdd((unsigned long long *)&P.tcnt[t.rbase + t.pos], (unsigned long long)add);
            done = true;
        } else {
            t.pos = (t.pos + 1) & t.rmask;
        }
    }
    // (a TCP message's record lives in the TCP pass's arena, not the batch the retry reads: fail)
    if (!done) table_overflow(P, slot, key, w, rep, ns == nullptr && !P.tcp_pass && !P.xmerge);
    if (created >= 0) atomicAdd(&P.tab_live[PV_TSLOT(slot, metric)], 1u);
    // (a multi-GPU owner merge knows no record: the name stays unknown, pv_comm_finalize fetches it)
    if (created >= 0 && metric != TM_IPV4) P.taux[created] = P.xmerge ? 0u : write_name(P, slot, metric, rep, ns, key);
}


// ------------------------------------------------------------------ LDS key cache
// Open-addressed key -> (count, min record index) cache shared by a workgroup's
// waves. Keys carry their bucket slot in bits 60..63 (local metric ids are < 16), so
// one cache serves every slot a workgroup touches and is flushed once, at the end.
// crep holds the smallest record index that touched the entry: a later record of the
// same key knows its CPC coupon (same key => same coupon) was already submitted with a
// smaller index, and the insert kernel uses it as the record a name is decoded from.
#ifndef PV_CACHE_PROBES
#define PV_CACHE_PROBES 4 // slots a key may probe before it goes to the update log
#endif
#define PV_LKEY(slot, lm, payload) (((uint64_t)(slot) << 60) | ((uint64_t)(lm) << 56) | ((uint64_t)(payload) & 0x00ffffffffffffffULL))
#ifndef PV_CACHE_BUCKET
#define PV_CACHE_BUCKET 1 // a key probes the aligned 4-entry bucket of its hash, read with two 16-B loads (0: four
                          // dependent single-entry probes; C3 DNS pass 1024 -> 997 us, C4 498 -> 484, profiles/r4/ab)
#endif
template <int N>
struct KeyCache {
    alignas(16) uint64_t key[N];
    uint32_t cnt[N];
    uint32_t rep[N];
    __device__ __forceinline__ void clear()
    {
        for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) { key[i] = 0; cnt[i] = 0; rep[i] = 0xffffffffu; }
    }
    // adds w to key's count; returns false if the probe window is full. first = the
    // entry's smallest record index before this call (0xffffffff if new)
    __device__ __forceinline__ bool add(uint64_t k, uint32_t w, uint32_t idx, uint32_t &first)
    {
#if PV_CACHE_BUCKET
        // one LDS round trip for the whole probe window (a miss used to cost four dependent reads)
        const uint32_t b = (uint32_t)(fmix64(k) >> 32) & (N - 4);
        const uint4 *kp = reinterpret_cast<const uint4 *>(&key[b]);
        const uint4 lo = kp[0], hi = kp[1];
        uint64_t cur4[4] = {(uint64_t)lo.x | ((uint64_t)lo.y << 32), (uint64_t)lo.z | ((uint64_t)lo.w << 32),
                            (uint64_t)hi.x | ((uint64_t)hi.y << 32), (uint64_t)hi.z | ((uint64_t)hi.w << 32)};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint64_t cur = cur4[j];
            if (cur == 0) {
                const uint64_t prev = atomicCAS((unsigned long long *)&key[b + j], 0ull, (unsigned long long)k);
                cur = prev == 0 ? k : prev;
            }
            if (cur == k) {
                if (w) atomicAdd(&cnt[b + j], w);
                first = atomicMin(&rep[b + j], idx);
                return true;
            }
        }
        return false;
#endif
        uint32_t h = (uint32_t)(fmix64(k) >> 32) & (N - 1);
        for (int probe = 0; probe < PV_CACHE_PROBES; probe++) {
            uint64_t cur = key[h];
            if (cur == 0) {
                const uint64_t prev = atomicCAS((unsigned long long *)&key[h], 0ull, (unsigned long long)k);
                cur = prev == 0 ? k : prev;
            }
            if (cur == k) {
                if (w) atomicAdd(&cnt[h], w);
                first = atomicMin(&rep[h], idx);
                return true;
            }
            h = (h + 1) & (N - 1);
        }
        return false;
    }
};

// Top-N updates the LDS cache does not absorb go to the update log of the grid range being
// processed (fire-and-forget stores, slot in key bits 60..63); the top-N merge kernels apply
// the logs to the global tables after the parse kernels, so no lane waits on an HBM round trip
// for a table update. mq_n: the range's LDS log count, then the range (a workgroup may walk
// several ranges of the logical grid).
__device__ __forceinline__ void log_put(PV_CREF(PvParams) P, uint32_t *mq_n, uint32_t slot, uint64_t key, uint32_t w,
                                        uint32_t rep)
{
    const uint32_t q = atomicAdd(mq_n, 1u);
    PV_G uint64_t *e = P.mq + ((uint64_t)mq_n[1] * P.mq_cap + q) * 2;
    e[0] = (key & ((1ull << 60) - 1)) | ((uint64_t)slot << 60);
    e[1] = (uint64_t)w | ((uint64_t)rep << 32);
}
// dense tables (payload sizes, ports, qtypes, rcodes): no-return HBM atomics
__device__ __forceinline__ void sum_add(PV_CREF(PvParams) P, uint32_t slot, uint32_t word, uint64_t w)
{
    __hip_atomic_fetch_add(P.sum + (uint64_t)slot * PV_SUM_WORDS + word, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t dense_word(uint32_t metric, uint64_t payload)
{
    return metric == TM_DENSE_PORT ? PV_OFF_PORT + (uint32_t)(payload & 0xffff)
         : metric == TM_DENSE_QTYPE ? PV_OFF_QTYPE + (uint32_t)(payload & 0xffff)
                                    : PV_OFF_RCODE + (uint32_t)(payload & 0xf);
}
// cache-local metric ids (cache keys hold metric ids < 16; these two never reach the
// global tables): payload-size histogram bins and CPC qname coupons
#define LM_HIST TM_SLOW_OUT
#define LM_CPCQ TM_SLOW_IN
// CPC first occurrence: no-return atomicMin of the global record index
__device__ __forceinline__ void cpc_min(PV_CREF(PvParams) P, uint32_t slot, uint32_t sketch, uint32_t coupon, int64_t gidx)
{
    __hip_atomic_fetch_min(P.cpc + (uint64_t)slot * PV_MIN_WORDS + (uint64_t)sketch * PV_CPC_COUPONS + coupon, gidx,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
#define PV_FLUSH1(s, word, v, on)                                                       \
    {                                                                                   \
        const uint32_t t_ = wave_sum(v);                                                \
        if ((threadIdx.x & 63) == 0 && t_ && (on)) sum_add(P, s, word, t_);             \
    }

// Net v1 counters of the wave's current slot, in registers
struct NetCtr {
    uint32_t nev, nin, nout, nunk, n4, n6, nudp, ntcp, nsyn, noth, nfilt;
    __device__ __forceinline__ void zero() { nev = nin = nout = nunk = n4 = n6 = nudp = ntcp = nsyn = noth = nfilt = 0; }
    __device__ __forceinline__ void add(const Parsed &o)
    {
        nev++;
        nin += o.dir == 0; nout += o.dir == 1; nunk += o.dir == 2;
        n4 += o.l3 == 4; n6 += o.l3 == 6;
        nudp += o.l4 == 17; ntcp += o.l4 == 6; nsyn += o.l4 == 6 && o.syn; noth += o.l4 == 0;
    }
};
__device__ void net_flush(PV_CREF(PvParams) P, uint32_t s, NetCtr &c)
{
    const bool nc = P.net_groups & PV_NET_COUNTERS_BIT;
    PV_FLUSH1(s, PV_OFF_NET + NC_EVENTS, c.nev, true) PV_FLUSH1(s, PV_OFF_NET + NC_SAMPLES, c.nev, true)
    PV_FLUSH1(s, PV_OFF_NET + NC_TOTAL, c.nev, nc) PV_FLUSH1(s, PV_OFF_NET + NC_IN, c.nin, nc)
    PV_FLUSH1(s, PV_OFF_NET + NC_OUT, c.nout, nc) PV_FLUSH1(s, PV_OFF_NET + NC_UNK, c.nunk, nc)
    PV_FLUSH1(s, PV_OFF_NET + NC_V4, c.n4, nc) PV_FLUSH1(s, PV_OFF_NET + NC_V6, c.n6, nc)
    PV_FLUSH1(s, PV_OFF_NET + NC_UDP, c.nudp, nc) PV_FLUSH1(s, PV_OFF_NET + NC_TCP, c.ntcp, nc)
    PV_FLUSH1(s, PV_OFF_NET + NC_SYN, c.nsyn, nc) PV_FLUSH1(s, PV_OFF_NET + NC_OTHER, c.noth, nc)
    c.zero();
}
// DNS v1 counters of the wave's current slot
struct DnsCtr {
    uint32_t dev, dq, dr, d4, d6, dnx, dref, dsrv, dnoerr, dnodata, dfilt, dqecs, dnd;
    __device__ __forceinline__ void zero() { dev = dq = dr = d4 = d6 = dnx = dref = dsrv = dnoerr = dnodata = dfilt = dqecs = dnd = 0; }
};
__device__ __forceinline__ void dns_flush(PV_CREF(PvParams) P, uint32_t s, DnsCtr &c)
{
    const bool dc = P.dns_groups & PV_DNS_COUNTERS_BIT;
    PV_FLUSH1(s, PV_OFF_DNS + DC_EVENTS, c.dev + c.dfilt, true) PV_FLUSH1(s, PV_OFF_DNS + DC_SAMPLES, c.dev + c.dfilt - c.dnd, true)
    PV_FLUSH1(s, PV_OFF_DNS + DC_TOTAL, c.dev, dc) PV_FLUSH1(s, PV_OFF_DNS + DC_UDP, c.dev, dc)
    if (P.f_flags) PV_FLUSH1(s, PV_OFF_DNS + DC_FILTERED, c.dfilt, dc || (P.dns2_groups & PV_D2G_COUNTERS))
    PV_FLUSH1(s, PV_OFF_DNS + DC_QUERIES, c.dq, dc) PV_FLUSH1(s, PV_OFF_DNS + DC_REPLIES, c.dr, dc)
    PV_FLUSH1(s, PV_OFF_DNS + DC_V4, c.d4, dc) PV_FLUSH1(s, PV_OFF_DNS + DC_V6, c.d6, dc)
    PV_FLUSH1(s, PV_OFF_DNS + DC_NX, c.dnx, dc) PV_FLUSH1(s, PV_OFF_DNS + DC_REFUSED, c.dref, dc)
    PV_FLUSH1(s, PV_OFF_DNS + DC_SRVFAIL, c.dsrv, dc) PV_FLUSH1(s, PV_OFF_DNS + DC_NOERROR, c.dnoerr, dc)
    PV_FLUSH1(s, PV_OFF_DNS + DC_NODATA, c.dnodata, dc)
    if (P.dns_groups & PV_DNS_TOP_ECS_BIT) PV_FLUSH1(s, PV_OFF_DNS + DC_QECS, c.dqecs, dc)
    c.zero();
}

__device__ __forceinline__ uint32_t period_of(PV_CREF(PvParams) P, uint64_t i)
{
    uint32_t p = 0;
    while (p < P.n_shift && i >= P.pstart[p]) p++;
    return p;
}
// DNS period of the DNS event of span record i (the DNS manager's own shifts, in stream order:
// the event that shifts and every event after it belong to the new period, whatever their
// timestamps, as AbstractMetricsManager::new_event decides per event)
__device__ __forceinline__ uint32_t dperiod_of(PV_CREF(PvParams) P, uint64_t i)
{
    uint32_t p = 0;
    while (p < P.n_dshift && 4 * i >= (uint64_t)P.dpos[p]) p++;
    return p;
}
__device__ __forceinline__ uint64_t uni64(uint64_t v)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

// DNS over UDP: the message of one record, located by the Net pass
// (DnsStreamHandler::process_udp_packet_cb, :270-302)
struct alignas(16) DnsMsg {
    uint32_t idx;     // record index in the batch
    uint32_t moff;    // absolute byte offset of the DNS header in the record blob
    uint16_t mlen;    // UDP payload length (IP-length trimmed)
    uint16_t mcap;    // bytes of the message inside the capture
    uint16_t port;    // metric port
    uint8_t flags;    // bit0-1 dir, bit2 IPv6, bit3 update buckets (period inside the window)
    uint8_t period;
    uint32_t fkey;    // hash5Tuple
    uint32_t sec;
    uint32_t nsec;
    uint32_t pad;
};
static_assert(sizeof(DnsMsg) == 32, "DnsMsg is two 16-B stores");
// a DnsMsg as its two 16-B words, composed dword by dword (field-wise stores of the
// struct would split into sub-dword stores)
struct DnsMsgW {
    uint4 a, b;
};
__device__ __forceinline__ DnsMsgW msg_words(const DnsMsg &d)
{
    DnsMsgW w;
    w.a = make_uint4(d.idx, d.moff, (uint32_t)d.mlen | ((uint32_t)d.mcap << 16),
                     (uint32_t)d.port | ((uint32_t)d.flags << 16) | ((uint32_t)d.period << 24));
    w.b = make_uint4(d.fkey, d.sec, d.nsec, 0u);
    return w;
}
__device__ __forceinline__ void put_msg(PV_G DnsMsg *dst, const DnsMsgW &w)
{
    PV_G uint4 *p = reinterpret_cast<PV_G uint4 *>(dst);
    p[0] = w.a;
    p[1] = w.b;
}

// Metric port of a UDP datagram (0 = not DNS), from the raw port word
__device__ __forceinline__ uint32_t dns_port(uint32_t pw)
{
    const uint32_t sport = ((pw & 0xff) << 8) | ((pw >> 8) & 0xff);
    const uint32_t dport = ((pw >> 8) & 0xff00) | (pw >> 24);
    if (dport == 53 || dport == 5353 || dport == 5355 || dport == 53000) return sport;
    if (sport == 53 || sport == 5353 || sport == 5355 || sport == 53000) return dport;
    return 0;
}
template <class A>
__device__ __forceinline__ DnsMsg dns_msg_of(PV_CREF(PvParams) P, const A &R, const Parsed &o, uint64_t i, uint32_t port,
                                             uint32_t period, bool upd, bool with_key = true)
{
    DnsMsg d;
    d.idx = (uint32_t)i;
    d.moff = (uint32_t)(o.l4off + 8);
    d.mlen = (uint16_t)(o.l4len - 8);
    const uint64_t cap_end = o.frame + o.caplen;
    d.mcap = (uint16_t)(cap_end > o.l4off + 8 ? min<uint64_t>(cap_end - (o.l4off + 8), 65535) : 0);
    d.port = (uint16_t)port;
    d.flags = (uint8_t)(o.dir | (o.l3 == 6 ? 4 : 0) | (upd ? 8 : 0));
    d.period = (uint8_t)period;
    d.fkey = with_key ? flowkey(R, o) : 0u;
    d.sec = (uint32_t)o.sec;
    d.nsec = (uint32_t)o.nsec;
    d.pad = 0;
    return d;
}

// The 12 header bytes of a DNS message as three little-endian words; bytes past the
// capture read as 0 (the reference over-reads there)
template <class A>
__device__ __forceinline__ void dns_header(const A &R, uint64_t m, uint32_t mcap, uint32_t &w0, uint32_t &w1, uint32_t &w2)
{
    if (mcap >= 12) { w0 = R.u32(m); w1 = R.u32(m + 4); w2 = R.u32(m + 8); return; }
    w0 = w1 = w2 = 0;
    for (uint32_t b = 0; b < 12; b++) {
        const uint32_t v = b < mcap ? R.u8(m + b) : 0;
        if (b < 4) w0 |= v << (8 * b); else if (b < 8) w1 |= v << (8 * (b - 4)); else w2 |= v << (8 * (b - 8));
    }
}
// The input proxy's UDP predicates (PcapInputEventProxy::process_udp_packet_cb,
// src/inputs/pcap/PcapInputStream.h:213-252, installed by DnsStreamHandler's
// _register_predicate_filter, dns/v1/DnsStreamHandler.cpp:485-537): only_rcode passes a
// response whose rcode is listed; only_qname a message whose lower-case first-query name is
// listed. A packet they reject never reaches the handler (no event, no window shift).
// only_qname: the lower-case first-query name is listed
template <class A>
__device__ __forceinline__ bool dns_qname_listed(PV_CREF(PvParams) P, const A &R, uint64_t m, uint32_t dlen, uint32_t w1,
                                                 uint32_t w2)
{
    const uint32_t qd = ((w1 & 0xff) << 8) | ((w1 >> 8) & 0xff), an = ((w1 >> 8) & 0xff00) | (w1 >> 24);
    const uint32_t ns = ((w2 & 0xff) << 8) | ((w2 >> 8) & 0xff), ar = ((w2 >> 8) & 0xff00) | (w2 >> 24);
    DnsInfo qi;
    dns_parse(R, m, dlen, qd, an, ns, ar, qi);
    bool hit = false;
    if (qi.ok && qi.has_query && qi.name_len_enc > 0) {
        NameStats st;
        st.init();
        name_stats(R, m, dlen, 12, st);
        const uint64_t fp = fp56(st.ph, st.n, 0);
        for (uint32_t k = 0; k < P.f_nqn; k++) hit |= st.n > 0 && fp == P.f_qn[k];
    }
    return hit;
}
template <class A>
__device__ __forceinline__ bool dns_predicates(PV_CREF(PvParams) P, const A &R, uint64_t m, uint32_t dlen, uint32_t w0,
                                               uint32_t w1, uint32_t w2)
{
    const uint32_t qr = (w0 >> 23) & 1, rcode = (w0 >> 24) & 15;
    if ((P.f_flags & PVDF_ONLY_RCODE) && (!qr || !((P.f_rcode_mask >> rcode) & 1))) return false;
    if ((P.f_flags & PVDF_ONLY_QNAME) && !dns_qname_listed(P, R, m, dlen, w1, w2)) return false;
    return true;
}

// DnsStreamHandler::_filtering, v1 (:538-648), for a message the input predicates passed: true
// when it is filtered (process_filtered). The deep-sampling prescans use it to know which events
// draw (a filtered one takes the manager's stale flag); it restates the filter block of
// dns_process below, with the suffix match (0xff: no listed suffix) computed here.
template <class A>
__device__ bool dns_v1_filtered(PV_CREF(PvParams) P, const A &R, uint64_t m, uint32_t dlen, uint32_t mcap, bool tcp)
{
    uint32_t w0, w1, w2;
    dns_header(R, m, mcap, w0, w1, w2);
    const uint32_t qr = (w0 >> 23) & 1, rcode = (w0 >> 24) & 15;
    const uint32_t qd = ((w1 & 0xff) << 8) | ((w1 >> 8) & 0xff);
    const uint32_t ancount = ((w1 >> 8) & 0xff00) | (w1 >> 24);
    const uint32_t ns = ((w2 & 0xff) << 8) | ((w2 >> 8) & 0xff);
    const uint32_t ar = ((w2 >> 8) & 0xff00) | (w2 >> 24);
    bool filt = ((P.f_flags & PVDF_EXCLUDE_NOERROR) && rcode == 0) ||
                (tcp && (P.f_flags & PVDF_ONLY_RCODE) && !((P.f_rcode_mask >> rcode) & 1)) ||
                ((P.f_flags & PVDF_ANSWER_COUNT) && ancount != P.f_ancount) ||
                ((P.f_flags & PVDF_ONLY_QUERIES) && qr) || ((P.f_flags & PVDF_ONLY_RESPONSES) && !qr) ||
                ((P.f_flags & PVDF_ONLY_DNSSEC) && (!qr || !ancount || !dns_dnssec(R, m, dlen, qd, ancount, ns, ar))) ||
                (P.f_flags & PVDF_FILTER_ALL);
    if (!filt && (P.f_flags & PVDF_ONLY_QTYPE)) {
        DnsInfo fd;
        dns_parse(R, m, dlen, qd, ancount, ns, ar, fd);
        bool hit = false;
        for (uint32_t k = 0; k < P.f_nq; k++) hit |= fd.qtype == P.f_qt[k];
        filt = !fd.ok || !fd.has_query || !hit;
    }
    if (!filt && tcp && (P.f_flags & PVDF_ONLY_QNAME)) filt = !dns_qname_listed(P, R, m, dlen, w1, w2);
    if (!filt && (P.f_flags & PVDF_ONLY_QSUFFIX)) filt = dns_suffix_of(P, R, m, dlen, qd, ancount, ns, ar) == 0xffu;
    return filt;
}
// DnsStreamHandler::_filtering, v2 (dns/v2/DnsStreamHandler.cpp:484-609), for the deep-sampling
// prescans: the filter block of dns_process's PVDF_V2 branch below, restated with the suffix
// match computed here. dir: 0 toHost, 1 fromHost, 2 unknown.
template <class A>
__device__ bool dns_v2_filtered(PV_CREF(PvParams) P, const A &R, uint64_t m, uint32_t dlen, uint32_t mcap, uint32_t dir)
{
    uint32_t w0, w1, w2;
    dns_header(R, m, mcap, w0, w1, w2);
    const uint32_t qr = (w0 >> 23) & 1, rcode = (w0 >> 24) & 15;
    const uint32_t qd = ((w1 & 0xff) << 8) | ((w1 >> 8) & 0xff);
    const uint32_t ancount = ((w1 >> 8) & 0xff00) | (w1 >> 24);
    const uint32_t ns = ((w2 & 0xff) << 8) | ((w2 >> 8) & 0xff);
    const uint32_t ar = ((w2 >> 8) & 0xff00) | (w2 >> 24);
    bool filt = (P.f_flags & PVDF2_NOUNK) && dir == 2;
    if (!filt && qr) {
        filt = ((P.f_flags & PVDF2_NOIN) && dir == 1) || ((P.f_flags & PVDF2_NOOUT) && dir == 0) ||
               ((P.f_flags & PVDF2_RCODE) && !((P.f_rcode_mask >> rcode) & 1)) ||
               ((P.f_flags & PVDF_ANSWER_COUNT) && ancount != P.f_ancount) ||
               ((P.f_flags & PVDF_ONLY_DNSSEC) && (!ancount || !dns_dnssec(R, m, dlen, qd, ancount, ns, ar)));
        if (!filt && (P.f_flags & PVDF_ONLY_QTYPE)) {
            DnsInfo fd;
            dns_parse(R, m, dlen, qd, ancount, ns, ar, fd);
            bool hit = false;
            for (uint32_t k = 0; k < P.f_nq; k++) hit |= fd.qtype == P.f_qt[k];
            filt = !fd.ok || !fd.has_query || !hit;
        }
    } else if (!filt) {
        filt = ((P.f_flags & PVDF2_NOIN) && dir == 0) || ((P.f_flags & PVDF2_NOOUT) && dir == 1);
        if (!filt && (P.f_flags & PVDF2_QNAME)) filt = !dns_qname_listed(P, R, m, dlen, w1, w2);
        if (!filt && (P.f_flags & PVDF_ONLY_QSUFFIX)) filt = dns_suffix_of(P, R, m, dlen, qd, ancount, ns, ar) == 0xffu;
    }
    return filt;
}
template <class A>
__device__ __forceinline__ bool dns_filtered(PV_CREF(PvParams) P, const A &R, uint64_t m, uint32_t dlen, uint32_t mcap, bool tcp,
                                             uint32_t dir)
{
    return (P.f_flags & PVDF_V2) ? dns_v2_filtered(P, R, m, dlen, mcap, dir) : dns_v1_filtered(P, R, m, dlen, mcap, tcp);
}

// DnsMetricsBucket::process_dns_layer (:910-1049) + the transaction event of one DNS
// message, in the bucket of its DNS period. Counters go to `c` when `own` (this lane's
// DNS slot is the wave's register slot), else straight to HBM.
// TAP: a dnstap event (DnsMetricsBucket::process_dnstap, :839-909): no filters, l3 / l4 from
// the socket fields (flags bit 4: l3 unknown; bits 5-6: 0 UDP, 1 TCP, 2 other), the query
// port as the port (top_udp_ports only when non-zero), no transaction event.
// FILT: the DNS filter blocks compiled in (the common pass of an unfiltered context has none:
// their code would cost it registers even when no filter is set)
template <bool TCP, bool TAP = false, bool SFX = true, bool FILT = true, class A, class Cache>
__device__ __forceinline__ void dns_process(PV_CREF(PvParams) P, Cache *cache, uint32_t *mq_n, uint32_t *nev,
                                            uint32_t *nresp, uint64_t ebase, const A &R, const DnsMsg &dm, bool own,
                                            DnsCtr &c)
{
    const bool upd = dm.flags & 8;
    const uint32_t period = dm.period;
    const uint32_t slot = dslot(P, period);
    const uint64_t m = dm.moff;
    const uint32_t dlen = dm.mlen;
    const uint32_t i = dm.idx;
    uint32_t w0, w1, w2;
    dns_header(R, m, dm.mcap, w0, w1, w2);
    const uint32_t txid = ((w0 & 0xff) << 8) | ((w0 >> 8) & 0xff);
    const uint32_t qr = (w0 >> 23) & 1;
    const uint32_t rcode = (w0 >> 24) & 15;
    const uint32_t qd = ((w1 & 0xff) << 8) | ((w1 >> 8) & 0xff);
    const uint32_t ancount = ((w1 >> 8) & 0xff00) | (w1 >> 24);
    const uint32_t ns = ((w2 & 0xff) << 8) | ((w2 >> 8) & 0xff);
    const uint32_t ar = ((w2 >> 8) & 0xff00) | (w2 >> 24);
    uint32_t sfx = 0; // only_qname_suffix's suffix_size for aggregateDomain
    // a message's order in the span: record * 4 (+ sub for a TCP message), for the CPC
    // first-occurrence index and the transaction sort rank
    const uint32_t ordr = (TCP || TAP) ? dm.pad - P.ord_base : (i << 2);
    // the message's transaction event (filtered: a DNS v2 event its filters rejected, which
    // still opens or ends a transaction, DnsMetricsManager::process_filtered, dns/v2 ...cpp:1147-1174)
    auto emit = [&](bool deep, bool filtered, uint32_t efam, uint64_t eaddr) {
        if (!P.want_events || TAP || (P.dbg & 1024)) return; // 1024: profiling knob, no events
        // the workgroup's event region; LDS counter, order irrelevant (sorted by key, index)
        const uint64_t e = ebase + atomicAdd(nev, 1u);
        if (qr) atomicAdd(nresp, 1u);
        PvXEvent ev;
        ev.key = ((uint64_t)dm.fkey << 16) | txid;
        ev.idx = TCP ? (i | PV_TCP_IDX) : i;
        ev.len = dlen;
        ev.sec = dm.sec;
        ev.nsec = (int32_t)dm.nsec;
        ev.qr = (uint8_t)qr;
        ev.dir = dm.flags & 3;
        ev.period = (uint8_t)period;
        ev.pad = deep ? 0 : 4; // v1: bit 2 = the event is not deep
        if (P.dns2_groups) {
            // DNS v2: one transaction map per direction (DnsMetricsManager::_pair_manager); a
            // response looks in the swapped direction's map (dns/v2 ...cpp:1100-1145). pad: the
            // query's CD bit, the message's l3 (bit 1: IPv6), bit 2: filtered, bits 3-4: the
            // ECS family, bit 5: not deep (a response's draw decides new_dns_transaction's deep part)
            const uint32_t dir = dm.flags & 3;
            const uint32_t xd = dir == 2 ? 2u : (qr ? dir ^ 1u : dir);
            ev.key |= (uint64_t)(xd + 1) << 48;
            ev.pad = (uint8_t)(((w0 >> 28) & 1) | ((dm.flags & 4) ? 2u : 0u) | (filtered ? 4u : 0u) | (efam << 3) |
                              (deep ? 0u : 32u));
            if (efam) P.eecs[e] = eaddr;
        }
        P.events[e] = ev;
        const uint64_t sk = xact_sort_key(ev.key, (P.ekey_base << 2) + ordr);
        if constexpr (!TCP && !TAP) {
            // the UDP pass: straight into the batch's key list at the range's reserved slots
            // (nev[1]: one per DNS message of the range; pv_xact_compact's work for these ranges)
            const uint64_t ks = (uint64_t)nev[1] + (e - ebase);
            P.skeys[ks] = sk;
            P.svals[ks] = (uint32_t)e;
        } else {
            P.ekeys[e] = sk;
        }
    };
    if (FILT && (P.f_flags & PVDF_V2) && !TAP) {
        // DnsStreamHandler::_filtering, DNS v2 (dns/v2/DnsStreamHandler.cpp:484-609): the
        // direction filters for both, the rcode / answer / DNSSEC / qtype filters on responses,
        // the qname filters on queries; no input predicate (every DNS packet is an event)
        const uint32_t dir = dm.flags & 3; // 0 toHost, 1 fromHost, 2 unknown
        bool filt = (P.f_flags & PVDF2_NOUNK) && dir == 2;
        if (!filt && qr) {
            filt = ((P.f_flags & PVDF2_NOIN) && dir == 1) || ((P.f_flags & PVDF2_NOOUT) && dir == 0) ||
                   ((P.f_flags & PVDF2_RCODE) && !((P.f_rcode_mask >> rcode) & 1)) ||
                   ((P.f_flags & PVDF_ANSWER_COUNT) && ancount != P.f_ancount) ||
                   ((P.f_flags & PVDF_ONLY_DNSSEC) && (!ancount || !dns_dnssec(R, m, dlen, qd, ancount, ns, ar)));
            if (!filt && (P.f_flags & PVDF_ONLY_QTYPE)) {
                DnsInfo fd;
                dns_parse(R, m, dlen, qd, ancount, ns, ar, fd);
                bool hit = false;
                for (uint32_t k = 0; k < P.f_nq; k++) hit |= fd.qtype == P.f_qt[k];
                filt = !fd.ok || !fd.has_query || !hit;
            }
        } else if (!filt) {
            filt = ((P.f_flags & PVDF2_NOIN) && dir == 0) || ((P.f_flags & PVDF2_NOOUT) && dir == 1);
            if (!filt && (P.f_flags & PVDF2_QNAME)) filt = !dns_qname_listed(P, R, m, dlen, w1, w2);
            if constexpr (SFX) {
                if (!filt && (P.f_flags & PVDF_ONLY_QSUFFIX)) filt = P.sfx_of[i] == 0xffu;
            }
        }
        if (filt) {
            // process_filtered: an event counted deep when the manager's stale flag is (the
            // not-deep bit deep sampling sets), `filtered`, and the transaction
            const bool fdeep = !(dm.flags & 16);
            if (upd) {
                if (own) { c.dfilt++; c.dnd += !fdeep; }
                else {
                    sum_add(P, slot, PV_OFF_DNS + DC_EVENTS, 1);
                    if (fdeep) sum_add(P, slot, PV_OFF_DNS + DC_SAMPLES, 1);
                    if (P.dns2_groups & PV_D2G_COUNTERS) sum_add(P, slot, PV_OFF_DNS + DC_FILTERED, 1);
                }
            }
            emit(true, true, 0, 0);
            return;
        }
    } else if (FILT && P.f_flags && !TAP) {
        // a TCP message takes no input predicate: _filtering applies only_rcode and only_qname
        // to it as ordinary filters (_predicate_filter_type stays FiltersMAX, :546-551,593-602)
        if (!TCP && (P.f_flags & (PVDF_ONLY_RCODE | PVDF_ONLY_QNAME)) && !dns_predicates(P, R, m, dlen, w0, w1, w2)) return;
        // DnsStreamHandler::_filtering (:538-648), in its order
        bool filt = ((P.f_flags & PVDF_EXCLUDE_NOERROR) && rcode == 0) ||
                    (TCP && (P.f_flags & PVDF_ONLY_RCODE) && !((P.f_rcode_mask >> rcode) & 1)) ||
                    ((P.f_flags & PVDF_ANSWER_COUNT) && ancount != P.f_ancount) ||
                    ((P.f_flags & PVDF_ONLY_QUERIES) && qr) || ((P.f_flags & PVDF_ONLY_RESPONSES) && !qr) ||
                    ((P.f_flags & PVDF_ONLY_DNSSEC) && (!qr || !ancount || !dns_dnssec(R, m, dlen, qd, ancount, ns, ar))) ||
                    (P.f_flags & PVDF_FILTER_ALL);
        if (!filt && (P.f_flags & PVDF_ONLY_QTYPE)) {
            DnsInfo fd;
            dns_parse(R, m, dlen, qd, ancount, ns, ar, fd);
            bool hit = false;
            for (uint32_t k = 0; k < P.f_nq; k++) hit |= fd.qtype == P.f_qt[k];
            filt = !fd.ok || !fd.has_query || !hit;
        }
        if (!filt && TCP && (P.f_flags & PVDF_ONLY_QNAME)) filt = !dns_qname_listed(P, R, m, dlen, w1, w2);
        // only_qname_suffix, or _configs' public_suffix_list (:648-657, never 0xff): matched by
        // pv_dns_suffix before this pass (0xff: no listed suffix); such runs use the SFX pass
        if constexpr (SFX) {
            if (!filt && (P.f_flags & (PVDF_ONLY_QSUFFIX | PVDF_PSL))) {
                const uint32_t r = P.sfx_of[i];
                filt = r == 0xffu;
                sfx = filt ? 0u : r;
            }
        } else if (!filt && (P.f_flags & PVDF_ONLY_QSUFFIX)) {
            const uint32_t r = P.sfx_of[i]; // not launched this way (host picks the SFX pass)
            filt = r == 0xffu;
            sfx = filt ? 0u : r;
        }
        if (filt) {
            // process_filtered (:1341-1347): an event, counted deep when the manager's stale
            // flag is (the not-deep bit deep sampling sets), and `filtered`
            const bool fdeep = !(dm.flags & 16);
            if (upd) {
                if (own) { c.dfilt++; c.dnd += !fdeep; }
                else {
                    sum_add(P, slot, PV_OFF_DNS + DC_EVENTS, 1);
                    if (fdeep) sum_add(P, slot, PV_OFF_DNS + DC_SAMPLES, 1);
                    if (P.dns_groups & PV_DNS_COUNTERS_BIT) sum_add(P, slot, PV_OFF_DNS + DC_FILTERED, 1);
                }
            }
            return;
        }
    }
    // top-N / dense update: cache, else log (hashed) or HBM atomic (dense); boundary: global table
    // (the UDP pass always has the cache: no call to global_add is compiled into it, so its
    // registers and scratch follow no call convention)
    auto top = [&](uint32_t metric, uint64_t payload, uint32_t w) {
        const uint64_t key = PV_KEY(metric, payload);
        if (P.dbg & 32) return; // profiling knob: no table updates
        if constexpr (!TCP && !TAP) {
            uint32_t first;
            if (cache->add(PV_LKEY(slot, metric, payload), w, i, first)) return;
            if (metric >= TM_DENSE_PORT) sum_add(P, slot, dense_word(metric, payload), w);
            else log_put(P, mq_n, slot, key, w, i);
        } else {
            global_add(P, slot, key, w, i);
        }
    };
    // deep sampling: an event that drew "not deep" counts as an event and in the counters only
    // (DnsMetricsBucket::process_dns_layer !deep, dns/v1/DnsStreamHandler.cpp:968-970); its
    // transaction still pairs, and a response's flag decides new_dns_transaction's deep part
    const bool deep = TAP || !(dm.flags & 16);
    if (upd) {
        const uint32_t l3u = TAP && (dm.flags & 16);
        const uint32_t d4 = !(dm.flags & 4) && !l3u, d6 = (dm.flags & 4) ? 1 : 0;
        const uint32_t l4c = TAP ? (dm.flags >> 5) & 3 : (TCP ? 1u : 0u); // 0 UDP, 1 TCP, 2 other
        if (own) {
            c.dev++;
            c.dnd += !deep;
            c.d4 += d4; c.d6 += d6;
            c.dq += !qr; c.dr += qr;
            c.dnoerr += qr && rcode == 0; c.dnodata += qr && rcode == 0 && ancount == 0;
            c.dsrv += qr && rcode == 2; c.dnx += qr && rcode == 3; c.dref += qr && rcode == 5;
        } else {
            const bool dc = P.dns_groups & PV_DNS_COUNTERS_BIT;
            sum_add(P, slot, PV_OFF_DNS + DC_EVENTS, 1);
            if (deep) sum_add(P, slot, PV_OFF_DNS + DC_SAMPLES, 1);
            if (dc) {
                sum_add(P, slot, PV_OFF_DNS + DC_TOTAL, 1);
                if (l4c < 2) sum_add(P, slot, PV_OFF_DNS + (l4c ? DC_TCP : DC_UDP), 1);
                if (d4 | d6) sum_add(P, slot, PV_OFF_DNS + (d6 ? DC_V6 : DC_V4), 1);
                sum_add(P, slot, PV_OFF_DNS + (qr ? DC_REPLIES : DC_QUERIES), 1);
                if (qr && rcode == 0) sum_add(P, slot, PV_OFF_DNS + DC_NOERROR, 1);
                if (qr && rcode == 0 && ancount == 0) sum_add(P, slot, PV_OFF_DNS + DC_NODATA, 1);
                if (qr && rcode == 2) sum_add(P, slot, PV_OFF_DNS + DC_SRVFAIL, 1);
                if (qr && rcode == 3) sum_add(P, slot, PV_OFF_DNS + DC_NX, 1);
                if (qr && rcode == 5) sum_add(P, slot, PV_OFF_DNS + DC_REFUSED, 1);
            }
        }
        if (deep) {
        DnsInfo d;
        dns_parse(R, m, dlen, qd, ancount, ns, ar, d);
        // client ports spread over 64 K values and rarely repeat inside a workgroup: a
        // no-return HBM atomic on the dense table, not an LDS cache probe (boundary: as before)
        if ((P.dns_groups & PV_DNS_TOP_PORTS_BIT) && (!TAP || dm.port)) {
            if (cache && !(P.dbg & 32)) sum_add(P, slot, PV_OFF_PORT + (dm.port & 0xffff), 1);
            else top(TM_DENSE_PORT, dm.port, 1);
        }
        if (d.ok) {
            if (qr) top(TM_DENSE_RCODE, rcode, 1);
            if (d.has_query) {
                NameStats st;
                st.init();
                if (d.name_len_enc > 0 && !(P.dbg & 16)) name_stats(R, m, dlen, 12, st);
                uint64_t h1, h2;
                st.mm.finish(h1, h2);
                if (st.n > 0 && (P.dns_groups & PV_DNS_CARDINALITY_BIT) && !(P.dbg & 512)) { // 512: knob, no qname CPC
                    const uint32_t coupon = cpc_coupon(h1, h2);
                    uint32_t first = 0xffffffffu;
                    // same name => same coupon: skip when a smaller record index already submitted it
                    if (!(cache && cache->add(PV_LKEY(slot, LM_CPCQ, coupon), 0, i, first) && first < i))
                        cpc_min(P, slot, CPC_QNAME, coupon, (int64_t)((P.gbase << 2) + ordr));
                }
                top(TM_DENSE_QTYPE, d.qtype, 1);
                if (P.dns_groups & PV_DNS_TOP_QNAMES_BIT) {
                    const uint64_t fp_full = fp56(st.ph, st.n, 0);
                    if (qr) {
                        if (rcode == 2) top(TM_SRVFAIL, fp_full, 1);
                        else if (rcode == 3) top(TM_NX, fp_full, 1);
                        else if (rcode == 5) top(TM_REFUSED, fp_full, 1);
                        else if (rcode == 0) {
                            if (P.dns_groups & PV_DNS_TOP_QNAMES_DETAILS_BIT) top(TM_NOERROR, fp_full, 1);
                            if (!ancount) top(TM_NODATA, fp_full, 1);
                        }
                        if (P.dns_groups & PV_DNS_TOP_QNAMES_DETAILS_BIT) top(TM_SIZED, fp_full, dlen);
                    }
                    int q2, q3;
                    uint64_t h2p, h3p;
                    // SFX: a suffix size may be set (only_qname_suffix / public_suffix_list runs);
                    // the common pass (sfx always 0) carries no re-walk code
                    if constexpr (SFX) agg_domain_r(R, m, dlen, st, q2, q3, h2p, h3p, sfx);
                    else agg_domain(st, q2, q3, h2p, h3p, sfx);
                    const uint64_t k2 = q2 == 0 ? st.ph : suffix_hash(st, q2, h2p);
                    top(TM_QNAME2, fp56(k2, st.n - q2, 0), 1);
                    if (q3 >= 0 && (uint32_t)q3 < st.n) {
                        const uint64_t k3 = q3 == 0 ? st.ph : suffix_hash(st, q3, h3p);
                        top(TM_QNAME3, fp56(k3, st.n - q3, 0), 1);
                    }
                }
            }
            // top_ecs (DnsMetricsBucket::process_dns_layer :1026-1048): a query's EDNS Client Subnet
            if ((P.dns_groups & PV_DNS_TOP_ECS_BIT) && !qr && ar) {
                uint64_t addr;
                const uint32_t fam = dns_ecs(R, m, dlen, qd, ancount, ns, ar, addr);
                if (fam) {
                    if (own) c.dqecs++;
                    else if (P.dns_groups & PV_DNS_COUNTERS_BIT) sum_add(P, slot, PV_OFF_DNS + DC_QECS, 1);
                    const uint64_t ek = PV_KEY(TM_ECS, fmix64(addr ^ ((uint64_t)fam << 62) ^ 0xec5ull));
                    if constexpr (TCP || TAP) global_add(P, slot, ek, 1, i);
                    else {
                        // listed for pv_dns_ecs (one per record at most: the list holds the batch)
                        const uint32_t q = atomicAdd(P.n_ecs, 1u);
                        if (q < P.ecs_cap) reinterpret_cast<PV_G uint4 *>(P.ecs_list)[q] = make_uint4((uint32_t)ek, (uint32_t)(ek >> 32), slot, (uint32_t)i);
                        else atomicOr(P.flags, PVF_TABLE_FULL);
                    }
                }
            }
        }
        }
    }
    if (!TAP && (P.dns2_groups & PV_D2G_TOP_ECS) && !qr && ar) {
        // DNS v2 top_ecs: the query's EDNS Client Subnet rides with its transaction event (the
        // subnet DnsMetricsManager::process_dns_layer hands start_transaction, dns/v2 ...cpp:1131-1144)
        uint64_t addr;
        const uint32_t fam = dns_ecs(R, m, dlen, qd, ancount, ns, ar, addr);
        emit(deep, false, fam, addr);
        return;
    }
    emit(deep, false, 0, 0);
}

// Flush a workgroup's key cache: hashed keys to the update log, dense keys to HBM.
template <class Cache>
__device__ __forceinline__ void cache_flush(PV_CREF(PvParams) P, Cache &C, uint32_t n, uint32_t *mq_n)
{
    for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
        const uint64_t k = C.key[j];
        if (!k || !C.cnt[j]) continue;
        const uint32_t slot = (uint32_t)(k >> 60), lm = (uint32_t)(k >> 56) & 15;
        const uint64_t pay = k & 0x00ffffffffffffffULL;
        if (lm >= TM_DENSE_PORT) sum_add(P, slot, dense_word(lm, pay), C.cnt[j]);
        else if (lm == LM_HIST) sum_add(P, slot, PV_OFF_PAYLOAD + (uint32_t)(pay & 0xffff), C.cnt[j]);
        else if (lm == TM_IPV4) log_put(P, mq_n, slot, PV_KEY(TM_IPV4, pay & 0xffffffffu), C.cnt[j], C.rep[j]);
        else if (lm == TM_IPV6) log_put(P, mq_n, slot, PV_KEY(TM_IPV6, pay & ((1ull << 55) - 1)), C.cnt[j], C.rep[j]);
        else if (lm != LM_CPCQ) log_put(P, mq_n, slot, PV_KEY(lm, pay), C.cnt[j], C.rep[j]);
    }
}

#define PV_WT 64      // records per wave tile
#define PV_WSTAGE 8192 // DNS pass: LDS staging bytes per wave (128-B message windows)
#ifndef PV_NCACHE
#define PV_NCACHE 4096 // DNS-pass key cache entries (4096: C3 combine + merge 573 -> 543 us, profiles/r3_s2/nc4096)
#endif
static_assert(PV_NCACHE <= PV_CACHE_MAX, "update log sized for PV_CACHE_MAX cache entries per flush");

#ifndef PV_HBINS
#define PV_HBINS 2048 // payload-size bins the Net pass keeps in LDS (larger sizes: HBM atomics)
#endif
#define PV_NOH 0xffffffffu
struct DnsState {
    uint32_t stage[PV_DNS_WAVES][PV_WSTAGE / 4];
    KeyCache<PV_NCACHE> C;
    uint4 desc[PV_DNS_WAVES][2][PV_WT]; // each wave's staged tile: its lanes' message descriptors (DnsMsgW words)
    uint32_t mq_n[2]; // the range's update-log count, the range
    uint32_t nev[2];  // the range's event count, its first slot in the batch's key list
    uint32_t nresp;
    uint32_t nlong;   // the range's messages past the LDS window (decoded after the range's tiles)
};
#ifndef PV_DNS_LACC
#define PV_DNS_LACC 1 // tuning: 0 decodes every message with the HBM-backed window accessor (TAcc)
#endif

// Adds one to bin v for every lane with v != PV_NOH: bins below PV_HBINS in the LDS
// histogram H, larger ones straight to the HBM table G (G[v]: the slot's payload-size words).
// The two most common values of the wave are added once each by a leader lane (packet sizes
// repeat: a whole wave often shares one), the rest per lane.
__device__ __forceinline__ void hist_add(uint32_t *H, PV_G uint64_t *G, uint32_t v, uint32_t lane)
{
    uint64_t m = __ballot(v != PV_NOH);
    for (int it = 0; it < 2 && m; it++) {
        const uint32_t ld = (uint32_t)__builtin_ctzll(m);
        const uint32_t lv = __builtin_amdgcn_readlane(v, ld);
        const uint64_t eq = __ballot(v == lv);
        if (lane == ld) {
            if (lv < PV_HBINS) atomicAdd(&H[lv], (uint32_t)__popcll(eq));
            else __hip_atomic_fetch_add(G + lv, (uint64_t)__popcll(eq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (v == lv) v = PV_NOH;
        m &= ~eq;
    }
    if (v != PV_NOH) {
        if (v < PV_HBINS) atomicAdd(&H[v], 1u);
        else __hip_atomic_fetch_add(G + v, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Loop-invariant values of the Net pass, read from the parameter block once: inside the
// record loop nothing waits on a scalar load (a scalar-load wait also drains the wave's
// LDS operations).
struct NetK {
    const PV_G uint8_t *recs;
    const PV_G uint32_t *offs;
    uint64_t n, rec_bytes, gbase;
    PV_G uint64_t *sum;
    PV_G int64_t *cpc;
    PV_G uint64_t *iplog;
    PV_G uint64_t *dq;
    PV_G uint32_t *flags;
    uint32_t n_shift, skip_before, slot0, net_groups, dbg, net_filter_all, n_dshift, dskip_before;
    uint32_t tcp_emit, tseg_cap;
    PV_G PvTcpSeg *tseg;
    PV_G uint32_t *tseg_cnt;
    PV_G uint64_t *tmask;
    const PV_G uint32_t *ndeep_net, *ndeep_dns; // deep sampling (general pass only)
};
// Net v1 counters of one record straight to HBM (a lane whose slot is not the wave's
// register slot: records of a 64-record tile that holds a period shift)
__device__ __noinline__ void knet_direct(PV_G uint64_t *sum, uint32_t net_groups, uint32_t s, uint32_t dir, uint32_t l3,
                                         uint32_t l4, uint32_t syn)
{
    PV_G uint64_t *b = sum + (uint64_t)s * PV_SUM_WORDS + PV_OFF_NET;
    auto add = [&](uint32_t w) { __hip_atomic_fetch_add(b + w, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    add(NC_EVENTS);
    add(NC_SAMPLES);
    if (!(net_groups & PV_NET_COUNTERS_BIT)) return;
    add(NC_TOTAL);
    add(dir == 0 ? NC_IN : (dir == 1 ? NC_OUT : NC_UNK));
    if (l3) add(l3 == 4 ? NC_V4 : NC_V6);
    add(l4 == 17 ? NC_UDP : (l4 == 6 ? NC_TCP : NC_OTHER));
    if (l4 == 6 && syn) add(NC_SYN);
}
__device__ __forceinline__ void ksum_add(const NetK &K, uint32_t slot, uint32_t word, uint64_t w)
{
    __hip_atomic_fetch_add(K.sum + (uint64_t)slot * PV_SUM_WORDS + word, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void kcpc_min(const NetK &K, uint32_t slot, uint32_t sketch, uint32_t coupon, uint64_t i)
{
    __hip_atomic_fetch_min(K.cpc + (uint64_t)slot * PV_MIN_WORDS + (uint64_t)sketch * PV_CPC_COUPONS + coupon,
                           (int64_t)(K.gbase + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#define PV_KFLUSH1(s, word, v, on)                                                      \
    {                                                                                   \
        const uint32_t t_ = wave_sum(v);                                                \
        if ((threadIdx.x & 63) == 0 && t_ && (on)) ksum_add(K, s, word, t_);            \
    }
__device__ void knet_flush(const NetK &K, uint32_t s, NetCtr &c)
{
    const bool nc = K.net_groups & PV_NET_COUNTERS_BIT;
    PV_KFLUSH1(s, PV_OFF_NET + NC_EVENTS, c.nev, true) PV_KFLUSH1(s, PV_OFF_NET + NC_SAMPLES, c.nev, true)
    PV_KFLUSH1(s, PV_OFF_NET + NC_TOTAL, c.nev - c.nfilt, nc) PV_KFLUSH1(s, PV_OFF_NET + NC_IN, c.nin, nc)
    PV_KFLUSH1(s, PV_OFF_NET + NC_OUT, c.nout, nc) PV_KFLUSH1(s, PV_OFF_NET + NC_UNK, c.nunk, nc)
    PV_KFLUSH1(s, PV_OFF_NET + NC_V4, c.n4, nc) PV_KFLUSH1(s, PV_OFF_NET + NC_V6, c.n6, nc)
    PV_KFLUSH1(s, PV_OFF_NET + NC_UDP, c.nudp, nc) PV_KFLUSH1(s, PV_OFF_NET + NC_TCP, c.ntcp, nc)
    PV_KFLUSH1(s, PV_OFF_NET + NC_SYN, c.nsyn, nc) PV_KFLUSH1(s, PV_OFF_NET + NC_OTHER, c.noth, nc)
    if (K.net_filter_all) PV_KFLUSH1(s, PV_OFF_NET + NC_FILTERED, c.nfilt, nc)
    c.zero();
}

// Dense IP log entry of one record for the top-N merge (0 = none):
//   IPv4  slot<<60 | TM_IPV4<<56 | card<<33 | dir<<32 | address
//   IPv6  slot<<60 | TM_IPV6<<56 | 55-bit address hash
// IPv4 cardinality is applied by pv_topn_merge, once per distinct address and batch,
// with the smallest record index; IPv6 cardinality (and cardinality without top IPs)
// goes straight to the first-occurrence table here.
// (NetworkMetricsBucket::process_net_layer :745-763)
template <class A>
__device__ __forceinline__ uint64_t net_ip_entry(const NetK &K, const A &R, const Parsed &o, uint64_t i, uint32_t slot)
{
    const bool card = K.net_groups & PV_NET_CARDINALITY_BIT, tops = K.net_groups & PV_NET_TOP_IPS_BIT;
    if (o.dir == 2 || !(card || tops)) return 0;
    uint64_t h1, h2;
    if (o.has4) {
        const uint32_t ip = R.u32(o.dir == 0 ? o.v4 + 12 : o.v4 + 16);
        if (!ip) return 0;
        if (tops)
            return ((uint64_t)slot << 60) | ((uint64_t)TM_IPV4 << 56) | ((uint64_t)card << 33) | ((uint64_t)o.dir << 32) | ip;
        murmur_8((uint64_t)(int64_t)(int32_t)ip, h1, h2);
        kcpc_min(K, slot, o.dir == 0 ? CPC_SRC : CPC_DST, cpc_coupon(h1, h2), i);
        return 0;
    }
    if (o.has6) {
        const uint64_t a = o.dir == 0 ? o.v6 + 8 : o.v6 + 24;
        const uint64_t w0 = (uint64_t)R.u32(a) | ((uint64_t)R.u32(a + 4) << 32);
        const uint64_t w1 = (uint64_t)R.u32(a + 8) | ((uint64_t)R.u32(a + 12) << 32);
        if (!(w0 | w1)) return 0;
        murmur_16(w0, w1, h1, h2);
        if (card) kcpc_min(K, slot, o.dir == 0 ? CPC_SRC : CPC_DST, cpc_coupon(h1, h2), i);
        if (tops) return ((uint64_t)slot << 60) | PV_KEY(TM_IPV6, (h1 ^ (h2 << 1)) & ((1ull << 55) - 1));
    }
    return 0;
}

// ------------------------------------------------------------------ Net pass staging
// Every wave streams its own tiles into a private LDS ring with LDS-DMA
// (global_load_lds: no VGPR holds data in flight) and keeps PV_NL_Q - 1 tiles in flight
// while it parses one. Per tile it issues, in this order, two row loads of record offsets
// (each lane's start and end) for the tile PV_NL_Q + 1 ahead and the tile's own DMA pieces.
// A tile's rows are thus issued two steps before its DMA needs them: loads retire in
// issue order, so rows issued only one step ahead would make every step wait one full
// memory latency and defeat the tile ring;
// every tile slot of the sequence is issued even past the range's end (a clamped copy),
// so the count of DMA operations younger than any tile is fixed and the wave waits for it
// with an exact vmcnt. The wave's other memory operations (stores, rare HBM reads) only
// make such a wait wait for a little more.
#ifndef PV_NL_Q
#define PV_NL_Q 3 // ring slots per wave (all of them in flight while the wave parses a tile)
#endif
#ifndef PV_NL_SLOT
#define PV_NL_SLOT 5120 // bytes per slot: the packed span of a tile, or 80-B windows
#endif
#define PV_NL_NJ (PV_NL_SLOT / 1024)     // 1-KiB DMA pieces per tile
#define PV_NL_OPS (PV_NL_NJ + 2)         // DMA operations per tile
#define PV_NL_OROWS (PV_NL_Q + 3)        // offset rows per wave (tiles k .. k + Q + 2)
static_assert(PV_NL_SLOT % 1024 == 0, "whole DMA pieces");
static_assert(PV_NL_SLOT / PV_WT >= 80, "window must cover Eth + IPv4 + UDP from a 16-B aligned start");

struct alignas(16) NetWave {
    uint32_t slot[PV_NL_Q][PV_NL_SLOT / 4];
    uint32_t lo[PV_NL_OROWS][PV_WT]; // each lane's record start
    uint32_t hi[PV_NL_OROWS];        // the tile's end (start of the record after its last)
    uint32_t pad[(4 - PV_NL_OROWS % 4) % 4];
};
// the batch's period tables, staged in LDS: lanes that need a per-record period (a tile that
// holds a shift, a DNS message's DNS period) read them with LDS loads; a per-lane load from
// the parameter block would be a vector load whose wait also drains the tiles in flight
struct PeriodTab {
    uint64_t pstart[PV_MAX_SHIFTS];
    int64_t dord[PV_MAX_SHIFTS]; // span ord of each DNS shift's event (P.dpos)
    uint32_t slot[PV_MAX_SHIFTS + 1];
};
struct NetState {
    NetWave w[4];
    uint32_t hist[PV_HBINS];
    uint32_t nd; // DNS messages found
    PeriodTab pt;
};

typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_u8 *)p);
}
// 64 lanes x 16 B from per-lane global addresses into LDS [m0 + lane * 16] (one 1-KiB piece)
__device__ __forceinline__ void dma16(const void *gsrc, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
// 64 lanes x 4 B into LDS [m0 + lane * 4]
__device__ __forceinline__ void dma4(const void *gsrc, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
#define PV_VMCNT(n) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory")
// Store flavours of the step's large writers. A plain store leaves its line dirty in the
// Infinity Cache until the read stream of a later kernel evicts it, and that kernel then pays for
// the write-back (tools/net_probe.hip, round 6: a pass over the C2 blob right after 160 MB of plain
// stores runs 158 us against 134 after the same bytes stored non-temporally, whose writer took
// 37 instead of 32 us). Non-temporal stores for the writers whose bytes no kernel of the same step
// reads back: the top-N merge's write-back. (The IP log and the combine list are read right after
// by the next kernel: non-temporal there measured slower, 87 -> 159 us for the combine list.)
#ifndef PV_NT_MERGE
#define PV_NT_MERGE 1 // pv_topn_merge's write-back of the table regions (read by the next batch's merge)
#endif
template <bool NT, class T>
__device__ __forceinline__ void st_nt(PV_G T *p, T v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// A workgroup barrier for LDS data only: the wave's LDS ops complete (lgkmcnt 0), then s_barrier.
// __syncthreads() also waits for every global store the wave has in flight (its release fence is a
// vmcnt(0)), and a store takes microseconds to complete under load; after a phase of global stores
// whose results no other wave of the workgroup reads, this barrier is the one to use.
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0); vmcnt / expcnt untouched
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(0) as the builtin (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15), which
// the compiler's wait insertion sees, unlike inline asm
#define PV_WAIT_VMCNT0 0x0F70

// Slot accessor: packed (dword d of the span at L[d]) or the lane's window as the DMA
// wrote it in 16-B pieces (dword d of lane l at L[(d >> 2) * 256 + l * 4 + (d & 3)]).
// Bytes outside the staged range come from HBM.
struct SAcc {
    const uint8_t *R;
    const uint32_t *L;
    uint64_t gbase;
    uint32_t lim, lane4, packed;
    PV_FN uint32_t idx(uint32_t d) const { return packed ? d : ((d >> 2) << 8) + lane4 + (d & 3); }
    PV_FN uint32_t u32(uint64_t off) const
    {
        const uint64_t rel = off - gbase;
        if (rel < lim) {
            const uint32_t r = (uint32_t)rel, d = r >> 2;
            return __builtin_amdgcn_alignbyte(L[idx(d + 1)], L[idx(d)], r & 3);
        }
        return pv_ld32(R, off);
    }
    PV_FN uint32_t u32a(uint64_t off) const // off 4-aligned
    {
        const uint64_t rel = off - gbase;
        if (rel < lim) return L[idx((uint32_t)rel >> 2)];
        return *reinterpret_cast<const uint32_t *>(R + off);
    }
    PV_FN uint32_t u8(uint64_t off) const
    {
        const uint64_t rel = off - gbase;
        if (rel < lim) {
            const uint32_t r = (uint32_t)rel;
            return (L[idx(r >> 2)] >> ((r & 3) * 8)) & 0xff;
        }
        return R[off];
    }
};

// Fast path of the per-record work: Ethernet II + IPv4 without options (and not
// IP-in-IP), the frame shape parse_record's own fast path takes. The record's first 64
// bytes are read from the slot into registers with independent LDS reads (one wait),
// and every field the Net pass needs is taken from them at a fixed offset; the results
// equal parse_record's, flowkey's and the accessor reads' on the same bytes.
struct RecW {
    uint32_t w[16]; // dwords at record offsets 0, 4, ..., 60
    PV_FN uint32_t at(int off) const // little-endian u32 at a constant record offset
    {
        return (off & 3) ? __builtin_amdgcn_alignbyte(w[(off >> 2) + 1], w[off >> 2], off & 3) : w[off >> 2];
    }
};
// the record's dwords d0 .. d0 + 16 (d0 < 4) from the five 16-B pieces that hold them, picked
// with two select levels, then byte-aligned
__device__ __forceinline__ void recw_pick(const uint32_t (&w)[20], uint32_t d0, uint32_t sh, RecW &r)
{
    // bit selects (v_bfi), not ternaries the compiler turns into a dynamically indexed
    // (scratch) array
    const uint32_t m0 = 0u - (d0 & 1), m1 = 0u - ((d0 >> 1) & 1);
    uint32_t a[19], x[17];
#pragma unroll
    for (int j = 0; j < 19; j++) a[j] = (w[j + 1] & m0) | (w[j] & ~m0);
#pragma unroll
    for (int j = 0; j < 17; j++) x[j] = (a[j + 2] & m1) | (a[j] & ~m1);
#pragma unroll
    for (int j = 0; j < 16; j++) r.w[j] = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);
}
// packed tile: the record's bytes are consecutive in the slot. Read as five ds_read_b128 from
// the record's 16-B aligned start (not 17 ds_read_b32 at the record's own dword: at an 80-B
// record stride those put 32 lanes on 8 of the 32 dword banks, a 4-way conflict on every
// read; b128 banks are (a/4) mod 64 in 16-lane groups, and 16 consecutive 80-B strides land
// on 16 distinct 16-B bank slots)
__device__ __forceinline__ void recw_load_packed(const uint32_t *L, uint32_t rel, RecW &r)
{
    const uint4 *q = reinterpret_cast<const uint4 *>(L + ((rel >> 4) << 2));
    uint32_t w[20];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint4 v = q[k];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
    recw_pick(w, (rel >> 2) & 3, rel & 3, r);
}
// window tile: the lane's 80-B window as five 16-B pieces (piece k at L[k * 256 + lane4]: lanes
// contiguous, so each ds_read_b128 is conflict-free), then the record's dwords d0 .. d0 + 16
// (d0 < 4) picked with two select levels
__device__ __forceinline__ void recw_load_window(const uint32_t *L, uint32_t d0, uint32_t sh, uint32_t lane4, RecW &r)
{
    const uint4 *q = reinterpret_cast<const uint4 *>(L + lane4);
    uint32_t w[20];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint4 v = q[k * 64];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
    recw_pick(w, d0, sh, r);
}
// parse_record's fast path from the words (o as parse_record sets it); false: not this shape
__device__ __forceinline__ bool fast_parse(const RecW &r, const ParseCfg &C, PV_CREF(PvParams) P, uint64_t rec, Parsed &o)
{
    o.caplen = r.w[2];
    o.sec = r.w[0];
    o.nsec = C.ts_nano ? (int32_t)r.w[1] : (int32_t)(r.w[1] * 1000u);
    o.frame = rec + 16;
    o.l3 = o.l4 = 0; o.has4 = o.has6 = 0; o.syn = 0; o.dir = 2;
    o.v4 = o.v6 = o.l4off = 0; o.l4len = 0;
    const uint32_t w3 = r.w[7], w4 = r.w[8], w5 = r.w[9];
    const uint32_t proto = w5 >> 24;
    if (!(C.linktype == 1 && o.caplen >= 34 && (w3 & 0xffffffu) == 0x450008u && proto != 4 && proto != 41)) return false;
    const uint32_t total = ((w4 & 0xff) << 8) | ((w4 >> 8) & 0xff);
    const uint32_t frag = ((w5 & 0xff) << 8) | ((w5 >> 8) & 0xff);
    uint32_t len = o.caplen - 14;
    if (total < len && total != 0) len = total;
    o.has4 = 1; o.l3 = 4; o.v4 = o.frame + 14;
    if (len > 20 && !(frag & 0x3fff)) {
        const uint64_t pl = o.frame + 34;
        const uint32_t pll = len - 20;
        if (proto == 17 && pll >= 8) { o.l4 = 17; o.l4off = pl; o.l4len = pll; }
        else if (proto == 6 && pll >= 20) {
            o.l4 = 6; o.l4off = pl; o.l4len = pll;
            o.syn = ((r.w[15] >> 24) & 2) ? 1 : 0; // TCP flags at record offset 63
        }
    }
    if (match4(C, P.nets, r.at(46))) o.dir = 0;
    else if (match4(C, P.nets, r.at(42))) o.dir = 1;
    return true;
}
// hash5Tuple of a fast-path record (flowkey on the same bytes)
__device__ __forceinline__ uint32_t fast_flowkey(const RecW &r)
{
    const uint32_t pw = r.at(50);
    const uint32_t ps = pw & 0xffff, pd = pw >> 16;
    int sp = pd < ps ? 1 : 0;
    uint32_t h = 0x811C9DC5u;
    const uint32_t p0 = sp ? pd : ps, p1 = sp ? ps : pd;
    h = fnv_bytes(h, p0, 2);
    h = fnv_bytes(h, p1, 2);
    const uint32_t sa = r.at(42), da = r.at(46);
    if (ps == pd && da < sa) sp = 1;
    h = fnv_bytes(h, sp ? da : sa, 4);
    h = fnv_bytes(h, sp ? sa : da, 4);
    return fnv_bytes(h, r.w[9] >> 24, 1);
}

// ---- DNS over TCP: the segment of a TCP packet of a DNS-port flow (PvTcpSeg; of any flow
// with `all`, the tcp_packet_reassembly_cache_limit replay's LRU holds every connection), or false
// when TcpReassembly would not look at it (no payload and none of SYN / FIN / RST: dropped
// before the connection lookup) or its header is not a TcpLayer (TcpLayer::isDataValid)
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xff) << 8) | ((x >> 8) & 0xff); }
__device__ __forceinline__ bool tcp_dns_pw(uint32_t pw)
{
    const uint32_t sp = bswap16(pw & 0xffff), dp = bswap16(pw >> 16);
    return sp == 53 || sp == 5353 || sp == 5355 || sp == 53000 || dp == 53 || dp == 5353 || dp == 5355 || dp == 53000;
}
// the side of a packet: its first IP layer's source address and source port
__device__ __forceinline__ uint64_t tcp_ep4(uint32_t a, uint32_t sport_raw)
{
    return fmix64((((uint64_t)a << 16) | sport_raw) ^ 0x7463703400000000ull);
}
__device__ __forceinline__ uint64_t tcp_ep6(uint64_t w0, uint64_t w1, uint32_t sport_raw)
{
    return fmix64(w0 ^ fmix64(w1 ^ ((uint64_t)sport_raw << 48) ^ 0x7463703600000000ull));
}
__device__ __forceinline__ bool tcp_seg_fill(PvTcpSeg &g, uint32_t pw, uint32_t w3, uint32_t seq_raw, uint32_t l4len, uint64_t l4off,
                                             uint64_t i, uint32_t fkey, int64_t sec, int32_t nsec, uint64_t ep, uint32_t dirv6,
                                             uint32_t mode)
{
    const uint32_t hl = ((w3 >> 4) & 0xf) * 4; // data offset (byte 12), flags (byte 13)
    const bool bad = hl < 20 || hl > l4len;
    uint32_t fl = (w3 >> 8) & 7;
    const uint32_t plen = bad ? 0u : l4len - hl;
    if (bad || (!plen && !fl)) {
        // ignored by reassembly; the exact LRU mode (mode bit 4) keeps it for the cleanup after it
        if (!(mode & 4)) return false;
        fl = PV_TF_NODATA;
    }
    g.idx = (uint32_t)i;
    g.poff = (uint32_t)(l4off + hl);
    g.seq = __builtin_bswap32(seq_raw);
    g.fkey = fkey;
    g.sec = (uint32_t)sec;
    g.usec = (uint32_t)nsec / 1000u;
    g.ep = ep;
    g.plen = (uint16_t)plen;
    g.sport = (uint16_t)bswap16(pw & 0xffff);
    g.dport = (uint16_t)bswap16(pw >> 16);
    g.flags = (uint8_t)fl;
    g.dirv6 = (uint8_t)dirv6;
    g.pad[0] = g.pad[1] = 0;
    return true;
}
template <class A>
__device__ __forceinline__ bool tcp_seg_of(const A &R, const Parsed &o, uint64_t i, PvTcpSeg &g, uint32_t mode = 1)
{
    if (o.l4 != 6) return false;
    const uint32_t pw = R.u32(o.l4off);
    if (!(mode & 2) && !tcp_dns_pw(pw)) return false;
    const bool v6first = o.has6 && (!o.has4 || o.v6 < o.v4);
    uint64_t ep;
    if (!v6first) ep = tcp_ep4(R.u32(o.v4 + 12), pw & 0xffff);
    else {
        const uint64_t a = o.v6 + 8;
        ep = tcp_ep6((uint64_t)R.u32(a) | ((uint64_t)R.u32(a + 4) << 32), (uint64_t)R.u32(a + 8) | ((uint64_t)R.u32(a + 12) << 32),
                     pw & 0xffff);
    }
    return tcp_seg_fill(g, pw, R.u32(o.l4off + 12), R.u32(o.l4off + 4), o.l4len, o.l4off, i, flowkey(R, o), o.sec, o.nsec, ep,
                        o.dir | (v6first ? 4u : 0u), mode);
}
// the same from a fast-path record's words (Ethernet + IPv4 without options: TCP at record offset 50)
__device__ __forceinline__ bool tcp_seg_fast(const RecW &r, const Parsed &o, uint64_t i, PvTcpSeg &g, uint32_t mode = 1)
{
    const uint32_t pw = r.at(50);
    if (!(mode & 2) && !tcp_dns_pw(pw)) return false;
    return tcp_seg_fill(g, pw, r.w[15] >> 16, r.at(54), o.l4len, o.l4off, i, fast_flowkey(r), o.sec, o.nsec,
                        tcp_ep4(r.at(42), pw & 0xffff), o.dir, mode);
}
// wave-compacted append of the lanes' segments (one atomic per wave), with their payload bytes
__device__ __forceinline__ void tcp_seg_store(PV_G PvTcpSeg *out, PV_G uint32_t *cnt, uint32_t cap, bool has, const PvTcpSeg &g,
                                              uint32_t lane)
{
    const uint64_t m = __ballot(has);
    if (!m) return;
    uint32_t bytes = has ? g.plen : 0u;
    for (int o = 32; o > 0; o >>= 1) bytes += __shfl_xor(bytes, o, 64);
    uint32_t q = 0;
    if (lane == 0) {
        q = atomicAdd(cnt, (uint32_t)__popcll(m));
        atomicAdd(cnt + 1, bytes);
    }
    q = __builtin_amdgcn_readlane(q, 0) + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (has) {
        if (q < cap) {
            PV_G uint4 *d = reinterpret_cast<PV_G uint4 *>(out + q);
            d[0] = make_uint4(g.idx, g.poff, g.seq, g.fkey);
            d[1] = make_uint4(g.sec, g.usec, (uint32_t)g.ep, (uint32_t)(g.ep >> 32));
            d[2] = make_uint4((uint32_t)g.plen | ((uint32_t)g.sport << 16), (uint32_t)g.dport | ((uint32_t)g.flags << 16) |
                              ((uint32_t)g.dirv6 << 24), 0u, 0u);
        }
    }
}

} // namespace

// The general per-record path (every frame the fast path does not take: VLAN, IPv6,
// options, tunnels, other link types), out of line. A call returns with its reads done, so
// the Net pass's loop never carries a register load pending across its edge; otherwise
// the compiler's vmcnt(0) before that register's next write, on the fast path too, would
// drain every tile in flight on every step. Fills what the caller's counters need and
// the record's dense IP log entry and DNS message.
struct SlowOut {
    uint64_t ek;
    DnsMsgW dm;
    uint32_t caplen, isdns;
    uint8_t dir, l3, l4, syn;
};
__device__ __forceinline__ SlowOut net_slow_body(const SAcc R, const ParseCfg C, PV_CREF(PvParams) P, const NetK K, uint64_t off,
                                                 uint64_t i, uint32_t slot, bool upd)
{
    SlowOut so;
    so.ek = 0;
    so.dm = DnsMsgW{};
    so.isdns = 0;
    Parsed o;
    parse_record(R, C, P, off, o);
    so.caplen = o.caplen; so.dir = o.dir; so.l3 = o.l3; so.l4 = o.l4; so.syn = o.syn;
    if (K.dbg & 2) return so;
    if (K.tcp_emit && o.l4 == 6) {
        // a DNS-port TCP segment of a general-path frame: appended by this lane alone
        PvTcpSeg g;
        if (tcp_seg_of(R, o, i, g, K.tcp_emit)) {
            const uint32_t q = atomicAdd(K.tseg_cnt, 1u);
            atomicAdd(K.tseg_cnt + 1, (uint32_t)g.plen);
            if (q < K.tseg_cap) K.tseg[q] = g;
        }
    }
    if (upd) so.ek = net_ip_entry(K, R, o, i, slot);
    if (o.l4 == 17 && !(K.dbg & 4)) {
        const uint32_t port = dns_port(R.u32(o.l4off));
        if (port) {
            const uint32_t dp = P.n_dshift ? dperiod_of(P, i) : 0u;
            so.dm = msg_words(dns_msg_of(P, R, o, i, port, dp, dp >= P.dskip_before, true));
            so.isdns = 1;
        }
    }
    return so;
}
// out of line for the general Net pass's rare records (its fast path keeps no frame for it)
__device__ __noinline__ SlowOut net_slow(const SAcc R, const ParseCfg C, PV_CREF(PvParams) P, const NetK K, uint64_t off,
                                         uint64_t i, uint32_t slot, bool upd)
{
    return net_slow_body(R, C, P, K, off, i, slot, upd);
}

// ------------------------------------------------------------------ the Net pass
// One lane per record; workgroup b owns the contiguous tile range [b*T, (b+1)*T) and its
// wave w takes the range's tiles w, w+4, ... (staging above). Counters stay in registers,
// payload sizes go to an LDS histogram, the IP of each record to the dense IP log
// (coalesced stores) and DNS messages to the workgroup's DNS work list. No table lookups
// and no atomics with a return on the per-record path.
#ifndef PV_NET_MINB
#define PV_NET_MINB 1 // tuning: resident workgroups per CU the register allocation must allow
#endif
// The Net pass body. GEN = false is the common batch, specialised: no period shift inside
// the batch, no filter-all mode and no profiling knobs, so the per-tile period and slot
// logic and the direct-update paths compile away (fewer live scalars in the tile loop).
template <bool GEN>
__device__ __forceinline__ void net_pass(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ NetState S;
    // wave index as a scalar: tile and period arithmetic stays uniform (no vector loads
    // whose vmcnt wait would also drain the tiles in flight)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (uint32_t b = threadIdx.x; b < PV_HBINS; b += blockDim.x) S.hist[b] = 0;
    if (threadIdx.x == 0) S.nd = 0;
    if (threadIdx.x < PV_MAX_SHIFTS) {
        S.pt.pstart[threadIdx.x] = P.pstart[threadIdx.x];
        S.pt.dord[threadIdx.x] = P.dpos[threadIdx.x];
    }
    if (threadIdx.x <= PV_MAX_SHIFTS) S.pt.slot[threadIdx.x] = P.slot_of[threadIdx.x];
    __syncthreads();
    NetK K;
    K.recs = P.recs; K.offs = P.offs; K.n = P.n; K.rec_bytes = P.rec_bytes; K.gbase = P.gbase;
    K.sum = P.sum; K.cpc = P.cpc; K.iplog = P.iplog; K.dq = P.dq; K.flags = P.flags;
    K.n_shift = GEN ? P.n_shift : 0u; K.skip_before = P.skip_before; K.slot0 = P.slot_of[0];
    K.net_groups = P.net_groups; K.dbg = GEN ? P.dbg : 0u; K.net_filter_all = GEN ? P.net_filter_all : 0u;
    K.n_dshift = P.n_dshift; K.dskip_before = P.dskip_before;
    K.tcp_emit = P.tcp_emit; K.tseg_cap = P.tseg_cap; K.tseg = P.tseg; K.tseg_cnt = P.tseg_cnt; K.tmask = P.tmask;
    K.ndeep_net = GEN ? P.ndeep_net : nullptr; K.ndeep_dns = GEN ? P.ndeep_dns : nullptr;
    const ParseCfg C = parse_cfg(P);
    const uint64_t n = K.n, last = n - 1;
    const uint64_t nwt = (n + PV_WT - 1) / PV_WT;
    const uint64_t wbeg = (uint64_t)blockIdx.x * P.wt_per_block;
    const uint64_t wend = min<uint64_t>(wbeg + P.wt_per_block, nwt);
    // this wave's tiles: t(k) = wbeg + wave + 4k, k < ntl
    const uint32_t ntl = wend > wbeg + wave ? (uint32_t)((wend - wbeg - wave + 3) / 4) : 0u;
    const uint64_t dq_base = wbeg * PV_WT; // this workgroup's DNS work-list region
    NetWave &NW = S.w[wave];
    auto tile_of = [&](uint32_t k) -> uint64_t { return wbeg + wave + 4ull * min(k, ntl - 1); };
    // offset rows of tile k (clamped), then its DMA pieces into slot k % Q
    auto issue_rows = [&](uint32_t k) {
        const uint64_t r = tile_of(k) * PV_WT + lane;
        const uint32_t row = k % PV_NL_OROWS;
        dma4(K.offs + min<uint64_t>(r, last), lds_addr(&NW.lo[row][0]));
        // the tile's end: lane 63's next offset, landing at hi[row] (LDS-DMA writes m0 + 4 * lane)
        const uint32_t ha = lds_addr(&NW.hi[row]) - 4 * 63;
        if (lane == 63) dma4(K.offs + min<uint64_t>(r + 1, last), ha);
    };
    auto issue_tile = [&](uint32_t k) {
        const uint32_t row = k % PV_NL_OROWS;
        const uint64_t t = tile_of(k);
        const uint32_t o = NW.lo[row][lane];
        const uint32_t b0 = __builtin_amdgcn_readfirstlane(NW.lo[row][0]);
        const uint32_t b1 = t * PV_WT + PV_WT >= n ? (uint32_t)K.rec_bytes : __builtin_amdgcn_readfirstlane(NW.hi[row]);
        const uint32_t base = b0 & ~15u, nch = (b1 - base + 15) >> 4;
        const bool packed = nch <= (uint32_t)(PV_NL_SLOT / 16);
        const uint32_t dst = lds_addr(&NW.slot[k % PV_NL_Q][0]);
#pragma unroll
        for (int j = 0; j < PV_NL_NJ; j++) {
            const uint32_t ch = (uint32_t)(j * 64) + lane;
            const uint32_t src = packed ? base + min(ch, nch - 1) * 16 : (o & ~15u) + 16u * j;
            dma16(K.recs + src, dst + j * 1024);
        }
    };
    auto period = [&](uint64_t r) -> uint32_t { return K.n_shift ? period_of(P, r) : 0u; };
    auto slot_of = [&](uint32_t p) -> uint32_t { return K.n_shift ? P.slot_of[p] : K.slot0; };
    // the LDS histogram belongs to the slot of the workgroup's first record
    const uint32_t hslot = slot_of(period(min<uint64_t>(wbeg * PV_WT, last)));
    const bool tops = K.net_groups & PV_NET_TOP_IPS_BIT;
    NetCtr c;
    c.zero();
    uint32_t wslot = 0xffffffffu;
    // The ring: step k waits for tile k, reads each lane's record words out of slot k % Q
    // into registers and, once no lane needs the slot any more (every lane took the fast
    // path: the common case), refills it at once with [rows k + Q + 2][tile k + Q]; a tile
    // with general-path records refills after its body. So Q tiles (not Q - 1) are in
    // flight while a wave parses, and Q = 2 slots per wave leave LDS for three workgroups per
    // CU. A tile's rows are issued two refills before the tile, so the wait for them is
    // for loads two steps old; every refill of the sequence is issued even past the range's
    // end (a clamped copy), so the count of DMA operations younger than any tile is fixed
    // and the waits are exact vmcnt counts (the wave's stores between them only make a wait
    // wait for a little more).
    auto refill = [&](uint32_t k) {
        issue_rows(k + PV_NL_Q + 2);
        PV_VMCNT(2 * PV_NL_OPS); // rows k + Q landed: younger are tile k + Q - 2, refill k - 1, rows k + Q + 2
        issue_tile(k + PV_NL_Q);
    };
    if (ntl) {
        // prologue: rows 0 and 1, then the refills of steps -Q .. -1, [rows j + 2][tile j] for
        // j = 0 .. Q - 1 (the steady state's pattern, so the counts hold from step 0 on)
        issue_rows(0);
        issue_rows(1);
        PV_VMCNT(0);
        for (uint32_t j = 0; j < PV_NL_Q; j++) {
            issue_rows(j + 2);
            if (j >= 2) PV_VMCNT(2 * PV_NL_OPS);
            issue_tile(j);
        }
    }
    STAMP_DECL
    // one tile's records from its staged copy Ls (off: this lane's record start, [b0, b1): the tile's span)
    auto tile_body = [&](uint32_t k, uint64_t off, uint32_t b0, uint32_t b1, const uint32_t *Ls) -> bool {
        const uint64_t t = tile_of(k);
        const uint64_t r0 = t * PV_WT;
        const uint64_t r1 = min<uint64_t>(r0 + PV_WT, n) - 1;
        const uint32_t p_lo = __builtin_amdgcn_readfirstlane(period(r0)), p_hi = __builtin_amdgcn_readfirstlane(period(r1));
        // a tile that holds a period shift: each lane resolves its own period, and lanes
        // outside the wave's register slot update HBM directly
        const bool straddle = p_lo != p_hi;
        const uint32_t tslot = slot_of(p_lo);
        if (p_lo >= K.skip_before && tslot != wslot) {
            if (wslot != 0xffffffffu) knet_flush(K, wslot, c);
            wslot = tslot;
        }
        const uint64_t i = r0 + lane;
        const bool active = i <= r1;
        uint32_t lp = p_lo, slot = tslot;
        if (straddle) {
            lp = 0;
            for (uint32_t q = 0; q < K.n_shift; q++) lp += i >= S.pt.pstart[q];
            slot = S.pt.slot[lp];
        }
        const bool upd = lp >= K.skip_before;
        const bool own = slot == wslot;
        // deep sampling: the Net manager's draw for this record's event, the DNS manager's for
        // its DNS event (bitmaps padded past the span, so inactive lanes read in bounds)
        bool deep = true, ddeep = true;
        if (GEN && K.ndeep_net) {
            deep = !((K.ndeep_net[i >> 5] >> (i & 31)) & 1);
            ddeep = !((K.ndeep_dns[i >> 5] >> (i & 31)) & 1);
        }
        const uint32_t base = b0 & ~15u, nch = (b1 - base + 15) >> 4;
        const bool packed = nch <= (uint32_t)(PV_NL_SLOT / 16);
        uint32_t hv = PV_NOH;
        uint64_t ek = 0;
        DnsMsgW dm{};
        bool isdns = false;
        bool istcp = false, hasseg = false, released = false;
        PvTcpSeg seg;
        const bool work = active && !(K.dbg & 1);
        const SAcc R = packed ? SAcc{K.recs, Ls, base, nch * 16 - 4, 0u, 1u}
                              : SAcc{K.recs, Ls, off & ~15ull, PV_NL_SLOT / PV_WT - 4, lane * 4, 0u};
        // fast path: the 17 staged dwords recw_load reads (the record's first 64 bytes
        // plus the alignment spill) are inside the staged range; in window mode that
        // holds for every record (start within 15 bytes of the 16-B aligned window)
        const uint32_t rel = (uint32_t)(off - R.gbase);
        RecW rw;
        Parsed o;
        bool fast = false;
        if (work && (rel >> 2) + 17 <= (R.lim + 4) >> 2) {
            if (packed) recw_load_packed(R.L, rel, rw);
            else recw_load_window(R.L, rel >> 2, rel & 3, lane * 4, rw);
            fast = fast_parse(rw, C, P, off, o);
        }
        // every lane's words are in registers: unless a general-path record still reads the
        // slot, it is refilled now (whole wave, uniform branch), before the body's work
        if (__ballot(work && !fast) == 0) {
            asm volatile("" ::: "memory");
            refill(k);
            released = true;
        }
        if (work) {
            if (!fast) {
                // a record that is not deep: no IPs, no SYN (NetworkMetricsBucket::process_packet
                // !deep, net/v1/NetStreamHandler.cpp:518-521)
                const SlowOut so = net_slow(R, C, P, K, off, i, slot, upd && !K.net_filter_all && deep);
                o.caplen = so.caplen; o.dir = so.dir; o.l3 = so.l3; o.l4 = so.l4; o.syn = so.syn && deep;
                ek = so.ek;
                dm = so.dm;
                isdns = so.isdns;
                if (!ddeep) dm.a.w |= 16u << 16; // DnsMsg flags bit 4: the DNS event is not deep
            } else if (K.tcp_emit && o.l4 == 6) {
                hasseg = tcp_seg_fast(rw, o, i, seg, GEN ? K.tcp_emit : 1u);
            }
            istcp = o.l4 == 6;
            if (!deep) o.syn = 0;
            if (GEN && K.ndeep_net) {
                // deep_samples counts deep events only: one subtraction per wave (per lane in a
                // tile whose records fall in several periods)
                const bool nd = upd && !deep && !(K.dbg & 2);
                const uint64_t m = __ballot(nd);
                if (m) {
                    if (!straddle) {
                        if (lane == (uint32_t)__builtin_ctzll(m))
                            ksum_add(K, slot, PV_OFF_NET + NC_SAMPLES, (uint64_t)0 - (uint64_t)__popcll(m));
                    } else if (nd) {
                        ksum_add(K, slot, PV_OFF_NET + NC_SAMPLES, ~0ull);
                    }
                }
            }
            STAMP(4)
            if (K.dbg & 2) {
                c.add(o);
            } else if (K.net_filter_all) {
                // process_filtered (net/v1/NetStreamHandler.cpp:507-514): an event and `filtered` only
                if (upd) {
                    if (own) { c.nev++; c.nfilt++; }
                    else {
                        ksum_add(K, slot, PV_OFF_NET + NC_EVENTS, 1);
                        ksum_add(K, slot, PV_OFF_NET + NC_SAMPLES, 1);
                        if (K.net_groups & PV_NET_COUNTERS_BIT) ksum_add(K, slot, PV_OFF_NET + NC_FILTERED, 1);
                    }
                }
                ek = 0;
            } else {
                if (upd) {
                    if (own) c.add(o);
                    else knet_direct(K.sum, K.net_groups, slot, o.dir, o.l3, o.l4, o.syn);
                    uint32_t cl = o.caplen;
                    if (cl > 65535) { atomicOr(K.flags, PVF_BIG_CAPLEN); cl = 65535; }
                    if (slot == hslot) hv = cl;
                    else ksum_add(K, slot, PV_OFF_PAYLOAD + cl, 1);
                    if (fast && deep) {
                        // net_ip_entry on the words (IPv4 only)
                        const bool card = K.net_groups & PV_NET_CARDINALITY_BIT;
                        const uint32_t ip = o.dir == 0 ? rw.at(42) : rw.at(46);
                        if (o.dir != 2 && ip && (card || tops)) {
                            if (tops)
                                ek = ((uint64_t)slot << 60) | ((uint64_t)TM_IPV4 << 56) | ((uint64_t)card << 33) |
                                     ((uint64_t)o.dir << 32) | ip;
                            else {
                                uint64_t h1, h2;
                                murmur_8((uint64_t)(int64_t)(int32_t)ip, h1, h2);
                                kcpc_min(K, slot, o.dir == 0 ? CPC_SRC : CPC_DST, cpc_coupon(h1, h2), i);
                            }
                        }
                    }
                }
            }
            // the DNS handler takes the pcap input's UDP signal itself (not chained behind Net)
            if (!(K.dbg & 2) && fast && o.l4 == 17 && !(K.dbg & 4)) {
                const uint32_t port = dns_port(rw.at(50));
                if (port) {
                    uint32_t dp = 0;
                    for (uint32_t q = 0; q < K.n_dshift; q++) dp += (int64_t)(4 * i) >= S.pt.dord[q];
                    DnsMsg d = dns_msg_of(P, R, o, i, port, dp, dp >= K.dskip_before, false);
                    d.fkey = fast_flowkey(rw);
                    dm = msg_words(d);
                    if (!ddeep) dm.a.w |= 16u << 16; // not deep
                    isdns = true;
                }
            }
        } else if (K.dbg & 1) {
            c.nev += active;
        }
        // all reads of slot sl are issued before the next step's DMA may overwrite it
        asm volatile("" ::: "memory");
        STAMP(5)
        if (!(K.dbg & 1)) {
            if (!(K.dbg & 64)) hist_add(S.hist, K.sum + (uint64_t)hslot * PV_SUM_WORDS + PV_OFF_PAYLOAD, hv, lane); // 64: profiling knob
            // DNS messages: wave-compacted into the workgroup's work list
            const uint64_t m = __ballot(isdns);
            if (m) {
                uint32_t q = 0;
                if (lane == 0) q = atomicAdd(&S.nd, (uint32_t)__popcll(m));
                q = __builtin_amdgcn_readlane(q, 0);
                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                if (isdns) {
                    PV_G uint4 *dd = reinterpret_cast<PV_G uint4 *>(K.dq) + 2 * (dq_base + q + below);
                    dd[0] = dm.a;
                    dd[1] = dm.b;
                }
            }
            if (tops && i <= r1 && !(K.dbg & 128)) K.iplog[i] = ek; // 128: profiling knob, no IP log
            if (K.tcp_emit) {
                // DNS over TCP: the tile's TCP records, then its DNS-port segments
                // (tiles without TCP keep the zero the batch's fill wrote: no store, so no
                // extra vector operation in the ring's exact vmcnt accounting on UDP-only tiles)
                const uint64_t tm = __ballot(istcp);
                if (tm) {
                    if (lane == 0) K.tmask[t] = tm;
                    tcp_seg_store(K.tseg, K.tseg_cnt, K.tseg_cap, hasseg, seg, lane);
                }
            }
        }
        STAMP(6)
        return released;
    };
    for (uint32_t k = 0; k < ntl; k++) {
        PV_VMCNT((PV_NL_Q - 1) * PV_NL_OPS); // tile k landed: younger are the refills of steps k - Q + 1 .. k - 1
        STAMP(1)
        const uint32_t sl = k % PV_NL_Q, row = k % PV_NL_OROWS;
        const bool rel = tile_body(k, NW.lo[row][lane], __builtin_amdgcn_readfirstlane(NW.lo[row][0]),
                                   tile_of(k) * PV_WT + PV_WT >= n ? (uint32_t)K.rec_bytes : __builtin_amdgcn_readfirstlane(NW.hi[row]),
                                   NW.slot[sl]);
        if (!rel) refill(k);
    }
    PV_VMCNT(0); // the sequence's trailing copies land before the workgroup ends
    if (wslot != 0xffffffffu) knet_flush(K, wslot, c);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < PV_HBINS; b += blockDim.x)
        if (S.hist[b]) ksum_add(K, hslot, PV_OFF_PAYLOAD + b, S.hist[b]);
    STAMP_FLUSH
    if (threadIdx.x == 0) {
        P.mq_cnt[blockIdx.x] = 0;
        P.dq_cnt[blockIdx.x] = S.nd;
        if (S.nd) atomicAdd(P.n_dns, S.nd);
    }
}


// ------------------------------------------------------------------ the lean Net pass
// The common batch: one Net period (no shift inside the batch), no filter-all, no deep
// sampling, no profiling knobs, Ethernet link type, at most two IPv4 host subnets. The same
// results as net_pass, with a tile's work written for the instruction budget: the general pass
// is issue-bound (rocprofv3 on C2: ~300 VALU and ~320 SALU wave-instructions per 64-record tile,
// each wave issuing 40 % of its cycles), most of it exec masking of nested per-lane branches and
// spilled scalars. Here the fast path (Ethernet II + IPv4 without options) is straight-line
// selects, the fast lanes' nine counters are three packed lane registers, every rarely taken
// piece (DNS messages, TCP segments, caplen > 65535, cardinality without top IPs) sits behind a
// uniform ballot branch, and general-path records (VLAN, IPv6, options, tunnels, other link
// types) are deferred to pv_net_slow_list, which parses every byte of them from HBM.
// (Measured and dropped, in the history of round 6: an LDS-DMA ring with producer waves, a
// per-grid-workgroup LDS ring, eight waves per workgroup, depth-2 and conditional-load
// pipelines, the general path as an out-of-line call in the loop)

// fast-path fields of one record (parse_record's fast path, branch-free)
struct FastRec {
    uint32_t ok, caplen, dir, l4, syn, l4len;
};
struct HostNets {
    uint32_t a0, m0, a1, m1, e0, e1; // e: subnet present (all-ones / zero)
};
PV_FN uint32_t hit4(const HostNets &h, uint32_t ip)
{
    const uint32_t m = (((ip ^ h.a0) & h.m0) == 0 ? h.e0 : 0u) | (((ip ^ h.a1) & h.m1) == 0 ? h.e1 : 0u);
    return ip ? m : 0u;
}
PV_FN FastRec fast_fields(const RecW &r, const HostNets &h)
{
    FastRec f;
    f.caplen = r.w[2];
    const uint32_t w3 = r.w[7], w4 = r.w[8], w5 = r.w[9];
    const uint32_t proto = w5 >> 24;
    f.ok = (f.caplen >= 34) & ((w3 & 0xffffffu) == 0x450008u) & (proto != 4) & (proto != 41);
    const uint32_t total = ((w4 & 0xff) << 8) | ((w4 >> 8) & 0xff);
    const uint32_t frag = ((w5 & 0xff) << 8) | ((w5 >> 8) & 0xff);
    const uint32_t l = f.caplen - 14;
    const uint32_t len = (total != 0 && total < l) ? total : l;
    const uint32_t pll = len - 20;
    const bool l4ok = (len > 20) & !(frag & 0x3fff);
    const bool udp = l4ok & (proto == 17) & (pll >= 8);
    const bool tcp = l4ok & (proto == 6) & (pll >= 20);
    f.l4 = udp ? 17u : (tcp ? 6u : 0u);
    f.syn = tcp ? (r.w[15] >> 25) & 1 : 0u; // TCP flags at record offset 63
    f.l4len = pll;
    const uint32_t dst = hit4(h, r.at(46)), src = hit4(h, r.at(42));
    f.dir = dst ? 0u : (src ? 1u : 2u);
    return f;
}
// dns_port without short-circuit branches
PV_FN uint32_t dns_port_bf(uint32_t pw)
{
    const uint32_t sport = ((pw & 0xff) << 8) | ((pw >> 8) & 0xff);
    const uint32_t dport = ((pw >> 8) & 0xff00) | (pw >> 24);
    const bool dd = (dport == 53) | (dport == 5353) | (dport == 5355) | (dport == 53000);
    const bool sd = (sport == 53) | (sport == 5353) | (sport == 5355) | (sport == 53000);
    return dd ? sport : (sd ? dport : 0u);
}
// the Parsed a fast record's consumers (DNS message, TCP segment) read
PV_FN Parsed fast_parsed(const FastRec &f, const RecW &r, uint32_t ts_nano, uint64_t off)
{
    Parsed o;
    o.caplen = f.caplen;
    o.sec = r.w[0];
    o.nsec = ts_nano ? (int32_t)r.w[1] : (int32_t)(r.w[1] * 1000u);
    o.frame = off + 16;
    o.l3 = 4; o.l4 = (uint8_t)f.l4; o.has4 = 1; o.has6 = 0; o.syn = (uint8_t)f.syn; o.dir = (uint8_t)f.dir;
    o.v4 = o.frame + 14; o.v6 = 0;
    o.l4off = f.l4 ? o.frame + 34 : 0;
    o.l4len = f.l4 ? f.l4len : 0;
    return o;
}
// a general-path record of the lean pass: net_slow with the parameters read here (inlined into
// pv_net_slow_list, which then makes no device call)
__device__ __forceinline__ SlowOut net_slow_p(const PvParams *__restrict__ Pp, const SAcc R, uint64_t off, uint64_t i)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    NetK K;
    K.recs = P.recs; K.offs = P.offs; K.n = P.n; K.rec_bytes = P.rec_bytes; K.gbase = P.gbase;
    K.sum = P.sum; K.cpc = P.cpc; K.iplog = P.iplog; K.dq = P.dq; K.flags = P.flags;
    K.n_shift = 0; K.skip_before = 0; K.slot0 = P.slot_of[0];
    K.net_groups = P.net_groups; K.dbg = 0; K.net_filter_all = 0;
    K.n_dshift = P.n_dshift; K.dskip_before = P.dskip_before;
    K.tcp_emit = P.tcp_emit; K.tseg_cap = P.tseg_cap; K.tseg = P.tseg; K.tseg_cnt = P.tseg_cnt; K.tmask = P.tmask;
    K.ndeep_net = nullptr; K.ndeep_dns = nullptr;
    return net_slow_body(R, parse_cfg(P), P, K, off, i, K.slot0, true);
}

// ------------------------------------------------------------------ the lean Net pass, register windows
// Each lane loads its own record's first 80 bytes straight into registers (five 16-B loads from
// the record's dword-aligned start, so the record's dwords are one alignbyte away: no selects),
// the windows of the next two tiles in flight while the wave parses this one. tools/stream_probe.hip
// measured the pattern alone at 5.8 TB/s (modes 7/8) against 4.2 TB/s for LDS-DMA staging; the
// LDS keeps only the histogram and the DNS / exception / deferred-record list counters.
#ifndef PV_REG_MINW
#define PV_REG_MINW 2 // waves per SIMD the register allocation must allow
#endif
struct NetRegState {
    uint32_t hist[PV_HBINS];
    uint32_t nd, nx, ns;
    int64_t dord[PV_MAX_SHIFTS];
};
__device__ __forceinline__ void win_load(const PV_G uint8_t *recs, uint32_t off, uint4 (&W)[5])
{
    const PV_G uint4 *p = reinterpret_cast<const PV_G uint4 *>(recs + (off & ~3u));
#pragma unroll
    for (int j = 0; j < 5; j++) W[j] = p[j];
}
__device__ __forceinline__ void win_words(const uint4 (&W)[5], uint32_t sh, RecW &r)
{
    uint32_t x[17];
#pragma unroll
    for (int k = 0; k < 4; k++) { x[4 * k] = W[k].x; x[4 * k + 1] = W[k].y; x[4 * k + 2] = W[k].z; x[4 * k + 3] = W[k].w; }
    x[16] = W[4].x;
#pragma unroll
    for (int j = 0; j < 16; j++) r.w[j] = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);
}
// NW: waves of the workgroup; wave w takes tiles w, w + NW, ... of each range.
// TC: top IPs on with the compact IP log (the default groups). Its two stores per tile are then
// unconditional instructions, so the compiler's counted vmcnt for the next tile's windows counts
// them as younger ops instead of waiting for them: a store takes microseconds to complete under
// the read stream, and a wait that covers the previous tile's stores (as the branchy form's
// does) stalls every tile on them (tools/ring_probe.hip: 138 -> 177 us on C2 with a 4-B store).
template <uint32_t NW, bool TC = false>
__device__ __forceinline__ void net_fast_reg(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ NetRegState S;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (uint32_t b = threadIdx.x; b < PV_HBINS; b += blockDim.x) S.hist[b] = 0;
    if (threadIdx.x == 0) { S.nd = 0; S.nx = 0; S.ns = 0; }
    if (threadIdx.x < PV_MAX_SHIFTS) S.dord[threadIdx.x] = P.dpos[threadIdx.x];
    __syncthreads();
    const PV_G uint8_t *const recs = P.recs;
    const bool compact = P.ip_compact;
    const PV_G uint32_t *const offs = P.offs;
    const uint64_t n = P.n, last = n - 1;
    const uint32_t slot = P.slot_of[0];
    const uint32_t groups = P.net_groups;
    const bool tops = groups & PV_NET_TOP_IPS_BIT, card = groups & PV_NET_CARDINALITY_BIT;
    const uint32_t ts_nano = P.ts_nano;
    HostNets h;
    {
        const uint32_t n4 = P.nets.n4;
        h.a0 = P.nets.v4_addr[0]; h.m0 = P.nets.v4_mask[0]; h.e0 = n4 > 0 ? ~0u : 0u;
        h.a1 = P.nets.v4_addr[1]; h.m1 = P.nets.v4_mask[1]; h.e1 = n4 > 1 ? ~0u : 0u;
    }
    const uint64_t nwt = (n + PV_WT - 1) / PV_WT;
    uint64_t cd = 0, cl = 0; // fast lanes' packed counters (net_fast)
    NetCtr c;
    c.zero();
    bool any = false;
    // each workgroup walks the ranges of several grid workgroups (lb = blockIdx.x, + gridDim.x,
    // ...): the DNS pass, combine and merge keep the grid's partition, while the Net pass runs
    // one workgroup per CU (fewer, longer streams measured faster: tools/gpu_reg2.sh)
    for (uint32_t lb = blockIdx.x; lb < P.grid_main; lb += gridDim.x) {
    const uint64_t wbeg = (uint64_t)lb * P.wt_per_block;
    const uint64_t wend = min<uint64_t>(wbeg + P.wt_per_block, nwt);
    const uint32_t ntl = wend > wbeg + wave ? (uint32_t)((wend - wbeg - wave + NW - 1) / NW) : 0u;
    any |= ntl != 0;
    auto tile_of = [&](uint32_t k) -> uint64_t { return wbeg + wave + (uint64_t)NW * min(k, ntl - 1); };
    auto off_of = [&](uint32_t k) -> uint32_t { return offs[min<uint64_t>(tile_of(k) * PV_WT + lane, last)]; };
    // one tile from its windows W (off: this lane's record start)
    // (a tile past the wave's last, live false, is a clamped copy: it parses nothing and its
    // unconditional stores go to the wave's trash line)
    PV_G uint64_t *const trash = P.trash + ((uint64_t)blockIdx.x * NW + wave) * 256;
    auto tile = [&](uint32_t k, uint32_t off, const uint4 (&W)[5]) {
        const bool live = k < ntl;
        const uint64_t t = tile_of(k);
        const uint64_t r0 = t * PV_WT, i = r0 + lane;
        const bool active = live && i < n;
        RecW rw;
        win_words(W, off & 3, rw);
        const FastRec f = fast_fields(rw, h);
        const bool fast = active & (f.ok != 0);
        const uint64_t slowm = __ballot(active & !fast);
        cd += fast ? 1ull << (f.dir * 16) : 0ull;
        cl += fast ? (1ull << (f.l4 == 17 ? 0u : (f.l4 == 6 ? 16u : 32u))) + ((uint64_t)f.syn << 48) : 0ull;
        uint32_t hv = fast ? f.caplen : PV_NOH;
        const uint32_t ip = f.dir == 0 ? rw.at(42) : rw.at(46);
        const bool ipok = fast & (f.dir != 2) & (ip != 0);
        uint64_t ek = tops && ipok ? ((uint64_t)slot << 60) | ((uint64_t)TM_IPV4 << 56) | ((uint64_t)card << 33) |
                                         ((uint64_t)f.dir << 32) | ip
                                   : 0ull;
        if (card && !tops) {
            if (ipok) {
                uint64_t h1, h2;
                murmur_8((uint64_t)(int64_t)(int32_t)ip, h1, h2);
                __hip_atomic_fetch_min(P.cpc + (uint64_t)slot * PV_MIN_WORDS + (uint64_t)(f.dir == 0 ? CPC_SRC : CPC_DST) * PV_CPC_COUPONS +
                                           cpc_coupon(h1, h2),
                                       (int64_t)(P.gbase + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        const uint32_t port = (fast & (f.l4 == 17)) ? dns_port_bf(rw.at(50)) : 0u;
        DnsMsgW dm{};
        bool isdns = port != 0;
        if (__ballot(isdns)) {
            if (isdns) {
                const Parsed o = fast_parsed(f, rw, ts_nano, off);
                uint32_t dp = 0;
                for (uint32_t q = 0; q < P.n_dshift; q++) dp += (int64_t)(4 * i) >= S.dord[q];
                const SAcc R{recs, nullptr, 0, 0, 0, 1};
                DnsMsg d = dns_msg_of(P, R, o, i, port, dp, dp >= P.dskip_before, false);
                d.fkey = fast_flowkey(rw);
                dm = msg_words(d);
            }
        }
        bool istcp = fast & (f.l4 == 6), hasseg = false;
        PvTcpSeg seg;
        const uint32_t temit = P.tcp_emit;
        if (temit && __ballot(istcp)) {
            if (istcp) hasseg = tcp_seg_fast(rw, fast_parsed(f, rw, ts_nano, off), i, seg);
        }
        if (slowm) {
            // general-path records (VLAN, IPv6, options, tunnels, other link types): their indices
            // to the range's list, which pv_net_slow_list parses after this pass (an out-of-line
            // call in the loop made the compiler give every wave a stack: 176 B of scratch a lane and
            // 167 VGPRs, against 101 without it, and C2 222 -> 208 us, profiles/r6/noslow); an LDS
            // reservation, since a returning global atomic would wait on every load in flight
            uint32_t q = 0;
            if (lane == 0) q = atomicAdd(&S.ns, (uint32_t)__popcll(slowm));
            q = __builtin_amdgcn_readlane(q, 0) + __builtin_amdgcn_mbcnt_hi((uint32_t)(slowm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)slowm, 0u));
            if (active && !fast) P.slow_list[wbeg * PV_WT + q] = (uint32_t)i;
        }
        if (__ballot(hv != PV_NOH && hv > 65535)) {
            if (hv != PV_NOH && hv > 65535) { atomicOr(P.flags, PVF_BIG_CAPLEN); hv = 65535; }
        }
        hist_add(S.hist, P.sum + (uint64_t)slot * PV_SUM_WORDS + PV_OFF_PAYLOAD, hv, lane);
        const uint64_t m = __ballot(isdns);
        if (m) {
            uint32_t q = 0;
            if (lane == 0) q = atomicAdd(&S.nd, (uint32_t)__popcll(m));
            q = __builtin_amdgcn_readlane(q, 0);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (isdns) {
                PV_G uint4 *dd = reinterpret_cast<PV_G uint4 *>(P.dq) + 2 * (wbeg * PV_WT + q + below);
                dd[0] = dm.a;
                dd[1] = dm.b;
            }
        }
        if (TC || tops) {
            if (TC || compact) {
                // the IPv4 entry as its address and a direction bit; anything else (an IPv6
                // key of a general-path record) into the range's exception list
                const bool v4 = ek && ((ek >> 32) & ~1ull) == (P.ip_base >> 32);
                const uint64_t xm = __ballot(active && ek && !v4);
                const uint64_t dbit = __ballot(v4 && ((ek >> 32) & 1));
                if (TC) {
                    // every lane (the log has 64 words of slack past the batch) and every lane
                    // the same direction word: two unconditional store instructions
                    PV_G uint32_t *const l32 = live ? P.iplog32 + i : reinterpret_cast<PV_G uint32_t *>(trash) + lane;
                    PV_G uint64_t *const ldw = live ? P.ipdir + t : trash + 32;
                    *l32 = active && v4 ? (uint32_t)ek : 0u;
                    *ldw = dbit;
                } else if (live) {
                    if (active) P.iplog32[i] = v4 ? (uint32_t)ek : 0u;
                    if (lane == 0) P.ipdir[t] = dbit;
                }
                if (xm) {
                    uint32_t q = 0;
                    if (lane == 0) q = atomicAdd(&S.nx, (uint32_t)__popcll(xm));
                    q = __builtin_amdgcn_readlane(q, 0);
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(xm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)xm, 0u));
                    if (active && ek && !v4) {
                        P.iplog[wbeg * PV_WT + q + below] = ek;
                        P.ipx_rep[wbeg * PV_WT + q + below] = (uint32_t)i;
                    }
                }
            } else if (active) {
                P.iplog[i] = ek;
            }
        }
        if (temit) {
            const uint64_t tm = __ballot(istcp);
            if (tm) {
                if (lane == 0) P.tmask[t] = tm;
                tcp_seg_store(P.tseg, P.tseg_cnt, P.tseg_cap, hasseg, seg, lane);
            }
        }
    };
    // software pipeline of depth 3 with unconditional loads: the windows of tiles k + 1 and k + 2
    // in flight while tile k is parsed, every load issued on every path (tile_of clamps past the
    // wave's last tile; tile() skips a clamped copy), so the compiler cannot sink a load behind the
    // parse it should overlap into a loop exit's branch (the conditional form: 237 -> 229 us on C2,
    // profiles/r6). Loads retire in order, so each counted wait the compiler places for a tile's
    // windows leaves the younger loads and the previous tiles' stores in flight.
    if (ntl) {
        uint4 W0[5], W1[5], W2[5];
        uint32_t o0 = off_of(0), o1 = off_of(1), o2 = off_of(2);
        win_load(recs, o0, W0);
        win_load(recs, o1, W1);
        for (uint32_t k = 0; k < ntl; k += 3) {
            const uint32_t oN = off_of(k + 3);
            win_load(recs, o2, W2);  // tile k + 2
            tile(k, o0, W0);
            const uint32_t oN1 = off_of(k + 4);
            win_load(recs, oN, W0);  // tile k + 3
            o0 = oN;
            tile(k + 1, o1, W1);
            const uint32_t oN2 = off_of(k + 5);
            win_load(recs, oN1, W1); // tile k + 4
            o1 = oN1;
            tile(k + 2, o2, W2);
            o2 = oN2;
        }
    }
    // this range's DNS list: its count, and the slot counter reset for the next range (LDS-only
    // barriers: the range's IP-log and DNS-list stores are other kernels' to read, and waiting
    // for them here would stall every wave on their completion)
    lds_barrier();
    if (threadIdx.x == 0) {
        P.mq_cnt[lb] = 0;
        P.dq_cnt[lb] = S.nd;
        if (compact) P.ipx_cnt[lb] = S.nx;
        P.slow_cnt[lb] = S.ns;
        if (S.nd) atomicAdd(P.n_dns, S.nd);
        if (S.ns) atomicAdd(P.n_slow, S.ns);
        S.nd = 0;
        S.nx = 0;
        S.ns = 0;
    }
    lds_barrier();
    }
    {
        const uint32_t fin = (uint32_t)(cd & 0xffff), fout = (uint32_t)((cd >> 16) & 0xffff), funk = (uint32_t)((cd >> 32) & 0xffff);
        const uint32_t nf = fin + fout + funk;
        c.nev += nf; c.n4 += nf;
        c.nin += fin; c.nout += fout; c.nunk += funk;
        c.nudp += (uint32_t)(cl & 0xffff); c.ntcp += (uint32_t)((cl >> 16) & 0xffff);
        c.noth += (uint32_t)((cl >> 32) & 0xffff); c.nsyn += (uint32_t)(cl >> 48);
    }
    NetK K;
    K.sum = P.sum; K.net_groups = groups; K.net_filter_all = 0;
    if (any) knet_flush(K, slot, c);
    lds_barrier();
    for (uint32_t b = threadIdx.x; b < PV_HBINS; b += blockDim.x)
        if (S.hist[b]) ksum_add(K, slot, PV_OFF_PAYLOAD + b, S.hist[b]);
}

// ------------------------------------------------------------------ the lean Net pass, span loads
// The register-window pass's loads touch ~40 lines per instruction at an 80-B record stride, and the
// second to fifth window instruction of a tile hit lines the first one is still fetching: the L1
// spends 57 % of the C2 pass in pending-miss stalls (profiles/r5/tcp_ta). This pass loads a tile
// whose 64 records lie in at most PV_SPAN_MAX bytes (C2: 64 x 80 B) as its span: six 16-B loads a
// lane, each instruction 1 KiB contiguous, one tile ahead; the wave writes the span into its LDS
// buffer and each lane reads its record's 96 bytes back with aligned 16-B reads (an 80-B stride
// puts 16 lanes on 16 distinct bank groups). Tiles spread wider load their windows per lane from
// HBM. Records the fast path does not take are not parsed here (the general path is an out-of-line
// call, and every value live across a call would be spilled with a wait on the whole load queue at
// each reload): their indices go to a list that pv_net_slow_list parses after this pass.
#ifndef PV_SPAN_MAX
#define PV_SPAN_MAX 6144
#endif
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
struct NetSpanState {
    uint32_t hist[PV_HBINS];
    uint32_t nd, ns;
    int64_t dord[PV_MAX_SHIFTS];
    v4u32 buf[4][PV_SPAN_MAX / 16 + 8];
};
// (six named registers of a native vector type: HIP's uint4 copies are byte copies, and the
// buffers they copy from stay in scratch)
struct SpanX {
    v4u32 v0, v1, v2, v3, v4, v5;
};
__device__ __forceinline__ void span_load(const PV_G uint8_t *recs, uint32_t o, uint32_t lane, SpanX &X, uint32_t &b)
{
    const uint32_t o0 = __builtin_amdgcn_readfirstlane(o), o63 = __builtin_amdgcn_readlane(o, 63);
    const uint32_t b16 = o0 & ~15u;
    const uint32_t len = o63 + 80u - b16;
    const PV_G v4u32 *ps = reinterpret_cast<const PV_G v4u32 *>(recs + b16);
    // a span: lane 0's and lane 63's records bound every lane's, within PV_SPAN_MAX bytes
    const bool sp = o63 >= o0 && len <= PV_SPAN_MAX && !__ballot(o < o0 || o > o63);
    b = sp ? b16 : 0xffffffffu;
    // (always six loads, so the compiler's vmcnt waits stay counted; past the span: chunk 0 again)
    const uint32_t lim = sp ? len : 0u;
#define PV_SPAN_LD(j) X.v##j = ps[16u * (lane + 64u * j) < lim ? lane + 64u * j : 0u]
    PV_SPAN_LD(0); PV_SPAN_LD(1); PV_SPAN_LD(2); PV_SPAN_LD(3); PV_SPAN_LD(4); PV_SPAN_LD(5);
#undef PV_SPAN_LD
}
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PV_REG_MINW))) pv_net_kernel_span(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ NetSpanState S;
    constexpr uint32_t NW = 4;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (uint32_t b = threadIdx.x; b < PV_HBINS; b += blockDim.x) S.hist[b] = 0;
    if (threadIdx.x == 0) { S.nd = 0; S.ns = 0; }
    if (threadIdx.x < PV_MAX_SHIFTS) S.dord[threadIdx.x] = P.dpos[threadIdx.x];
    __syncthreads();
    const PV_G uint8_t *const recs = P.recs;
    const PV_G uint32_t *const offs = P.offs;
    const uint64_t n = P.n, last = n - 1;
    const uint32_t slot = P.slot_of[0];
    const uint32_t groups = P.net_groups;
    const bool card = groups & PV_NET_CARDINALITY_BIT;
    const uint32_t ts_nano = P.ts_nano;
    HostNets h;
    {
        const uint32_t n4 = P.nets.n4;
        h.a0 = P.nets.v4_addr[0]; h.m0 = P.nets.v4_mask[0]; h.e0 = n4 > 0 ? ~0u : 0u;
        h.a1 = P.nets.v4_addr[1]; h.m1 = P.nets.v4_mask[1]; h.e1 = n4 > 1 ? ~0u : 0u;
    }
    const uint64_t nwt = (n + PV_WT - 1) / PV_WT;
    uint64_t cd = 0, cl = 0; // fast lanes' packed counters (net_fast_reg's)
    v4u32 *Lq = S.buf[wave];
    for (uint32_t lb = blockIdx.x; lb < P.grid_main; lb += gridDim.x) {
    const uint64_t wbeg = (uint64_t)lb * P.wt_per_block;
    const uint64_t wend = min<uint64_t>(wbeg + P.wt_per_block, nwt);
    const uint32_t ntl = wend > wbeg + wave ? (uint32_t)((wend - wbeg - wave + NW - 1) / NW) : 0u;
    auto tile_of = [&](uint32_t k) -> uint64_t { return wbeg + wave + (uint64_t)NW * min(k, ntl - 1); };
    auto off_of = [&](uint32_t k) -> uint32_t { return offs[min<uint64_t>(tile_of(k) * PV_WT + lane, last)]; };
    auto tile = [&](uint32_t k, uint32_t off, const SpanX &X, uint32_t b) {
        const uint64_t t = tile_of(k);
        const uint64_t i = t * PV_WT + lane;
        const bool active = i < n;
        RecW rw;
        if (b != 0xffffffffu) {
            Lq[lane] = X.v0; Lq[lane + 64] = X.v1; Lq[lane + 128] = X.v2;
            Lq[lane + 192] = X.v3; Lq[lane + 256] = X.v4; Lq[lane + 320] = X.v5;
            // (a wave's LDS operations execute in issue order: only the compiler's order matters)
            asm volatile("" ::: "memory");
            const uint32_t rel = off - b;
            const v4u32 *q = Lq + (rel >> 4);
            uint32_t x[24];
#pragma unroll
            for (int j = 0; j < 6; j++) {
                const v4u32 v = q[j];
                x[4 * j] = v.x; x[4 * j + 1] = v.y; x[4 * j + 2] = v.z; x[4 * j + 3] = v.w;
            }
            // the record's dwords from its dword-aligned start: x[d + m], d = (rel >> 2) & 3
            // (bit selects on opaque masks: written as selects, the compiler indexes the array
            // with d and puts it in scratch)
            uint32_t m1 = 0u - ((rel >> 2) & 1), m2 = 0u - ((rel >> 3) & 1);
            asm volatile("" : "+v"(m1), "+v"(m2));
            uint32_t y[19], z[17];
#pragma unroll
            for (int m = 0; m < 19; m++) y[m] = (x[m + 1] & m1) | (x[m] & ~m1);
#pragma unroll
            for (int m = 0; m < 17; m++) z[m] = (y[m + 2] & m2) | (y[m] & ~m2);
#pragma unroll
            for (int j = 0; j < 16; j++) rw.w[j] = __builtin_amdgcn_alignbyte(z[j + 1], z[j], rel & 3);
            asm volatile("" ::: "memory");
        } else {
            uint4 W[5];
            win_load(recs, off, W);
            win_words(W, off & 3, rw);
        }
        const FastRec f = fast_fields(rw, h);
        const bool fast = active & (f.ok != 0);
        cd += fast ? 1ull << (f.dir * 16) : 0ull;
        cl += fast ? (1ull << (f.l4 == 17 ? 0u : (f.l4 == 6 ? 16u : 32u))) + ((uint64_t)f.syn << 48) : 0ull;
        // the records the fast path does not take: the range's list for pv_net_slow_list (an LDS
        // reservation: a returning global atomic would wait on every load in flight)
        {
            const uint64_t sm = __ballot(active & !fast);
            if (sm) {
                uint32_t q = 0;
                if (lane == 0) q = atomicAdd(&S.ns, (uint32_t)__popcll(sm));
                q = __builtin_amdgcn_readlane(q, 0) + __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                if (active && !fast) P.slow_list[wbeg * PV_WT + q] = (uint32_t)i;
            }
        }
        uint32_t hv = fast ? f.caplen : PV_NOH;
        const uint32_t ip = f.dir == 0 ? rw.at(42) : rw.at(46);
        const bool ipok = fast & (f.dir != 2) & (ip != 0);
        const uint32_t port = (fast & (f.l4 == 17)) ? dns_port_bf(rw.at(50)) : 0u;
        DnsMsgW dm{};
        const bool isdns = port != 0;
        if (__ballot(isdns)) {
            if (isdns) {
                const Parsed o = fast_parsed(f, rw, ts_nano, off);
                uint32_t dp = 0;
                for (uint32_t q = 0; q < P.n_dshift; q++) dp += (int64_t)(4 * i) >= S.dord[q];
                const SAcc R{recs, nullptr, 0, 0, 0, 1};
                DnsMsg dmsg = dns_msg_of(P, R, o, i, port, dp, dp >= P.dskip_before, false);
                dmsg.fkey = fast_flowkey(rw);
                dm = msg_words(dmsg);
            }
        }
        const bool istcp = fast & (f.l4 == 6);
        bool hasseg = false;
        PvTcpSeg seg;
        const uint32_t temit = P.tcp_emit;
        if (temit && __ballot(istcp)) {
            if (istcp) hasseg = tcp_seg_fast(rw, fast_parsed(f, rw, ts_nano, off), i, seg);
        }
        if (__ballot(hv != PV_NOH && hv > 65535)) {
            if (hv != PV_NOH && hv > 65535) { atomicOr(P.flags, PVF_BIG_CAPLEN); hv = 65535; }
        }
        hist_add(S.hist, P.sum + (uint64_t)slot * PV_SUM_WORDS + PV_OFF_PAYLOAD, hv, lane);
        const uint64_t m = __ballot(isdns);
        if (m) {
            uint32_t q = 0;
            if (lane == 0) q = atomicAdd(&S.nd, (uint32_t)__popcll(m));
            q = __builtin_amdgcn_readlane(q, 0);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (isdns) {
                PV_G uint4 *dd = reinterpret_cast<PV_G uint4 *>(P.dq) + 2 * (wbeg * PV_WT + q + below);
                dd[0] = dm.a;
                dd[1] = dm.b;
            }
        }
        // the compact IP log: every lane's word (the log has 64 words of slack past the batch;
        // a deferred record's word is pv_net_slow_list's), the tile's direction word
        const uint64_t ek = ipok ? ((uint64_t)card << 33) | ((uint64_t)f.dir << 32) | ip : 0ull;
        P.iplog32[i] = (uint32_t)ek;
        P.ipdir[t] = __ballot(ipok && f.dir == 1);
        if (temit) {
            const uint64_t tm = __ballot(istcp);
            if (tm) {
                if (lane == 0) P.tmask[t] = tm;
                tcp_seg_store(P.tseg, P.tseg_cnt, P.tseg_cap, hasseg, seg, lane);
            }
        }
    };
    SpanX XA, XB;
    uint32_t oA = 0, oB = 0, bA = 0xffffffffu, bB = 0xffffffffu;
    if (ntl) {
        oA = off_of(0);
        oB = off_of(1);
        span_load(recs, oA, lane, XA, bA);
    }
    for (uint32_t k = 0; k < ntl; k += 2) {
        const uint32_t oN = off_of(k + 2);
        span_load(recs, oB, lane, XB, bB);   // tile k + 1 (a clamped copy past the range's end)
        tile(k, oA, XA, bA);
        if (k + 1 >= ntl) break;
        const uint32_t oN2 = off_of(k + 3);
        span_load(recs, oN, lane, XA, bA);   // tile k + 2
        oA = oN;
        tile(k + 1, oB, XB, bB);
        oB = oN2;
    }
    // this range's DNS list count; the exception list is pv_net_slow_list's (0 here)
    lds_barrier();
    if (threadIdx.x == 0) {
        P.mq_cnt[lb] = 0;
        P.dq_cnt[lb] = S.nd;
        P.ipx_cnt[lb] = 0;
        P.slow_cnt[lb] = S.ns;
        if (S.nd) atomicAdd(P.n_dns, S.nd);
        if (S.ns) atomicAdd(P.n_slow, S.ns);
        S.nd = 0;
        S.ns = 0;
    }
    lds_barrier();
    }
    NetCtr c;
    c.zero();
    {
        const uint32_t fin = (uint32_t)(cd & 0xffff), fout = (uint32_t)((cd >> 16) & 0xffff), funk = (uint32_t)((cd >> 32) & 0xffff);
        const uint32_t nf = fin + fout + funk;
        c.nev += nf; c.n4 += nf;
        c.nin += fin; c.nout += fout; c.nunk += funk;
        c.nudp += (uint32_t)(cl & 0xffff); c.ntcp += (uint32_t)((cl >> 16) & 0xffff);
        c.noth += (uint32_t)((cl >> 32) & 0xffff); c.nsyn += (uint32_t)(cl >> 48);
    }
    NetK K;
    K.sum = P.sum; K.net_groups = groups; K.net_filter_all = 0;
    knet_flush(K, slot, c);
    lds_barrier();
    for (uint32_t b = threadIdx.x; b < PV_HBINS; b += blockDim.x)
        if (S.hist[b]) ksum_add(K, slot, PV_OFF_PAYLOAD + b, S.hist[b]);
}

// The span pass's deferred records (VLAN, IPv6, options, tunnels, other link types), one lane
// each: the general path (net_slow_p: counters' fields, IP entry, DNS message, TCP segment), then
// what the span pass does for a fast record, through atomics (the records' ranges have closed):
// payload histogram, compact IP log word or exception entry, direction bit, DNS list entry, TCP
// tile mask. A persistent grid walks the list.
extern "C" __global__ void __launch_bounds__(256) pv_net_slow_list(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    if (!*P.n_slow) return; // (the common batch: Ethernet + IPv4 only, nothing deferred)
    const uint32_t slot = P.slot_of[0];
    const uint64_t per_range = (uint64_t)P.wt_per_block * PV_WT;
    NetCtr c;
    c.zero();
    for (uint32_t r = blockIdx.x; r < P.grid_main; r += gridDim.x)
    for (uint32_t j = threadIdx.x; j < P.slow_cnt[r]; j += blockDim.x) {
        const uint64_t i = P.slow_list[r * per_range + j];
        const SAcc R{P.recs, nullptr, 0, 0, 0, 1};
        const SlowOut so = net_slow_p(Pp, R, P.offs[i], i);
        Parsed o;
        o.dir = so.dir; o.l3 = so.l3; o.l4 = so.l4; o.syn = so.syn;
        c.add(o);
        uint32_t hv = so.caplen;
        if (hv != PV_NOH) {
            if (hv > 65535) { atomicOr(P.flags, PVF_BIG_CAPLEN); hv = 65535; }
            __hip_atomic_fetch_add(P.sum + (uint64_t)slot * PV_SUM_WORDS + PV_OFF_PAYLOAD + hv, 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint64_t lb = r, t = i / PV_WT;
        if (so.isdns) {
            const uint32_t q = atomicAdd(P.dq_cnt + lb, 1u);
            PV_G uint4 *dd = reinterpret_cast<PV_G uint4 *>(P.dq) + 2 * (lb * per_range + q);
            dd[0] = so.dm.a;
            dd[1] = so.dm.b;
            atomicAdd(P.n_dns, 1u);
        }
        const uint64_t ek = so.ek;
        if (ek) {
            if (((ek >> 32) & ~1ull) == (P.ip_base >> 32)) {
                P.iplog32[i] = (uint32_t)ek;
                if ((ek >> 32) & 1) atomicOr(reinterpret_cast<unsigned long long *>(P.ipdir + t), 1ull << (i & 63));
            } else {
                const uint32_t q = atomicAdd(P.ipx_cnt + lb, 1u);
                P.iplog[lb * per_range + q] = ek;
                P.ipx_rep[lb * per_range + q] = (uint32_t)i;
            }
        }
        if (P.tcp_emit && so.l4 == 6) atomicOr(reinterpret_cast<unsigned long long *>(P.tmask + t), 1ull << (i & 63));
    }
    NetK K;
    K.sum = P.sum; K.net_groups = P.net_groups; K.net_filter_all = 0;
    knet_flush(K, slot, c);
}

extern "C" __global__ void __launch_bounds__(256, PV_NET_MINB) pv_net_kernel(const PvParams *__restrict__ Pp) { net_pass<true>(Pp); }
extern "C" __global__ void __launch_bounds__(256, PV_NET_MINB) pv_net_kernel_ns(const PvParams *__restrict__ Pp) { net_pass<false>(Pp); }
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PV_REG_MINW))) pv_net_kernel_reg(const PvParams *__restrict__ Pp) { net_fast_reg<4>(Pp); }
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PV_REG_MINW))) pv_net_kernel_reg_tc(const PvParams *__restrict__ Pp) { net_fast_reg<4, true>(Pp); }

// ------------------------------------------------------------------ the DNS pass
// One lane per DNS message of the Net pass's work list (same workgroup mapping).
// Each wave stages 128-B windows of its 64 messages in LDS (names past the window
// come from HBM) while the next messages' windows are in flight.
// only_qname_suffix (filter-enabled runs only): the suffix match of every message on the
// DNS work lists, one lane per message, into sfx_of[record], so the DNS pass itself carries
// no suffix code (it cost that pass 11% on C3 when inlined)
extern "C" __global__ void __launch_bounds__(256) pv_dns_suffix(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint32_t nd = P.dq_cnt[blockIdx.x];
    const uint64_t region = (uint64_t)blockIdx.x * P.wt_per_block * PV_WT;
    const PV_G DnsMsg *Q = reinterpret_cast<const PV_G DnsMsg *>(P.dq) + region;
    const GAcc R{P.recs};
    for (uint32_t t = threadIdx.x; t < nd; t += blockDim.x) {
        const DnsMsg dm = Q[t];
        const uint64_t m = dm.moff;
        // header words as dns_process reads them (bytes past the capture read as 0)
        uint32_t w1 = 0, w2 = 0;
        if (dm.mcap >= 12) { w1 = R.u32(m + 4); w2 = R.u32(m + 8); }
        else {
            for (uint32_t b = 4; b < 12; b++) {
                const uint32_t v = b < dm.mcap ? R.u8(m + b) : 0;
                if (b < 8) w1 |= v << (8 * (b - 4)); else w2 |= v << (8 * (b - 8));
            }
        }
        const uint32_t qd = ((w1 & 0xff) << 8) | ((w1 >> 8) & 0xff);
        const uint32_t an = ((w1 >> 8) & 0xff00) | (w1 >> 24);
        const uint32_t ns = ((w2 & 0xff) << 8) | ((w2 >> 8) & 0xff);
        const uint32_t ar = ((w2 >> 8) & 0xff00) | (w2 >> 24);
        P.sfx_of[dm.idx] = (uint8_t)dns_suffix_of(P, R, m, dm.mlen, qd, an, ns, ar);
    }
}

#ifndef PV_DNS_MINW
#define PV_DNS_MINW 1 // tuning: waves per SIMD the DNS pass's register allocation must allow
#endif
// The DNS pass: each workgroup (PV_DNS_WAVES waves, one resident per CU at this kernel's register
// count) walks ranges of the logical grid (lb = blockIdx.x, + gridDim.x), so the grid's three
// ranges per CU are three per workgroup and no partial round of workgroups idles part of the
// chip. Per range: its DNS list, its event region and update log; the key cache and the register
// counters span the workgroup's ranges (the cache is flushed once, into the last range's log).
template <bool SFX, bool FILT>
__device__ __forceinline__ void dns_pass(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ DnsState S;
    // no DNS message in the batch (the Net pass counted them): nothing to do (the update-log
    // counters stay as the Net pass reset them, the key list stays empty)
    if (*P.n_dns == 0) return;
    S.C.clear();
    if (threadIdx.x == 0) S.nresp = 0;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t *L = S.stage[wave];
    DnsCtr c;
    c.zero();
    uint32_t wslot = 0xffffffffu;
    for (uint32_t lb = blockIdx.x; lb < P.grid_main; lb += gridDim.x) {
        const uint32_t nd = P.dq_cnt[lb];
        if (threadIdx.x == 0) {
            S.mq_n[0] = P.mq_cnt[lb];
            S.mq_n[1] = lb;
            S.nev[0] = 0;
            S.nlong = 0;
            // the range's slots in the key list: at most one event per message
            if (P.want_events && nd) S.nev[1] = atomicAdd(P.n_keys, nd);
        }
        __syncthreads();
        const uint64_t region = (uint64_t)lb * P.wt_per_block * PV_WT;
        const PV_G DnsMsg *Q = reinterpret_cast<const PV_G DnsMsg *>(P.dq) + region;
        const uint32_t ntl = (nd + PV_WT - 1) / PV_WT;
        // message and window loads are unconditional (clamped index; an inactive lane's copy is
        // never read), so every iteration issues the same number of loads in the same order and
        // the compiler's vmcnt waits stay exact instead of falling back to vmcnt(0)
        constexpr uint32_t NW = PV_DNS_WAVES;
        uint32_t t = wave;
        uint4 pf[8];
        auto issue = [&](const DnsMsg &d, bool) {
            const uint4 *src = reinterpret_cast<const uint4 *>(P.recs + ((uint64_t)d.moff & ~15ull));
#pragma unroll
            for (int j = 0; j < 8; j++) pf[j] = src[j];
        };
        // The staged tile's descriptors sit in LDS (desc, as raw words) next to its windows; one
        // descriptor is in registers, loaded a tile ahead of its windows. So the only loop-carried
        // loads are the windows (pf) and that descriptor's words (mw), both consumed behind the one
        // wait at the top of the next iteration, and nothing in the decode waits on them.
        const PV_G uint4 *Qw = reinterpret_cast<const PV_G uint4 *>(Q);
        auto msgw = [&](uint32_t t, uint4 &a, uint4 &b) {
            const uint32_t j = min(t * PV_WT + lane, nd - 1);
            a = Qw[2 * (uint64_t)j];
            b = Qw[2 * (uint64_t)j + 1];
        };
        auto win = [&](uint32_t moff) {
            const uint4 *src = reinterpret_cast<const uint4 *>(P.recs + ((uint64_t)moff & ~15ull));
#pragma unroll
            for (int j = 0; j < 8; j++) pf[j] = src[j];
        };
        uint4 mwa{}, mwb{};
        if (t < ntl) {
            uint4 a, b;
            msgw(t, a, b);
            S.desc[wave][0][lane] = a;
            S.desc[wave][1][lane] = b;
            win(a.y);
            msgw(t + NW, mwa, mwb);
        }
        for (; t < ntl; t += NW) {
            t = __builtin_amdgcn_readfirstlane(t);
            const bool active = t * PV_WT + lane < nd;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                L[(4 * j + 0) * PV_WT + lane] = pf[j].x;
                L[(4 * j + 1) * PV_WT + lane] = pf[j].y;
                L[(4 * j + 2) * PV_WT + lane] = pf[j].z;
                L[(4 * j + 3) * PV_WT + lane] = pf[j].w;
            }
            const uint4 da = S.desc[wave][0][lane], db = S.desc[wave][1][lane];
            if (t + NW < ntl) {
                // (a wave's LDS operations retire in order: the reads above see the old words)
                S.desc[wave][0][lane] = mwa;
                S.desc[wave][1][lane] = mwb;
                win(mwa.y);
                msgw(t + 2 * NW, mwa, mwb);
            }
            DnsMsg dm;
            dm.idx = da.x;
            dm.moff = da.y;
            dm.mlen = (uint16_t)(da.z & 0xffff);
            dm.mcap = (uint16_t)(da.z >> 16);
            dm.port = (uint16_t)(da.w & 0xffff);
            dm.flags = (uint8_t)((da.w >> 16) & 0xff);
            dm.period = (uint8_t)(da.w >> 24);
            dm.fkey = db.x;
            dm.sec = db.y;
            dm.nsec = db.z;
            dm.pad = db.w;
            // the wave's register counters follow the slot of its first message
            const uint32_t s0 = P.dslot_of[__builtin_amdgcn_readfirstlane((uint32_t)dm.period)];
            if (s0 != wslot) {
                if (wslot != 0xffffffffu) dns_flush(P, wslot, c);
                wslot = s0;
            }
            const uint64_t wbase = (uint64_t)dm.moff & ~15ull;
            if (PV_DNS_LACC) {
                // a message the window holds whole (every byte the decoder reads lies in
                // [moff, moff + max(mlen, mcap))) decodes from LDS alone; the rest wait for the
                // range's long pass, where no prefetch is in flight
                const bool fits = (uint64_t)dm.moff + max((uint32_t)dm.mlen, (uint32_t)dm.mcap) - wbase <= (uint64_t)(PV_WIN - 4);
                if (active && fits) {
                    const LAcc R{L, wbase, (uint32_t)PV_WT, lane};
                    dns_process<false, false, SFX, FILT>(P, &S.C, S.mq_n, S.nev, &S.nresp, region, R, dm, dslot(P, dm.period) == wslot, c);
                } else if (active) {
                    reinterpret_cast<PV_G uint32_t *>(P.ekeys + region)[atomicAdd(&S.nlong, 1u)] = t * PV_WT + lane;
                }
            } else if (active) {
                const TAcc R{P.recs, L, wbase, PV_WIN - 4, (uint32_t)PV_WT, lane};
                dns_process<false, false, SFX, FILT>(P, &S.C, S.mq_n, S.nev, &S.nresp, region, R, dm, dslot(P, dm.period) == wslot, c);
            }
        }
        __syncthreads();
        if (PV_DNS_LACC && S.nlong) {
            // the long pass: one wave per 64 long messages, their windows staged as above, bytes past
            // the window from HBM (TAcc)
            const uint32_t nl = S.nlong;
            const PV_G uint32_t *lq = reinterpret_cast<const PV_G uint32_t *>(P.ekeys + region);
            for (uint32_t u = wave; u * PV_WT < nl; u += NW) {
                u = __builtin_amdgcn_readfirstlane(u);
                const bool active = u * PV_WT + lane < nl;
                const DnsMsg dm = Q[lq[min(u * PV_WT + lane, nl - 1)]];
                issue(dm, active);
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    L[(4 * j + 0) * PV_WT + lane] = pf[j].x;
                    L[(4 * j + 1) * PV_WT + lane] = pf[j].y;
                    L[(4 * j + 2) * PV_WT + lane] = pf[j].z;
                    L[(4 * j + 3) * PV_WT + lane] = pf[j].w;
                }
                const uint32_t s0 = P.dslot_of[__builtin_amdgcn_readfirstlane((uint32_t)dm.period)];
                if (s0 != wslot) {
                    if (wslot != 0xffffffffu) dns_flush(P, wslot, c);
                    wslot = s0;
                }
                if (active) {
                    const TAcc R{P.recs, L, (uint64_t)dm.moff & ~15ull, PV_WIN - 4, (uint32_t)PV_WT, lane};
                    dns_process<false, false, SFX, FILT>(P, &S.C, S.mq_n, S.nev, &S.nresp, region, R, dm, dslot(P, dm.period) == wslot, c);
                }
            }
            __syncthreads();
        }
        if (lb + gridDim.x >= P.grid_main) {
            cache_flush(P, S.C, PV_NCACHE, S.mq_n);
            __syncthreads();
        }
        if (P.want_events) {
            // messages without an event leave their reserved key slots as sentinels (all ones:
            // sorted behind every event key, whose top bit is clear)
            const uint32_t ne = S.nev[0];
            for (uint32_t j = ne + threadIdx.x; j < nd; j += blockDim.x) {
                P.skeys[(uint64_t)S.nev[1] + j] = ~0ull;
                P.svals[(uint64_t)S.nev[1] + j] = 0;
            }
            if (threadIdx.x == 0 && ne) atomicAdd(P.n_events, ne);
        }
        if (threadIdx.x == 0) P.mq_cnt[lb] = S.mq_n[0];
    }
    if (wslot != 0xffffffffu) dns_flush(P, wslot, c);
    if (threadIdx.x == 0 && S.nresp) atomicAdd(P.n_events + 1, S.nresp);
}
extern "C" __global__ void __launch_bounds__(64 * PV_DNS_WAVES, PV_DNS_MINW) pv_dns_kernel(const PvParams *__restrict__ Pp)
{
    dns_pass<false, false>(Pp);
}
// the UDP DNS pass's top_ecs updates into the global table (global_add, as the TCP pass inserts
// its own): kept out of the pass, whose registers then follow no device-call convention
extern "C" __global__ void __launch_bounds__(256) pv_dns_ecs(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint32_t n = min(*P.n_ecs, P.ecs_cap);
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const uint4 e = reinterpret_cast<const PV_G uint4 *>(P.ecs_list)[j];
        global_add(P, e.z, (uint64_t)e.x | (uint64_t)e.y << 32, 1, e.w);
    }
}
// a context with DNS filters (v1 or v2), no suffix
extern "C" __global__ void __launch_bounds__(64 * PV_DNS_WAVES, PV_DNS_MINW) pv_dns_kernel_f(const PvParams *__restrict__ Pp)
{
    dns_pass<false, true>(Pp);
}
// only_qname_suffix / public_suffix_list runs: suffix sizes of any length (agg_domain_r)
extern "C" __global__ void __launch_bounds__(64 * PV_DNS_WAVES, PV_DNS_MINW) pv_dns_kernel_sfx(const PvParams *__restrict__ Pp)
{
    dns_pass<true, true>(Pp);
}

// ------------------------------------------------------------------ Net v2
// record range of workgroup b (the Net pass mapping), clipped to the batch
__device__ __forceinline__ void wg_records(PV_CREF(PvParams) P, uint32_t b, uint64_t &r0, uint64_t &r1)
{
    r0 = min<uint64_t>((uint64_t)b * P.wt_per_block * PV_WT, P.n);
    r1 = min<uint64_t>(r0 + (uint64_t)P.wt_per_block * PV_WT, P.n);
}
// NetworkMetricsBucket v2 (src/handlers/net/v2/NetStreamHandler.cpp:494-532,650-716): every
// metric per direction (in = toHost, out = fromHost, unknown). In: the source address, out:
// the destination, unknown: both. Counters, payload sizes, IP cardinality and top IPv4 /
// IPv6. The v2 manager sees the same events as v1's (every packet), so its periods are the
// Net window's and it lives in the Net part of each slot. One lane per record over the Net
// pass's workgroup ranges (same grid), records parsed straight from HBM; counters and the
// payload histogram of the range's first period in LDS, top-N keys and CPC coupons through
// an LDS key cache into the workgroup's update log (after the DNS pass's entries).
#define PV_N2_HBINS 1024
#define LM2_CPC 3 // cache-local: CPC coupon of a direction (payload dir << 17 | coupon)
struct Net2State {
    KeyCache<PV_NCACHE> C;
    uint32_t ctr[PV_MAX_SHIFTS + 1][PV_NET2_CTRS];
    uint32_t hist[3][PV_N2_HBINS];
    uint32_t mq_n[2];
};
__device__ __forceinline__ void n2_key(PV_CREF(PvParams) P, Net2State &S, uint32_t slot, uint64_t key, uint32_t idx)
{
    uint32_t first;
    if (!S.C.add((key & ((1ull << 60) - 1)) | ((uint64_t)slot << 60), 1, idx, first)) log_put(P, S.mq_n, slot, key, 1, idx);
}
__device__ __forceinline__ void n2_coupon(PV_CREF(PvParams) P, Net2State &S, uint32_t slot, uint32_t dir, uint32_t coupon,
                                          uint32_t idx)
{
    uint32_t first;
    if (!S.C.add(PV_LKEY(slot, LM2_CPC, ((uint64_t)dir << 17) | coupon), 1, idx, first))
        cpc_min(P, slot, CPC_V2 + dir, coupon, (int64_t)(P.gbase + idx));
}
extern "C" __global__ void __launch_bounds__(256) pv_net2_kernel(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ Net2State S;
    S.C.clear();
    for (uint32_t i = threadIdx.x; i < (PV_MAX_SHIFTS + 1) * PV_NET2_CTRS; i += blockDim.x) (&S.ctr[0][0])[i] = 0;
    for (uint32_t i = threadIdx.x; i < 3 * PV_N2_HBINS; i += blockDim.x) (&S.hist[0][0])[i] = 0;
    if (threadIdx.x == 0) { S.mq_n[0] = P.mq_cnt[blockIdx.x]; S.mq_n[1] = blockIdx.x; }
    __syncthreads();
    const uint32_t g = P.net2_groups;
    const bool card = g & PV_N2G_CARDINALITY, tops = g & PV_N2G_TOP_IPS;
    uint64_t r0, r1;
    wg_records(P, blockIdx.x, r0, r1);
    const uint32_t p0 = r0 < r1 ? period_of(P, r0) : 0u;
    const ParseCfg C = parse_cfg(P);
    const GAcc R{P.recs};
    for (uint64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
        const uint32_t p = period_of(P, i);
        if (p < P.skip_before) continue; // a period already outside the window
        const uint32_t slot = P.slot_of[p];
        uint32_t *ctr = S.ctr[p];
        // deep sampling: the v2 manager's draws equal v1's (same generator seed, one draw per
        // packet); not deep: counters without SYN and the payload size only (net/v2 ...cpp:494-500)
        const bool deep = !P.ndeep_net || !((P.ndeep_net[i >> 5] >> (i & 31)) & 1);
        atomicAdd(&ctr[N2_EVENTS], 1u);
        if (deep) atomicAdd(&ctr[N2_SAMPLES], 1u);
        Parsed o;
        parse_record(R, C, P, P.offs[i], o);
        const uint32_t d = o.dir;
        uint32_t *dc = ctr + N2_DIR + 8 * d;
        atomicAdd(&dc[N2_TOTAL], 1u);
        if (o.l3 == 4) atomicAdd(&dc[N2_V4], 1u);
        else if (o.l3 == 6) atomicAdd(&dc[N2_V6], 1u);
        if (o.l4 == 17) atomicAdd(&dc[N2_UDP], 1u);
        else if (o.l4 == 6) {
            atomicAdd(&dc[N2_TCP], 1u);
            if (o.syn && deep) atomicAdd(&dc[N2_SYN], 1u);
        } else atomicAdd(&dc[N2_OTHER], 1u);
        const uint32_t cl = min(o.caplen, 65535u);
        if (p == p0 && cl < PV_N2_HBINS) atomicAdd(&S.hist[d][cl], 1u);
        else sum_add(P, slot, PV_OFF_PAYLOAD2 + d * PV_PAYLOAD_BINS + cl, 1);
        if (!(card || tops) || !deep) continue;
        const uint32_t idx = (uint32_t)i;
        if (o.has4) {
            if (o.l3 != 4) continue;
            for (uint32_t side = 0; side < 2; side++) { // source, then destination
                if (side == 0 ? d == 1 : d == 0) continue;
                const uint32_t ip = R.u32(o.v4 + (side ? 16 : 12));
                if (!ip) continue;
                if (card) {
                    uint64_t h1, h2;
                    murmur_8((uint64_t)(int64_t)(int32_t)ip, h1, h2);
                    n2_coupon(P, S, slot, d, cpc_coupon(h1, h2), idx);
                }
                if (tops) n2_key(P, S, slot, PV_V2_IP4(d, ip), idx);
            }
        } else if (o.has6) {
            if (o.l3 != 6) continue;
            for (uint32_t side = 0; side < 2; side++) {
                if (side == 0 ? d == 1 : d == 0) continue;
                const uint64_t a = side ? o.v6 + 24 : o.v6 + 8;
                const uint64_t w0 = (uint64_t)R.u32(a) | ((uint64_t)R.u32(a + 4) << 32);
                const uint64_t w1 = (uint64_t)R.u32(a + 8) | ((uint64_t)R.u32(a + 12) << 32);
                if (!(w0 | w1)) continue;
                uint64_t h1, h2;
                murmur_16(w0, w1, h1, h2);
                if (card) n2_coupon(P, S, slot, d, cpc_coupon(h1, h2), idx);
                if (tops) n2_key(P, S, slot, PV_V2_IP6(d, h1 ^ (h2 << 1)), idx);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < (P.n_shift + 1) * PV_NET2_CTRS; i += blockDim.x) {
        const uint32_t p = i / PV_NET2_CTRS, w = i % PV_NET2_CTRS;
        if (S.ctr[p][w]) sum_add(P, P.slot_of[p], PV_OFF_NET2 + w, S.ctr[p][w]);
    }
    if (r0 < r1 && p0 >= P.skip_before)
        for (uint32_t i = threadIdx.x; i < 3 * PV_N2_HBINS; i += blockDim.x)
            if ((&S.hist[0][0])[i])
                sum_add(P, P.slot_of[p0], PV_OFF_PAYLOAD2 + (i / PV_N2_HBINS) * PV_PAYLOAD_BINS + i % PV_N2_HBINS,
                        (&S.hist[0][0])[i]);
    for (uint32_t j = threadIdx.x; j < PV_NCACHE; j += blockDim.x) {
        const uint64_t k = S.C.key[j];
        if (!k || !S.C.cnt[j]) continue;
        const uint32_t slot = (uint32_t)(k >> 60), lm = (uint32_t)(k >> 56) & 15;
        const uint64_t pay = k & 0x00ffffffffffffffULL;
        if (lm == LM2_CPC) cpc_min(P, slot, CPC_V2 + (uint32_t)(pay >> 17), (uint32_t)(pay & 0x1ffff), (int64_t)(P.gbase + S.C.rep[j]));
        else log_put(P, S.mq_n, slot, PV_KEY(lm, pay), S.C.cnt[j], S.C.rep[j]);
    }
    __syncthreads();
    if (threadIdx.x == 0) P.mq_cnt[blockIdx.x] = S.mq_n[0];
}

// ------------------------------------------------------------------ top-N merge
// The parse passes leave per-workgroup update logs. They are bucketed by table region
// (count -> scan -> scatter); then one workgroup per region merges the region's updates:
// it loads the region (keys, counts) into LDS, applies every update with LDS atomics,
// writes the region back with coalesced stores and lists the entries it created, whose
// names pv_topn_names decodes. No update waits on an HBM round trip and no update
// issues an HBM atomic (regions with only a few updates take the direct path).
#define PV_RS (1u << PV_REGION_LOG2)
// Visits j in [0, n) with this thread's stride-blockDim.x share, U loads in flight per
// thread: the loops below are bound by load latency, not by their LDS work.
template <int U, class Ld, class Body>
__device__ __forceinline__ void batched(uint64_t n, Ld ld, Body body)
{
    for (uint64_t j0 = threadIdx.x; j0 < n; j0 += (uint64_t)U * blockDim.x) {
        decltype(ld(0)) v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t j = j0 + (uint64_t)u * blockDim.x;
            if (j < n) v[u] = ld(j);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t j = j0 + (uint64_t)u * blockDim.x;
            if (j < n) body(j, v[u]);
        }
    }
}
#define PV_E16(q) reinterpret_cast<const PV_G ulonglong2 *>(q)
#define PV_W_IP4 (1u << 31)  // weight word of a combined IPv4 entry: flag | dir << 30 | card << 29 | count

// CPC coupon of an IPv4 address (cpc_sketch update of the int32 address)
__device__ __forceinline__ uint32_t ip4_coupon(uint32_t ip)
{
    uint64_t h1, h2;
    murmur_8((uint64_t)(int64_t)(int32_t)ip, h1, h2);
    return cpc_coupon(h1, h2);
}

// table of an update-log entry (slot in bits 60..63, the key's metric)
__device__ __forceinline__ uint32_t entry_table(uint64_t e0)
{
    return PV_TSLOT((uint32_t)(e0 >> 60), PV_KEY_METRIC(e0 & ((1ull << 60) - 1)));
}
__device__ __forceinline__ uint32_t log_region(PV_CREF(PvParams) P, uint64_t e0)
{
    return tregion(P, tkey_hash(e0 & ((1ull << 60) - 1)));
}
// run table word: start (24 bits) | count (24 bits) << 24 | the handler's tables << 48
__device__ __forceinline__ uint64_t pv_run_word(uint32_t start, uint32_t cnt, uint32_t tabs)
{
    return (uint64_t)start | (uint64_t)cnt << 24 | (uint64_t)((tabs | tabs >> PV_SLOTS) & 0xffffu) << 48;
}
// run key of an entry: its table region, split by handler (Net tables, DNS tables), so a
// merge workgroup reads only entries of its own handler's tables (one table, usually)
__device__ __forceinline__ uint32_t run_key(PV_CREF(PvParams) P, uint64_t e0)
{
    return (entry_table(e0) / PV_SLOTS) << P.reg_log2 | log_region(P, e0);
}
// table key (slot bits kept) of a dense IP log entry: IPv4 drops the card / dir bits
__device__ __forceinline__ uint64_t ip_tkey(uint64_t e)
{
    return PV_KEY_METRIC(e & ((1ull << 60) - 1)) == TM_IPV4 ? (e & (0xffull << 56)) | (e & 0xffffffffull) : e;
}

// Combine: one workgroup per Net/DNS workgroup range aggregates its update log and its
// records' dense IP entries in an LDS table (key -> weight, smallest record index), so a
// heavy hitter leaves one entry per range instead of one per packet; entries the table
// cannot take spill to the workgroup's part of tp_buf. Then the workgroup writes its
// combined list sorted by table region (counting sort in LDS) and publishes, per region,
// where its run starts and how long it is (cb_run): pv_topn_merge reads each region's runs
// straight from the lists, so no bucketing pass over the entries is needed.
#define PV_W_CNT ((1u << 29) - 1) // weight bits of a dense IPv4 entry
#ifndef PV_CB_U
#define PV_CB_U 8 // tuning: dense IP log loads in flight per combine thread
#endif
#ifndef PV_MG_U
#define PV_MG_U 8 // tuning: run entries in flight per merge thread
#endif
template <uint32_t CN, uint32_t NR>
struct CombState {
    alignas(16) uint64_t key[CN];
    uint32_t cnt[CN];
    uint32_t rep[CN];
    uint32_t h[NR];   // entries per region, then the placement cursors
    uint32_t tb[NR / 2]; // tables among each region's entries (16 bits a region: the run word's
                         // folded PV_TSLOT bit), two regions a word
    uint32_t wsum[PV_CB_THREADS / 64];
    uint32_t nsp;
    uint32_t hm; // handlers among the entries (bit 0 Net, 1 DNS)
};
// combined entry (e0 = slot | table key, e1 = weight word | rep << 32) of a cache key;
// IPv4 cache keys are dense entries (card << 33 | dir << 32 | address)
__device__ __forceinline__ ulonglong2 comb_entry(uint64_t ck, uint32_t w, uint32_t rep)
{
    uint64_t e0 = ck;
    if (PV_KEY_METRIC(ck & ((1ull << 60) - 1)) == TM_IPV4 && !PV_IS_V2_IP4(ck & ((1ull << 60) - 1))) {
        // a dense IP log entry (v1): table key without the card / dir bits
        e0 = ip_tkey(ck);
        w = PV_W_IP4 | ((uint32_t)(ck >> 32) & 1u) << 30 | ((uint32_t)(ck >> 33) & 1u) << 29 | (w & PV_W_CNT);
    }
    return make_ulonglong2(e0, (uint64_t)w | ((uint64_t)rep << 32));
}
template <class St>
__device__ __forceinline__ void comb_count(PV_CREF(PvParams) P, St &S, uint64_t e0)
{
    const uint32_t r = run_key(P, e0);
    atomicAdd(&S.h[r], 1u);
    const uint32_t bit = 1u << ((entry_table(e0) & 15u) + 16u * (r & 1u));
    if (!(S.tb[r >> 1] & bit)) atomicOr(&S.tb[r >> 1], bit);
}
#ifndef PV_CB_BUCKET
#define PV_CB_BUCKET 1 // probe aligned 4-entry buckets (two 16-B LDS reads each), at most 4 (0: 16 dependent
                       // single-entry probes; C3 combine 307 -> 271 us, C4 229 -> 216, profiles/r4/ab)
#endif
// one aligned 4-entry bucket of the combine table: match or claim; false = the bucket is full of
// other keys
template <class St>
__device__ __forceinline__ bool comb_bucket(PV_CREF(PvParams) P, St &S, uint32_t b, uint64_t ck, uint32_t w, uint32_t rep)
{
    const uint4 *kp = reinterpret_cast<const uint4 *>(&S.key[b]);
    const uint4 lo = kp[0], hi = kp[1];
    const uint64_t cur4[4] = {(uint64_t)lo.x | ((uint64_t)lo.y << 32), (uint64_t)lo.z | ((uint64_t)lo.w << 32),
                              (uint64_t)hi.x | ((uint64_t)hi.y << 32), (uint64_t)hi.z | ((uint64_t)hi.w << 32)};
#pragma unroll
    for (int j = 0; j < 4; j++) {
        uint64_t cur = cur4[j];
        if (cur == 0) {
            const uint64_t prev = atomicCAS((unsigned long long *)&S.key[b + j], 0ull, (unsigned long long)ck);
            cur = prev == 0 ? ck : prev;
        }
        if (cur == ck) {
            atomicAdd(&S.cnt[b + j], w);
            if (rep < S.rep[b + j]) atomicMin(&S.rep[b + j], rep);
            return true;
        }
    }
    return false;
}
// an entry the LDS table cannot take: to the workgroup's spill list, counted
template <class St>
__device__ __forceinline__ void comb_spill(PV_CREF(PvParams) P, St &S, PV_G ulonglong2 *sp, uint64_t ck, uint32_t w,
                                           uint32_t rep)
{
    const ulonglong2 e = comb_entry(ck, w, rep);
    sp[atomicAdd(&S.nsp, 1u)] = e;
    comb_count(P, S, e.x);
}
template <uint32_t CN, class St>
__device__ __forceinline__ void comb_add(PV_CREF(PvParams) P, St &S, PV_G ulonglong2 *sp, uint64_t ck, uint32_t w,
                                         uint32_t rep)
{
    uint32_t pos = (uint32_t)(fmix64(ck) >> 20) & (CN - 1);
#if PV_CB_BUCKET
    for (int g = 0; g < 4; g++)
        if (comb_bucket(P, S, ((pos & ~3u) + 4u * g) & (CN - 1), ck, w, rep)) return;
    comb_spill(P, S, sp, ck, w, rep);
    return;
#endif
    for (int probe = 0; probe < 16; probe++) {
        uint64_t cur = S.key[pos];
        if (cur == 0) {
            const uint64_t prev = atomicCAS((unsigned long long *)&S.key[pos], 0ull, (unsigned long long)ck);
            cur = prev == 0 ? ck : prev;
        }
        if (cur == ck) {
            atomicAdd(&S.cnt[pos], w);
            if (rep < S.rep[pos]) atomicMin(&S.rep[pos], rep);
            return;
        }
        pos = (pos + 1) & (CN - 1);
    }
    comb_spill(P, S, sp, ck, w, rep);
}

// comb_add with the first probe's key and rep words already read (cur0 / rep0, read for a whole
// batch at once so the LDS round trips overlap)
template <uint32_t CN, class St>
__device__ __forceinline__ void comb_add_pre(PV_CREF(PvParams) P, St &S, PV_G ulonglong2 *sp, uint64_t ck, uint32_t w,
                                             uint32_t rep, uint32_t pos, uint64_t cur0, uint32_t rep0)
{
    uint64_t cur = cur0;
#if PV_CB_BUCKET
    // the pre-read first probe, then the aligned buckets after it
    if (cur == 0) {
        const uint64_t prev = atomicCAS((unsigned long long *)&S.key[pos], 0ull, (unsigned long long)ck);
        cur = prev == 0 ? ck : prev;
        rep0 = 0xffffffffu;
    }
    if (cur == ck) {
        atomicAdd(&S.cnt[pos], w);
        if (rep < rep0) atomicMin(&S.rep[pos], rep);
        return;
    }
    for (int g = 1; g <= 4; g++)
        if (comb_bucket(P, S, ((pos & ~3u) + 4u * g) & (CN - 1), ck, w, rep)) return;
    comb_spill(P, S, sp, ck, w, rep);
    return;
#endif
    for (int probe = 0; probe < 16; probe++) {
        if (probe) { cur = S.key[pos]; rep0 = 0; }
        if (cur == 0) {
            const uint64_t prev = atomicCAS((unsigned long long *)&S.key[pos], 0ull, (unsigned long long)ck);
            cur = prev == 0 ? ck : prev;
            rep0 = 0xffffffffu;
        }
        if (cur == ck) {
            atomicAdd(&S.cnt[pos], w);
            if (rep < rep0 || probe) atomicMin(&S.rep[pos], rep);
            return;
        }
        pos = (pos + 1) & (CN - 1);
    }
    comb_spill(P, S, sp, ck, w, rep);
}

// exclusive prefix of v over the workgroup (all threads call it); *total = the sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *wsum, uint32_t &total)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (uint32_t k = 0; k < nw; k++) {
        const uint32_t s = wsum[k];
        if (k < wv) base += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return base + incl - v;
}

template <uint32_t CN, uint32_t NR>
__device__ __forceinline__ void topn_combine(PV_CREF(PvParams) P)
{
    using St = CombState<CN, NR>;
    __shared__ St S;
    TST_DECL
    const uint32_t nreg = 2u << P.reg_log2; // run keys
    for (uint32_t j = threadIdx.x; j < CN; j += blockDim.x) { S.key[j] = 0; S.cnt[j] = 0; S.rep[j] = 0xffffffffu; }
    for (uint32_t r = threadIdx.x; r < nreg; r += blockDim.x) {
        S.h[r] = 0;
        if (!(r & 1)) S.tb[r >> 1] = 0;
    }
    if (threadIdx.x == 0) S.nsp = 0;
    __syncthreads();
    TST(0)
    // this workgroup's grid ranges [g0, g1) (cb_fan of them): their update logs and IP logs into
    // one table, one list at the first range's place
    const uint32_t g0 = blockIdx.x * P.cb_fan, g1 = min(g0 + P.cb_fan, P.grid_main);
    const uint64_t wbase = (uint64_t)g0 * P.mq_cap;
    PV_G ulonglong2 *sp = reinterpret_cast<PV_G ulonglong2 *>(P.tp_buf) + wbase;
    PV_G ulonglong2 *out = reinterpret_cast<PV_G ulonglong2 *>(P.cb) + wbase;
    for (uint32_t gr = g0; gr < g1; gr++) {
    const uint32_t cnt = P.mq_cnt[gr];
    const PV_G uint64_t *q = P.mq + (uint64_t)gr * P.mq_cap * 2;
    batched<8>(cnt, [&](uint64_t j) { return PV_E16(q)[j]; },
               [&](uint64_t, ulonglong2 e) { comb_add<CN>(P, S, sp, e.x, (uint32_t)e.y, (uint32_t)(e.y >> 32)); });
    if (P.net_groups & PV_NET_TOP_IPS_BIT) {
        uint64_t a, z;
        wg_records(P, gr, a, z);
        const PV_G uint64_t *ipl = P.iplog + a;
        if (P.ip_compact) {
            // the register-window pass's compact log: address + direction bit, then the
            // range's exception entries
            // software-pipelined per batch of PV_CB_U entries a thread: the log words and their
            // direction words in flight together, then every entry's first-probe key and rep
            // words read from LDS together, then the inserts (most end at that first probe)
            const PV_G uint32_t *ip4 = P.iplog32;
            const uint64_t nn = z - a, bd = blockDim.x;
            const uint64_t ipb = P.ip_base;
            for (uint64_t j0 = threadIdx.x; j0 < nn; j0 += (uint64_t)PV_CB_U * bd) {
                uint32_t ipv[PV_CB_U];
                uint64_t dw[PV_CB_U];
#pragma unroll
                for (int u = 0; u < PV_CB_U; u++) {
                    const uint64_t j = j0 + (uint64_t)u * bd;
                    ipv[u] = j < nn ? ip4[a + j] : 0u;
                    dw[u] = j < nn ? P.ipdir[(a + j) >> 6] : 0ull;
                }
                uint64_t ck[PV_CB_U], cur[PV_CB_U];
                uint32_t pos[PV_CB_U], rp[PV_CB_U];
#pragma unroll
                for (int u = 0; u < PV_CB_U; u++) {
                    const uint64_t r = a + j0 + (uint64_t)u * bd;
                    ck[u] = ipb | ((dw[u] >> (r & 63)) & 1) << 32 | ipv[u];
                    pos[u] = (uint32_t)(fmix64(ck[u]) >> 20) & (CN - 1);
                    cur[u] = ipv[u] ? S.key[pos[u]] : 0ull;
                    rp[u] = ipv[u] ? S.rep[pos[u]] : 0u;
                }
#pragma unroll
                for (int u = 0; u < PV_CB_U; u++)
                    if (ipv[u]) comb_add_pre<CN>(P, S, sp, ck[u], 1u, (uint32_t)(a + j0 + (uint64_t)u * bd), pos[u], cur[u], rp[u]);
            }
            const uint32_t nx = P.ipx_cnt[gr];
            for (uint32_t q = threadIdx.x; q < nx; q += blockDim.x) comb_add<CN>(P, S, sp, ipl[q], 1u, P.ipx_rep[a + q]);
        } else {
            batched<PV_CB_U>(z - a, [&](uint64_t j) { return ipl[j]; }, [&](uint64_t j, uint64_t e) {
                if (e) comb_add<CN>(P, S, sp, e, 1u, (uint32_t)(a + j));
            });
        }
    }
    }
    if (threadIdx.x == 0) S.hm = 0;
    __syncthreads();
    TST(1)
    // the table's entries per region (the spilled ones were counted as they spilled)
    for (uint32_t j = threadIdx.x; j < CN; j += blockDim.x)
        if (S.key[j]) comb_count(P, S, comb_entry(S.key[j], S.cnt[j], S.rep[j]).x);
    __syncthreads();
    TST(2)
    // region run starts: each thread scans a contiguous share of the regions
    const uint32_t per = (nreg + blockDim.x - 1) / blockDim.x;
    const uint32_t r0 = min(threadIdx.x * per, nreg), r1 = min(r0 + per, nreg);
    uint32_t s = 0;
    for (uint32_t r = r0; r < r1; r++) s += S.h[r];
    // handlers with entries in this workgroup (a share never straddles the two halves: per | half)
    {
        const uint32_t hb = s ? 1u << (r0 >> P.reg_log2) : 0u;
        const uint64_t b0 = __ballot(hb & 1), b1 = __ballot(hb & 2);
        if ((threadIdx.x & 63) == 0 && (b0 | b1)) atomicOr(&S.hm, (b0 ? 1u : 0u) | (b1 ? 2u : 0u));
    }
    uint32_t total;
    uint32_t run = block_excl_scan(s, S.wsum, total); // (its barriers publish S.hm)
    const uint32_t hm = S.hm;
    // handlers with entries in this batch (pv_topn_merge's workgroups of the other exit early)
    if (threadIdx.x < 2 && ((hm >> threadIdx.x) & 1)) atomicOr(P.tp_hands, 1u << threadIdx.x);
    if (threadIdx.x == 0) P.cb_hm[blockIdx.x] = hm;
    // this workgroup's column of the run table: [run key][XCD][workgroup / 8], so the
    // workgroups of one XCD (blockIdx % 8) fill whole lines of its L2; a handler without entries
    // here writes no words (the merge reads cb_hm first)
    const uint32_t ng8 = (P.cb_grid + 7) / 8;
    PV_G uint64_t *col = P.cb_run + (blockIdx.x % 8) * ng8 + blockIdx.x / 8;
    for (uint32_t r = r0; r < r1; r++) {
        const uint32_t c = S.h[r];
        if ((hm >> (r >> P.reg_log2)) & 1) col[(uint64_t)r * 8 * ng8] = pv_run_word(run, c, (S.tb[r >> 1] >> (16u * (r & 1u))) & 0xffffu);
        S.h[r] = run; // the placement cursor
        run += c;
    }
    lds_barrier(); // the run-table stores are the merge kernel's to read
    TST(3)
    for (uint32_t j = threadIdx.x; j < CN; j += blockDim.x)
        if (S.key[j]) {
            const ulonglong2 e = comb_entry(S.key[j], S.cnt[j], S.rep[j]);
            out[atomicAdd(&S.h[run_key(P, e.x)], 1u)] = e;
        }
    // spilled entries (this workgroup's own writes: same CU, coherent after the barrier)
    const uint32_t nsp = S.nsp;
    batched<8>(nsp, [&](uint64_t j) { return sp[j]; },
               [&](uint64_t, ulonglong2 e) { out[atomicAdd(&S.h[run_key(P, e.x)], 1u)] = e; });
    if (threadIdx.x == 0) P.cb_cnt[blockIdx.x] = total;
#ifdef PV_TSTAMPS
    __syncthreads();
#endif
    TST(4)
    TST_FLUSH(0)
}
// LDS: an 8192-entry table with up to 2^10 regions per table (152 KiB), 2048 entries with
// more (128 KiB); two run keys per region
#ifndef PV_CB_CN
#define PV_CB_CN 8192
#endif
static_assert(PV_SLOTS == 16, "pv_topn_combine folds a table bit to 16 bits a region");
extern "C" __global__ void __launch_bounds__(PV_CB_THREADS) pv_topn_combine(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    topn_combine<PV_CB_CN, 2048>(P);
}
extern "C" __global__ void __launch_bounds__(PV_CB_THREADS) pv_topn_combine_r12(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    topn_combine<2048, 2u << PV_MAX_REGIONS_LOG2>(P);
}

// Merge, round 5: a region's keys (32 KiB) and this batch's weight per entry (32 KiB) in LDS, so two
// workgroups share a CU (one's loads overlap the other's inserts); the count words are read at
// write-back for the existing entries the batch changed, never for the others; the IPv4 CPC
// minima were applied by the combine. PV_CREATED marks an entry this batch claimed.
#define PV_MG_THREADS 512
#ifndef PV_MG_U2
#define PV_MG_U2 4 // tuning: run entries in flight per merge thread
#endif
#define PV_MG_NN 640 // created named entries a workgroup lists in LDS (more go straight to the list)
#define PV_CREATED (1ull << 63)
#define PV_MV4 (1ull << 62)              // LDS key word of a v1 IPv4 entry (minima inside)
#define PV_MN1 (0xffffffull << 32)       // its direction-1 minimum (0xffffff: none)
#define PV_DL0 (0xffffffffull << 32)     // a weight word's start: direction-0 minimum unset
// a v1 IPv4 table key (bits 32..55 zero; Net v2 keys set bit 40)
__device__ __forceinline__ bool mv4_key(uint64_t k) { return PV_KEY_METRIC(k) == TM_IPV4 && !((k >> 40) & 1); }
// an LDS key word without its batch state (created bit, direction-1 minimum)
__device__ __forceinline__ uint64_t mv4_norm(uint64_t w) { return w & ~(PV_CREATED | ((w & PV_MV4) ? PV_MN1 : 0ull)); }
struct MergeState {
    alignas(16) uint64_t key[PV_RS];
    uint64_t dl[PV_RS];
    uint32_t nrep[PV_MG_NN]; // created named entries: source record, region index (past the list's
    uint16_t nidx[PV_MG_NN]; // capacity the source record waits in the entry's aux word)
    uint32_t nnew, nbase, ncr;
    uint32_t ip4c; // the run key has IPv4 entries with a cardinality update
};
// The region's runs in the combine workgroups' region-sorted lists (cb_run): run i holds
// entries [pref[i], pref[i+1]) of the region, from list list[i] at start[i].
struct MergeRuns {
    uint32_t start[PV_MAX_GRID + 8];
    uint32_t pref[PV_MAX_GRID + 9];
    uint16_t list[PV_MAX_GRID + 8];
    uint32_t wsum[16];
    uint32_t tabs;
};
static_assert(2 * PV_MG_THREADS >= (PV_MAX_GRID + 7) / 8 * 8, "two runs per merge thread");
static_assert(sizeof(MergeState) + sizeof(MergeRuns) <= 80 * 1024, "pv_topn_merge: two workgroups per CU");
extern "C" uint32_t pv_topn_merge_threads() { return PV_MG_THREADS; }
// (waves_per_eu 4: two 8-wave workgroups per CU need at most 128 VGPRs a lane)
extern "C" __global__ void __launch_bounds__(PV_MG_THREADS) __attribute__((amdgpu_waves_per_eu(4))) pv_topn_merge(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint32_t rk = blockIdx.x;                  // run key: handler << reg_log2 | region
    const uint32_t r = rk & ((1u << P.reg_log2) - 1);
    const uint32_t hd = rk >> P.reg_log2;            // 0 Net tables, 1 DNS tables
    if (!((*P.tp_hands >> hd) & 1)) return; // no entry of this handler in the batch
    if (P.xmerge && (r < P.x_lo || r >= P.x_hi)) return; // (multi-GPU owner merge: this rank's regions)
    __shared__ MergeRuns U;
    __shared__ MergeState S;
    TST_DECL
    const uint32_t ng8 = (P.cb_grid + 7) / 8, ng = 8 * ng8;
    const uint64_t lcap = (uint64_t)P.cb_fan * P.mq_cap; // a combine workgroup's list capacity
    const uint32_t rsl = P.tcap_log2 - P.reg_log2;
    const uint32_t rs = 1u << rsl;
    const uint32_t tbg = hd ? PV_SLOTS + P.dslot_of[0] : P.slot_of[0];
    const uint64_t rbg = ((uint64_t)tbg << P.tcap_log2) + ((uint64_t)r << rsl);
    const bool pf = rs == PV_RS;
    if (pf) {
        // the keys of the region this run key almost always holds (the handler's first period
        // slot), LDS-DMA'd in flight with the run words: 32 1-KiB pieces, four per wave
        static_assert(PV_RS * 8 == 32 * 1024 && PV_MG_THREADS == 512, "four pieces per wave");
        const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t pc = wv * 4 + q;
            dma16(P.tkeys + rbg + pc * 128 + ln * 2, lds_addr(&S.key[pc * 128]));
        }
    }
    uint32_t n;
    {
        // runs 2t and 2t + 1 of the column (one 16-B load); a combine workgroup without entries of
        // this handler wrote no words
        uint32_t c0 = 0, c1 = 0, tb = 0;
        if (threadIdx.x == 0) U.tabs = 0;
        const uint32_t i0 = 2 * threadIdx.x;
        if (i0 < ng) {
            const ulonglong2 v = *reinterpret_cast<const PV_G ulonglong2 *>(P.cb_run + (uint64_t)rk * ng + i0);
            const uint32_t w0 = (i0 % ng8) * 8 + i0 / ng8, w1 = ((i0 + 1) % ng8) * 8 + (i0 + 1) / ng8;
            const bool h0 = w0 < P.cb_grid && ((P.cb_hm[w0] >> hd) & 1);
            const bool h1 = w1 < P.cb_grid && ((P.cb_hm[w1] >> hd) & 1);
            U.start[i0] = (uint32_t)v.x & 0xffffffu;
            U.start[i0 + 1] = (uint32_t)v.y & 0xffffffu;
            U.list[i0] = (uint16_t)w0;
            U.list[i0 + 1] = (uint16_t)w1;
            c0 = h0 ? (uint32_t)(v.x >> 24) & 0xffffffu : 0u;
            c1 = h1 ? (uint32_t)(v.y >> 24) & 0xffffffu : 0u;
            tb = (h0 ? (uint32_t)(v.x >> 48) : 0u) | (h1 ? (uint32_t)(v.y >> 48) : 0u);
        }
        uint32_t total;
        PV_VMCNT(0); // the region DMA too, before the barriers below
        const uint32_t pre = block_excl_scan(c0 + c1, U.wsum, total);
        if (i0 < ng) { U.pref[i0] = pre; U.pref[i0 + 1] = pre + c0; }
        if (threadIdx.x == 0) U.pref[ng] = total;
        if (tb) atomicOr(&U.tabs, tb);
        __syncthreads();
        n = total;
    }
    TST(0)
    if (n == 0) return;
    // entry j of the region: its run by binary search over the run prefixes
    uint32_t top = 1;
    while (top * 2 < ng) top *= 2;
    const PV_G ulonglong2 *cb = reinterpret_cast<const PV_G ulonglong2 *>(P.cb);
    auto ld = [&](uint64_t j) -> ulonglong2 {
        uint32_t lo = 0;
        for (uint32_t st = top; st; st >>= 1) {
            const uint32_t m = lo + st;
            if (m < ng && U.pref[m] <= (uint32_t)j) lo = m;
        }
        return cb[(uint64_t)U.list[lo] * lcap + U.start[lo] + ((uint32_t)j - U.pref[lo])];
    };
    // (every run key takes the LDS path, however few its entries: a direct global insert here
    // would bind the kernel to the device-call convention)
    static_assert(PV_TABLES <= 32, "table mask");
    constexpr uint32_t PF = PV_RS / PV_MG_THREADS; // region entries per thread
    // IPv4 cardinality minima in the insert pass (batches of at most 2^24 records): a v1 IPv4
    // entry's LDS key word carries PV_MV4 and direction 1's smallest record index in bits
    // 32..55 (the key's own bits there are zero; the word's atomicMin lowers that field alone,
    // the other bits being the entry's constants), its weight word the count in the low half and
    // direction 0's smallest index in the high half. Longer batches take a second pass.
    const bool narrow = P.n <= (1ull << 24) && !P.xmerge;
    const bool xm = P.xmerge != 0; // multi-GPU owner merge: 64-bit weights, no names, no CPC
    uint32_t tabs = U.tabs << (hd * PV_SLOTS); // the tables among this run key's entries
    const bool one = !(tabs & (tabs - 1));
    bool fresh = true; // S.key still holds the DMA'd region
    while (tabs) {
        const uint32_t tb = __builtin_ctz(tabs);
        const uint32_t s = tb % PV_SLOTS; // the handler slot (Net for tb < PV_SLOTS, else DNS)
        tabs &= tabs - 1;
        const uint64_t rbase = ((uint64_t)tb << P.tcap_log2) + ((uint64_t)r << rsl);
        if (!(pf && tb == tbg && fresh)) batched<4>(rs, [&](uint64_t i) { return P.tkeys[rbase + i]; }, [&](uint64_t i, uint64_t k) { S.key[i] = k; });
        // the LDS forms of the loaded keys; weights start at PV_DL0 (direction 0's minimum unset)
        for (uint32_t i = threadIdx.x; i < rs; i += blockDim.x) {
            const uint64_t k = S.key[i];
            if (narrow && mv4_key(k)) S.key[i] = k | PV_MV4 | PV_MN1;
            S.dl[i] = PV_DL0;
        }
        if (threadIdx.x == 0) { S.nnew = 0; S.ncr = 0; S.ip4c = 0; }
        lds_barrier();
        TST(1)
        auto ins = [&](ulonglong2 e) __attribute__((always_inline)) {
            const uint64_t e0 = e.x;
            if (!one && entry_table(e0) != tb) return;
            const uint32_t w32 = (uint32_t)e.y, rep = (uint32_t)(e.y >> 32);
            const uint64_t w = xm ? e.y : (w32 & PV_W_IP4) ? (uint64_t)(w32 & PV_W_CNT) : (uint64_t)w32;
            const uint64_t key = e0 & ((1ull << 60) - 1);
            const bool v4 = narrow && mv4_key(key);
            const bool card = !xm && (w32 & PV_W_IP4) && ((w32 >> 29) & 1);
            if (card && !v4) S.ip4c = 1; // (a long batch: the second pass)
            const uint64_t pk = v4 ? key | PV_MV4 : key;
            uint32_t pos = (uint32_t)tkey_hash(key) & (rs - 1);
            for (int probe = 0; probe < PV_PROBES; probe++) {
                uint64_t cur = S.key[pos];
                bool created = false;
                if (cur == 0) {
                    const uint64_t nw = pk | (v4 ? PV_MN1 : 0ull) | PV_CREATED;
                    const uint64_t prev = atomicCAS((unsigned long long *)&S.key[pos], 0ull, (unsigned long long)nw);
                    created = prev == 0;
                    cur = created ? nw : prev;
                }
                if (mv4_norm(cur) == pk) {
                    if (v4) {
                        atomicAdd(reinterpret_cast<uint32_t *>(&S.dl[pos]), (uint32_t)w);
                        if (card) {
                            if ((w32 >> 30) & 1) atomicMin((unsigned long long *)&S.key[pos], (unsigned long long)((cur & ~PV_MN1) | ((uint64_t)rep << 32)));
                            else atomicMin(reinterpret_cast<uint32_t *>(&S.dl[pos]) + 1, rep);
                        }
                    } else {
                        atomicAdd((unsigned long long *)&S.dl[pos], (unsigned long long)w);
                    }
                    if (created) {
                        atomicAdd(&S.ncr, 1u);
                        if (PV_KEY_METRIC(key) != TM_IPV4 && !xm) {
                            // (past the list's capacity the names phase scans the region instead)
                            const uint32_t k = atomicAdd(&S.nnew, 1u);
                            if (k < PV_MG_NN) { S.nidx[k] = (uint16_t)pos; S.nrep[k] = rep; }
                            else P.taux[rbase + pos] = rep;
                        }
                    }
                    return;
                }
                pos = (pos + 1) & (rs - 1);
            }
            if (card && v4) cpc_min(P, s, ((w32 >> 30) & 1) ? CPC_DST : CPC_SRC, ip4_coupon((uint32_t)key), (int64_t)(P.gbase + rep));
            table_overflow(P, s, key, w, rep, !xm);
        };
        batched<PV_MG_U2>(n, ld, [&](uint64_t, ulonglong2 e) { ins(e); });
        __syncthreads();
        TST(2)
        // the created named entries' slots in the new-name list (pv_topn_names decodes them)
        const uint32_t nnew = S.nnew;
        auto new_name = [&](uint32_t g, uint32_t i, uint32_t rep) {
            if (g < P.nn_cap) P.nn[g] = PvNewName{tb, rep, rbase + i};
            else {
                // past the list: the record waits in the aux word for pv_topn_name_fix
                P.taux[rbase + i] = PV_AUX_PENDING | rep;
                atomicOr(P.flags, (uint32_t)PVF_NAMES_PENDING);
            }
        };
        if (nnew && nnew <= PV_MG_NN) {
            if (threadIdx.x == 0) S.nbase = atomicAdd(P.nn_cnt, nnew);
            lds_barrier();
            for (uint32_t k = threadIdx.x; k < nnew; k += blockDim.x) new_name(S.nbase + k, S.nidx[k], S.nrep[k]);
        } else if (nnew) {
            // more than the list holds: every thread lists its share of the region's created entries
            uint32_t mine = 0;
            for (uint32_t i = threadIdx.x; i < rs; i += blockDim.x) {
                const uint64_t k = S.key[i];
                mine += (k & PV_CREATED) && PV_KEY_METRIC(k & ~PV_CREATED) != TM_IPV4;
            }
            uint32_t tot;
            uint32_t g = block_excl_scan(mine, U.wsum, tot);
            if (threadIdx.x == 0) S.nbase = atomicAdd(P.nn_cnt, tot);
            // the listed entries' source records to their aux words too (visible to the
            // workgroup after the barrier; read past L1)
            for (uint32_t k = threadIdx.x; k < PV_MG_NN; k += blockDim.x) P.taux[rbase + S.nidx[k]] = S.nrep[k];
            __syncthreads();
            g += S.nbase;
            for (uint32_t i = threadIdx.x; i < rs; i += blockDim.x) {
                const uint64_t k = S.key[i];
                if ((k & PV_CREATED) && PV_KEY_METRIC(k & ~PV_CREATED) != TM_IPV4)
                    new_name(g++, i, __hip_atomic_load(&P.taux[rbase + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            }
        }
        TST(3)
        // write-back of the entries this batch changed: a created entry's key and weight; an
        // existing one's count word read (all of a thread's reads in flight together) and stored
        // with the weight added. Then the IPv4 cardinality minima of the changed v1 entries.
        constexpr uint32_t WB = PF < 4 ? PF : 4;
        for (uint32_t q0 = 0; q0 < PF; q0 += WB) {
            uint64_t kk[WB], dd[WB], cc[WB];
#pragma unroll
            for (uint32_t q = 0; q < WB; q++) {
                const uint32_t i = threadIdx.x + (q0 + q) * PV_MG_THREADS;
                kk[q] = i < rs ? S.key[i] : 0;
                const uint64_t d = i < rs ? S.dl[i] : PV_DL0;
                dd[q] = (kk[q] & PV_MV4) ? (d & 0xffffffffull) : d - PV_DL0;
            }
#pragma unroll
            for (uint32_t q = 0; q < WB; q++) {
                const uint32_t i = threadIdx.x + (q0 + q) * PV_MG_THREADS;
                cc[q] = (dd[q] && !(kk[q] & PV_CREATED)) ? P.tcnt[rbase + i] : 0;
            }
#pragma unroll
            for (uint32_t q = 0; q < WB; q++) {
                const uint32_t i = threadIdx.x + (q0 + q) * PV_MG_THREADS;
                if (kk[q] & PV_CREATED) {
                    st_nt<PV_NT_MERGE, uint64_t>(P.tkeys + rbase + i, mv4_norm(kk[q]) & ~PV_MV4);
                    if (xm && PV_KEY_METRIC(kk[q] & ~PV_CREATED) != TM_IPV4) P.taux[rbase + i] = 0; // name unknown here
                }
                if (dd[q]) st_nt<PV_NT_MERGE, uint64_t>(P.tcnt + rbase + i, cc[q] + dd[q]);
                if ((kk[q] & PV_MV4) && dd[q]) {
                    const uint32_t m0 = (uint32_t)(S.dl[i] >> 32), m1 = (uint32_t)(kk[q] >> 32) & 0xffffffu;
                    if (m0 != 0xffffffffu || m1 != 0xffffffu) {
                        const uint32_t cp = ip4_coupon((uint32_t)kk[q]);
                        if (m0 != 0xffffffffu) cpc_min(P, s, CPC_SRC, cp, (int64_t)(P.gbase + m0));
                        if (m1 != 0xffffffu) cpc_min(P, s, CPC_DST, cp, (int64_t)(P.gbase + m1));
                    }
                }
            }
        }
        if (threadIdx.x == 0 && S.ncr) atomicAdd(&P.tab_live[tb], S.ncr);
        // batches longer than 2^24 records: the minima by a second pass over the run's entries,
        // in dl (now free: the low word direction 0, the high word direction 1)
        if (S.ip4c) {
            lds_barrier(); // the write-back's reads of dl
            for (uint32_t i = threadIdx.x; i < rs; i += blockDim.x) S.dl[i] = ~0ull;
            lds_barrier();
            batched<PV_MG_U2>(n, ld, [&](uint64_t, ulonglong2 e) {
                const uint32_t w32 = (uint32_t)e.y, rep = (uint32_t)(e.y >> 32), d = (w32 >> 30) & 1;
                if (!(w32 & PV_W_IP4) || !((w32 >> 29) & 1) || (!one && entry_table(e.x) != tb)) return;
                const uint64_t key = e.x & ((1ull << 60) - 1);
                uint32_t pos = (uint32_t)tkey_hash(key) & (rs - 1);
                for (int probe = 0; probe < PV_PROBES; probe++) {
                    const uint64_t cur = S.key[pos] & ~PV_CREATED;
                    if (cur == key) {
                        atomicMin(reinterpret_cast<uint32_t *>(&S.dl[pos]) + d, rep);
                        return;
                    }
                    if (cur == 0) break;
                    pos = (pos + 1) & (rs - 1);
                }
                // (an update the full region could not take, gone to the overflow list)
                cpc_min(P, s, d ? CPC_DST : CPC_SRC, ip4_coupon((uint32_t)key), (int64_t)(P.gbase + rep));
            });
            lds_barrier();
            for (uint32_t i = threadIdx.x; i < rs; i += blockDim.x) {
                const uint64_t m = S.dl[i];
                if (m == ~0ull) continue;
                const uint32_t cp = ip4_coupon((uint32_t)S.key[i]);
                if ((uint32_t)m != 0xffffffffu) cpc_min(P, s, CPC_SRC, cp, (int64_t)(P.gbase + (uint32_t)m));
                if ((uint32_t)(m >> 32) != 0xffffffffu) cpc_min(P, s, CPC_DST, cp, (int64_t)(P.gbase + (uint32_t)(m >> 32)));
            }
        }
        if (tabs) lds_barrier(); // another table's region reuses S
        TST(4)
        fresh = false;
    }
    TST_FLUSH(65536)
}

// ------------------------------------------------------------------ multi-GPU top-N exchange
// The regions of every table are partitioned over the ranks in contiguous blocks (the owner of
// region r: r * W / nreg). A rank sends the live entries of the regions it does not own to
// their owners, ordered (owner, handler, region, slot), with the counts of each (handler,
// region, slot) as a header; each owner merges what it receives into its own regions with
// pv_topn_merge (xmerge: 64-bit weights, no names), the analog of the frequent-items merge of
// AbstractMetricsBucket::merge (src/AbstractMetricsManager.h:177-195, src/Metrics.h:534-538)
// over shards of one stream.
__device__ __forceinline__ uint32_t x_owner(uint32_t r, uint32_t reg_log2, uint32_t W) { return (uint32_t)(((uint64_t)r * W) >> reg_log2); }
__device__ __forceinline__ uint32_t x_lo(uint32_t d, uint32_t reg_log2, uint32_t W) { return (uint32_t)((((uint64_t)d << reg_log2) + W - 1) / W); }
#define PV_XC(hd, r, slot, reg_log2) ((((uint32_t)(hd) << (reg_log2)) + (r)) * PV_SLOTS + (slot))

// live entries per (table, region) of the regions other ranks own
extern "C" __global__ void __launch_bounds__(256) pv_topn_xcount(const PvParams *__restrict__ Pp, PvXTabs T, uint32_t *__restrict__ cnt)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ uint32_t wsum[16];
    const uint32_t r = blockIdx.x & ((1u << P.reg_log2) - 1), tb = T.tb[blockIdx.x >> P.reg_log2];
    const uint32_t rs = 1u << (P.tcap_log2 - P.reg_log2);
    uint32_t c = 0;
    if (x_owner(r, P.reg_log2, T.W) != T.me) {
        const PV_G uint64_t *k = P.tkeys + ((uint64_t)tb << P.tcap_log2) + ((uint64_t)r << (P.tcap_log2 - P.reg_log2));
        for (uint32_t i = threadIdx.x; i < rs; i += blockDim.x) c += k[i] != 0;
    }
    uint32_t tot;
    block_excl_scan(c, wsum, tot);
    if (threadIdx.x == 0) cnt[PV_XC(tb / PV_SLOTS, r, tb % PV_SLOTS, P.reg_log2)] = tot;
}

// One workgroup: the counts in (owner, handler, region, slot) order: each cell's offset in the
// send list and the header stream (the counts in that order; an owner's slice is its header)
extern "C" __global__ void __launch_bounds__(1024) pv_topn_xscan(uint32_t reg_log2, uint32_t W, const uint32_t *__restrict__ cnt,
                                                                 uint32_t *__restrict__ off, uint32_t *__restrict__ hdr)
{
    __shared__ uint32_t wsum[16];
    const uint32_t E = (2u << reg_log2) * PV_SLOTS, per = (E + blockDim.x - 1) / blockDim.x;
    const uint32_t p0 = min(threadIdx.x * per, E), p1 = min(p0 + per, E);
    auto cell = [&](uint32_t p) {
        const uint32_t d = x_owner(p / (2 * PV_SLOTS), reg_log2, W);
        const uint32_t lo = x_lo(d, reg_log2, W), len = x_lo(d + 1, reg_log2, W) - lo;
        const uint32_t rem = p - 2 * PV_SLOTS * lo, hd = rem / (PV_SLOTS * len);
        return PV_XC(hd, lo + (rem % (PV_SLOTS * len)) / PV_SLOTS, rem % PV_SLOTS, reg_log2);
    };
    uint32_t s = 0;
    for (uint32_t p = p0; p < p1; p++) s += cnt[cell(p)];
    uint32_t tot;
    uint32_t at = block_excl_scan(s, wsum, tot);
    for (uint32_t p = p0; p < p1; p++) {
        const uint32_t i = cell(p), c = cnt[i];
        off[i] = at;
        hdr[p] = c;
        at += c;
    }
}

// the live entries of the regions other ranks own into the send list: {key | slot << 60, count}
extern "C" __global__ void __launch_bounds__(256) pv_topn_xwrite(const PvParams *__restrict__ Pp, PvXTabs T, const uint32_t *__restrict__ off,
                                                                 ulonglong2 *__restrict__ out)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ uint32_t wsum[16];
    const uint32_t r = blockIdx.x & ((1u << P.reg_log2) - 1), tb = T.tb[blockIdx.x >> P.reg_log2];
    if (x_owner(r, P.reg_log2, T.W) == T.me) return;
    const uint32_t rsl = P.tcap_log2 - P.reg_log2, rs = 1u << rsl;
    const uint64_t rb = ((uint64_t)tb << P.tcap_log2) + ((uint64_t)r << rsl);
    const uint32_t per = rs / blockDim.x; // contiguous positions per thread
    const uint32_t i0 = threadIdx.x * per;
    uint32_t c = 0;
    for (uint32_t i = i0; i < i0 + per; i++) c += P.tkeys[rb + i] != 0;
    uint32_t tot;
    uint32_t at = off[PV_XC(tb / PV_SLOTS, r, tb % PV_SLOTS, P.reg_log2)] + block_excl_scan(c, wsum, tot);
    for (uint32_t i = i0; i < i0 + per; i++) {
        const uint64_t k = P.tkeys[rb + i];
        if (k) out[at++] = make_ulonglong2(k | ((uint64_t)(tb % PV_SLOTS) << 60), P.tcnt[rb + i]);
    }
}

// The run table of the received lists for pv_topn_merge: workgroup q scans source q's header
// (this rank's regions, (handler, region, slot) order) into one run word per (handler, region):
// start in q's list, count, the slots present. Source me sends nothing: zero words.
extern "C" __global__ void __launch_bounds__(1024) pv_topn_xruns(uint32_t reg_log2, uint32_t W, uint32_t me, const uint32_t *__restrict__ hdr,
                                                                 uint32_t hdr_stride, uint64_t *__restrict__ cb_run)
{
    __shared__ uint32_t wsum[16];
    const uint32_t q = blockIdx.x, lo = x_lo(me, reg_log2, W), len = x_lo(me + 1, reg_log2, W) - lo;
    const uint32_t ng8 = (W + 7) / 8, ng = 8 * ng8, col = (q % 8) * ng8 + q / 8;
    const uint32_t E = 2 * len; // (handler, region) runs
    const uint32_t per = (E + blockDim.x - 1) / blockDim.x, e0 = min(threadIdx.x * per, E), e1 = min(e0 + per, E);
    const uint32_t *h = hdr + (uint64_t)q * hdr_stride;
    uint32_t s = 0;
    if (q != me)
        for (uint32_t e = e0; e < e1; e++)
            for (uint32_t k = 0; k < PV_SLOTS; k++) s += h[e * PV_SLOTS + k];
    uint32_t tot;
    uint32_t at = block_excl_scan(s, wsum, tot);
    for (uint32_t e = e0; e < e1; e++) {
        uint32_t c = 0, tabs = 0;
        if (q != me)
            for (uint32_t k = 0; k < PV_SLOTS; k++) {
                const uint32_t v = h[e * PV_SLOTS + k];
                c += v;
                if (v) tabs |= 1u << k;
            }
        const uint32_t hd = e / len, rk = (hd << reg_log2) | (lo + e % len);
        cb_run[(uint64_t)rk * ng + col] = pv_run_word(at, c, tabs);
        at += c;
    }
}

// Finalize support: the aux word (name record) of each listed (table, key) in this rank's
// tables, 0 when absent or unnamed
// Name records of table entries for the multi-GPU read view (pv_topn_x_candidates / _names), in
// two launches: each record's length (its 2-byte header; ~0 for none), then, at the host's prefix
// offsets, its bytes, so the host reads every name with two copies instead of two per name.
extern "C" __global__ void pv_xname_len(const uint8_t *__restrict__ arena, uint64_t arena_cap, const uint32_t *__restrict__ tb,
                                        const uint32_t *__restrict__ aux, uint32_t n, uint32_t *__restrict__ len)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    if (!aux[j]) { len[j] = 0xffffffffu; return; }
    const uint8_t *b = arena + (uint64_t)tb[j] * arena_cap + (aux[j] - 1);
    len[j] = (uint32_t)b[0] | ((uint32_t)b[1] << 8);
}
extern "C" __global__ void pv_xname_copy(const uint8_t *__restrict__ arena, uint64_t arena_cap, const uint32_t *__restrict__ tb,
                                         const uint32_t *__restrict__ aux, const uint32_t *__restrict__ len,
                                         const uint64_t *__restrict__ off, uint32_t n, uint8_t *__restrict__ out)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n || len[j] == 0xffffffffu) return;
    const uint8_t *b = arena + (uint64_t)tb[j] * arena_cap + (aux[j] - 1) + 2;
    for (uint32_t k = 0; k < len[j]; k++) out[off[j] + k] = b[k];
}

extern "C" __global__ void pv_topn_xlookup(const PvParams *__restrict__ Pp, const uint64_t *__restrict__ keys, const uint32_t *__restrict__ tbs,
                                           uint32_t n, uint32_t *__restrict__ aux)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t key = keys[j];
    const uint32_t tb = tbs[j], rsl = P.tcap_log2 - P.reg_log2;
    const uint64_t h = tkey_hash(key);
    const uint64_t rb = ((uint64_t)tb << P.tcap_log2) + ((uint64_t)tregion(P, h) << rsl);
    uint32_t pos = (uint32_t)h & ((1u << rsl) - 1), a = 0;
    for (int probe = 0; probe < PV_PROBES; probe++) {
        const uint64_t k = P.tkeys[rb + pos];
        if (k == key) { a = P.taux[rb + pos]; break; }
        if (k == 0) break;
        pos = (pos + 1) & ((1u << rsl) - 1);
    }
    aux[j] = a;
}

// The updates full regions could not take in this batch, once the host has purged their tables:
// inserted again (those that still find no room go back to the overflow list for another round)
extern "C" __global__ void pv_topn_retry(const PvParams *__restrict__ Pp, const PvOvf *__restrict__ src, uint32_t n)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const PvOvf e = src[j];
    if (e.pad) global_add(P, e.slot, e.key, (uint64_t)e.w | ((uint64_t)e.rep << 32), 0u); // an owner merge's entry
    else global_add(P, e.slot, e.key, e.w, e.rep);
}

// Bounded top-N tables: the frequent-items sketch's purge (Apache DataSketches
// frequent_items_sketch / reverse_purge_hash_map, as TopN holds it, src/Metrics.h:488-538;
// the library is not vendored in the reference). Once a table holds more than half its
// capacity between batches, every region of it takes its median count theta, subtracts it
// from every entry and drops those left at zero or below, rehashing the survivors; theta is
// added to the region's offset. The host reports count + offset: exact for a key never
// dropped, and for any key an upper bound on its true count with count as the lower bound,
// as the sketch's get_estimate / get_lower_bound are. Each purge removes at least
// theta x (half the region) of stored weight, so the offset stays below 4 x (the region's
// updates) / (region size).
extern "C" __global__ void __launch_bounds__(1024) pv_topn_purge(const PvParams *__restrict__ Pp, uint32_t tb,
                                                                 uint32_t *theta_out)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint32_t r = blockIdx.x;
    const uint32_t rsl = P.tcap_log2 - P.reg_log2;
    const uint32_t rs = 1u << rsl;
    const uint64_t rbase = ((uint64_t)tb << P.tcap_log2) + ((uint64_t)r << rsl);
    __shared__ uint64_t K[PV_RS];
    __shared__ uint64_t C[PV_RS];
    __shared__ uint32_t A[PV_RS];
    __shared__ uint32_t hist[1024];
    __shared__ uint32_t live, theta, removed;
    for (uint32_t b = threadIdx.x; b < 1024; b += blockDim.x) hist[b] = 0;
    if (threadIdx.x == 0) { live = 0; removed = 0; theta = 0; }
    __syncthreads();
    // this thread's entries (rs / blockDim.x of them) stay in registers across the rebuild
    constexpr uint32_t PER = PV_RS / 1024;
    uint64_t k[PER], c[PER];
    uint32_t a[PER];
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
        const uint32_t i = threadIdx.x + q * blockDim.x;
        k[q] = i < rs ? P.tkeys[rbase + i] : 0;
        c[q] = i < rs ? P.tcnt[rbase + i] : 0;
        a[q] = i < rs ? P.taux[rbase + i] : 0;
        if (k[q]) {
            atomicAdd(&live, 1u);
            atomicAdd(&hist[c[q] < 1023 ? (uint32_t)c[q] : 1023u], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && live) {
        // smallest theta with at least half the entries at count <= theta
        uint32_t acc = 0, t = 0;
        while (t < 1023 && acc + hist[t] < (live + 1) / 2) acc += hist[t++];
        theta = t;
    }
    __syncthreads();
    const uint32_t th = theta;
    if (!live) { if (threadIdx.x == 0) theta_out[r] = 0; return; }
    for (uint32_t i = threadIdx.x; i < rs; i += blockDim.x) { K[i] = 0; C[i] = 0; A[i] = 0; }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
        if (!k[q]) continue;
        if (c[q] <= th) { atomicAdd(&removed, 1u); continue; }
        uint32_t pos = (uint32_t)tkey_hash(k[q]) & (rs - 1);
        for (uint32_t probe = 0; probe < rs; probe++) {
            if (atomicCAS((unsigned long long *)&K[pos], 0ull, (unsigned long long)k[q]) == 0) {
                C[pos] = c[q] - th;
                A[pos] = a[q];
                break;
            }
            pos = (pos + 1) & (rs - 1);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < rs; i += blockDim.x) {
        P.tkeys[rbase + i] = K[i];
        P.tcnt[rbase + i] = C[i];
        P.taux[rbase + i] = A[i];
    }
    if (threadIdx.x == 0) {
        theta_out[r] = th;
        atomicSub(&P.tab_live[tb], removed);
    }
}

// Name-arena compaction of one table after a purge: every live entry's name record moves,
// within its own partition, to a scratch arena packed from the partition start, and its aux
// is re-pointed; the host copies the scratch over the table's arena and takes the scratch
// tops as the partitions' new tops. A partition never grows, so nothing can overflow.
extern "C" __global__ void pv_topn_compact(const PvParams *__restrict__ Pp, uint32_t tb, uint8_t *tmp,
                                           unsigned long long *tmp_top)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint64_t tcap = 1ull << P.tcap_log2;
    const uint64_t pcap = P.arena_cap / PV_ARENA_PARTS;
    const uint8_t *arena = P.arena + (uint64_t)tb * P.arena_cap;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < tcap; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t at = ((uint64_t)tb << P.tcap_log2) + i;
        const uint64_t key = P.tkeys[at];
        if (!key || PV_KEY_METRIC(key) == TM_IPV4) continue; // IPv4 entries have no name (stale aux)
        const uint32_t aux = P.taux[at];
        if (!aux) continue;
        const uint64_t part = (aux - 1) / pcap;
        const uint8_t *src = arena + (aux - 1);
        const uint32_t len = src[0] | (src[1] << 8);
        const uint32_t bytes = (len + 2 + 3) & ~3u;
        const uint64_t pos = part * pcap + atomicAdd(&tmp_top[part], (unsigned long long)bytes);
        for (uint32_t b = 0; b < len + 2; b++) tmp[pos + b] = src[b];
        P.taux[at] = (uint32_t)pos + 1;
    }
}

// Name records of the entries pv_topn_merge created, one lane per entry: the record
// is parsed again, the first PV_WIN bytes of its DNS message are staged into the lane's
// LDS window with independent 16-B loads, and the name is decoded from there (bytes past
// the window come from HBM). Each wave reserves its lanes' arena bytes with one atomic.
// SFX: suffix sizes in play (only_qname_suffix / public_suffix_list): qname2/3 may need the
// name walked again (agg_domain_r's out-of-line dots_up_to); without them the kernel makes
// no device call
template <bool SFX>
__device__ __forceinline__ void topn_names(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    // each lane stages PV_NWIN bytes from its record's 16-B aligned start: the frame
    // headers and, for a plain DNS message, the whole first question, so the record is
    // parsed and its name decoded from LDS after one round of loads
    __shared__ uint32_t stage[4][PV_NWIN / 4 * 64];
    // the wave's name records, packed as they will lie in the arena, then copied out with
    // coalesced dword stores (byte stores of each lane's name were one write request per byte)
    __shared__ uint32_t obuf[4][PV_NOUT / 4];
    const uint32_t n = min(*P.nn_cnt, P.nn_cap);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t *L = stage[threadIdx.x >> 6];
    uint8_t *O = reinterpret_cast<uint8_t *>(obuf[threadIdx.x >> 6]);
    const uint64_t pcap = P.arena_cap / PV_ARENA_PARTS;
    const GAcc G{P.recs};
    // Software pipeline over the lane's entries i, i + step, ...: the window of the next entry
    // and the table key / record offset of the one after are loaded while this entry's arena
    // reservation (a returning atomic the wave waits for anyway) is in flight, and the new-name
    // record two ahead right after it, so each iteration waits for memory once.
    const uint32_t step = gridDim.x * blockDim.x;
    auto ld_e = [&](uint32_t j) { return j < n ? P.nn[j] : PvNewName{0, 0, 0}; };
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    PvNewName e = ld_e(i);
    uint64_t tkey = i < n ? P.tkeys[e.pos] : 0, roff = i < n ? P.offs[e.rep] : 0;
    uint4 pf[PV_NWIN / 16];
    auto ld_win = [&](uint64_t ro, bool a) {
        const uint4 *src = reinterpret_cast<const uint4 *>(P.recs + (ro & ~15ull));
#pragma unroll
        for (int j = 0; j < PV_NWIN / 16; j++) pf[j] = a ? src[j] : make_uint4(0, 0, 0, 0);
    };
    ld_win(roff, i < n);
    PvNewName e_n = ld_e(i + step);
    uint64_t tkey_n = i + step < n ? P.tkeys[e_n.pos] : 0, roff_n = i + step < n ? P.offs[e_n.rep] : 0;
    PvNewName e_nn = ld_e(i + 2 * step);
    for (uint32_t b = blockIdx.x * blockDim.x; b < n; b += step, i += step) {
        const bool act = i < n;
        const uint32_t metric = PV_KEY_METRIC(tkey);
        uint32_t size = 0, start = 0, nl = 0, mlen = 0;
        uint64_t m = 0, a6 = 0;
        Parsed o;
        const uint64_t wbase = roff & ~15ull;
#pragma unroll
        for (int j = 0; j < PV_NWIN / 16; j++) {
            L[(4 * j + 0) * 64 + lane] = pf[j].x;
            L[(4 * j + 1) * 64 + lane] = pf[j].y;
            L[(4 * j + 2) * 64 + lane] = pf[j].z;
            L[(4 * j + 3) * 64 + lane] = pf[j].w;
        }
        // the next entry's window: in flight through this entry's decode, which reads LDS alone
        // (LAccT); the reservation's wait below lands it
        const uint32_t i_n = i + step, i_nn = i + 2 * step;
        ld_win(roff_n, i_n < n);
        const TAcc R{P.recs, L, wbase, PV_NWIN - 4, 64u, lane};
        uint32_t hi = 0;
        const LAccT RL{L, wbase, 64u, lane, &hi};
        auto decode = [&](const auto &A) {
            parse_record(A, P, roff, o);
            m = o.l4off + 8;
            mlen = o.l4len - 8;
            if (metric == TM_IPV6) {
                a6 = ip6_name_addr(A, o, tkey);
                size = 18;
            } else {
                NameStats st;
                st.init();
                nl = name_len_l1(A, m, mlen, 12);
                if (nl > 0) name_stats(A, m, mlen, 12, st);
                const uint32_t nch = nl > 0 ? st.n : 0;
                start = 0;
                if (metric == TM_QNAME2 || metric == TM_QNAME3) {
                    int q2, q3;
                    uint64_t h2, h3;
                    if (nl == 0) { q2 = 0; q3 = -1; }
                    else if constexpr (SFX) agg_domain_r(A, m, mlen, st, q2, q3, h2, h3, name_sfx(P, e.rep, P.sfx_of));
                    else agg_domain(st, q2, q3, h2, h3, 0);
                    const int st0 = metric == TM_QNAME2 ? q2 : q3;
                    start = st0 < 0 ? nch : (uint32_t)st0;
                }
                size = nch - start + 2;
            }
        };
        if (act) decode(RL);
        // a record whose decode read past the window (rare: long names, IP options) is decoded
        // again with the HBM path, whose waits also land the prefetch
        const bool inwin = hi <= PV_NWIN;
        if (act && !inwin) decode(R);
        // wave prefix sum of the sizes; one arena reservation per wave when its lanes
        // share a slot (the common case), else one per lane
        uint32_t incl = size;
        for (int o2 = 1; o2 < 64; o2 <<= 1) {
            const uint32_t v = __shfl_up(incl, o2, 64);
            if (lane >= (uint32_t)o2) incl += v;
        }
        const uint32_t tot = __shfl(incl, 63, 64);
        const uint32_t tot4 = (tot + 3) & ~3u; // arena allocations are dword multiples
        const uint32_t part = (blockIdx.x * 4 + (threadIdx.x >> 6)) & (PV_ARENA_PARTS - 1);
        const uint32_t s0 = __shfl(e.slot, 0, 64);
        const bool uniform = __all(!act || e.slot == s0);
        const bool packed = uniform && tot4 <= PV_NOUT;
        // the key / record offset of the entry after next: landed by the reservation's wait
        const uint64_t tkey_nn = i_nn < n ? P.tkeys[e_nn.pos] : 0, roff_nn = i_nn < n ? P.offs[e_nn.rep] : 0;
        auto emit_to = [&](uint8_t *dst) {
            const uint32_t slen = size - 2;
            dst[0] = (uint8_t)(slen & 0xff);
            dst[1] = (uint8_t)(slen >> 8);
            if (metric == TM_IPV6) {
                for (int k = 0; k < 16; k++) dst[2 + k] = (uint8_t)G.u8(a6 + k);
            } else if (slen > 0 && nl > 0) {
                CopyEmit ce{dst + 2, start, 0, (metric == TM_SLOW_IN || metric == TM_SLOW_OUT) ? 1u : 0u};
                if (inwin) name_emit(RL, m, mlen, 12, ce);
                else name_emit(R, m, mlen, 12, ce);
            }
        };
        if (uniform) {
            unsigned long long wb = 0;
            if (lane == 0 && tot) wb = atomicAdd((unsigned long long *)&P.arena_top[s0 * PV_ARENA_PARTS + part], (unsigned long long)tot4);
            wb = __shfl(wb, 0, 64);
            const bool room = wb + tot4 <= pcap;
            if (!room) {
                if (act) {
                    atomicOr(P.flags, PVF_ARENA_FULL);
                    P.taux[e.pos] = 0;
                }
            } else {
                uint8_t *arena = P.arena + (uint64_t)s0 * P.arena_cap + part * pcap + wb;
                if (packed) {
                    if (act) emit_to(O + incl - size);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    for (uint32_t k = lane * 4; k < tot4; k += 256)
                        *reinterpret_cast<uint32_t *>(arena + k) = *reinterpret_cast<const uint32_t *>(O + k);
                    __builtin_amdgcn_wave_barrier();
                } else if (act) {
                    emit_to(arena + incl - size);
                }
                if (act) P.taux[e.pos] = (uint32_t)(part * pcap + wb + incl - size) + 1;
            }
        } else if (act) {
            const uint64_t pos = atomicAdd((unsigned long long *)&P.arena_top[e.slot * PV_ARENA_PARTS + part],
                                           (unsigned long long)((size + 3) & ~3u));
            if (pos + size > pcap) {
                atomicOr(P.flags, PVF_ARENA_FULL);
                P.taux[e.pos] = 0;
            } else {
                emit_to(P.arena + (uint64_t)e.slot * P.arena_cap + part * pcap + pos);
                P.taux[e.pos] = (uint32_t)(part * pcap + pos) + 1;
            }
        }
        e = e_n; tkey = tkey_n; roff = roff_n;
        e_n = e_nn; tkey_n = tkey_nn; roff_n = roff_nn;
        e_nn = ld_e(i + 3 * step);
    }
}
extern "C" __global__ void __launch_bounds__(256) pv_topn_names(const PvParams *__restrict__ Pp)
{
    topn_names<false>(Pp);
}
// Names of the entries the merge created past the new-name list (PVF_NAMES_PENDING, rare): every
// aux word of table tb holding PV_AUX_PENDING | record gets its name record (write_name)
extern "C" __global__ void __launch_bounds__(256) pv_topn_name_fix(const PvParams *__restrict__ Pp, uint32_t tb)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const uint64_t tcap = 1ull << P.tcap_log2, base = (uint64_t)tb * tcap;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < tcap; i += (uint64_t)gridDim.x * blockDim.x) {
        // (only named entries: an IPv4 entry's aux word is never written, and an empty slot's is
        // whatever its last occupant left)
        const uint64_t key = P.tkeys[base + i];
        if (!key || PV_KEY_METRIC(key) == TM_IPV4) continue;
        const uint32_t a = P.taux[base + i];
        if (!(a & PV_AUX_PENDING)) continue;
        const uint32_t rep = a & ~PV_AUX_PENDING;
        P.taux[base + i] = rep < P.n ? write_name(P, tb % PV_SLOTS, PV_KEY_METRIC(key), rep, nullptr, key) : 0u;
    }
}
extern "C" __global__ void __launch_bounds__(256) pv_topn_names_sfx(const PvParams *__restrict__ Pp)
{
    topn_names<true>(Pp);
}

// DNS events of a batch for the DNS manager's own window (AbstractMetricsManager::new_event,
// src/AbstractMetricsManager.h:318-333): bit i of dbits is set when record i reaches the DNS
// handler as an event: a UDP datagram on a DNS port with a non-zero metric port
// (DnsStreamHandler::process_udp_packet_cb, dns/v1/DnsStreamHandler.cpp:270-302) that the
// input predicates pass (only_rcode / only_qname). The host walks the bits for the DNS
// period shifts. One lane per record, one 64-bit store per 64-record tile.
extern "C" __global__ void __launch_bounds__(256) pv_dns_prescan(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const GAcc R{P.recs};
    const uint64_t ntiles = (P.n + 63) / 64;
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < ntiles; t += (uint64_t)gridDim.x * 4) {
        const uint64_t i = t * 64 + (threadIdx.x & 63);
        bool ev = false, istcp = false, hasseg = false;
        PvTcpSeg g;
        if (i < P.n) {
            Parsed o;
            parse_record(R, P, P.offs[i], o);
            istcp = o.l4 == 6;
            if (P.tcp_emit && istcp) hasseg = tcp_seg_of(R, o, i, g, P.tcp_emit);
            if (o.l4 == 17 && dns_port(R.u32(o.l4off))) {
                ev = true;
                if (P.f_flags & (PVDF_ONLY_RCODE | PVDF_ONLY_QNAME)) {
                    const uint64_t m = o.l4off + 8;
                    const uint64_t cap_end = o.frame + o.caplen;
                    const uint32_t mcap = cap_end > m ? (uint32_t)min<uint64_t>(cap_end - m, 65535) : 0u;
                    uint32_t w0, w1, w2;
                    dns_header(R, m, mcap, w0, w1, w2);
                    ev = dns_predicates(P, R, m, o.l4len - 8, w0, w1, w2);
                }
            }
        }
        const uint64_t b = __ballot(ev);
        if ((threadIdx.x & 63) == 0) P.dbits[t] = b;
        if (P.fbits) {
            // deep sampling with DNS filters: which of these events _filtering rejects
            bool f = false;
            if (ev) {
                Parsed o;
                parse_record(R, P, P.offs[i], o);
                const uint64_t m = o.l4off + 8;
                const uint64_t cap_end = o.frame + o.caplen;
                const uint32_t mcap = cap_end > m ? (uint32_t)min<uint64_t>(cap_end - m, 65535) : 0u;
                f = dns_filtered(P, R, m, o.l4len - 8, mcap, false, o.dir);
            }
            const uint64_t fb = __ballot(f);
            if ((threadIdx.x & 63) == 0) P.fbits[t] = fb;
        }
        if (P.tcp_emit) {
            // DNS over TCP for a batch the TCP stage runs ahead of the Net pass (pv_tcp.hip)
            const uint64_t tm = __ballot(istcp);
            if ((threadIdx.x & 63) == 0) P.tmask[t] = tm;
            if (tm) tcp_seg_store(P.tseg, P.tseg_cnt, P.tseg_cap, hasseg, g, threadIdx.x & 63);
        }
    }
}

// ------------------------------------------------------------------ the TCP DNS pass
// The DNS messages pv_tcp_flow cut from reassembled streams, through the same per-message
// work as UDP datagrams (DnsStreamHandler::tcp_message_ready_cb -> _filtering ->
// process_dns_layer, dns/v1/DnsStreamHandler.cpp:375-436). P is the span's parameter block
// with recs / offs replaced by the message records (linktype 101) and dq by the message
// list; the messages of this span (ord in [ord_lo, ord_hi)) take the DNS period of their
// position. Workgroup b handles messages [b * region, (b + 1) * region) and appends its
// events to the event region of workgroup grid_main + b, so pv_xact_compact packs them
// with the UDP events. Top-N updates go straight to the global tables (names decoded from
// the message records at once), the counters to HBM: TCP messages are few.
extern "C" __global__ void __launch_bounds__(256) pv_dns_tcp(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ uint32_t nev, nresp;
    if (threadIdx.x == 0) { nev = 0; nresp = 0; }
    __syncthreads();
    const uint64_t region = (uint64_t)P.wt_per_block * PV_WT;
    const uint64_t j0 = (uint64_t)blockIdx.x * region, j1 = min<uint64_t>(j0 + region, P.tcp_nmsg);
    const GAcc R{P.recs};
    DnsCtr c;
    c.zero();
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
        const PV_G uint4 *q = reinterpret_cast<const PV_G uint4 *>(P.dq) + 2 * j;
        const uint4 a = q[0], b = q[1];
        DnsMsg dm;
        dm.idx = a.x; dm.moff = a.y; dm.mlen = (uint16_t)(a.z & 0xffff); dm.mcap = (uint16_t)(a.z >> 16);
        dm.port = (uint16_t)(a.w & 0xffff); dm.flags = (uint8_t)((a.w >> 16) & 0xff);
        dm.fkey = b.x; dm.sec = b.y; dm.nsec = b.z; dm.pad = b.w;
        if (dm.pad < P.ord_lo || dm.pad >= P.ord_hi) continue;
        if (P.ndeep_dns && ((P.ndeep_dns[j >> 5] >> (j & 31)) & 1)) dm.flags |= 16; // deep sampling: not deep
        const uint32_t ordr = dm.pad - P.ord_base;
        uint32_t p = 0;
        for (uint32_t k = 0; k < P.n_dshift; k++) p += ordr >= P.dpos[k];
        dm.period = (uint8_t)p;
        if (p >= P.dskip_before) dm.flags |= 8;
        if (P.f_flags & (PVDF_ONLY_QSUFFIX | PVDF_PSL)) {
            const uint64_t m = dm.moff;
            P.sfx_of[dm.idx] = (uint8_t)dns_suffix_of(P, R, m, dm.mlen, be16(R, m + 4), be16(R, m + 6), be16(R, m + 8),
                                                      be16(R, m + 10));
        }
        dns_process<true>(P, (KeyCache<PV_NCACHE> *)nullptr, nullptr, &nev, &nresp, (uint64_t)(P.grid_main + blockIdx.x) * region, R,
                    dm, false, c);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        P.blk_events[P.grid_main + blockIdx.x] = nev;
        if (nresp) atomicAdd(P.n_events + 1, nresp);
    }
}

// Deep sampling with DNS filters over the messages of the TCP stage (P: the TCP pass's block,
// recs / offs the message records, dq the message list): bit j of fbits set when message j is
// filtered (dns_v1_filtered, or dns_v2_filtered in a DNS v2 context), so the host knows which
// events draw.
extern "C" __global__ void __launch_bounds__(256) pv_dns_tcp_filter(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    const GAcc R{P.recs};
    const uint64_t nt = ((uint64_t)P.tcp_nmsg + 63) / 64;
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < nt; t += (uint64_t)gridDim.x * 4) {
        const uint64_t j = t * 64 + (threadIdx.x & 63);
        bool f = false;
        if (j < P.tcp_nmsg) {
            const uint4 a = reinterpret_cast<const PV_G uint4 *>(P.dq)[2 * j];
            f = dns_filtered(P, R, a.y, a.z & 0xffff, a.z >> 16, true, (a.w >> 16) & 3);
        }
        const uint64_t fb = __ballot(f);
        if ((threadIdx.x & 63) == 0) P.fbits[t] = fb;
    }
}

// ------------------------------------------------------------------ dnstap events
// One lane per dnstap event, in the bucket of the span's period (spans hold no shift): the
// Net handler's NetworkMetricsBucket::process_dnstap (net/v1 ...cpp:549-620: direction by
// message type, l3 / l4 from the socket fields, the frame length as the payload size, the
// query address as "in" and the response address as "out", no SYN) and the DNS handler's
// DnsMetricsManager / DnsMetricsBucket::process_dnstap (dns/v1 ...cpp:839-909,1376-1412:
// dnstap_msg_type filter, counters by side without a message, else process_dns_layer on the
// message). Events are few next to packets: counters and tables are updated in HBM directly.
__device__ void dnstap_event(PV_CREF(PvParams) P, uint32_t j, uint32_t *nev, uint32_t *nresp);
extern "C" __global__ void __launch_bounds__(256) pv_dnstap_kernel(const PvParams *__restrict__ Pp)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ uint32_t nev, nresp;
    if (threadIdx.x == 0) { nev = 0; nresp = 0; }
    __syncthreads();
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < P.n) dnstap_event(P, j, &nev, &nresp);
    if (!P.want_events) return;
    // DNS v2: this block's transaction events (pv_xact_compact packs the regions)
    __syncthreads();
    if (threadIdx.x == 0) {
        P.blk_events[blockIdx.x] = nev;
        if (nresp) atomicAdd(P.n_events + 1, nresp);
    }
}
__device__ void dnstap_event(PV_CREF(PvParams) P, uint32_t j, uint32_t *nev, uint32_t *nresp)
{
    const PvDtEv e = reinterpret_cast<const PV_G PvDtEv *>(P.dq)[j];
    const GAcc R{P.recs};
    const uint64_t gidx = P.gbase + j;
    // ---- Net v1
    {
        const uint32_t s = P.slot_of[0];
        // deep sampling, not deep: process_net_layer(dir, l3, l4, size) only (net/v1 ...cpp:599-602)
        const bool deep = !(e.pad[0] & 1);
        sum_add(P, s, PV_OFF_NET + NC_EVENTS, 1);
        if (deep) sum_add(P, s, PV_OFF_NET + NC_SAMPLES, 1);
        if (P.net_groups & PV_NET_COUNTERS_BIT) {
            sum_add(P, s, PV_OFF_NET + NC_TOTAL, 1);
            sum_add(P, s, PV_OFF_NET + (e.dir == 0 ? NC_IN : (e.dir == 1 ? NC_OUT : NC_UNK)), 1);
            if (e.l3) sum_add(P, s, PV_OFF_NET + (e.l3 == 4 ? NC_V4 : NC_V6), 1);
            sum_add(P, s, PV_OFF_NET + (e.l4 == 17 ? NC_UDP : (e.l4 == 6 ? NC_TCP : NC_OTHER)), 1);
        }
        sum_add(P, s, PV_OFF_PAYLOAD + min(e.size, 65535u), 1);
        const bool card = P.net_groups & PV_NET_CARDINALITY_BIT, tops = P.net_groups & PV_NET_TOP_IPS_BIT;
        for (int side = 0; side < 2 && deep; side++) {
            const uint8_t *a = side ? e.raddr : e.qaddr;
            const uint32_t alen = side ? e.rlen : e.qlen;
            const uint32_t sketch = side ? CPC_DST : CPC_SRC;
            if (e.l3 == 4 && alen == 4) {
                const uint32_t ip = (uint32_t)a[0] | ((uint32_t)a[1] << 8) | ((uint32_t)a[2] << 16) | ((uint32_t)a[3] << 24);
                if (!ip) continue;
                if (card) cpc_min(P, s, sketch, ip4_coupon(ip), (int64_t)gidx);
                if (tops) global_add(P, s, PV_KEY(TM_IPV4, ip), 1, j);
            } else if (e.l3 == 6 && alen == 16) {
                uint64_t w0 = 0, w1 = 0;
                for (int b = 0; b < 8; b++) { w0 |= (uint64_t)a[b] << (8 * b); w1 |= (uint64_t)a[8 + b] << (8 * b); }
                if (!(w0 | w1)) continue;
                uint64_t h1, h2;
                murmur_16(w0, w1, h1, h2);
                if (card) cpc_min(P, s, sketch, cpc_coupon(h1, h2), (int64_t)gidx);
                if (tops) global_add(P, s, PV_KEY(TM_IPV6, (h1 ^ (h2 << 1)) & ((1ull << 55) - 1)), 1, j);
            }
        }
    }
    // ---- Net v2 (net/v2/NetStreamHandler.cpp:533-604): the same events by direction; deep, the
    // query address as the source and the response address as the destination, both counted
    if (P.net2_groups) {
        const uint32_t s = P.slot_of[0], d = e.dir;
        const bool deep = !(e.pad[0] & 1);
        sum_add(P, s, PV_OFF_NET2 + N2_EVENTS, 1);
        if (deep) sum_add(P, s, PV_OFF_NET2 + N2_SAMPLES, 1);
        const uint32_t dc = PV_OFF_NET2 + N2_DIR + 8 * d;
        sum_add(P, s, dc + N2_TOTAL, 1);
        if (e.l3) sum_add(P, s, dc + (e.l3 == 4 ? N2_V4 : N2_V6), 1);
        sum_add(P, s, dc + (e.l4 == 17 ? N2_UDP : (e.l4 == 6 ? N2_TCP : N2_OTHER)), 1);
        sum_add(P, s, PV_OFF_PAYLOAD2 + d * PV_PAYLOAD_BINS + min(e.size, 65535u), 1);
        const bool card = P.net2_groups & PV_N2G_CARDINALITY, tops = P.net2_groups & PV_N2G_TOP_IPS;
        for (int side = 0; side < 2 && deep; side++) {
            const uint8_t *a = side ? e.raddr : e.qaddr;
            const uint32_t alen = side ? e.rlen : e.qlen;
            if (e.l3 == 4 && alen == 4) {
                const uint32_t ip = (uint32_t)a[0] | ((uint32_t)a[1] << 8) | ((uint32_t)a[2] << 16) | ((uint32_t)a[3] << 24);
                if (!ip) continue;
                if (card) cpc_min(P, s, CPC_V2 + d, ip4_coupon(ip), (int64_t)(P.gbase + j));
                if (tops) global_add(P, s, PV_V2_IP4(d, ip), 1, j);
            } else if (e.l3 == 6 && alen == 16) {
                uint64_t w0 = 0, w1 = 0;
                for (int b = 0; b < 8; b++) { w0 |= (uint64_t)a[b] << (8 * b); w1 |= (uint64_t)a[8 + b] << (8 * b); }
                if (!(w0 | w1)) continue;
                uint64_t h1, h2;
                murmur_16(w0, w1, h1, h2);
                if (card) cpc_min(P, s, CPC_V2 + d, cpc_coupon(h1, h2), (int64_t)(P.gbase + j));
                if (tops) global_add(P, s, PV_V2_IP6(d, h1 ^ (h2 << 1)), 1, j);
            }
        }
    }
    // ---- DNS v2 (DnsMetricsManager::process_dnstap, dns/v2/DnsStreamHandler.cpp:1176-1270): the
    // transaction direction by message type; a response with its message ends the transaction
    // DnsXactID(transactionID, 2) of that direction's map, else a query message starts one
    if (P.dns2_groups) {
        const uint32_t s = P.dslot_of[0];
        const bool ddeep = !(e.pad[0] & 2);
        sum_add(P, s, PV_OFF_DNS + DC_EVENTS, 1);
        if (ddeep) sum_add(P, s, PV_OFF_DNS + DC_SAMPLES, 1);
        if (e.filtered) {
            if (P.dns2_groups & PV_D2G_COUNTERS) sum_add(P, s, PV_OFF_DNS + DC_FILTERED, 1);
            return;
        }
        const uint32_t v2 = e.pad[1]; // xd | qr << 2 | has a message << 3 | socket protocol << 4
        if (!(v2 & 8) || !P.want_events) return;
        const GAcc R{P.recs};
        const uint32_t txid = e.mlen >= 2 ? (R.u8(e.moff) << 8) | R.u8(e.moff + 1) : 0u;
        PvXEvent ev;
        ev.key = ((uint64_t)txid << 16) | 2u | ((uint64_t)((v2 & 3) + 1) << 48);
        ev.idx = j;
        ev.len = e.mlen;
        ev.sec = e.sec;
        ev.nsec = (int32_t)e.nsec;
        ev.qr = (uint8_t)((v2 >> 2) & 1);
        ev.dir = (uint8_t)(0x80u | ((e.l3 == 4 ? 1u : (e.l3 == 6 ? 2u : 0u)) << 4) | ((v2 >> 4) & 7));
        ev.period = 0;
        ev.pad = ddeep ? 0 : 32; // a dnstap query: CD false, no subnet (start_transaction :1265-1268)
        const uint64_t eidx = (uint64_t)blockIdx.x * P.wt_per_block * PV_WT + atomicAdd(nev, 1u);
        if (ev.qr) atomicAdd(nresp, 1u);
        P.events[eidx] = ev;
        P.ekeys[eidx] = xact_sort_key(ev.key, (P.ekey_base << 2) + (j << 2));
        return;
    }
    // ---- DNS v1
    {
        const uint32_t s = P.dslot_of[0];
        const bool dc = P.dns_groups & PV_DNS_COUNTERS_BIT;
        // deep sampling: a not-deep event takes process_dns_layer(l3, l4, side) (dns/v1 ...cpp:882-885);
        // a filtered one counts the manager's last flag
        const bool ddeep = !(e.pad[0] & 2);
        if (e.filtered || e.dns_mode != PV_DT_MESSAGE || !ddeep) {
            sum_add(P, s, PV_OFF_DNS + DC_EVENTS, 1);
            if (ddeep) sum_add(P, s, PV_OFF_DNS + DC_SAMPLES, 1);
            if (e.filtered) {
                if (dc) sum_add(P, s, PV_OFF_DNS + DC_FILTERED, 1);
            } else if ((e.dns_mode == PV_DT_SIDE || !ddeep) && dc) {
                // process_dns_layer(l3, l4, side) (:1051-1091)
                sum_add(P, s, PV_OFF_DNS + DC_TOTAL, 1);
                if (e.l3) sum_add(P, s, PV_OFF_DNS + (e.l3 == 6 ? DC_V6 : DC_V4), 1);
                if (e.l4 == 17 || e.l4 == 6) sum_add(P, s, PV_OFF_DNS + (e.l4 == 6 ? DC_TCP : DC_UDP), 1);
                sum_add(P, s, PV_OFF_DNS + (e.side ? DC_REPLIES : DC_QUERIES), 1);
            }
            return;
        }
        DnsMsg dm;
        dm.idx = j;
        dm.moff = e.moff;
        dm.mlen = (uint16_t)min(e.mlen, 65535u);
        dm.mcap = dm.mlen;
        dm.port = e.qport;
        dm.flags = (uint8_t)(8u | (e.l3 == 6 ? 4u : 0u) | (e.l3 == 0 ? 16u : 0u) |
                             ((e.l4 == 17 ? 0u : (e.l4 == 6 ? 1u : 2u)) << 5));
        dm.period = 0;
        dm.fkey = 0;
        dm.sec = e.sec;
        dm.nsec = e.nsec;
        dm.pad = j << 2;
        DnsCtr c;
        c.zero();
        dns_process<false, true, false>(P, (KeyCache<PV_NCACHE> *)nullptr, nullptr, nullptr, nullptr, 0, R, dm, false, c);
    }
}

// Packs the event regions of workgroups b0 .. b0 + gridDim.x - 1 (the TCP pass's, dnstap's; the
// UDP DNS pass writes its keys in place) into one dense run of the key list from kbase, adding
// their total to n_events[0] and setting the key list's length n_keys (region order is
// irrelevant: events are sorted by (key, index)).
extern "C" __global__ void pv_xact_compact(const PvParams *__restrict__ Pp, uint32_t b0, uint32_t kbase)
{
    PV_CREF(PvParams) P = *(const PV_C PvParams *)Pp;
    __shared__ uint32_t part[4];
    // this block's base: the events of all earlier blocks, summed by the whole block
    uint32_t b = 0;
    for (uint32_t j = threadIdx.x; j < blockIdx.x; j += blockDim.x) b += P.blk_events[b0 + j];
    b = wave_sum(b);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = b;
    __syncthreads();
    const uint32_t base = part[0] + part[1] + part[2] + part[3];
    const uint32_t cnt = P.blk_events[b0 + blockIdx.x];
    if (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1) {
        if (base + cnt) atomicAdd(P.n_events, base + cnt);
        *P.n_keys = kbase + base + cnt;
    }
    const uint64_t src = (uint64_t)(b0 + blockIdx.x) * P.wt_per_block * PV_WT;
    for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) {
        P.skeys[kbase + base + j] = P.ekeys[src + j];
        P.svals[kbase + base + j] = (uint32_t)(src + j);
    }
}

// Fills a list of device regions in one launch (bucket-slot clears and the per-batch
// status reset), grid-stride over every segment.
__device__ __forceinline__ void fill_segs(const PvFillList &L);
extern "C" __global__ void pv_fill_multi(PvFillList L) { fill_segs(L); }
// the fills and a parameter block (pv_store_blob's store) in one launch: the batch's first
extern "C" __global__ void pv_fill_store(PvFillList L, PvBlob b, uint4 *dst, uint32_t n16)
{
    const uint32_t t = threadIdx.x;
    if (blockIdx.x == 0 && t < n16) dst[t] = make_uint4(b.w[4 * t], b.w[4 * t + 1], b.w[4 * t + 2], b.w[4 * t + 3]);
    fill_segs(L);
}
__device__ __forceinline__ void fill_segs(const PvFillList &L)
{
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint32_t k = 0; k < L.n; k++) {
        const PvFillSeg &f = L.s[k];
        if (f.w32) {
            uint32_t *p = reinterpret_cast<uint32_t *>(f.p);
            for (uint64_t i = g; i < f.n; i += gs) p[i] = (uint32_t)f.v;
        } else {
            uint64_t *p = reinterpret_cast<uint64_t *>(f.p);
            for (uint64_t i = g; i < f.n; i += gs) p[i] = f.v;
        }
    }
}

// Stores a by-value parameter block (n16 16-B words) to device memory: one workgroup.
extern "C" __global__ void __launch_bounds__(PV_BLOB_WORDS) pv_store_blob(PvBlob b, uint4 *dst, uint32_t n16)
{
    const uint32_t t = threadIdx.x;
    if (t < n16) dst[t] = make_uint4(b.w[4 * t], b.w[4 * t + 1], b.w[4 * t + 2], b.w[4 * t + 3]);
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
// a whole batch at once: events sorted by (24-bit hash of (flow,txid), stream rank); a
// response pairs with the immediately preceding event of the same key iff that
// event is a query (start_transaction overwrites, maybe_end_transaction erases).
// Period shifts purge queries older than the TTL (DnsStreamHandler.h:252-267).
namespace {
// first shift k (1-based period index) after period `a` whose threshold purges a
// query started at `sec`; returns 0 if none inside this batch
__device__ __forceinline__ uint32_t purge_period(PV_CREF(PvParams) P, uint32_t ttl_s, uint32_t a, int64_t sec)
{
    for (uint32_t k = a + 1; k <= P.n_dshift; k++)
        if (P.dthresh[k - 1] >= (int64_t)ttl_s + sec) return k;
    return 0;
}
// Workgroup-local staging: transaction counters per period and the quantile / slow
// lists are gathered in LDS and reserved in global memory once per workgroup, so no
// global address sees more than one atomic per workgroup.
enum { XC_TOTAL, XC_OUT, XC_IN, XC_TIMEOUT, XC_N };
struct XState {
    uint32_t ctr[PV_MAX_SHIFTS + 1][XC_N];
    uint32_t c2[PV_MAX_SHIFTS + 1][3][D2_N]; // DNS v2 counters per period and direction
    PvXValue val[PV_BLOCK * 3];
    PvXValid valid[PV_BLOCK];
    uint32_t nval, nvalid, vbase, dbase;
};
// Lanes of a wave adding to one LDS word serialise there (most transactions of a batch bump the
// same few counters): one add per distinct word instead, each by the lowest lane that holds it.
// Callable in divergent code: the loop runs over the active lanes' words, uniformly.
__device__ __forceinline__ void lds_inc(uint32_t *a)
{
    const uint32_t lane = __lane_id();
    const uint64_t ad = (uint64_t)(uintptr_t)a;
    uint64_t pend = __ballot(1);
    while (pend) {
        const uint32_t ld = (uint32_t)__builtin_ctzll(pend);
        const uint64_t la = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(ad >> 32), ld) << 32) |
                            __builtin_amdgcn_readlane((uint32_t)ad, ld);
        const uint64_t eq = __ballot(ad == la);
        if (lane == ld) atomicAdd(a, (uint32_t)__popcll(eq));
        pend &= ~eq;
    }
}
// one slot of an LDS-counted list per active lane: one add per wave
__device__ __forceinline__ uint32_t lds_reserve(uint32_t *ctr)
{
    const uint64_t m = __ballot(1);
    const uint32_t ld = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (__lane_id() == ld) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __builtin_amdgcn_readlane(base, ld);
    return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ void xctr(XState &T, uint32_t period, uint32_t c) { lds_inc(&T.ctr[period][c]); }
__device__ __forceinline__ void xval(PV_CREF(PvXactParams) X, XState &T, uint32_t period, uint32_t kind, uint64_t bits)
{
    T.val[lds_reserve(&T.nval)] = PvXValue{bits, X.slot_gen[period], kind};
}
// DnsMetricsBucket::new_dns_transaction slow branch (dns/v1 ...cpp:1126-1136): the
// response's first query name (getName(), case kept) into top_slow
__device__ void slow_check(PV_CREF(PvXactParams) X, uint32_t idx, uint32_t period, uint32_t dir, uint64_t us)
{
    const float thr = dir == 0 ? X.thr_from[period] : (dir == 1 ? X.thr_to[period] : 0.0f);
    if (!(thr > 0.0f && (float)us >= thr)) return;
    PV_CREF(PvParams) P = X.P;
    Parsed o;
    const bool tcp = idx & PV_TCP_IDX;
    const GAcc R{tcp ? X.trecs : P.recs};
    if (tcp) {
        ParseCfg C = parse_cfg(P);
        C.linktype = 101;
        idx &= ~PV_TCP_IDX;
        parse_record(R, C, P, X.toffs[idx], o);
    } else {
        parse_record(R, P, P.offs[idx], o);
    }
    uint64_t m = o.l4off + 8;
    uint32_t len = o.l4len - 8;
    DnsInfo d;
    dns_parse(R, m, len, be16(R, m + 4), be16(R, m + 6), be16(R, m + 8), be16(R, m + 10), d);
    if (!(d.ok && d.has_query)) return;
    RawName rn{0, 0};
    if (d.name_len_enc > 0) name_emit(R, m, len, 12, rn);
    const uint32_t metric = dir == 0 ? TM_SLOW_OUT : TM_SLOW_IN;
    const NameSrc ns{X.trecs, X.toffs};
    global_add(P, P.dslot_of[period], PV_KEY(metric, fp56(rn.ph, rn.n, 1)), 1, idx, tcp ? &ns : nullptr);
}
// DnsMetricsBucket::new_dns_transaction, DNS v2 (dns/v2/DnsStreamHandler.cpp:925-1089): a
// valid, kept transaction accounted on its response (record e.idx of this batch) in the
// response's transaction direction xd; qe is its query. Name tops and dense tables go
// straight to the period's tables (v2 keys carry the direction).
__device__ void dns2_xact(PV_CREF(PvXactParams) X, XState &T, const PvXEvent &e, const PvXEvent &qe, uint32_t xd,
                          uint64_t us, int64_t order, uint64_t qaddr)
{
    PV_CREF(PvParams) P = X.P;
    const uint32_t g = P.dns2_groups;
    const uint32_t period = e.period, slot = P.dslot_of[period];
    const bool tcp = e.idx & PV_TCP_IDX;
    const uint32_t idx = e.idx & ~PV_TCP_IDX;
    Parsed o;
    const GAcc R{tcp ? X.trecs : P.recs};
    if (tcp) {
        ParseCfg C = parse_cfg(P);
        C.linktype = 101;
        parse_record(R, C, P, X.toffs[idx], o);
    } else {
        parse_record(R, P, P.offs[idx], o);
    }
    const uint64_t m = o.l4off + 8;
    const uint32_t len = e.len;
    const uint32_t b23 = R.u32(m) >> 16; // header bytes 2, 3
    const uint32_t rcode = (b23 >> 8) & 15;
    const uint32_t qd = be16(R, m + 4), an = be16(R, m + 6), ns = be16(R, m + 8), ar = be16(R, m + 10);
    uint32_t *c = T.c2[period][xd];
    if (g & PV_D2G_COUNTERS) {
        lds_inc(&c[D2_XACTS]);
        if (e.dir & 0x80) {
            // a dnstap event: l3 from socket_family, l4 the socket protocol (new_dns_transaction :936-970)
            const uint32_t l3 = (e.dir >> 4) & 3, pr = e.dir & 7;
            if (l3) lds_inc(&c[l3 == 2 ? D2_V6 : D2_V4]);
            if (pr) {
                const uint32_t w[8] = {0, D2_UDP, D2_TCP, D2_DOT, D2_DOH, D2_CRYPT_UDP, D2_CRYPT_TCP, D2_DOQ};
                lds_inc(&c[w[pr]]);
            }
        } else {
            lds_inc(&c[(e.pad & 2) ? D2_V6 : D2_V4]);
            lds_inc(&c[tcp ? D2_TCP : D2_UDP]);
        }
        if (qe.pad & 1) lds_inc(&c[D2_CD]);
        if (rcode == 0) { lds_inc(&c[D2_NOERROR]); if (!an) lds_inc(&c[D2_NODATA]); }
        else if (rcode == 2) lds_inc(&c[D2_SRVFAIL]);
        else if (rcode == 3) lds_inc(&c[D2_NX]);
        else if (rcode == 5) lds_inc(&c[D2_REFUSED]);
        if (b23 & 0x04) lds_inc(&c[D2_AA]);
        if (b23 & 0x2000) lds_inc(&c[D2_AD]);
    }
    // deep sampling: a response that drew "not deep" stops after the counters (:1006-1008)
    if (e.pad & 32) return;
    if (qe.len && (g & PV_D2G_TOP_SIZE))
        xval(X, T, period, XV2_RATIO + xd, (uint64_t)__double_as_longlong((double)len / (double)qe.len));
    const uint32_t port = dns_port(R.u32(o.l4off));
    if (port && (g & PV_D2G_TOP_PORTS)) sum_add(P, slot, PV_OFF_PORT2 + xd * PV_PORT_BINS + port, 1);
    if (g & PV_D2G_XACT_TIMES) xval(X, T, period, XV2_TIME + xd, us);
    DnsInfo d;
    dns_parse(R, m, len, qd, an, ns, ar, d);
    if (!d.ok) return;
    sum_add(P, slot, PV_OFF_RCODE2 + xd * PV_RCODE_BINS + rcode, 1);
    // top_ecs (:1077-1089): the query's subnet, past the resources parse and with or without a
    // question; its name record straight from the carried address
    const uint32_t qfam = (qe.pad >> 3) & 3;
    if ((g & PV_D2G_TOP_ECS) && qfam) {
        if (g & PV_D2G_COUNTERS) lds_inc(&c[D2_ECS]);
        const NameSrc es{nullptr, nullptr, qaddr, qfam};
        global_add(P, slot, PV_V2_DKEY(TM_ECS, xd, fmix64(qaddr ^ ((uint64_t)qfam << 62) ^ 0xec5ull)), 1, idx, &es);
    }
    if (!d.has_query) return;
    NameStats st;
    st.init();
    if (d.name_len_enc > 0) name_stats(R, m, len, 12, st);
    uint64_t h1, h2;
    st.mm.finish(h1, h2);
    if (st.n > 0 && (g & PV_D2G_CARDINALITY)) cpc_min(P, slot, CPC_QNAME2 + xd, cpc_coupon(h1, h2), order);
    sum_add(P, slot, PV_OFF_QTYPE2 + xd * PV_QTYPE_BINS + (d.qtype & 0xffff), 1);
    const NameSrc ns_{X.trecs, X.toffs, 0, 0, X.tsfx};
    const NameSrc *nsp = tcp ? &ns_ : nullptr;
    const uint64_t fp = fp56(st.ph, st.n, 0);
    auto add = [&](uint32_t metric, uint64_t f, uint32_t w) { global_add(P, slot, PV_V2_DKEY(metric, xd, f), w, idx, nsp); };
    if (g & PV_D2G_TOP_RCODES) {
        if (rcode == 2) add(TM_SRVFAIL, fp, 1);
        else if (rcode == 3) add(TM_NX, fp, 1);
        else if (rcode == 5) add(TM_REFUSED, fp, 1);
        else if (rcode == 0) { add(TM_NOERROR, fp, 1); if (!an) add(TM_NODATA, fp, 1); }
    }
    if (g & PV_D2G_TOP_SIZE) add(TM_SIZED, fp, len);
    if (g & PV_D2G_XACT_TIMES) {
        const float thr = X.thr2[period][xd];
        if (thr < 0.0f) T.valid[lds_reserve(&T.nvalid)] = PvXValid{e.idx, (uint8_t)period, (uint8_t)(4 + xd), 0, 0, us};
        else if (thr > 0.0f && (float)us >= thr) add(TM_SLOW_OUT, fp, 1);
    }
    if (g & PV_D2G_TOP_QNAMES) {
        int q2, q3;
        uint64_t h2p, h3p;
        // public_suffix_list: the response's own suffix size (_configs, v2 :612-619)
        const uint32_t sfx = name_sfx(P, idx, tcp ? X.tsfx : P.sfx_of);
        if (sfx) agg_domain_r(R, m, len, st, q2, q3, h2p, h3p, sfx);
        else agg_domain(st, q2, q3, h2p, h3p, 0);
        const uint64_t k2 = q2 == 0 ? st.ph : suffix_hash(st, q2, h2p);
        add(TM_QNAME2, fp56(k2, st.n - q2, 0), 1);
        if (q3 >= 0 && (uint32_t)q3 < st.n) {
            const uint64_t k3 = q3 == 0 ? st.ph : suffix_hash(st, q3, h3p);
            add(TM_QNAME3, fp56(k3, st.n - q3, 0), 1);
        }
    }
}
// the deferred slow check of a DNS v2 transaction (its period's p90 was not known at resolve)
__device__ void dns2_slow(PV_CREF(PvXactParams) X, uint32_t eidx, uint32_t period, uint32_t xd, uint64_t us)
{
    const float thr = X.thr2[period][xd];
    if (!(thr > 0.0f && (float)us >= thr)) return;
    PV_CREF(PvParams) P = X.P;
    const bool tcp = eidx & PV_TCP_IDX;
    const uint32_t idx = eidx & ~PV_TCP_IDX;
    Parsed o;
    const GAcc R{tcp ? X.trecs : P.recs};
    if (tcp) {
        ParseCfg C = parse_cfg(P);
        C.linktype = 101;
        parse_record(R, C, P, X.toffs[idx], o);
    } else {
        parse_record(R, P, P.offs[idx], o);
    }
    const uint64_t m = o.l4off + 8;
    const uint32_t len = o.l4len - 8;
    DnsInfo d;
    dns_parse(R, m, len, be16(R, m + 4), be16(R, m + 6), be16(R, m + 8), be16(R, m + 10), d);
    if (!(d.ok && d.has_query)) return;
    NameStats st;
    st.init();
    if (d.name_len_enc > 0) name_stats(R, m, len, 12, st);
    const NameSrc ns_{X.trecs, X.toffs};
    global_add(P, P.dslot_of[period], PV_V2_DKEY(TM_SLOW_OUT, xd, fp56(st.ph, st.n, 0)), 1, idx, tcp ? &ns_ : nullptr);
}
} // namespace

// event of a sorted position: this batch's events, or a query carried in from an earlier batch
__device__ __forceinline__ PvXEvent xev(PV_CREF(PvXactParams) X, uint32_t p)
{
    const uint32_t v = X.svals[p];
    return (v & PV_PEND_FLAG) ? X.pend[v & ~PV_PEND_FLAG] : X.events[v];
}
// the ECS address of a DNS v2 query event (top_ecs), carried or of this batch
__device__ __forceinline__ uint64_t xecs(PV_CREF(PvXactParams) X, uint32_t p)
{
    const uint32_t v = X.svals[p];
    return (v & PV_PEND_FLAG) ? X.pecs[v & ~PV_PEND_FLAG] : X.P.eecs[v];
}

__device__ void resolve_one(PV_CREF(PvXactParams) X, XState &T, uint32_t p)
{
    PV_CREF(PvParams) P = X.P;
    const PvXEvent e = xev(X, p);
    const uint32_t h = (uint32_t)(X.skeys[p] >> 32);
    if (e.qr) {
        // predecessor on the same (flow, txid)
        int q = (int)p - 1;
        for (; q >= 0 && (uint32_t)(X.skeys[q] >> 32) == h; q--)
            if (xev(X, q).key == e.key) break;
        if (q < 0 || (uint32_t)(X.skeys[q] >> 32) != h) {
            // NotExist here; a shard-edge stub for the multi-GPU merge
            const uint32_t k = atomicAdd(X.n_orph, 1u);
            if (k < X.orph_cap) {
                PvXEvent o = e;
                o.pad = (uint8_t)(P.dslot_of[e.period] | (e.period >= P.dskip_before ? 0x80u : 0u) | ((e.pad & 4) ? 0x40u : 0u));
                X.orph[k] = o;
            }
            return;
        }
        const PvXEvent qe = xev(X, q);
        if (qe.qr) return; // previous event was a response: erased => NotExist
        uint32_t kp = purge_period(P, X.ttl_s, qe.period, qe.sec);
        if (kp && kp <= e.period) return; // purged at a period shift before this response
        const bool kept = e.period >= P.dskip_before;
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
        // a response that is not deep: counts only (new_dns_transaction !deep, :1105-1121)
        const bool rdeep = !(e.pad & 4);
        // quantile inputs of every period (skipped ones still feed the next period's p90)
        if (X.quantiles && rdeep) {
            if (e.dir == 0) xval(X, T, e.period, XV_FROM_US, us);
            else if (e.dir == 1) xval(X, T, e.period, XV_TO_US, us);
        }
        if ((X.quantiles & 1) && qe.len && kept && rdeep)
            xval(X, T, e.period, XV_RATIO, (uint64_t)__double_as_longlong((double)e.len / (double)qe.len));
        if (!kept || e.dir == 2 || !rdeep) return;
        // top_slow: a period without a threshold yet defers every candidate; with one, only the
        // slow transactions are listed. pv_xact_slow_dev names them after the resolve (the record
        // parse and the table insert stay out of this kernel, which then makes no device call)
        const float thr = e.dir == 0 ? X.thr_from[e.period] : X.thr_to[e.period];
        if (X.thr_from[e.period] < 0.0f || (thr > 0.0f && (float)us >= thr))
            T.valid[lds_reserve(&T.nvalid)] = PvXValid{e.idx, (uint8_t)e.period, (uint8_t)e.dir, 0, 0, us};
    } else {
        if (X.edge_h && e.sec < X.edge_h) {
            // sharded runs: the first query of its key may overwrite an open query of an earlier
            // shard (the stub list holds it next to the orphan responses)
            int q = (int)p - 1;
            for (; q >= 0 && (uint32_t)(X.skeys[q] >> 32) == h; q--)
                if (xev(X, q).key == e.key) break;
            if (q < 0 || (uint32_t)(X.skeys[q] >> 32) != h) {
                const uint32_t k = atomicAdd(X.n_orph, 1u);
                if (k < X.orph_cap) {
                    PvXEvent o = e;
                    o.pad = (uint8_t)(P.dslot_of[e.period] | (e.period >= P.dskip_before ? 0x80u : 0u) | ((e.pad & 4) ? 0x40u : 0u));
                    X.orph[k] = o;
                }
            }
        }
        // an open query purged at a later period shift counts as timed out there
        uint32_t kp = purge_period(P, X.ttl_s, e.period, e.sec);
        if (!kp) return;
        uint32_t q = p + 1;
        for (; q < X.n && (uint32_t)(X.skeys[q] >> 32) == h; q++)
            if (xev(X, q).key == e.key) break;
        if (q < X.n && (uint32_t)(X.skeys[q] >> 32) == h && xev(X, q).period < kp) return;
        if (kp < P.dskip_before) return;
        xctr(T, kp, XC_TIMEOUT);
    }
}

// A DNS v2 shard-edge stub (sharded runs, X.orph_ord set): the first event of its key in this
// context's stream, kept whole (pad intact: the edge pair's accounting reads it) with the kept
// flag in period bit 7, and its first-occurrence order
__device__ __forceinline__ void stub2(PV_CREF(PvXactParams) X, const PvXEvent &e, uint32_t p, bool kept)
{
    PV_CREF(PvParams) P = X.P;
    const uint32_t k = atomicAdd(X.n_orph, 1u);
    if (k >= X.orph_cap) return;
    PvXEvent o = e;
    o.period = (uint8_t)(e.period | (kept ? 0x80u : 0u));
    X.orph[k] = o;
    X.orph_ord[k] = (int64_t)((P.gbase << 2) + ((uint32_t)X.skeys[p] - (P.ekey_base << 2)));
}
// TransactionManager per direction, DNS v2 (dns/v2/DnsStreamHandler.cpp:1100-1145 and the
// manager's on_period_shift, .h:440-453): a response of transaction direction xd is
// Valid, TimedOut or NotExist (orphan) against the latest event of its key (the key holds
// xd); every outcome sets the direction up in the response's bucket. An open query
// purged at a later shift is a time-out of that period. Queries account nothing.
__device__ void resolve_one2(PV_CREF(PvXactParams) X, XState &T, uint32_t p)
{
    PV_CREF(PvParams) P = X.P;
    const PvXEvent e = xev(X, p);
    const uint32_t h = (uint32_t)(X.skeys[p] >> 32);
    const uint32_t xd = (uint32_t)((e.key >> 48) & 3) - 1;
    if (e.qr) {
        const bool kept = e.period >= P.dskip_before;
        uint32_t *c = T.c2[e.period][xd];
        if (kept) lds_inc(&c[D2_SEEN]);
        int q = (int)p - 1;
        for (; q >= 0 && (uint32_t)(X.skeys[q] >> 32) == h; q--)
            if (xev(X, q).key == e.key) break;
        const bool first = q < 0 || (uint32_t)(X.skeys[q] >> 32) != h;
        if (first && X.orph_ord) stub2(X, e, p, kept); // may answer a query an earlier shard left open
        const bool found = !first && !xev(X, q).qr;
        const PvXEvent qe = found ? xev(X, q) : e;
        const uint32_t kp = found ? purge_period(P, X.ttl_s, qe.period, qe.sec) : 0u;
        const bool rf = e.pad & 4, qf = found && (qe.pad & 4); // filtered response / query (v2 filters)
        // process_filtered's second `filtered` (a valid pair with an unfiltered query), or a
        // response to a filtered query (dns/v2 ...cpp:1115-1119,1160-1164)
        auto filtered = [&]() {
            if (kept && (P.dns2_groups & PV_D2G_COUNTERS)) sum_add(P, P.dslot_of[e.period], PV_OFF_DNS + DC_FILTERED, 1);
        };
        if (!found || (kp && kp <= e.period)) { if (kept && !rf) lds_inc(&c[D2_ORPHAN]); return; }
        int64_t dsec = e.sec > qe.sec ? e.sec - qe.sec : qe.sec - e.sec;
        int64_t dnsec = (int64_t)e.nsec - (int64_t)qe.nsec;
        if (dnsec < 0) { dsec--; dnsec += 1000000000LL; }
        const bool timed_out = dsec > (int64_t)X.ttl_s || (dsec == (int64_t)X.ttl_s && ((double)dnsec / 1.0e6) >= (double)X.ttl_ms);
        if (rf) { if (!timed_out && !qf) filtered(); return; }
        if (qf) { filtered(); return; }
        if (timed_out) { if (kept) lds_inc(&c[D2_TIMEOUT]); return; }
        const uint64_t us = (uint64_t)((dsec * 1000000000LL) + dnsec) / 1000;
        if (!kept) {
            // a period outside the window still feeds the next period's p90
            if (P.dns2_groups & PV_D2G_XACT_TIMES) xval(X, T, e.period, XV2_TIME + xd, us);
            return;
        }
        // the response's first-occurrence order (the DNS pass's CPC order: batch base * 4 + rank)
        const int64_t order = (int64_t)((P.gbase << 2) + ((uint32_t)X.skeys[p] - (P.ekey_base << 2)));
        dns2_xact(X, T, e, qe, xd, us, order, ((qe.pad >> 3) & 3) ? xecs(X, q) : 0ull);
    } else {
        if (X.orph_ord && X.edge_h && e.sec < X.edge_h) {
            // sharded runs: the first query of its key may overwrite an open query of an earlier shard
            int q = (int)p - 1;
            for (; q >= 0 && (uint32_t)(X.skeys[q] >> 32) == h; q--)
                if (xev(X, q).key == e.key) break;
            if (q < 0 || (uint32_t)(X.skeys[q] >> 32) != h) stub2(X, e, p, e.period >= P.dskip_before);
        }
        const uint32_t kp = purge_period(P, X.ttl_s, e.period, e.sec);
        if (!kp) return;
        uint32_t q = p + 1;
        for (; q < X.n && (uint32_t)(X.skeys[q] >> 32) == h; q++)
            if (xev(X, q).key == e.key) break;
        if (q < X.n && (uint32_t)(X.skeys[q] >> 32) == h && xev(X, q).period < kp) return;
        if (kp < P.dskip_before) return;
        lds_inc(&T.c2[kp][xd][D2_TIMEOUT]);
        lds_inc(&T.c2[kp][xd][D2_SEEN]);
    }
}

// Queries still open after this batch (the latest event of their (flow, txid) is a query
// not purged by a period shift here) move to the carried list for the next batch, as
// period 0 with sort rank 0: TransactionManager's map surviving the batch edge. Run by the
// resolve kernel's threads on their own sorted positions (one pass over the events).
__device__ __forceinline__ void carry_one(PV_CREF(PvXactParams) X, uint32_t p)
{
    PvXEvent e = xev(X, p);
    if (e.qr || purge_period(X.P, X.ttl_s, e.period, e.sec)) return;
    const uint32_t h = (uint32_t)(X.skeys[p] >> 32);
    for (uint32_t q = p + 1; q < X.n && (uint32_t)(X.skeys[q] >> 32) == h; q++)
        if (xev(X, q).key == e.key) return;
    e.period = 0;
    const uint32_t k = atomicAdd(X.n_pend_out, 1u);
    X.pend_out[k] = e;
    if (X.pecs_out) X.pecs_out[k] = ((e.pad >> 3) & 3) ? xecs(X, p) : 0ull;
    X.pkeys_out[k] = (uint64_t)h << 32;
    X.pvals_out[k] = k;
}
extern "C" __global__ void pv_xact_carry(const PvXactParams *__restrict__ Xp)
{
    PV_CREF(PvXactParams) X = *(const PV_C PvXactParams *)Xp;
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < X.n) carry_one(X, p);
}

__device__ __forceinline__ void xstate_init(XState &T)
{
    for (uint32_t j = threadIdx.x; j < (PV_MAX_SHIFTS + 1) * XC_N; j += blockDim.x) (&T.ctr[0][0])[j] = 0;
    for (uint32_t j = threadIdx.x; j < (PV_MAX_SHIFTS + 1) * 3 * D2_N; j += blockDim.x) (&T.c2[0][0][0])[j] = 0;
    if (threadIdx.x == 0) { T.nval = 0; T.nvalid = 0; }
    __syncthreads();
}
// the block's transaction counters into the periods' buckets, its values and deferred slow
// candidates appended to the context's lists (after a __syncthreads)
__device__ __forceinline__ void xstate_flush(PV_CREF(PvXactParams) X, XState &T)
{
    PV_CREF(PvParams) P = X.P;
    if (P.dns2_groups)
        for (uint32_t j = threadIdx.x; j < (P.n_dshift + 1) * 3 * D2_N; j += blockDim.x) {
            const uint32_t per = j / (3 * D2_N), w = j % (3 * D2_N);
            const uint32_t v = (&T.c2[0][0][0])[j];
            if (v) sum_add(P, P.dslot_of[per], PV_OFF_DNS2 + (w / D2_N) * PV_DNS2_CTRS + w % D2_N, v);
        }
    static const uint8_t dc[XC_N] = {DC_XTOTAL, DC_XOUT, DC_XIN, DC_XTIMEOUT};
    if (threadIdx.x < (PV_MAX_SHIFTS + 1) * XC_N) {
        const uint32_t per = threadIdx.x / XC_N, c = threadIdx.x % XC_N;
        const uint32_t v = T.ctr[per][c];
        if (v && per <= P.n_dshift)
            atomicAdd((unsigned long long *)&P.sum[(uint64_t)P.dslot_of[per] * PV_SUM_WORDS + PV_OFF_DNS + dc[c]],
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

template <bool V2>
__device__ __forceinline__ void xact_resolve(const PvXactParams *__restrict__ Xp)
{
    PV_CREF(PvXactParams) X = *(const PV_C PvXactParams *)Xp;
    __shared__ XState T;
    xstate_init(T);
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < X.n) {
        if constexpr (V2) resolve_one2(X, T, p);
        else resolve_one(X, T, p);
        if (X.pend_out) carry_one(X, p); // the queries still open go on to the next batch
    }
    __syncthreads();
    xstate_flush(X, T);
}
// DNS v1 (a context without the v2 handler) and DNS v2: one kernel each, so the v1 one carries
// none of the v2 accounting's table inserts
extern "C" __global__ void __launch_bounds__(PV_BLOCK) pv_xact_resolve(const PvXactParams *__restrict__ Xp)
{
    xact_resolve<false>(Xp);
}
extern "C" __global__ void __launch_bounds__(PV_BLOCK) pv_xact_resolve2(const PvXactParams *__restrict__ Xp)
{
    xact_resolve<true>(Xp);
}

// DNS v2 transactions across a shard edge (pv_edge_carry): each pair as resolve_one2 accounts a
// valid, kept transaction (dns2_xact), the response's record in the run's blobs (P.recs / offs,
// TCP message records X.trecs / toffs), its period r.period of the run's table. With
// public_suffix_list the response's suffix size is matched here first (pv_dns_suffix's rule).
extern "C" __global__ void __launch_bounds__(PV_BLOCK) pv_xact_edge2(const PvXactParams *__restrict__ Xp,
                                                                     const PvEdgePair *__restrict__ pairs, uint32_t n,
                                                                     uint8_t *sfx, uint8_t *tsfx)
{
    PV_CREF(PvXactParams) X = *(const PV_C PvXactParams *)Xp;
    PV_CREF(PvParams) P = X.P;
    __shared__ XState T;
    xstate_init(T);
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) {
        const PvEdgePair e = pairs[p];
        const uint32_t xd = (uint32_t)((e.r.key >> 48) & 3) - 1;
        if ((P.f_flags & PVDF_PSL) && !(P.f_flags & PVDF_ONLY_QSUFFIX)) {
            const bool tcp = e.r.idx & PV_TCP_IDX;
            const uint32_t idx = e.r.idx & ~PV_TCP_IDX;
            const GAcc R{tcp ? X.trecs : P.recs};
            Parsed o;
            if (tcp) {
                ParseCfg C = parse_cfg(P);
                C.linktype = 101;
                parse_record(R, C, P, X.toffs[idx], o);
            } else {
                parse_record(R, P, P.offs[idx], o);
            }
            const uint64_t m = o.l4off + 8;
            (tcp ? tsfx : sfx)[idx] = (uint8_t)dns_suffix_of(P, R, m, e.r.len, be16(R, m + 4), be16(R, m + 6), be16(R, m + 8),
                                                             be16(R, m + 10));
        }
        if (xd < 3) dns2_xact(X, T, e.r, e.q, xd, e.us, e.order, e.qaddr);
    }
    __syncthreads();
    xstate_flush(X, T);
}

// A batch with queries only and no period shift pairs nothing: its events join the
// carried list unresolved. With nothing carried the host hands the batch's event store, keys
// and values over to the carried list as they lie (no copy); otherwise this kernel appends them
// (the key list's sentinel slots left out): keys at `at`, events densely at `ehi` of the store,
// in the order of a wave-aggregated counter (ctr, zero at launch).
extern "C" __global__ void pv_xact_defer(const uint64_t *skeys, const uint32_t *svals, const PvXEvent *events, uint32_t n,
                                         PvXEvent *pend, uint64_t *pkeys, uint32_t *pvals, uint32_t at, uint32_t ehi,
                                         const uint64_t *eecs, uint64_t *pecs, uint32_t *ctr)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
    const uint64_t k = j < n ? skeys[j] : ~0ull;
    const bool ok = k != ~0ull;
    const uint64_t m = __ballot(ok);
    if (!m) return;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader, 64);
    if (!ok) return;
    const uint32_t q = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    const uint32_t v = svals[j];
    const PvXEvent ev = events[v];
    pend[ehi + q] = ev;
    pkeys[at + q] = k;
    pvals[at + q] = ehi + q;
    if (pecs) pecs[ehi + q] = ((ev.pad >> 3) & 3) ? eecs[v] : 0ull;
}
// the carried list's keys behind this batch's compacted keys, values flagged
extern "C" __global__ void pv_xact_pend_in(uint64_t *skeys, uint32_t *svals, const uint64_t *pkeys, const uint32_t *pvals,
                                           uint32_t n_pend, uint32_t at)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_pend) return;
    skeys[at + j] = pkeys[j];
    svals[at + j] = PV_PEND_FLAG | pvals[j];
}

// top_slow of the resolve's listed transactions (its count read on the device): the slow ones of
// periods with a threshold, and the candidates of periods whose threshold the host set after it
extern "C" __global__ void __launch_bounds__(256) pv_xact_slow_dev(const PvXactParams *__restrict__ Xp)
{
    PV_CREF(PvXactParams) X = *(const PV_C PvXactParams *)Xp;
    const uint32_t n = *X.n_valid;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const PvXValid v = X.valid[i];
        if (v.dir >= 4) dns2_slow(X, v.idx, v.period, v.dir - 4, v.us);
        else slow_check(X, v.idx, v.period, v.dir, v.us);
    }
}
// top_slow for transactions of periods whose threshold became known after the resolve
extern "C" __global__ void pv_xact_slow(const PvXactParams *__restrict__ Xp, uint32_t n_valid)
{
    PV_CREF(PvXactParams) X = *(const PV_C PvXactParams *)Xp;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_valid) return;
    const PvXValid v = X.valid[i];
    if (v.dir >= 4) dns2_slow(X, v.idx, v.period, v.dir - 4, v.us);
    else slow_check(X, v.idx, v.period, v.dir, v.us);
}

// Stable LSD radix sort of (key, value) pairs over the transaction keys' bits [0, 32 + 24)
// (rocPRIM onesweep; the all-ones sentinel is all ones there too, so it still sorts last)
extern "C" hipError_t pv_radix_sort_pairs(void *tmp, size_t *tmp_bytes, uint64_t *kin, uint64_t *kout, uint32_t *vin,
                                          uint32_t *vout, size_t n, hipStream_t s)
{
    return rocprim::radix_sort_pairs(tmp, *tmp_bytes, kin, kout, vin, vout, n, 0, 32 + PV_XHASH_BITS, s);
}

// ------------------------------------------------------------------ period-shift thresholds
// A DNS period shift sets the slow-transaction thresholds to the p90 of the transaction times of
// the bucket that closed (dns/v1/DnsStreamHandler.h:259-266, v2 :440-453). The rank-r value of
// each selected kind is found by radix selection over the device value buffer: a pass
// histograms byte `shift` of the values of slot sg (slot | generation << 8) whose higher bytes
// equal their kind's prefix so far; the host picks the byte holding the rank and the next pass
// narrows to it. Eight passes over the buffer instead of copying it to the host and sorting.
__device__ __forceinline__ int xv_sel_kind(uint32_t kind)
{
    return kind == XV_FROM_US ? 0 : kind == XV_TO_US ? 1 : (kind >= XV2_TIME && kind < XV2_TIME + 3) ? 2 + (int)(kind - XV2_TIME) : -1;
}
extern "C" __global__ void __launch_bounds__(256) pv_xv_hist(const PvXValue *__restrict__ v, const uint32_t *__restrict__ n_vals,
                                                          uint32_t cap, uint32_t sg, uint32_t shift, PvXvSel sel,
                                                          uint32_t *__restrict__ hist)
{
    __shared__ uint32_t h[PV_XV_SEL * 256];
    for (uint32_t i = threadIdx.x; i < PV_XV_SEL * 256; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint32_t n = min(*n_vals, cap); // the buffer's values (a full buffer counts past its end)
    const uint64_t hm = shift >= 56 ? 0ull : ~0ull << (shift + 8);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const PvXValue x = v[i];
        if (x.slot != sg) continue;
        const int k = xv_sel_kind(x.kind);
        if (k < 0 || (x.bits & hm) != (sel.prefix[k] & hm)) continue;
        atomicAdd(&h[k * 256 + (uint32_t)((x.bits >> shift) & 255)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < PV_XV_SEL * 256; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// ------------------------------------------------------------------ record gather (sharded top_slow)
// The records of a list of batch record indices (idx[i * stride], PV_TCP_IDX: a TCP message
// record of the batch's message arena), copied whole (16-B header + capture, 4-B padded) into
// one blob: the deferred slow-transaction candidates of a sharded run keep their response
// records this way until the merge knows every period's threshold (pv_slow_finish).
extern "C" __global__ void pv_rec_sizes(const uint8_t *recs, const uint32_t *offs, const uint8_t *trecs, const uint32_t *toffs,
                                        const uint32_t *idx, uint32_t stride, uint32_t n, uint32_t *sizes)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t id = idx[(uint64_t)i * stride];
    const bool tcp = id & PV_TCP_IDX;
    const uint8_t *r = tcp ? trecs + toffs[id & ~PV_TCP_IDX] : recs + offs[id];
    const uint32_t cap = min((uint32_t)r[8] | (uint32_t)r[9] << 8 | (uint32_t)r[10] << 16 | (uint32_t)r[11] << 24, 65535u);
    sizes[i] = (16u + cap + 3u) & ~3u;
}
extern "C" __global__ void pv_rec_gather(const uint8_t *recs, const uint32_t *offs, const uint8_t *trecs, const uint32_t *toffs,
                                         const uint32_t *idx, uint32_t stride, uint32_t n, const uint32_t *dst_off, uint8_t *out)
{
    // one wave per record, dword copies
    const uint32_t i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= n) return;
    const uint32_t id = idx[(uint64_t)i * stride];
    const bool tcp = id & PV_TCP_IDX;
    const uint8_t *r = tcp ? trecs + toffs[id & ~PV_TCP_IDX] : recs + offs[id];
    const uint32_t cap = min((uint32_t)r[8] | (uint32_t)r[9] << 8 | (uint32_t)r[10] << 16 | (uint32_t)r[11] << 24, 65535u);
    const uint32_t bytes = 16u + cap;
    uint8_t *o = out + dst_off[i];
    for (uint32_t b = lane; b < bytes; b += 64) o[b] = r[b];
    if (lane == 0) *reinterpret_cast<uint32_t *>(o + 8) = cap; // a clamped capture length stays consistent
    for (uint32_t b = bytes + lane; b < ((bytes + 3u) & ~3u); b += 64) o[b] = 0;
}

// ------------------------------------------------------------------ pcap BPF filter on the device
// The pcap input's filter (PcapInputStream::_open_pcap: reader->setFilter(bpf),
// src/inputs/pcap/PcapInputStream.cpp:485-488; libpcap runs the compiled classic-BPF program on
// every record, bpf_filter with the capture length as the buffer and the wire length for
// BPF_LEN) over a batch already in HBM: one lane per record runs the machine (pv_bpf.cpp's
// restatement; the program in LDS), the kept records are compacted into a new blob (sizes and
// record ranks by exclusive scans, one wave per 64 records copying each record with its 64 lanes)
// and the kept run's ts_sec change points found, so pv_process_device then takes the kept
// records as its batch.
struct PvBpfIns {
    uint16_t code;
    uint8_t jt, jf;
    uint32_t k;
};
#define PV_BPF_LDS 1024 // program instructions held in LDS (longer programs read the rest from HBM)
__device__ __forceinline__ bool bpf_ld(const uint8_t *p, uint32_t buflen, uint64_t k, uint32_t n, uint32_t &v)
{
    if (k + n > buflen) return false;
    v = 0;
    for (uint32_t i = 0; i < n; i++) v = (v << 8) | p[k + i];
    return true;
}
__device__ uint32_t bpf_run_dev(const PvBpfIns *lds, const PvBpfIns *prog, const uint8_t *p, uint32_t wirelen,
                                uint32_t buflen)
{
    uint32_t a = 0, x = 0, mem[16];
    for (int i = 0; i < 16; i++) mem[i] = 0;
    for (uint32_t pc = 0;; pc++) {
        const PvBpfIns f = pc < PV_BPF_LDS ? lds[pc] : prog[pc];
        const uint16_t c = f.code;
        uint32_t v;
        switch (c & 7) {
        case 0: { // LD
            const uint16_t mode = c & 0xe0;
            const uint32_t n = (c & 0x18) == 0 ? 4 : (c & 0x18) == 8 ? 2 : 1;
            if (mode == 0x00) a = f.k;
            else if (mode == 0x80) a = wirelen;
            else if (mode == 0x60) a = mem[f.k & 15];
            else {
                if (!bpf_ld(p, buflen, (mode == 0x40 ? (uint64_t)x : 0) + f.k, n, v)) return 0;
                a = v;
            }
            break;
        }
        case 1: { // LDX
            const uint16_t mode = c & 0xe0;
            if (mode == 0x00) x = f.k;
            else if (mode == 0x80) x = wirelen;
            else if (mode == 0x60) x = mem[f.k & 15];
            else {
                if (!bpf_ld(p, buflen, f.k, 1, v)) return 0;
                x = (v & 0xf) << 2;
            }
            break;
        }
        case 2: mem[f.k & 15] = a; break;
        case 3: mem[f.k & 15] = x; break;
        case 4: { // ALU
            const uint32_t s = (c & 8) ? x : f.k;
            switch (c & 0xf0) {
            case 0x00: a += s; break;
            case 0x10: a -= s; break;
            case 0x20: a *= s; break;
            case 0x30: if (!s) return 0; a /= s; break;
            case 0x90: if (!s) return 0; a %= s; break;
            case 0x40: a |= s; break;
            case 0x50: a &= s; break;
            case 0xa0: a ^= s; break;
            case 0x60: a <<= (s & 31); break;
            case 0x70: a >>= (s & 31); break;
            case 0x80: a = 0u - a; break;
            }
            break;
        }
        case 5: { // JMP
            const uint16_t op = c & 0xf0;
            if (op == 0x00) { pc += f.k; break; }
            const uint32_t s = (c & 8) ? x : f.k;
            const bool t = op == 0x10 ? a == s : op == 0x20 ? a > s : op == 0x30 ? a >= s : (a & s) != 0;
            pc += t ? f.jt : f.jf;
            break;
        }
        case 6: return (c & 0x18) == 0x10 ? a : f.k; // RET
        default: if ((c & 0xf8) == 0x80) a = x; else x = a; break; // MISC: TXA / TAX
        }
    }
}
__device__ __forceinline__ uint32_t rec_u32(const uint8_t *r, uint64_t p)
{
    return (uint32_t)r[p] | ((uint32_t)r[p + 1] << 8) | ((uint32_t)r[p + 2] << 16) | ((uint32_t)r[p + 3] << 24);
}
// sz[i]: 16 + caplen of a kept record, else 0; kf[i]: 1 if kept
extern "C" __global__ void __launch_bounds__(256) pv_bpf_keep(const uint8_t *__restrict__ recs, const uint32_t *__restrict__ offs, uint32_t n,
                                                              const PvBpfIns *__restrict__ prog, uint32_t ninsn, uint32_t *__restrict__ sz,
                                                              uint32_t *__restrict__ kf)
{
    __shared__ PvBpfIns lp[PV_BPF_LDS];
    for (uint32_t j = threadIdx.x; j < min(ninsn, (uint32_t)PV_BPF_LDS); j += blockDim.x) lp[j] = prog[j];
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = offs[i];
    const uint32_t cap = rec_u32(recs, o + 8), len = rec_u32(recs, o + 12);
    const bool keep = bpf_run_dev(lp, prog, recs + o + 16, len, cap) != 0;
    sz[i] = keep ? 16 + cap : 0;
    kf[i] = keep ? 1u : 0u;
}
// kept record i to out at boff[i], its offset to ooffs[rank[i]]: one wave per 64 records
extern "C" __global__ void __launch_bounds__(256) pv_bpf_gather(const uint8_t *__restrict__ recs, const uint32_t *__restrict__ offs, uint32_t n,
                                                                const uint32_t *__restrict__ sz, const uint32_t *__restrict__ boff,
                                                                const uint32_t *__restrict__ rank, uint8_t *__restrict__ out,
                                                                uint32_t *__restrict__ ooffs)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u;
    const uint32_t mi = w0 + lane;
    const uint32_t my_sz = mi < n ? sz[mi] : 0u, my_off = mi < n ? offs[mi] : 0u, my_b = mi < n ? boff[mi] : 0u;
    if (my_sz) ooffs[rank[mi]] = my_b;
    for (uint32_t r = 0; r < 64 && w0 + r < n; r++) {
        const uint32_t s = __shfl(my_sz, r, 64);
        if (!s) continue;
        const uint32_t so = __shfl(my_off, r, 64), d = __shfl(my_b, r, 64);
        for (uint32_t b = lane; b < s; b += 64) out[(uint64_t)d + b] = recs[(uint64_t)so + b];
    }
}
// ts_sec change points of the kept run: flag[j] = 1 where record j's second differs from j - 1's
// (record 0 always); sec[j] its second; down[0] counts decreases (non-monotone)
extern "C" __global__ void __launch_bounds__(256) pv_bpf_secs(const uint8_t *__restrict__ out, const uint32_t *__restrict__ ooffs, uint32_t nk,
                                                              uint32_t *__restrict__ flag, uint32_t *__restrict__ sec, uint32_t *__restrict__ down)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nk) return;
    const uint32_t s = rec_u32(out, ooffs[j]);
    const uint32_t p = j ? rec_u32(out, ooffs[j - 1]) : 0u;
    flag[j] = (j == 0 || s != p) ? 1u : 0u;
    sec[j] = s;
    if (j && s < p) atomicAdd(down, 1u);
}
// the change points, compacted by the flags' exclusive scan
extern "C" __global__ void __launch_bounds__(256) pv_bpf_secs_compact(const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                                                                      const uint32_t *__restrict__ sec, uint32_t nk, uint32_t cap,
                                                                      uint32_t *__restrict__ sci, uint32_t *__restrict__ scs)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nk || !flag[j] || pos[j] >= cap) return;
    sci[pos[j]] = j;
    scs[pos[j]] = sec[j];
}
// Exclusive prefix sum of n u32 (rocPRIM), tmp sized by a first call with tmp == nullptr.
extern "C" hipError_t pv_exclusive_scan_u32(void *tmp, size_t *tmp_bytes, const uint32_t *in, uint32_t *out, size_t n, hipStream_t s)
{
    return rocprim::exclusive_scan(tmp, *tmp_bytes, in, out, 0u, n, rocprim::plus<uint32_t>(), s);
}
