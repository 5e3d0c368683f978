// SPDX-License-Identifier: MPL-2.0
// pv_parse.h — per-packet parse, DNS decode and hashing logic of the hot path.
//
// Included by pv_kernels.hip (device code) and by the CPU test harness
// tests/native/parse_harness.cpp, which fuzzes this exact source against the
// oracle. The includer defines:
//   PV_FN                      function qualifiers (__device__ __forceinline__ / inline)
//   pv_clz64(x)                count leading zeros of a non-zero u64
//   pv_alignbyte(hi, lo, s)    bytes s..s+3 of the little-endian pair (lo, hi), s < 4
// Byte access goes through an accessor object A with
//   A.u32(off)  little-endian u32 at any absolute byte offset of the record blob
//   A.u32a(off) the same at a 4-aligned offset (one LDS / memory word)
//   A.u8(off)   one byte
// (the kernel uses an LDS window over each record's first bytes, falling back to
// HBM; the CPU harness reads plain memory).
#pragma once
#include <stdint.h>

#include "pv_layout.h"

template <class A>
PV_FN uint32_t be16(const A &R, uint64_t off)
{
    uint32_t w = R.u32(off);
    return ((w & 0xff) << 8) | ((w >> 8) & 0xff);
}

// ------------------------------------------------------------------ hashing
PV_FN uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
PV_FN uint64_t fmix64(uint64_t k)
{
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}
#define MM_C1 0x87c37b91114253d5ULL
#define MM_C2 0x4cf5ad432745937fULL

// Streaming MurmurHash3_x64_128 (seed 9001, datasketches DEFAULT_SEED).
struct Murmur {
    uint64_t h1, h2, k1, k2;
    uint32_t n;
    PV_FN void init() { h1 = h2 = 9001; k1 = k2 = 0; n = 0; }
    PV_FN void block()
    {
        k1 *= MM_C1; k1 = rotl64(k1, 31); k1 *= MM_C2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= MM_C2; k2 = rotl64(k2, 33); k2 *= MM_C1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
        k1 = k2 = 0;
    }
    PV_FN void put(uint32_t c)
    {
        uint32_t j = n & 15;
        if (j < 8) k1 |= (uint64_t)c << (8 * j);
        else k2 |= (uint64_t)c << (8 * (j - 8));
        n++;
        if ((n & 15) == 0) block();
    }
    PV_FN void finish(uint64_t &o1, uint64_t &o2)
    {
        uint32_t r = n & 15;
        if (r > 8) { k2 *= MM_C2; k2 = rotl64(k2, 33); k2 *= MM_C1; h2 ^= k2; }
        if (r > 0) { k1 *= MM_C1; k1 = rotl64(k1, 31); k1 *= MM_C2; h1 ^= k1; }
        h1 ^= n; h2 ^= n;
        h1 += h2; h2 += h1;
        h1 = fmix64(h1); h2 = fmix64(h2);
        h1 += h2; h2 += h1;
        o1 = h1; o2 = h2;
    }
};

// Fixed-length murmur for 8 and 16 byte items (one/one-and-a-half blocks).
PV_FN void murmur_8(uint64_t v, uint64_t &o1, uint64_t &o2)
{
    uint64_t h1 = 9001, h2 = 9001, k1 = v;
    k1 *= MM_C1; k1 = rotl64(k1, 31); k1 *= MM_C2; h1 ^= k1;
    h1 ^= 8; h2 ^= 8;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    o1 = h1; o2 = h2;
}
PV_FN void murmur_16(uint64_t a, uint64_t b, uint64_t &o1, uint64_t &o2)
{
    uint64_t h1 = 9001, h2 = 9001, k1 = a, k2 = b;
    k1 *= MM_C1; k1 = rotl64(k1, 31); k1 *= MM_C2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= MM_C2; k2 = rotl64(k2, 33); k2 *= MM_C1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    h1 ^= 16; h2 ^= 16;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    o1 = h1; o2 = h2;
}

// CPC coupon index from the two hash halves (cpc_sketch_impl.hpp:175-185), lg_k = 11.
PV_FN uint32_t cpc_coupon(uint64_t h1, uint64_t h2)
{
    uint32_t col = h2 ? pv_clz64(h2) : 63;
    if (col > 63) col = 63;
    uint32_t row = (uint32_t)(h1 & 2047);
    return (row << 6) | col;
}

// Name fingerprint state: two polynomial string hashes over Z/2^32 with odd bases, packed
// as lo | hi << 32. Prefix hashes give suffix hashes by H(s[i:n]) = H(s[:n]) - H(s[:i]) *
// B^(n-i) in each lane. Names are <= 255 chars. The bases are primes below 2^8, so B, B^2 and
// B^3 fit 24 bits: a dword of four characters costs one quarter-rate multiply per lane (h * B^4)
// and three full-rate 24-bit multiply-adds (v_mad_u32_u24) for its characters, where 32-bit
// bases cost four quarter-rate multiplies per lane (C3 DNS pass). Distinct
// strings of up to four characters never collide in both lanes (the difference polynomial
// would need both bases as roots with coefficients below 2^8); longer ones wrap mod 2^32 in
// each lane, and fp56 mixes the 64 bits with the length.
#define PB1 251u
#define PB2 239u
PV_FN uint64_t ph_step(uint64_t h, uint32_t c)
{
    const uint32_t lo = (uint32_t)h * PB1 + (c + 1), hi = (uint32_t)(h >> 32) * PB2 + (c + 1);
    return ((uint64_t)hi << 32) | lo;
}
// four ph_steps over the bytes of x (low byte first), in one Horner step per lane:
// h * B^4 + (c0+1) B^3 + (c1+1) B^2 + (c2+1) B + (c3+1)  (mod 2^32 per lane)
#define PB1_2 (PB1 * PB1)
#define PB1_3 (PB1_2 * PB1)
#define PB1_4 (PB1_2 * PB1_2)
#define PB2_2 (PB2 * PB2)
#define PB2_3 (PB2_2 * PB2)
#define PB2_4 (PB2_2 * PB2_2)
static_assert(PB1_3 < (1u << 24) && PB2_3 < (1u << 24), "24-bit multiply-adds");
PV_FN uint64_t ph_step4(uint64_t h, uint32_t x)
{
    // (c + 1) B^k = c B^k + B^k: the ones folded into one constant per lane
    const uint32_t c0 = x & 0xff, c1 = (x >> 8) & 0xff, c2 = (x >> 16) & 0xff, c3 = x >> 24;
    const uint32_t lo = (uint32_t)h * PB1_4 + c0 * PB1_3 + c1 * PB1_2 + c2 * PB1 + c3 + (PB1_3 + PB1_2 + PB1 + 1u);
    const uint32_t hi = (uint32_t)(h >> 32) * PB2_4 + c0 * PB2_3 + c1 * PB2_2 + c2 * PB2 + c3 + (PB2_3 + PB2_2 + PB2 + 1u);
    return ((uint64_t)hi << 32) | lo;
}
PV_FN uint64_t powb(uint32_t e) // (PB1^e, PB2^e)
{
    uint32_t r1 = 1, r2 = 1, b1 = PB1, b2 = PB2;
    while (e) {
        if (e & 1) { r1 *= b1; r2 *= b2; }
        b1 *= b1; b2 *= b2;
        e >>= 1;
    }
    return ((uint64_t)r2 << 32) | r1;
}
// a - b * p, lane by lane
PV_FN uint64_t ph_submul(uint64_t a, uint64_t b, uint64_t p)
{
    const uint32_t lo = (uint32_t)a - (uint32_t)b * (uint32_t)p;
    const uint32_t hi = (uint32_t)(a >> 32) - (uint32_t)(b >> 32) * (uint32_t)(p >> 32);
    return ((uint64_t)hi << 32) | lo;
}
// 56-bit fingerprint of a byte string from its polynomial hash and length
PV_FN uint64_t fp56(uint64_t poly, uint32_t len, uint32_t salt)
{
    return fmix64(poly ^ ((uint64_t)len << 48) ^ ((uint64_t)salt << 40) ^ 0x9e3779b97f4a7c15ULL) & 0x00ffffffffffffffULL;
}
PV_FN uint32_t hash32(uint64_t k) { return (uint32_t)(fmix64(k) >> 17); }
// transaction sort key: a 24-bit hash of the (flow, txid) key above the 32-bit stream rank, so
// the radix sort covers bits [0, 56): seven 8-bit passes instead of eight (the pairing compares
// the keys themselves inside a hash group, so a narrower hash only lengthens a few groups)
#define PV_XHASH_BITS 24
PV_FN uint64_t xact_sort_key(uint64_t key, uint32_t rank) { return ((fmix64(key) >> (64 - PV_XHASH_BITS)) << 32) | rank; }

// ------------------------------------------------------------------ packet parse
struct Parsed {
    uint32_t caplen;
    int64_t sec;
    int32_t nsec;
    uint64_t frame;    // absolute offset of frame byte 0
    uint8_t l3, l4;    // 0/4/6, 0/6/17
    uint8_t has4, has6;
    uint8_t syn, dir;
    uint64_t v4;       // absolute offset of first IPv4 header
    uint64_t v6;       // absolute offset of first IPv6 header
    uint64_t l4off;    // absolute offset of the TCP/UDP header
    uint32_t l4len;    // IP-length-trimmed L4 layer length
};

// Parse configuration: the link type and the first two IPv4 host subnets held in
// registers (the kernels build it once per thread); further subnets and IPv6 subnets
// are read from the parameter block. A /0 subnet has mask 0, so the mask test alone
// reproduces the reference's match-all rule.
struct ParseCfg {
    uint32_t linktype, ts_nano, n4;
    uint32_t a0, m0, a1, m1;
};
PV_FN ParseCfg parse_cfg(PV_CREF(PvParams) P)
{
    ParseCfg c;
    c.linktype = P.linktype;
    c.ts_nano = P.ts_nano;
    c.n4 = P.nets.n4;
    c.a0 = P.nets.v4_addr[0]; c.m0 = c.n4 > 0 ? P.nets.v4_mask[0] : 0xffffffffu;
    c.a1 = P.nets.v4_addr[1]; c.m1 = c.n4 > 1 ? P.nets.v4_mask[1] : 0xffffffffu;
    return c;
}
PV_FN bool match4(const ParseCfg &c, PV_CREF(PvSubnets) s, uint32_t ip)
{
    if (!ip) return false;
    if (c.n4 > 0 && ((ip ^ c.a0) & c.m0) == 0) return true;
    if (c.n4 > 1 && ((ip ^ c.a1) & c.m1) == 0) return true;
    for (uint32_t i = 2; i < c.n4; i++)
        if (s.v4_all[i] || ((ip ^ s.v4_addr[i]) & s.v4_mask[i]) == 0) return true;
    return false;
}
template <class A>
PV_FN bool match6(PV_CREF(PvSubnets) s, const A &R, uint64_t a)
{
    for (uint32_t i = 0; i < s.n6; i++) {
        uint32_t cidr = s.v6_cidr[i], bytes = cidr / 8, bits = cidr % 8;
        bool r = false;
        if (bytes > 0) {
            r = true;
            for (uint32_t b = 0; b < bytes; b++)
                if (R.u8(a + b) != s.v6_addr[i][b]) { r = false; break; }
        }
        if ((r || cidr < 8) && bits > 0) r = (s.v6_addr[i][bytes] >> (8 - bits)) == (R.u8(a + bytes) >> (8 - bits));
        if (r) return true;
    }
    return false;
}

template <class A>
PV_FN void parse_dir(const A &R, const ParseCfg &C, PV_CREF(PvParams) P, Parsed &o);

template <class A>
PV_FN void parse_record(const A &R, const ParseCfg &C, PV_CREF(PvParams) P, uint64_t rec, Parsed &o)
{
    uint32_t tsec = R.u32(rec), tfrac = R.u32(rec + 4);
    o.caplen = R.u32(rec + 8);
    o.sec = tsec;
    o.nsec = C.ts_nano ? (int32_t)tfrac : (int32_t)(tfrac * 1000u);
    o.frame = rec + 16;
    o.l3 = o.l4 = 0; o.has4 = o.has6 = 0; o.syn = 0; o.dir = 2;
    o.v4 = o.v6 = o.l4off = 0; o.l4len = 0;
    // fast path: Ethernet II + IPv4 without options (the overwhelmingly common frame);
    // identical results to the general walk below, which handles everything else
    if (C.linktype == 1 && o.caplen >= 34) {
        const uint32_t w3 = R.u32(o.frame + 12); // ethertype, version/IHL
        if ((w3 & 0xffffffu) == 0x450008u) {
            const uint32_t w4 = R.u32(o.frame + 16), w5 = R.u32(o.frame + 20);
            const uint32_t proto = w5 >> 24;
            if (proto != 4 && proto != 41) {
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
                        o.syn = (R.u8(pl + 13) & 2) ? 1 : 0;
                    }
                }
                if (match4(C, P.nets, R.u32(o.frame + 30))) o.dir = 0;
                else if (match4(C, P.nets, R.u32(o.frame + 26))) o.dir = 1;
                return;
            }
        }
    }
    uint64_t cur = o.frame;
    uint32_t len = o.caplen;
    uint32_t kind = 0; // 4 or 6 once an IP header is located
    uint32_t et = 0;
    bool l2ok = false;
    if (C.linktype == 1) {
        if (len >= 14) {
            et = be16(R, cur + 12);
            if (et >= 0x600 && len > 14) { cur += 14; len -= 14; l2ok = true; }
        }
    } else if (C.linktype == 113) {
        if (len > 16) { et = be16(R, cur + 14); cur += 16; len -= 16; l2ok = true; }
    } else if (C.linktype == 101 || C.linktype == 12 || C.linktype == 14 || C.linktype == 228 || C.linktype == 229) {
        if (len >= 1) { uint32_t v = R.u8(cur) >> 4; kind = (v == 4 || v == 6) ? v : 0; }
    }
    if (l2ok) {
        for (int d = 0; d < 8 && (et == 0x8100 || et == 0x88A8); d++) {
            if (len <= 4) { et = 0; break; }
            et = be16(R, cur + 2);
            cur += 4; len -= 4;
        }
        kind = et == 0x0800 ? 4 : (et == 0x86DD ? 6 : 0);
    }
    for (int depth = 0; depth < 4 && kind; depth++) {
        uint32_t proto, hl;
        if (kind == 4) {
            uint32_t b0 = R.u8(cur);
            if (!(len >= 20 && (b0 >> 4) == 4 && (b0 & 15) >= 5)) break;
            if (!o.has4) { o.has4 = 1; o.v4 = cur; }
            uint32_t total = be16(R, cur + 2);
            if (total < len && total != 0) len = total;
            hl = (b0 & 15) * 4;
            if (len <= hl) break;
            uint32_t frag = be16(R, cur + 6);
            if ((frag & 0x2000) || (frag & 0x1fff)) break;
            proto = R.u8(cur + 9);
        } else {
            if (len < 40) break;
            if (!o.has6) { o.has6 = 1; o.v6 = cur; }
            uint32_t next = R.u8(cur + 6);
            uint32_t off = 40;
            bool frag = false;
            for (int e = 0; e < 8 && len >= 2 && off <= len - 2; e++) {
                uint32_t elen;
                if (next == 44) elen = 8;
                else if (next == 0 || next == 60 || next == 43) elen = (R.u8(cur + off + 1) + 1) * 8;
                else if (next == 51) elen = (R.u8(cur + off + 1) + 2) * 4;
                else break;
                frag = next == 44;
                next = R.u8(cur + off);
                off += elen;
            }
            uint32_t total = be16(R, cur + 4) + off;
            if (total < len) len = total;
            hl = off;
            if (len <= hl || frag) break;
            proto = next;
        }
        uint64_t pl = cur + hl;
        uint32_t pll = len - hl;
        if (proto == 17) {
            if (pll >= 8) { o.l4 = 17; o.l4off = pl; o.l4len = pll; }
            break;
        }
        if (proto == 6) {
            if (pll >= 20) { o.l4 = 6; o.l4off = pl; o.l4len = pll; o.syn = (R.u8(pl + 13) & 2) ? 1 : 0; }
            break;
        }
        if ((proto == 4 || proto == 41) && pll >= 1) {
            uint32_t v = R.u8(pl) >> 4;
            kind = (v == 4 || v == 6) ? v : 0;
            cur = pl; len = pll;
            continue;
        }
        break;
    }
    o.l3 = o.has4 ? 4 : (o.has6 ? 6 : 0);
    parse_dir(R, C, P, o);
}
// direction (PcapInputStream.cpp:401-416) for the general walk
template <class A>
PV_FN void parse_dir(const A &R, const ParseCfg &C, PV_CREF(PvParams) P, Parsed &o)
{
    if (o.has4) {
        if (match4(C, P.nets, R.u32(o.v4 + 16))) o.dir = 0;
        else if (match4(C, P.nets, R.u32(o.v4 + 12))) o.dir = 1;
    } else if (o.has6) {
        if (match6(P.nets, R, o.v6 + 24)) o.dir = 0;
        else if (match6(P.nets, R, o.v6 + 8)) o.dir = 1;
    }
}

template <class A>
PV_FN void parse_record(const A &R, PV_CREF(PvParams) P, uint64_t rec, Parsed &o)
{
    parse_record(R, parse_cfg(P), P, rec, o);
}

// PcapPlusPlus hash5Tuple(packet, directionUnique=false): FNV-1 32-bit.
PV_FN uint32_t fnv_bytes(uint32_t h, uint32_t v, int n)
{
    for (int i = 0; i < n; i++) { h *= 0x01000193u; h ^= (v >> (8 * i)) & 0xff; }
    return h;
}
template <class A>
PV_FN uint32_t flowkey(const A &R, const Parsed &o)
{
    uint32_t pw = R.u32(o.l4off);
    uint32_t ps = pw & 0xffff, pd = pw >> 16; // raw network-order u16 read little-endian
    int sp = pd < ps ? 1 : 0;
    uint32_t h = 0x811C9DC5u;
    uint32_t p0 = sp ? pd : ps, p1 = sp ? ps : pd;
    h = fnv_bytes(h, p0, 2);
    h = fnv_bytes(h, p1, 2);
    if (o.has4) {
        uint32_t s = R.u32(o.v4 + 12), d = R.u32(o.v4 + 16);
        if (ps == pd && d < s) sp = 1;
        uint32_t a = sp ? d : s, b = sp ? s : d;
        h = fnv_bytes(h, a, 4);
        h = fnv_bytes(h, b, 4);
        h = fnv_bytes(h, R.u8(o.v4 + 9), 1);
    } else {
        uint64_t a = sp ? o.v6 + 24 : o.v6 + 8, b = sp ? o.v6 + 8 : o.v6 + 24;
        for (int i = 0; i < 16; i += 4) h = fnv_bytes(h, R.u32(a + i), 4);
        for (int i = 0; i < 16; i += 4) h = fnv_bytes(h, R.u32(b + i), 4);
        h = fnv_bytes(h, R.u8(o.v6 + 6), 1);
    }
    return h;
}

// ------------------------------------------------------------------ DNS name decode
// Level-1 structural walk of decodeName: returns m_NameLength (encoded length)
// and whether the name text is forced empty (illegal top-level pointer => 0).
template <class A>
PV_FN uint32_t name_len_l1(const A &R, uint64_t m, uint32_t len, uint32_t off)
{
    uint32_t enc = 0, cur = off;
    if (cur + 1 > len) return 0;
    uint32_t wl = R.u8(m + cur);
    while (wl != 0) {
        if ((wl & 0xc0) == 0xc0) {
            if (cur + 2 > len || enc > 255) return enc;
            uint32_t ptr = ((wl & 0x3f) << 8) | R.u8(m + cur + 1);
            if (ptr < 12 || ptr >= len) return 0;
            return enc + 2;
        }
        if (cur + wl + 1 > len || enc + wl > 255) return enc == 256 ? enc : enc + 1;
        cur += wl + 1;
        enc += wl + 1;
        if (cur + 1 > len) return enc == 256 ? enc : enc + 1;
        wl = R.u8(m + cur);
    }
    return enc + 1;
}

// Iterative decodeName producing the characters of the final std::string
// (NUL-truncated, per-level 255-char copy limits, trailing-dot rules).
// E::put(c) receives each character; returns false when the name is empty.
template <class A, class E>
PV_FN void name_emit(const A &R, uint64_t m, uint32_t len, uint32_t off, E &e)
{
    uint32_t cur = off, enc = 0, dec = 0, level = 1;
    int budget = 1 << 30; // chars that can still travel up to the top-level buffer
    bool pending = false, stop = false;
    auto emit = [&](uint32_t c) {
        if (stop) return;
        if (c == 0) { stop = true; return; }
        if (level >= 2) {
            if (budget <= 0) { stop = true; return; }
            budget--;
        }
        e.put(c);
    };
    if (cur + 1 > len) return;
    uint32_t wl = R.u8(m + cur);
    for (int guard = 0; guard < 4096 && !stop; guard++) {
        if (wl == 0) return; // normal termination: trailing '.' dropped
        if ((wl & 0xc0) == 0xc0) {
            if (cur + 2 > len || enc > 255) { if (pending) emit('.'); return; }
            uint32_t ptr = ((wl & 0x3f) << 8) | R.u8(m + cur + 1);
            if (ptr < 12 || ptr >= len) { if (level >= 2 && pending) emit('.'); return; }
            if (pending) { emit('.'); pending = false; }
            int cap = 255 - (int)dec;
            if (level >= 2 && budget < cap) cap = budget;
            budget = cap;
            level++;
            if (level > 20) return; // decodeName(iteration > 20) returns an empty string
            cur = ptr; enc = 0; dec = 0;
            wl = R.u8(m + cur);
            continue;
        }
        if (cur + wl + 1 > len || enc + wl > 255) { if (enc != 256 && pending) emit('.'); return; }
        if (pending) emit('.');
        for (uint32_t i = 0; i < wl && !stop; i++) emit(R.u8(m + cur + 1 + i));
        pending = true;
        dec += wl + 1;
        cur += wl + 1;
        enc += wl + 1;
        if (cur + 1 > len) { if (enc != 256 && pending) emit('.'); return; }
        wl = R.u8(m + cur);
    }
}

PV_FN uint32_t lower(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

// Per-packet name statistics: murmur for CPC, length, the last four dots with the
// prefix hash in front of each (newest first, registers only), full prefix hash.
struct NameStats {
    Murmur mm;
    uint64_t ph;                     // polynomial prefix hash of the chars so far
    uint32_t n;                      // chars so far
    int32_t d0, d1, d2, d3;          // positions of the last dots, newest first (-1 = none)
    uint64_t h0, h1, h2, h3;         // prefix hash before each of those dots
    uint32_t last_c;
    PV_FN void init()
    {
        mm.init(); ph = 0; n = 0; last_c = 0;
        d0 = d1 = d2 = d3 = -1; h0 = h1 = h2 = h3 = 0;
    }
    PV_FN void put(uint32_t c)
    {
        c = lower(c);
        if (c == '.') { d3 = d2; h3 = h2; d2 = d1; h2 = h1; d1 = d0; h1 = h0; d0 = (int32_t)n; h0 = ph; }
        mm.put(c);
        ph = ph_step(ph, c);
        n++;
        last_c = c;
    }
    // last dot at position <= lim among the tracked ones (std::string::rfind), -1 if none
    PV_FN int rfind(int lim, uint64_t &pph) const
    {
        if (d0 >= 0 && d0 <= lim) { pph = h0; return d0; }
        if (d1 >= 0 && d1 <= lim) { pph = h1; return d1; }
        if (d2 >= 0 && d2 <= lim) { pph = h2; return d2; }
        if (d3 >= 0 && d3 <= lim) { pph = h3; return d3; }
        return -1;
    }
};

// aggregateDomain(name, 0): suffix start positions for qname2 / qname3 (-1 = empty)
// (suffix_size > 0: aggregateDomain(name, suffix_size), libs/visor_dns/dns.cpp:19-23)
PV_FN void agg_domain(const NameStats &s, int &q2, int &q3, uint64_t &ph2, uint64_t &ph3, uint32_t suffix_size = 0)
{
    int n = (int)s.n;
    q2 = 0; q3 = 0; ph2 = 0; ph3 = 0;
    if (n < 5) { q3 = -1; return; }
    int endDot = 1 << 30;
    if (suffix_size > 0 && (uint32_t)n > suffix_size) endDot = n - (int)suffix_size;
    else if (s.last_c == '.') endDot = n - 2;
    uint64_t x1;
    int first = s.rfind(endDot, x1);
    if (first > 0) {
        uint64_t x2;
        int second = s.rfind(first - 1, x2);
        if (second >= 0) {
            q2 = second; ph2 = x2;
            if (second > 0) {
                uint64_t x3;
                int third = s.rfind(second - 1, x3);
                if (third >= 0) { q3 = third; ph3 = x3; }
            }
        } else {
            q3 = -1;
        }
    }
}
// polynomial hash of the suffix [start, n) given the prefix hash at start
PV_FN uint64_t suffix_hash(const NameStats &s, int start, uint64_t ph_start)
{
    return ph_submul(s.ph, ph_start, powb(s.n - (uint32_t)start));
}

// The dots of a name at positions <= lim, newest first, with the prefix hash in front of
// each. aggregateDomain's rfinds (libs/visor_dns/dns.cpp:20-36) never look past endDot, so
// these are the only dots it can use; NameStats keeps the last four dots of the whole name,
// which is too few once a suffix (only_qname_suffix, public_suffix_list) covers two of them.
struct DotsUpTo {
    uint64_t ph = 0;
    uint32_t n = 0;
    int32_t lim;
    int32_t d0 = -1, d1 = -1, d2 = -1;
    uint64_t h0 = 0, h1 = 0, h2 = 0;
    PV_FN void put(uint32_t c)
    {
        c = lower(c);
        if (c == '.' && (int32_t)n <= lim) { d2 = d1; h2 = h1; d1 = d0; h1 = h0; d0 = (int32_t)n; h0 = ph; }
        ph = ph_step(ph, c);
        n++;
    }
};
#ifndef PV_OOL
#if defined(__HIP__)
#define PV_OOL __host__ __device__ __noinline__
#else
#define PV_OOL __attribute__((noinline))
#endif
#endif
struct DotsOut {
    int32_t d0, d1, d2;
    uint64_t h0, h1, h2;
};
// out of line with by-value arguments and result, so the DNS pass keeps no stack frame for it
template <class A>
PV_OOL DotsOut dots_up_to(A R, uint64_t m, uint32_t len, int32_t lim)
{
    DotsUpTo d;
    d.lim = lim;
    name_emit(R, m, len, 12, d);
    return DotsOut{d.d0, d.d1, d.d2, d.h0, d.h1, d.h2};
}
// agg_domain with any suffix size: when two or more of the tracked dots lie past endDot, the
// name is walked again for the dots at or before it (rare: long suffixes on many-label names)
template <class A>
PV_FN void agg_domain_r(const A &R, uint64_t m, uint32_t len, const NameStats &s, int &q2, int &q3, uint64_t &ph2,
                        uint64_t &ph3, uint32_t suffix_size)
{
    agg_domain(s, q2, q3, ph2, ph3, suffix_size);
    if (suffix_size > 0 && s.n > suffix_size && s.d3 >= 0 && s.d1 > (int)(s.n - suffix_size)) {
        const DotsOut d = dots_up_to(R, m, len, (int32_t)(s.n - suffix_size));
        NameStats t = s;
        t.d0 = d.d0; t.h0 = d.h0; t.d1 = d.d1; t.h1 = d.h1; t.d2 = d.d2; t.h2 = d.h2; t.d3 = -1; t.h3 = 0;
        agg_domain(t, q2, q3, ph2, ph3, suffix_size);
    }
}
// the lower-case name into a buffer (public_suffix_list)
struct BufEmit {
    uint8_t *d;
    uint32_t n, cap;
    PV_FN void put(uint32_t c)
    {
        if (n < cap) d[n] = (uint8_t)lower(c);
        n++;
    }
};

// ------------------------------------------------------------------ name fast path
// A level-1 name made of plain labels (lengths 1..63, no pointer, no NUL and no '.'
// byte inside a label, at most 8 inner dots, terminated inside the message within the
// 255-byte limit) decodes, under name_emit's rules, to the wire bytes
// [off + 1, off + 1 + n) with each inner length byte read as '.'. name_stats_fast
// computes NameStats of that text four bytes at a time (SWAR lower-casing, dot
// substitution from the label walk, murmur over 16-byte blocks, prefix hashes at the
// last four dots taken from the running Horner values); it returns false, st untouched,
// for every other name.
PV_FN uint32_t lower4(uint32_t w)
{
    const uint32_t t = w & 0x7f7f7f7fu;
    const uint32_t up = (t + 0x3f3f3f3fu) & ~(t + 0x25252525u) & ~w & 0x80808080u; // 'A' <= byte <= 'Z'
    return w | (up >> 2);
}
PV_FN uint32_t nonzero4(uint32_t w) { return (((w & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w) & 0x80808080u; }
PV_FN uint32_t nibble_bytes(uint32_t x) { return ((x * 0x00204081u) & 0x01010101u) * 0xffu; }

template <class A>
PV_FN bool name_stats_fast(const A &R, uint64_t m, uint32_t len, uint32_t off, NameStats &st)
{
    // label walk: inner dot positions of the decoded text, newest in the low byte (0xff = none)
    uint32_t cur = off, enc = 0, nb = 0;
    uint64_t bp = ~0ull;
    if (cur + 1 > len) return false;
    uint32_t wl = R.u8(m + cur);
    while (wl != 0) {
        if (wl > 63 || cur + wl + 1 > len || enc + wl > 255) return false;
        if (enc) {
            if (nb == 8) return false;
            bp = (bp << 8) | (enc - 1);
            nb++;
        }
        cur += wl + 1;
        enc += wl + 1;
        if (cur + 1 > len) return false;
        wl = R.u8(m + cur);
    }
    const uint32_t n = enc ? enc - 1 : 0;
    uint32_t t[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t b = (uint32_t)(bp >> (8 * k)) & 0xff;
        t[k] = b == 0xff ? 0xffffffffu : b;
    }
    Murmur mm;
    mm.init();
    uint64_t ph = 0, hk[4] = {0, 0, 0, 0};
    const uint64_t src = m + off + 1;
    const uint64_t abase = src & ~3ull;
    const uint32_t sh = (uint32_t)(src & 3);
    uint32_t prev = R.u32a(abase);
    bool bad = false;
    for (uint32_t j = 0; j * 16 < n; j++) {
        // inner dots inside this 16-byte block (none for a single-label name)
        uint32_t bm = 0;
        if (nb) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t rel = ((uint32_t)(bp >> (8 * k)) & 0xff) - 16 * j;
                bm |= rel < 16 ? 1u << rel : 0u;
            }
        }
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t p = 16 * j + 4 * q;
            const uint32_t nv = n > p + 4 ? 4u : n > p ? n - p : 0u;
            const uint32_t vm = nv >= 4 ? 0xffffffffu : (1u << (8 * nv)) - 1u;
            const uint32_t dm = nibble_bytes((bm >> (4 * q)) & 15);
            const uint32_t nxt = R.u32a(abase + p + 4);
            uint32_t x = lower4(pv_alignbyte(nxt, prev, sh));
            prev = nxt;
            const uint32_t ok = nonzero4(x) & nonzero4(x ^ 0x2e2e2e2eu);
            bad |= ((~ok & 0x80808080u) & vm & ~dm) != 0;
            x = ((x & ~dm) | (0x2e2e2e2eu & dm)) & vm;
            w[q] = x;
            // Horner over the valid bytes; a tracked dot takes the hash before its byte. A
            // whole dword without a tracked dot (the common case) is one ph_step4.
            const bool tracked = ((t[0] - p) < 4) | ((t[1] - p) < 4) | ((t[2] - p) < 4) | ((t[3] - p) < 4);
            if (nv == 4 && !tracked) {
                ph = ph_step4(ph, x);
            } else {
                uint64_t hv[4];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    hv[r] = ph;
                    if ((uint32_t)r < nv) ph = ph_step(ph, (x >> (8 * r)) & 0xff);
                }
                if (tracked) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t rel = t[k] - p;
                        if (rel < 4) hk[k] = rel == 0 ? hv[0] : rel == 1 ? hv[1] : rel == 2 ? hv[2] : hv[3];
                    }
                }
            }
        }
        mm.k1 = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
        mm.k2 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
#ifndef PV_NO_MM // tuning knob: no Murmur blocks (the qname CPC coupons are then wrong)
        if (16 * j + 16 <= n) mm.block();
#endif
    }
    if (bad) return false;
    mm.n = n;
    st.mm = mm;
    st.ph = ph;
    st.n = n;
    st.d0 = (int32_t)t[0]; st.d1 = (int32_t)t[1]; st.d2 = (int32_t)t[2]; st.d3 = (int32_t)t[3];
    st.h0 = hk[0]; st.h1 = hk[1]; st.h2 = hk[2]; st.h3 = hk[3];
    st.last_c = n ? lower(R.u8(src + n - 1)) : 0;
    return true;
}
// NameStats of the first query name (name_emit's result, by the fast path where it applies)
template <class A>
PV_FN void name_stats(const A &R, uint64_t m, uint32_t len, uint32_t off, NameStats &st)
{
    if (!name_stats_fast(R, m, len, off, st)) name_emit(R, m, len, off, st);
}

struct CountEmit {
    uint32_t n;
    PV_FN void put(uint32_t) { n++; }
};
struct CopyEmit {
    uint8_t *dst;
    uint32_t from, n;
    uint32_t raw; // 1: keep case (DnsQuery::getName), 0: lower case (getNameLower)
    PV_FN void put(uint32_t c)
    {
        if (n >= from) dst[n - from] = (uint8_t)(raw ? c : lower(c));
        n++;
    }
};
// case-preserving polynomial hash of a name (top_slow keys use getName())
struct RawName {
    uint64_t ph;
    uint32_t n;
    PV_FN void put(uint32_t c)
    {
        ph = ph_step(ph, c);
        n++;
    }
};

// prefix hash of the lower-case name at position tgt (only_qname_suffix: the hash of the
// last L chars is H(name) - H(name[:n-L]) * B^L)
struct SuffixCap {
    uint64_t ph, cap;
    uint32_t n, tgt;
    PV_FN void put(uint32_t c)
    {
        if (n == tgt) cap = ph;
        ph = ph_step(ph, lower(c));
        n++;
    }
};

// ------------------------------------------------------------------ DNS message
struct DnsInfo {
    bool ok;          // parseResources(queryOnly) succeeded
    bool has_query;
    uint32_t name_off; // offset of the first query name in the message
    uint32_t name_len_enc;
    uint32_t qtype;
};

// only_dnssec_response (dns/v1/DnsStreamHandler.cpp:573-595): parseResources(false, true,
// true) walks questions, answers, authorities and the first additional (DnsLayer.cpp:119-209);
// true if that walk stays in bounds and an answer has type RRSIG (46)
template <class A>
PV_FN bool dns_dnssec(const A &R, uint64_t m, uint32_t len, uint32_t qd, uint32_t an, uint32_t ns, uint32_t ar)
{
    const uint32_t total = qd + an + ns + ar;
    if (total > 100 || len < 12) return false;
    uint32_t off = 12;
    bool sig = false;
    for (uint32_t i = 0; i < total; i++) {
        const uint32_t nl = name_len_l1(R, m, len, off);
        const uint32_t start = off;
        if (i < qd) off += nl + 4;
        else {
            const uint32_t dl = (off + nl + 10 <= len) ? be16(R, m + off + nl + 8) : 0u;
            off += nl + 10 + dl;
        }
        if (off > len) return false;
        if (i >= qd && i < qd + an && be16(R, m + start + nl) == 46) sig = true;
        if (i >= qd + an + ns) break; // the first additional record ends the walk
    }
    return sig;
}

// Offset of the first additional record as DnsLayer::parseResources(false, true, true) reaches
// it (questions, answers, authorities, then the first additional, each in bounds;
// libs/visor_dns/DnsLayer.cpp:119-209), 0 if none
template <class A>
PV_FN uint32_t dns_first_additional(const A &R, uint64_t m, uint32_t len, uint32_t qd, uint32_t an, uint32_t ns,
                                    uint32_t ar)
{
    const uint32_t total = qd + an + ns + ar;
    if (total > 100 || len < 12 || ar == 0) return 0;
    uint32_t off = 12;
    for (uint32_t i = 0; i < total; i++) {
        const uint32_t nl = name_len_l1(R, m, len, off);
        const uint32_t start = off;
        if (i < qd) off += nl + 4;
        else {
            const uint32_t dl = (off + nl + 10 <= len) ? be16(R, m + off + nl + 8) : 0u;
            off += nl + 10 + dl;
        }
        if (off > len) return 0;
        if (i == qd + an + ns) return start;
    }
    return 0;
}
// parse_additional_records_ecs (libs/visor_dns/DnsAdditionalRecord.h:49-101) on a query's
// first additional record: an OPT record whose data (>= 9 bytes) opens with option CSUBNET
// (8). Returns the family (1 IPv4, 2 IPv6; 0 = no ECS) and the address bytes the reference
// keeps, little-endian in lo | hi: IPv4 data bytes 8 .. 12 (it copies them all into a 4-byte
// array; bytes past 4 are not kept), IPv6 data bytes 8 .. min(len, 16).
template <class A>
PV_FN uint32_t dns_ecs(const A &R, uint64_t m, uint32_t len, uint32_t qd, uint32_t an, uint32_t ns, uint32_t ar,
                       uint64_t &addr)
{
    addr = 0;
    const uint32_t a = dns_first_additional(R, m, len, qd, an, ns, ar);
    if (!a) return 0;
    const uint32_t nl = name_len_l1(R, m, len, a);
    const uint32_t type = be16(R, m + a + nl), dlen = be16(R, m + a + nl + 8);
    if (type != 41 || dlen < 9) return 0;
    const uint64_t x = m + a + nl + 10;
    if (be16(R, x) != 8) return 0;
    const uint32_t family = be16(R, x + 4);
    const uint32_t lim = family == 1 ? (dlen < 12 ? dlen : 12u) : (family == 2 ? (dlen < 16 ? dlen : 16u) : 8u);
    for (uint32_t i = 8; i < lim; i++) addr |= (uint64_t)R.u8(x + i) << (8 * (i - 8));
    return family == 1 || family == 2 ? family : 0u;
}

template <class A>
PV_FN void dns_parse(const A &R, uint64_t m, uint32_t len, uint32_t qd, uint32_t an, uint32_t ns,
                          uint32_t ar, DnsInfo &d)
{
    d.ok = false; d.has_query = false; d.qtype = 0; d.name_off = 12; d.name_len_enc = 0;
    uint32_t total = qd + an + ns + ar;
    if (total > 100) return;
    if (total == 0) { d.ok = true; return; }
    if (len < 12) return;
    if (qd > 0) {
        uint32_t nl = name_len_l1(R, m, len, 12);
        if (12 + nl + 4 > len) return;
        d.ok = true; d.has_query = true; d.name_len_enc = nl;
        d.qtype = be16(R, m + 12 + nl);
        return;
    }
    uint32_t off = 12;
    for (uint32_t i = 0; i < total; i++) {
        uint32_t nl = name_len_l1(R, m, len, off);
        uint32_t dl = 0;
        if (off + nl + 10 <= len) dl = be16(R, m + off + nl + 8);
        off += nl + 10 + dl;
        if (off > len) return;
    }
    d.ok = true;
}

