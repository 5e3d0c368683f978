// tests/native/parse_harness.cpp — TEST ONLY: compiles the product's parse/decode
// source (pktvisor_amd/csrc/pv_parse.h, the code the HIP kernel runs) for the CPU
// so it can be fuzzed against the oracle without a GPU. Not a fallback: nothing in
// the product loads this library.
#include <cstring>
#include <stdint.h>

#define PV_FN inline
#define PV_CREF(T) const T &
inline uint32_t pv_clz64(uint64_t x) { return (uint32_t)__builtin_clzll(x); }
inline uint32_t pv_alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) { return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh)); }
#include "../../pktvisor_amd/csrc/pv_parse.h"

// plain-memory accessor (the kernel uses an LDS-window accessor with the same interface)
struct HAcc {
    const uint8_t *R;
    uint32_t u32(uint64_t off) const { uint32_t v; memcpy(&v, R + off, 4); return v; }
    uint32_t u32a(uint64_t off) const { return u32(off); }
    uint32_t u8(uint64_t off) const { return R[off]; }
};

extern "C" {

// first query name of a DNS message (buffer must be readable 8 bytes past len):
// returns m_NameLength, writes the raw name bytes (as the final std::string) to out
uint32_t h_decode_qname(const uint8_t *msg, uint32_t len, char *out, uint32_t *outlen)
{
    struct Coll {
        char *o;
        uint32_t n;
        void put(uint32_t c) { o[n++] = (char)c; }
    } col{out, 0};
    const HAcc R{msg};
    uint32_t nl = name_len_l1(R, 0, len, 12);
    if (nl > 0) name_emit(R, 0, len, 12, col);
    *outlen = col.n;
    return nl;
}

// parseResources(queryOnly) outcome: ok, has_query, qtype
void h_dns_parse(const uint8_t *msg, uint32_t len, int *ok, int *has_query, uint32_t *qtype)
{
    DnsInfo d;
    const HAcc R{msg};
    uint32_t qd = be16(R, 4), an = be16(R, 6), ns = be16(R, 8), ar = be16(R, 10);
    dns_parse(R, 0, len, qd, an, ns, ar, d);
    *ok = d.ok; *has_query = d.has_query; *qtype = d.qtype;
}

// lower-case name stats: length, murmur (CPC) halves, aggregateDomain suffix starts
void h_name_stats(const uint8_t *msg, uint32_t len, uint32_t *n, uint64_t *h1, uint64_t *h2, int *q2, int *q3)
{
    NameStats st;
    st.init();
    const HAcc R{msg};
    uint32_t nl = name_len_l1(R, 0, len, 12);
    if (nl > 0) name_emit(R, 0, len, 12, st);
    *n = st.n;
    st.mm.finish(*h1, *h2);
    uint64_t a, b;
    if (st.n) agg_domain(st, *q2, *q3, a, b); else { *q2 = 0; *q3 = -1; }
}
}

extern "C" {
// name_stats_fast against name_emit + NameStats on the same message:
// -1 = the fast path declined, 1 = every NameStats field equal, 0 = a field differs
int h_name_fast_check(const uint8_t *msg, uint32_t len)
{
    const HAcc R{msg};
    uint32_t nl = name_len_l1(R, 0, len, 12);
    if (nl == 0) return -1;
    NameStats a, b;
    a.init();
    b.init();
    if (!name_stats_fast(R, 0, len, 12, a)) return -1;
    name_emit(R, 0, len, 12, b);
    uint64_t a1, a2, b1, b2;
    a.mm.finish(a1, a2);
    b.mm.finish(b1, b2);
    return a1 == b1 && a2 == b2 && a.ph == b.ph && a.n == b.n && a.last_c == b.last_c && a.d0 == b.d0 &&
           a.d1 == b.d1 && a.d2 == b.d2 && a.d3 == b.d3 && a.h0 == b.h0 && a.h1 == b.h1 && a.h2 == b.h2 &&
           a.h3 == b.h3;
}
}
