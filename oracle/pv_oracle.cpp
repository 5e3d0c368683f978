// SPDX-License-Identifier: MPL-2.0
//
// oracle/pv_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// A single-threaded CPU restatement of pktvisor's per-packet hot path, written
// from the reference source as a specification (not copied):
//   * pcap record loop ............ src/inputs/pcap/PcapInputStream.cpp:471-527
//   * L2/L3/L4 classify + dir ..... src/inputs/pcap/PcapInputStream.cpp:380-428,
//                                   libs/visor_utils/utils.cpp:26-69,105-164
//   * hash5Tuple flowkey .......... PcapPlusPlus 23.09 PacketUtils (not vendored;
//                                   restated, parity unpinned)
//   * Net v1 bucket ............... src/handlers/net/v1/NetStreamHandler.cpp:161-169,
//                                   516-548,682-764
//   * DNS wire decoder ............ libs/visor_dns/DnsLayer.cpp:119-209,
//                                   libs/visor_dns/DnsResource.cpp:19-32,53-148
//   * DNS v1 bucket + xacts ....... src/handlers/dns/v1/DnsStreamHandler.cpp:270-302,
//                                   910-1049,1093-1138,1350-1370,
//                                   libs/visor_transaction/TransactionManager.h:24-117
//   * aggregateDomain ............. libs/visor_dns/dns.cpp:9-43
//   * window / period shift ....... src/AbstractMetricsManager.h:177-206,276-333,423-437,601-647
//   * sketches: CPC (HIP/ICON), exact top-N counts, exact quantiles with the
//     KLL rank rule — 3rd/datasketches/cpc/include/cpc_sketch_impl.hpp:75-385,
//     icon_estimator.hpp:225-270, common/include/quantiles_sorted_view_impl.hpp:76-84.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this code, and only as the checker / CPU baseline. The product path
// (pktvisor_amd, libpvgpu.so) never links or calls it.
//
// Parity status: pinned against the reference's own known-answer tests on the
// UDP fixtures (tests/golden/, see tests/test_oracle_kat.py) and, for the sketch
// estimators, against the vendored datasketches library compiled by
// oracle/Makefile into oracle/_ref/ (tests/test_ref_sketch.py).

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>
#include <arpa/inet.h>

namespace pvo {

// ---------------------------------------------------------------- utilities
static inline uint16_t rd16be(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t rd32le(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

struct TS {
    int64_t sec = 0;
    int64_t nsec = 0;
};

// ---------------------------------------------------------------- MurmurHash3_x64_128
// Standard public-domain algorithm; datasketches uses it with seed 9001
// (3rd/datasketches/common/include/common_defs.hpp:34).
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t k)
{
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}
static void murmur3_128(const uint8_t *data, size_t len, uint64_t seed, uint64_t &o1, uint64_t &o2)
{
    const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    uint64_t h1 = seed, h2 = seed;
    size_t nb = len / 16;
    for (size_t i = 0; i < nb; i++) {
        uint64_t k1, k2;
        memcpy(&k1, data + 16 * i, 8);
        memcpy(&k2, data + 16 * i + 8, 8);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t *t = data + nb * 16;
    uint64_t k1 = 0, k2 = 0;
    size_t r = len & 15;
    for (size_t i = r; i > 8; i--) k2 ^= (uint64_t)t[i - 1] << (8 * (i - 9));
    if (r > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
    for (size_t i = std::min<size_t>(r, 8); i > 0; i--) k1 ^= (uint64_t)t[i - 1] << (8 * (i - 1));
    if (r > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
    h1 ^= len; h2 ^= len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    o1 = h1; o2 = h2;
}

// ---------------------------------------------------------------- CPC (lg_k = 11)
// Restatement of the coupon/HIP/ICON logic of cpc_sketch_impl.hpp. The sketch
// state is the set of coupons; HIP depends on the order in which coupons first
// appear plus the periodic kxp refresh at window offsets that are multiples of 8.
static const int CPC_LGK = 11;
static const uint32_t CPC_K = 1u << CPC_LGK;

// icon_estimator.hpp:98-102 (log K = 11 row) — the published polynomial.
static const double ICON_COEF_LGK11[20] = {
    0.9999186020796150265, 0.3333249054574359826, 0.126791713589799987, -0.06662487271699729652,
    -0.07335552427910230211, 0.3316370184815959909, -1.434143797561290068, 4.180260309967409604,
    -8.593906870708760692, 12.95088874800289958, -14.56876092520539956, 12.37074367531410068,
    -7.969152075707960137, 3.888774396648960074, -1.424923326506990051, 0.385084561785229984,
    -0.07435541911616409816, 0.009695363567476529554, -0.0007644375960047160388, 2.75156194717188011e-05};

double icon_estimate(uint32_t c)
{
    if (c < 2) return c == 0 ? 0.0 : 1.0;
    const double k = (double)CPC_K, dc = (double)c;
    if (dc > 5.7 * k) return 0.7940236163830469 * k * pow(2.0, dc / k);
    const double x = dc / (2.0 * k);
    double total = ICON_COEF_LGK11[19];
    for (int j = 18; j >= 0; j--) { total *= x; total += ICON_COEF_LGK11[j]; }
    const double ratio = dc / k;
    const double term = 1.0 + (ratio * ratio * ratio / 66.774757);
    const double result = dc * total * term;
    return result >= dc ? result : dc;
}

static double kxp_byte(uint8_t b)
{
    double s = 0;
    for (int col = 0; col < 8; col++)
        if (((b >> col) & 1) == 0) s += ldexp(1.0, -(col + 1));
    return s;
}

struct Cpc {
    std::vector<uint64_t> rows = std::vector<uint64_t>(CPC_K, 0);
    uint32_t num_coupons = 0;
    double kxp = (double)CPC_K;
    double hip = 0;
    int window_offset = 0;
    bool windowed = false;
    bool merged = false;

    void refresh_kxp()
    {
        double byte_sums[8] = {0};
        for (uint32_t i = 0; i < CPC_K; i++) {
            uint64_t w = rows[i];
            for (int j = 0; j < 8; j++) { byte_sums[j] += kxp_byte(w & 0xff); w >>= 8; }
        }
        double total = 0;
        for (int j = 7; j >= 0; j--) total += ldexp(1.0, -8 * j) * byte_sums[j];
        kxp = total;
    }
    void coupon(uint32_t row, uint32_t col)
    {
        if ((rows[row] >> col) & 1) return;
        rows[row] |= 1ULL << col;
        num_coupons++;
        hip += (double)CPC_K / kxp;
        kxp -= ldexp(1.0, -(int)(col + 1));
        if (!windowed) {
            if (((uint64_t)num_coupons << 5) >= 3ULL * CPC_K) windowed = true;
        } else {
            if (((uint64_t)num_coupons << 3) >= (27ULL + ((uint64_t)window_offset << 3)) * CPC_K) {
                window_offset++;
                if ((window_offset & 7) == 0) refresh_kxp();
            }
        }
    }
    void update_bytes(const void *p, size_t n)
    {
        uint64_t h1, h2;
        murmur3_128((const uint8_t *)p, n, 9001, h1, h2);
        uint32_t col = h2 ? (uint32_t)__builtin_clzll(h2) : 64;
        if (col > 63) col = 63;
        coupon((uint32_t)(h1 & (CPC_K - 1)), col);
    }
    // cpc_sketch_impl.hpp:124-132: uint32 -> int32 -> int64 (sign extension), 8 bytes
    void update_u32(uint32_t v)
    {
        int64_t x = (int64_t)(int32_t)v;
        update_bytes(&x, 8);
    }
    void update_str(const std::string &s)
    {
        if (s.empty()) return; // cpc_sketch_impl.hpp:109-112
        update_bytes(s.data(), s.size());
    }
    void merge(const Cpc &o)
    {
        for (uint32_t i = 0; i < CPC_K; i++) rows[i] |= o.rows[i];
        num_coupons = 0;
        for (uint32_t i = 0; i < CPC_K; i++) num_coupons += __builtin_popcountll(rows[i]);
        merged = true;
    }
    double estimate() const { return merged ? icon_estimate(num_coupons) : hip; }
};

// ---------------------------------------------------------------- exact quantiles
// Same rank rule as the KLL sorted view in exact mode
// (quantiles_sorted_view_impl.hpp:76-84, inclusive=true): item at ceil(rank*n)-1.
template <typename T>
struct ExactQuantile {
    std::vector<T> v;
    std::vector<T> qsum; // Quantile::_quantiles_sum (src/Metrics.h:338-372)
    void update(T x) { v.push_back(x); }
    void merge(const ExactQuantile &o) { v.insert(v.end(), o.v.begin(), o.v.end()); }
    // Quantile::merge(other, Aggregate::SUM) (src/Metrics.h:356-372): once this sketch holds
    // data, the p50..p99 of every further non-empty sketch are added p-wise to a sum that the
    // output prefers; the sketch itself stays as it was. An empty sketch merges as usual.
    void merge_sum(const ExactQuantile &o)
    {
        if (v.empty()) { merge(o); return; }
        if (o.v.empty()) return;
        const std::vector<T> oq = o.quantiles_of_sketch();
        if (qsum.empty()) qsum = quantiles_of_sketch();
        for (int i = 0; i < 4; i++) qsum[i] += oq[i];
    }
    bool empty() const { return v.empty(); }
    std::vector<T> quantiles() const { return qsum.empty() ? quantiles_of_sketch() : qsum; }
    std::vector<T> quantiles_of_sketch() const
    {
        std::vector<T> s = v;
        std::sort(s.begin(), s.end());
        std::vector<T> out;
        const double ranks[4] = {0.50, 0.90, 0.95, 0.99};
        for (double r : ranks) {
            uint64_t w = (uint64_t)std::ceil(r * (double)s.size());
            size_t idx = w == 0 ? 0 : (size_t)(w - 1);
            if (idx >= s.size()) idx = s.size() - 1;
            out.push_back(s[idx]);
        }
        return out;
    }
    T p(double r) const
    {
        std::vector<T> s = v;
        std::sort(s.begin(), s.end());
        uint64_t w = (uint64_t)std::ceil(r * (double)s.size());
        size_t idx = w == 0 ? 0 : (size_t)(w - 1);
        if (idx >= s.size()) idx = s.size() - 1;
        return s[idx];
    }
};

// ---------------------------------------------------------------- exact top-N
template <typename K>
struct ExactTop {
    std::map<K, uint64_t> m;
    void update(const K &k, uint64_t w = 1) { m[k] += w; }
    void merge(const ExactTop &o)
    {
        for (auto &kv : o.m) m[kv.first] += kv.second;
    }
};

// ---------------------------------------------------------------- JSON writer
struct J {
    std::string s;
    std::vector<bool> first{true};
    void comma()
    {
        if (!first.back()) s += ',';
        first.back() = false;
    }
    void key(const std::string &k)
    {
        comma();
        str_(k);
        s += ':';
        first.back() = true; // value follows immediately
        pending_value = true;
    }
    bool pending_value = false;
    void pre_value()
    {
        if (pending_value) { pending_value = false; first.back() = false; return; }
        comma();
    }
    void str_(const std::string &v)
    {
        s += '"';
        for (unsigned char c : v) {
            if (c == '"') s += "\\\"";
            else if (c == '\\') s += "\\\\";
            else if (c < 0x20 || c >= 0x80) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); s += b; } // bytes >= 0x80 as U+0080..U+00FF
            else s += (char)c;
        }
        s += '"';
    }
    void str(const std::string &v) { pre_value(); str_(v); }
    void u64(uint64_t v) { pre_value(); s += std::to_string(v); }
    void i64(int64_t v) { pre_value(); s += std::to_string(v); }
    void dbl(double v)
    {
        pre_value();
        char b[40];
        snprintf(b, sizeof b, "%.17g", v);
        s += b;
        if (!strpbrk(b, ".eEn")) s += ".0";
    }
    void obj() { pre_value(); s += '{'; first.push_back(true); }
    void end_obj() { s += '}'; first.pop_back(); }
    void arr() { pre_value(); s += '['; first.push_back(true); }
    void end_arr() { s += ']'; first.pop_back(); }
};

// ---------------------------------------------------------------- name tables
// libs/visor_dns/dns.h:31-265 (QTypeNames / RCodeNames); restated for the
// codes the decoder can emit names for.
static const std::map<uint16_t, std::string> &qtype_names()
{
    static const std::map<uint16_t, std::string> m = {
        {0, "Reserved (0)"}, {1, "A"}, {2, "NS"}, {3, "MD"}, {4, "MF"}, {5, "CNAME"}, {6, "SOA"}, {7, "MB"}, {8, "MG"}, {9, "MR"},
        {10, "NULL"}, {11, "WKS"}, {12, "PTR"}, {13, "HINFO"}, {14, "MINFO"}, {15, "MX"}, {16, "TXT"},
        {17, "RP"}, {18, "AFSDB"}, {19, "X25"}, {20, "ISDN"}, {21, "RT"}, {22, "NSAP"}, {23, "NSAP-PTR"},
        {24, "SIG"}, {25, "KEY"}, {26, "PX"}, {27, "GPOS"}, {28, "AAAA"}, {29, "LOC"}, {30, "NXT"},
        {31, "EID"}, {32, "NIMLOC"}, {33, "SRV"}, {34, "ATMA"}, {35, "NAPTR"}, {36, "KX"}, {37, "CERT"},
        {38, "A6"}, {39, "DNAME"}, {40, "SINK"}, {41, "OPT"}, {42, "APL"}, {43, "DS"}, {44, "SSHFP"},
        {45, "IPSECKEY"}, {46, "RRSIG"}, {47, "NSEC"}, {48, "DNSKEY"}, {49, "DHCID"}, {50, "NSEC3"},
        {51, "NSEC3PARAM"}, {52, "TLSA"}, {53, "SMIMEA"}, {55, "HIP"}, {56, "NINFO"}, {57, "RKEY"},
        {58, "TALINK"}, {59, "CDS"}, {60, "CDNSKEY"}, {61, "OPENPGPKEY"}, {62, "CSYNC"}, {63, "ZONEMD"},
        {64, "SVCB"}, {65, "HTTPS"}, {99, "SPF"}, {100, "UINFO"}, {101, "UID"}, {102, "GID"}, {103, "UNSPEC"},
        {104, "NID"}, {105, "L32"}, {106, "L64"}, {107, "LP"}, {108, "EUI48"}, {109, "EUI64"},
        {249, "TKEY"}, {250, "TSIG"}, {251, "IXFR"}, {252, "AXFR"}, {253, "MAILB"}, {254, "MAILA"},
        {255, "*"}, {256, "URI"}, {257, "CAA"}, {258, "AVC"}, {259, "DOA"}, {260, "AMTRELAY"},
        {32768, "TA"}, {32769, "DLV"}, {65535, "Reserved (65535)"}};
    return m;
}
static const std::map<uint16_t, std::string> &rcode_names()
{
    static const std::map<uint16_t, std::string> m = {
        {0, "NOERROR"}, {1, "FORMERR"}, {2, "SRVFAIL"}, {3, "NXDOMAIN"}, {4, "NOTIMP"}, {5, "REFUSED"},
        {6, "YXDOMAIN"}, {7, "YXRRSET"}, {8, "NXRRSET"}, {9, "NOTAUTH"}, {10, "NOTZONE"}, {11, "DSOTYPENI"},
        {16, "BADVERS"}, {17, "BADKEY"}, {18, "BADTIME"}, {19, "BADMODE"}, {20, "BADNAME"}, {21, "BADALG"},
        {22, "BADTRUNC"}, {23, "BADCOOKIE"}};
    return m;
}

// ---------------------------------------------------------------- config
enum { NG_COUNTERS = 1, NG_CARDINALITY = 2, NG_TOP_GEO = 4, NG_TOP_IPS = 8 };
// DNS v2 groups (src/handlers/dns/v2/DnsStreamHandler.h:40-52, _group_defs :565-575)
enum { D2G_CARDINALITY = 1, D2G_COUNTERS = 2, D2G_QUANTILES = 4, D2G_TOP_ECS = 8, D2G_TOP_QTYPES = 16,
       D2G_TOP_RCODES = 32, D2G_TOP_SIZE = 64, D2G_TOP_QNAMES = 128, D2G_TOP_PORTS = 256, D2G_XACT_TIMES = 512 };
// Net v2 groups (src/handlers/net/v2/NetStreamHandler.h:25-31): Counters, Cardinality, Quantiles, TopGeo, TopIps
enum { N2G_COUNTERS = 1, N2G_CARDINALITY = 2, N2G_QUANTILES = 4, N2G_TOP_GEO = 8, N2G_TOP_IPS = 16 };
enum { DG_CARDINALITY = 1, DG_COUNTERS = 2, DG_QUANTILES = 4, DG_HISTOGRAMS = 8, DG_TRANSACTIONS = 16, DG_TOP_ECS = 32,
       DG_TOP_QNAMES = 64, DG_TOP_QNAMES_DETAILS = 128, DG_TOP_PORTS = 256 };
struct V4Net { uint32_t addr; uint8_t cidr; };  // addr: network-order bytes as LE u32 (in_addr.s_addr)
struct V6Net { uint8_t addr[16]; uint8_t cidr; };

struct Config {
    std::vector<V4Net> v4;
    std::vector<V6Net> v6;
    unsigned num_periods = 5;
    unsigned window = 5; // output window: 1 => single bucket 0 ("1m"), N>=2 => merged N ("Nm")
    size_t topn_count = 10;
    uint32_t xact_ttl_ms = 5000;
    // PcapInputStream's tcp_packet_reassembly_cache_limit (PcapInputStream.cpp:97-99): the LRU
    // list's capacity, DEFAULT_LRULIST_SIZE = TCP_TIMEOUT * 10000 without it (PcapInputStream.h:99)
    uint64_t tcp_cache_limit = 30 * 10000;
    bool recorded_stream = true;
    // metric groups (StreamMetricsHandler::process_groups, src/StreamHandler.h:111-133), as the
    // handler's _groups bits: net v1 defaults (NetStreamHandler.cpp:53-56), dns v1 defaults
    // (DnsStreamHandler.cpp:52-57); "dns_details=1" adds top_qnames_details
    uint32_t net_groups = NG_COUNTERS | NG_CARDINALITY | NG_TOP_GEO | NG_TOP_IPS;
    uint32_t dns_groups = DG_CARDINALITY | DG_COUNTERS | DG_QUANTILES | DG_TRANSACTIONS | DG_TOP_QNAMES | DG_TOP_PORTS;
    uint32_t topn_pct = 0;   // topn_percentile_threshold
    bool net_filter_all = false; // net geo / ASN filters with no geo database: every packet filtered (:223-283)
    unsigned deep_sample_rate = 100; // window config "deep_sample_rate" (AbstractMetricsManager.h:357-365), clamped 1..100
    // Net v2 handler attached ("net"): its groups (N2G_*), 0 = not attached
    uint32_t net2_groups = 0;
    // DNS v2 handler in place of v1 ("dns" is both versions' schema key): its groups (D2G_*), 0 = v1
    uint32_t dns2_groups = 0;
    bool filter_all = false; // geoloc_notfound / asn_notfound with no geo database: every packet filtered (:619-642)
    // DNS v1 filters (DnsStreamHandler::start, dns/v1/DnsStreamHandler.cpp:60-160)
    bool exclude_noerror = false;   // "exclude_noerror" (:61-63)
    uint32_t only_rcode_mask = 0;   // "only_rcode": bit r set = rcode r wanted (:64-113); predicate mode
    bool has_answer_count = false;  // "answer_count" (:123-130)
    uint32_t answer_count = 0;
    bool only_queries = false, only_responses = false; // (:114-119)
    bool only_dnssec = false;                           // "only_dnssec_response" (:120-122)
    bool psl = false;                                   // "public_suffix_list" config (:187-189)
    std::vector<int64_t> heartbeats; // heartbeat stamps (seconds, ascending): each fires before the first
                                     // packet past it (or at the end of the capture, before end_tstamp)
    int single = -1;                 // >= 0: output bucket `single` alone (window_single_json)
    std::vector<uint16_t> only_qtype;                   // "only_qtype" (:131-150)
    std::vector<std::string> only_qname;                // "only_qname" (:151-160), lower-case; predicate mode
    std::vector<std::string> only_qname_suffix;         // "only_qname_suffix" (:161-169), lower-case
    // DNS v2 (dns/v2/DnsStreamHandler.cpp:61-170): the filter keys above read with v2's
    // semantics (_filtering :484-609), plus only_xact_directions: bit 0 in, 1 out, 2 unknown off
    uint32_t xact_dirs_disabled = 0;
};

// libs/visor_utils/utils.cpp:128-164
static bool parse_host_specs(const std::string &spec, Config &c, std::string &err)
{
    size_t pos = 0;
    while (pos <= spec.size() && !spec.empty()) {
        size_t e = spec.find(',', pos);
        std::string host = spec.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
        pos = e == std::string::npos ? spec.size() + 1 : e + 1;
        if (host.empty()) continue;
        size_t d = host.find('/');
        if (d == std::string::npos) { err = "invalid CIDR: " + host; return false; }
        std::string ip = host.substr(0, d), cs = host.substr(d + 1);
        if (cs.empty() || !std::all_of(cs.begin(), cs.end(), ::isdigit)) { err = "invalid CIDR: " + host; return false; }
        int cidr = atoi(cs.c_str());
        if (ip.find(':') != std::string::npos) {
            if (cidr < 0 || cidr > 128) { err = "invalid CIDR: " + host; return false; }
            V6Net n;
            if (inet_pton(AF_INET6, ip.c_str(), n.addr) != 1) { err = "invalid IPv6 address: " + ip; return false; }
            n.cidr = (uint8_t)cidr;
            c.v6.push_back(n);
        } else {
            if (cidr < 0 || cidr > 32) { err = "invalid CIDR: " + host; return false; }
            in_addr a;
            if (inet_pton(AF_INET, ip.c_str(), &a) != 1) { err = "invalid IPv4 address: " + ip; return false; }
            c.v4.push_back({a.s_addr, (uint8_t)cidr});
        }
    }
    return true;
}

// utils.cpp:26-43 — value 0 never matches; cidr 0 matches everything.
static bool match_v4(const Config &c, uint32_t ip)
{
    if (!ip) return false;
    for (auto &n : c.v4) {
        if (n.cidr == 0) return true;
        uint32_t mask = htonl(0xFFFFFFFFu << (32 - n.cidr));
        if (((ip ^ n.addr) & mask) == 0) return true;
    }
    return false;
}
// utils.cpp:45-69 — byte compare then bit compare; prefix 0 never matches.
static bool match_v6(const Config &c, const uint8_t *ip)
{
    for (auto &n : c.v6) {
        uint8_t bytes = n.cidr / 8, bits = n.cidr % 8;
        bool r = false;
        if (bytes > 0) r = memcmp(n.addr, ip, bytes) == 0;
        if ((r || n.cidr < 8) && bits > 0) r = (n.addr[bytes] >> (8 - bits)) == (ip[bytes] >> (8 - bits));
        if (r) return true;
    }
    return false;
}

// ---------------------------------------------------------------- packet parse
// PcapPlusPlus 23.09 `Packet(raw, TCP|UDP)` semantics restated.
enum { L3_UNKNOWN = 0, L3_IPV4 = 4, L3_IPV6 = 6 };
enum { L4_UNKNOWN = 0, L4_TCP = 6, L4_UDP = 17 };
enum Dir { DIR_TO_HOST = 0, DIR_FROM_HOST = 1, DIR_UNKNOWN = 2 };

struct Pkt {
    const uint8_t *data = nullptr;
    uint32_t caplen = 0;
    TS ts;
    int l3 = L3_UNKNOWN, l4 = L4_UNKNOWN;
    bool has_v4 = false, has_v6 = false;
    const uint8_t *v4hdr = nullptr; // first IPv4 layer header
    const uint8_t *v6hdr = nullptr; // first IPv6 layer header
    const uint8_t *ip1 = nullptr;   // first IP layer of either version (getLayerOfType<IPLayer>)
    bool ip1_v6 = false;
    const uint8_t *l4hdr = nullptr;
    uint32_t l4len = 0; // L4 layer data length (incl. L4 header), IP-length trimmed
    bool syn = false;
    Dir dir = DIR_UNKNOWN;
};

static void parse_ip(Pkt &p, const uint8_t *d, size_t len, int depth);

static bool ipv4_valid(const uint8_t *d, size_t len) { return len >= 20 && (d[0] >> 4) == 4 && (d[0] & 0x0f) >= 5; }
static bool ipv6_valid(const uint8_t *, size_t len) { return len >= 40; }

static void parse_l4(Pkt &p, int proto, const uint8_t *d, size_t len)
{
    if (proto == 17) {
        if (len >= 8) { p.l4 = L4_UDP; p.l4hdr = d; p.l4len = (uint32_t)len; }
    } else if (proto == 6) {
        if (len >= 20) {
            p.l4 = L4_TCP; p.l4hdr = d; p.l4len = (uint32_t)len;
            p.syn = (d[13] & 0x02) != 0;
        }
    }
}

static void parse_ipv4(Pkt &p, const uint8_t *d, size_t len, int depth)
{
    if (!p.has_v4) { p.has_v4 = true; p.v4hdr = d; }
    if (!p.ip1) { p.ip1 = d; p.ip1_v6 = false; }
    size_t total = rd16be(d + 2);
    if (total < len && total != 0) len = total; // IPv4Layer ctor trims to totalLength
    size_t hl = (size_t)(d[0] & 0x0f) * 4;
    if (len <= hl) return;
    const uint8_t *pl = d + hl;
    size_t pll = len - hl;
    uint16_t frag = rd16be(d + 6);
    if ((frag & 0x2000) || (frag & 0x1fff)) return; // fragment -> payload layer, no L4
    uint8_t proto = d[9];
    if (proto == 17 || proto == 6) parse_l4(p, proto, pl, pll);
    else if (proto == 4 || proto == 41) parse_ip(p, pl, pll, depth + 1);
}

static void parse_ipv6(Pkt &p, const uint8_t *d, size_t len, int depth)
{
    if (!p.has_v6) { p.has_v6 = true; p.v6hdr = d; }
    if (!p.ip1) { p.ip1 = d; p.ip1_v6 = true; }
    // IPv6Layer::parseExtensions
    uint8_t next = d[6];
    size_t off = 40;
    bool frag = false;
    while (len >= 2 && off <= len - 2) {
        size_t elen;
        if (next == 44) elen = 8;
        else if (next == 0 || next == 60 || next == 43) elen = ((size_t)d[off + 1] + 1) * 8;
        else if (next == 51) elen = ((size_t)d[off + 1] + 2) * 4;
        else break;
        frag = (next == 44);
        next = d[off];
        off += elen;
    }
    size_t hdrlen = off;
    size_t total = (size_t)rd16be(d + 4) + hdrlen;
    if (total < len) len = total;
    if (len <= hdrlen) return;
    const uint8_t *pl = d + hdrlen;
    size_t pll = len - hdrlen;
    if (frag) return;
    if (next == 17 || next == 6) parse_l4(p, next, pl, pll);
    else if (next == 4 || next == 41) parse_ip(p, pl, pll, depth + 1);
}

static void parse_ip(Pkt &p, const uint8_t *d, size_t len, int depth)
{
    if (depth > 4 || len < 1) return;
    int v = d[0] >> 4;
    if (v == 4 && ipv4_valid(d, len)) parse_ipv4(p, d, len, depth);
    else if (v == 6 && ipv6_valid(d, len)) parse_ipv6(p, d, len, depth);
}

static void parse_ether_payload(Pkt &p, uint16_t et, const uint8_t *d, size_t len, int depth)
{
    if (et == 0x0800) { if (ipv4_valid(d, len)) parse_ipv4(p, d, len, 0); }
    else if (et == 0x86DD) { if (ipv6_valid(d, len)) parse_ipv6(p, d, len, 0); }
    else if ((et == 0x8100 || et == 0x88A8) && depth < 8) {
        if (len <= 4) return;
        parse_ether_payload(p, rd16be(d + 2), d + 4, len - 4, depth + 1);
    }
}

static void parse_packet(Pkt &p, uint32_t linktype)
{
    const uint8_t *d = p.data;
    size_t len = p.caplen;
    if (linktype == 1) {
        if (len < 14 || rd16be(d + 12) < 0x600) return;
        if (len <= 14) return;
        parse_ether_payload(p, rd16be(d + 12), d + 14, len - 14, 0);
    } else if (linktype == 101 || linktype == 12 || linktype == 14 || linktype == 228 || linktype == 229) {
        parse_ip(p, d, len, 0);
    } else if (linktype == 113) {
        if (len <= 16) return;
        parse_ether_payload(p, rd16be(d + 14), d + 16, len - 16, 0);
    }
    if (p.has_v4) p.l3 = L3_IPV4;
    else if (p.has_v6) p.l3 = L3_IPV6;
}

// PcapInputStream.cpp:401-416
static void set_direction(Pkt &p, const Config &c)
{
    p.dir = DIR_UNKNOWN;
    if (p.has_v4) {
        if (match_v4(c, rd32le(p.v4hdr + 16))) p.dir = DIR_TO_HOST;
        else if (match_v4(c, rd32le(p.v4hdr + 12))) p.dir = DIR_FROM_HOST;
    } else if (p.has_v6) {
        if (match_v6(c, p.v6hdr + 24)) p.dir = DIR_TO_HOST;
        else if (match_v6(c, p.v6hdr + 8)) p.dir = DIR_FROM_HOST;
    }
}

// PcapPlusPlus hash5Tuple (directionUnique=false), FNV-1 32-bit. Restated.
static uint32_t hash5tuple(const Pkt &p)
{
    if (!p.has_v4 && !p.has_v6) return 0;
    if (p.l4 != L4_TCP && p.l4 != L4_UDP) return 0;
    uint16_t ps, pd;
    memcpy(&ps, p.l4hdr, 2);
    memcpy(&pd, p.l4hdr + 2, 2);
    int sp = (pd < ps) ? 1 : 0;
    const uint8_t *vec[5];
    size_t vl[5];
    vec[0 + sp] = (const uint8_t *)&ps; vl[0 + sp] = 2;
    vec[1 - sp] = (const uint8_t *)&pd; vl[1 - sp] = 2;
    if (p.has_v4) {
        uint32_t s = rd32le(p.v4hdr + 12), dd = rd32le(p.v4hdr + 16);
        if (ps == pd && dd < s) sp = 1;
        vec[2 + sp] = p.v4hdr + 12; vl[2 + sp] = 4;
        vec[3 - sp] = p.v4hdr + 16; vl[3 - sp] = 4;
        vec[4] = p.v4hdr + 9; vl[4] = 1;
    } else {
        // the reference compares the two array addresses, never true
        vec[2 + sp] = p.v6hdr + 8; vl[2 + sp] = 16;
        vec[3 - sp] = p.v6hdr + 24; vl[3 - sp] = 16;
        vec[4] = p.v6hdr + 6; vl[4] = 1;
    }
    uint32_t h = 0x811C9DC5u;
    for (int i = 0; i < 5; i++)
        for (size_t j = 0; j < vl[i]; j++) { h *= 0x01000193u; h ^= vec[i][j]; }
    return h;
}

static std::string ipv4_str(uint32_t le)
{
    char b[20];
    snprintf(b, sizeof b, "%u.%u.%u.%u", le & 0xff, (le >> 8) & 0xff, (le >> 16) & 0xff, le >> 24);
    return b;
}
static std::string ipv6_str(const uint8_t *a)
{
    char b[64];
    inet_ntop(AF_INET6, a, b, sizeof b);
    return b;
}

// ---------------------------------------------------------------- DNS decoder
// libs/visor_dns/DnsResource.cpp:53-148 decodeName, restated with identical
// bounds/truncation/pointer rules. Returns the encoded length; `out` receives
// the decoded bytes (not NUL-truncated here; callers truncate as std::string did).
struct DnsMsg {
    const uint8_t *d;
    size_t len;
    uint8_t byte(size_t off) const { return d[off]; }
};

static size_t decode_name(const DnsMsg &m, size_t off, std::string &out, int iteration)
{
    size_t enc = 0, dec = 0;
    out.clear();
    size_t cur = off;
    if (cur + 1 > m.len) return enc;
    if (iteration > 20) return enc;
    uint8_t wl = m.byte(cur);
    while (wl != 0) {
        if ((wl & 0xc0) == 0xc0) {
            if (cur + 2 > m.len || enc > 255) return enc;
            uint16_t ptr = (uint16_t)((wl & 0x3f) * 256 + m.byte(cur + 1));
            // illegal pointer: return 0. At the top level the caller discards the text
            // (m_NameLength == 0); a nested caller copies what this level already wrote
            // into its zero-filled tempResult (labels with their trailing '.').
            if (ptr < 12 || ptr >= m.len) return 0;
            std::string tmp;
            decode_name(m, ptr, tmp, iteration + 1);
            // tempResult is a zero-filled buffer: copy stops at the first NUL
            size_t i = 0;
            while (i < tmp.size() && tmp[i] != 0 && dec < 255) { out.push_back(tmp[i++]); dec++; }
            return enc + 2;
        } else {
            if (cur + wl + 1 > m.len || enc + wl > 255) {
                if (enc == 256) { out.pop_back(); dec--; }
                else enc++;
                return enc;
            }
            out.append((const char *)m.d + cur + 1, wl);
            out.push_back('.');
            dec += wl + 1;
            cur += wl + 1;
            enc += wl + 1;
            if (cur + 1 > m.len) {
                if (enc == 256) { dec--; out.pop_back(); }
                else enc++;
                return enc;
            }
            wl = m.byte(cur);
        }
    }
    if (!out.empty()) out.pop_back(); // remove the last '.'
    enc++;
    return enc;
}

struct DnsParse {
    bool ok = false;        // parseResources(queryOnly=true) result
    bool has_query = false;
    std::string name;       // getName() (NUL-truncated like std::string(char*))
    uint16_t qtype = 0;
};

// DnsLayer.cpp:119-209 with queryOnly=true.
// only_dnssec_response (dns/v1/DnsStreamHandler.cpp:573-595): parseResources(false, true, true)
// walks questions, answers, authorities and the first additional (DnsLayer.cpp:119-209); the
// packet passes if that walk stays in bounds and an answer has type RRSIG (46)
static bool dnssec_answer(const DnsMsg &m)
{
    uint16_t qd = rd16be(m.d + 4), an = rd16be(m.d + 6), ns = rd16be(m.d + 8), ar = rd16be(m.d + 10);
    uint32_t total = (uint32_t)qd + an + ns + ar;
    if (total > 100 || m.len < 12) return false;
    size_t off = 12;
    bool sig = false;
    for (uint32_t i = 0; i < total; i++) {
        int kind = 0; // 0 query, 1 answer, 2 authority, 3 additional
        if (qd > 0) qd--;
        else if (an > 0) { an--; kind = 1; }
        else if (ns > 0) { ns--; kind = 2; }
        else { ar--; kind = 3; }
        std::string nm;
        size_t nl = decode_name(m, off, nm, 1);
        size_t sz;
        if (kind == 0) sz = nl + 4;
        else {
            size_t dl_off = off + nl + 8;
            uint16_t dl = (dl_off + 2 <= m.len) ? rd16be(m.d + dl_off) : 0;
            sz = nl + 10 + dl;
        }
        const size_t start = off;
        off += sz;
        if (off > m.len) return false;
        if (kind == 1 && rd16be(m.d + start + nl) == 46) sig = true;
        if (kind == 3) break;
    }
    return sig;
}

static DnsParse parse_resources(const DnsMsg &m)
{
    DnsParse r;
    uint16_t qd = rd16be(m.d + 4), an = rd16be(m.d + 6), ns = rd16be(m.d + 8), ar = rd16be(m.d + 10);
    uint32_t total = (uint32_t)qd + an + ns + ar;
    if (total > 100) return r;
    size_t off = 12;
    for (uint32_t i = 0; i < total; i++) {
        bool is_q = false;
        if (qd > 0) { is_q = true; qd--; }
        else if (an > 0) an--;
        else if (ns > 0) ns--;
        else ar--;
        std::string nm;
        size_t nl = decode_name(m, off, nm, 1);
        size_t sz;
        if (is_q) sz = nl + 4;
        else {
            size_t dl_off = off + nl + 8;
            uint16_t dl = (dl_off + 2 <= m.len) ? rd16be(m.d + dl_off) : 0;
            sz = nl + 10 + dl;
        }
        size_t start = off;
        off += sz;
        if (off > m.len) return r;
        if (is_q) {
            r.has_query = true;
            if (nl > 0) {
                size_t z = nm.find('\0');
                r.name = z == std::string::npos ? nm : nm.substr(0, z);
            }
            r.qtype = rd16be(m.d + start + nl);
            break;
        }
    }
    r.ok = true;
    return r;
}

// The first additional record, as DnsLayer::parseResources(false, true, true) finds it
// (libs/visor_dns/DnsLayer.cpp:119-209): questions, answers, authorities, then the first
// additional, each in bounds; its offset or -1.
static long first_additional(const DnsMsg &m)
{
    uint16_t qd = rd16be(m.d + 4), an = rd16be(m.d + 6), ns = rd16be(m.d + 8), ar = rd16be(m.d + 10);
    uint32_t total = (uint32_t)qd + an + ns + ar;
    if (total > 100 || m.len < 12 || ar == 0) return -1;
    size_t off = 12;
    for (uint32_t i = 0; i < total; i++) {
        const bool is_q = i < qd;
        std::string nm;
        size_t nl = decode_name(m, off, nm, 1);
        size_t sz;
        if (is_q) sz = nl + 4;
        else {
            size_t dl_off = off + nl + 8;
            uint16_t dl = (dl_off + 2 <= m.len) ? rd16be(m.d + dl_off) : 0;
            sz = nl + 10 + dl;
        }
        const size_t start = off;
        off += sz;
        if (off > m.len) return -1;
        if (i == (uint32_t)qd + an + ns) return (long)start;
    }
    return -1;
}

// parse_additional_records_ecs (libs/visor_dns/DnsAdditionalRecord.h:49-101): an OPT record
// whose data (at least 9 bytes) opens with option CSUBNET (8); family 1 takes the data bytes
// from offset 8 as the IPv4 address (the reference copies them all into a 4-byte array: only
// the first 4 are kept here), family 2 takes data bytes 8 .. min(len, 16) as the start of
// the IPv6 address. inet_ntop text, empty for other families.
static std::string ecs_subnet(const DnsMsg &m)
{
    const long a = first_additional(m);
    if (a < 0) return "";
    std::string nm;
    const size_t nl = decode_name(m, (size_t)a, nm, 1);
    const uint8_t *r = m.d + a + nl;
    const uint16_t type = rd16be(r), dlen = rd16be(r + 8);
    if (type != 41 || dlen < 9) return "";
    const uint8_t *x = r + 10;
    if (rd16be(x) != 8) return "";
    const uint16_t family = rd16be(x + 4);
    char buf[64];
    if (family == 1) {
        uint8_t v4[4] = {0, 0, 0, 0};
        for (size_t i = 8; i < dlen && i < 12; i++) v4[i - 8] = x[i];
        inet_ntop(AF_INET, v4, buf, sizeof buf);
        return buf;
    }
    if (family == 2) {
        uint8_t v6[16] = {0};
        for (size_t i = 8; i < std::min<size_t>(dlen, 16); i++) v6[i - 8] = x[i];
        inet_ntop(AF_INET6, v6, buf, sizeof buf);
        return buf;
    }
    return "";
}

static std::string lower(const std::string &s)
{
    std::string o = s;
    for (auto &c : o) c = (char)tolower((unsigned char)c);
    return o;
}

// match_public_suffix (libs/visor_dns/PublicSuffixList.h:226-250): the last label picks a
// list; the first listed suffix the whole name ends with (a byte compare, no label
// boundary) gives its size + 1, else the label's size + 1; 0 without a listed label.
// The table is pv_psl_data.h, generated from the reference's ICANN section (tools/gen_psl.py).
#include "../pktvisor_amd/csrc/pv_psl_data.h"
static size_t match_public_suffix(const std::string &str)
{
    static const std::unordered_map<std::string, std::pair<uint32_t, uint32_t>> icann = [] {
        std::unordered_map<std::string, std::pair<uint32_t, uint32_t>> m;
        uint32_t first = 0;
        for (uint32_t t = 0; t < PV_PSL_NTLD; t++) {
            m.emplace(pv_psl_tld[t], std::make_pair(first, (uint32_t)pv_psl_count[t]));
            first += pv_psl_count[t];
        }
        return m;
    }();
    const size_t pos = str.find_last_of('.');
    if (pos == std::string::npos || pos + 1 == str.size()) return 0;
    auto it = icann.find(str.substr(pos + 1));
    if (it == icann.end()) return 0;
    for (uint32_t k = it->second.first; k < it->second.first + it->second.second; k++) {
        const std::string sub = pv_psl_sfx[k];
        if (str.size() >= sub.size() && str.compare(str.size() - sub.size(), sub.size(), sub) == 0) return sub.size() + 1;
    }
    return it->first.size() + 1;
}

// libs/visor_dns/dns.cpp:9-43
static void aggregate_domain(const std::string &domain, size_t suffix_size, std::string &q2, std::string &q3)
{
    q2 = domain;
    q3 = domain;
    if (domain.size() < 5) { q3 = ""; return; }
    size_t endDot = std::string::npos;
    if (suffix_size > 0 && domain.size() > suffix_size) endDot = domain.size() - suffix_size;
    else if (domain.back() == '.') endDot = domain.size() - 2;
    size_t first_dot = domain.rfind('.', endDot);
    if (first_dot != std::string::npos && first_dot > 0) {
        size_t second_dot = domain.rfind('.', first_dot - 1);
        if (second_dot != std::string::npos) {
            q2 = domain.substr(second_dot);
            if (second_dot > 0) {
                size_t third_dot = domain.rfind('.', second_dot - 1);
                if (third_dot != std::string::npos) q3 = domain.substr(third_dot);
            }
        } else {
            q3 = "";
        }
    }
}

// ---------------------------------------------------------------- buckets
struct BaseBucket {
    TS start, end;
    unsigned period_length = 0;
    bool read_only = false;
    uint64_t num_events = 0, num_samples = 0;
    void set_read_only(TS s)
    {
        end = s;
        period_length = (unsigned)(end.sec - start.sec);
        read_only = true;
    }
};

struct NetBucket : BaseBucket {
    uint64_t UDP = 0, TCP = 0, OtherL4 = 0, IPv4 = 0, IPv6 = 0, TCP_SYN = 0, in = 0, out = 0, unk = 0, total = 0,
             filtered = 0;
    ExactQuantile<uint64_t> payload;
    Cpc src, dst;
    ExactTop<uint32_t> top4;
    ExactTop<std::string> top6;

    // NetworkMetricsBucket::specialized_merge (net/v1/NetStreamHandler.cpp:285-330); sum:
    // Aggregate::SUM, the quantile rule of a policy's merged handlers
    void merge(const NetBucket &o, bool sum = false)
    {
        UDP += o.UDP; TCP += o.TCP; OtherL4 += o.OtherL4; IPv4 += o.IPv4; IPv6 += o.IPv6; TCP_SYN += o.TCP_SYN;
        in += o.in; out += o.out; unk += o.unk; total += o.total; filtered += o.filtered;
        if (sum) payload.merge_sum(o.payload);
        else payload.merge(o.payload);
        src.merge(o.src);
        dst.merge(o.dst);
        top4.merge(o.top4);
        top6.merge(o.top6);
    }
};

// Net v2 (src/handlers/net/v2/NetStreamHandler.h:61-156): every metric per direction
struct Net2Dir {
    uint64_t UDP = 0, TCP = 0, OtherL4 = 0, IPv4 = 0, IPv6 = 0, TCP_SYN = 0, total = 0;
    uint64_t seen = 0; // packets of this direction (the reference's _net map entry exists once one arrived)
    ExactQuantile<uint64_t> payload;
    Cpc ips;
    ExactTop<uint32_t> top4;
    ExactTop<std::string> top6;
    // NetworkMetricsBucket::specialized_merge, v2 (net/v2/NetStreamHandler.cpp:286-331); sum:
    // Aggregate::SUM (a policy's merged handlers)
    void merge(const Net2Dir &o, bool sum = false)
    {
        UDP += o.UDP; TCP += o.TCP; OtherL4 += o.OtherL4; IPv4 += o.IPv4; IPv6 += o.IPv6; TCP_SYN += o.TCP_SYN;
        total += o.total; seen += o.seen;
        if (sum) payload.merge_sum(o.payload);
        else payload.merge(o.payload);
        ips.merge(o.ips);
        top4.merge(o.top4);
        top6.merge(o.top6);
    }
};
struct Net2Bucket : BaseBucket {
    uint64_t filtered = 0;
    Net2Dir dir[3]; // in (toHost), out (fromHost), unknown
    void merge(const Net2Bucket &o, bool sum = false)
    {
        filtered += o.filtered;
        for (int d = 0; d < 3; d++) dir[d].merge(o.dir[d], sum);
    }
};

// DNS v2 (src/handlers/dns/v2/DnsStreamHandler.h:75-291): transaction-centric, per direction
struct Dns2Dir {
    uint64_t xacts = 0, UDP = 0, TCP = 0, IPv4 = 0, IPv6 = 0, NX = 0, ECS = 0, REFUSED = 0, SRVFAIL = 0, NOERROR = 0,
             NODATA = 0, AD = 0, AA = 0, CD = 0, timeout = 0, orphan = 0;
    bool seen = false; // DnsMetricsBucket::dir_setup ran for this direction
    ExactQuantile<uint64_t> time;
    ExactQuantile<uint64_t> hist; // dnsHistTimeUs (a Histogram: its sketch merges under any aggregate)
    ExactQuantile<double> ratio;
    Cpc qname;
    ExactTop<std::string> ecs, qname2, qname3, nx, refused, sized, srvfail, nodata, noerror, slow;
    ExactTop<uint16_t> port, qtype, rcode;
    // DnsMetricsBucket::specialized_merge, v2 (dns/v2/DnsStreamHandler.cpp:619-676); sum: Aggregate::SUM
    void merge(const Dns2Dir &o, bool sum = false)
    {
        xacts += o.xacts; UDP += o.UDP; TCP += o.TCP; IPv4 += o.IPv4; IPv6 += o.IPv6; NX += o.NX; ECS += o.ECS;
        REFUSED += o.REFUSED; SRVFAIL += o.SRVFAIL; NOERROR += o.NOERROR; NODATA += o.NODATA; AD += o.AD; AA += o.AA;
        CD += o.CD; timeout += o.timeout; orphan += o.orphan;
        seen = seen || o.seen;
        if (sum) { time.merge_sum(o.time); ratio.merge_sum(o.ratio); }
        else { time.merge(o.time); ratio.merge(o.ratio); }
        hist.merge(o.hist);
        qname.merge(o.qname);
        ecs.merge(o.ecs); qname2.merge(o.qname2); qname3.merge(o.qname3); nx.merge(o.nx); refused.merge(o.refused);
        sized.merge(o.sized); srvfail.merge(o.srvfail); nodata.merge(o.nodata); noerror.merge(o.noerror);
        slow.merge(o.slow); port.merge(o.port); qtype.merge(o.qtype); rcode.merge(o.rcode);
    }
};
struct Dns2Bucket : BaseBucket {
    uint64_t filtered = 0;
    Dns2Dir dir[3]; // in, out, unknown
    void merge(const Dns2Bucket &o, bool sum = false)
    {
        filtered += o.filtered;
        for (int d = 0; d < 3; d++) dir[d].merge(o.dir[d], sum);
    }
};

struct DnsBucket : BaseBucket {
    uint64_t xacts_total = 0, xacts_in = 0, xacts_out = 0, xacts_timed_out = 0, queries = 0, replies = 0, UDP = 0,
             TCP = 0, IPv4 = 0, IPv6 = 0, NX = 0, REFUSED = 0, SRVFAIL = 0, NOERROR = 0, NODATA = 0, total = 0,
             filtered = 0, query_ecs = 0;
    ExactQuantile<uint64_t> xact_from, xact_to; // "out" / "in" quantiles_us
    ExactQuantile<uint64_t> hist_from, hist_to; // "out" / "in" histogram_us (Histogram, src/Metrics.h:189-327)
    ExactQuantile<double> ratio;
    Cpc qname;
    ExactTop<std::string> qname2, qname3, nx, refused, srvfail, nodata, noerror, sized_resp, slow_in, slow_out, ecs;
    ExactTop<uint16_t> udp_port, qtype, rcode;

    // DnsMetricsBucket::specialized_merge (dns/v1/DnsStreamHandler.cpp:658-733); sum: Aggregate::SUM
    void merge(const DnsBucket &o, bool sum = false)
    {
        xacts_total += o.xacts_total; xacts_in += o.xacts_in; xacts_out += o.xacts_out;
        xacts_timed_out += o.xacts_timed_out; queries += o.queries; replies += o.replies; UDP += o.UDP;
        TCP += o.TCP; IPv4 += o.IPv4; IPv6 += o.IPv6; NX += o.NX; REFUSED += o.REFUSED; SRVFAIL += o.SRVFAIL;
        NOERROR += o.NOERROR; NODATA += o.NODATA; total += o.total; filtered += o.filtered; query_ecs += o.query_ecs;
        if (sum) { xact_from.merge_sum(o.xact_from); xact_to.merge_sum(o.xact_to); ratio.merge_sum(o.ratio); }
        else { xact_from.merge(o.xact_from); xact_to.merge(o.xact_to); ratio.merge(o.ratio); }
        hist_from.merge(o.hist_from); hist_to.merge(o.hist_to); ecs.merge(o.ecs);
        qname.merge(o.qname);
        qname2.merge(o.qname2); qname3.merge(o.qname3); nx.merge(o.nx); refused.merge(o.refused);
        srvfail.merge(o.srvfail); nodata.merge(o.nodata); noerror.merge(o.noerror); sized_resp.merge(o.sized_resp);
        slow_in.merge(o.slow_in); slow_out.merge(o.slow_out);
        udp_port.merge(o.udp_port); qtype.merge(o.qtype); rcode.merge(o.rcode);
    }
};

// AbstractMetricsManager window/period engine (src/AbstractMetricsManager.h:276-333)
template <typename B>
struct Window {
    std::deque<std::unique_ptr<B>> buckets;
    unsigned num_periods;
    int64_t next_shift_sec = 0;
    explicit Window(unsigned np) : num_periods(std::max(1u, std::min(np, 10u))) { buckets.emplace_front(new B()); }
    B &live() { return *buckets.front(); }
    void set_start(TS ts)
    {
        next_shift_sec = ts.sec + 60;
        buckets.front()->start = ts;
    }
    void set_end(TS ts) { buckets.front()->set_read_only(ts); }
    // returns true if a period shift happened
    bool maybe_shift(TS ts)
    {
        if (!(num_periods > 1 && ts.sec >= next_shift_sec)) return false;
        buckets.emplace_front(new B());
        buckets.front()->start = ts;
        buckets[1]->set_read_only(ts);
        if (buckets.size() > num_periods) buckets.pop_back();
        next_shift_sec = ts.sec + 60;
        return true;
    }
    void new_event(bool deep)
    {
        live().num_events++;
        if (deep) live().num_samples++;
    }
};

// jsf32 (3rd/rng/jsf.h:38-70,111,151: jsf<uint32_t, uint32_t, 27, 17, 0>, seed 1, 20 rounds)
struct Jsf32 {
    uint32_t a = 0xf1ea5eedu, b = 1, c = 1, d = 1;
    Jsf32() { for (int i = 0; i < 20; i++) (*this)(); }
    static uint32_t rot(uint32_t x, unsigned k) { return (x << k) | (x >> (32 - k)); }
    uint32_t operator()()
    {
        uint32_t e = a - rot(b, 27);
        a = b ^ rot(c, 17);
        b = c + d;
        c = d + e;
        d = e + a;
        return d;
    }
};

// AbstractMetricsManager::new_event's sampling (src/AbstractMetricsManager.h:318-333): each
// manager draws once per sampled event when the rate is not 100 and keeps the flag; an event
// with sample=false (process_filtered) counts the stale flag
struct Sampler {
    Jsf32 rng;
    unsigned rate = 100;
    bool now = true;
    bool draw(bool sample)
    {
        if (sample && rate != 100) now = rng() % 100u < rate;
        return now;
    }
};

struct XactKey {
    uint32_t flow;
    uint16_t txid;
    bool operator==(const XactKey &o) const { return flow == o.flow && txid == o.txid; }
};
struct XactKeyHash {
    size_t operator()(const XactKey &k) const { return std::hash<uint64_t>()(((uint64_t)k.flow << 16) | k.txid); }
};
struct Xact {
    TS start;
    size_t query_size;
};

// ---------------------------------------------------------------- the engine
struct Engine {
    Config cfg;
    uint32_t linktype = 1;
    Window<NetBucket> net;
    Window<Net2Bucket> net2;
    Window<DnsBucket> dns;
    Window<Dns2Bucket> dns2;
    std::unordered_map<XactKey, Xact, XactKeyHash> xacts;
    // DNS v2: one TransactionManager per direction (DnsMetricsManager::_pair_manager, v2 .h:421-437)
    struct Xact2 {
        TS start;
        size_t query_size;
        bool cd;
        std::string ecs;
        bool filtered = false; // DnsTransaction::filtered (dns/v2/DnsStreamHandler.h:55-60)
    };
    std::unordered_map<XactKey, Xact2, XactKeyHash> xacts2[3];
    float per90_2[3] = {0.0f, 0.0f, 0.0f};
    uint32_t ttl_s = 0, ttl_ms = 0;
    float to90 = 0.0f, from90 = 0.0f;
    Sampler net_s, dns_s;   // the Net and DNS managers' generators
    Sampler net2_s, dns2_s; // the v2 managers' own (same default seed: jsf32 default-constructed)

    explicit Engine(const Config &c) : cfg(c), net(c.num_periods), net2(c.num_periods), dns(c.num_periods), dns2(c.num_periods)
    {
        net_s.rate = dns_s.rate = net2_s.rate = dns2_s.rate = c.deep_sample_rate;
        // TransactionManager.h:60-68
        if (c.xact_ttl_ms > 1000) { ttl_s = c.xact_ttl_ms / 1000; ttl_ms = c.xact_ttl_ms - ttl_s * 1000; }
        else ttl_ms = c.xact_ttl_ms;
    }

    // heartbeat_signal -> check_period_shift in each handler (src/AbstractMetricsManager.h:462-470;
    // net/v1/NetStreamHandler.cpp:99-102, dns/v1/DnsStreamHandler.cpp:219-222): a shift with no
    // event, the DNS manager's on_period_shift included
    void heartbeat(TS ts)
    {
        net.maybe_shift(ts);
        net2.maybe_shift(ts);
        if (dns.maybe_shift(ts)) on_dns_period_shift(ts);
        if (dns2.maybe_shift(ts)) on_dns2_period_shift(ts);
    }
    void start(TS ts)
    {
        net.set_start(ts);
        net2.set_start(ts);
        dns.set_start(ts);
        dns2.set_start(ts);
    }
    void end(TS ts)
    {
        net.set_end(ts);
        net2.set_end(ts);
        dns.set_end(ts);
        dns2.set_end(ts);
    }

    // NetworkMetricsManager::process_packet + bucket (net/v1 ...cpp:516-548,682-764)
    void net_packet(const Pkt &p)
    {
        const bool deep = net_s.draw(!cfg.net_filter_all);
        net.maybe_shift(p.ts);
        net.new_event(deep);
        NetBucket &b = net.live();
        if (cfg.net_filter_all) { // process_filtered (net/v1/NetStreamHandler.cpp:507-514)
            if (cfg.net_groups & NG_COUNTERS) b.filtered++;
            return;
        }
        // not deep: process_net_layer(dir, l3, l4, size) — counters without SYN, payload size (:518-521,620-680)
        if (cfg.net_groups & NG_COUNTERS) {
            b.total++;
            if (p.dir == DIR_FROM_HOST) b.out++;
            else if (p.dir == DIR_TO_HOST) b.in++;
            else b.unk++;
            if (p.l3 == L3_IPV6) b.IPv6++;
            else if (p.l3 == L3_IPV4) b.IPv4++;
            if (p.l4 == L4_UDP) b.UDP++;
            else if (p.l4 == L4_TCP) { b.TCP++; if (p.syn && deep) b.TCP_SYN++; }
            else b.OtherL4++;
        }
        b.payload.update(p.caplen);
        if (!deep) return;
        const bool card = cfg.net_groups & NG_CARDINALITY, tops = cfg.net_groups & NG_TOP_IPS;
        if (p.has_v4) {
            uint32_t in = 0, out = 0;
            if (p.dir == DIR_TO_HOST) in = rd32le(p.v4hdr + 12);
            else if (p.dir == DIR_FROM_HOST) out = rd32le(p.v4hdr + 16);
            if (p.l3 == L3_IPV4 && in) { if (card) b.src.update_u32(in); if (tops) b.top4.update(in); }
            if (p.l3 == L3_IPV4 && out) { if (card) b.dst.update_u32(out); if (tops) b.top4.update(out); }
        } else if (p.has_v6) {
            static const uint8_t zero[16] = {0};
            const uint8_t *in = nullptr, *out = nullptr;
            if (p.dir == DIR_TO_HOST) in = p.v6hdr + 8;
            else if (p.dir == DIR_FROM_HOST) out = p.v6hdr + 24;
            if (p.l3 == L3_IPV6 && in && memcmp(in, zero, 16)) { if (card) b.src.update_bytes(in, 16); if (tops) b.top6.update(ipv6_str(in)); }
            if (p.l3 == L3_IPV6 && out && memcmp(out, zero, 16)) { if (card) b.dst.update_bytes(out, 16); if (tops) b.top6.update(ipv6_str(out)); }
        }
    }

    // Net v2: NetworkMetricsManager::process_packet + NetworkMetricsBucket::process_packet /
    // process_net_layer(NetworkPacket&) (net/v2/NetStreamHandler.cpp:494-532,650-716,756-762).
    // Deep path (deep_sample_rate 100): toHost keeps the source address, fromHost the
    // destination, unknown both; an address counts only when the packet's l3 matches its
    // layer and it is not the unspecified address (isValid)
    // Not deep (deep_sample_rate < 100, :494-500): process_net_layer(dir, l3, l4, size), the
    // counters without SYN and the payload size
    void net2_packet(const Pkt &p)
    {
        const bool deep = net2_s.draw(true);
        net2.maybe_shift(p.ts);
        net2.new_event(deep);
        Net2Bucket &b = net2.live();
        const int d = p.dir == DIR_TO_HOST ? 0 : (p.dir == DIR_FROM_HOST ? 1 : 2);
        Net2Dir &x = b.dir[d];
        x.seen++;
        const uint32_t g = cfg.net2_groups;
        if (g & N2G_COUNTERS) {
            x.total++;
            if (p.l3 == L3_IPV6) x.IPv6++;
            else if (p.l3 == L3_IPV4) x.IPv4++;
            if (p.l4 == L4_UDP) x.UDP++;
            else if (p.l4 == L4_TCP) { x.TCP++; if (p.syn && deep) x.TCP_SYN++; }
            else x.OtherL4++;
        }
        x.payload.update(p.caplen);
        if (!deep) return;
        const bool card = g & N2G_CARDINALITY, tops = g & N2G_TOP_IPS;
        const bool want_src = d != 1, want_dst = d != 0;
        if (p.has_v4) {
            if (p.l3 != L3_IPV4) return;
            for (int side = 0; side < 2; side++) {
                if (side == 0 ? !want_src : !want_dst) continue;
                const uint32_t ip = rd32le(p.v4hdr + (side ? 16 : 12));
                if (!ip) continue;
                if (card) x.ips.update_u32(ip);
                if (tops) x.top4.update(ip);
            }
        } else if (p.has_v6) {
            if (p.l3 != L3_IPV6) return;
            static const uint8_t zero[16] = {0};
            for (int side = 0; side < 2; side++) {
                if (side == 0 ? !want_src : !want_dst) continue;
                const uint8_t *a = p.v6hdr + (side ? 24 : 8);
                if (!memcmp(a, zero, 16)) continue;
                if (card) x.ips.update_bytes(a, 16);
                if (tops) x.top6.update(ipv6_str(a));
            }
        }
    }

    // DnsStreamHandler::process_udp_packet_cb (dns/v1 ...cpp:270-302) and the manager/bucket path
    void dns_udp_packet(const Pkt &p, uint32_t flowkey)
    {
        uint16_t sport = rd16be(p.l4hdr), dport = rd16be(p.l4hdr + 2);
        auto is_dns = [](uint16_t x) { return x == 53 || x == 5353 || x == 5355 || x == 53000; };
        uint16_t metric_port = 0;
        if (is_dns(dport)) metric_port = sport;
        else if (is_dns(sport)) metric_port = dport;
        if (!metric_port) return;
        DnsEv e;
        e.msg = p.l4hdr + 8; e.len = p.l4len - 8; e.cap_end = p.data + p.caplen;
        e.ts = p.ts; e.l3 = p.l3; e.dir = p.dir; e.flowkey = flowkey; e.port = metric_port; e.tcp = false;
        dns_event(e);
    }

    // One DNS message into the handler: a UDP payload, or a message the DnsTcpSessionData
    // framing cut from a reassembled TCP stream (dns/v1 ...cpp:406-429)
    struct DnsEv {
        const uint8_t *msg, *cap_end;
        size_t len;
        TS ts;
        int l3;
        Dir dir;
        uint32_t flowkey;
        uint16_t port;
        bool tcp;
    };
    void dns_event(const DnsEv &p)
    {
        const uint32_t flowkey = p.flowkey;
        const uint16_t metric_port = p.port;
        DnsMsg m{p.msg, p.len};
        // A DNS message shorter than the 12-byte header is read past its end by
        // the reference (UB); we read the bytes that follow inside the capture, else 0.
        uint8_t hdr_buf[12];
        const uint8_t *cap_end = p.cap_end;
        for (int i = 0; i < 12; i++) hdr_buf[i] = (m.d + i < cap_end) ? m.d[i] : 0;
        DnsMsg hm = m;
        std::vector<uint8_t> tmp;
        if (m.len < 12) {
            tmp.assign(hdr_buf, hdr_buf + 12);
            hm = DnsMsg{tmp.data(), m.len};
        }
        const uint8_t *h = hm.d;
        uint16_t txid = rd16be(h);
        bool qr = (h[2] & 0x80) != 0;
        uint8_t rcode = h[3] & 0x0f;
        uint16_t ancount = rd16be(h + 6);
        if (cfg.dns2_groups) { // DNS v2: its own filters, no input predicate
            dns2_event(p, m, hm, hdr_buf, qr, rcode, ancount, txid);
            return;
        }

        // only_rcode installs a UDP predicate in the input proxy (dns/v1 ...cpp:485-508): a
        // non-response or a response whose rcode is not listed never reaches the handler
        // A TCP message takes no predicate: _filtering applies only_rcode and only_qname as
        // ordinary filters there (_predicate_filter_type stays FiltersMAX, :546-551,593-602)
        if (!p.tcp && cfg.only_rcode_mask && !cfg.exclude_noerror && (!qr || !((cfg.only_rcode_mask >> rcode) & 1))) return;
        // only_qname's predicate (:509-524): parse failure or no query never matches a listed name
        auto qname_listed = [&]() {
            DnsParse qp = m.len >= 12 ? parse_resources(m) : parse_resources_short(DnsMsg{hdr_buf, m.len});
            if (!qp.ok || !qp.has_query) return false;
            return std::find(cfg.only_qname.begin(), cfg.only_qname.end(), lower(qp.name)) != cfg.only_qname.end();
        };
        if (!p.tcp && !cfg.only_qname.empty() && !qname_listed()) return;
        // DnsStreamHandler::_filtering (:538-648) in its order; a filtered packet is
        // process_filtered: an event without a sample of its own and the `filtered` counter
        bool filt = false;
        if (cfg.exclude_noerror && rcode == 0) filt = true;
        else if (p.tcp && cfg.only_rcode_mask && !cfg.exclude_noerror && !((cfg.only_rcode_mask >> rcode) & 1)) filt = true;
        else if (cfg.has_answer_count && ancount != cfg.answer_count) filt = true;
        else if (cfg.only_queries && qr) filt = true;
        else if (cfg.only_responses && !qr) filt = true;
        else if (cfg.only_dnssec && (!qr || !ancount || !dnssec_answer(m))) filt = true;
        else if (!cfg.only_qtype.empty()) {
            DnsParse fr = m.len >= 12 ? parse_resources(m) : parse_resources_short(DnsMsg{hdr_buf, m.len});
            if (!fr.ok || !fr.has_query) filt = true;
            else if (std::find(cfg.only_qtype.begin(), cfg.only_qtype.end(), fr.qtype) == cfg.only_qtype.end()) filt = true;
        }
        else if (p.tcp && !cfg.only_qname.empty() && !qname_listed()) filt = true;
        // only_qname_suffix (:615-630): the first listed suffix the name ends with sets suffix_size
        size_t suffix_size = 0;
        if (!filt && !cfg.only_qname_suffix.empty()) {
            DnsParse sp = m.len >= 12 ? parse_resources(m) : parse_resources_short(DnsMsg{hdr_buf, m.len});
            bool hit = false;
            if (sp.ok && sp.has_query) {
                const std::string nl = lower(sp.name);
                for (const auto &sfx : cfg.only_qname_suffix)
                    if (nl.size() >= sfx.size() && nl.compare(nl.size() - sfx.size(), sfx.size(), sfx) == 0) {
                        suffix_size = sfx.size();
                        hit = true;
                        break;
                    }
            }
            filt = !hit;
        }
        if (!filt && cfg.filter_all) filt = true;
        if (filt) {
            const bool stale = dns_s.draw(false);
            if (dns.maybe_shift(p.ts)) on_dns_period_shift(p.ts);
            dns.new_event(stale);
            if (cfg.dns_groups & DG_COUNTERS) dns.live().filtered++;
            return;
        }

        // DnsStreamHandler::_configs (:648-657): public_suffix_list sets suffix_size from the
        // first query's lower-case name, only while only_qname_suffix is off
        if (cfg.psl && cfg.only_qname_suffix.empty()) {
            DnsParse pp = m.len >= 12 ? parse_resources(m) : parse_resources_short(DnsMsg{hdr_buf, m.len});
            if (pp.ok && pp.has_query) suffix_size = match_public_suffix(lower(pp.name));
        }
        // DnsMetricsManager::process_dns_layer (:1350-1370)
        const bool deep = dns_s.draw(true);
        if (dns.maybe_shift(p.ts)) on_dns_period_shift(p.ts);
        dns.new_event(deep);
        DnsBucket &b = dns.live();
        const uint32_t g = cfg.dns_groups;
        if (g & DG_COUNTERS) {
            b.total++;
            if (p.l3 == L3_IPV6) b.IPv6++;
            else if (p.l3 == L3_IPV4) b.IPv4++;
            if (p.tcp) b.TCP++;
            else b.UDP++;
            if (qr) {
                b.replies++;
                if (rcode == 0) { b.NOERROR++; if (!ancount) b.NODATA++; }
                else if (rcode == 2) b.SRVFAIL++;
                else if (rcode == 3) b.NX++;
                else if (rcode == 5) b.REFUSED++;
            } else b.queries++;
        }
        DnsParse r;
        if (deep) {
        if (g & DG_TOP_PORTS) b.udp_port.update(metric_port);
        if (m.len >= 12) r = parse_resources(m);
        else {
            DnsMsg mm{hdr_buf, m.len};
            r = parse_resources_short(mm);
        }
        }
        std::string name_lower;
        if (deep && r.ok) {
            if (qr) b.rcode.update(rcode);
            if (r.has_query) {
                name_lower = lower(r.name);
                if (g & DG_CARDINALITY) b.qname.update_str(name_lower);
                b.qtype.update(r.qtype);
                if (g & DG_TOP_QNAMES) {
                    const bool det = g & DG_TOP_QNAMES_DETAILS;
                    if (qr) {
                        if (rcode == 2) b.srvfail.update(name_lower);
                        else if (rcode == 3) b.nx.update(name_lower);
                        else if (rcode == 5) b.refused.update(name_lower);
                        else if (rcode == 0) {
                            if (det) b.noerror.update(name_lower);
                            if (!ancount) b.nodata.update(name_lower);
                        }
                        if (det) b.sized_resp.update(name_lower, m.len);
                    }
                    std::string q2, q3;
                    aggregate_domain(name_lower, suffix_size, q2, q3);
                    b.qname2.update(q2);
                    if (!q3.empty()) b.qname3.update(q3);
                }
            }
            // top_ecs (:1026-1048): a query's first additional record, its EDNS Client Subnet
            if ((g & DG_TOP_ECS) && !qr && rd16be(hm.d + 10) > 0) {
                std::string subnet = ecs_subnet(m);
                if (!subnet.empty()) {
                    if (g & DG_COUNTERS) b.query_ecs++;
                    b.ecs.update(subnet);
                }
            }
        }
        if (!(g & DG_TRANSACTIONS)) return;
        // transactions
        XactKey k{flowkey, txid};
        if (qr) {
            auto it = xacts.find(k);
            if (it != xacts.end()) {
                Xact x = it->second;
                xacts.erase(it);
                // timespec_diff (TransactionManager.h:24-37)
                TS d;
                d.sec = p.ts.sec > x.start.sec ? p.ts.sec - x.start.sec : x.start.sec - p.ts.sec;
                d.nsec = p.ts.nsec - x.start.nsec;
                if (d.nsec < 0) { d.sec--; d.nsec += 1000000000L; }
                bool timed_out = false;
                if (d.sec > (int64_t)ttl_s) timed_out = true;
                else if (d.sec == (int64_t)ttl_s && (d.nsec / 1.0e6) >= ttl_ms) timed_out = true;
                if (timed_out) b.xacts_timed_out++;
                else new_xact(b, p, d, x, r, deep);
            }
        } else {
            xacts[k] = Xact{p.ts, m.len};
        }
    }

    // ---------------------------------------------------------------- DNS v2
    // DnsMetricsManager::process_dns_layer, v2 (dns/v2/DnsStreamHandler.cpp:1100-1145): every
    // message is an event; a query opens a transaction in its direction's map (toHost query:
    // "in"), a response looks in the swapped direction's map and accounts the transaction
    // DnsStreamHandler::_filtering, v2 (dns/v2/DnsStreamHandler.cpp:484-609): the direction
    // filters for both kinds, rcode / answer_count / DNSSEC / qtype on responses, qname and
    // qname suffix on queries (the suffix size it sets is consumed by the query's own
    // process_dns_layer, which does not use it: a response always aggregates with 0)
    bool dns2_filtering(const DnsEv &p, const DnsMsg &m, const uint8_t *hdr12, bool qr, uint8_t rcode, uint16_t ancount)
    {
        const uint32_t dis = cfg.xact_dirs_disabled;
        if ((dis & 4) && p.dir == DIR_UNKNOWN) return true;
        auto parsed = [&]() { return m.len >= 12 ? parse_resources(m) : parse_resources_short(DnsMsg{hdr12, m.len}); };
        if (qr) {
            if ((dis & 1) && p.dir == DIR_FROM_HOST) return true;
            if ((dis & 2) && p.dir == DIR_TO_HOST) return true;
            if (cfg.exclude_noerror) { if (rcode == 0) return true; }
            else if (cfg.only_rcode_mask && !((cfg.only_rcode_mask >> rcode) & 1)) return true;
            if (cfg.has_answer_count && ancount != cfg.answer_count) return true;
            if (cfg.only_dnssec && (!ancount || !dnssec_answer(m))) return true;
            if (!cfg.only_qtype.empty()) {
                DnsParse fr = parsed();
                if (!fr.ok || !fr.has_query) return true;
                if (std::find(cfg.only_qtype.begin(), cfg.only_qtype.end(), fr.qtype) == cfg.only_qtype.end()) return true;
            }
        } else {
            if ((dis & 1) && p.dir == DIR_TO_HOST) return true;
            if ((dis & 2) && p.dir == DIR_FROM_HOST) return true;
            if (!cfg.only_qname.empty()) {
                DnsParse qp = parsed();
                if (!qp.ok || !qp.has_query) return true;
                if (std::find(cfg.only_qname.begin(), cfg.only_qname.end(), lower(qp.name)) == cfg.only_qname.end()) return true;
            }
            if (!cfg.only_qname_suffix.empty()) {
                DnsParse sp = parsed();
                if (!sp.ok || !sp.has_query) return true;
                const std::string nl = lower(sp.name);
                bool hit = false;
                for (const auto &sfx : cfg.only_qname_suffix)
                    if (nl.size() >= sfx.size() && nl.compare(nl.size() - sfx.size(), sfx.size(), sfx) == 0) { hit = true; break; }
                if (!hit) return true;
            }
        }
        return false;
    }

    void dns2_event(const DnsEv &p, const DnsMsg &m, const DnsMsg &hm, const uint8_t *hdr12, bool qr, uint8_t rcode,
                    uint16_t ancount, uint16_t txid)
    {
        const uint8_t *h = hm.d;
        size_t suffix_size = 0; // DnsStreamHandler::_configs, v2 (:612-619): set below for a response
        const bool filt = dns2_filtering(p, m, hdr12, qr, rcode, ancount);
        // new_event(stamp) draws; process_filtered's new_event(stamp, false) keeps the last flag
        const bool deep = dns2_s.draw(!filt);
        if (dns2.maybe_shift(p.ts)) on_dns2_period_shift(p.ts);
        dns2.new_event(deep);
        Dns2Bucket &b = dns2.live();
        const uint32_t g = cfg.dns2_groups;
        const XactKey k{p.flowkey, txid};
        auto elapsed = [&](const Xact2 &q) {
            TS d;
            d.sec = p.ts.sec > q.start.sec ? p.ts.sec - q.start.sec : q.start.sec - p.ts.sec;
            d.nsec = p.ts.nsec - q.start.nsec;
            if (d.nsec < 0) { d.sec--; d.nsec += 1000000000L; }
            return d;
        };
        auto timed_out = [&](const TS &d) { return d.sec > (int64_t)ttl_s || (d.sec == (int64_t)ttl_s && (d.nsec / 1.0e6) >= ttl_ms); };
        if (filt) {
            // DnsMetricsManager::process_filtered, v2 (:1147-1174)
            if (qr) {
                const int xd = p.dir == DIR_TO_HOST ? 1 : (p.dir == DIR_FROM_HOST ? 0 : 2);
                auto it = xacts2[xd].find(k);
                b.dir[xd].seen = true;
                if (it != xacts2[xd].end()) {
                    const Xact2 q = it->second;
                    xacts2[xd].erase(it);
                    if (!timed_out(elapsed(q)) && !q.filtered && (g & D2G_COUNTERS)) b.filtered++;
                }
            } else {
                const int xd = p.dir == DIR_TO_HOST ? 0 : (p.dir == DIR_FROM_HOST ? 1 : 2);
                Xact2 q{p.ts, 0, false, std::string()};
                q.filtered = true;
                xacts2[xd][k] = q;
            }
            if (g & D2G_COUNTERS) b.filtered++;
            return;
        }
        if (qr) {
            const int xd = p.dir == DIR_TO_HOST ? 1 : (p.dir == DIR_FROM_HOST ? 0 : 2);
            Dns2Dir &x = b.dir[xd];
            x.seen = true;
            auto it = xacts2[xd].find(k);
            if (it == xacts2[xd].end()) { x.orphan++; return; }
            Xact2 q = it->second;
            xacts2[xd].erase(it);
            const TS d = elapsed(q);
            if (q.filtered) { if (g & D2G_COUNTERS) b.filtered++; return; } // the query was filtered out
            if (timed_out(d)) { x.timeout++; return; }
            // DnsMetricsBucket::new_dns_transaction, v2 (:925-1089)
            const uint64_t us = (uint64_t)((d.sec * 1000000000LL) + d.nsec) / 1000;
            if (g & D2G_COUNTERS) {
                x.xacts++;
                if (p.l3 == L3_IPV6) x.IPv6++;
                else if (p.l3 == L3_IPV4) x.IPv4++;
                if (p.tcp) x.TCP++;
                else x.UDP++;
                if (q.cd) x.CD++;
                if (rcode == 0) { x.NOERROR++; if (!ancount) x.NODATA++; }
                else if (rcode == 2) x.SRVFAIL++;
                else if (rcode == 3) x.NX++;
                else if (rcode == 5) x.REFUSED++;
                if (h[2] & 0x04) x.AA++;
                if (h[3] & 0x20) x.AD++;
            }
            if (!deep) return; // new_dns_transaction v2 (:1006-1008): the rest only when deep
            if (q.query_size && (g & D2G_TOP_SIZE)) x.ratio.update((double)m.len / (double)q.query_size);
            if (p.port && (g & D2G_TOP_PORTS)) x.port.update(p.port);
            if (g & D2G_XACT_TIMES) { x.time.update(us); x.hist.update(us); }
            DnsParse r = m.len >= 12 ? parse_resources(m) : parse_resources_short(DnsMsg{h, m.len});
            if (r.ok) {
                x.rcode.update(rcode);
                if (r.has_query) {
                    const std::string name = lower(r.name);
                    // public_suffix_list while only_qname_suffix is off: match_public_suffix of the
                    // response's first query name, new_dns_transaction's suffix_size (:1067-1072)
                    if (cfg.psl && cfg.only_qname_suffix.empty()) suffix_size = match_public_suffix(name);
                    if (g & D2G_CARDINALITY) x.qname.update_str(name);
                    x.qtype.update(r.qtype);
                    if (g & D2G_TOP_RCODES) {
                        if (rcode == 2) x.srvfail.update(name);
                        else if (rcode == 3) x.nx.update(name);
                        else if (rcode == 5) x.refused.update(name);
                        else if (rcode == 0) { x.noerror.update(name); if (!ancount) x.nodata.update(name); }
                    }
                    if (g & D2G_TOP_SIZE) x.sized.update(name, m.len);
                    if (per90_2[xd] > 0 && (float)us >= per90_2[xd] && (g & D2G_XACT_TIMES)) x.slow.update(name);
                    if (g & D2G_TOP_QNAMES) {
                        std::string q2, q3;
                        aggregate_domain(name, suffix_size, q2, q3);
                        x.qname2.update(q2);
                        if (!q3.empty()) x.qname3.update(q3);
                    }
                }
                if ((g & D2G_TOP_ECS) && !q.ecs.empty()) {
                    if (g & D2G_COUNTERS) x.ECS++;
                    x.ecs.update(q.ecs);
                }
            }
        } else {
            const int xd = p.dir == DIR_TO_HOST ? 0 : (p.dir == DIR_FROM_HOST ? 1 : 2);
            std::string subnet;
            if ((g & D2G_TOP_ECS) && m.len >= 12 && rd16be(h + 10) > 0) subnet = ecs_subnet(m);
            xacts2[xd][k] = Xact2{p.ts, m.len, (h[3] & 0x10) != 0, subnet};
        }
    }

    // DnsMetricsManager::on_period_shift, v2 (dns/v2/DnsStreamHandler.h:440-453)
    void on_dns2_period_shift(TS ts)
    {
        for (int d = 0; d < 3; d++) {
            uint64_t timed_out = 0;
            for (auto it = xacts2[d].begin(); it != xacts2[d].end();) {
                if (ts.sec >= (int64_t)ttl_s + it->second.start.sec) { it = xacts2[d].erase(it); timed_out++; }
                else ++it;
            }
            if (timed_out) { dns2.live().dir[d].seen = true; dns2.live().dir[d].timeout += timed_out; }
            const Dns2Bucket &b1 = *dns2.buckets.at(1);
            if (b1.dir[d].seen && !b1.dir[d].time.empty()) per90_2[d] = (float)b1.dir[d].time.p(0.90);
        }
    }

    // header-only message (< 12 bytes): the counts come from the padded header copy
    DnsParse parse_resources_short(const DnsMsg &m)
    {
        DnsParse r;
        uint16_t qd = rd16be(m.d + 4), an = rd16be(m.d + 6), ns = rd16be(m.d + 8), ar = rd16be(m.d + 10);
        uint32_t total = (uint32_t)qd + an + ns + ar;
        if (total > 100) return r;
        if (total == 0) { r.ok = true; return r; }
        return r; // first resource starts at offset 12 > len: out of bounds
    }

    // DnsMetricsBucket::new_dns_transaction (:1093-1138)
    void new_xact(DnsBucket &b, const DnsEv &p, TS d, const Xact &x, const DnsParse &r, bool deep)
    {
        uint64_t us = (uint64_t)((d.sec * 1000000000LL) + d.nsec) / 1000;
        const bool q = deep && (cfg.dns_groups & DG_QUANTILES), h = deep && (cfg.dns_groups & DG_HISTOGRAMS);
        b.xacts_total++;
        if (p.dir == DIR_TO_HOST) { b.xacts_out++; if (q) b.xact_from.update(us); if (h) b.hist_from.update(us); }
        else if (p.dir == DIR_FROM_HOST) { b.xacts_in++; if (q) b.xact_to.update(us); if (h) b.hist_to.update(us); }
        if (!deep) return; // new_dns_transaction (:1121-1136): ratio and slow tops only when deep
        size_t resp_len = p.len;
        if (x.query_size) b.ratio.update((double)resp_len / (double)x.query_size);
        if (r.ok && r.has_query) {
            if (p.dir == DIR_TO_HOST && from90 > 0 && (float)us >= from90) b.slow_out.update(r.name);
            else if (p.dir == DIR_FROM_HOST && to90 > 0 && (float)us >= to90) b.slow_in.update(r.name);
        }
    }

    // DnsMetricsManager::on_period_shift (dns/v1/DnsStreamHandler.h:252-267)
    void on_dns_period_shift(TS ts)
    {
        uint64_t timed_out = 0;
        for (auto it = xacts.begin(); it != xacts.end();) {
            if (ts.sec >= (int64_t)ttl_s + it->second.start.sec) { it = xacts.erase(it); timed_out++; }
            else ++it;
        }
        if (timed_out) dns.live().xacts_timed_out += timed_out;
        const DnsBucket &b1 = *dns.buckets.at(1);
        if (!b1.xact_from.empty()) from90 = (float)b1.xact_from.p(0.90);
        if (!b1.xact_to.empty()) to90 = (float)b1.xact_to.p(0.90);
    }

    // ------------------------------------------------------------ DNS over TCP
    // PcapPlusPlus 23.09 TcpReassembly (third-party, not vendored in the reference; its
    // algorithm restated here) as PcapInputStream drives it (PcapInputStream.cpp:75-79,
    // 254-283, 429-465): config removeConnInfo, closedConnectionDelay 1 s, maxOutOfOrder 50.
    // A closed connection's info is purged by wall clock (time(nullptr)), which a replay
    // cannot reproduce; here a closed flow stays closed for the rest of the run.
    struct TcpFrag {
        uint32_t seq;
        std::vector<uint8_t> data;
    };
    struct TcpSide {
        uint8_t ip[16] = {0};
        bool v6 = false;
        uint16_t port = 0;
        uint32_t seq = 0;
        bool fin = false; // gotFinOrRst
        std::vector<TcpFrag> frags;
    };
    struct DnsTcpSession { // DnsTcpSessionData (dns/v1/DnsStreamHandler.cpp:337-373)
        std::vector<uint8_t> buf;
        bool invalid = false;
    };
    struct TcpConn {
        TcpSide side[2];
        int nsides = 0, prev = -1;
        bool closed = false;
        TS end;                 // ConnectionData::endTime (timeval precision), {0,0} until a 2nd packet
        uint16_t sport = 0, dport = 0;
        bool v4 = true;
        // DnsStreamHandler::_tcp_connections entry (TcpFlowData)
        bool tracked = false;
        uint16_t port = 0;
        std::unique_ptr<DnsTcpSession> sess[2];
    };
    static constexpr size_t MIN_DNS_QUERY_SIZE = 17;
    static constexpr size_t TCP_MAX_OOO = 50;
    static constexpr int64_t TCP_TIMEOUT = 30;       // PcapInputStream.h:97
    static constexpr int MAX_TCP_CLEANUPS = 100;     // PcapInputStream.h:98
    std::unordered_map<uint32_t, TcpConn> tcp_conns;
    std::list<std::pair<uint32_t, TS>> lru; // VisorLRUList: front = most recently put
    std::unordered_map<uint32_t, std::list<std::pair<uint32_t, TS>>::iterator> lru_at;
    std::vector<uint32_t> lru_overflow;
    Dir tcp_dir = DIR_UNKNOWN; // _packet_dir_cache of the packet being reassembled
    uint64_t rec_no = 0;       // records seen (debug log of TCP messages: PVO_TCP_LOG)
    FILE *tcp_log = nullptr;
    bool ooo_busy = false;     // m_ProcessingOutOfOrder

    static bool seq_lt(uint32_t a, uint32_t b) { return (int32_t)(a - b) < 0; }
    static bool seq_gt(uint32_t a, uint32_t b) { return (int32_t)(b - a) < 0; }
    static bool is_dns_port(uint16_t x) { return x == 53 || x == 5353 || x == 5355 || x == 53000; }

    void lru_put(uint32_t fk, TS t)
    {
        auto it = lru_at.find(fk);
        if (it != lru_at.end()) lru.erase(it->second);
        lru.emplace_front(fk, t);
        lru_at[fk] = lru.begin();
        if (cfg.tcp_cache_limit && lru_at.size() > cfg.tcp_cache_limit) {
            uint32_t old = lru.back().first;
            lru_at.erase(old);
            lru.pop_back();
            lru_overflow.push_back(old);
        }
    }
    void lru_erase(uint32_t fk)
    {
        auto it = lru_at.find(fk);
        if (it == lru_at.end()) return;
        lru.erase(it->second);
        lru_at.erase(it);
    }

    // DnsStreamHandler::tcp_connection_start_cb (:438-455) / tcp_connection_end_cb (:457-469)
    void conn_track(TcpConn &c)
    {
        uint16_t mp = is_dns_port(c.dport) ? c.sport : (is_dns_port(c.sport) ? c.dport : 0);
        if (!c.tracked && mp) { c.tracked = true; c.port = mp; }
    }
    void conn_untrack(TcpConn &c)
    {
        c.tracked = false;
        c.sess[0].reset();
        c.sess[1].reset();
    }

    // onMessageReady -> PcapInputStream::tcp_message_ready (PcapInputStream.cpp:254-263) ->
    // DnsStreamHandler::tcp_message_ready_cb (:375-436) -> DnsTcpSessionData framing
    void tcp_deliver(uint32_t fk, TcpConn &c, int side, const uint8_t *d, size_t n)
    {
        conn_track(c);
        if (c.tracked) {
            if (!c.sess[side]) c.sess[side].reset(new DnsTcpSession());
            DnsTcpSession &s = *c.sess[side];
            if (!s.invalid) {
                s.buf.insert(s.buf.end(), d, d + n);
                size_t pos = 0;
                for (;;) {
                    if (s.buf.size() - pos < MIN_DNS_QUERY_SIZE + 2) break;
                    size_t size = ((size_t)s.buf[pos] << 8) | s.buf[pos + 1];
                    if (size < MIN_DNS_QUERY_SIZE) { s.buf.clear(); pos = 0; s.invalid = true; break; }
                    if (s.buf.size() - pos < 2 + size) break;
                    std::vector<uint8_t> msg(s.buf.begin() + pos + 2, s.buf.begin() + pos + 2 + size);
                    pos += 2 + size;
                    if (tcp_log) fprintf(tcp_log, "%llu %u %u %lld %lld\n", (unsigned long long)rec_no, (unsigned)size,
                                         (unsigned)((msg[0] << 8) | msg[1]), (long long)c.end.sec, (long long)c.end.nsec);
                    DnsEv e;
                    e.msg = msg.data(); e.len = size; e.cap_end = msg.data() + size;
                    e.ts = c.end; e.l3 = c.v4 ? L3_IPV4 : L3_IPV6; e.dir = tcp_dir;
                    e.flowkey = fk; e.port = c.port; e.tcp = true;
                    dns_event(e);
                }
                if (pos) s.buf.erase(s.buf.begin(), s.buf.begin() + pos);
            }
        }
        lru_put(fk, c.end);
    }

    // TcpReassembly::checkOutOfOrderFragments
    void tcp_check_ooo(uint32_t fk, TcpConn &c, int side, bool clean)
    {
        if (ooo_busy) return;
        ooo_busy = true;
        TcpSide &s = c.side[side];
        bool found;
        do {
            do {
                found = false;
                size_t i = 0;
                while (i < s.frags.size()) {
                    TcpFrag &f = s.frags[i];
                    if (f.seq == s.seq) {
                        s.seq += (uint32_t)f.data.size();
                        std::vector<uint8_t> d = std::move(f.data);
                        s.frags.erase(s.frags.begin() + i);
                        tcp_deliver(fk, c, side, d.data(), d.size());
                        found = true;
                        continue;
                    }
                    if (seq_lt(f.seq, s.seq)) {
                        uint32_t nseq = f.seq + (uint32_t)f.data.size();
                        std::vector<uint8_t> d = std::move(f.data);
                        s.frags.erase(s.frags.begin() + i);
                        if (seq_gt(nseq, s.seq)) {
                            uint32_t nl = s.seq - (nseq - (uint32_t)d.size());
                            s.seq += (uint32_t)d.size() - nl;
                            tcp_deliver(fk, c, side, d.data() + nl, d.size() - nl);
                            found = true;
                        }
                        continue;
                    }
                    i++;
                }
            } while (found);
            if (!clean && s.frags.size() <= TCP_MAX_OOO) break;
            // missing data: deliver the fragment with the lowest sequence behind a
            // "[N bytes missing]" text, then start over
            int best = -1;
            uint32_t closest = 0xffffffffu;
            for (size_t i = 0; i < s.frags.size(); i++)
                if (best < 0 || seq_lt(s.frags[i].seq, closest)) { closest = s.frags[i].seq; best = (int)i; }
            if (best >= 0) {
                TcpFrag f = std::move(s.frags[best]);
                s.frags.erase(s.frags.begin() + best);
                uint32_t missing = f.seq - s.seq;
                s.seq = f.seq + (uint32_t)f.data.size();
                std::string text = "[" + std::to_string(missing) + " bytes missing]";
                std::vector<uint8_t> d(text.begin(), text.end());
                d.insert(d.end(), f.data.begin(), f.data.end());
                tcp_deliver(fk, c, side, d.data(), d.size());
                found = true;
            }
        } while (found);
        ooo_busy = false;
    }

    // TcpReassembly::closeConnectionInternal
    void tcp_close(uint32_t fk)
    {
        auto it = tcp_conns.find(fk);
        if (it == tcp_conns.end() || it->second.closed) return;
        TcpConn &c = it->second;
        tcp_check_ooo(fk, c, 0, true);
        tcp_check_ooo(fk, c, 1, true);
        conn_untrack(c);  // onConnectionEnd -> tcp_connection_end
        lru_erase(fk);
        c.closed = true;
    }

    // TcpReassembly::handleFinOrRst
    void tcp_fin_rst(uint32_t fk, TcpConn &c, int side, bool rst)
    {
        if (c.side[side].fin) return;
        c.side[side].fin = true;
        if (c.side[1 - side].fin || rst) tcp_close(fk);
        else tcp_check_ooo(fk, c, side, true);
    }

    // TcpReassembly::reassemblePacket
    void tcp_reassemble(const Pkt &p)
    {
        if (!p.ip1) return;                          // NonIpPacket
        const uint8_t *th = p.l4hdr;
        size_t hl = (size_t)(th[12] >> 4) * 4;
        if (hl < 20 || hl > p.l4len) return;         // no TcpLayer (TcpLayer::isDataValid)
        const uint8_t *pl = th + hl;
        const uint32_t plen = (uint32_t)(p.l4len - hl);
        const bool syn = th[13] & 0x02, fin = th[13] & 0x01, rst = th[13] & 0x04;
        if (plen == 0 && !syn && !fin && !rst) return; // Ignore_PacketWithNoData
        const uint32_t fk = hash5tuple(p);
        const uint16_t sport = rd16be(th), dport = rd16be(th + 2);
        const uint8_t *src = p.ip1 + (p.ip1_v6 ? 8 : 12);
        const size_t alen = p.ip1_v6 ? 16 : 4;
        TS now{p.ts.sec, p.ts.nsec / 1000 * 1000}; // timespec -> ConnectionData timeval
        auto it = tcp_conns.find(fk);
        TcpConn *cp;
        if (it == tcp_conns.end()) {
            cp = &tcp_conns[fk];
            cp->sport = sport; cp->dport = dport; cp->v4 = !p.ip1_v6;
            // onConnectionStart -> tcp_connection_start (PcapInputStream.cpp:265-274)
            conn_track(*cp);
            lru_put(fk, now);
        } else {
            cp = &it->second;
            if (cp->closed) return;                  // Ignore_PacketOfClosedFlow
            if (now.sec > cp->end.sec || (now.sec == cp->end.sec && now.nsec > cp->end.nsec)) cp->end = now;
        }
        TcpConn &c = *cp;
        int side = -1;
        bool first = false;
        auto is_side = [&](int k) {
            return c.side[k].port == sport && c.side[k].v6 == p.ip1_v6 && !memcmp(c.side[k].ip, src, alen);
        };
        if (c.nsides < 2 && !(c.nsides == 1 && is_side(0))) {
            side = c.nsides++;
            memcpy(c.side[side].ip, src, alen);
            c.side[side].v6 = p.ip1_v6;
            c.side[side].port = sport;
            first = true;
        } else if (is_side(0)) side = 0;
        else if (c.nsides == 2 && is_side(1)) side = 1;
        else return;                                 // Error_PacketDoesNotMatchFlow
        TcpSide &s = c.side[side];
        if (s.fin) return;
        if ((fin || rst) && plen == 0) { tcp_fin_rst(fk, c, side, rst); return; }
        if (c.prev != -1 && c.prev != side) tcp_check_ooo(fk, c, c.prev, true);
        c.prev = side;
        const uint32_t seq = ((uint32_t)th[4] << 24) | ((uint32_t)th[5] << 16) | ((uint32_t)th[6] << 8) | th[7];
        if (first) {
            s.seq = seq + plen + (syn ? 1 : 0);
            if (plen) tcp_deliver(fk, c, side, pl, plen);
        } else if (seq_lt(seq, s.seq)) {
            uint32_t nseq = seq + plen;
            if (seq_gt(nseq, s.seq)) {
                uint32_t nl = s.seq - seq;
                s.seq += plen - nl;
                tcp_deliver(fk, c, side, pl + nl, plen - nl);
            }
        } else if (seq == s.seq) {
            if (plen) {
                s.seq += plen + (syn ? 1 : 0);
                tcp_deliver(fk, c, side, pl, plen);
                tcp_check_ooo(fk, c, side, false);
            }
        } else if (plen) {
            s.frags.push_back(TcpFrag{seq, std::vector<uint8_t>(pl, pl + plen)});
            if (s.frags.size() > TCP_MAX_OOO) tcp_check_ooo(fk, c, side, true);
        }
        if (fin || rst) tcp_fin_rst(fk, c, side, rst);
    }

    // PcapInputStream::process_raw_packet, TCP branch (PcapInputStream.cpp:429-465)
    void tcp_packet(const Pkt &p)
    {
        tcp_reassemble(p);
        for (int k = 0; k < MAX_TCP_CLEANUPS && !lru.empty(); k++) {
            auto back = lru.back();
            if (p.ts.sec < back.second.sec + TCP_TIMEOUT) break;
            tcp_close(back.first);
            lru_erase(back.first);
        }
        // indexed: a close can flush data whose LRU put overflows again
        for (size_t k = 0; k < lru_overflow.size(); k++) tcp_close(lru_overflow[k]);
        lru_overflow.clear();
    }

    // TcpReassembly::closeAllConnections at the end of the capture (PcapInputStream.cpp:243-244)
    void tcp_close_all()
    {
        std::vector<uint32_t> keys;
        for (auto &kv : tcp_conns)
            if (!kv.second.closed) keys.push_back(kv.first);
        std::sort(keys.begin(), keys.end());
        for (uint32_t fk : keys) tcp_close(fk);
    }

    void process(const Pkt &p0)
    {
        Pkt p = p0;
        parse_packet(p, linktype);
        set_direction(p, cfg);
        tcp_dir = p.dir;
        net_packet(p);
        if (cfg.net2_groups) net2_packet(p);
        if (p.l4 == L4_UDP) dns_udp_packet(p, hash5tuple(p));
        else if (p.l4 == L4_TCP) tcp_packet(p);
        rec_no++;
    }
};

// ---------------------------------------------------------------- JSON rendering
static thread_local uint32_t topn_pct = 0; // topn_percentile_threshold of the current run

// TopN::to_json (src/Metrics.h:510-521,577-590): the first n by estimate, cut at the first one
// below the topn_percentile_threshold quantile (KLL inclusive rule) of those n estimates
template <typename K, typename F>
static void top_json(J &j, const std::string &key, const ExactTop<K> &t, size_t n, F fmt)
{
    std::vector<std::pair<std::string, uint64_t>> v;
    for (auto &kv : t.m) v.push_back({fmt(kv.first), kv.second});
    std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) {
        if (a.second != b.second) return a.second > b.second;
        return a.first < b.first;
    });
    const size_t k = std::min(n, v.size());
    ExactQuantile<uint64_t> est;
    for (size_t i = 0; i < k; i++) est.update(v[i].second);
    const uint64_t thr = k ? est.p((double)topn_pct / 100.0) : 0;
    j.key(key);
    j.arr();
    for (size_t i = 0; i < k && v[i].second >= thr; i++) {
        j.obj();
        j.key("name"); j.str(v[i].first);
        j.key("estimate"); j.u64(v[i].second);
        j.end_obj();
    }
    j.end_arr();
}

template <typename T>
static void quant_json(J &j, const std::string &key, const ExactQuantile<T> &q)
{
    if (q.empty()) return;
    auto v = q.quantiles();
    const char *names[4] = {"p50", "p90", "p95", "p99"};
    j.key(key);
    j.obj();
    for (int i = 0; i < 4; i++) {
        j.key(names[i]);
        if constexpr (std::is_floating_point<T>::value) j.dbl(v[i]);
        else j.u64((uint64_t)v[i]);
    }
    j.end_obj();
}

static std::string id_str(const std::string &s) { return s; }

// Histogram::to_json (src/Metrics.h:243-262) on exact data: the split points are the distinct
// uint64 values of 10^(b/18) * 10^e (e in [-9, 18), b in [0, 18)); a point is kept when the
// inclusive PMF interval ending at it holds an item; each kept point's value is the inclusive
// CDF times n (a double), then "+Inf" = n
static void hist_json(J &j, const std::string &key, const ExactQuantile<uint64_t> &h)
{
    if (h.empty()) return;
    std::vector<uint64_t> pts;
    for (int e = -9; e < 18; e++)
        for (int k = 0; k < 18; k++) {
            const float f = static_cast<float>(k) / 18;
            const uint64_t v = static_cast<uint64_t>(std::pow(10.0, f) * std::pow(10.0, e));
            if (pts.empty() || pts.back() != v) pts.push_back(v);
        }
    std::vector<uint64_t> s = h.v;
    std::sort(s.begin(), s.end());
    const double n = (double)s.size();
    auto le = [&](uint64_t x) { return (uint64_t)(std::upper_bound(s.begin(), s.end(), x) - s.begin()); };
    j.key(key); j.obj();
    j.key("buckets"); j.obj();
    uint64_t prev = 0;
    for (uint64_t x : pts) {
        const uint64_t c = le(x);
        if (c != prev) { j.key(std::to_string(x)); j.dbl(((double)c / n) * n); }
        prev = c;
    }
    j.key("+Inf"); j.dbl(1.0 * n);
    j.end_obj();
    j.end_obj();
}

static void net_json(J &j, const NetBucket &b, size_t topn, uint32_t g)
{
    j.key("period"); j.obj();
    j.key("start_ts"); j.i64(b.start.sec);
    j.key("length"); j.u64(b.period_length);
    j.end_obj();
    j.key("events"); j.u64(b.num_events);
    j.key("deep_samples"); j.u64(b.num_samples);
    if (g & NG_COUNTERS) {
        j.key("udp"); j.u64(b.UDP);
        j.key("tcp"); j.u64(b.TCP);
        j.key("protocol"); j.obj(); j.key("tcp"); j.obj(); j.key("syn"); j.u64(b.TCP_SYN); j.end_obj(); j.end_obj();
        j.key("other_l4"); j.u64(b.OtherL4);
        j.key("ipv4"); j.u64(b.IPv4);
        j.key("ipv6"); j.u64(b.IPv6);
        j.key("in"); j.u64(b.in);
        j.key("out"); j.u64(b.out);
        j.key("unknown_dir"); j.u64(b.unk);
        j.key("total"); j.u64(b.total);
        j.key("filtered"); j.u64(b.filtered);
    }
    if (g & NG_CARDINALITY) {
        j.key("cardinality"); j.obj();
        j.key("src_ips_in"); j.i64(lround(b.src.estimate()));
        j.key("dst_ips_out"); j.i64(lround(b.dst.estimate()));
        j.end_obj();
    }
    if (g & NG_TOP_IPS) {
        top_json(j, "top_ipv4", b.top4, topn, ipv4_str);
        top_json(j, "top_ipv6", b.top6, topn, id_str);
    }
    if (g & NG_TOP_GEO) {
        j.key("top_geoLoc"); j.arr(); j.end_arr();
        j.key("top_ASN"); j.arr(); j.end_arr();
    }
    quant_json(j, "payload_size", b.payload);
}

// NetworkMetricsBucket::to_json, Net v2 (net/v2/NetStreamHandler.cpp:436-484); rates excluded
static void net2_json(J &j, const Net2Bucket &b, size_t topn, uint32_t g)
{
    j.key("period"); j.obj();
    j.key("start_ts"); j.i64(b.start.sec);
    j.key("length"); j.u64(b.period_length);
    j.end_obj();
    j.key("observed_packets"); j.u64(b.num_events);
    j.key("deep_sampled_packets"); j.u64(b.num_samples);
    if (g & N2G_COUNTERS) { j.key("filtered_packets"); j.u64(b.filtered); }
    static const char *names[3] = {"in", "out", "unknown"};
    for (int d = 0; d < 3; d++) {
        const Net2Dir &x = b.dir[d];
        if (!x.seen) continue;
        j.key(names[d]); j.obj();
        if (g & N2G_COUNTERS) {
            j.key("udp_packets"); j.u64(x.UDP);
            j.key("tcp_packets"); j.u64(x.TCP);
            j.key("other_l4_packets"); j.u64(x.OtherL4);
            j.key("ipv4_packets"); j.u64(x.IPv4);
            j.key("ipv6_packets"); j.u64(x.IPv6);
            j.key("tcp"); j.obj(); j.key("syn_packets"); j.u64(x.TCP_SYN); j.end_obj();
            j.key("total_packets"); j.u64(x.total);
        }
        if (g & N2G_CARDINALITY) {
            j.key("cardinality"); j.obj();
            j.key("ips"); j.i64(lround(x.ips.estimate()));
            j.end_obj();
        }
        if (g & N2G_TOP_IPS) {
            top_json(j, "top_ipv4_packets", x.top4, topn, ipv4_str);
            top_json(j, "top_ipv6_packets", x.top6, topn, id_str);
        }
        if (g & N2G_TOP_GEO) {
            j.key("top_geo_loc_packets"); j.arr(); j.end_arr();
            j.key("top_asn_packets"); j.arr(); j.end_arr();
        }
        if (g & N2G_QUANTILES) quant_json(j, "payload_size_bytes", x.payload);
        j.end_obj();
    }
}

// DnsMetricsBucket::to_json, DNS v2 (dns/v2/DnsStreamHandler.cpp:678-757); rates excluded
static void dns2_json(J &j, const Dns2Bucket &b, size_t topn, uint32_t g)
{
    auto u16s = [](const uint16_t &v) { return std::to_string(v); };
    auto rc = [](const uint16_t &v) { auto &m = rcode_names(); auto it = m.find(v); return it != m.end() ? it->second : std::to_string(v); };
    auto qt = [](const uint16_t &v) { auto &m = qtype_names(); auto it = m.find(v); return it != m.end() ? it->second : std::to_string(v); };
    j.key("period"); j.obj();
    j.key("start_ts"); j.i64(b.start.sec);
    j.key("length"); j.u64(b.period_length);
    j.end_obj();
    j.key("observed_packets"); j.u64(b.num_events);
    j.key("deep_sampled_packets"); j.u64(b.num_samples);
    if (g & D2G_COUNTERS) { j.key("filtered_packets"); j.u64(b.filtered); }
    static const char *names[3] = {"in", "out", "unknown"};
    for (int d = 0; d < 3; d++) {
        const Dns2Dir &x = b.dir[d];
        if (!x.seen) continue;
        j.key(names[d]); j.obj();
        if (g & D2G_COUNTERS) {
            const std::pair<const char *, uint64_t> ctr[] = {
                {"xacts", x.xacts}, {"udp_xacts", x.UDP}, {"tcp_xacts", x.TCP}, {"dot_xacts", 0}, {"doh_xacts", 0},
                {"dnscrypt_udp_xacts", 0}, {"dnscrypt_tcp_xacts", 0}, {"doq_xacts", 0}, {"ipv4_xacts", x.IPv4},
                {"ipv6_xacts", x.IPv6}, {"nxdomain_xacts", x.NX}, {"ecs_xacts", x.ECS}, {"refused_xacts", x.REFUSED},
                {"srvfail_xacts", x.SRVFAIL}, {"noerror_xacts", x.NOERROR}, {"nodata_xacts", x.NODATA},
                {"authenticated_data_xacts", x.AD}, {"authoritative_answer_xacts", x.AA},
                {"checking_disabled_xacts", x.CD}, {"timeout_queries", x.timeout}, {"orphan_responses", x.orphan}};
            for (auto &c : ctr) { j.key(c.first); j.u64(c.second); }
        }
        if (g & D2G_CARDINALITY) { j.key("cardinality"); j.obj(); j.key("qname"); j.i64(lround(x.qname.estimate())); j.end_obj(); }
        if (g & D2G_TOP_PORTS) top_json(j, "top_udp_ports_xacts", x.port, topn, u16s);
        if (g & D2G_TOP_ECS) {
            j.key("top_geo_loc_ecs_xacts"); j.arr(); j.end_arr();
            j.key("top_asn_ecs_xacts"); j.arr(); j.end_arr();
            top_json(j, "top_ecs_xacts", x.ecs, topn, id_str);
        }
        if (g & D2G_TOP_RCODES) {
            top_json(j, "top_nxdomain_xacts", x.nx, topn, id_str);
            top_json(j, "top_refused_xacts", x.refused, topn, id_str);
            top_json(j, "top_srvfail_xacts", x.srvfail, topn, id_str);
            top_json(j, "top_nodata_xacts", x.nodata, topn, id_str);
            top_json(j, "top_noerror_xacts", x.noerror, topn, id_str);
            top_json(j, "top_rcode_xacts", x.rcode, topn, rc);
        }
        if (g & D2G_TOP_QNAMES) {
            top_json(j, "top_qname2_xacts", x.qname2, topn, id_str);
            top_json(j, "top_qname3_xacts", x.qname3, topn, id_str);
        }
        if (g & D2G_TOP_SIZE) {
            top_json(j, "top_response_bytes", x.sized, topn, id_str);
            quant_json(j, "response_query_size_ratio", x.ratio);
        }
        if (g & D2G_TOP_QTYPES) top_json(j, "top_qtype_xacts", x.qtype, topn, qt);
        if (g & D2G_XACT_TIMES) {
            quant_json(j, "xact_time_us", x.time);
            hist_json(j, "xact_histogram_us", x.hist);
            top_json(j, "top_slow_xacts", x.slow, topn, id_str);
        }
        j.end_obj();
    }
}

static void dns_json(J &j, const DnsBucket &b, size_t topn, uint32_t g)
{
    auto u16s = [](const uint16_t &v) { return std::to_string(v); };
    auto rc = [](const uint16_t &v) { auto &m = rcode_names(); auto it = m.find(v); return it != m.end() ? it->second : std::to_string(v); };
    auto qt = [](const uint16_t &v) { auto &m = qtype_names(); auto it = m.find(v); return it != m.end() ? it->second : std::to_string(v); };
    j.key("period"); j.obj();
    j.key("start_ts"); j.i64(b.start.sec);
    j.key("length"); j.u64(b.period_length);
    j.end_obj();
    j.key("wire_packets"); j.obj();
    j.key("events"); j.u64(b.num_events);
    j.key("deep_samples"); j.u64(b.num_samples);
    if (g & DG_COUNTERS) {
        j.key("queries"); j.u64(b.queries);
        j.key("replies"); j.u64(b.replies);
        j.key("tcp"); j.u64(b.TCP);
        j.key("udp"); j.u64(b.UDP);
        j.key("ipv4"); j.u64(b.IPv4);
        j.key("ipv6"); j.u64(b.IPv6);
        j.key("nxdomain"); j.u64(b.NX);
        j.key("refused"); j.u64(b.REFUSED);
        j.key("srvfail"); j.u64(b.SRVFAIL);
        j.key("noerror"); j.u64(b.NOERROR);
        j.key("nodata"); j.u64(b.NODATA);
        j.key("total"); j.u64(b.total);
        j.key("filtered"); j.u64(b.filtered);
        if (g & DG_TOP_ECS) { j.key("query_ecs"); j.u64(b.query_ecs); }
    }
    j.end_obj();
    if (g & DG_CARDINALITY) { j.key("cardinality"); j.obj(); j.key("qname"); j.i64(lround(b.qname.estimate())); j.end_obj(); }
    if (g & DG_TRANSACTIONS) {
        j.key("xact"); j.obj();
        j.key("counts"); j.obj(); j.key("total"); j.u64(b.xacts_total); j.key("timed_out"); j.u64(b.xacts_timed_out); j.end_obj();
        j.key("in"); j.obj(); j.key("total"); j.u64(b.xacts_in);
        top_json(j, "top_slow", b.slow_in, topn, id_str);
        if (g & DG_QUANTILES) quant_json(j, "quantiles_us", b.xact_to);
        if (g & DG_HISTOGRAMS) hist_json(j, "histogram_us", b.hist_to);
        j.end_obj();
        j.key("out"); j.obj(); j.key("total"); j.u64(b.xacts_out);
        top_json(j, "top_slow", b.slow_out, topn, id_str);
        if (g & DG_QUANTILES) quant_json(j, "quantiles_us", b.xact_from);
        if (g & DG_HISTOGRAMS) hist_json(j, "histogram_us", b.hist_from);
        j.end_obj();
        if ((g & DG_QUANTILES) && !b.ratio.empty()) { j.key("ratio"); j.obj(); quant_json(j, "quantiles", b.ratio); j.end_obj(); }
        j.end_obj();
    }
    if (g & DG_TOP_PORTS) top_json(j, "top_udp_ports", b.udp_port, topn, u16s);
    if (g & DG_TOP_ECS) {
        // geo / ASN lookups need a MaxMind database: none is enabled (HandlerModulePlugin::city/asn)
        j.key("top_geoLoc_ecs"); j.arr(); j.end_arr();
        j.key("top_asn_ecs"); j.arr(); j.end_arr();
        top_json(j, "top_query_ecs", b.ecs, topn, id_str);
    }
    if (g & DG_TOP_QNAMES) {
        top_json(j, "top_qname2", b.qname2, topn, id_str);
        top_json(j, "top_qname3", b.qname3, topn, id_str);
        top_json(j, "top_nxdomain", b.nx, topn, id_str);
        top_json(j, "top_refused", b.refused, topn, id_str);
        top_json(j, "top_srvfail", b.srvfail, topn, id_str);
        top_json(j, "top_nodata", b.nodata, topn, id_str);
        if (g & DG_TOP_QNAMES_DETAILS) {
            top_json(j, "top_qname_by_resp_bytes", b.sized_resp, topn, id_str);
            top_json(j, "top_noerror", b.noerror, topn, id_str);
        }
    }
    top_json(j, "top_rcode", b.rcode, topn, rc);
    top_json(j, "top_qtype", b.qtype, topn, qt);
}

// merged window (AbstractMetricsManager::window_merged_json) or a single bucket
// AbstractMetricsBucket::merge (src/AbstractMetricsManager.h:177-195): base fields, then the
// handler's specialized_merge (sum: Aggregate::SUM)
template <typename B>
static void bucket_merge(B &out, const B &m, bool firstb, bool sum = false)
{
    out.num_events += m.num_events;
    out.num_samples += m.num_samples;
    out.period_length += m.period_length;
    if (firstb || m.start.sec < out.start.sec) out.start.sec = m.start.sec;
    if (firstb || m.end.sec > out.end.sec) out.end.sec = m.end.sec;
    out.merge(m, sum);
}
// a fresh bucket folding buckets [from, from + count) of the window (DEFAULT aggregate); a
// union of CPC sketches reports the ICON estimate even for one input
template <typename B>
static std::unique_ptr<B> fold_buckets(const Window<B> &w, unsigned from, unsigned count)
{
    std::unique_ptr<B> out(new B());
    bool firstb = true;
    for (unsigned k = from; k < from + count && k < w.buckets.size(); k++) {
        bucket_merge(*out, *w.buckets[k], firstb);
        firstb = false;
    }
    return out;
}
template <typename B>
static std::unique_ptr<B> window_bucket(const Window<B> &w, unsigned window, int single = -1)
{
    std::unique_ptr<B> out(new B());
    if (single >= 0) {
        *out = *w.buckets.at((size_t)single);
        return out;
    }
    if (window <= 1) {
        *out = *w.buckets.at(0);
        return out;
    }
    return fold_buckets(w, 0, window);
}

// ---------------------------------------------------------------- pcap reader
struct PcapFile {
    bool swapped = false, nano = false;
    uint32_t linktype = 1;
    const uint8_t *p = nullptr;
    size_t len = 0, pos = 24;
    bool open(const uint8_t *d, size_t n, std::string &err)
    {
        p = d; len = n;
        if (n < 24) { err = "Cannot open pcap/pcapng file"; return false; }
        uint32_t magic = rd32le(d);
        if (magic == 0xa1b2c3d4) {} else if (magic == 0xa1b23c4d) nano = true;
        else if (magic == 0xd4c3b2a1) swapped = true;
        else if (magic == 0x4d3cb2a1) { swapped = true; nano = true; }
        else { err = "Cannot open pcap/pcapng file"; return false; }
        linktype = u32(d + 20);
        return true;
    }
    uint32_t u32(const uint8_t *q) const { uint32_t v = rd32le(q); return swapped ? __builtin_bswap32(v) : v; }
    bool next(Pkt &pk)
    {
        if (pos + 16 > len) return false;
        const uint8_t *h = p + pos;
        uint32_t incl = u32(h + 8);
        if (pos + 16 + incl > len) return false;
        pk = Pkt();
        pk.ts.sec = u32(h);
        pk.ts.nsec = nano ? u32(h + 4) : (int64_t)u32(h + 4) * 1000;
        pk.caplen = incl;
        pk.data = h + 16;
        pos += 16 + incl;
        return true;
    }
};

static bool parse_config(const char *s, Config &c, std::string &err)
{
    std::string str = s ? s : "";
    size_t pos = 0;
    while (pos < str.size()) {
        size_t e = str.find(';', pos);
        std::string kv = str.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
        pos = e == std::string::npos ? str.size() : e + 1;
        if (kv.empty()) continue;
        size_t eq = kv.find('=');
        std::string k = kv.substr(0, eq), v = eq == std::string::npos ? "" : kv.substr(eq + 1);
        if (k == "host_spec") { if (!parse_host_specs(v, c, err)) return false; }
        else if (k == "num_periods") c.num_periods = (unsigned)atoi(v.c_str());
        else if (k == "window") c.window = (unsigned)atoi(v.c_str());
        else if (k == "topn_count") c.topn_count = (size_t)atoll(v.c_str());
        else if (k == "xact_ttl_ms") c.xact_ttl_ms = (uint32_t)atoll(v.c_str());
        else if (k == "tcp_packet_reassembly_cache_limit") c.tcp_cache_limit = (uint64_t)strtoull(v.c_str(), nullptr, 0);
        else if (k == "dns_details") { if (atoi(v.c_str())) c.dns_groups |= DG_TOP_QNAMES_DETAILS; }
        else if (k == "net_groups") c.net_groups = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "dns_groups") c.dns_groups = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "filter_all") c.filter_all = atoi(v.c_str()) != 0;
        else if (k == "net_filter_all") c.net_filter_all = atoi(v.c_str()) != 0;
        else if (k == "deep_sample_rate") c.deep_sample_rate = std::max(1, std::min(100, atoi(v.c_str())));
        else if (k == "net2_groups") c.net2_groups = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "dns2_groups") c.dns2_groups = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "topn_pct") c.topn_pct = (uint32_t)atoi(v.c_str());
        else if (k == "exclude_noerror") c.exclude_noerror = atoi(v.c_str()) != 0;
        else if (k == "only_rcode_mask") c.only_rcode_mask = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "answer_count") { c.has_answer_count = true; c.answer_count = (uint32_t)atoll(v.c_str()); }
        else if (k == "only_queries") c.only_queries = atoi(v.c_str()) != 0;
        else if (k == "only_responses") c.only_responses = atoi(v.c_str()) != 0;
        else if (k == "only_dnssec_response") c.only_dnssec = atoi(v.c_str()) != 0;
        else if (k == "public_suffix_list") c.psl = atoi(v.c_str()) != 0;
        else if (k == "xact_dirs_disabled") c.xact_dirs_disabled = (uint32_t)atoi(v.c_str());
        else if (k == "single") c.single = atoi(v.c_str());
        else if (k == "heartbeats") {
            size_t q = 0;
            while (q < v.size()) {
                size_t e2 = v.find(',', q);
                c.heartbeats.push_back(atoll(v.substr(q, e2 == std::string::npos ? std::string::npos : e2 - q).c_str()));
                q = e2 == std::string::npos ? v.size() : e2 + 1;
            }
        }
        else if (k == "only_qname_suffix") {
            size_t q = 0;
            while (q < v.size()) {
                size_t e2 = v.find(',', q);
                c.only_qname_suffix.push_back(lower(v.substr(q, e2 == std::string::npos ? std::string::npos : e2 - q)));
                q = e2 == std::string::npos ? v.size() : e2 + 1;
            }
        }
        else if (k == "only_qname") {
            size_t q = 0;
            while (q < v.size()) {
                size_t e2 = v.find(',', q);
                std::string t = v.substr(q, e2 == std::string::npos ? std::string::npos : e2 - q);
                if (!t.empty()) c.only_qname.push_back(lower(t));
                q = e2 == std::string::npos ? v.size() : e2 + 1;
            }
        }
        else if (k == "only_qtype") {
            size_t q = 0;
            while (q < v.size()) {
                size_t e2 = v.find(',', q);
                std::string t = v.substr(q, e2 == std::string::npos ? std::string::npos : e2 - q);
                if (!t.empty()) c.only_qtype.push_back((uint16_t)atoi(t.c_str()));
                q = e2 == std::string::npos ? v.size() : e2 + 1;
            }
        }
        else { err = "unknown config key: " + k; return false; }
    }
    return true;
}

} // namespace pvo

// ---------------------------------------------------------------- C ABI (tests / cpu_baseline only)
extern "C" {

// Runs the restated pktvisor-reader pipeline (net v1 + dns v1) on an in-memory
// pcap file image. `cfg` is "key=value;..." (host_spec, num_periods, window,
// topn_count, xact_ttl_ms, dns_details). On success returns 0 and *out holds a
// malloc'd JSON document {"<W>m": {"packets": {...}, "dns": {...}}}.
int pvo_run(const uint8_t *file, size_t len, const char *cfg, char **out)
{
    using namespace pvo;
    Config c;
    std::string err;
    *out = nullptr;
    if (!parse_config(cfg, c, err)) { *out = strdup(err.c_str()); return -1; }
    PcapFile f;
    if (!f.open(file, len, err)) { *out = strdup(err.c_str()); return -2; }
    Engine e(c);
    e.linktype = f.linktype;
    if (const char *lp = getenv("PVO_TCP_LOG")) e.tcp_log = fopen(lp, "w");
    topn_pct = c.topn_pct;
    Pkt pk;
    TS last;
    bool first = true;
    size_t hb = 0;
    while (f.next(pk)) {
        if (first) { e.start(pk.ts); first = false; }
        for (; hb < c.heartbeats.size() && c.heartbeats[hb] < pk.ts.sec; hb++) e.heartbeat(TS{c.heartbeats[hb], 0});
        e.process(pk);
        last = pk.ts;
    }
    if (!first)
        for (; hb < c.heartbeats.size(); hb++) e.heartbeat(TS{c.heartbeats[hb], 0});
    if (!first) e.end(last);
    e.tcp_close_all(); // after end_tstamp_cb (PcapInputStream.cpp:514-522)
    if (e.tcp_log) fclose(e.tcp_log);
    J j;
    j.obj();
    unsigned w = c.window <= 1 ? 1 : c.window;
    j.key(c.single >= 0 ? "p" + std::to_string(c.single) : std::to_string(w) + "m");
    j.obj();
    if (c.single >= 0 && ((size_t)c.single >= e.net.buckets.size() || (size_t)c.single >= e.dns.buckets.size())) {
        *out = strdup("requested metrics period has not yet accumulated");
        return -3;
    }
    auto nb = window_bucket(e.net, w, c.single);
    j.key("packets"); j.obj(); net_json(j, *nb, c.topn_count, c.net_groups); j.end_obj();
    if (c.net2_groups) {
        auto n2 = window_bucket(e.net2, w, c.single);
        j.key("net"); j.obj(); net2_json(j, *n2, c.topn_count, c.net2_groups); j.end_obj();
    }
    if (c.dns2_groups) {
        auto d2 = window_bucket(e.dns2, w, c.single);
        j.key("dns"); j.obj(); dns2_json(j, *d2, c.topn_count, c.dns2_groups); j.end_obj();
    } else {
        auto db = window_bucket(e.dns, w, c.single);
        j.key("dns"); j.obj(); dns_json(j, *db, c.topn_count, c.dns_groups); j.end_obj();
    }
    j.end_obj();
    j.end_obj();
    *out = strdup(j.s.c_str());
    return 0;
}

void pvo_free(char *p) { free(p); }

// Policy::_get_merged_buckets (src/Policies.cpp:420-446) over like handlers, one per capture:
// StreamMetricsHandler::merge(bucket, period, prometheus, merged) (src/StreamHandler.h:259-269)
// -> simple_merge / multiple_merge (src/AbstractMetricsManager.h:649-706). The first handler
// makes a fresh bucket of its period (or of its `period` newest buckets, merged); each further
// one folds its own into it with Aggregate::SUM. prometheus: period 1 of a manager holding more
// than one, else 0, never merged. Output {"packets": {...}, "dns": {...}} (window_external_json).
int pvo_run_policy(const uint8_t *const *files, const size_t *lens, uint32_t n, const char *cfg, uint32_t period,
                   int merged, int prometheus, char **out)
{
    using namespace pvo;
    Config c;
    std::string err;
    *out = nullptr;
    if (!parse_config(cfg, c, err)) { *out = strdup(err.c_str()); return -1; }
    topn_pct = c.topn_pct;
    std::vector<std::unique_ptr<Engine>> engines;
    for (uint32_t i = 0; i < n; i++) {
        PcapFile f;
        if (!f.open(files[i], lens[i], err)) { *out = strdup(err.c_str()); return -2; }
        engines.emplace_back(new Engine(c));
        Engine &e = *engines.back();
        e.linktype = f.linktype;
        Pkt pk;
        TS last;
        bool first = true;
        size_t hb = 0;
        while (f.next(pk)) {
            if (first) { e.start(pk.ts); first = false; }
            for (; hb < c.heartbeats.size() && c.heartbeats[hb] < pk.ts.sec; hb++) e.heartbeat(TS{c.heartbeats[hb], 0});
            e.process(pk);
            last = pk.ts;
        }
        if (!first) e.end(last);
        e.tcp_close_all();
    }
    auto pick = [&](auto &win, std::unique_ptr<typename std::remove_reference<decltype(*win.buckets[0])>::type> &acc, bool firstb) {
        uint64_t p = period;
        bool m = merged != 0;
        if (prometheus) { p = win.buckets.size() > 1 ? 1 : 0; m = false; }
        auto b = m ? fold_buckets(win, 0, (unsigned)p) : fold_buckets(win, (unsigned)p, 1);
        if (firstb) acc = std::move(b);
        else bucket_merge(*acc, *b, false, true);
    };
    std::unique_ptr<NetBucket> nb;
    std::unique_ptr<DnsBucket> db;
    std::unique_ptr<Net2Bucket> n2b;
    std::unique_ptr<Dns2Bucket> d2b;
    for (uint32_t i = 0; i < n; i++) {
        pick(engines[i]->net, nb, i == 0);
        pick(engines[i]->dns, db, i == 0);
        if (c.net2_groups) pick(engines[i]->net2, n2b, i == 0);
        if (c.dns2_groups) pick(engines[i]->dns2, d2b, i == 0);
    }
    J j;
    j.obj();
    j.key("packets"); j.obj(); net_json(j, *nb, c.topn_count, c.net_groups); j.end_obj();
    if (c.net2_groups) { j.key("net"); j.obj(); net2_json(j, *n2b, c.topn_count, c.net2_groups); j.end_obj(); }
    j.key("dns"); j.obj();
    if (c.dns2_groups) dns2_json(j, *d2b, c.topn_count, c.dns2_groups);
    else dns_json(j, *db, c.topn_count, c.dns_groups);
    j.end_obj();
    j.end_obj();
    *out = strdup(j.s.c_str());
    return 0;
}

// Exposed for the sketch pinning tests: estimate of a CPC sketch fed with the
// given sequence of uint32 values (update(uint32_t)) or byte strings.
double pvo_cpc_u32(const uint32_t *v, size_t n, int merged)
{
    pvo::Cpc c;
    for (size_t i = 0; i < n; i++) c.update_u32(v[i]);
    if (merged) { pvo::Cpc u; u.merge(c); return u.estimate(); }
    return c.estimate();
}

void pvo_murmur3(const uint8_t *d, size_t n, uint64_t seed, uint64_t *out2)
{
    pvo::murmur3_128(d, n, seed, out2[0], out2[1]);
}

double pvo_icon(uint32_t c) { return pvo::icon_estimate(c); }

// First query name as DnsQuery would hold it (NUL-truncated) and m_NameLength.
uint32_t pvo_decode_qname(const uint8_t *msg, uint32_t len, char *out, uint32_t *outlen)
{
    pvo::DnsMsg m{msg, len};
    std::string nm;
    size_t nl = pvo::decode_name(m, 12, nm, 1);
    std::string name;
    if (nl > 0) { size_t z = nm.find('\0'); name = z == std::string::npos ? nm : nm.substr(0, z); }
    memcpy(out, name.data(), name.size());
    *outlen = (uint32_t)name.size();
    return (uint32_t)nl;
}

void pvo_dns_parse(const uint8_t *msg, uint32_t len, int *ok, int *has_query, uint32_t *qtype)
{
    pvo::DnsMsg m{msg, len};
    pvo::DnsParse r = pvo::parse_resources(m);
    *ok = r.ok; *has_query = r.has_query; *qtype = r.qtype;
}

void pvo_aggregate_domain(const char *name, size_t n, size_t suffix, size_t *q2_start, long *q3_start)
{
    std::string d(name, n), q2, q3;
    pvo::aggregate_domain(d, suffix, q2, q3);
    *q2_start = d.size() - q2.size();
    *q3_start = q3.empty() ? -1 : (long)(d.size() - q3.size());
}

// the oracle's jsf32 restatement, first n draws (pinned against oracle/_ref/ref_jsf)
int pvo_jsf32(uint32_t n, uint32_t *out)
{
    pvo::Jsf32 r;
    for (uint32_t i = 0; i < n; i++) out[i] = r();
    return 0;
}

} // extern "C"

#ifdef PVO_MAIN
// CLI mirroring cmd/pktvisor-reader/main.cpp:28-51 for the options the hot path
// uses: pvo_reader [-H HOST_SPEC] [--periods N] FILE
#include <fstream>
#include <iterator>
int main(int argc, char **argv)
{
    std::string host, file;
    unsigned periods = 5;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "-H" && i + 1 < argc) host = argv[++i];
        else if (a == "--periods" && i + 1 < argc) periods = (unsigned)atoi(argv[++i]);
        else file = a;
    }
    std::ifstream f(file, std::ios::binary);
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::string cfg = "num_periods=" + std::to_string(periods) + ";window=" + std::to_string(periods);
    if (!host.empty()) cfg += ";host_spec=" + host;
    char *out = nullptr;
    int rc = pvo_run(buf.data(), buf.size(), cfg.c_str(), &out);
    printf("%s\n", out ? out : "");
    pvo_free(out);
    return rc ? 1 : 0;
}
#endif
