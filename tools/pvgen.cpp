// SPDX-License-Identifier: MPL-2.0
// tools/pvgen.cpp — seeded synthetic classic-pcap generator for the BASELINE.json
// configs (test / bench infrastructure; not part of the product path).
//
//   cfg 1  C1: 1k DNS packets, 500 queries + 500 paired responses, A/AAAA/MX/TXT,
//              rcodes {0,2,3,5}, clients in 10.0.0.0/8           (seed 0x5eed0001)
//   cfg 2  C2: Net only, caplen 64 = Eth+IPv4+UDP+22B, non-DNS ports, Zipf(1.1)
//              over 2^20 addresses in 10/8 and 172.16/12, 1 us steps (0x5eed0002)
//   cfg 3  C3: UDP/53 queries, QD=1 type A, one mixed-case label L~U[51,63] drawn
//              Zipf over 1M names + EDNS0 OPT RR => frame 71+L, mean 128 B (0x5eed0003)
//   cfg 4  C4: IMIX 70% non-DNS UDP/TCP {64:7,576:4,1500:1} + 30% DNS query/response
//              pairs (0xC00C answers, rcodes 0/2/3/5, ANCOUNT 0..3)      (0x5eed0004)
//   cfg 9  edge-case mix for parity: VLAN/QinQ, IPv6 (+ext headers), IP-in-IP,
//              fragments, short/truncated frames, malformed DNS names, pointer
//              loops, NULs, upper case, QD=0 messages, Ethernet padding
//
// Timestamps start at 1700000000.000000 and advance by `ts_step_us` per record.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed ^ 0x9e3779b97f4a7c15ULL) {}
    uint64_t next()
    {
        uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        return z ^ (z >> 31);
    }
    uint32_t u32() { return (uint32_t)next(); }
    uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
    double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct Zipf {
    std::vector<double> cdf;
    Zipf(size_t n, double s)
    {
        cdf.resize(n);
        double acc = 0;
        for (size_t k = 0; k < n; k++) { acc += pow((double)(k + 1), -s); cdf[k] = acc; }
        for (auto &c : cdf) c /= acc;
    }
    size_t draw(Rng &r) const { return std::lower_bound(cdf.begin(), cdf.end(), r.unit()) - cdf.begin(); }
};

struct Out {
    uint8_t *buf;
    size_t cap, used = 0;
    uint32_t *offs;
    uint64_t nrec = 0;
    uint64_t ts_us;
    uint32_t step;
    bool ok = true;
    void rec(const uint8_t *frame, uint32_t len)
    {
        if (used + 16 + len > cap) { ok = false; return; }
        if (offs) offs[nrec] = (uint32_t)used;
        uint32_t h[4] = {(uint32_t)(ts_us / 1000000), (uint32_t)(ts_us % 1000000), len, len};
        memcpy(buf + used, h, 16);
        memcpy(buf + used + 16, frame, len);
        used += 16 + len;
        nrec++;
        ts_us += step;
    }
};

inline void put16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
inline void put32(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v; }

// Ethernet + IPv4 header; returns offset of L4. ip addresses in host order.
uint32_t eth_ipv4(uint8_t *f, uint32_t src, uint32_t dst, uint8_t proto, uint32_t l4len)
{
    memset(f, 0, 34);
    f[0] = 0x02; f[5] = 0x01; f[6] = 0x02; f[11] = 0x02;
    put16(f + 12, 0x0800);
    uint8_t *ip = f + 14;
    ip[0] = 0x45;
    put16(ip + 2, 20 + l4len);
    put16(ip + 4, 0x1234);
    put16(ip + 6, 0x4000); // DF
    ip[8] = 64;
    ip[9] = proto;
    put32(ip + 12, src);
    put32(ip + 16, dst);
    return 34;
}

uint32_t udp(uint8_t *p, uint32_t sport, uint32_t dport, uint32_t paylen)
{
    put16(p, sport);
    put16(p + 2, dport);
    put16(p + 4, 8 + paylen);
    put16(p + 6, 0);
    return 8;
}

bool dns_port(uint32_t p) { return p == 53 || p == 5353 || p == 5355 || p == 53000; }
uint32_t rand_port(Rng &r)
{
    for (;;) { uint32_t p = 1024 + r.below(65536 - 1024); if (!dns_port(p)) return p; }
}

const char ALNUM[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";

// deterministic name for a catalogue id
std::string label_for(uint64_t id, uint32_t len, bool mixed)
{
    Rng r(id * 0x2545F4914F6CDD1DULL + 17);
    std::string s(len, 'a');
    for (auto &c : s) c = mixed ? ALNUM[r.below(62)] : ALNUM[r.below(26)];
    return s;
}

uint32_t encode_name(uint8_t *p, const std::string &name)
{
    uint32_t o = 0;
    size_t start = 0;
    while (start <= name.size()) {
        size_t dot = name.find('.', start);
        if (dot == std::string::npos) dot = name.size();
        size_t l = dot - start;
        if (l == 0) break;
        p[o++] = (uint8_t)l;
        memcpy(p + o, name.data() + start, l);
        o += (uint32_t)l;
        start = dot + 1;
    }
    p[o++] = 0;
    return o;
}

const uint16_t QTYPES[] = {1, 28, 15, 16, 5, 2, 6};

struct Dns {
    // builds a DNS query or response message; returns length
    static uint32_t msg(uint8_t *m, uint16_t txid, bool resp, uint32_t rcode, uint32_t ancount, const std::string &qname,
                        uint16_t qtype, bool opt, Rng &r)
    {
        put16(m, txid);
        m[2] = resp ? 0x81 : 0x01;
        m[3] = resp ? (uint8_t)(0x80 | (rcode & 15)) : 0x00;
        put16(m + 4, 1);
        put16(m + 6, ancount);
        put16(m + 8, 0);
        put16(m + 10, opt ? 1 : 0);
        uint32_t o = 12;
        o += encode_name(m + o, qname);
        put16(m + o, qtype); put16(m + o + 2, 1);
        o += 4;
        for (uint32_t a = 0; a < ancount; a++) {
            m[o] = 0xc0; m[o + 1] = 0x0c;
            put16(m + o + 2, 1); put16(m + o + 4, 1); put32(m + o + 6, 300);
            put16(m + o + 10, 4); put32(m + o + 12, r.u32());
            o += 16;
        }
        if (opt) {
            m[o] = 0; put16(m + o + 1, 41); put16(m + o + 3, 4096); put32(m + o + 5, 0); put16(m + o + 9, 0);
            o += 11;
        }
        return o;
    }
};

void gen_c2(Out &o, uint64_t n, Rng &r)
{
    Zipf z(1u << 20, 1.1);
    std::vector<uint32_t> addrs(1u << 20);
    for (uint32_t i = 0; i < addrs.size(); i++)
        addrs[i] = (i & 1) ? (0x0A000000u | (r.u32() & 0x00ffffffu)) : (0xAC100000u | (r.u32() & 0x000fffffu));
    uint8_t f[64];
    for (uint64_t i = 0; i < n && o.ok; i++) {
        uint32_t src = addrs[z.draw(r)], dst = addrs[z.draw(r)];
        uint32_t l4 = eth_ipv4(f, src, dst, 17, 8 + 22);
        l4 += udp(f + l4, rand_port(r), rand_port(r), 22);
        for (int k = 0; k < 22; k++) f[l4 + k] = (uint8_t)r.u32();
        o.rec(f, 64);
    }
}

void gen_c3(Out &o, uint64_t n, Rng &r)
{
    Zipf z(1000000, 1.1);
    uint8_t f[256];
    for (uint64_t i = 0; i < n && o.ok; i++) {
        uint64_t id = z.draw(r);
        uint32_t L = 51 + (uint32_t)(Rng(id + 99).below(13));
        std::string name = label_for(id, L, true);
        uint32_t client = 0x0A000000u | (r.u32() & 0x00ffffffu);
        uint32_t server = 0xC0000200u | (r.u32() & 0xff);
        uint8_t m[200];
        uint32_t dl = Dns::msg(m, (uint16_t)r.u32(), false, 0, 0, name, 1, true, r);
        uint32_t l4 = eth_ipv4(f, client, server, 17, 8 + dl);
        uint32_t sport = 1 + r.below(65535);
        if (dns_port(sport)) sport = 1024;
        l4 += udp(f + l4, sport, 53, dl);
        memcpy(f + l4, m, dl);
        o.rec(f, l4 + dl);
    }
}

// C1 / C4: DNS query/response pairs interleaved with non-DNS traffic
void gen_mix(Out &o, uint64_t n, Rng &r, double dns_frac, uint32_t domains)
{
    Zipf zd(domains, 1.1);
    const char *tlds[] = {"com", "net", "org", "io", "test"};
    struct Open { uint32_t client, server, sport; uint16_t txid; std::string name; uint16_t qtype; uint64_t due; };
    std::vector<Open> open;
    uint8_t f[1600];
    uint64_t i = 0;
    while (i < n && o.ok) {
        // a pending response that is due goes first
        if (!open.empty() && open.front().due <= i) {
            Open q = open.front();
            open.erase(open.begin());
            uint32_t u = r.below(10), rcode = u < 7 ? 0 : (u == 7 ? 2 : (u == 8 ? 3 : 5));
            uint32_t an = rcode == 0 ? r.below(4) : 0;
            uint8_t m[512];
            uint32_t dl = Dns::msg(m, q.txid, true, rcode, an, q.name, q.qtype, false, r);
            uint32_t l4 = eth_ipv4(f, q.server, q.client, 17, 8 + dl);
            l4 += udp(f + l4, 53, q.sport, dl);
            memcpy(f + l4, m, dl);
            o.rec(f, l4 + dl);
            o.ts_us += r.below(50);
            i++;
            continue;
        }
        if (r.unit() < dns_frac / 2 && open.size() < 4096) {
            uint64_t d = zd.draw(r);
            std::string name = label_for(r.below(1u << 20), 3 + r.below(10), r.below(4) == 0) + "." +
                               label_for(d, 4 + (uint32_t)(d % 9), false) + "." + tlds[d % 5];
            uint32_t client = 0x0A000000u | (r.u32() & 0x00ffffffu);
            uint32_t server = 0x08080800u | r.below(8);
            uint32_t sport = 1024 + r.below(60000);
            if (dns_port(sport)) sport = 2000;
            uint16_t txid = (uint16_t)r.u32();
            uint16_t qtype = QTYPES[r.below(4)];
            uint8_t m[512];
            uint32_t dl = Dns::msg(m, txid, false, 0, 0, name, qtype, false, r);
            uint32_t l4 = eth_ipv4(f, client, server, 17, 8 + dl);
            l4 += udp(f + l4, sport, 53, dl);
            memcpy(f + l4, m, dl);
            o.rec(f, l4 + dl);
            open.push_back(Open{client, server, sport, txid, name, qtype, i + 1 + r.below(40)});
            i++;
            continue;
        }
        // non-DNS IMIX packet
        uint32_t u = r.below(12), size = u < 7 ? 64 : (u < 11 ? 576 : 1500);
        uint32_t src = (r.below(2) ? 0x0A000000u : 0xC6336400u) | (r.u32() & 0xffff);
        uint32_t dst = (r.below(2) ? 0x0A000000u : 0x5DB8D800u) | (r.u32() & 0xffff);
        if (r.below(2)) {
            uint32_t l4 = eth_ipv4(f, src, dst, 17, size - 34);
            udp(f + l4, rand_port(r), rand_port(r), size - 42);
            for (uint32_t k = l4 + 8; k < size; k++) f[k] = (uint8_t)k;
        } else {
            uint32_t l4 = eth_ipv4(f, src, dst, 6, size - 34);
            memset(f + l4, 0, 20);
            put16(f + l4, rand_port(r)); put16(f + l4 + 2, r.below(2) ? 443 : 80);
            put32(f + l4 + 4, r.u32());
            f[l4 + 12] = 0x50;
            f[l4 + 13] = r.below(10) == 0 ? 0x02 : 0x10;
            for (uint32_t k = l4 + 20; k < size; k++) f[k] = (uint8_t)k;
        }
        o.rec(f, size);
        i++;
    }
}

// edge cases for parity (not a BASELINE config)
void gen_edge(Out &o, uint64_t n, Rng &r)
{
    uint8_t f[1600];
    for (uint64_t i = 0; i < n && o.ok; i++) {
        uint32_t kind = r.below(16);
        uint32_t len = 0;
        uint32_t src = (r.below(2) ? 0x0A000000u : 0xC0A80000u) | (r.u32() & 0xffff);
        uint32_t dst = (r.below(2) ? 0x0A000000u : 0x08080000u) | (r.u32() & 0xffff);
        if (r.below(50) == 0) src = 0; // 0.0.0.0 is never recorded
        // DNS payload with random structure
        uint8_t m[600];
        uint32_t dl = 0;
        {
            uint32_t mk = r.below(12);
            std::string name = label_for(r.below(5000), 1 + r.below(20), true) + "." + label_for(r.below(50), 3, false) +
                               (r.below(3) ? ".com" : "") + (r.below(8) == 0 ? "." : "");
            bool resp = r.below(2);
            dl = Dns::msg(m, (uint16_t)r.below(4), resp, r.below(6), resp ? r.below(3) : 0, name, QTYPES[r.below(7)],
                          r.below(4) == 0, r);
            if (mk == 0) { m[12] = 0xc0; m[13] = (uint8_t)r.below(40); }             // pointer as first label
            else if (mk == 1) { m[12] = 0xc0; m[13] = 12; }                         // self loop
            else if (mk == 2) dl = 12 + r.below(dl - 12);                           // truncated
            else if (mk == 3) { for (uint32_t k = 12; k < dl; k++) if (r.below(6) == 0) m[k] = (uint8_t)r.u32(); }
            else if (mk == 4) { put16(m + 4, 0); }                                 // QD=0 with answers
            else if (mk == 5) { put16(m + 4, 60); put16(m + 6, 60); }              // counts > 100
            else if (mk == 6) { m[13] = 0; }                                        // NUL inside first label
            else if (mk == 7) dl = r.below(12);                                     // shorter than the header
            else if (mk == 8) { m[12] = 63; for (int k = 0; k < 63; k++) m[13 + k] = 'A'; m[76] = 0xc0; m[77] = 12; dl = std::max(dl, 90u); }
            else if (mk == 9) { m[12] = 0x80 | r.below(64); }                       // 0x40-0xbf length byte
        }
        uint32_t sport = r.below(3) == 0 ? 53 : 1 + r.below(65535), dport = r.below(2) ? 53 : (r.below(4) ? 5353 : r.below(65536));
        if (r.below(40) == 0) sport = 0;
        memset(f, 0, sizeof f);
        f[0] = 2; put16(f + 12, 0x0800);
        uint32_t l3 = 14;
        if (kind == 1 || kind == 2) { // VLAN / QinQ
            put16(f + 12, kind == 1 ? 0x8100 : 0x88A8);
            put16(f + 14, r.below(4096));
            put16(f + 16, kind == 1 ? 0x0800 : 0x8100);
            l3 = 18;
            if (kind == 2) { put16(f + 18, 7); put16(f + 20, 0x0800); l3 = 22; }
        }
        if (kind == 3 || kind == 4 || kind == 5) { // IPv6 (+ hop-by-hop / fragment ext)
            put16(f + 12, 0x86DD);
            uint8_t *ip = f + 14;
            ip[0] = 0x60;
            uint32_t ext = kind == 4 ? 8 : (kind == 5 ? 8 : 0);
            ip[6] = kind == 4 ? 0 : (kind == 5 ? 44 : 17);
            ip[7] = 64;
            for (int k = 0; k < 16; k++) { ip[8 + k] = (uint8_t)(r.below(3) ? 0x20 + k : r.u32()); ip[24 + k] = (uint8_t)(k == 0 ? (r.below(2) ? 0x20 : 0xfe) : r.u32()); }
            if (r.below(3) == 0) memset(ip + 8, 0, 16);
            uint32_t l4 = 14 + 40 + ext;
            if (ext) { f[54] = 17; f[55] = 0; if (kind == 5) { put16(f + 56, r.below(2) ? 0 : 8); } }
            l4 += udp(f + l4, sport, dport, dl);
            memcpy(f + l4, m, dl);
            put16(ip + 4, ext + 8 + dl);
            len = l4 + dl;
        } else if (kind == 6) { // TCP SYN / short TCP
            uint32_t l4 = eth_ipv4(f, src, dst, 6, 20);
            put16(f + l4, r.below(65536)); put16(f + l4 + 2, 53);
            f[l4 + 12] = 0x50; f[l4 + 13] = (uint8_t)r.below(64);
            len = l4 + (r.below(4) ? 20 : r.below(20));
            if (len < l4 + 20) put16(f + 16, 20 + (len - l4));
        } else if (kind == 7) { // fragment
            uint32_t l4 = eth_ipv4(f, src, dst, 17, 8 + dl);
            put16(f + 20, r.below(2) ? 0x2000 : 0x0010);
            l4 += udp(f + l4, sport, dport, dl);
            memcpy(f + l4, m, dl);
            len = l4 + dl;
        } else if (kind == 8) { // IP-in-IP
            uint32_t inner = eth_ipv4(f, src, dst, 4, 20 + 8 + dl);
            uint8_t *ip2 = f + inner;
            ip2[0] = 0x45; put16(ip2 + 2, 20 + 8 + dl); ip2[8] = 64; ip2[9] = 17;
            put32(ip2 + 12, dst ^ 0x55); put32(ip2 + 16, src ^ 0x33);
            uint32_t l4 = inner + 20;
            l4 += udp(f + l4, sport, dport, dl);
            memcpy(f + l4, m, dl);
            len = l4 + dl;
        } else if (kind == 9) { // short frames
            len = r.below(60);
            for (uint32_t k = 0; k < len; k++) f[k] = (uint8_t)r.u32();
            if (len > 13) put16(f + 12, r.below(2) ? 0x0800 : 0x86DD);
        } else if (kind == 10) { // non-IP ethertype / 802.3 length
            put16(f + 12, r.below(2) ? 0x0806 : 0x0100);
            len = 60;
        } else { // plain IPv4 UDP (with optional padding / options / bad lengths)
            uint32_t opt = r.below(6) == 0 ? 4 * r.below(4) : 0;
            uint8_t *ip = f + l3;
            ip[0] = (uint8_t)(0x45 + opt / 4);
            ip[8] = 64; ip[9] = r.below(8) == 0 ? 6 : 17;
            put32(ip + 12, src); put32(ip + 16, dst);
            uint32_t l4 = l3 + 20 + opt;
            l4 += udp(f + l4, sport, dport, dl);
            memcpy(f + l4, m, dl);
            uint32_t total = l4 + dl - l3;
            put16(ip + 2, r.below(10) == 0 ? (r.below(2) ? 0 : total - r.below(10)) : total);
            len = l4 + dl + (r.below(4) == 0 ? r.below(20) : 0); // Ethernet padding
            if (ip[9] == 6) ip[l4 - l3 - 8 + 13 - 0] = 0x02;
        }
        if (len > sizeof f) len = sizeof f;
        o.rec(f, len);
    }
}

} // namespace

extern "C" {

// Generates `n` records for config `cfg` into buf[cap] (classic-pcap record
// format, no global header). offs (optional) receives each record's offset.
// Returns the number of records written, or -1 if cap was too small.
int64_t pvgen_records_at(int cfg, uint64_t n, uint64_t seed, uint32_t ts_step_us, uint64_t start_us, uint8_t *buf, size_t cap,
                         size_t *used, uint32_t *offs)
{
    Out o{buf, cap, 0, offs, 0, start_us, ts_step_us ? ts_step_us : 1u};
    Rng r(seed);
    switch (cfg) {
    case 1: gen_mix(o, n, r, 1.0, 200); break;
    case 2: gen_c2(o, n, r); break;
    case 3: gen_c3(o, n, r); break;
    case 4: case 5: gen_mix(o, n, r, 0.30, 100000); break;
    case 9: gen_edge(o, n, r); break;
    default: return -1;
    }
    *used = o.used;
    return o.ok ? (int64_t)o.nrec : -1;
}

int64_t pvgen_records(int cfg, uint64_t n, uint64_t seed, uint32_t ts_step_us, uint8_t *buf, size_t cap, size_t *used,
                      uint32_t *offs)
{
    return pvgen_records_at(cfg, n, seed, ts_step_us, 1700000000ull * 1000000ull, buf, cap, used, offs);
}

// Upper bound of bytes needed for n records of a config.
uint64_t pvgen_bound(int cfg, uint64_t n) { return n * (16 + (cfg == 2 ? 64 : (cfg == 3 ? 160 : 1600))) + 256; }

} // extern "C"
