// SPDX-License-Identifier: MPL-2.0
//
// pv_pcapng.cpp — pcapng capture files into the record blob the device path reads.
//
// The reference opens "pcap or pcapng" through PcapPlusPlus IFileReaderDevice::getReader
// (src/inputs/pcap/PcapInputStream.cpp:475-481; PcapPlusPlus 23.09 reads pcapng with
// LightPcapNg), and every packet reaches process_raw_packet as raw bytes plus a timespec.
// Neither library is in this image; the format (IETF draft-tuexen-opsawg-pcapng) is restated:
// blocks of (type, total length, body, total length), 32-bit aligned, in the byte order the
// Section Header Block's magic gives:
//   - 0x0A0D0D0A Section Header: byte-order magic 0x1A2B3C4D; starts a new interface list;
//   - 0x00000001 Interface Description: linktype (u16), snaplen, options (if_tsresol, code 9:
//     a byte v, units of 10^-v s, or 2^-(v & 0x7f) s when the top bit is set; default 10^-6);
//   - 0x00000006 Enhanced Packet: interface id, 64-bit timestamp (high, low), captured and
//     original length, the data padded to 4 bytes;
//   - 0x00000003 Simple Packet: original length and data (captured = min(original, snaplen of
//     interface 0)), no timestamp (0);
//   - 0x00000002 (obsolete) Packet: interface id (u16), drops (u16), timestamp, lengths, data;
//   - any other block is skipped.
// Each packet becomes a classic pcap record with a nanosecond fraction (ts_nano = 1), so the
// ingest and kernels see exactly what they see for a pcap file.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "pv_pcapng.h"

namespace pvi {

namespace {

struct Iface {
    uint32_t linktype = 0, snaplen = 0;
    bool pow2 = false;
    uint32_t tsres = 6; // 10^-6 s
};

struct Sec {
    bool swap = false;
    uint32_t u32(const uint8_t *p) const
    {
        uint32_t v;
        memcpy(&v, p, 4);
        return swap ? __builtin_bswap32(v) : v;
    }
    uint16_t u16(const uint8_t *p) const
    {
        uint16_t v;
        memcpy(&v, p, 2);
        return swap ? __builtin_bswap16(v) : v;
    }
};

// the interface's timestamp units -> (seconds, nanoseconds)
void ts_of(const Iface &f, uint64_t t, uint32_t &sec, uint32_t &nsec)
{
    if (f.pow2) {
        const uint32_t b = f.tsres;
        const uint64_t s = b >= 64 ? 0 : t >> b;
        const uint64_t frac = b >= 64 ? t : t & ((1ull << b) - 1);
        sec = (uint32_t)s;
        nsec = b == 0 ? 0 : (uint32_t)(((unsigned __int128)frac * 1000000000ull) >> b);
        return;
    }
    uint64_t div = 1;
    for (uint32_t k = 0; k < f.tsres; k++) div *= 10; // tsres <= 19 (checked at the IDB)
    sec = (uint32_t)(t / div);
    const uint64_t frac = t % div;
    if (f.tsres <= 9) {
        uint64_t mul = 1;
        for (uint32_t k = f.tsres; k < 9; k++) mul *= 10;
        nsec = (uint32_t)(frac * mul);
    } else {
        uint64_t d2 = 1;
        for (uint32_t k = 9; k < f.tsres; k++) d2 *= 10;
        nsec = (uint32_t)(frac / d2);
    }
}

} // namespace

int pcapng_to_records(const uint8_t *buf, size_t bytes, std::vector<uint8_t> *out, uint32_t *linktype,
                      uint64_t *n_records)
{
    Sec sec;
    std::vector<Iface> ifs;
    bool have_section = false;
    int64_t lt = -1;
    uint64_t n = 0;
    size_t p = 0;
    auto emit = [&](const uint8_t *data, uint32_t cap, uint32_t orig, uint32_t s, uint32_t ns) {
        n++;
        if (!out) return;
        const size_t o = out->size();
        out->resize(o + 16 + cap);
        const uint32_t h[4] = {s, ns, cap, orig};
        memcpy(out->data() + o, h, 16);
        if (cap) memcpy(out->data() + o + 16, data, cap);
    };
    while (p + 12 <= bytes) {
        uint32_t type;
        memcpy(&type, buf + p, 4);
        if (type == 0x0A0D0D0Au) {
            // the byte-order magic decides how this section is read
            uint32_t bom;
            memcpy(&bom, buf + p + 8, 4);
            if (bom == 0x1A2B3C4Du) sec.swap = false;
            else if (bom == 0x4D3C2B1Au) sec.swap = true;
            else return PVNG_EFORMAT;
            ifs.clear();
            have_section = true;
        } else {
            type = sec.u32(buf + p);
            if (!have_section) return PVNG_EFORMAT;
        }
        const uint32_t len = sec.u32(buf + p + 4);
        if (len < 12 || (len & 3) || p + len > bytes) break; // a truncated last block ends the file
        const uint8_t *b = buf + p + 8;     // body
        const uint32_t blen = len - 12;
        if (type == 1) {
            if (blen < 8) return PVNG_EFORMAT;
            Iface f;
            f.linktype = sec.u16(b);
            f.snaplen = sec.u32(b + 4);
            // options: (code u16, length u16, value padded to 4)
            uint32_t q = 8;
            while (q + 4 <= blen) {
                const uint16_t code = sec.u16(b + q), olen = sec.u16(b + q + 2);
                if (code == 0) break;
                if (q + 4 + olen > blen) break;
                if (code == 9 && olen >= 1) {
                    const uint8_t v = b[q + 4];
                    f.pow2 = (v & 0x80) != 0;
                    f.tsres = v & 0x7f;
                    // 10^-20 s and finer do not fit the 64-bit timestamp arithmetic (and no
                    // capture writes them): refused, not silently wrapped
                    if (!f.pow2 && f.tsres > 19) return PVNG_EFORMAT;
                }
                q += 4 + ((olen + 3u) & ~3u);
            }
            if (lt < 0) lt = f.linktype;
            else if ((uint32_t)lt != f.linktype) return PVNG_ELINKTYPES;
            ifs.push_back(f);
        } else if (type == 6 || type == 2) {
            if (blen < 20) return PVNG_EFORMAT;
            const uint32_t ifid = type == 6 ? sec.u32(b) : sec.u16(b);
            if (ifid >= ifs.size()) return PVNG_EFORMAT;
            const uint64_t t = ((uint64_t)sec.u32(b + 4) << 32) | sec.u32(b + 8);
            uint32_t cap = sec.u32(b + 12);
            const uint32_t orig = sec.u32(b + 16);
            if (cap > blen - 20) return PVNG_EFORMAT;
            uint32_t s, ns;
            ts_of(ifs[ifid], t, s, ns);
            emit(b + 20, cap, orig, s, ns);
        } else if (type == 3) {
            if (blen < 4 || ifs.empty()) return PVNG_EFORMAT;
            const uint32_t orig = sec.u32(b);
            uint32_t cap = orig;
            if (ifs[0].snaplen && cap > ifs[0].snaplen) cap = ifs[0].snaplen;
            if (cap > blen - 4) cap = blen - 4;
            emit(b + 4, cap, orig, 0, 0);
        }
        p += len;
    }
    if (linktype) *linktype = lt < 0 ? 1u : (uint32_t)lt;
    if (n_records) *n_records = n;
    return 0;
}

} // namespace pvi
