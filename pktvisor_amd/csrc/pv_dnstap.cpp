// SPDX-License-Identifier: MPL-2.0
//
// pv_dnstap.cpp — dnstap input decoding (host side of pv_process_dnstap).
//
// The reference reads a Frame Streams file with libfstrm (DnstapInputStream::_read_frame_stream_file,
// src/inputs/dnstap/DnstapInputStream.cpp:33-92) and parses each data frame as the protobuf
// message dnstap.Dnstap (src/inputs/dnstap/pb/dnstap.proto) with libprotobuf: frames that do
// not parse, are not of type MESSAGE or carry no message are skipped (:62-69). Neither library
// is in this image; this is the wire format restated:
//   - Frame Streams: a data frame is a big-endian u32 length (> 0) and the payload; a control
//     frame is an escape (u32 0), a u32 length and the control payload (its first u32 is the
//     control type: 2 START, 3 STOP ...). Reading ends at STOP or at the end of the bytes.
//   - protobuf (proto2): fields as (tag << 3 | wire type) varint keys, wire types 0 varint,
//     1 fixed64, 2 length-delimited, 5 fixed32; unknown fields skipped; a missing required
//     field (Dnstap.type, Message.type) fails the parse.
// The decoded events feed pv_dnstap_kernel (pv_kernels.hip) through pv_process_dnstap.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "pv_dnstap.h"

namespace pvi {

namespace {

struct Rd {
    const uint8_t *p, *e;
    bool ok = true;
    uint64_t varint()
    {
        uint64_t v = 0;
        for (int s = 0; s < 64; s += 7) {
            if (p >= e) { ok = false; return 0; }
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7f) << s;
            if (!(b & 0x80)) return v;
        }
        ok = false;
        return 0;
    }
    uint32_t fixed32()
    {
        if (e - p < 4) { ok = false; return 0; }
        uint32_t v;
        memcpy(&v, p, 4);
        p += 4;
        return v;
    }
    bool bytes(const uint8_t *&b, size_t &n)
    {
        const uint64_t l = varint();
        if (!ok || (uint64_t)(e - p) < l) { ok = false; return false; }
        b = p;
        n = (size_t)l;
        p += l;
        return true;
    }
    // skips a field of wire type wt
    void skip(uint32_t wt)
    {
        const uint8_t *b;
        size_t n;
        switch (wt) {
        case 0: varint(); break;
        case 1: if (e - p < 8) ok = false; else p += 8; break;
        case 2: bytes(b, n); break;
        case 5: fixed32(); break;
        default: ok = false; // groups (3, 4) are not used by dnstap.proto
        }
    }
};

bool parse_message(const uint8_t *b, size_t n, DtMessage &m)
{
    Rd r{b, b + n};
    bool has_type = false;
    while (r.ok && r.p < r.e) {
        const uint64_t key = r.varint();
        if (!r.ok) break;
        const uint32_t tag = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
        const uint8_t *q;
        size_t ql;
        switch (tag) {
        case 1: if (wt != 0) { r.skip(wt); break; } m.type = (uint32_t)r.varint(); has_type = true; break;
        case 2: if (wt != 0) { r.skip(wt); break; } m.family = (uint32_t)r.varint(); m.has_family = true; break;
        case 3: if (wt != 0) { r.skip(wt); break; } m.protocol = (uint32_t)r.varint(); m.has_protocol = true; break;
        case 4: if (wt != 2) { r.skip(wt); break; } if (r.bytes(q, ql)) { m.qaddr.assign(q, q + ql); m.has_qaddr = true; } break;
        case 5: if (wt != 2) { r.skip(wt); break; } if (r.bytes(q, ql)) { m.raddr.assign(q, q + ql); m.has_raddr = true; } break;
        case 6: if (wt != 0) { r.skip(wt); break; } m.qport = (uint32_t)r.varint(); m.has_qport = true; break;
        case 8: if (wt != 0) { r.skip(wt); break; } m.qsec = r.varint(); m.has_qsec = true; break;
        case 9: if (wt != 5) { r.skip(wt); break; } m.qnsec = r.fixed32(); break;
        case 10: if (wt != 2) { r.skip(wt); break; } if (r.bytes(q, ql)) { m.qmsg = q; m.qmsg_len = ql; m.has_qmsg = true; } break;
        case 12: if (wt != 0) { r.skip(wt); break; } m.rsec = r.varint(); m.has_rsec = true; break;
        case 13: if (wt != 5) { r.skip(wt); break; } m.rnsec = r.fixed32(); break;
        case 14: if (wt != 2) { r.skip(wt); break; } if (r.bytes(q, ql)) { m.rmsg = q; m.rmsg_len = ql; m.has_rmsg = true; } break;
        default: r.skip(wt);
        }
    }
    return r.ok && has_type;
}

// dnstap.Dnstap: type (15, required), message (14); true when it parses as the reference's
// ParseFromArray would and is a MESSAGE with a message
bool parse_dnstap(const uint8_t *b, size_t n, DtMessage &m)
{
    Rd r{b, b + n};
    bool has_type = false, has_msg = false, msg_ok = true;
    uint64_t type = 0;
    while (r.ok && r.p < r.e) {
        const uint64_t key = r.varint();
        if (!r.ok) break;
        const uint32_t tag = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
        if (tag == 15 && wt == 0) {
            type = r.varint();
            has_type = true;
        } else if (tag == 14 && wt == 2) {
            const uint8_t *q;
            size_t ql;
            if (r.bytes(q, ql)) {
                // a repeated occurrence of an embedded message merges; dnstap writers emit one
                m = DtMessage();
                msg_ok = parse_message(q, ql, m);
                has_msg = true;
            }
        } else {
            r.skip(wt);
        }
    }
    return r.ok && has_type && msg_ok && type == 1 && has_msg;
}

inline uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

} // namespace

int dnstap_decode(const uint8_t *buf, size_t bytes, std::vector<DtMessage> &out, uint32_t *frames)
{
    out.clear();
    uint32_t nf = 0;
    size_t p = 0;
    while (p + 4 <= bytes) {
        const uint32_t len = be32(buf + p);
        p += 4;
        if (len == 0) {
            // control frame: length, then the control type
            if (p + 4 > bytes) break;
            const uint32_t cl = be32(buf + p);
            p += 4;
            if (p + cl > bytes) break;
            const uint32_t ctype = cl >= 4 ? be32(buf + p) : 0;
            p += cl;
            if (ctype == 3) break; // STOP
            continue;
        }
        if (p + len > bytes) break; // a truncated data frame ends the stream
        nf++;
        DtMessage m;
        if (parse_dnstap(buf + p, len, m)) {
            m.frame_len = len;
            out.push_back(std::move(m));
        }
        p += len;
    }
    if (frames) *frames = nf;
    return 0;
}

} // namespace pvi
