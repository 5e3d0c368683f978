// SPDX-License-Identifier: MPL-2.0
// pv_bpf.cpp — the pcap input's BPF filter (PcapInputStream::_open_pcap: reader->setFilter(bpf),
// src/inputs/pcap/PcapInputStream.cpp:485-488) for records handed to pv_process_host.
//
// libpcap compiles the filter expression to a classic-BPF program and runs it on every record
// it reads (pcap_offline_filter → bpf_filter: the frame from its link layer, the capture length
// as the buffer, the wire length for BPF_LEN); a record the program answers 0 for never reaches
// the input's handlers. libpcap is not in this image, so the ABI takes the compiled program
// (struct sock_filter, what `tcpdump -dd EXPR` prints and AF_PACKET's SO_ATTACH_FILTER takes)
// and this file is the interpreter, restating the classic-BPF machine (linux/filter.h opcodes;
// the checks of the kernel's bpf_check_classic / libpcap's bpf_validate).
#include <string.h>

#include <vector>

#include "../../include/pvgpu.h"

namespace {

// opcode fields (linux/bpf_common.h)
enum : uint16_t {
    LD = 0x00, LDX = 0x01, ST = 0x02, STX = 0x03, ALU = 0x04, JMP = 0x05, RET = 0x06, MISC = 0x07,
    W = 0x00, H = 0x08, B = 0x10,
    IMM = 0x00, ABS = 0x20, IND = 0x40, MEM = 0x60, LEN = 0x80, MSH = 0xa0,
    ADD = 0x00, SUB = 0x10, MUL = 0x20, DIV = 0x30, OR = 0x40, AND = 0x50, LSH = 0x60, RSH = 0x70, NEG = 0x80,
    MOD = 0x90, XOR = 0xa0,
    JA = 0x00, JEQ = 0x10, JGT = 0x20, JGE = 0x30, JSET = 0x40,
    K = 0x00, X = 0x08, A = 0x10,
    TAX = 0x00, TXA = 0x80,
};
constexpr uint32_t MEMWORDS = 16;
constexpr uint32_t MAXINSNS = 4096;

inline uint32_t cls(uint16_t c) { return c & 0x07; }

// bytes [k, k + n) of the frame, big-endian; false past the capture (the program returns 0)
inline bool load(const uint8_t *p, uint32_t buflen, uint64_t k, uint32_t n, uint32_t &v)
{
    if (k + n > buflen) return false;
    v = 0;
    for (uint32_t i = 0; i < n; i++) v = (v << 8) | p[k + i];
    return true;
}

} // namespace

extern "C" int pv_bpf_validate(const pv_bpf_insn *prog, uint32_t n)
{
    if (!prog || n == 0 || n > MAXINSNS) return PV_EINVAL;
    for (uint32_t pc = 0; pc < n; pc++) {
        const pv_bpf_insn &f = prog[pc];
        const uint16_t c = f.code;
        switch (cls(c)) {
        case LD:
        case LDX: {
            const uint16_t mode = c & 0xe0, size = c & 0x18;
            if (cls(c) == LD) {
                if (mode == ABS || mode == IND) { if (size != W && size != H && size != B) return PV_EINVAL; }
                else if (mode == MEM) { if (f.k >= MEMWORDS) return PV_EINVAL; }
                else if (mode != IMM && mode != LEN) return PV_EINVAL;
                if ((mode == IMM || mode == LEN || mode == MEM) && size != W) return PV_EINVAL;
            } else {
                if (mode == MEM) { if (f.k >= MEMWORDS || size != W) return PV_EINVAL; }
                else if (mode == MSH) { if (size != B) return PV_EINVAL; }
                else if ((mode != IMM && mode != LEN) || size != W) return PV_EINVAL;
            }
            if (c & ~0xffu) return PV_EINVAL;
            break;
        }
        case ST:
        case STX:
            if (c != cls(c) || f.k >= MEMWORDS) return PV_EINVAL;
            break;
        case ALU: {
            const uint16_t op = c & 0xf0;
            if (c & ~0xffu || (c & 0x07) != ALU) return PV_EINVAL;
            if (op > XOR) return PV_EINVAL;
            if (op == NEG) { if (c & X) return PV_EINVAL; }
            else if ((op == DIV || op == MOD) && !(c & X) && f.k == 0) return PV_EINVAL; // division by a constant 0
            break;
        }
        case JMP: {
            const uint16_t op = c & 0xf0;
            if (c & ~0xffu) return PV_EINVAL;
            if (op == JA) {
                if ((c & X) || (uint64_t)pc + 1 + f.k >= n) return PV_EINVAL;
            } else if (op == JEQ || op == JGT || op == JGE || op == JSET) {
                if ((uint64_t)pc + 1 + f.jt >= n || (uint64_t)pc + 1 + f.jf >= n) return PV_EINVAL;
            } else {
                return PV_EINVAL;
            }
            break;
        }
        case RET: {
            const uint16_t src = c & 0x18;
            if (c & ~0xffu || (src != K && src != A) || (c & 0xe0)) return PV_EINVAL;
            break;
        }
        case MISC:
            if (c != (MISC | TAX) && c != (MISC | TXA)) return PV_EINVAL;
            break;
        }
    }
    return cls(prog[n - 1].code) == RET ? PV_OK : PV_EINVAL;
}

// bpf_filter: the program's answer for one frame (0 = drop); the program must validate
extern "C" uint32_t pv_bpf_run(const pv_bpf_insn *prog, const uint8_t *p, uint32_t wirelen, uint32_t buflen)
{
    uint32_t a = 0, x = 0, mem[MEMWORDS] = {0};
    for (uint32_t pc = 0;; pc++) {
        const pv_bpf_insn &f = prog[pc];
        const uint16_t c = f.code;
        uint32_t v;
        switch (cls(c)) {
        case LD: {
            const uint16_t mode = c & 0xe0;
            const uint32_t n = (c & 0x18) == W ? 4 : (c & 0x18) == H ? 2 : 1;
            if (mode == IMM) a = f.k;
            else if (mode == LEN) a = wirelen;
            else if (mode == MEM) a = mem[f.k];
            else {
                const uint64_t off = (mode == IND ? (uint64_t)x : 0) + f.k;
                if (!load(p, buflen, off, n, v)) return 0;
                a = v;
            }
            break;
        }
        case LDX: {
            const uint16_t mode = c & 0xe0;
            if (mode == IMM) x = f.k;
            else if (mode == LEN) x = wirelen;
            else if (mode == MEM) x = mem[f.k];
            else { // MSH: 4 * (low nibble of the byte at k), the IPv4 header length
                if (!load(p, buflen, f.k, 1, v)) return 0;
                x = (v & 0xf) << 2;
            }
            break;
        }
        case ST: mem[f.k] = a; break;
        case STX: mem[f.k] = x; break;
        case ALU: {
            const uint32_t s = (c & X) ? x : f.k;
            switch (c & 0xf0) {
            case ADD: a += s; break;
            case SUB: a -= s; break;
            case MUL: a *= s; break;
            case DIV: if (!s) return 0; a /= s; break;
            case MOD: if (!s) return 0; a %= s; break;
            case OR: a |= s; break;
            case AND: a &= s; break;
            case XOR: a ^= s; break;
            case LSH: a <<= (s & 31); break; // libpcap's C shift on x86: the count taken mod 32
            case RSH: a >>= (s & 31); break;
            case NEG: a = 0u - a; break;
            }
            break;
        }
        case JMP: {
            const uint16_t op = c & 0xf0;
            if (op == JA) { pc += f.k; break; }
            const uint32_t s = (c & X) ? x : f.k;
            const bool t = op == JEQ ? a == s : op == JGT ? a > s : op == JGE ? a >= s : (a & s) != 0;
            pc += t ? f.jt : f.jf;
            break;
        }
        case RET: return (c & 0x18) == A ? a : f.k;
        case MISC: if ((c & 0xf8) == TXA) a = x; else x = a; break;
        }
    }
}

// The records of [recs, recs + bytes) the program keeps, copied in order to out (at most bytes
// long); *out_bytes and *kept report them. A record cut short by the end of the block is left
// out with everything after it (pv_index_records' rule); records are classic-pcap, host order.
extern "C" int pv_bpf_filter_records(const pv_bpf_insn *prog, uint32_t n, const uint8_t *recs, size_t bytes, uint8_t *out,
                                     size_t *out_bytes, uint64_t *kept)
{
    if (int rc = pv_bpf_validate(prog, n)) return rc;
    if ((!recs && bytes) || !out_bytes) return PV_EINVAL;
    size_t pos = 0, o = 0;
    uint64_t k = 0;
    while (pos + 16 <= bytes) {
        uint32_t incl, orig;
        memcpy(&incl, recs + pos + 8, 4);
        memcpy(&orig, recs + pos + 12, 4);
        if (pos + 16 + (size_t)incl > bytes) break;
        if (pv_bpf_run(prog, recs + pos + 16, orig, incl)) {
            if (out && out + o != recs + pos) memmove(out + o, recs + pos, 16 + (size_t)incl);
            o += 16 + (size_t)incl;
            k++;
        }
        pos += 16 + (size_t)incl;
    }
    *out_bytes = o;
    if (kept) *kept = k;
    return PV_OK;
}
