"""Classic-BPF programs (struct sock_filter tuples, as `tcpdump -dd` prints them) for the pcap
input's "bpf" filter tests, and an independent restatement of the classic-BPF machine
(linux/filter.h; libpcap's bpf_filter) the library's interpreter is checked against.
Parity unpinned: no reference fixture holds a filtered run (the reference compiles filter
expressions with libpcap, which this image lacks); the machine's semantics are the kernel's."""

# tcpdump -dd udp (Ethernet): IPv6 next header 17, or IPv6 fragment header then 17, or IPv4 proto 17
UDP = [(0x28, 0, 0, 12), (0x15, 0, 5, 0x86dd), (0x30, 0, 0, 20), (0x15, 6, 0, 17), (0x15, 0, 6, 0x2c),
       (0x30, 0, 0, 54), (0x15, 3, 4, 17), (0x15, 0, 3, 0x800), (0x30, 0, 0, 23), (0x15, 0, 1, 17),
       (0x6, 0, 0, 262144), (0x6, 0, 0, 0)]
# IPv4 UDP, not a fragment, either port 53 (ldxb 4*([14]&0xf), indexed half-word loads)
UDP53 = [(0x28, 0, 0, 12), (0x15, 0, 9, 0x800), (0x30, 0, 0, 23), (0x15, 0, 7, 17), (0x28, 0, 0, 20),
         (0x45, 5, 0, 0x1fff), (0xb1, 0, 0, 14), (0x48, 0, 0, 14), (0x15, 3, 0, 53), (0x48, 0, 0, 16),
         (0x15, 1, 0, 53), (0x6, 0, 0, 0), (0x6, 0, 0, 262144)]
# len <= 200
SHORT = [(0x80, 0, 0, 0), (0x25, 1, 0, 200), (0x6, 0, 0, 262144), (0x6, 0, 0, 0)]
# IPv4 with ((2 * (total length - 20)) / 4 % 1000 ^ 5) << 1 > 60: scratch memory, X, ALU ops, ret A
ARITH = [(0x28, 0, 0, 12), (0x15, 0, 11, 0x800), (0x28, 0, 0, 16), (0x14, 0, 0, 20), (0x02, 0, 0, 3),
         (0x61, 0, 0, 3), (0x0c, 0, 0, 0), (0x34, 0, 0, 4), (0x94, 0, 0, 1000), (0xa4, 0, 0, 5), (0x64, 0, 0, 1),
         (0x25, 0, 1, 60), (0x16, 0, 0, 0), (0x6, 0, 0, 0)]
PROGRAMS = {"udp": UDP, "udp53": UDP53, "short": SHORT, "arith": ARITH}
INVALID = {"empty": [], "no_ret": [(0x28, 0, 0, 12)], "jump_out": [(0x15, 5, 0, 1), (0x6, 0, 0, 0)],
           "div_zero": [(0x34, 0, 0, 0), (0x6, 0, 0, 0)], "mem_16": [(0x60, 0, 0, 16), (0x16, 0, 0, 0)],
           "bad_op": [(0xff, 0, 0, 0), (0x6, 0, 0, 0)]}


def run(prog, pkt: bytes, wirelen: int) -> int:
    """bpf_filter(prog, pkt, wirelen, len(pkt))"""
    a = x = 0
    mem = [0] * 16
    pc = 0
    n = len(pkt)
    m32 = 0xFFFFFFFF
    while True:
        code, jt, jf, k = prog[pc]
        c = code & 7
        if c in (0, 1):
            mode, size = code & 0xE0, code & 0x18
            if mode == 0x00:
                v = k
            elif mode == 0x80:
                v = wirelen
            elif mode == 0x60:
                v = mem[k]
            elif mode == 0xA0:
                if k >= n:
                    return 0
                v = (pkt[k] & 0xF) * 4
            else:
                off = (x if mode == 0x40 else 0) + k
                w = {0x00: 4, 0x08: 2, 0x10: 1}[size]
                if off + w > n:
                    return 0
                v = int.from_bytes(pkt[off:off + w], "big")
            if c == 0:
                a = v
            else:
                x = v
        elif c == 2:
            mem[k] = a
        elif c == 3:
            mem[k] = x
        elif c == 4:
            s = x if code & 8 else k
            op = code & 0xF0
            if op == 0x00:
                a = (a + s) & m32
            elif op == 0x10:
                a = (a - s) & m32
            elif op == 0x20:
                a = (a * s) & m32
            elif op == 0x30:
                if s == 0:
                    return 0
                a //= s
            elif op == 0x90:
                if s == 0:
                    return 0
                a %= s
            elif op == 0x40:
                a |= s
            elif op == 0x50:
                a &= s
            elif op == 0xA0:
                a ^= s
            elif op == 0x60:
                a = (a << (s & 31)) & m32
            elif op == 0x70:
                a >>= (s & 31)
            elif op == 0x80:
                a = (-a) & m32
        elif c == 5:
            op = code & 0xF0
            if op == 0x00:
                pc += k
            else:
                s = x if code & 8 else k
                t = a == s if op == 0x10 else a > s if op == 0x20 else a >= s if op == 0x30 else (a & s) != 0
                pc += jt if t else jf
        elif c == 6:
            return a if code & 0x18 == 0x10 else k
        elif c == 7:
            if code & 0xF8 == 0x80:
                a = x
            else:
                x = a
        pc += 1


def filter_records(recs: bytes, prog) -> bytes:
    """the classic-pcap records (host order) the program keeps"""
    import struct
    out = bytearray()
    pos = 0
    while pos + 16 <= len(recs):
        incl, orig = struct.unpack_from("<II", recs, pos + 8)
        if pos + 16 + incl > len(recs):
            break
        if run(prog, recs[pos + 16:pos + 16 + incl], orig):
            out += recs[pos:pos + 16 + incl]
        pos += 16 + incl
    return bytes(out)
