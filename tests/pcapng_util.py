"""Test helper: write a classic pcap's packets as pcapng (IETF draft-tuexen-opsawg-pcapng), in
the block kinds and options pv_pcapng_records must read (not a fixture of the reference: the
reference's tests hold no pcapng file)."""
import struct


def pcap_packets(pcap: bytes):
    magic, = struct.unpack_from("<I", pcap, 0)
    nano = magic == 0xA1B23C4D
    lt, = struct.unpack_from("<I", pcap, 20)
    p, out = 24, []
    while p + 16 <= len(pcap):
        s, f, cl, ol = struct.unpack_from("<IIII", pcap, p)
        out.append((s, f * (1 if nano else 1000), cl, ol, pcap[p + 16:p + 16 + cl]))
        p += 16 + cl
    return lt, out


def _blk(t, body, be=False):
    e = ">" if be else "<"
    body += b"\0" * (-len(body) % 4)
    n = len(body) + 12
    return struct.pack(e + "II", t, n) + body + struct.pack(e + "I", n)


def _opt(code, val, be=False):
    e = ">" if be else "<"
    return struct.pack(e + "HH", code, len(val)) + val + b"\0" * (-len(val) % 4)


def to_pcapng(pcap: bytes, tsresol=None, be=False, sections=1, simple=False, options=True):
    """tsresol: None = default 10^-6, else the if_tsresol byte (9 = ns, 0x80|k = 2^-k);
    sections: packets split over this many sections; simple: Simple Packet Blocks (no ts)"""
    e = ">" if be else "<"
    lt, pk = pcap_packets(pcap)
    out = b""
    per = -(-len(pk) // sections) if pk else 0
    for k in range(sections):
        shb = struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1)
        if options:
            shb += _opt(4, b"pvgpu test\0", be) + _opt(0, b"", be)
        out += _blk(0x0A0D0D0A, shb, be)
        idb = struct.pack(e + "HHI", lt, 0, 262144)
        if tsresol is not None:
            idb += _opt(9, bytes([tsresol]), be)
        if options or tsresol is not None:
            idb += _opt(2, b"eth0", be) + _opt(0, b"", be)
        out += _blk(1, idb, be)
        if options:
            out += _blk(0x00000BAD, b"custom block", be)  # unknown block: skipped
        for s, ns, cl, ol, data in pk[k * per:(k + 1) * per]:
            if simple:
                out += _blk(3, struct.pack(e + "I", ol) + data, be)
                continue
            if tsresol is None:
                t = s * 1000000 + ns // 1000
            elif tsresol & 0x80:
                b = tsresol & 0x7f
                t = (s << b) + (ns << b) // 1000000000
            else:
                t = s * 10 ** tsresol + ns * 10 ** tsresol // 1000000000
            body = struct.pack(e + "IIIII", 0, t >> 32, t & 0xffffffff, cl, ol) + data
            if options:
                body += b"\0" * (-len(body) % 4) + _opt(1, b"c", be) + _opt(0, b"", be)
            out += _blk(6, body, be)
    return out
