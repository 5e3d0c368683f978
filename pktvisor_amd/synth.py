"""Seeded synthetic pcaps for the BASELINE.json configs (via tools/libpvgen.so).

Test and bench infrastructure only: the product never generates traffic.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "tools", "libpvgen.so")

SEEDS = {1: 0x5EED0001, 2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005, 9: 0x5EED0009}
HOST_SPEC = "10.0.0.0/8"

_gen = None


def _lib():
    global _gen
    if _gen is None:
        if not os.path.exists(GEN):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "tools")])
        g = ctypes.CDLL(GEN)
        g.pvgen_records.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                                    ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
        g.pvgen_records.restype = ctypes.c_int64
        g.pvgen_records_at.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
        g.pvgen_records_at.restype = ctypes.c_int64
        g.pvgen_bound.argtypes = [ctypes.c_int, ctypes.c_uint64]
        g.pvgen_bound.restype = ctypes.c_uint64
        _gen = g
    return _gen


def records(cfg: int, n: int, seed: int | None = None, ts_step_us: int = 1, with_offsets: bool = False):
    """Returns (record bytes as np.uint8 array incl. 256 B zero padding, offsets or None, used bytes)."""
    g = _lib()
    cap = int(g.pvgen_bound(cfg, n))
    buf = np.zeros(cap, dtype=np.uint8)
    offs = np.empty(n, dtype=np.uint32) if with_offsets else None
    used = ctypes.c_size_t()
    got = g.pvgen_records(cfg, n, SEEDS.get(cfg, 1) if seed is None else seed, ts_step_us, buf.ctypes.data, cap,
                          ctypes.byref(used), offs.ctypes.data if offs is not None else None)
    if got != n:
        raise RuntimeError(f"pvgen failed for cfg {cfg}: {got}")
    return buf[: used.value + 256], offs, used.value


T0_US = 1700000000 * 1000000  # the generator's first timestamp


def stream_shard(cfg: int, lo: int, hi: int, seed: int, ts_step_us: int = 1, chunk: int = 10_000_000, progress=None):
    """Records [lo, hi) of a synthetic stream of the config's shape at ts_step_us per record:
    generated in chunks of `chunk` records (each its own seed, timestamps continuing at
    T0 + index * step), returned as one np.uint8 array (+256 B zero padding) and its used bytes."""
    g = _lib()
    parts, total = [], 0
    for a in range(lo, hi, chunk):
        b = min(hi, a + chunk)
        cap = int(g.pvgen_bound(cfg, b - a))
        buf = np.zeros(cap, dtype=np.uint8)
        used = ctypes.c_size_t()
        got = g.pvgen_records_at(cfg, b - a, seed + 104729 * (a // chunk), ts_step_us, T0_US + a * ts_step_us,
                                 buf.ctypes.data, cap, ctypes.byref(used), None)
        if got != b - a:
            raise RuntimeError(f"pvgen failed for cfg {cfg}: {got}")
        parts.append(buf[: used.value].copy())
        del buf
        total += used.value
        if progress:
            progress(b - lo)
    out = np.zeros(total + 256, dtype=np.uint8)
    at = 0
    for p in parts:
        out[at:at + len(p)] = p
        at += len(p)
    return out, total


def pcap_bytes(cfg: int, n: int, seed: int | None = None, ts_step_us: int = 1) -> bytes:
    from pktvisor_amd import pcap_file_bytes
    buf, _, used = records(cfg, n, seed, ts_step_us)
    return pcap_file_bytes(buf[:used].tobytes())


def records_of(pcap: bytes):
    """[(ts_sec, ts_usec, record bytes)] of a classic little-endian pcap image"""
    import struct
    out, pos = [], 24
    while pos + 16 <= len(pcap):
        sec, usec, incl, _ = struct.unpack_from("<IIII", pcap, pos)
        out.append((sec, usec, pcap[pos:pos + 16 + incl]))
        pos += 16 + incl
    return out


def is_udp_dns(rec: bytes) -> bool:
    """Ethernet + IPv4 (no options) UDP datagram on port 53 (the generator's DNS frames)"""
    f = rec[16:]
    return (len(f) >= 38 and f[12:14] == b"\x08\x00" and f[14] == 0x45 and f[23] == 17
            and (f[34:36] == b"\x00\x35" or f[36:38] == b"\x00\x35"))


def sparse_dns_pcap(n: int = 120000, ts_step_us: int = 2500, quiet=(52, 9), seed: int | None = None) -> bytes:
    """C4 traffic spanning several minutes with no DNS packet in the seconds around every 60 s
    mark after the capture's start (second offsets whose remainder mod 60 is >= quiet[0] or
    < quiet[1]): the DNS manager then shifts seconds after the Net manager, and the gap between
    the two boundaries drifts from one period to the next."""
    from pktvisor_amd import pcap_file_bytes
    recs = records_of(pcap_bytes(4, n, seed=seed, ts_step_us=ts_step_us))
    t0 = recs[0][0]
    keep = [r for s, _, r in recs if not (is_udp_dns(r) and ((s - t0) % 60 >= quiet[0] or (s - t0) % 60 < quiet[1]))]
    return pcap_file_bytes(b"".join(keep))


def merged_pcap(*pcaps) -> bytes:
    """the records of several classic pcaps in one capture, in timestamp order (ties: argument
    order, then each capture's own order)"""
    from pktvisor_amd import pcap_file_bytes
    allr = []
    for k, pc in enumerate(pcaps):
        allr += [(s, u, k, i, r) for i, (s, u, r) in enumerate(records_of(pc))]
    allr.sort(key=lambda x: x[:4])
    return pcap_file_bytes(b"".join(x[4] for x in allr))


def c4_tcp_pcap(n: int = 120000, ts_step_us: int = 2500, flows: int = 300, seed: int = 3) -> bytes:
    """C4 traffic over n * ts_step_us (300 s by default: several 60 s marks) with DNS-over-TCP
    connections (tcp_dns_pcap) spread over the same span"""
    dur = n * ts_step_us / 1e6
    return merged_pcap(pcap_bytes(4, n, ts_step_us=ts_step_us), tcp_dns_pcap(seed=seed, flows=flows, duration_s=dur * 0.95))


# ---------------------------------------------------------------- DNS over TCP
def _dns_msg(rng, txid: int, qr: bool, name: str, qtype: int, rcode: int = 0, answers: int = 0) -> bytes:
    import struct
    q = b"".join(bytes([len(l)]) + l.encode() for l in name.split(".")) + b"\x00" + struct.pack(">HH", qtype, 1)
    flags = (0x8180 | rcode) if qr else 0x0100
    hdr = struct.pack(">HHHHHH", txid, flags, 1, answers, 0, 0)
    ans = b"".join(struct.pack(">HHHIH", 0xC00C, 1, 1, 300, 4) + bytes(rng.integers(0, 256, 4, dtype=np.uint8))
                   for _ in range(answers))
    return hdr + q + ans


def _frame(src, dst, sport, dport, seq, flags, payload, v6):
    """Ethernet + IPv4 / IPv6 + TCP (ack 0, window 0) carrying payload"""
    import struct
    tcp = struct.pack(">HHIIBBHHH", sport, dport, seq & 0xffffffff, 0, 0x50, flags, 65535, 0, 0) + payload
    if v6:
        ip = struct.pack(">IHBB", 0x60000000, len(tcp), 6, 64) + src + dst
        return b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb\x86\xdd" + ip + tcp
    ip = struct.pack(">BBHHHBBH", 0x45, 0, 20 + len(tcp), 0, 0, 64, 6, 0) + src + dst
    return b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb\x08\x00" + ip + tcp


def tcp_dns_pcap(seed: int = 1, flows: int = 60, duration_s: float = 20.0, udp_share: float = 0.3,
                 noise_share: float = 0.3, pauses: int = 0, open_tails: int = 0) -> bytes:
    """DNS over TCP traffic for the reassembly parity tests: connections to port 53 (IPv4 and
    IPv6) carrying pipelined queries and responses that are cut into segments at random byte
    boundaries, with out-of-order segments, duplicate and overlapping retransmissions, a
    lost SYN (the first captured packet carries data), invalid framing (a length below 17),
    FIN and RST closes, a reused client port after a close; interleaved with UDP DNS and
    non-DNS TCP noise (port 443). With pauses > 0 that many connections fall silent for 35 s
    while the noise goes on (PcapInputStream's 30 s TCP timeout). Timestamps are monotone.
    Every connection with a gap left in its stream ends with FIN or RST, except with
    open_tails > 0: that many connections lose one data segment for good and send no FIN or
    RST, so the segments after the hole are still held when the capture ends and only the
    end-of-capture flush delivers them (PcapInputStream closes every connection when the
    file is read, TcpReassembly::closeAllConnections; the device path emits those closes
    with pv_set_end_of_capture, pv_tcp.hip)."""
    import struct
    from pktvisor_amd import pcap_file_bytes
    rng = np.random.default_rng(seed)
    names = [f"{''.join(chr(97 + int(c)) for c in rng.integers(0, 26, 6))}.example.{tld}" for tld in ("com", "net", "org")
             for _ in range(7)]

    def addr(v6, server):
        if v6:
            return (bytes.fromhex("20014860000000000000000000008888") if server else
                    bytes.fromhex("20010db8") + bytes(rng.integers(0, 256, 12, dtype=np.uint8)))
        return bytes([8, 8, 8, 8]) if server else bytes([10, int(rng.integers(0, 256)), int(rng.integers(0, 256)),
                                                         int(rng.integers(1, 255))])

    streams = []  # per connection: its packets in send order
    used_ports = []
    # connections that fall silent for 35 s keep their segments in order (a timeout that
    # flushes buffered data is ordered differently on the device, see pv_tcp.hip)
    pause_flows = set(rng.choice(flows, size=min(pauses, flows), replace=False).tolist()) if pauses else set()
    tail_rng = np.random.default_rng(seed + 7919)  # keeps the other flows as without open_tails
    open_flows = set(tail_rng.choice([f for f in range(flows) if f not in pause_flows],
                                     size=min(open_tails, flows - len(pause_flows)), replace=False).tolist()) \
        if open_tails else set()
    for f in range(flows):
        v6 = bool(rng.random() < 0.3)
        cli, srv = addr(v6, False), addr(v6, True)
        cport = int(rng.integers(1024, 60000))
        if cport in (5353, 5355, 53000):
            cport += 1
        if used_ports and rng.random() < 0.05:  # a client port reused after a close
            cli, srv, cport, v6 = used_ports[int(rng.integers(0, len(used_ports)))]
        used_ports.append((cli, srv, cport, v6))
        cseq, sseq = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
        ntx = int(rng.integers(1, 6))
        cbytes, sbytes = b"", b""
        for t in range(ntx):
            name = names[int(rng.integers(0, len(names)))]
            qt = [1, 28, 15, 16][int(rng.integers(0, 4))]
            txid = int(rng.integers(0, 65536))
            q = _dns_msg(rng, txid, False, name, qt)
            r = _dns_msg(rng, txid, True, name, qt, [0, 0, 0, 3, 2][int(rng.integers(0, 5))], int(rng.integers(0, 3)))
            cbytes += struct.pack(">H", len(q)) + q
            sbytes += struct.pack(">H", len(r)) + r
        if rng.random() < 0.05:  # invalid framing on the client side: a length below 17
            cbytes += b"\x00\x05" + bytes(30)
        pkts = []
        lost_syn = rng.random() < 0.08 and f not in pause_flows
        if not lost_syn:
            pkts.append((cli, srv, cport, 53, cseq, 0x02, b""))
            pkts.append((srv, cli, 53, cport, sseq, 0x12, b""))
        cseq += 1
        sseq += 1

        def cut(data, seq0, src, dst, sp, dp):
            out, pos = [], 0
            while pos < len(data):
                n = int(rng.integers(1, 120)) if rng.random() < 0.7 else len(data) - pos
                out.append((src, dst, sp, dp, seq0 + pos, 0x18, data[pos:pos + n]))
                pos += n
            return out

        csegs = cut(cbytes, cseq, cli, srv, cport, 53)
        ssegs = cut(sbytes, sseq, srv, cli, 53, cport)
        gaps = False
        for segs in (csegs, ssegs):
            # out-of-order pairs, duplicates and overlapping retransmissions
            for k in range(len(segs) - 1):
                if rng.random() < 0.12 and f not in pause_flows:
                    segs[k], segs[k + 1] = segs[k + 1], segs[k]
                    gaps = True
            k = 0
            while k < len(segs):
                if rng.random() < 0.06:
                    s = segs[k]
                    if rng.random() < 0.5 or k + 1 >= len(segs):
                        segs.insert(k + 1, s)  # duplicate
                    else:
                        nxt = segs[k + 1]
                        segs.insert(k + 1, (s[0], s[1], s[2], s[3], s[4], 0x18, s[6] + nxt[6][:max(1, len(nxt[6]) // 2)]))
                    k += 1
                k += 1
        if f in open_flows:
            # one data segment never arrives: what follows it waits for the end of the capture
            sides = [x for x in (csegs, ssegs) if len(x) >= 2]
            if sides:
                segs = sides[int(tail_rng.integers(0, len(sides)))]
                del segs[int(tail_rng.integers(0, len(segs) - 1))]
        pkts += csegs + ssegs if rng.random() < 0.5 else [p for pair in zip(csegs, ssegs) for p in pair] + \
            csegs[len(ssegs):] + ssegs[len(csegs):]
        end = rng.random()
        if f in open_flows:
            streams.append(list(pkts))
            continue
        if end < 0.6 or gaps:
            pkts.append((cli, srv, cport, 53, cseq + len(cbytes), 0x11, b""))
            pkts.append((srv, cli, 53, cport, sseq + len(sbytes), 0x11, b""))
        elif end < 0.85:
            pkts.append((srv, cli, 53, cport, sseq + len(sbytes), 0x04, b""))
        streams.append([p for p in pkts])
    # interleave: connections start at random times, their packets keep order
    t0 = 1700000000.0
    n_total = sum(len(s) for s in streams)
    events = []
    for f, s in enumerate(streams):
        start = rng.random() * duration_s
        t = start
        for k, p in enumerate(s):
            t += float(rng.exponential(0.02))
            if f in pause_flows and k == len(s) // 2:
                t += 35.0
            events.append((t, f, k, p))
    tmax = max(e[0] for e in events) if events else 0.0
    # UDP DNS and non-DNS TCP noise over the whole span (the noise carries the clock)
    n_udp, n_noise = int(n_total * udp_share), int(n_total * noise_share) + (int(tmax * 20) if pauses else 0)
    for _ in range(n_udp):
        t = rng.random() * tmax
        name = names[int(rng.integers(0, len(names)))]
        m = _dns_msg(rng, int(rng.integers(0, 65536)), bool(rng.random() < 0.5), name, 1)
        sp = int(rng.integers(1024, 60000))
        udp = struct.pack(">HHHH", sp, 53, 8 + len(m), 0) + m
        ip = struct.pack(">BBHHHBBH", 0x45, 0, 20 + len(udp), 0, 0, 64, 17, 0) + bytes([10, 9, 9, 9]) + bytes([8, 8, 8, 8])
        events.append((t, -1, 0, b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb\x08\x00" + ip + udp))
    # noise: eight long-lived port-443 connections (SYN, then in-order data), and every 20 s an
    # "anchor" connection that opens and stays silent. PcapInputStream closes the LRU list's
    # least recently used connection once it is 30 s old; a connection whose first captured
    # packet carries data enters that list with time 0 (ConnectionData::endTime is unset
    # until a second packet), and dies as soon as it is the list's oldest: an anchor keeps
    # an older entry alive, as a busy capture does (the device path dates that entry by
    # the packet instead, pv_tcp.hip).
    nseq = [int(rng.integers(0, 2**32)) for _ in range(8)]
    for c in range(8):
        events.append((0.0, -2, -100 + c, _frame(bytes([10, 1, 1, 1]), bytes([1, 2, 3, c]), 40000 + c, 443, nseq[c], 0x02, b"", False)))
        nseq[c] += 1
    for a in range(int(tmax // 20) + 2):
        events.append((a * 20.0, -2, -200 + a, _frame(bytes([10, 1, 1, 2]), bytes([1, 2, 4, 4]), 30000 + a, 443, 7, 0x02, b"", False)))
    for k in range(n_noise):
        t = (k + rng.random()) * tmax / max(n_noise, 1)
        c = k % 8
        pl = bytes(int(rng.integers(1, 40)))
        events.append((t, -2, k, _frame(bytes([10, 1, 1, 1]), bytes([1, 2, 3, c]), 40000 + c, 443, nseq[c], 0x18, pl, False)))
        nseq[c] += len(pl)
    events.sort(key=lambda e: (e[0], e[1], e[2]))
    out = bytearray()
    for t, f, k, p in events:
        fr = _frame(*p[:6], p[6], len(p[0]) == 16) if f >= 0 else p
        us = int(round((t0 + t) * 1e6))
        out += struct.pack("<IIII", us // 1000000, us % 1000000, len(fr), len(fr)) + fr
    return pcap_file_bytes(bytes(out))


def _pcap_of(events) -> bytes:
    """(seconds, frame) pairs, sorted by time, as a classic pcap file"""
    import struct
    from pktvisor_amd import pcap_file_bytes
    out = bytearray()
    for t, fr in sorted(events, key=lambda e: e[0]):
        us = int(round((1700000000.0 + t) * 1e6))
        out += struct.pack("<IIII", us // 1000000, us % 1000000, len(fr), len(fr)) + fr
    return pcap_file_bytes(bytes(out))


def tcp_reput_pcap() -> bytes:
    """Three DNS-over-TCP connections under tcp_packet_reassembly_cache_limit = 2, one second
    apart (PcapInputStream.cpp:254-283,429-465):
      A: SYN, then a segment 10 bytes past the next sequence (held out of order);
      B: SYN, then the first 10 bytes of a framed 24-byte query (length + 8 bytes);
      C: SYN: its put overflows the list [C, B, A] and evicts A. Closing A flushes the held
         fragment behind "[10 bytes missing]", whose delivery puts A into the list again
         ([A, C, B]): that put evicts B, which the same overflow loop closes;
      B: the remaining 16 bytes of the query: a packet of a closed flow, ignored.
    So no TCP query is counted; a replay without the flush's put keeps B open and counts one."""
    import struct
    srv = bytes([8, 8, 8, 8])
    q = _dns_msg(np.random.default_rng(0), 0x1234, False, "ab.com", 1)
    assert len(q) == 24
    framed = struct.pack(">H", len(q)) + q
    a, b, c = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2]), bytes([10, 0, 0, 3])
    sa, sb, sc = 1000, 5000, 9000
    ev = [(0.0, _frame(a, srv, 1001, 53, sa, 0x02, b"", False)),
          (1.0, _frame(a, srv, 1001, 53, sa + 1 + 10, 0x18, bytes(range(1, 21)), False)),
          (2.0, _frame(b, srv, 1002, 53, sb, 0x02, b"", False)),
          (3.0, _frame(b, srv, 1002, 53, sb + 1, 0x18, framed[:10], False)),
          (4.0, _frame(c, srv, 1003, 53, sc, 0x02, b"", False)),
          (5.0, _frame(b, srv, 1002, 53, sb + 11, 0x18, framed[10:], False))]
    return _pcap_of(ev)


def tcp_held_evict_pcap(seed: int = 1, flows: int = 48, duration_s: float = 12.0) -> bytes:
    """DNS-over-TCP connections that hold out-of-order fragments for a long time while many
    others start: each client sends its framed queries cut into 3-6 segments, the second one
    delayed by 0.3-3 s behind the later ones, then FIN; the server answers in order. Under a
    small tcp_packet_reassembly_cache_limit the list evicts connections that hold fragments,
    whose closes put them into the list again (tcp_reput_pcap)."""
    import struct
    rng = np.random.default_rng(seed)
    srv = bytes([8, 8, 8, 8])
    names = [f"h{k}.example.{tld}" for k in range(6) for tld in ("com", "net")]
    ev = []
    for f in range(flows):
        cli = bytes([10, 1, int(rng.integers(0, 256)), int(rng.integers(1, 255))])
        cp = 2000 + f
        cs, ss = int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))
        cb, sb = b"", b""
        for _ in range(int(rng.integers(1, 4))):
            name = names[int(rng.integers(0, len(names)))]
            txid = int(rng.integers(0, 65536))
            qm = _dns_msg(rng, txid, False, name, 1)
            rm = _dns_msg(rng, txid, True, name, 1, 0, int(rng.integers(0, 3)))
            cb += struct.pack(">H", len(qm)) + qm
            sb += struct.pack(">H", len(rm)) + rm
        cuts = sorted(set(int(x) for x in rng.integers(1, len(cb), int(rng.integers(2, 6)))))
        bounds = [0] + cuts + [len(cb)]
        segs = [(cs + 1 + bounds[k], cb[bounds[k]:bounds[k + 1]]) for k in range(len(bounds) - 1)]
        t = float(rng.random() * duration_s)
        ev.append((t, _frame(cli, srv, cp, 53, cs, 0x02, b"", False)))
        t += float(rng.exponential(0.05))
        ev.append((t, _frame(srv, cli, 53, cp, ss, 0x12, b"", False)))
        late = 1 if len(segs) > 2 else len(segs) - 1
        for k, (sq, pl) in enumerate(segs):
            if k == late:
                continue
            t += float(rng.exponential(0.05))
            ev.append((t, _frame(cli, srv, cp, 53, sq, 0x18, pl, False)))
        t += 0.3 + float(rng.random()) * 2.7
        ev.append((t, _frame(cli, srv, cp, 53, segs[late][0], 0x18, segs[late][1], False)))
        t += float(rng.exponential(0.05))
        ev.append((t, _frame(srv, cli, 53, cp, ss + 1, 0x18, sb, False)))
        t += float(rng.exponential(0.05))
        ev.append((t, _frame(cli, srv, cp, 53, cs + 1 + len(cb), 0x11, b"", False)))
        ev.append((t + 0.01, _frame(srv, cli, 53, cp, ss + 1 + len(sb), 0x11, b"", False)))
    return _pcap_of(ev)


# ---------------------------------------------------------------- random-subdomain flood
def qname_flood_pcap(seed: int = 1, heavy: int = 24, flood: int = 40000, duration_s: float = 40.0):
    """UDP DNS queries for a random-subdomain flood: `flood` distinct one-off names
    <random>.victim.example next to `heavy` repeated names www<i>.victim.example with
    Zipf-like counts, interleaved at random over duration_s (inside one 60 s period).
    Returns (pcap bytes, {heavy name: count}, total queries)."""
    import struct
    from pktvisor_amd import pcap_file_bytes
    rng = np.random.default_rng(seed)
    counts = {f"www{i}.victim.example": int(3000 // (i + 1)) + 40 for i in range(heavy)}
    names = [n for n, c in counts.items() for _ in range(c)]
    names += [f"{rng.integers(1 << 40):010x}.victim.example" for _ in range(flood)]
    order = rng.permutation(len(names))
    t0 = 1_700_000_000_000_000
    step = int(duration_s * 1e6 / len(names))
    out = []
    for k, j in enumerate(order):
        msg = _dns_msg(rng, int(rng.integers(65536)), False, names[j], 1)
        udp = struct.pack(">HHHH", 1024 + k % 50000, 53, 8 + len(msg), 0) + msg
        ip = struct.pack(">BBHHHBBH", 0x45, 0, 20 + len(udp), 0, 0, 64, 17, 0) + bytes([10, 0, k % 200, 1]) + bytes([8, 8, 8, 8])
        f = b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb\x08\x00" + ip + udp
        ts = t0 + k * step
        out.append(struct.pack("<IIII", ts // 1_000_000, ts % 1_000_000, len(f), len(f)) + f)
    return pcap_file_bytes(b"".join(out)), counts, len(names)
