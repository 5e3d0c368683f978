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
