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
