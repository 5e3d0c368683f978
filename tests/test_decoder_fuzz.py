"""CPU fuzz: the product's DNS decode source (pv_parse.h, compiled for the host by
tests/native) against the oracle's restatement of DnsResource::decodeName /
DnsLayer::parseResources / aggregateDomain, on random and adversarial messages."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native", "libpvparse_host.so")


@pytest.fixture(scope="module")
def harness():
    if not os.path.exists(NATIVE):
        subprocess.check_call(["make", "-C", os.path.dirname(NATIVE)])
    h = ctypes.CDLL(NATIVE)
    h.h_decode_qname.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32)]
    h.h_decode_qname.restype = ctypes.c_uint32
    h.h_dns_parse.argtypes = [ctypes.c_char_p, ctypes.c_uint32] + [ctypes.POINTER(ctypes.c_int)] * 2 + [ctypes.POINTER(ctypes.c_uint32)]
    h.h_name_stats.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                               ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    return h


def oracle_fns(oracle):
    lib = oracle.lib
    lib.pvo_decode_qname.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32)]
    lib.pvo_decode_qname.restype = ctypes.c_uint32
    lib.pvo_dns_parse.argtypes = [ctypes.c_char_p, ctypes.c_uint32] + [ctypes.POINTER(ctypes.c_int)] * 2 + [ctypes.POINTER(ctypes.c_uint32)]
    lib.pvo_aggregate_domain.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_long)]
    lib.pvo_murmur3.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    return lib


def random_message(rng):
    """12-byte header + a name region built from labels, pointers and junk."""
    n = int(rng.integers(0, 300))
    kind = rng.integers(0, 6)
    hdr = bytearray(rng.integers(0, 256, 12, dtype=np.uint8).tobytes())
    hdr[4:6] = int(rng.integers(0, 3)).to_bytes(2, "big")
    if rng.integers(0, 3) == 0:
        hdr[6:12] = bytes(int(x) for x in rng.integers(0, 3, 6))
    body = bytearray()
    while len(body) < n:
        r = rng.integers(0, 10)
        if r < 5:  # label
            ln = int(rng.integers(0, 70)) if kind == 0 else int(rng.integers(1, 64))
            body.append(ln)
            alphabet = b"abcXYZ09-_." if kind != 1 else bytes(range(256))
            body += bytes(alphabet[int(i)] for i in rng.integers(0, len(alphabet), ln))
        elif r < 7:  # pointer (often into the message, sometimes illegal / self)
            target = int(rng.integers(0, max(13, 12 + len(body) + 20)))
            body += bytes([0xC0 | ((target >> 8) & 0x3F), target & 0xFF])
        elif r < 8:
            body.append(0)
        elif r < 9:
            body.append(int(rng.integers(0x40, 0xC0)))
        else:
            body += rng.integers(0, 256, int(rng.integers(1, 8)), dtype=np.uint8).tobytes()
    msg = bytes(hdr) + bytes(body)
    if rng.integers(0, 4) == 0:
        msg = msg[: int(rng.integers(0, len(msg) + 1))]
    return msg


def test_decode_name_matches_oracle(harness, oracle):
    lib = oracle_fns(oracle)
    rng = np.random.default_rng(12345)
    out_a, out_b = ctypes.create_string_buffer(4096), ctypes.create_string_buffer(4096)
    la, lb = ctypes.c_uint32(), ctypes.c_uint32()
    checked = 0
    for _ in range(60000):
        msg = random_message(rng)
        if len(msg) < 12:
            continue
        buf = msg + b"\0" * 16
        na = harness.h_decode_qname(buf, len(msg), out_a, ctypes.byref(la))
        nb = lib.pvo_decode_qname(buf, len(msg), out_b, ctypes.byref(lb))
        a, b = out_a.raw[: la.value], out_b.raw[: lb.value]
        assert (na, a) == (nb, b), (msg.hex(), na, a, nb, b)
        checked += 1
    assert checked > 40000


def test_parse_resources_matches_oracle(harness, oracle):
    lib = oracle_fns(oracle)
    rng = np.random.default_rng(777)
    ok1, hq1, ok2, hq2 = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    qt1, qt2 = ctypes.c_uint32(), ctypes.c_uint32()
    for _ in range(40000):
        msg = random_message(rng)
        if len(msg) < 12:
            continue
        buf = msg + b"\0" * 16
        harness.h_dns_parse(buf, len(msg), ctypes.byref(ok1), ctypes.byref(hq1), ctypes.byref(qt1))
        lib.pvo_dns_parse(buf, len(msg), ctypes.byref(ok2), ctypes.byref(hq2), ctypes.byref(qt2))
        assert (ok1.value, hq1.value) == (ok2.value, hq2.value), msg.hex()
        if ok1.value and hq1.value:
            assert qt1.value == qt2.value, msg.hex()


def test_name_stats_match_oracle(harness, oracle):
    """CPC hash of the lower-cased name and the aggregateDomain suffix positions."""
    lib = oracle_fns(oracle)
    rng = np.random.default_rng(99)
    n, q2, q3 = ctypes.c_uint32(), ctypes.c_int(), ctypes.c_int()
    h1, h2 = ctypes.c_uint64(), ctypes.c_uint64()
    out_b, lb = ctypes.create_string_buffer(4096), ctypes.c_uint32()
    mm = (ctypes.c_uint64 * 2)()
    s2, s3 = ctypes.c_size_t(), ctypes.c_long()
    for _ in range(30000):
        msg = random_message(rng)
        if len(msg) < 12:
            continue
        buf = msg + b"\0" * 16
        harness.h_name_stats(buf, len(msg), ctypes.byref(n), ctypes.byref(h1), ctypes.byref(h2), ctypes.byref(q2),
                             ctypes.byref(q3))
        nb = lib.pvo_decode_qname(buf, len(msg), out_b, ctypes.byref(lb))
        name = out_b.raw[: lb.value].lower() if nb > 0 else b""
        name = bytes(c + 32 if 65 <= c <= 90 else c for c in out_b.raw[: lb.value]) if nb > 0 else b""
        assert n.value == len(name), msg.hex()
        lib.pvo_murmur3(name, len(name), 9001, mm)
        assert (h1.value, h2.value) == (mm[0], mm[1]), msg.hex()
        if name:
            lib.pvo_aggregate_domain(name, len(name), 0, ctypes.byref(s2), ctypes.byref(s3))
            assert (q2.value, q3.value) == (s2.value, s3.value), (name, q2.value, q3.value, s2.value, s3.value)


def plain_name_message(rng):
    """A query whose name is plain labels (the name fast path's domain) or a near miss:
    NUL / '.' inside a label, 64+ length bytes, pointers, truncation, 255-byte limit."""
    labels = []
    nl = int(rng.integers(0, 12))
    alphabet = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_\x7f\x80\xc1\xff"
    for _ in range(nl):
        ln = int(rng.integers(1, 64)) if rng.integers(0, 4) else int(rng.integers(1, 6))
        lab = bytearray(alphabet[int(i)] for i in rng.integers(0, len(alphabet), ln))
        r = rng.integers(0, 40)
        if r == 0:
            lab[int(rng.integers(0, ln))] = 0
        elif r == 1:
            lab[int(rng.integers(0, ln))] = ord(".")
        labels.append(bytes([ln]) + bytes(lab))
    body = b"".join(labels)
    r = rng.integers(0, 12)
    if r == 0:
        body += bytes([0xC0, 12])
    elif r == 1:
        body += bytes([int(rng.integers(64, 192))])
    else:
        body += b"\x00"
    body += b"\x00\x01\x00\x01"
    hdr = bytes([1, 2, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0])
    msg = hdr + body
    if rng.integers(0, 6) == 0:
        msg = msg[: int(rng.integers(12, len(msg) + 1))]
    return msg


def test_name_fast_path_matches_general_decode(harness):
    """pv_parse.h name_stats_fast (the DNS pass's word-at-a-time path) equals the general
    byte-at-a-time decodeName walk field for field wherever it applies."""
    harness.h_name_fast_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    harness.h_name_fast_check.restype = ctypes.c_int
    rng = np.random.default_rng(777)
    took = 0
    for _ in range(40000):
        msg = plain_name_message(rng)
        buf = msg + bytes(32)  # readable past len, as the record blob's padding is
        r = harness.h_name_fast_check(buf, len(msg))
        assert r != 0, msg.hex()
        took += r == 1
    assert took > 15000, took
