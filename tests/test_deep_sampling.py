"""Deep sampling (deep_sample_rate < 100, AbstractMetricsManager::new_event,
src/AbstractMetricsManager.h:318-333): the jsf32 restatements pinned against the reference's
own generator (tests/golden/jsf32_seed1.json from oracle/_ref/ref_jsf, 3rd/rng/jsf.h compiled
in place), and the oracle's sampled paths (no GPU)."""
import ctypes
import json
import os

import numpy as np
import pytest

from tests.oracle_ctypes import jget

GOLD = os.path.join(os.path.dirname(__file__), "golden")
VEC = json.load(open(os.path.join(GOLD, "jsf32_seed1.json")))


def jsf32(n):
    """Python restatement (3rd/rng/jsf.h:38-70: jsf<uint32_t, uint32_t, 27, 17, 0>, seed 1)"""
    M = 0xffffffff
    rot = lambda x, k: ((x << k) | (x >> (32 - k))) & M
    a, b, c, d = 0xf1ea5eed, 1, 1, 1
    out = []
    for i in range(20 + n):
        e = (a - rot(b, 27)) & M
        a = b ^ rot(c, 17)
        b = (c + d) & M
        c = (d + e) & M
        d = (e + a) & M
        if i >= 20:
            out.append(d)
    return out


def test_python_restatement_matches_reference():
    assert jsf32(256) == VEC["first"]


def test_oracle_restatement_matches_reference(oracle):
    n = VEC["n"]
    out = (ctypes.c_uint32 * n)()
    oracle.lib.pvo_jsf32(n, out)
    v = np.frombuffer(out, dtype=np.uint32)
    assert list(v[:256]) == VEC["first"]
    assert int(v[-1]) == VEC["last"]
    assert int((v % 100 < 50).sum()) == VEC["pct_lt_50"]


@pytest.mark.parametrize("rate", [1, 37, 100])
def test_oracle_sampled_counts(oracle, rate):
    pcap = open(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), "rb").read()
    full = oracle.run_bytes(pcap, num_periods=1, window=1)
    s = oracle.run_bytes(pcap, num_periods=1, window=1, deep_sample_rate=rate)
    # events and counters do not depend on sampling; deep samples are the draws below the rate
    for k in ("events", "udp", "ipv4", "in", "out", "total"):
        assert jget(s, "1m.packets." + k) == jget(full, "1m.packets." + k), k
    for k in ("events", "queries", "replies", "noerror", "nxdomain", "srvfail", "refused", "udp"):
        assert jget(s, "1m.dns.wire_packets." + k) == jget(full, "1m.dns.wire_packets." + k), k
    v = jsf32(int(jget(full, "1m.packets.events")))
    assert jget(s, "1m.packets.deep_samples") == (sum(1 for x in v if x % 100 < rate) if rate < 100
                                                   else jget(full, "1m.packets.events"))
    if rate == 100:
        assert s == full
