"""Pins the oracle's sketch restatements (CPC HIP/ICON, exact-mode KLL rank rule)
against the reference's own datasketches library: committed vectors everywhere,
plus live comparisons when oracle/_ref/ref_sketch is built."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "ref_sketch")
VEC = json.load(open(os.path.join(ROOT, "tests", "golden", "cpc_vectors.json")))["cases"]


@pytest.mark.parametrize("case", VEC, ids=[str(c["n"]) for c in VEC])
def test_cpc_matches_reference_vectors(oracle, case):
    v = np.random.default_rng(case["seed"]).integers(0, 2**32, size=case["n"], dtype=np.uint64).astype(np.uint32)
    assert oracle.lib.pvo_cpc_u32(v.ctypes.data, len(v), 0) == case["hip"]
    assert oracle.lib.pvo_cpc_u32(v.ctypes.data, len(v), 1) == case["icon"]


def _ref(cmd):
    return subprocess.run([REF], input=cmd.encode(), capture_output=True, check=True).stdout.decode()


@pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref not built")
def test_kll_exact_mode_rank_rule():
    # For n <= 200 KLL keeps every item: the quantile rule is deterministic.
    from tests.oracle_ctypes import ROOT as _  # noqa: F401
    rng = np.random.default_rng(7)
    for n in [1, 2, 3, 10, 99, 100, 101, 140, 200]:
        v = rng.integers(0, 5000, size=n).tolist()
        got = [int(x) for x in _ref(f"kll_u64 {n} " + " ".join(map(str, v)) + "\n").split()]
        s = sorted(v)
        want = []
        for r in (0.5, 0.9, 0.95, 0.99):
            w = int(np.ceil(r * n))
            want.append(s[max(w, 1) - 1])
        assert got == want, n


@pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref not built")
def test_fi_exact_below_purge_threshold():
    # Below 0.75 * 2^13 distinct items the FI sketch never purges: estimates are exact counts.
    rng = np.random.default_rng(3)
    items = [f"k{x}" for x in rng.zipf(1.3, size=20000) if x < 5000]
    out = _ref(f"fi_str {len(items)} " + " ".join(items) + "\n").split()
    assert out[0] == "maxerr" and out[1] == "0"
    got = {kv.rsplit(":", 1)[0]: int(kv.rsplit(":", 1)[1]) for kv in out[2:]}
    from collections import Counter
    assert got == dict(Counter(items))
