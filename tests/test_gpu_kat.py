"""The HIP path against the reference's own known-answer tests (tests/golden/kat_reference.json),
each case run through the C-ABI with the handler config the reference test sets."""
import json
import os

import pytest

import pktvisor_amd as pa
from tests.oracle_ctypes import jget

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat_reference.json")))["cases"]


@pytest.mark.parametrize("case", KAT, ids=[c["fixture"] + str(i) for i, c in enumerate(KAT)])
def test_gpu_matches_reference_kats(case):
    out = pa.pktvisor_reader(os.path.join(GOLD, case["fixture"]), host_spec=case["host_spec"] or None,
                             periods=case["periods"], net_config={}, dns_config=case.get("dns_config", {}),
                             net2_config=case.get("net2_config"), dns2_config=case.get("dns2_config"),
                             **case.get("input_config", {}))
    for path, want in case["checks"]:
        assert jget(out, path) == want, (case["cite"], path)
    for path, lo in case.get("ge", []):
        assert jget(out, path) >= lo, (case["cite"], path)
    for path, n in case.get("len", []):
        assert len(jget(out, path)) == n, (case["cite"], path)
    for paths, want in case.get("sums", []):
        assert sum(jget(out, q) for q in paths) == want, (case["cite"], paths)
    for path in case.get("absent", []):
        with pytest.raises((KeyError, IndexError, TypeError)):
            jget(out, path)
