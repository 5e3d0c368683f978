"""The oracle (CPU restatement) against the reference's own known-answer tests."""
import json
import os

import pytest

from tests.oracle_ctypes import jget

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KAT = json.load(open(os.path.join(GOLD, "kat_reference.json")))["cases"]


@pytest.mark.parametrize("case", KAT, ids=[c["fixture"] + str(i) for i, c in enumerate(KAT)])
def test_oracle_matches_reference_kats(oracle, case):
    out = oracle.run_file(os.path.join(GOLD, case["fixture"]), host_spec=case["host_spec"],
                          num_periods=case["periods"], window=case["periods"], **case.get("cfg", {}))
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


def test_readme_sample_shape(oracle):
    # README.md:407-431 sample (dns_ipv4_udp, default 5m merged window). The README's
    # qname cardinality (70) was produced by an older sketch library; the vendored
    # datasketches gives 69 for these 70 names (pinned in test_ref_sketch.py).
    out = oracle.run_file(os.path.join(GOLD, "dns_ipv4_udp.pcap"), num_periods=5, window=5)
    d = out["5m"]["dns"]
    assert d["period"] == {"start_ts": 1567706414, "length": 6}
    assert d["top_qname2"] == [{"name": ".test.com", "estimate": 140}]
    assert d["top_nxdomain"] == []
    assert d["cardinality"]["qname"] in (69, 70)
