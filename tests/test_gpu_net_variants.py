"""The Net pass's A/B variants (PV_NET_KERNEL), each in a process of its own
(tests/net_variant_worker.py), against the oracle: the span-load pass with deferred general-path
records, the shift-free and the general pass must stay parity-green while they are kept."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("variant,kernel", [("span", "pv_net_kernel_span"), ("ns", "pv_net_kernel_ns"),
                                            ("general", "pv_net_kernel")])
def test_net_variant_parity(variant, kernel):
    env = dict(os.environ, PV_NET_KERNEL=variant)
    r = subprocess.run([sys.executable, "-m", "tests.net_variant_worker"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert kernel in out, out[-3000:]
