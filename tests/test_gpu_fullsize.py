"""The exact workloads bench.py times, checked bit-exact against the oracle's single pass:
C2 (10M x 64 B UDP) and C3 (10M DNS queries), 5 periods, default groups (the
10M bench configs were only checked for their event counts)."""
import pytest

from pktvisor_amd import synth
from tests.test_gpu_parity import diff, run_both

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", [2, 3])
def test_bench_workload_full_size(oracle, tmp_path, cfg):
    pcap = synth.pcap_bytes(cfg, 10_000_000)
    gpu, ref = run_both(oracle, pcap, synth.HOST_SPEC, 5, tmp_path)
    del pcap
    assert diff(gpu, ref) is None, diff(gpu, ref)
