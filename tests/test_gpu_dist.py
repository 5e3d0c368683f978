"""Multi-rank parity on the GPU box: W ranks (gloo; they share the box's GPU) each
process a contiguous shard of a capture, merge with pktvisor_amd.dist.merge_window
(bucket SUM/MIN, top-N, quantile inputs, DNS transactions across shard edges), and
rank 0's window must equal the oracle's single pass over the whole capture."""
import json
import os

import pytest

from pktvisor_amd import synth
from tests.dist_launch import run_ranks
from tests.test_gpu_parity import GOLD, diff

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", ["c4", "c1", "fixture"])
def test_sharded_merge_matches_single_pass(oracle, tmp_path, world, case):
    if case == "fixture":
        pcap, host = open(os.path.join(GOLD, "dns_ipv4_udp.pcap"), "rb").read(), ""
    else:
        pcap, host = (synth.pcap_bytes(4, 60000) if case == "c4" else synth.pcap_bytes(1, 1000)), synth.HOST_SPEC
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    out = tmp_path / "out.json"
    run_ranks(world, ["gpu", str(p), str(out), host, "1"])
    gpu = json.load(open(out))
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=1, window=1)
    assert diff(gpu, ref) is None, diff(gpu, ref)
