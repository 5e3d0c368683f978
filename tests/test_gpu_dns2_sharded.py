"""Sharded DNS v2: contiguous shards of one capture on W ranks, merged with
pktvisor_amd.dist.merge_window, equal the oracle's single pass bit-exactly. A v2 transaction whose
query and response fall in different shards pairs rank by rank (pv_edge_carry: the response this
shard counted as an orphan is accounted as the single stream's TransactionManager per direction
would, src/handlers/dns/v2/DnsStreamHandler.cpp:1100-1145, libs/visor_transaction/
TransactionManager.h:51-106), open queries time out at the purging shard's shifts, and top_slow
per direction is judged against the whole stream's p90 of each closed bucket (pv_slow_finish)."""
import json

import pytest

from pktvisor_amd import synth
from tests.dist_launch import run_ranks
from tests.test_gpu_dns2 import ALL, ALL_NAMES
from tests.test_gpu_parity import diff

pytestmark = pytest.mark.gpu


def run(oracle, tmp_path, pcap, world, timeout=240):
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    out = tmp_path / "out.json"
    run_ranks(world, ["gpu", str(p), str(out), synth.HOST_SPEC, "5", "100", "null", json.dumps({"enable": ALL_NAMES})],
              timeout=timeout)
    gpu = json.load(open(out))
    ref = oracle.run_bytes(pcap, host_spec=synth.HOST_SPEC, num_periods=5, window=5, dns2_groups=ALL)
    return gpu, ref


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_dns2_c4_300s(oracle, tmp_path, world):
    """C4 traffic over 300 s (transactions crossing every shard edge, several DNS shifts)"""
    gpu, ref = run(oracle, tmp_path, synth.pcap_bytes(4, 120000, ts_step_us=2500), world)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_sharded_dns2_world8_c4_tcp(oracle, tmp_path):
    """8 ranks sharing the GPU over C4 traffic with DNS-over-TCP connections"""
    gpu, ref = run(oracle, tmp_path, synth.c4_tcp_pcap(), 8, timeout=400)
    assert diff(gpu, ref) is None, diff(gpu, ref)
