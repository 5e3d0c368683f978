"""Oracle sanity on the synthetic configs (CPU)."""
import pytest

from pktvisor_amd import synth


def test_c2_shape(oracle):
    out = oracle.run_bytes(synth.pcap_bytes(2, 20000), host_spec=synth.HOST_SPEC, num_periods=1, window=1)["1m"]
    p = out["packets"]
    assert p["events"] == p["udp"] == p["ipv4"] == 20000
    assert p["in"] + p["out"] + p["unknown_dir"] == 20000
    assert p["payload_size"] == {"p50": 64, "p90": 64, "p95": 64, "p99": 64}
    assert out["dns"]["wire_packets"]["events"] == 0
    assert p["cardinality"]["src_ips_in"] > 1000


def test_c3_shape(oracle):
    out = oracle.run_bytes(synth.pcap_bytes(3, 20000), host_spec=synth.HOST_SPEC, num_periods=1, window=1)["1m"]
    d = out["dns"]["wire_packets"]
    assert d["events"] == d["queries"] == 20000 and d["replies"] == 0
    assert out["dns"]["top_qtype"][0] == {"name": "A", "estimate": 20000}
    sizes = out["packets"]["payload_size"]
    assert 122 <= sizes["p50"] <= 134


@pytest.mark.parametrize("cfg", [1, 4])
def test_paired_configs(oracle, cfg):
    out = oracle.run_bytes(synth.pcap_bytes(cfg, 5000), host_spec=synth.HOST_SPEC, num_periods=1, window=1)["1m"]
    d = out["dns"]
    assert d["wire_packets"]["replies"] > 0
    assert d["xact"]["counts"]["total"] > 0.9 * d["wire_packets"]["replies"]
    assert d["xact"]["out"]["total"] == d["xact"]["counts"]["total"]


def test_edge_mix_runs(oracle):
    out = oracle.run_bytes(synth.pcap_bytes(9, 20000), host_spec="10.0.0.0/8,2000::/3", num_periods=1, window=1)
    assert out["1m"]["packets"]["events"] == 20000


@pytest.mark.parametrize("limit,tcp", [(2, 0), (3, 1), (None, 1)])
def test_tcp_reput_crafted(oracle, limit, tcp):
    """The oracle against the reference's LRU order derived by hand (synth.tcp_reput_pcap): with
    the list capped at 2, closing the evicted A flushes its held fragment, that delivery's put
    evicts B, and B's last segment then belongs to a closed flow (PcapInputStream.cpp:254-263,
    449-465; TcpReassembly::closeConnection). Without the cap, or at 3, B's query counts."""
    out = oracle.run_bytes(synth.tcp_reput_pcap(), num_periods=1, window=1, tcp_packet_reassembly_cache_limit=limit)
    d = out["1m"]["dns"]["wire_packets"]
    assert (d["tcp"], d["queries"]) == (tcp, tcp)
