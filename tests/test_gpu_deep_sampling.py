"""deep_sample_rate < 100 on the GPU path against the oracle's restatement (jsf32 draws per
manager in stream order; not-deep events count in the counters only; a not-deep response
pairs but feeds no quantile, ratio or slow top): reference fixtures and a synthetic C4 capture
over many ingest batches. Combinations that are not built fail loudly."""
import os

import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.test_gpu_parity import GOLD, diff

pytestmark = pytest.mark.gpu


def both(oracle, pcap, tmp_path, host, periods, rate, **kw):
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host or None, periods=periods, deep_sample_rate=rate, **kw)
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods, deep_sample_rate=rate)
    return gpu, ref


@pytest.mark.parametrize("fixture,host", [("dns_ipv4_udp.pcap", ""), ("dns_ipv6_udp.pcap", ""),
                                          ("dns_udp_mixed_rcode.pcap", "")])
@pytest.mark.parametrize("rate", [1, 50, 99])
@pytest.mark.parametrize("periods", [1, 5])
def test_fixture_sampled_parity(oracle, tmp_path, fixture, host, rate, periods):
    gpu, ref = both(oracle, open(os.path.join(GOLD, fixture), "rb").read(), tmp_path, host, periods, rate)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("rate", [33, 80])
def test_synthetic_sampled_parity_many_batches(oracle, tmp_path, monkeypatch, rate):
    monkeypatch.setenv("PV_INGEST_CHUNK_MB", "1")
    pcap = synth.pcap_bytes(4, 60000, ts_step_us=1500)
    gpu, ref = both(oracle, pcap, tmp_path, synth.HOST_SPEC, 5, rate)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_sampling_refusals(tmp_path):
    with pytest.raises(pa.PvError, match="DNS filters"):
        pa.PvHandlers(deep_sample_rate=50, dns_filters={"only_queries": True})
    p = os.path.join(GOLD, "dns_ipv4_tcp.pcap")
    with pytest.raises(pa.PvError, match="DNS over TCP"):
        pa.pktvisor_reader(p, periods=1, deep_sample_rate=50)
