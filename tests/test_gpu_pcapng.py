"""pcapng input end to end: the reference's pcap fixtures written as pcapng (tests/pcapng_util.py)
through pktvisor_reader give the same windows as the pcap files (ns-resolution records)."""
import os

import pytest

import pktvisor_amd as pa
from tests.pcapng_util import to_pcapng
from tests.test_gpu_parity import diff

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("fixture,host", [("dns_ipv4_udp.pcap", ""), ("dns_udp_tcp_random.pcap", "192.168.0.0/24"),
                                          ("ecs.pcap", "")])
@pytest.mark.parametrize("periods", [1, 5])
@pytest.mark.parametrize("kw", [{}, {"tsresol": 9, "sections": 2}])
def test_pcapng_same_windows(tmp_path, fixture, host, periods, kw):
    src = os.path.join(GOLD, fixture)
    ng = tmp_path / (fixture + "ng")
    ng.write_bytes(to_pcapng(open(src, "rb").read(), **kw))
    a = pa.pktvisor_reader(src, host_spec=host or None, periods=periods)
    b = pa.pktvisor_reader(str(ng), host_spec=host or None, periods=periods)
    assert diff(b, a) is None, diff(b, a)
