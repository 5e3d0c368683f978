"""DNS v1 filters: the oracle against the reference's filter known-answer tests
(src/handlers/dns/v1/tests/test_dns_layer.cpp:271-366,524-705), and the host-side
config parsing against the reference's ConfigException messages (:869-896)."""
import os

import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MIXED = os.path.join(GOLD, "dns_udp_mixed_rcode.pcap")

# (cite, oracle filter config, expected wire_packets counters, expected top names)
KAT = [
    ("test_dns_layer.cpp:485-522 only_qname_suffix", dict(only_qname_suffix="GooGle.com"),
     dict(udp=10, noerror=4, srvfail=0, refused=0, nxdomain=1, nodata=2, total=10, filtered=14), {}),
    ("test_dns_layer.cpp:446-483 only_qname (predicate)", dict(only_qname="play.GooGle.com,nonexistent.google.com"),
     dict(udp=6, noerror=2, srvfail=0, refused=0, nxdomain=1, nodata=2, total=6, filtered=0),
     dict(top_qname2=".google.com", top_qname3="play.google.com")),
    ("test_dns_layer.cpp:271-302 exclude_noerror", dict(exclude_noerror=1),
     dict(noerror=0, srvfail=0, refused=1, nxdomain=1, nodata=0, filtered=22), {}),
    ("test_dns_layer.cpp:304-334 only_rcode nx (predicate)", dict(only_rcode_mask=1 << 3),
     dict(noerror=0, srvfail=0, refused=0, nxdomain=1, nodata=0, filtered=0), {}),
    ("test_dns_layer.cpp:336-366 only_rcode nx + refused", dict(only_rcode_mask=(1 << 3) | (1 << 5)),
     dict(noerror=0, srvfail=0, refused=1, nxdomain=1, nodata=0, filtered=0), {}),
    ("test_dns_layer.cpp:524-556 only_rcode noerror + answer_count 0", dict(only_rcode_mask=1, answer_count=0),
     dict(udp=4, noerror=4, srvfail=0, refused=0, nxdomain=0, nodata=4, filtered=6), {}),
    ("test_dns_layer.cpp:639-673 only_queries", dict(only_queries=1),
     dict(udp=12, noerror=0, srvfail=0, refused=0, nxdomain=0, filtered=12),
     dict(top_qname2=".mwbsys.com", top_qname3="sirius.mwbsys.com")),
    ("test_dns_layer.cpp:603-637 public_suffix_list", dict(public_suffix_list=1),
     dict(udp=24, noerror=10, srvfail=0, refused=1, nxdomain=1, filtered=0),
     dict(top_qname2=".mwbsys.com", top_qname3="sirius.mwbsys.com")),
    ("test_dns_layer.cpp:675-705 only_responses", dict(only_responses=1),
     dict(udp=12, noerror=10, srvfail=0, refused=1, nxdomain=1, filtered=12), {}),
]


@pytest.mark.parametrize("cite,cfg,want,tops", KAT, ids=[k[0].split()[-1] + str(i) for i, k in enumerate(KAT)])
def test_oracle_filter_kats(oracle, cite, cfg, want, tops):
    d = oracle.run_file(MIXED, host_spec="192.168.0.0/24", num_periods=1, window=1, **cfg)["1m"]["dns"]
    for k, v in want.items():
        assert d["wire_packets"][k] == v, (cite, k)
    for k, v in tops.items():
        assert d[k][0]["name"] == v, (cite, k)
    if "only_qname_suffix" in cfg:  # :520-521
        assert "google.com" in d["top_qname2"][0]["name"] and d["top_qname3"] == []


def test_filter_config_parsing():
    """DnsStreamHandler::start filter parsing (dns/v1/DnsStreamHandler.cpp:60-150): names and
    numbers, case-insensitive, and the reference's error messages."""
    from pktvisor_amd import ConfigError, dns_filter_config
    f = dns_filter_config({"only_rcode": ["nxdomain", "5"]})
    assert f["only_rcode_mask"] == (1 << 3) | (1 << 5)
    assert dns_filter_config({"only_rcode": 3})["only_rcode_mask"] == 1 << 3
    f = dns_filter_config({"only_qtype": ["AAAA", "TxT", "15"]})
    assert f["only_qtype"] == [28, 16, 15]
    # exclude_noerror wins over only_rcode (:61-64 else-if)
    f = dns_filter_config({"exclude_noerror": True, "only_rcode": 3})
    assert f["exclude_noerror"] and f["only_rcode_mask"] == 0
    assert dns_filter_config({"answer_count": 0})["answer_count"] == 0
    cases = [
        ({"only_rcode": "1"}, "DnsStreamHandler: wrong value type for only_rcode filter. It should be an integer or an array"),
        ({"only_rcode": 133}, "DnsStreamHandler: only_rcode filter contained an invalid/unsupported rcode"),
        ({"only_qtype": ["AAAA", "TEXT"]}, "DnsStreamHandler: only_qtype filter contained an invalid/unsupported qtype: TEXT"),
        ({"only_qtype": ["AAAA", "270"]}, "DnsStreamHandler: only_qtype filter contained an invalid/unsupported qtype: 270"),
        ({"answer_count": "1"}, "DnsStreamHandler: wrong value type for answer_count filter. It should be an integer"),
    ]
    for cfg, msg in cases:
        with pytest.raises(ConfigError) as e:
            dns_filter_config(cfg)
        assert str(e.value) == msg
    assert dns_filter_config({"only_qname": ["play.GooGle.com"]})["only_qname"] == ["play.google.com"]
    assert dns_filter_config({"only_qname_suffix": ["GooGle.com"]})["only_qname_suffix"] == ["google.com"]
    assert dns_filter_config({"public_suffix_list": True})["public_suffix_list"] == 1
    with pytest.raises(ConfigError) as e:
        dns_filter_config({"public_suffix_list": 1})  # config_get<bool> of an int
    assert str(e.value) == "wrong type for key: public_suffix_list"


def test_oracle_dnssec_kat(oracle):
    """test_dns_layer.cpp:558-596 only_dnssec_response on dnssec.pcap"""
    d = oracle.run_file(os.path.join(GOLD, "dnssec.pcap"), host_spec="192.168.0.0/24", num_periods=1, window=1,
                        only_dnssec_response=1)["1m"]["dns"]
    w = d["wire_packets"]
    assert (w["events"], w["deep_samples"], w["tcp"], w["udp"], w["ipv4"], w["ipv6"]) == (14, 14, 0, 6, 6, 0)
    assert (w["queries"], w["replies"], w["noerror"]) == (0, 6, 6)
    assert d["cardinality"]["qname"] == 3
    assert [(e["name"], e["estimate"]) for e in d["top_qtype"][:3]] == [("DNSKEY", 3), ("DS", 2), ("A", 1)]
