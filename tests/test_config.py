"""The handler config surface: the reference's group and config validation with its exact
texts (StreamMetricsHandler, src/StreamHandler.h:94-152; KATs
src/handlers/dns/v1/tests/test_dns_layer.cpp:856-1017, net/v1/tests/test_net_layer.cpp),
and the oracle's window JSON against the reference's window schemas (the reference's
test_json_schema.cpp configs). No GPU."""
import json
import os

import pytest

from pktvisor_amd import config as pvcfg
from tests.schema_check import errors

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DNS_GROUPS_MSG = ("dns_top_wired is an invalid/unsupported metric group. The valid groups are: all, cardinality, counters, "
                  "dns_transaction, histograms, quantiles, top_ecs, top_ports, top_qnames, top_qnames_details")
DNS_CONFIG_MSG = ("invalid_config is an invalid/unsupported config or filter. The valid configs/filters are: exclude_noerror, "
                  "only_rcode, only_queries, only_responses, only_dnssec_response, answer_count, only_qtype, only_qname, "
                  "only_qname_suffix, geoloc_notfound, asn_notfound, dnstap_msg_type, public_suffix_list, recorded_stream, "
                  "xact_ttl_secs, xact_ttl_ms, deep_sample_rate, num_periods, topn_count, topn_percentile_threshold")


@pytest.mark.parametrize("key", ["disable", "enable"])
def test_dns_invalid_group_text(key):
    # test_dns_layer.cpp:980-990
    with pytest.raises(pvcfg.StreamHandlerException) as e:
        pvcfg.dns_start({key: ["top_qnames", "dns_top_wired"]})
    assert str(e.value) == DNS_GROUPS_MSG


def test_dns_invalid_config_text():
    # test_dns_layer.cpp:993-1004
    with pytest.raises(pvcfg.StreamHandlerException) as e:
        pvcfg.dns_start({"invalid_config": True})
    assert str(e.value) == DNS_CONFIG_MSG


def test_dns_config_ttl():
    # test_dns_layer.cpp:1006-1017: xact_ttl_secs accepted (2 s)
    assert pvcfg.dns_start({"xact_ttl_secs": 2})["xact_ttl_ms"] == 2000
    assert pvcfg.dns_start({"xact_ttl_ms": 1500, "xact_ttl_secs": 2})["xact_ttl_ms"] == 1500


def test_net_invalid_group_and_config_text():
    with pytest.raises(pvcfg.StreamHandlerException) as e:
        pvcfg.net_start({"enable": ["top_ips", "net_top_wired"]})
    assert str(e.value) == ("net_top_wired is an invalid/unsupported metric group. The valid groups are: all, cardinality, "
                            "counters, top_geo, top_ips")
    with pytest.raises(pvcfg.StreamHandlerException) as e:
        pvcfg.net_start({"invalid_config": True})
    assert str(e.value) == ("invalid_config is an invalid/unsupported config or filter. The valid configs/filters are: "
                            "geoloc_notfound, asn_notfound, only_geoloc_prefix, only_asn_number, recorded_stream, "
                            "deep_sample_rate, num_periods, topn_count, topn_percentile_threshold")
    with pytest.raises(pvcfg.ConfigException) as e:
        pvcfg.net_start({"only_asn_number": ["16509", "AS1"]})
    assert str(e.value) == "NetStreamHandler: only_asn_number filter contained an invalid/unsupported value: AS1"


def test_group_processing_order():
    G = pvcfg.DNS_GROUP_DEFS
    base = pvcfg.dns_start({})["groups"] & ~pvcfg.GROUPS_SET
    assert base == sum(G[g] for g in pvcfg.DNS_DEFAULT_GROUPS)
    g = pvcfg.dns_start({"disable": ["cardinality", "counters"], "enable": ["histograms"]})["groups"]
    assert g & ~pvcfg.GROUPS_SET == (base & ~(G["cardinality"] | G["counters"])) | G["histograms"]
    # "all" stops its list: disable all then enable one
    g = pvcfg.dns_start({"disable": ["all", "not_checked"], "enable": ["top_ecs"]})["groups"]
    assert g == pvcfg.GROUPS_SET | G["top_ecs"]
    assert pvcfg.dns_start({"enable": ["all"]})["groups"] & ~pvcfg.GROUPS_SET == sum(G.values())
    assert pvcfg.dns_start({"disable": ["all"]})["groups"] == pvcfg.GROUPS_SET


def test_config_value_types():
    # Configurable::config_get<T> (src/Configurable.h:101-112)
    for bad in ({"only_qname_suffix": "com"}, {"only_qname": "a.com"}, {"only_qtype": "A"}, {"only_queries": 1},
                {"enable": "top_ecs"}):
        with pytest.raises(pvcfg.ConfigException, match="wrong type for key"):
            pvcfg.dns_start(bad)
    with pytest.raises(pvcfg.ConfigException) as e:
        pvcfg.dns_start({"only_rcode": "1"})
    assert str(e.value) == "DnsStreamHandler: wrong value type for only_rcode filter. It should be an integer or an array"
    with pytest.raises(pvcfg.ConfigException) as e:
        pvcfg.dns_start({"answer_count": "1"})
    assert str(e.value) == "DnsStreamHandler: wrong value type for answer_count filter. It should be an integer"
    with pytest.raises(pvcfg.ConfigException) as e:
        pvcfg.dns_start({"dnstap_msg_type": "bogus"})
    assert str(e.value).startswith("DnsStreamHandler: dnstap_msg_type contained an invalid/unsupported type. Valid types: auth")


def test_geo_filters_without_database_filter_everything():
    assert pvcfg.dns_start({"geoloc_notfound": True})["filters"]["filter_all"] == 1
    assert pvcfg.dns_start({"asn_notfound": False})["filters"]["filter_all"] == 0
    assert pvcfg.net_start({"asn_notfound": True})["filter_all"]
    assert pvcfg.net_start({"only_geoloc_prefix": ["NA/US"]})["filter_all"]


def _schema(name):
    return json.load(open(os.path.join(GOLD, f"{name}_v1_window-schema.json")))


def test_oracle_window_json_matches_reference_schemas(oracle):
    """the reference's schema tests: dns_udp_tcp_random.pcap, 5 periods merged, dns with
    top_ecs + top_ports + top_qnames_details enabled (dns/v1/tests/test_json_schema.cpp:24-39)"""
    G = pvcfg.DNS_GROUP_DEFS
    dns_groups = sum(G[g] for g in pvcfg.DNS_DEFAULT_GROUPS) | G["top_ecs"] | G["top_qnames_details"]
    out = oracle.run_file(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), host_spec="192.168.0.0/24", num_periods=5,
                          window=5, dns_groups=dns_groups)["5m"]
    assert errors(_schema("dns"), {"dns": out["dns"]}) == []
    assert errors(_schema("net"), {"packets": out["packets"]}) == []


def test_schema_checker_catches_missing_keys(oracle):
    out = oracle.run_file(os.path.join(GOLD, "dns_udp_tcp_random.pcap"), host_spec="192.168.0.0/24", num_periods=5,
                          window=5)["5m"]
    # default groups: no top_ecs / details keys, which the reference's schema requires
    errs = errors(_schema("dns"), {"dns": out["dns"]})
    assert any("top_query_ecs" in e for e in errs) and any("top_noerror" in e for e in errs)


def test_dns2_filter_config():
    """DnsStreamHandler v2 start (dns/v2/DnsStreamHandler.cpp:61-170): typed filters with v2's
    key set, only_xact_directions to disabled bits, the reference's error texts"""
    from pktvisor_amd.config import ConfigException, dns2_start
    d = dns2_start({"exclude_noerror": True, "only_xact_directions": ["in", "unknown"]})
    assert d["filters"]["v2"] == 1 and d["filters"]["exclude_noerror"] == 1 and d["filters"]["xact_dirs_disabled"] == 2
    d = dns2_start({"only_rcode": ["nxdomain", "5"], "only_qname": ["A.b"]})
    assert d["filters"]["only_rcode_mask"] == (1 << 3) | (1 << 5) and d["filters"]["only_qname"] == ["a.b"]
    assert dns2_start({})["filters"] is None
    with pytest.raises(ConfigException, match="only_xact_directions filter contained an invalid/unsupported direction: up"):
        dns2_start({"only_xact_directions": ["up"]})
    with pytest.raises(ConfigException, match="geoloc_notfound is not supported"):
        dns2_start({"geoloc_notfound": True})
