"""dnstap input (pv_process_dnstap) against the reference's own dnstap KATs on its fixture
(tests/golden/fixture.dnstap = src/inputs/dnstap/tests/fixtures/fixture.dnstap):
src/handlers/dns/v1/tests/test_dnstap.cpp:12-151 and
src/handlers/net/v1/tests/test_net_layer.cpp:324-361."""
import os

import pytest

import pktvisor_amd as pa
from tests.oracle_ctypes import jget

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "golden", "fixture.dnstap")


def run(dns_config=None):
    return pa.dnstap_reader(FIX, periods=1, net_config={}, dns_config=dns_config or {})


def test_dns_dnstap_kat():
    """test_dnstap.cpp:12-63 "Parse DNSTAP" """
    out = run()
    want = {"events": 153, "deep_samples": 153, "tcp": 0, "udp": 153, "ipv4": 153, "ipv6": 0, "queries": 79,
            "replies": 74, "noerror": 70, "nxdomain": 0, "refused": 0, "srvfail": 4, "filtered": 0}
    for k, v in want.items():
        assert jget(out, "1m.dns.wire_packets." + k) == v, k
    for k in ("total", "in.total", "out.total"):
        assert jget(out, "1m.dns.xact." + ("counts." + k if k == "total" else k)) == 0, k
    assert jget(out, "1m.dns.xact.counts.timed_out") == 0
    assert jget(out, "1m.dns.cardinality.qname") == 70
    assert jget(out, "1m.dns.top_qname2.0.name") == ".google.com"
    assert jget(out, "1m.dns.top_qname2.0.estimate") == 18
    assert jget(out, "1m.dns.top_udp_ports.0.name") == "33000"
    assert jget(out, "1m.dns.top_udp_ports.0.estimate") == 4
    assert jget(out, "1m.dns.top_qtype.0.name") == "A"
    assert jget(out, "1m.dns.top_qtype.0.estimate") == 149
    assert jget(out, "1m.dns.top_qtype.1.name") == "HTTPS"
    assert jget(out, "1m.dns.top_qtype.1.estimate") == 4


def test_dns_dnstap_filtered_empty():
    """test_dnstap.cpp:65-101: dnstap_msg_type "auth" filters every (client) message"""
    out = run({"dnstap_msg_type": "auth"})
    assert jget(out, "1m.dns.wire_packets.events") == 153
    assert jget(out, "1m.dns.wire_packets.deep_samples") == 153
    for k in ("tcp", "udp", "ipv4", "ipv6", "queries", "replies", "noerror", "nxdomain", "refused", "srvfail"):
        assert jget(out, "1m.dns.wire_packets." + k) == 0, k
    assert jget(out, "1m.dns.wire_packets.filtered") == 153


def test_dns_dnstap_filtered_with_data():
    """test_dnstap.cpp:103-151: dnstap_msg_type "client" keeps them"""
    out = run({"dnstap_msg_type": "client"})
    want = {"events": 153, "deep_samples": 153, "tcp": 0, "udp": 153, "ipv4": 153, "ipv6": 0, "queries": 79,
            "replies": 74, "noerror": 70, "srvfail": 4, "filtered": 0}
    for k, v in want.items():
        assert jget(out, "1m.dns.wire_packets." + k) == v, k


def test_net_dnstap_kat():
    """test_net_layer.cpp:324-361 "Parse net dnstap stream" """
    out = run()
    want = {"events": 153, "deep_samples": 153, "tcp": 0, "udp": 153, "ipv4": 153, "ipv6": 0, "in": 79,
            "out": 74, "protocol.tcp.syn": 0}
    for k, v in want.items():
        assert jget(out, "1m.packets." + k) == v, k
    assert jget(out, "1m.packets.cardinality.dst_ips_out") == 1
    assert jget(out, "1m.packets.cardinality.src_ips_in") == 1
    assert jget(out, "1m.packets.top_ipv4.0.name") == "192.168.0.54"
    assert jget(out, "1m.packets.top_ipv4.0.estimate") == 153
    assert jget(out, "1m.packets.payload_size.p50") == 100


def test_dnstap_invalid_msg_type():
    with pytest.raises(Exception, match="dnstap_msg_type contained an invalid/unsupported type. Valid types: auth, "
                                        "client, forwarder, resolver, stub, tool, update"):
        run({"dnstap_msg_type": "bogus"})


@pytest.mark.parametrize("rate", [1, 30, 70, 99])
@pytest.mark.parametrize("msg_type", [None, "auth"])
def test_dnstap_deep_sampling(rate, msg_type):
    """deep_sample_rate < 100 over dnstap: each manager draws per event in stream order
    (new_event, net/v1 ...cpp:840, dns/v1 ...cpp:1409); a dnstap_msg_type-filtered event draws
    nothing in the DNS manager (process_filtered) and counts its last flag. A not-deep event
    takes the Net handler's process_net_layer(dir, l3, l4, size) and the DNS handler's
    process_dns_layer(l3, l4, side) (net/v1 ...cpp:599-602, dns/v1 ...cpp:882-885). The oracle has
    no dnstap path: the expected numbers come from the reference generator's draws
    (tests/golden/jsf32_seed1.json, oracle/_ref/ref_jsf) and the unsampled KATs above."""
    import json
    first = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "jsf32_seed1.json")))["first"]
    deep = sum(1 for x in first[:153] if x % 100 < rate)
    out = pa.dnstap_reader(FIX, periods=1, net_config={}, dns_config={"dnstap_msg_type": msg_type} if msg_type else {},
                           deep_sample_rate=rate)
    # Net: every event draws; counters and payload sizes for all, addresses for the deep ones
    for k, v in {"events": 153, "deep_samples": deep, "udp": 153, "ipv4": 153, "in": 79, "out": 74}.items():
        assert jget(out, "1m.packets." + k) == v, k
    assert jget(out, "1m.packets.top_ipv4.0.estimate") == deep
    assert jget(out, "1m.packets.payload_size.p50") == 100
    dns = jget(out, "1m.dns.wire_packets")
    if msg_type == "auth":
        # every event filtered: no DNS draw, the manager's initial flag (deep) on each
        assert (dns["events"], dns["deep_samples"], dns["filtered"], dns["queries"]) == (153, 153, 153, 0)
    else:
        # counters by side for every event; the message's rcode and names for the deep ones
        for k, v in {"events": 153, "deep_samples": deep, "udp": 153, "ipv4": 153, "queries": 79, "replies": 74}.items():
            assert dns[k] == v, k
        assert dns["noerror"] + dns["srvfail"] <= 74
        q = sum(e["estimate"] for e in jget(out, "1m.dns.top_qtype"))
        assert q <= deep and (deep == 0 or q > 0)


# ---- the dnstap input proxy's only_hosts (src/inputs/dnstap/DnstapInputStream.h:96-146)
@pytest.mark.parametrize("hosts", [["192.168.0.0/24"], ["192.168.0.12/32"], ["192.168.0.0/24", "2001:db8::/48"]])
def test_dnstap_only_hosts(hosts):
    """the proxy's match_subnet(..., std::string) reads the raw address bytes as text, so no
    fixture message (all carry both addresses, 4-byte binary) matches and none reaches the
    handlers: test_dnstap.cpp:150-169 "filter by invalid subnet" (0 callbacks); the "valid
    subnet" case (:128-148) is [!mayfail] in the reference and fails there the same way"""
    frames = open(FIX, "rb").read()
    h = pa.PvHandlers(num_periods=1, net_config={}, dns_config={})
    try:
        h._check(h.lib.pv_set_dnstap_only_hosts(h.ctx, ",".join(hosts).encode()), "pv_set_dnstap_only_hosts")
        h.process_dnstap(frames)
        with pytest.raises(pa.PvError, match="no data"):
            h.window_json(0)
        # cleared: every message again
        h._check(h.lib.pv_set_dnstap_only_hosts(h.ctx, None), "pv_set_dnstap_only_hosts")
        h.process_dnstap(frames)
        assert jget({"w": h.window_json(0)}, "w.dns.wire_packets.events") == 153
    finally:
        h.close()


@pytest.mark.parametrize("spec,err", [("192.168.0.0/24/12ac", "invalid CIDR: 192.168.0.0/24/12ac"),
                                      ("192.168.0.0/64", "invalid CIDR: 192.168.0.0/64"),
                                      ("192.168.AE.0/24", "invalid IPv4 address: 192.168.AE.0"),
                                      ("2001:db8::/48/12ac", "invalid CIDR: 2001:db8::/48/12ac"),
                                      ("2001:db8::/256", "invalid CIDR: 2001:db8::/256"),
                                      ("fe80:2030:31:24/12", "invalid IPv6 address: fe80:2030:31:24")])
def test_dnstap_only_hosts_invalid(spec, err):
    """test_dnstap.cpp:171-211 "dnstap invalid filters": parse_host_specs' texts"""
    h = pa.PvHandlers(num_periods=1)
    try:
        with pytest.raises(pa.PvError, match=err.replace(".", r"\.")):
            h._check(h.lib.pv_set_dnstap_only_hosts(h.ctx, spec.encode()), "pv_set_dnstap_only_hosts")
    finally:
        h.close()


# ---- the v2 handlers over dnstap (net/v2 ...cpp:533-604, dns/v2 ...cpp:1176-1270)
def test_dns2_dnstap_kat():
    """src/handlers/dns/v2/tests/test_dnstap.cpp:12-64 "Parse DNSTAP" (enable top_size, top_ports):
    transactions DnsXactID(transactionID, 2) per direction of the message type"""
    out = pa.dnstap_reader(FIX, periods=1, dns2_config={"enable": ["top_size", "top_ports"]})
    d = out["1m"]["dns"]
    assert (d["observed_packets"], d["deep_sampled_packets"]) == (153, 153)
    want = {"tcp_xacts": 0, "udp_xacts": 72, "dot_xacts": 0, "doh_xacts": 0, "dnscrypt_udp_xacts": 0,
            "dnscrypt_tcp_xacts": 0, "doq_xacts": 0, "ipv4_xacts": 72, "ipv6_xacts": 0, "xacts": 72,
            "timeout_queries": 0, "orphan_responses": 2, "noerror_xacts": 68, "nxdomain_xacts": 0,
            "refused_xacts": 0, "srvfail_xacts": 4}
    for k, v in want.items():
        assert d["in"][k] == v, k
    assert d["in"]["cardinality"]["qname"] == 65
    assert d["in"]["top_qname2_xacts"][0] == {"name": ".google.com", "estimate": 9}
    assert d["in"]["top_udp_ports_xacts"][0]["estimate"] == 2
    assert d["in"]["top_qtype_xacts"][:2] == [{"name": "A", "estimate": 70}, {"name": "HTTPS", "estimate": 2}]


def test_net2_dnstap_kat():
    """src/handlers/net/v2/tests/test_net_layer.cpp:321-358 "Parse net dnstap stream" """
    out = pa.dnstap_reader(FIX, periods=1, net2_config={})
    n = out["1m"]["net"]
    assert (n["observed_packets"], n["deep_sampled_packets"]) == (153, 153)
    for k, v in {"tcp_packets": 0, "udp_packets": 79, "ipv4_packets": 79, "ipv6_packets": 0, "total_packets": 79}.items():
        assert n["in"][k] == v, k
    assert n["in"]["tcp"]["syn_packets"] == 0
    assert n["in"]["cardinality"]["ips"] == 2
    assert n["in"]["top_ipv4_packets"][0] == {"name": "192.168.0.54", "estimate": 79}
    assert n["in"]["payload_size_bytes"]["p50"] == 89


@pytest.mark.parametrize("periods", [1, 3])
def test_dns2_dnstap_windows_and_filter(periods):
    """dnstap_msg_type with DNS v2 (process_filtered(stamp): an event, `filtered_packets`, no
    transaction) and the window shifts between dnstap spans (the open transactions' purge)"""
    out = pa.dnstap_reader(FIX, periods=periods, dns2_config={"dnstap_msg_type": "auth"})
    d = out[f"{periods}m"]["dns"]
    assert (d["observed_packets"], d["filtered_packets"]) == (153, 153)
    assert "in" not in d and "out" not in d
    out = pa.dnstap_reader(FIX, periods=periods, dns2_config={})
    d = out[f"{periods}m"]["dns"]
    assert d["observed_packets"] == 153 and d["in"]["xacts"] == 72


def test_dnstap_only_hosts_failed_call_keeps_state():
    """a spec list that fails to parse leaves the previous only_hosts state as it was
    (the reference's parse_host_specs throws before any proxy filters with a partial list)"""
    frames = open(FIX, "rb").read()
    h = pa.PvHandlers(num_periods=1, net_config={}, dns_config={})
    try:
        # no filter, then a failing call: every message still reaches the handlers
        with pytest.raises(pa.PvError, match="invalid CIDR"):
            h._check(h.lib.pv_set_dnstap_only_hosts(h.ctx, b"192.168.0.0/24,10.0.0.0/99"), "pv_set_dnstap_only_hosts")
        h.process_dnstap(frames)
        assert jget({"w": h.window_json(0)}, "w.dns.wire_packets.events") == 153
        # a filter, then a failing call: the filter stays (no message matches it, as above)
        h.reset()
        h._check(h.lib.pv_set_dnstap_only_hosts(h.ctx, b"192.168.0.0/24"), "pv_set_dnstap_only_hosts")
        with pytest.raises(pa.PvError, match="invalid IPv4 address"):
            h._check(h.lib.pv_set_dnstap_only_hosts(h.ctx, b"192.168.AE.0/24"), "pv_set_dnstap_only_hosts")
        h.process_dnstap(frames)
        with pytest.raises(pa.PvError, match="no data"):
            h.window_json(0)
    finally:
        h.close()
