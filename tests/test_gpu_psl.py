"""DNS v1 `public_suffix_list` (DnsStreamHandler::_configs, src/handlers/dns/v1/DnsStreamHandler.cpp:648-657;
match_public_suffix, libs/visor_dns/PublicSuffixList.h:226-250) on the GPU path against the oracle, the
reference KAT (test_dns_layer.cpp:603-637), and only_qname_suffix with many-dot suffixes (the DNS pass's
re-walk for suffixes covering two or more of a name's last four dots)."""
import os
import struct

import pytest

import pktvisor_amd as pa
from tests.test_gpu_parity import diff

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

# names chosen around the table's quirks: listed multi-label suffixes, byte (not label) suffix
# matches ("xcom.ac" ends with "com.ac"), unlisted labels, a key holding a dot ("ac.za"), the
# literal "*.sch.uk", trailing dots, upper case, one-label and very long names
NAMES = ["www.example.co.uk", "a.b.c.d.example.co.uk", "mail.xcom.ac", "x.y.z.k12.ak.us", "deep.a.b.c.d.e.f.k12.ak.us",
         "host.uk", "uk", "foo.ac.za", "q.w.e.r.sth.ac.at", "One.Two.GOV.AU", "a.b.c.d.e.f.g.h.i.example.com",
         "trailing.example.co.jp.", "s.t.u.v.w.x.*.sch.uk", "pref.tokyo.jp", "a.b.c.d.kawasaki.jp", "www.google.com",
         "x" * 60 + ".y.z.co.nz", "sub.domain.blogspot.co.uk", "k.l.m.n.o.p.com.br", "a.b.city.kawasaki.jp"]


def _name(n: str) -> bytes:
    out = b""
    for lab in n.rstrip(".").split("."):
        out += bytes([len(lab)]) + lab.encode()
    return out + b"\0"


def psl_pcap(reps: int = 40) -> bytes:
    recs, ts, txid = [], 1_600_000_000_000_000, 1
    for r in range(reps):
        for k, n in enumerate(NAMES):
            for qr in (0, 1):
                flags = 0x8180 if qr else 0x0100
                msg = struct.pack(">HHHHHH", txid, flags, 1, 0, 0, 0) + _name(n) + struct.pack(">HH", 1, 1)
                sport, dport = (53, 40000 + k) if qr else (40000 + k, 53)
                src, dst = (bytes([8, 8, 8, 8]), bytes([192, 168, 0, 10])) if qr else (bytes([192, 168, 0, 10]), bytes([8, 8, 8, 8]))
                udp = struct.pack(">HHHH", sport, dport, 8 + len(msg), 0) + msg
                ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + len(udp), txid & 0xffff, 0, 64, 17, 0, src, dst) + udp
                fr = b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb\x08\x00" + ip
                recs.append(struct.pack("<IIII", ts // 1_000_000, ts % 1_000_000, len(fr), len(fr)) + fr)
                ts += 250
            txid = (txid + 1) & 0xffff
    return struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1) + b"".join(recs)


def _both(oracle, tmp_path, pcap, f, okw, periods=1):
    p = tmp_path / "psl.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec="192.168.0.0/24", periods=periods, dns_filters=f)
    ref = oracle.run_bytes(pcap, host_spec="192.168.0.0/24", num_periods=periods, window=periods, **okw)
    return gpu, ref


def test_psl_synthetic_parity(oracle, tmp_path):
    gpu, ref = _both(oracle, tmp_path, psl_pcap(), {"public_suffix_list": True}, {"public_suffix_list": 1})
    assert diff(gpu, ref) is None, diff(gpu, ref)
    names = {e["name"] for e in ref["1m"]["dns"]["top_qname2"]}
    assert ".example.co.uk" in names and ".k12.ak.us" in names  # listed suffixes took effect


def test_psl_ignored_with_only_qname_suffix(oracle, tmp_path):
    f = {"public_suffix_list": True, "only_qname_suffix": ["co.uk", ".ak.us"]}
    gpu, ref = _both(oracle, tmp_path, psl_pcap(8), f, {"public_suffix_list": 1, "only_qname_suffix": "co.uk,.ak.us"})
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("sfx", [["www.google.com"], [".k12.ak.us", "c.d.e.f.k12.ak.us"], ["y.z.co.nz", "a.b.city.kawasaki.jp"]])
def test_many_dot_qname_suffix_parity(oracle, tmp_path, sfx):
    """only_qname_suffix with two or more dots after the first character (refused before this change)"""
    gpu, ref = _both(oracle, tmp_path, psl_pcap(8), {"only_qname_suffix": sfx}, {"only_qname_suffix": ",".join(sfx)}, periods=5)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_psl_reference_kat():
    """test_dns_layer.cpp:603-637 on dns_udp_mixed_rcode.pcap"""
    j = pa.pktvisor_reader(os.path.join(GOLD, "dns_udp_mixed_rcode.pcap"), host_spec="192.168.0.0/24", periods=1,
                           dns_filters={"public_suffix_list": True})["1m"]["dns"]
    w = j["wire_packets"]
    assert (w["udp"], w["noerror"], w["srvfail"], w["refused"], w["nxdomain"], w["filtered"]) == (24, 10, 0, 1, 1, 0)
    assert j["top_qname2"][0]["name"] == ".mwbsys.com" and j["top_qname3"][0]["name"] == "sirius.mwbsys.com"


# ---- DNS v2 (dns/v2/DnsStreamHandler.cpp:192-194 config, _configs :612-619, new_dns_transaction
# :1067-1072): the response's own suffix size aggregates its transaction's top_qname2/3
V2_ALL = ["cardinality", "counters", "quantiles", "top_ecs", "top_qtypes", "top_rcodes", "top_size", "top_qnames",
          "top_ports", "xact_times"]


def _both_v2(oracle, tmp_path, pcap, cfg, okw, periods=1, host="192.168.0.0/24"):
    p = tmp_path / "psl2.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec=host, periods=periods, dns2_config={"enable": V2_ALL, **cfg})
    ref = oracle.run_bytes(pcap, host_spec=host, num_periods=periods, window=periods, dns2_groups=0x3ff, **okw)
    return gpu, ref


@pytest.mark.parametrize("periods", [1, 5])
def test_psl_v2_synthetic_parity(oracle, tmp_path, periods):
    gpu, ref = _both_v2(oracle, tmp_path, psl_pcap(), {"public_suffix_list": True}, {"public_suffix_list": 1}, periods)
    assert diff(gpu, ref) is None, diff(gpu, ref)
    key = "1m" if periods == 1 else f"{periods}m"
    names = {e["name"] for e in ref[key]["dns"]["out"]["top_qname2_xacts"]}
    assert ".example.co.uk" in names and ".k12.ak.us" in names  # listed suffixes took effect


@pytest.mark.parametrize("fixture", ["dns_udp_tcp_random.pcap", "dns_ipv6_tcp.pcap", "dns_udp_mixed_rcode.pcap"])
def test_psl_v2_fixture_parity(oracle, tmp_path, fixture):
    """UDP and DNS-over-TCP transactions (a TCP response's suffix size comes from the TCP pass)"""
    pcap = open(os.path.join(GOLD, fixture), "rb").read()
    gpu, ref = _both_v2(oracle, tmp_path, pcap, {"public_suffix_list": True}, {"public_suffix_list": 1})
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_psl_v2_ignored_with_only_qname_suffix(oracle, tmp_path):
    cfg = {"public_suffix_list": True, "only_qname_suffix": ["co.uk", ".ak.us"]}
    gpu, ref = _both_v2(oracle, tmp_path, psl_pcap(8), cfg, {"public_suffix_list": 1, "only_qname_suffix": "co.uk,.ak.us"})
    assert diff(gpu, ref) is None, diff(gpu, ref)
