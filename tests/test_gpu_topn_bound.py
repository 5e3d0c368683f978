"""Bounded top-N tables under a random-subdomain flood (pv_topn_purge, the frequent-items
sketch's purge that TopN relies on, src/Metrics.h:488-538): with a table far smaller than the
flood's distinct names, the heavy names still come out on top with estimates in
[true count, true count + the sketch's error bound], while a table large enough for every
name keeps the result exact (the oracle's counts)."""
import numpy as np
import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests.test_gpu_parity import diff

pytestmark = pytest.mark.gpu


def _run(pcap, table_log2, batch):
    recs = pcap[24:]
    idx = pa.RecordIndex(recs)
    offs = list(idx.offsets) + [len(recs)]
    h = pa.PvHandlers(host_spec="10.0.0.0/8", num_periods=1, table_log2=table_log2, max_records=1 << 17,
                      topn_count=10)
    try:
        for i in range(0, idx.n, batch):
            h.process_host(recs[offs[i]:offs[min(idx.n, i + batch)]])
        return h.window_json(0)
    finally:
        h.close()


@pytest.mark.parametrize("table_log2,batch", [(12, 1000), (13, 1500)])
def test_flood_bounded_estimates(table_log2, batch):
    pcap, heavy, total = synth.qname_flood_pcap(7, flood=60000)
    w = _run(pcap, table_log2, batch)
    dns = w["dns"]
    top3 = dns["top_qname3"]
    assert [e["name"] for e in top3] == sorted(heavy, key=lambda n: -heavy[n])[:10]
    # offset bound: each purge removes theta x (half a region) of stored weight
    rs = 1 << min(table_log2, 12)
    bound = 4 * total * rs // (1 << table_log2) // rs + 2
    for e in top3:
        t = heavy[e["name"]]
        assert t <= e["estimate"] <= t + bound, (e, t, bound)
    # the second-level name is one key, never purged: exact
    assert dns["top_qname2"][0] == {"name": ".victim.example", "estimate": total}
    assert dns["wire_packets"]["total"] == total


def test_flood_large_table_exact(oracle, tmp_path):
    """no purge when the table holds every name: bit-exact with the oracle"""
    pcap, heavy, total = synth.qname_flood_pcap(3, flood=20000)
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    gpu = pa.pktvisor_reader(str(p), host_spec="10.0.0.0/8", periods=1)
    ref = oracle.run_bytes(pcap, host_spec="10.0.0.0/8", num_periods=1, window=1)
    assert diff(gpu, ref) is None, diff(gpu, ref)


@pytest.mark.parametrize("table_log2", [10, 12])
def test_flood_one_batch_degrades(table_log2):
    """the whole flood in ONE batch, far more distinct names than the table holds: full regions
    hand their updates to the overflow list, the table is purged and they are inserted again
    (drain_overflow) instead of the batch failing; the same bounds hold"""
    pcap, heavy, total = synth.qname_flood_pcap(11, flood=60000)
    w = _run(pcap, table_log2, 1 << 17)
    dns = w["dns"]
    top3 = dns["top_qname3"]
    assert [e["name"] for e in top3] == sorted(heavy, key=lambda n: -heavy[n])[:10]
    rounds_bound = 64  # drain_overflow's rounds, each adds one theta (1 here: singletons)
    for e in top3:
        t = heavy[e["name"]]
        assert t <= e["estimate"] <= t + rounds_bound, (e, t)
    assert dns["top_qname2"][0] == {"name": ".victim.example", "estimate": total}
    assert dns["wire_packets"]["total"] == total


def test_dirty_writeback_after_purge():
    """pv_topn_merge writes back only the entries a batch changed (a dirty byte per
    entry). After a flood has purged the table, batches that touch only the heavy names must move
    each heavy estimate by exactly its new count (no purge runs: 24 live keys), so the merge wrote
    every changed entry back and left the others as the purge left them."""
    import struct
    pcap, heavy, total = synth.qname_flood_pcap(7, flood=60000)
    extra, heavy2, total2 = synth.qname_flood_pcap(8, flood=0, duration_s=5.0)
    more = bytearray(extra[24:])
    p = 0
    while p < len(more):  # 45 s later: the same 60 s period, after the flood
        s, us, cl, ol = struct.unpack_from("<IIII", more, p)
        struct.pack_into("<I", more, p, s + 45)
        p += 16 + cl
    h = pa.PvHandlers(host_spec="10.0.0.0/8", num_periods=1, table_log2=12, max_records=1 << 17, topn_count=24)
    try:
        def feed(recs, batch):
            idx = pa.RecordIndex(recs)
            offs = list(idx.offsets) + [len(recs)]
            for i in range(0, idx.n, batch):
                h.process_host(recs[offs[i]:offs[min(idx.n, i + batch)]])
        feed(pcap[24:], 1000)
        e1 = {e["name"]: e["estimate"] for e in h.window_json(0)["dns"]["top_qname3"]}
        feed(bytes(more), 300)
        e2 = {e["name"]: e["estimate"] for e in h.window_json(0)["dns"]["top_qname3"]}
    finally:
        h.close()
    common = [n for n in heavy if n in e1 and n in e2]
    assert len(common) >= 20
    for n in common:
        assert e2[n] - e1[n] == heavy2[n], (n, e1[n], e2[n], heavy2[n])


def test_sharded_flood_owner_merge_purges(tmp_path, monkeypatch):
    """Three ranks each see a third of the flood in a 4096-entry table; the top-N owner merge
    receives more distinct names than a region holds, so full regions purge (the frequent-items
    merge's purge) and take the rest again instead of failing; the heavy names stay on top with
    estimates no lower than their true counts"""
    import json
    from tests.dist_launch import run_ranks
    pcap, heavy, total = synth.qname_flood_pcap(7, flood=60000)
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    out = tmp_path / "merged.json"
    monkeypatch.setenv("PV_TEST_TABLE_LOG2", "12")
    run_ranks(3, ["gpu", str(p), str(out), "10.0.0.0/8", "1"])
    dns = json.load(open(out))["1m"]["dns"]
    top3 = dns["top_qname3"]
    assert [e["name"] for e in top3] == sorted(heavy, key=lambda n: -heavy[n])[:10]
    bound = 3 * (4 * total // 4096 + 2) + 64
    for e in top3:
        t = heavy[e["name"]]
        assert t <= e["estimate"] <= t + bound, (e, t, bound)
    assert dns["top_qname2"][0] == {"name": ".victim.example", "estimate": total}
    assert dns["wire_packets"]["total"] == total


def _v6_query_pcap(n, seed):
    """UDP DNS queries from n random IPv6 clients (2001:db8::/32) to one server, each asking
    h<k>.n<k % 997>.example.com"""
    import ipaddress
    import struct
    rng = np.random.default_rng(seed)
    dst = bytes.fromhex("20014860000000000000000000008888")
    out, srcs = bytearray(), set()
    for k in range(n):
        src = bytes.fromhex("20010db8") + rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        srcs.add(str(ipaddress.IPv6Address(src)))
        q = synth._dns_msg(rng, k & 0xffff, False, f"h{k}.n{k % 997}.example.com", 1)
        udp = struct.pack(">HHHH", 1024 + k % 50000, 53, 8 + len(q), 0) + q
        fr = b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb\x86\xdd" + struct.pack(">IHBB", 0x60000000, len(udp), 17, 64) + src + dst + udp
        us = 1700000000 * 10**6 + 10 * k
        out += struct.pack("<IIII", us // 10**6, us % 10**6, len(fr), len(fr)) + fr
    return pa.pcap_file_bytes(bytes(out)), srcs | {str(ipaddress.IPv6Address(dst))}


def test_new_name_list_overflow(monkeypatch, capfd):
    """one batch creating more named entries than the new-name list holds (table_log2 8: 256
    entries a table and in the list; the Net table's IPv6 keys and the DNS table's names fill
    512): the merge leaves the rest pending in their aux words and pv_topn_name_fix names them,
    so every listed entry carries its own name"""
    n = 6000
    pcap, addrs = _v6_query_pcap(n, 5)
    monkeypatch.setenv("PV_NAMEFIX_TRACE", "1")
    h = pa.PvHandlers(host_spec="2001:db8::/32", num_periods=1, table_log2=8, max_records=1 << 14, topn_count=10)
    try:
        h.process_host(pcap[24:])
        w = h.window_json(0)
    finally:
        h.close()
    assert "pending top-N names written" in capfd.readouterr().err  # the path under test ran
    v6 = w["packets"]["top_ipv6"]
    assert v6 and v6[0]["name"] == "2001:4860::8888" and v6[0]["estimate"] >= n
    assert all(e["name"] in addrs for e in v6), v6
    q3 = w["dns"]["top_qname3"]
    assert q3 and all(e["name"] in {f".n{j}.example.com" for j in range(997)} for e in q3), q3
    assert w["dns"]["top_qname2"][0] == {"name": ".example.com", "estimate": n}
    assert w["dns"]["wire_packets"]["total"] == n
