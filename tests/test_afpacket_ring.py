"""f2: the AF_PACKET TPACKET_V3 capture loop (pv_afpacket_*, AFPacket::start_capture /
walk_block / flush_block, src/inputs/pcap/afpacket.cpp:72-86,214-243) over a ring laid out as
the kernel fills it (linux/if_packet.h), driven by a producer thread that plays the kernel's
part: it writes a block, hands it over with TP_STATUS_USER, signals an eventfd (the socket's
POLLIN) and reuses the block only once the loop gave it back (TP_STATUS_KERNEL).

CPU tests: records reach the sink in capture order with the block's ts_last_pkt, across ring
wrap-around and several staging batches; blocks are returned; the loop stops on request and on a
failing sink. The GPU test feeds pv_process_host and compares the window with the oracle."""
import ctypes
import mmap
import os
import struct
import threading
import time

import pytest

import pktvisor_amd as pa
from tests.pcapng_util import pcap_packets
from tests.test_tpacket3 import block

GOLD = os.path.join(os.path.dirname(__file__), "golden")
BS = 1 << 16  # ring block bytes


class FakeKernel:
    """num_blocks ring blocks in an anonymous mapping and the kernel's side of the protocol"""

    def __init__(self, num_blocks=4, block_size=BS):
        self.nb, self.bs = num_blocks, block_size
        self.mm = mmap.mmap(-1, num_blocks * block_size)
        self.addr = ctypes.addressof(ctypes.c_char.from_buffer(self.mm))
        self.efd = os.eventfd(0, os.EFD_NONBLOCK)
        self.next = 0
        self.handed = 0

    def status(self, k):
        return struct.unpack_from("<I", self.mm, k * self.bs + 8)[0]

    def put(self, raw, timeout=20.0, stopped=lambda: False):
        k = self.next
        t0 = time.time()
        while self.status(k) != 0:  # TP_STATUS_KERNEL: the loop gave it back
            if stopped():
                return False  # the loop ended (a failing sink): no one returns blocks any more
            if time.time() - t0 > timeout:
                raise TimeoutError("ring block never returned")
            time.sleep(0.0005)
        body = bytearray(raw[: self.bs])
        struct.pack_into("<I", body, 8, 0)
        self.mm[k * self.bs:(k + 1) * self.bs] = bytes(body) + b"\0" * (self.bs - len(body))
        struct.pack_into("<I", self.mm, k * self.bs + 8, 1)  # TP_STATUS_USER, last
        os.eventfd_write(self.efd, 1)
        self.next = (k + 1) % self.nb
        self.handed += 1
        return True

    def close(self):
        os.close(self.efd)


def fixture_blocks(name="dns_udp_tcp_random.pcap", per=37):
    pcap = open(os.path.join(GOLD, name), "rb").read()
    _, pk = pcap_packets(pcap)
    frames = [p[4] for p in pk]
    blocks = []
    for j in range(0, len(frames), per):
        part = frames[j:j + per]
        blocks.append((part, (1700000000 + j // 500, 1000 * j)))
    return blocks


def parse_records(recs):
    out, p = [], 0
    while p < len(recs):
        s, ns, cl, ol = struct.unpack_from("<IIII", recs, p)
        out.append((s, ns, recs[p + 16:p + 16 + cl]))
        p += 16 + cl
    return out


def run_capture(blocks, num_blocks=4, batch_bytes=1 << 15, sink_fail_after=None):
    fk = FakeKernel(num_blocks)
    cap = pa.AfPacket.attach(fk.addr, BS, num_blocks, fk.efd, batch_bytes=batch_bytes, flush_ms=20)
    got, batches = [], []
    rc = [None]

    def sink(recs, n):
        batches.append(n)
        got.extend(parse_records(recs))
        if sink_fail_after is not None and len(batches) > sink_fail_after:
            return 1
        return 0

    t = threading.Thread(target=lambda: rc.__setitem__(0, cap.run(sink)))
    t.start()
    try:
        for part, ts in blocks:
            if not fk.put(block(part, ts_last=ts, size=BS), stopped=lambda: rc[0] is not None) or rc[0] is not None:
                break
        want = sum(len(p) for p, _ in blocks)
        t0 = time.time()
        while len(got) < want and rc[0] is None and time.time() - t0 < 20:
            time.sleep(0.01)
    finally:
        cap.stop()
        t.join(timeout=30)
    st = cap.stats()
    cap.close()
    fk.close()
    return got, batches, rc[0], st


def test_ring_loop_records_in_order():
    blocks = fixture_blocks()
    got, batches, rc, st = run_capture(blocks)
    assert rc == 0
    want = [(ts[0], ts[1], f) for part, ts in blocks for f in part]
    assert len(got) == len(want)
    assert got == want  # capture order, the block's ts_last_pkt, frames intact
    assert len(batches) > 3 and sum(batches) == len(want)
    assert st["blocks"] == len(blocks) > 4  # the ring wrapped
    assert st["packets"] == len(want) and st["batches"] == len(batches)


def test_ring_loop_equals_block_walk():
    blocks = fixture_blocks("dns_udp_mixed_rcode.pcap", per=5)
    got, _, rc, _ = run_capture(blocks, num_blocks=2, batch_bytes=1 << 12)
    assert rc == 0
    ref = parse_records(pa.tpacket3_records([block(p, ts_last=ts, size=BS) for p, ts in blocks]))
    assert got == ref


def test_ring_loop_failing_sink_stops():
    blocks = fixture_blocks(per=20)
    got, batches, rc, _ = run_capture(blocks, batch_bytes=1 << 12, sink_fail_after=1)
    assert rc == 1
    assert len(batches) == 2


def test_open_unknown_interface():
    with pytest.raises(pa.PvError):
        pa.AfPacket.open("pv-no-such-if0")


@pytest.mark.gpu
def test_ring_loop_into_handlers(oracle):
    """records from the ring through pv_process_host (linktype 1, ns timestamps) equal the oracle
    on the same records written as a nanosecond pcap"""
    blocks = fixture_blocks(per=64)
    fk = FakeKernel(4)
    h = pa.PvHandlers(host_spec="192.168.0.0/24", num_periods=1, linktype=1, ts_nano=1, max_records=1 << 16)
    cap = pa.AfPacket.attach(fk.addr, BS, 4, fk.efd, batch_bytes=1 << 16, flush_ms=20)
    try:
        cap.start(h)
        for part, ts in blocks:
            fk.put(block(part, ts_last=ts, size=BS))
        want = sum(len(p) for p, _ in blocks)
        t0 = time.time()
        while cap.stats()["packets"] < want and time.time() - t0 < 60:
            time.sleep(0.01)
        assert cap.stop() == 0
        recs = pa.tpacket3_records([block(p, ts_last=ts, size=BS) for p, ts in blocks])
        last = parse_records(recs)[-1]
        h.set_end_tstamp(last[0], last[1])
        gpu = h.window_json(0)
        ref = oracle.run_bytes(pa.pcap_file_bytes(recs, linktype=1, ts_nano=1), host_spec="192.168.0.0/24",
                               num_periods=1, window=1)["1m"]
        assert gpu == ref
    finally:
        cap.close()
        h.close()
        fk.close()
