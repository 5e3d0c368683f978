"""The pcap input's "bpf" filter end to end (PcapInputStream::_open_pcap's setFilter,
src/inputs/pcap/PcapInputStream.cpp:485-488): a capture read with a compiled classic-BPF program
gives the windows of the capture holding only the records the program keeps (the oracle run on
that capture). Parity unpinned for the filter itself (tests/bpf_progs.py)."""
import os

import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests import bpf_progs
from tests.test_gpu_parity import GOLD, diff

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prog,src", [("udp53", "dns_udp_tcp_random.pcap"), ("short", "dns_udp_tcp_random.pcap"),
                                      ("arith", "dns_udp_mixed_rcode.pcap"), ("udp53", "c4"), ("short", "c4"),
                                      ("arith", "c4")])
def test_bpf_reader_parity(oracle, tmp_path, prog, src):
    pcap = open(os.path.join(GOLD, src), "rb").read() if src.endswith(".pcap") else synth.pcap_bytes(4, 20000)
    p = tmp_path / "in.pcap"
    p.write_bytes(pcap)
    insns = bpf_progs.PROGRAMS[prog]
    host = "192.168.0.0/24" if src.endswith(".pcap") else synth.HOST_SPEC
    gpu = pa.pktvisor_reader(str(p), host_spec=host, periods=1, bpf=insns)
    kept = pcap[:24] + bpf_progs.filter_records(pcap[24:], insns)
    assert len(kept) < len(pcap)
    ref = oracle.run_bytes(kept, host_spec=host, num_periods=1, window=1)
    assert diff(gpu, ref) is None, diff(gpu, ref)


def test_bpf_context_filter(oracle):
    """pv_set_bpf on a context: pv_process_host drops the rejected records of every block"""
    pcap = synth.pcap_bytes(4, 20000)
    recs = pcap[24:]
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=1, max_records=1 << 15, bpf=bpf_progs.UDP53)
    try:
        half = len(recs) // 2
        cut = 0
        while cut < half:  # a record boundary near the middle
            cut += 16 + int.from_bytes(recs[cut + 8:cut + 12], "little")
        h.process_host(recs[:cut])
        h.process_host(recs[cut:])
        kept = bpf_progs.filter_records(recs, bpf_progs.UDP53)
        idx = pa.RecordIndex(kept)
        h.set_end_tstamp(*pa.last_record_ts(kept, idx))
        got = {"1m": h.window_json(0)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap[:24] + kept, host_spec=synth.HOST_SPEC, num_periods=1, window=1)
    assert diff(got, ref) is None, diff(got, ref)


@pytest.mark.parametrize("prog", ["udp53", "short", "arith"])
def test_bpf_device_resident(oracle, prog):
    """pv_process_device with a program set: the filter runs on the batch in HBM (pv_bpf_keep /
    pv_bpf_gather), so device-resident input is filtered as the pcap input filters its reader"""
    import numpy as np
    import torch
    pcap = synth.pcap_bytes(4, 30000)
    recs = pcap[24:]
    insns = bpf_progs.PROGRAMS[prog]
    idx = pa.RecordIndex(recs)
    d_recs = torch.from_numpy(np.frombuffer(recs + bytes(256), dtype=np.uint8).copy()).cuda()
    d_offs = torch.from_numpy(np.ascontiguousarray(idx.offsets[: idx.n])).cuda()
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=1, max_records=idx.n, bpf=insns)
    try:
        h.process_device(d_recs.data_ptr(), d_offs.data_ptr(), idx)
        h.synchronize()
        kept = bpf_progs.filter_records(recs, insns)
        assert 0 < len(kept) < len(recs)
        kidx = pa.RecordIndex(kept)
        h.set_end_tstamp(*pa.last_record_ts(kept, kidx))
        got = {"1m": h.window_json(0)}
    finally:
        h.close()
    ref = oracle.run_bytes(pcap[:24] + kept, host_spec=synth.HOST_SPEC, num_periods=1, window=1)
    assert diff(got, ref) is None, diff(got, ref)
