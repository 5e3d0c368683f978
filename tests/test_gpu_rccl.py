"""The library's own RCCL communicator (pv_comm_*, include/pvgpu.h): a C++ host shards across
GPUs without torch. One GPU on the test box, so world size 1: the window all-reduce and the
all-gather run through RCCL and leave a single shard's window unchanged."""
import os

import pytest

import pktvisor_amd as pa
from pktvisor_amd import dist as pvdist
from pktvisor_amd import synth

pytestmark = pytest.mark.gpu


def test_comm_world1_merge_window_identity(tmp_path):
    import torch
    p = tmp_path / "c4.pcap"
    p.write_bytes(synth.pcap_bytes(4, 20000))
    linktype, ts_nano, recs = pa.read_pcap(str(p))
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=5, max_records=20000)
    try:
        h.process_host(recs)
        before = h.window_json(5, merged=True)
        h.comm_init(pa.comm_unique_id(), 1, 0)
        assert h.comm_allgather(b"shard-0") == [b"shard-0"]
        assert h.comm_allgather(b"") == [b""]
        pvdist.merge_window(h, torch.device("cuda", 0), comm="pv")
        after = h.window_json(5, merged=True)
        assert after == before
        h.comm_destroy()
    finally:
        h.close()


def test_comm_requires_init():
    h = pa.PvHandlers(host_spec=synth.HOST_SPEC, num_periods=1, max_records=16)
    try:
        with pytest.raises(pa.PvError):
            h.comm_allreduce_window()
    finally:
        h.close()
