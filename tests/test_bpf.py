"""The pcap input's "bpf" filter (PcapInputStream.cpp:485-488) on the host side of the ABI:
the library's classic-BPF interpreter (pv_bpf_run / pv_bpf_filter_records, pv_bpf.cpp) against
the independent restatement in tests/bpf_progs.py over every record of the reference fixture
pcaps and a synthetic mix, and the checker's refusals (pv_bpf_validate, pv_set_bpf)."""
import ctypes
import os

import numpy as np
import pytest

import pktvisor_amd as pa
from pktvisor_amd import synth
from tests import bpf_progs

GOLD = os.path.join(os.path.dirname(__file__), "golden")
PCAPS = ["dns_ipv4_udp.pcap", "dns_ipv4_tcp.pcap", "dns_ipv6_udp.pcap", "dns_udp_mixed_rcode.pcap"]


def blobs():
    for name in PCAPS:
        p = os.path.join(GOLD, name)
        if os.path.exists(p):
            yield name, pa.read_pcap(p)[2]
    yield "c4", synth.pcap_bytes(4, 3000)[24:]
    yield "edge", synth.pcap_bytes(9, 2000)[24:]


@pytest.mark.parametrize("prog", sorted(bpf_progs.PROGRAMS))
def test_filter_matches_restatement(prog):
    insns = bpf_progs.PROGRAMS[prog]
    lib = pa.load_library()
    arr = pa.bpf_program(insns)
    assert lib.pv_bpf_validate(arr, len(insns)) == 0
    kept_any = dropped_any = False
    for name, recs in blobs():
        want = bpf_progs.filter_records(recs, insns)
        got = pa.bpf_filter(recs, insns)
        assert got == want, (prog, name)
        kept_any |= len(want) > 0
        dropped_any |= len(want) < len(recs)
        # per frame, the program's answer itself (snap length or A)
        buf = np.frombuffer(recs, dtype=np.uint8)
        pos = 0
        while pos + 16 <= len(recs):
            incl, orig = np.frombuffer(recs[pos + 8:pos + 16], dtype="<u4")
            frame = recs[pos + 16:pos + 16 + int(incl)]
            r = lib.pv_bpf_run(arr, buf.ctypes.data + pos + 16, int(orig), int(incl))
            assert r == bpf_progs.run(insns, frame, int(orig)), (prog, name, pos)
            pos += 16 + int(incl)
    assert kept_any and dropped_any, prog


@pytest.mark.parametrize("bad", sorted(bpf_progs.INVALID))
def test_checker_refuses(bad):
    insns = bpf_progs.INVALID[bad]
    lib = pa.load_library()
    assert lib.pv_bpf_validate(pa.bpf_program(insns) if insns else None, len(insns)) != 0
    with pytest.raises(pa.PvError):
        pa.bpf_filter(b"", insns)


def test_truncated_tail_dropped():
    recs = synth.pcap_bytes(2, 10)[24:]
    cut = recs[:-5]
    want = bpf_progs.filter_records(cut, bpf_progs.SHORT)
    assert pa.bpf_filter(cut, bpf_progs.SHORT) == want
    assert len(want) < len(recs)
