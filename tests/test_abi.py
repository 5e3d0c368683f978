"""The C-ABI library loads, exports every symbol include/pvgpu.h declares, and its
pure-host entry points behave (no GPU needed)."""
import ctypes
import os
import re
import struct

import numpy as np
import pytest

import pktvisor_amd as pa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "pvgpu.h")).read()
    return sorted(set(re.findall(r"\b(pv_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_python_export_list():
    assert header_symbols() == sorted(pa.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = pa.load_library()
    for sym in header_symbols():
        assert hasattr(lib, sym), sym
    assert lib.pv_version().decode().startswith("pvgpu")


def test_index_records_matches_python_walk():
    _, _, recs = pa.read_pcap(os.path.join(ROOT, "tests", "golden", "dns_udp_tcp_random.pcap"))
    idx = pa.RecordIndex(recs)
    offs, pos, secs = [], 0, []
    while pos + 16 <= len(recs):
        s, us, incl, _ = struct.unpack_from("<IIII", recs, pos)
        offs.append(pos)
        secs.append(s)
        pos += 16 + incl
    assert idx.n == len(offs) == 16147
    assert np.array_equal(idx.offsets, np.array(offs, dtype=np.uint32))
    assert idx.info.monotone == 1
    assert idx.info.first_sec == secs[0] and idx.info.last_sec == secs[-1]
    changes = [i for i in range(len(secs)) if i == 0 or secs[i] != secs[i - 1]]
    assert idx.info.n_sec_changes == len(changes)
    assert list(idx.sc_idx[: len(changes)]) == changes


def test_index_records_detects_non_monotone():
    from pktvisor_amd import synth
    buf, _, used = synth.records(2, 100)
    b = bytearray(buf[:used].tobytes())
    struct.pack_into("<I", b, 80 * 50, 1600000000)  # record 50 goes back in time
    idx = pa.RecordIndex(bytes(b))
    assert idx.n == 100 and idx.info.monotone == 0


@pytest.mark.skipif(pa.device_count() > 0, reason="a GPU is present")
def test_create_fails_loudly_without_gpu():
    with pytest.raises(pa.PvError):
        pa.PvHandlers(host_spec="10.0.0.0/8")


def test_bad_host_spec_error_strings():
    # error strings of libs/visor_utils/utils.cpp:128-164 (checked before any device work)
    for spec, msg in [("10.0.0.0", "invalid CIDR: 10.0.0.0"), ("10.0.0.0/33", "invalid CIDR: 10.0.0.0/33"),
                      ("10.0.0.300/8", "invalid IPv4 address: 10.0.0.300"), ("fe80::zz/64", "invalid IPv6 address: fe80::zz")]:
        with pytest.raises(pa.PvError, match=re.escape(msg)):
            pa.PvHandlers(host_spec=spec)
