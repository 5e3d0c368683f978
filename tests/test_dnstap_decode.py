"""Frame Streams / dnstap protobuf decoding on the host (pv_dnstap_count, no GPU): the
reference fixture's frames, and malformed input that must neither crash nor over-read."""
import os
import struct

import pktvisor_amd as pa

FIX = os.path.join(os.path.dirname(__file__), "golden", "fixture.dnstap")


def test_fixture_frames_and_events():
    data = open(FIX, "rb").read()
    assert pa.dnstap_count(data) == (153, 153)  # test_dnstap.cpp:30: 153 events


def test_truncated_and_garbage():
    data = open(FIX, "rb").read()
    for cut in (0, 3, 7, 50, 1000, len(data) - 5):
        nf, ne = pa.dnstap_count(data[:cut])
        assert ne <= nf <= 153
    # a data frame that is not a dnstap protobuf is skipped, not an event
    junk = struct.pack(">I", 5) + b"\xff\xff\xff\xff\xff"
    assert pa.dnstap_count(junk) == (1, 0)
    # Dnstap of type MESSAGE (15: 1) without a message: skipped
    assert pa.dnstap_count(struct.pack(">I", 2) + b"\x78\x01") == (1, 0)
    # a minimal MESSAGE: message {type CLIENT_QUERY}
    msg = b"\x72\x02\x08\x05" + b"\x78\x01"
    assert pa.dnstap_count(struct.pack(">I", len(msg)) + msg) == (1, 1)
    # Message without its required type field: the parse fails (proto2 required)
    msg = b"\x72\x02\x10\x01" + b"\x78\x01"
    assert pa.dnstap_count(struct.pack(">I", len(msg)) + msg) == (1, 0)
