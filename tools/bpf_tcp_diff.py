"""Diagnostic: the windows of dns_udp_tcp_random.pcap read with a BPF program that drops the small
packets (every TCP handshake / ACK / FIN segment), GPU against the oracle: all differing keys."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pktvisor_amd as pa
from tests import bpf_progs
from tests.oracle_ctypes import load


def walk(a, b, path, out):
    if isinstance(a, dict) and isinstance(b, dict):
        for k in sorted(set(a) | set(b)):
            walk(a.get(k), b.get(k), f"{path}.{k}", out)
    elif isinstance(a, list) and isinstance(b, list) and len(a) == len(b):
        for i, (x, y) in enumerate(zip(a, b)):
            walk(x, y, f"{path}[{i}]", out)
    elif a != b:
        out.append((path, a, b))


pcap = open("tests/golden/dns_udp_tcp_random.pcap", "rb").read()
open("/tmp/in.pcap", "wb").write(pcap)
insns = bpf_progs.ARITH
gpu = pa.pktvisor_reader("/tmp/in.pcap", host_spec="192.168.0.0/24", periods=1, bpf=insns)
kept = pcap[:24] + bpf_progs.filter_records(pcap[24:], insns)
ref = load().run_bytes(kept, host_spec="192.168.0.0/24", num_periods=1, window=1)
out = []
walk(gpu, ref, "", out)
print(len(out), "differences")
for d in out[:60]:
    print(d)
