"""Parity of one Net-pass variant selected by the environment (PV_NET_KERNEL is read once per
process, so each variant runs in a process of its own; test_gpu_net_variants.py starts them).

usage: PV_NET_KERNEL=<variant> python -m tests.net_variant_worker
Checks the variant against the oracle on a reference fixture and synthetic C2 / C4 / edge-mix
traffic; prints the kernel the library launched and exits 0 when every case matches."""
import os
import sys


def main():
    import torch
    if torch.cuda.device_count() > 0:
        torch.cuda.init()  # torch's HIP runtime first (tests/conftest.py)
    import pktvisor_amd as pa
    from pktvisor_amd import synth
    from tests.oracle_ctypes import load as load_oracle
    from tests.test_gpu_parity import diff
    oracle = load_oracle()
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dns_udp_tcp_random.pcap")
    cases = [("dns_udp_tcp_random", open(gold, "rb").read(), "192.168.0.0/24"),
             ("c2", synth.pcap_bytes(2, 60000), synth.HOST_SPEC),
             ("c4", synth.pcap_bytes(4, 60000), synth.HOST_SPEC),
             ("edge_mix", synth.pcap_bytes(9, 20000), "10.0.0.0/8,2000::/3,192.168.0.0/16")]
    kernels = set()
    bad = []
    for name, pcap, host in cases:
        recs = pcap[24:]
        idx = pa.RecordIndex(recs)
        h = pa.PvHandlers(host_spec=host, num_periods=1, max_records=max(1, idx.n))
        try:
            h.process_host(recs)
            h.set_end_tstamp(*pa.last_record_ts(recs, idx))
            kernels.add(h.net_kernel_name())
            gpu = h.window_json(0)
        finally:
            h.close()
        ref = oracle.run_bytes(pcap, host_spec=host, num_periods=1, window=1)["1m"]
        d = diff(gpu, ref)
        if d:
            bad.append(f"{name}: {d}")
    print("kernels:", sorted(kernels))
    for b in bad:
        print("MISMATCH", b)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
