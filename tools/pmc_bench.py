"""Fold a pmc_summary.py JSON (per-kernel means of one bench config) into the file bench.py reads
for its roofline.traffic / step_traffic: profiles/pmc_c<cfg>_<records>.json.

HBM bytes of a kernel = FETCH_SIZE x 2 (gfx950 counts half of a wide streaming read,
MI355X_MICROARCH.md HBM section) + WRITE_SIZE, KB x 1024. The step's bytes sum every pv_* kernel
of the summary, each counted once per step (pmc_summary.py reports per-dispatch means; the bench
steps launch each pv_* kernel once, except where --launches says otherwise).

  python tools/pmc_bench.py profiles/r4/pmc_c2.json 2 10000000 pv_net_kernel_ring "C2 10M x 64 B" > profiles/pmc_c2_10000000.json
"""
import json
import sys


def hbm(m):
    return m.get("FETCH_SIZE", 0) * 1024 * 2 + m.get("WRITE_SIZE", 0) * 1024


def main():
    src, cfg, n, kern, workload = sys.argv[1:6]
    d = json.load(open(src))["kernels"]
    per = {k: round(hbm(m)) for k, m in d.items() if k.startswith("pv_")}
    m = d[kern]
    out = {
        "kernel": kern,
        "workload": workload,
        "fetch_bytes_per_launch": round(m.get("FETCH_SIZE", 0) * 1024 * 2),
        "write_bytes_per_launch": round(m.get("WRITE_SIZE", 0) * 1024),
        "hbm_bytes_per_launch": per[kern],
        "hbm_bytes_per_step": sum(per.values()),
        "hbm_bytes_per_kernel": per,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE+TCC_HIT+TCC_MISS in separate runs (tools/gpu_pmc.sh); "
                  "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section), KB x 1024; step = every pv_* kernel once",
        "source": src,
    }
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
