"""Fold a pmc_summary.py JSON (per-kernel means of one bench config) into the file bench.py reads
for its roofline.traffic / step_traffic: profiles/pmc_c<cfg>_<records>.json.

HBM bytes of a kernel = FETCH_SIZE x 2 for the 16-B streaming-read kernels (gfx950 counts half of a
wide streaming read, MI355X_MICROARCH.md HBM section), x 1 for the others (STREAMING below), +
WRITE_SIZE, KB x 1024. The step's bytes sum every pv_* kernel
of the summary, each counted once per step (pmc_summary.py reports per-dispatch means; the bench
steps launch each pv_* kernel once, except where --launches says otherwise).

  python tools/pmc_bench.py profiles/r4/pmc_c2.json 2 10000000 pv_net_kernel_reg_tc "C2 10M x 64 B" > profiles/pmc_c2_10000000.json
"""
import json
import sys


# Kernels whose reads are wide streaming reads (16 B per lane, global_load_dwordx4 or LDS-DMA
# dwordx4 over consecutive records or messages): FETCH_SIZE counts half their bytes on gfx950
# (MI355X_MICROARCH.md HBM section), so x2. Every other kernel's reads are gathers or 4/8-B loads,
# for which the guide gives no calibration: FETCH_SIZE is taken as it reads (x1), the lower figure
# (the merge's raw fetch matches its expected region + list bytes).
STREAMING = {
    "pv_net_kernel_reg_tc": "record windows, 5 x 16 B per lane, lanes on consecutive records",
    "pv_net_kernel_reg": "record windows, 5 x 16 B per lane, lanes on consecutive records",
    "pv_net_kernel": "LDS-DMA dwordx4 of packed tiles",
    "pv_net_kernel_ns": "LDS-DMA dwordx4 of packed tiles",
    "pv_dns_kernel": "128-B message windows, 8 x 16 B per lane into registers, lanes on consecutive messages",
    "pv_dns_kernel_f": "128-B message windows, 8 x 16 B per lane into registers, lanes on consecutive messages",
    "pv_dns_kernel_sfx": "128-B message windows, 8 x 16 B per lane into registers, lanes on consecutive messages",
    "pv_net_kernel_span": "each tile's packed span, 16 B per lane, consecutive",
}


def rule(k):
    return 2 if k in STREAMING else 1


def hbm(k, m):
    return m.get("FETCH_SIZE", 0) * 1024 * rule(k) + m.get("WRITE_SIZE", 0) * 1024


def main():
    src, cfg, n, kern, workload = sys.argv[1:6]
    d = json.load(open(src))["kernels"]
    per = {k: round(hbm(k, m)) for k, m in d.items() if k.startswith("pv_")}
    detail = {k: {"fetch_raw": round(m.get("FETCH_SIZE", 0) * 1024), "fetch_rule": f"x{rule(k)}",
                  "why": STREAMING.get(k, "gathers / narrow loads: uncalibrated, raw"),
                  "write": round(m.get("WRITE_SIZE", 0) * 1024), "hbm": per[k]}
              for k, m in d.items() if k.startswith("pv_")}
    m = d[kern]
    out = {
        "kernel": kern,
        "workload": workload,
        "fetch_bytes_per_launch": round(m.get("FETCH_SIZE", 0) * 1024 * rule(kern)),
        "write_bytes_per_launch": round(m.get("WRITE_SIZE", 0) * 1024),
        "hbm_bytes_per_launch": per[kern],
        "hbm_bytes_per_step": sum(per.values()),
        "hbm_bytes_per_kernel": per,
        "per_kernel": detail,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE+TCC_HIT+TCC_MISS in separate runs (tools/gpu_pmc.sh); "
                  "FETCH_SIZE x2 for the 16-B streaming-read kernels only (MI355X_MICROARCH.md HBM section), x1 for the "
                  "others (per_kernel.fetch_rule), KB x 1024; step = every pv_* kernel once (sum of hbm_bytes_per_kernel)",
        "source": src,
    }
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
