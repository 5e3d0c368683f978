"""Per-kernel means of the rocprofv3 --pmc passes of tools/gpu_pmc.sh (counter_collection.csv).

FETCH_SIZE is reported raw and x2: on gfx950 it counts half the bytes of wide (16 B/lane)
coalesced streaming reads (MI355X_MICROARCH.md, HBM section); other access widths are
uncalibrated, so the x2 figure is an upper estimate for gathers. Usage:
  python tools/pmc_summary.py gpurun_out/pmc 2 > profiles/r2/pmc_c2.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = (row.get("Dispatch_Id") or row.get("Correlation_Id"), row["Counter_Name"])
                per[k] += float(row["Counter_Value"])
                names[k[0]] = row["Kernel_Name"].split("(")[0]
        for (disp, ctr), v in per.items():
            vals[names[disp]][ctr].append(v)
    return vals


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    out = {}
    for p in (1, 2, 3, 4):
        for kern, ctrs in load(os.path.join(root, f"c{cfg}_p{p}")).items():
            for ctr, v in ctrs.items():
                out.setdefault(kern, {})[ctr] = sum(v) / len(v)
    for kern, m in out.items():
        if "FETCH_SIZE" in m:
            m["fetch_bytes_x2"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            m["write_bytes"] = m["WRITE_SIZE"] * 1024
        if m.get("SQ_WAVE_CYCLES"):
            w = m["SQ_WAVE_CYCLES"]
            m["frac_active_valu"] = m.get("SQ_ACTIVE_INST_VALU", 0) / w
            m["frac_active_any"] = m.get("SQ_ACTIVE_INST_ANY", 0) / w
            m["frac_wait_any"] = m.get("SQ_WAIT_ANY", 0) / w
            m["frac_wait_inst_any"] = m.get("SQ_WAIT_INST_ANY", 0) / w
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("TCC_HIT", 0) + m.get("TCC_MISS", 0):
            m["l2_hit_rate"] = m["TCC_HIT"] / (m["TCC_HIT"] + m["TCC_MISS"])
    json.dump({"config": f"C{cfg}", "method": "rocprofv3 --pmc, one counter group per run (tools/gpu_pmc.sh); per-dispatch means",
               "kernels": out}, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
