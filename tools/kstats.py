"""Print the per-kernel average time (us) of rocprofv3 --stats csv files: kstats.py dir..."""
import csv, glob, os, sys
for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        print(d, "no stats"); continue
    rows = list(csv.DictReader(open(f[0])))
    parts = []
    for x in rows:
        nm = x["Name"].split("(")[0].replace("void rocprim::ROCPRIM_400200_NS::detail::", "")[:22]
        if "rocclr" in nm or "fill" in nm: continue
        parts.append(f"{nm}={float(x['AverageNs'])/1000:.0f}")
    print(os.path.basename(d.rstrip('/')).ljust(12), " ".join(parts))
