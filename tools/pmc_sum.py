"""Average PMC counter values per dispatch of one kernel from rocprofv3 --pmc csv dirs:
pmc_sum.py KERNEL dir..."""
import csv, glob, os, sys
from collections import defaultdict
kern = sys.argv[1]
for d in sys.argv[2:]:
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        print(d, "no counters"); continue
    acc = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if kern in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d.rstrip("/")), " ".join(f"{k}={sum(v)/len(v):.4g}" for k, v in sorted(acc.items())))
