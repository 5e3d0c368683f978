#!/bin/bash
# ksum.sh <dir>: per-config kernel averages (us) of rocprofv3 --stats csv files + bench lines
d=$1
for f in $(ls $d/prof/*_kernel_stats.csv $d/*/*_kernel_stats.csv 2>/dev/null); do
python3 - "$f" <<'P'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[1].split('/')[-2]+'/'+sys.argv[1].split('/')[-1][:2], " ".join(f"{r['Name'][:18].replace('void rocprim::','')}={float(r['AverageNs'])/1e3:.0f}" for r in rows[:11] if 'copyBuffer' not in r['Name']))
P
done
for c in 2 3 4; do f=$d/bench_c$c.json; [ -f $f ] && python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('C$c', d['value'], 'ms', d['ms_per_step'], 'med', d.get('ms_per_step_median'), 'net', d['roofline']['kernel_ms'], d['roofline']['frac'])"; done
