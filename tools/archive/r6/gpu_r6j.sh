#!/bin/bash
# Round 6: kernel stats of C2 with the deferred general path (reg pass + pv_net_slow_list)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6j}; mkdir -p $O
export TMPDIR=/tmp
for c in 2 4; do
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c > $O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
echo "c$c $(python3 tools/kstats.py $O/prof_c$c 2>/dev/null | cut -c1-300)"
done
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r6j/prof_c2/k_kernel_trace.csv' if False else __import__('glob').glob('gpurun_out/r6j/prof_c2/**/*kernel_trace.csv', recursive=True)[0])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
prev=None
for r in rows[-16:]:
    s=int(r['Start_Timestamp']); e=int(r['End_Timestamp'])
    print(f"{r['Kernel_Name'].split('(')[0][:36]:36s} dur {(e-s)/1000:7.1f} gap {((s-prev)/1000 if prev else 0):7.1f}")
    prev=e
PY
