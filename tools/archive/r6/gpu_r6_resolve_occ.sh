#!/bin/bash
# The v1 resolve's occupancy: dynamic LDS padding per workgroup on C4, rocprofv3 (two runs: 0 / 20 / 40 KiB,
# then 30 / 80 / 40 KiB; the padding came from PV_RESOLVE_LDS, a probe knob since replaced by PV_RESOLVE_PAD)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6resolve_occ; mkdir -p $O
export TMPDIR=/tmp
for l in 30000 80000 40960; do
  PV_RESOLVE_LDS=$l timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$l -o k -- python3 -u bench.py --config 4 --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --reset-each-step > $O/prof_$l.log 2>&1 || { tail -5 $O/prof_$l.log; exit 1; }
  f=$(find $O/prof_$l -name '*kernel_stats.csv' | head -1); cp $f $O/c4_kernel_stats_$l.csv
  echo "lds $l: $(grep -E 'pv_xact_resolve' $O/c4_kernel_stats_$l.csv | cut -d, -f1-4)"
done
