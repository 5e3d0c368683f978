#!/bin/bash
# Round 5: C3 bench repeatability (three runs on one box).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5hh}; mkdir -p $O
export TMPDIR=/tmp
for k in 1 2 3; do
  timeout -k 10 400 python3 -u bench.py --config 3 --no-e2e --no-cpu-baseline > $O/bench_c3_$k.log 2>&1 || { tail -20 $O/bench_c3_$k.log; exit 1; }
  grep '^{' $O/bench_c3_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], d["ms_per_step_median"], r["kernel_ms"])'
done
echo done
