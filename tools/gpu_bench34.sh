#!/bin/bash
# clean (unprofiled) bench lines of C3 and C4, each under its own time limit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3_${PTAG:-final}; mkdir -p $O
for c in 3 4; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-e2e > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  tail -1 $O/bench_c$c.log
done
