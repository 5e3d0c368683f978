#!/bin/bash
# quick bench + kernel stats for C2/C3/C4 (run on the GPU box via gpurun)
set -o pipefail
mkdir -p gpurun_out/q
export TMPDIR=/tmp
for c in 2 3 4; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/q/bench_c$c.json 2> gpurun_out/q/bench_c$c.err || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/q/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/q/prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > /dev/null 2>&1 || exit 1
