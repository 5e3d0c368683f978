#!/bin/bash
# kernel-trace stats for C2/C3/C4 bench commands (round-2 profiles)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/prof2}
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e"
for c in 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c$c -o c$c -- $B --config $c > $OUT/trace_c$c.log 2>&1 || exit 1
done
