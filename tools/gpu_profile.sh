#!/bin/bash
# Round profile: default bench line (with cpu_baseline), rocprofv3 kernel-trace stats,
# and separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the same C2 command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --read-ceiling > gpurun_out/prof/bench_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o c2 -- $B > gpurun_out/prof/trace_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o c2 -- $B > gpurun_out/prof/fetch_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d gpurun_out/prof/write -o c2 -- $B > gpurun_out/prof/write_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace3 -o c3 -- $B --config 3 > gpurun_out/prof/trace_c3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace4 -o c4 -- $B --config 4 --records 4000000 > gpurun_out/prof/trace_c4.log 2>&1
echo "exit $?"
