#!/bin/bash
# quick perf check: C2 default, C3, C4 (kernel ms), plus GPU parity tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 $B > gpurun_out/q_c2.log 2>&1 &&
timeout -k 10 200 $B --config 3 > gpurun_out/q_c3.log 2>&1 &&
timeout -k 10 200 $B --config 4 --records 4000000 > gpurun_out/q_c4.log 2>&1
echo "chain exit $?"
