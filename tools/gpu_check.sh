#!/bin/bash
# GPU-box check of HEAD: smoke, GPU parity tests, default bench line, kernel-trace stats
# for C2/C3/C4. Every GPU step has its own limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/chk
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk/smoke.log 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/chk/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > gpurun_out/chk/bench_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chk/t2 -o c2 -- $B > gpurun_out/chk/trace_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chk/t3 -o c3 -- $B --config 3 > gpurun_out/chk/trace_c3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chk/t4 -o c4 -- $B --config 4 --records 4000000 > gpurun_out/chk/trace_c4.log 2>&1
rc=$?
echo "chain exit $rc"
exit $rc
