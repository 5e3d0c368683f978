#!/bin/bash
# Iteration check: GPU parity tests, then kernel-trace stats of C2 / C3 / C4 benches.
# usage: gpu_iter.sh TAG  -> gpurun_out/it_TAG/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-x}
O=gpurun_out/it_$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
R="rocprofv3 --kernel-trace --stats --output-format csv"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 $R -d $O/c2 -o k -- $B > $O/c2.log 2>&1 &&
timeout -k 10 300 $R -d $O/c3 -o k -- $B --config 3 > $O/c3.log 2>&1 &&
timeout -k 10 300 $R -d $O/c4 -o k -- $B --config 4 --records 4000000 > $O/c4.log 2>&1
rc=$?
echo "chain exit $rc"
# staging floor and parse floor of the Net pass (kernel_ms in the bench line)
[ $rc -eq 0 ] && [ -n "$STAGES" ] && (export PV_DEBUG_STAGES=1; timeout -k 10 200 $B > $O/c2_stage.log 2>&1) && (export PV_DEBUG_STAGES=2; timeout -k 10 200 $B > $O/c2_parse.log 2>&1)
exit $rc
