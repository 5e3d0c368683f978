#!/bin/bash
# Iteration check with DNS attribution: GPU parity tests, C2/C3/C4 kernel stats, then
# C3 with no DNS table updates (knob 32) and with neither names nor tables (knob 48).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-x}
O=gpurun_out/it_$T
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
R="rocprofv3 --kernel-trace --stats --output-format csv"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 $R -d $O/c2 -o k -- $B > $O/c2.log 2>&1 &&
timeout -k 10 300 $R -d $O/c3 -o k -- $B --config 3 > $O/c3.log 2>&1 &&
timeout -k 10 300 $R -d $O/c4 -o k -- $B --config 4 --records 4000000 > $O/c4.log 2>&1 &&
(export PV_DEBUG_STAGES=32; timeout -k 10 300 $R -d $O/c3_notab -o k -- $B --config 3 > $O/c3_notab.log 2>&1) &&
(export PV_DEBUG_STAGES=48; timeout -k 10 300 $R -d $O/c3_none -o k -- $B --config 3 > $O/c3_none.log 2>&1)
rc=$?
echo "chain exit $rc"
exit $rc
