#!/bin/bash
# Per-kernel attribution on C2 and C3: stage knobs (PV_DEBUG_STAGES 1 = staging only,
# 2 = parse + counters) and metric-group ablations, each under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
R="rocprofv3 --kernel-trace --stats --output-format csv"
run() { # name, env, args
  local nm=$1; shift
  ( export PV_DEBUG_STAGES=$1; timeout -k 10 200 $R -d gpurun_out/abl/$nm -o k -- $B "${@:2}" > gpurun_out/abl/$nm.log 2>&1 )
}
run c2_stage 1 --config 2 &&
run c2_parse 2 --config 2 &&
run c2_ctr 0 --config 2 --net-groups 1 --dns-groups 2 &&
run c2_card 0 --config 2 --net-groups 3 --dns-groups 2 &&
run c2_top 0 --config 2 --net-groups 9 --dns-groups 2 &&
run c3_ctr 0 --config 3 --net-groups 1 --dns-groups 2 &&
run c3_card 0 --config 3 --net-groups 1 --dns-groups 3 &&
run c3_qn 0 --config 3 --net-groups 1 --dns-groups 66 &&
run c3_xact 0 --config 3 --net-groups 1 --dns-groups 18
echo "chain exit $?"
