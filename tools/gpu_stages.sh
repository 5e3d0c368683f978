#!/bin/bash
# kernel time per pipeline stage (PV_DEBUG_STAGES) on C2 and C3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for cfg in 2 3; do
  for st in 1 2 4 0; do
    PV_DEBUG_STAGES=$st timeout -k 10 200 $B --config $cfg > gpurun_out/st_c${cfg}_$st.log 2>&1 || exit 1
  done
  timeout -k 10 200 $B --config $cfg --net-groups 1 --dns-groups 2 > gpurun_out/st_c${cfg}_ctr.log 2>&1 || exit 1
done
echo done
