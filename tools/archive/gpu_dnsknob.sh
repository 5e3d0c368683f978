#!/bin/bash
# C3 DNS-pass attribution by runtime profiling knobs (PV_DEBUG_STAGES bits, pv_kernels.hip
# dns_process): 16 no name statistics, 32 no table updates, 256 no LDS key cache, 512 no qname
# CPC, 1024 no transaction events. Kernel stats per setting under gpurun_out/r4_knob/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/r4_knob
mkdir -p $O
export TMPDIR=/tmp
for k in ${KNOBS:-0 16 32 256 512 1024 48}; do
  echo "[$(date +%T)] knob $k"
  (cd /tmp && PV_DEBUG_STAGES=$k timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$k -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 --config ${CFG:-3} > $O/k$k.log 2>&1) || { tail -5 $O/k$k.log; echo "knob $k: rc $?"; }
  python3 tools/kstats.py $O/k$k 2>/dev/null | grep -E "pv_dns_kernel|pv_topn|pv_xact" | head -6
done
