#!/bin/bash
# DNS pass cost split on C3: PV_DEBUG_STAGES knobs (16: no name decode, 32: no table updates)
set -o pipefail
mkdir -p gpurun_out/dbg
for d in 0 16 32 48; do
  PV_DEBUG_STAGES=$d timeout -k 10 200 python bench.py --config ${CFG:-3} --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/dbg/c${CFG:-3}_d$d.json 2>/dev/null || true
  cd /tmp && PV_DEBUG_STAGES=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dbg/p$d -o s -- python3 $GRAFT_REPO_ROOT/bench.py --config ${CFG:-3} --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > /dev/null 2>&1; cd $GRAFT_REPO_ROOT
  f=$(find gpurun_out/dbg/p$d -name "*kernel_stats.csv" | head -1)
  echo "== d$d"; grep -E "pv_dns_kernel|pv_topn|pv_net" $f | cut -d, -f1,4
done
