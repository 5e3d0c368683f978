#!/bin/bash
# Round-3 iteration on one GPU box: optional test files, the C2 bench line, rocprofv3 kernel
# stats of C2/C3/C4 and (PMC=1) the C2 LDS / memory counter passes. Every GPU step has its own
# time limit and the chain stops at the first failure.
#   bash tools/gpu_r3.sh TAG [pytest targets...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
TAG=${1:-x}; shift
O=$R/gpurun_out/r3_$TAG
mkdir -p $O
export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-e2e"
step() { echo "[$(date +%T)] $*"; }
if [ $# -gt 0 ]; then
  step tests "$@"
  timeout -k 10 900 python3 -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
step bench c2
timeout -k 10 300 python3 $B > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log
for c in ${CFGS:-2 3 4}; do
  step prof c$c
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 $B --steps 10 --config $c > $O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
  python3 tools/kstats.py $O/prof_c$c 2>/dev/null | head -12
done
if [ "${PMC:-0}" = 1 ]; then
  step pmc
  OUT=gpurun_out/r3_$TAG/pmc CFGS="${PMC_CFGS:-2}" bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
  for c in ${PMC_CFGS:-2}; do python3 tools/pmc_summary.py $O/pmc $c > $O/pmc_c$c.json; done
fi
step done
