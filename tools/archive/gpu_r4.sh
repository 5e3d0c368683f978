#!/bin/bash
# Round-4 iteration on one GPU box. Every GPU step has its own time limit and the chain stops
# at the first failure.
#   PROBE=1 : tools/ring_probe (Net-pass staging variants)
#   TESTS="tests/x.py ..." : GPU tests first
#   BENCH="2 3 4" : bench lines (CPU=1 adds cpu_baseline, E2E=1 the host-memory path)
#   PROF="2 3 4" : rocprofv3 kernel stats per config
#   PMC="2" : PMC passes (tools/gpu_pmc.sh) per config
#   bash tools/gpu_r4.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
TAG=${1:-x}
O=$R/gpurun_out/r4_$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
if [ "${PROBE:-0}" = 1 ]; then
  step probe
  timeout -k 10 180 ./tools/ring_probe > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
  cat $O/probe.log
fi
if [ -n "$TESTS" ]; then
  step tests $TESTS
  timeout -k 10 900 python3 -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
for c in $BENCH; do
  F="--no-e2e"; [ "${E2E:-0}" = 1 ] && [ $c = 2 ] && F=""
  [ "${CPU:-0}" = 1 ] || F="$F --no-cpu-baseline"
  step bench c$c
  timeout -k 10 300 python3 $R/bench.py --config $c $F $BENCH_ARGS > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  tail -1 $O/bench_c$c.log
done
for c in $PROF; do
  step prof c$c
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c > $O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
  python3 tools/kstats.py $O/prof_c$c 2>/dev/null | head -12
done
if [ -n "$PMC" ]; then
  step pmc $PMC
  OUT=gpurun_out/r4_$TAG/pmc CFGS="$PMC" bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
  for c in $PMC; do python3 tools/pmc_summary.py $O/pmc $c > $O/pmc_c$c.json; done
fi
step done
