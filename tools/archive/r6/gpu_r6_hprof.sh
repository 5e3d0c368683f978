#!/bin/bash
# Host-side time split of the bench step (PV_HOST_PROF: pv_destroy prints the per-phase sums)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6hprof; mkdir -p $O
export TMPDIR=/tmp PV_HOST_PROF=1
timeout -k 10 300 python3 -u bench.py --steps 200 --no-cpu-baseline --no-e2e > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
grep -E '^\{|hostprof' $O/c2.log | cut -c1-400
timeout -k 10 300 python3 -u bench.py --config 4 --steps 40 --warmup 3 --no-e2e --no-cpu-baseline --reset-each-step > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
grep -E '^\{|hostprof' $O/c4.log | cut -c1-400
