#!/bin/bash
# Round-1 evidence pass: e2e (host-memory) rate on C2/C3, stage ablation of the Net pass,
# FETCH_SIZE / WRITE_SIZE PMC passes for pv_net_kernel (separate runs, kernel-trace only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r1e
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
P="rocprofv3 --kernel-trace --output-format csv"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --e2e --read-ceiling > $O/c2_e2e.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --e2e --no-cpu-baseline --config 3 > $O/c3_e2e.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --e2e --no-cpu-baseline --config 4 --records 4000000 > $O/c4_e2e.log 2>&1 &&
(export PV_DEBUG_STAGES=1; timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_stage.log 2>&1) &&
(export PV_DEBUG_STAGES=2; timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_parse.log 2>&1) &&
timeout -s KILL 90 $P --pmc FETCH_SIZE -d $O/f -o k -- $B > $O/f.log 2>&1 &&
timeout -s KILL 90 $P --pmc WRITE_SIZE -d $O/w -o k -- $B > $O/w.log 2>&1
echo "chain exit $?"
