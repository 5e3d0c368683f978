#!/bin/bash
# Round-3 evidence: bench + rocprofv3 kernel stats of C2/C3/C4 and the PMC passes (HBM bytes,
# LDS, instruction mix) of the same three workloads, then the default bench line (with the
# CPU baseline and the end-to-end host-memory path) and C5 (100M-record stream from host
# memory, one GPU), each under its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PMC=1 PMC_CFGS="${PMC_CFGS:-2 3 4}" CFGS="2 3 4" bash tools/gpu_r3.sh ${PTAG:-final} || exit 1
O=gpurun_out/r3_${PTAG:-final}
echo "[$(date +%T)] bench default"
timeout -k 10 600 python3 bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
if [ "${C5:-1}" = 1 ]; then
  echo "[$(date +%T)] bench c5"
  timeout -k 10 900 python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
  tail -1 $O/bench_c5.log
fi
