#!/bin/bash
# Round-4 evidence, part 2: the C5 line (100M-record stream from page-locked host memory, 1 GPU)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_ev; mkdir -p $O
echo "[$(date +%T)] bench c5"
timeout -k 10 1000 python3 -u bench.py --config 5 --steps 2 --warmup 1 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | cut -c1-500
