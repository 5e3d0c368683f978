#!/bin/bash
# Round 5: PMC passes for C2-C4 (tools/gpu_pmc.sh), the C5 ingest chunk size A/B, and the TA /
# TCP counters of the C2 Net pass (tools/archive/gpu_r5n.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5o}; mkdir -p $O
export TMPDIR=/tmp
OUT=gpurun_out/r5_pmc bash tools/gpu_pmc.sh || exit 1
for mb in 128 256; do
  PV_INGEST_CHUNK_MB=$mb timeout -k 10 600 python3 -u bench.py --config 5 --steps 2 --warmup 1 > $O/c5_chunk$mb.log 2>&1 || { tail -20 $O/c5_chunk$mb.log; exit 1; }
  echo "chunk $mb: $(tail -1 $O/c5_chunk$mb.log | cut -c1-330)"
done
R5_DIR=r5n bash tools/archive/gpu_r5n.sh || exit 1
echo done
