#!/bin/bash
# C5 (C4-shape stream from page-locked host memory) against the ingest chunk size, 30M records
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4_v; mkdir -p $O
for mb in 64 256 512; do
  echo "[$(date +%T)] chunk $mb MB"
  PV_INGEST_CHUNK_MB=$mb timeout -k 10 400 python3 -u bench.py --config 5 --stream-records 30000000 --steps 2 --warmup 1 \
    > $O/c5_$mb.log 2>&1 || { tail -5 $O/c5_$mb.log; exit 1; }
  tail -1 $O/c5_$mb.log | cut -c1-260
done
