#!/bin/bash
# C5 30M traces (kernels + copies) at chunk 64 / ring 6 and chunk 128 / ring 4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_z; mkdir -p $O
for cfg in "64 6" "128 4"; do
  set -- $cfg
  (cd /tmp && PV_INGEST_CHUNK_MB=$1 PV_INGEST_RING=$2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_$1_$2 -o k -- python3 $R/bench.py --config 5 --stream-records 30000000 --steps 1 --warmup 0 > $O/prof_$1_$2.log 2>&1) || { tail -5 $O/prof_$1_$2.log; exit 1; }
  tail -1 $O/prof_$1_$2.log | cut -c1-200
done
