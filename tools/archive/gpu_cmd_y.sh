#!/bin/bash
# ingest ring depth and chunk size on C5 (30M records)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_y; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_index.py > $O/tests.log 2>&1 || { tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "64 3" "64 4" "64 6" "128 4" "256 4" "256 6"; do
  set -- $cfg
  PV_INGEST_CHUNK_MB=$1 PV_INGEST_RING=$2 timeout -k 10 300 python3 -u bench.py --config 5 --stream-records 30000000 --steps 2 --warmup 1 > $O/c5_$1_$2.log 2>&1 || { tail -5 $O/c5_$1_$2.log; exit 1; }
  echo -n "chunk $1 ring $2: "; tail -1 $O/c5_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ingest_ms'])"
done
