#!/bin/bash
# C5 30M: pair-stage host marks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_hp3; mkdir -p $O
for cfg in "64 6"; do
  set -- $cfg
  PV_HOST_PROF=1 PV_INGEST_CHUNK_MB=$1 PV_INGEST_RING=$2 timeout -k 10 300 python3 -u bench.py --config 5 --stream-records 30000000 --steps 1 --warmup 1 > $O/c5_$1_$2.log 2>&1 || { tail -5 $O/c5_$1_$2.log; exit 1; }
  echo "chunk $1 ring $2"; grep pv_hostprof $O/c5_$1_$2.log; tail -1 $O/c5_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ingest_ms'])"
done
