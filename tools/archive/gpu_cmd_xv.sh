#!/bin/bash
# value buffer growth: transaction parity tests, then C5 at 100M and 30M
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_xv; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_windows.py tests/test_gpu_dns2.py tests/test_gpu_v2_outputs.py tests/test_gpu_dns2_sharded.py tests/test_gpu_boundary.py > $O/tests.log 2>&1 || { tail -25 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 -u bench.py --config 5 --steps 2 --warmup 1 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('100M', d['value'], d['ms_per_step'], d['ingest_ms'])"
PV_HOST_PROF=1 timeout -k 10 300 python3 -u bench.py --config 5 --stream-records 30000000 --steps 2 --warmup 1 > $O/c5_30m.log 2>&1 || { tail -5 $O/c5_30m.log; exit 1; }
grep pv_hostprof $O/c5_30m.log; tail -1 $O/c5_30m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('30M', d['value'], d['ms_per_step'], d['ingest_ms'])"
