#!/bin/bash
# merge direct-region threshold (PV_MERGE_DIRECT 64 / 256 / 1024): parity with 1024, then C5 30M and C4 10M
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_dir; mkdir -p $O
PVGPU_LIB=$R/pktvisor_amd/variants/libpvgpu_d1024.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_topn_bound.py tests/test_gpu_windows.py > $O/tests.log 2>&1 || { tail -25 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in main d256 d1024; do
  L=$R/pktvisor_amd/libpvgpu.so; [ $v = main ] || L=$R/pktvisor_amd/variants/libpvgpu_$v.so
  PVGPU_LIB=$L timeout -k 10 300 python3 -u bench.py --config 5 --stream-records 30000000 --steps 2 --warmup 1 > $O/c5_$v.log 2>&1 || { tail -5 $O/c5_$v.log; exit 1; }
  echo -n "$v c5: "; tail -1 $O/c5_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ingest_ms'])"
  PVGPU_LIB=$L timeout -k 10 300 python3 -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/c4_$v.log 2>&1 || { tail -5 $O/c4_$v.log; exit 1; }
  echo -n "$v c4: "; tail -1 $O/c4_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
