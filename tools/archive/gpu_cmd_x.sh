#!/bin/bash
# device index rewrite: index tests, C5 at 30M (bench line, merge phase stamps, kernel stats)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_x; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_index.py tests/test_gpu_boundary.py > $O/tests.log 2>&1 || { tail -15 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u bench.py --config 5 --stream-records 30000000 --steps 1 --warmup 1 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ingest_ms'])"
PV_TSTAMPS=1 PVGPU_LIB=$R/pktvisor_amd/variants/libpvgpu_tst.so timeout -k 10 300 python3 -u bench.py --config 5 --stream-records 30000000 --steps 1 --warmup 0 > $O/c5_tst.log 2>&1 || { tail -5 $O/c5_tst.log; exit 1; }
grep pv_tstamps $O/c5_tst.log | tail -3 | cut -c1-400
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k -- python3 $R/bench.py --config 5 --stream-records 30000000 --steps 1 --warmup 0 > $O/prof.log 2>&1) || { tail -5 $O/prof.log; exit 1; }
python3 tools/kstats.py $O/prof | cut -c1-300
