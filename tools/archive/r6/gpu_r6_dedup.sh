#!/bin/bash
# The combine's wave-level key dedup of IP-log inserts (PV_CB_DEDUP distinct keys an insert):
# 0 / 3 (product) / 6, C2 bench line and rocprofv3 kernel stats, then the parity tests at 3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6dedup; mkdir -p $O
export TMPDIR=/tmp
for v in dd0 main dd6; do
  if [ $v = main ]; then L=$R/pktvisor_amd/libpvgpu.so; else L=$R/pktvisor_amd/variants/libpvgpu_$v.so; fi
  PVGPU_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 100 --no-e2e --no-cpu-baseline > $O/bench_c2_$v.log 2>&1 || { tail -5 $O/bench_c2_$v.log; exit 1; }
  echo "$v c2 $(grep '^{' $O/bench_c2_$v.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  PVGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o k -- python3 -u bench.py --steps 10 --warmup 2 --no-e2e --no-cpu-baseline > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -1); cp $f $O/c2_kernel_stats_$v.csv
  grep -E 'pv_topn_combine|pv_topn_merge' $O/c2_kernel_stats_$v.csv | cut -d, -f1-4
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_shape.py tests/test_gpu_topn_bound.py tests/test_gpu_net2.py > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -20 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
