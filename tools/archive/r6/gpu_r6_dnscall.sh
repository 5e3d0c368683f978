#!/bin/bash
# DNS pass without device-function calls (cache path only, top_ecs listed for pv_dns_ecs, the
# cache flush inlined): DNS GPU tests, then HEAD build vs this one, C3 / C4 bench lines and
# rocprofv3 kernel stats of C3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6dnscall; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_contract.py tests/test_gpu_parity.py tests/test_gpu_dns2.py tests/test_gpu_boundary.py tests/test_gpu_deep_sampling.py tests/test_gpu_psl.py > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -20 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
for v in head main; do
  if [ $v = main ]; then L=$R/pktvisor_amd/libpvgpu.so; else L=$R/pktvisor_amd/variants/libpvgpu_$v.so; fi
  for c in 3 4; do
    PVGPU_LIB=$L timeout -k 10 300 python3 -u bench.py --config $c --steps 30 --warmup 3 --no-e2e --no-cpu-baseline --reset-each-step > $O/bench_c${c}_$v.log 2>&1 || { tail -5 $O/bench_c${c}_$v.log; exit 1; }
    echo "$v c$c $(grep '^{' $O/bench_c${c}_$v.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  done
  PVGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o k -- python3 -u bench.py --config 3 --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --reset-each-step > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; exit 1; }
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -1); cp $f $O/c3_kernel_stats_$v.csv
  grep -E '"pv_dns_kernel"|pv_dns_kernel,' $O/c3_kernel_stats_$v.csv | cut -d, -f1-6
done
