#!/bin/bash
# pv_net_slow_list without a device call (the general path inlined): Net parity / variants / bench
# shape GPU tests, then C2 and C3 bench lines and rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6slowlist; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_net_variants.py tests/test_gpu_bench_shape.py tests/test_gpu_kat.py tests/test_gpu_tcp.py > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -20 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --steps 100 --no-e2e --no-cpu-baseline > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 1; }
echo "c2 $(grep '^{' $O/bench_c2.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
for c in 2 3; do
  x=""; [ $c != 2 ] && x="--reset-each-step"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 -u bench.py --config $c --steps 10 --warmup 2 --no-e2e --no-cpu-baseline $x > $O/prof_c$c.log 2>&1 || { tail -5 $O/prof_c$c.log; exit 1; }
  f=$(find $O/prof_c$c -name '*kernel_stats.csv' | head -1); cp $f $O/c${c}_kernel_stats.csv
  grep -E 'pv_net' $O/c${c}_kernel_stats.csv | cut -d, -f1-4
done
