#!/bin/bash
# pv_topn_names without device calls (suffix sizes in their own instance, pv_topn_names_sfx):
# parity / PSL / filter GPU tests, C3 and C4 bench lines, rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6names; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_psl.py tests/test_gpu_filters.py tests/test_gpu_topn_bound.py tests/test_gpu_dns2.py > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -20 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
for c in 3 4; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 40 --warmup 3 --no-e2e --no-cpu-baseline --reset-each-step > $O/bench_c$c.log 2>&1 || { tail -5 $O/bench_c$c.log; exit 1; }
  echo "c$c $(grep '^{' $O/bench_c$c.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 -u bench.py --config $c --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --reset-each-step > $O/prof_c$c.log 2>&1 || { tail -5 $O/prof_c$c.log; exit 1; }
  f=$(find $O/prof_c$c -name '*kernel_stats.csv' | head -1); cp $f $O/c${c}_kernel_stats.csv
  grep -E 'pv_topn_names|pv_xact_resolve|pv_dns_kernel' $O/c${c}_kernel_stats.csv | cut -d, -f1-4
done
