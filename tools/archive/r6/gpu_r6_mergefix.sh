#!/bin/bash
# pv_topn_merge without device calls (every run key on the LDS path; entries past the new-name
# list named by pv_topn_name_fix): the whole GPU suite, then C2-C4 kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6mergefix; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -20 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
for c in 2 3 4; do
  x=""; [ $c != 2 ] && x="--reset-each-step"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 -u bench.py --config $c --steps 10 --warmup 2 --no-e2e --no-cpu-baseline $x > $O/prof_c$c.log 2>&1 || { tail -5 $O/prof_c$c.log; exit 1; }
  f=$(find $O/prof_c$c -name '*kernel_stats.csv' | head -1); cp $f $O/c${c}_kernel_stats.csv
  grep -E 'pv_topn_merge' $O/c${c}_kernel_stats.csv | cut -d, -f1-4
done
