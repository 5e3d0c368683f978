#!/bin/bash
# The DNS v1 resolve without device calls (slow transactions listed for pv_xact_slow_dev, the v2
# accounting in its own kernel): transaction / window / v2 / sharded GPU tests, C4 bench line and
# rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6resolve; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_windows.py tests/test_gpu_dns2.py tests/test_gpu_dns2_sharded.py tests/test_gpu_dist.py tests/test_gpu_bench_shape.py tests/test_gpu_topn_bound.py tests/test_gpu_tcp.py tests/test_gpu_v2_outputs.py > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -20 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --config 4 --steps 40 --warmup 3 --no-e2e --no-cpu-baseline --reset-each-step > $O/bench_c4.log 2>&1 || { tail -5 $O/bench_c4.log; exit 1; }
grep '^{' $O/bench_c4.log | tail -1 | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o k -- python3 -u bench.py --config 4 --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --reset-each-step > $O/prof_c4.log 2>&1 || { tail -5 $O/prof_c4.log; exit 1; }
f=$(find $O/prof_c4 -name '*kernel_stats.csv' | head -1); cp $f $O/c4_kernel_stats.csv
grep -E 'pv_xact|pv_dns_kernel' $O/c4_kernel_stats.csv | cut -d, -f1-5
