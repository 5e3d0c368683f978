#!/bin/bash
# The transaction stage's single read-back: DNS / TCP / window GPU tests, then C4 and C3 bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6ovf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_topn_bound.py tests/test_gpu_windows.py tests/test_gpu_dns2.py tests/test_gpu_tcp.py tests/test_gpu_bench_shape.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -n 2 $O/gpu_tests.log
for c in 4 3; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 40 --warmup 3 --no-e2e --no-cpu-baseline --reset-each-step > $O/bench_c$c.log 2>&1 || { tail -5 $O/bench_c$c.log; exit 1; }
  grep '^{' $O/bench_c$c.log | tail -1 | cut -c1-200
done
