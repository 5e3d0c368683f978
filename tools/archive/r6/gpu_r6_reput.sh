#!/bin/bash
# Exact LRU replay with the close flush's re-puts: the TCP limit / TCP / KAT GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6reput; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tcp_limit.py tests/test_gpu_tcp.py tests/test_gpu_kat.py > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; tail -30 $O/gpu_tests.log; exit 1; }
tail -n 2 $O/gpu_tests.log
