#!/bin/bash
# key list written by the DNS pass + carried-list hand-over: GPU tests of the transaction stage,
# C3 bench + kernel stats, the sharded DNS v2 tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4_o
TESTS="tests/test_gpu_parity.py tests/test_gpu_dns2.py tests/test_gpu_windows.py tests/test_gpu_tcp.py tests/test_gpu_dnstap.py" \
  BENCH="3" PROF="3" bash tools/gpu_r4.sh o || exit 1
echo "[$(date +%T)] new tests"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dns2_sharded.py tests/test_gpu_concurrency.py -q --timeout 500 \
  --timeout-method thread -p no:cacheprovider > $O/tests_new.log 2>&1
rc=$?
tail -5 $O/tests_new.log
# test failures (1) leave the GPU usable; anything else ends the call here
exit $rc
