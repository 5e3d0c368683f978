#!/bin/bash
# LDS-only DNS decode + key list in place + carried-list hand-over: the transaction-stage and
# full-size GPU tests, then the C3 bench line and kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TESTS="tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dns2.py tests/test_gpu_windows.py tests/test_gpu_tcp.py tests/test_gpu_dnstap.py tests/test_gpu_bpf.py tests/test_gpu_psl.py tests/test_gpu_topn_bound.py" \
  BENCH="3" PROF="3" bash tools/gpu_r4.sh q1
