#!/bin/bash
# The pending-name path of the merge (new-name list overflow): the top-N bound tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6namefix; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_topn_bound.py > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -n 3 $O/gpu_tests.log
