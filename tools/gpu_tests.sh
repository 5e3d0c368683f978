#!/bin/bash
# GPU test suite only
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/t_${1:-x}
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
echo "chain exit $rc"
exit $rc
