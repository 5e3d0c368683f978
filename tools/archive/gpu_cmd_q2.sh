#!/bin/bash
# A/B of the DNS decode accessor (tacc: the HBM-backed window everywhere) and the bucketed key
# cache (bkt), C3/C4/C2 kernel stats; then the sharded DNS v2 and concurrency tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export GRAFT_REPO_ROOT=$(pwd)
TAG=r4q CFGS="3 4 2" VARS="tacc:tacc:- bkt:bkt:- cbkt:cbkt:-" bash tools/gpu_var.sh || exit 1
O=gpurun_out/r4_q2; mkdir -p $O
echo "[$(date +%T)] new tests"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_dns2_sharded.py tests/test_gpu_concurrency.py -q --timeout 500 \
  --timeout-method thread -p no:cacheprovider > $O/tests_new.log 2>&1
rc=$?
tail -5 $O/tests_new.log
exit $rc
