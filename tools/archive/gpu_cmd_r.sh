#!/bin/bash
# the rest of the round-4 GPU tests, the BPF/TCP diagnostic, C3 bench + kernel stats, then the
# A/B variants (tacc / bkt / cbkt) on C3, C4, C2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export GRAFT_REPO_ROOT=$(pwd)
O=gpurun_out/r4_r; mkdir -p $O
echo "[$(date +%T)] tests"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bpf.py tests/test_gpu_psl.py tests/test_gpu_topn_bound.py \
  tests/test_gpu_dns2_sharded.py tests/test_gpu_concurrency.py -q --timeout 500 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -4 $O/tests.log
[ $rc -le 1 ] || exit $rc
echo "[$(date +%T)] diag"
timeout -k 10 300 python3 tools/bpf_tcp_diff.py > $O/bpf_tcp_diff.log 2>&1 || { tail -5 $O/bpf_tcp_diff.log; exit 1; }
head -30 $O/bpf_tcp_diff.log
BENCH="3" PROF="3" bash tools/gpu_r4.sh r || exit 1
TAG=r4r CFGS="3 4 2" VARS="tacc:tacc:- bkt:bkt:- cbkt:cbkt:-" bash tools/gpu_var.sh
