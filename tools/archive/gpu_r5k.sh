#!/bin/bash
# Round 5: the multi-GPU merge paths (sharded parity tests) after the candidate / selection
# rewrites, then the world-8 merge measurement with per-step times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5k}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_windows.py tests/test_gpu_dist.py tests/test_gpu_dns2_sharded.py tests/test_gpu_topn_bound.py tests/test_gpu_rccl.py \
  > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 -u tools/merge_world8.py --records 100000000 > $O/merge_world8.log 2>&1 || { tail -30 $O/merge_world8.log; exit 1; }
grep merge_world8 $O/merge_world8.log
echo done
