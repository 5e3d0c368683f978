#!/bin/bash
# Round 5: GPU test subsets by name (default: TCP, KAT, BPF, windows), then the world-8 merge
# measurement with ranks sharing the GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5t}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_tcp.py tests/test_gpu_tcp_limit.py tests/test_gpu_kat.py tests/test_gpu_bpf.py tests/test_gpu_windows.py} \
  > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
if [ -n "$MERGE8" ]; then
  timeout -k 10 900 python3 -u tools/merge_world8.py --records ${MERGE8} > $O/merge_world8.log 2>&1 || { tail -30 $O/merge_world8.log; exit 1; }
  tail -2 $O/merge_world8.log
fi
echo done
