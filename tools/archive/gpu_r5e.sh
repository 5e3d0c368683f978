#!/bin/bash
# Round 5: sharded merges through the device top-N exchange and the distributed selection.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5e}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bpf.py tests/test_gpu_dist.py tests/test_gpu_windows.py tests/test_gpu_dns2_sharded.py tests/test_gpu_rccl.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -30; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
step bench c2
timeout -k 10 300 python3 -u bench.py --config 2 --no-cpu-baseline --no-e2e > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-200
step done
