#!/bin/bash
# Round 6 evidence B: the whole GPU suite and smoke() at HEAD, then the C2 bench line as the driver
# runs it (python bench.py: C2, CPU baseline, end-to-end rates).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6final}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -n 2 $O/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 2 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 1; }
grep '^{' $O/bench_c2.log | tail -1 | cut -c1-200
