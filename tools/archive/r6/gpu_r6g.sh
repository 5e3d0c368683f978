#!/bin/bash
# Round 6: the whole GPU suite on the depth-3 unconditional-load Net pass with non-temporal merge
# write-back (plus the bench-shape tests), then smoke.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6g}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
trc=$?
tail -3 $O/gpu_tests.log
grep -E "^(FAILED|ERROR)" $O/gpu_tests.log | head -20
[ $trc -le 1 ] || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
[ $trc -eq 0 ] || exit 1
