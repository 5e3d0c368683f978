#!/bin/bash
# One GPU box call: the whole -m gpu suite (every failure listed), smoke(), then the C2 bench line
# and rocprofv3 kernel stats of C2/C3/C4 (tools/gpu_r3.sh). Stops at a time limit / abort / fault.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-check}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 ${SUITE_TIMEOUT:-700} python3 -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -12 $O/tests.log
case $rc in 0|1) ;; *) echo "suite ended with $rc: stopping"; exit $rc;; esac
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
[ "${BENCH:-1}" = 1 ] && { bash tools/gpu_r3.sh $TAG || exit 1; }
exit $rc
