#!/bin/bash
# The whole -m gpu suite without -x (every failure listed), then optional follow-up script(s)
# unless the suite ended by a time limit, abort or fault.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-suite}; mkdir -p $O
timeout -k 10 ${SUITE_TIMEOUT:-900} python3 -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -15 $O/tests.log
case $rc in 0|1) ;; *) echo "suite ended with $rc: stopping"; exit $rc;; esac
for s in "$@"; do bash $s || exit 1; done
exit $rc
