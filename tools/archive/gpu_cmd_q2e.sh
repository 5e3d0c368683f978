#!/bin/bash
# A/B variants (C3/C4/C2 kernel stats), the new multi-rank and concurrency tests, then the
# evidence benches (smoke, default C2 line, C3 / C4 lines with CPU baselines)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_cmd_q2.sh; rc=$?
[ $rc -le 1 ] || exit $rc
bash tools/gpu_cmd_ev1.sh
