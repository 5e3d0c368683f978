#!/bin/bash
# GPU parity tests, then the host-memory (e2e) rates on C2/C3/C4 next to the
# device-resident bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/e2e_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --config 3 > $O/c3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --config 4 --records 4000000 > $O/c4.log 2>&1
rc=$?
echo "chain exit $rc"
exit $rc
