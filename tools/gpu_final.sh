#!/bin/bash
# Round evidence: GPU suite, smoke(), the default bench line (as the driver runs it), and
# the rocprofv3 kernel-trace stats of the same command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/final_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k -- python3 bench.py --no-cpu-baseline --no-e2e > $O/bench_prof.log 2>&1
rc=$?
echo "chain exit $rc"
exit $rc
