#!/bin/bash
# Round-2 evidence on the current tree: the GPU suite, smoke(), the default bench line (as
# the driver runs it), rocprofv3 kernel-trace stats of the C2/C3/C4 benches, and the C2
# FETCH_SIZE / WRITE_SIZE passes (separate runs) for the roofline's traffic figure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2f_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-e2e"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o k -- $B > $O/prof_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o k -- $B --config 3 > $O/prof_c3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o k -- $B --config 4 > $O/prof_c4.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/pmc_f -o k -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/pmc_f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/pmc_w -o k -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/pmc_w.log 2>&1
rc=$?
echo "chain exit $rc"
exit $rc
