#!/bin/bash
# public_suffix_list session: the GPU suite (incl. tests/test_gpu_psl.py), the default bench line and
# C3 kernel stats (the DNS pass's cost after the SFX split)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/psl; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --config 3 > $O/prof_c3.log 2>&1
rc=$?; echo "chain exit $rc"; exit $rc
