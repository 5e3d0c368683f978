#!/bin/bash
# Round 5: the Net-pass variants' parity (one process each), smoke, bench C5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5ff}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_net_variants.py > $O/tests.log 2>&1
trc=$?
tail -1 $O/tests.log; grep -E "^(FAILED|ERROR)|MISMATCH|kernels:" $O/tests.log | head -20
[ $trc -le 1 ] || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u bench.py --config 5 --steps 2 --warmup 1 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | cut -c1-300
echo done
