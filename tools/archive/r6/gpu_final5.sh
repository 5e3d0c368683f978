#!/bin/bash
# Round-5 final evidence on HEAD: GPU suite, smoke, bench lines C2-C4 (with CPU baselines), C5 at
# 100M, kernel stats C2-C4 and C5 (30M). Every GPU step has its own limit; the chain stops at the
# first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${FIN_DIR:-r5_fin}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step tests
# (no -x: every failure at once; a failing test does not stop the evidence below, a hang or a
# crash of the suite does)
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
trc=$?
tail -1 $O/gpu_tests.log
grep -E "^(FAILED|ERROR)" $O/gpu_tests.log | head -20
[ $trc -le 1 ] || exit 1
step smoke
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in 2 3 4; do
  step bench c$c
  F="--no-e2e"; [ $c = 2 ] && F=""
  timeout -k 10 400 python3 -u bench.py --config $c $F > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  tail -1 $O/bench_c$c.log | cut -c1-300
done
step bench c5
timeout -k 10 600 python3 -u bench.py --config 5 --steps 2 --warmup 1 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | cut -c1-400
for c in 2 3 4; do
  step prof c$c
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c > $O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
  python3 tools/kstats.py $O/prof_c$c 2>/dev/null | cut -c1-300
done
step prof c5
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o k -- python3 $R/bench.py --config 5 --stream-records 30000000 --steps 1 --warmup 1 > $O/prof_c5.log 2>&1) || { tail -20 $O/prof_c5.log; exit 1; }
python3 tools/kstats.py $O/prof_c5 2>/dev/null | cut -c1-300
step done
[ $trc -eq 0 ] || exit 1
