#!/bin/bash
# Round-4 evidence, part 1: smoke, the default bench line (C2 + cpu_baseline + e2e), C3 and C4
# bench lines with their CPU baselines, kernel stats of C2/C3/C4 (each step under its own limit)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r4_ev; mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step bench default
timeout -k 10 400 python3 bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-400
for c in 3 4; do
  step bench c$c
  timeout -k 10 400 python3 bench.py --config $c --no-e2e > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  tail -1 $O/bench_c$c.log | cut -c1-300
done
for c in 2 3 4; do
  step prof c$c
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c > $O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
  python3 tools/kstats.py $O/prof_c$c | cut -c1-240
done
step done
