#!/bin/bash
# Round 6: kernel stats of C2 (accumulate), C3 and C4 (reset each step) on HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6n}; mkdir -p $O
export TMPDIR=/tmp
for c in 2 3 4; do
  x=""; [ $c != 2 ] && x="--reset-each-step"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c $x > $O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
  echo "c$c $(python3 tools/kstats.py $O/prof_c$c 2>/dev/null | cut -c1-600)"
done
