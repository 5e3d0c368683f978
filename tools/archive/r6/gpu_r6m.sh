#!/bin/bash
# Round 6: the whole GPU suite and smoke() after the Net-pass clean-up (ring / fast / reg8 passes,
# lean levels and ablation macros removed) and the TCP end-of-capture flush; then C2-C4 bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6m}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for c in 2 3 4; do
  x=""; [ $c != 2 ] && x="--reset-each-step"
  timeout -k 10 300 python3 -u bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-e2e $x > $O/c$c.log 2>&1 || { tail -5 $O/c$c.log; exit 1; }
  echo "c$c: $(grep '^{' $O/c$c.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"], d["ms_per_step_median"])')"
done
echo done
