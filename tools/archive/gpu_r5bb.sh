#!/bin/bash
# Round 5: bench lines C2 / C3 / C4 with the Net pass's 80-B header-window bytes rule.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5bb}; mkdir -p $O
export TMPDIR=/tmp
for c in 2 3 4; do
  F="--no-e2e"; [ $c = 2 ] && F=""
  timeout -k 10 400 python3 -u bench.py --config $c $F > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  grep '^{' $O/bench_c$c.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["config"]["workload"][:3], d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], r["bytes_per_launch"], r["step_frac"], d["cpu_baseline"]["value"])'
done
echo done
