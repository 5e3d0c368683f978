#!/bin/bash
# Round 6: status read-back waited for by polling an event vs a blocking stream synchronisation,
# C2 alternating twice on one box, C3 once each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6x}; mkdir -p $O
run() { # name cfg env...
  local n=$1 c=$2; shift 2
  local x=""; [ $c != 2 ] && x="--reset-each-step"
  env "$@" timeout -k 10 300 python3 -u bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-e2e $x > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel_ms"], d["ms_per_step"], d["ms_per_step_median"])')"
}
for k in 1 2 3; do
  run c2_spin_$k 2 PV_X=1
  run c2_block_$k 2 PV_SYNC=block
done
run c3_spin 3 PV_X=1
run c3_block 3 PV_SYNC=block
