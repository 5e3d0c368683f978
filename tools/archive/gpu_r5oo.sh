#!/bin/bash
# Round 5: grid ranges per CU (PV_NET_WGCU: the batch's partition for the DNS pass, combine and
# merge) on C2 / C3 / C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5oo}; mkdir -p $O
export TMPDIR=/tmp
for cfg in ${CFGS:-2 3 4}; do
  for g in 2 3 4; do
    PV_NET_WGCU=$g timeout -k 10 400 python3 -u bench.py --config $cfg --no-e2e --no-cpu-baseline > $O/c${cfg}_g$g.log 2>&1 || { tail -20 $O/c${cfg}_g$g.log; exit 1; }
    echo "C$cfg wgcu=$g: $(grep '^{' $O/c${cfg}_g$g.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_step_median"], d["roofline"]["kernel_ms"])')"
  done
done
echo done
