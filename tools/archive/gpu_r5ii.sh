#!/bin/bash
# Round 5: fills + parameter block in one launch vs two (PV_FILL_FUSE=0), C3 and C2, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5ii}; mkdir -p $O
export TMPDIR=/tmp
for cfg in 3 2; do
for k in 1 2; do
  for f in 1 0; do
    PV_FILL_FUSE=$f timeout -k 10 400 python3 -u bench.py --config $cfg --no-e2e --no-cpu-baseline > $O/c${cfg}_f${f}_$k.log 2>&1 || { tail -20 $O/c${cfg}_f${f}_$k.log; exit 1; }
    echo "C$cfg fuse=$f: $(grep '^{' $O/c${cfg}_f${f}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], d["ms_per_step_median"], r["kernel_ms"])')"
  done
done
done
echo done
