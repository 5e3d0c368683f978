#!/bin/bash
# Round 5: grid ranges per top-N combine workgroup (PV_CB_FAN) on C2 / C3: kernel statistics of
# combine and merge per setting, and the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5w}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for cfg in ${CFGS:-2 3}; do
  for fan in ${FANS:-1 2 3 4}; do
    n=c${cfg}_fan$fan
    PV_CB_FAN=$fan timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $R/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
    f=$(find $O/$n -name '*kernel_stats.csv' | head -1); cp "$f" $O/${n}_stats.csv
    echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])') $(grep -E 'pv_topn_(combine|merge)"' $O/${n}_stats.csv | cut -d, -f1,4 | tr '\n' ' ')"
  done
done
echo done
