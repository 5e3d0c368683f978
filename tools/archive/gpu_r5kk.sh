#!/bin/bash
# Round 5: the Net pass launched without timing stamps (PV_NET_TIMING=0) vs with: C2 kernel traces
# (the gaps around the Net pass) and step times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5kk}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for t in 1 0; do
  PV_NET_TIMING=$t timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_t$t -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 2 > $O/prof_t$t.log 2>&1 || { tail -20 $O/prof_t$t.log; exit 1; }
done
cd $R
for k in 1 2; do for t in 1 0; do
  PV_NET_TIMING=$t timeout -k 10 300 python3 -u bench.py --config 2 --no-e2e --no-cpu-baseline > $O/c2_t${t}_$k.log 2>&1 || { tail -20 $O/c2_t${t}_$k.log; exit 1; }
  echo "C2 timing=$t: $(grep '^{' $O/c2_t${t}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_step_median"])')"
done; done
echo done
