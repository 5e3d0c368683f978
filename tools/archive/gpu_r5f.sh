#!/bin/bash
# Round 5: C2 A/B of runtime knobs (Net-pass kernel and occupancy, batch partition), kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5f}; mkdir -p $O
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config 2 --no-cpu-baseline --no-e2e > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; return 1; }
  echo "$name $(tail -1 $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["kernel_ms"])')"
}
run default PV_X=0 && run ring PV_NET_KERNEL=ring && run regwg2 PV_REG_WGCU=2 && run reg8 PV_REG_WAVES=8 && run netwg2 PV_NET_WGCU=2 && run netwg4 PV_NET_WGCU=4 || exit 1
for v in "ring PV_NET_KERNEL=ring" "netwg2 PV_NET_WGCU=2"; do
  set -- $v
  (cd /tmp && env $2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$1 -o k -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 2 > $GRAFT_REPO_ROOT/$O/prof_$1.log 2>&1) || { tail -20 $O/prof_$1.log; exit 1; }
  python3 tools/kstats.py $O/prof_$1 2>/dev/null | cut -c1-200
done
echo done
