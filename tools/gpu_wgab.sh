#!/bin/bash
# A/B of the logical grid (PV_NET_WGCU workgroups per CU: the DNS pass, combine and merge
# partition) on C2/C3/C4 kernel stats: bash tools/gpu_wgab.sh TAG "2 3 4"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/r3_${1:-wg}
mkdir -p $O
export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-e2e"
for w in ${2:-2 3 4}; do
  for c in ${CFGS:-2 3 4}; do
    echo "[$(date +%T)] prof c$c wgcu $w"
    (cd /tmp && PV_NET_WGCU=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c${c}_w$w -o k -- python3 $B --steps 10 --config $c > $O/prof_c${c}_w$w.log 2>&1) || { tail -20 $O/prof_c${c}_w$w.log; exit 1; }
    python3 tools/kstats.py $O/prof_c${c}_w$w 2>/dev/null
    tail -1 $O/prof_c${c}_w$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  ms_per_step', d['ms_per_step'], 'median', d.get('ms_per_step_median'))"
  done
done
echo "[$(date +%T)] done"
