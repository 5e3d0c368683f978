#!/bin/bash
# A/B of a tuning build (pktvisor_amd/variants/libpvgpu_$1.so) against the product library on
# C3 and C4: rocprofv3 kernel stats and the bench line of each. Stops on a time limit / fault.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
V=$1
O=$R/gpurun_out/var_$V
mkdir -p $O
export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 2"
for lib in base $V; do
  for c in ${CFGS:-3 4}; do
    (cd /tmp && { [ $lib != base ] && export PVGPU_LIB=$R/pktvisor_amd/variants/libpvgpu_$lib.so; true; } && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${lib}_c$c -o k -- python3 $B --config $c > $O/${lib}_c$c.log 2>&1) || { echo "$lib c$c failed"; tail -5 $O/${lib}_c$c.log; exit 1; }
    python3 tools/kstats.py $O/${lib}_c$c | head -2
    python3 -c "import json; d=json.loads(open('$O/${lib}_c$c.log').read().strip().splitlines()[-1]); print('  ', '$lib', 'c$c', d['ms_per_step'])"
  done
done
