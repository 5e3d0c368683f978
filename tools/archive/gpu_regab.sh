#!/bin/bash
# A/B of the register-window Net pass's waves per workgroup (PV_REG_WAVES=4|8, one workgroup
# per CU): C2 bench lines and rocprofv3 kernel stats of C2 and C3 per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/regab_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-e2e"
for w in ${WAVES:-4 8}; do
  for c in 2 3; do
    echo "[$(date +%T)] waves $w c$c"
    (cd /tmp && PV_REG_WAVES=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w${w}_c$c -o k -- python3 $B --steps 10 --config $c > $O/w${w}_c$c.log 2>&1) || { tail -20 $O/w${w}_c$c.log; exit 1; }
    python3 tools/kstats.py $O/w${w}_c$c | head -2
  done
  PV_REG_WAVES=$w timeout -k 10 300 python3 $B > $O/bench_w$w.log 2>&1 || { tail -20 $O/bench_w$w.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_w$w.log').read().strip().splitlines()[-1]); print('w$w', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
