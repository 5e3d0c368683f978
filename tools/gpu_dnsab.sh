#!/bin/bash
# A/B of the DNS pass on C3 under each Net-pass kernel (PV_NET_KERNEL=ns|fast vs the register
# pass), after the deep-sampling tests: bash tools/gpu_dnsab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/r3_${1:-ab}
mkdir -p $O
export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-e2e"
echo "[$(date +%T)] tests"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_deep_sampling.py tests/test_gpu_windows.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in reg ns fast; do
  echo "[$(date +%T)] prof c3 $k"
  (cd /tmp && PV_NET_KERNEL=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$k -o k -- python3 $B --steps 10 --config 3 > $O/prof_c3_$k.log 2>&1) || { tail -20 $O/prof_c3_$k.log; exit 1; }
  python3 tools/kstats.py $O/prof_c3_$k 2>/dev/null
done
echo "[$(date +%T)] done"
