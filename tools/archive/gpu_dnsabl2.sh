#!/bin/bash
# DNS-pass attribution on C3 (rocprofv3 kernel stats per variant): full, no name hashing (16),
# no table updates (32), neither (48), no transactions group, counters group only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/dnsabl2_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python3 $PWD/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --config ${CFG:-3}"
run() { local nm=$1 dbg=$2; shift 2
  ( export PV_DEBUG_STAGES=$dbg; cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/$nm -o k -- $B "$@" > $OLDPWD/$O/$nm.log 2>&1 ) || return 1
  python3 tools/kstats.py $O/$nm | head -3; }
run full 0 && run noname 16 && run notab 32 && run none 48 && run notrans 0 --dns-groups 2147483975 && run ctronly 0 --dns-groups 2147483650
echo "chain exit $?"
