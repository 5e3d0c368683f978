#!/bin/bash
# DNS-pass attribution on C3 (kernel-trace stats per variant): default groups, no name
# decode (knob 16), no table updates (knob 32), both, and metric-group subsets.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/dnsabl_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --config 3"
R="rocprofv3 --kernel-trace --stats --output-format csv"
run() { local nm=$1 dbg=$2; shift 2
  ( export PV_DEBUG_STAGES=$dbg; timeout -k 10 200 $R -d $O/$nm -o k -- $B "$@" > $O/$nm.log 2>&1 ) }
run full 0 && run noname 16 && run notab 32 && run none 48 &&
run ctr 0 --net-groups 1 --dns-groups 2 && run card 0 --net-groups 1 --dns-groups 3 &&
run qn 0 --net-groups 1 --dns-groups 66 && run xact 0 --net-groups 1 --dns-groups 18
echo "chain exit $?"
