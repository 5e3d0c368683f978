#!/bin/bash
# DNS-pass attribution on C3: full, no names (16), no tables (32), neither (48), no transactions
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/dnsabl2_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --config 3"
R="rocprofv3 --kernel-trace --stats --output-format csv"
run() { local nm=$1 dbg=$2; shift 2
  ( export PV_DEBUG_STAGES=$dbg; timeout -k 10 200 $R -d $O/$nm -o k -- $B "$@" > $O/$nm.log 2>&1 ) }
run full 0 && run noname 16 && run notab 32 && run none 48 && run noxact 0 --dns-groups $2 && run nonex 48 --dns-groups $2
echo "chain exit $?"
