#!/bin/bash
# Net-pass attribution on C2: the register pass built with PV_LEAN_LEVEL 1..4 (loads only, +
# parse and counters, + histogram, + IP log; pktvisor_amd/variants/libpvgpu_lean*.so) against
# the product build. The lean builds skip work, so bench's parity check fails after timing: the
# rocprofv3 kernel stats are the result. Stops on a time limit, abort or fault.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/lean_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 2"
for L in 0 1 2 3 4; do
  lib=""; [ $L != 0 ] && lib=$R/pktvisor_amd/variants/libpvgpu_lean$L.so
  (cd /tmp && { [ -n "$lib" ] && export PVGPU_LIB=$lib; true; } && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/l$L -o k -- python3 $B > $O/l$L.log 2>&1)
  rc=$?
  case $rc in 0|1) ;; *) echo "level $L ended with $rc"; exit $rc;; esac
  python3 tools/kstats.py $O/l$L | head -2
done
