#!/bin/bash
# Round 5: is the C2 Net pass bound by the texture-address path? TA / TCP counters of one bench run
# (each pass its own run and limit).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5n}; mkdir -p $O
export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --config 2"
pass() {  # name counters...
  local n=$1; shift
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex 'pv_net.*' --output-format csv -d $O/$n -o run -- python3 $B > $O/$n.log 2>&1) || { echo "pass $n failed"; tail -5 $O/$n.log; return 1; }
  echo "pass $n done"
}
pass ta TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum || exit 1
echo done
