#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on the C2 bench, stage-only
# and full, for the Net pass: instruction mix, waits, LDS, memory.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pmc_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
P="rocprofv3 --kernel-trace --output-format csv"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
G2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
for mode in 1 0; do
  ( export PV_DEBUG_STAGES=$mode
    timeout -s KILL 90 $P --pmc $G1 -d $O/g1_$mode -o k -- $B > $O/g1_$mode.log 2>&1 &&
    timeout -s KILL 90 $P --pmc $G2 -d $O/g2_$mode -o k -- $B > $O/g2_$mode.log 2>&1 &&
    timeout -s KILL 90 $P --pmc FETCH_SIZE -d $O/f_$mode -o k -- $B > $O/f_$mode.log 2>&1 &&
    timeout -s KILL 90 $P --pmc WRITE_SIZE -d $O/w_$mode -o k -- $B > $O/w_$mode.log 2>&1 ) || exit 1
done
echo done
