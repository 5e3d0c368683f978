#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, each under its own time limit) over the
# bench's C2 / C3 / C4 steps; tools/pmc_summary.py folds them into per-kernel means.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
B="$PWD/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
P1="FETCH_SIZE"
P2="WRITE_SIZE TCC_HIT TCC_MISS"
P3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P4="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"
for c in ${CFGS:-2 3 4}; do
  for p in 1 2 3 4; do
    eval "CTR=\$P$p"
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-include-regex 'pv_.*' --output-format csv \
        -d $GRAFT_REPO_ROOT/$OUT/c${c}_p$p -o run -- python3 $B --config $c > $GRAFT_REPO_ROOT/$OUT/c${c}_p$p.log 2>&1) || exit 1
    echo "c$c p$p done"
  done
done
