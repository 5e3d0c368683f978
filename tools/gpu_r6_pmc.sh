#!/bin/bash
# Round 6 evidence: rocprofv3 PMC passes (one counter group per run, each under its own limit;
# MI355X_MICROARCH.md HBM section) over C2 and C3 / C4 (reset each step, as their bench lines),
# then kernel stats of C2-C4 at HEAD. tools/pmc_summary.py + tools/pmc_bench.py fold them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6pmc}; mkdir -p $O
export TMPDIR=/tmp
P1="FETCH_SIZE"
P2="WRITE_SIZE TCC_HIT TCC_MISS"
P3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P4="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"
for c in 2 3 4; do
  x=""; [ $c != 2 ] && x="--reset-each-step"
  for p in 1 2 3 4; do
    eval "CTR=\$P$p"
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-include-regex 'pv_.*' --output-format csv \
        -d $O/c${c}_p$p -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --config $c $x > $O/c${c}_p$p.log 2>&1) || { echo "c$c p$p failed"; tail -5 $O/c${c}_p$p.log; exit 1; }
    echo "c$c p$p done"
  done
done
for c in 2 3 4; do
  x=""; [ $c != 2 ] && x="--reset-each-step"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c $x > $O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
  echo "c$c $(python3 tools/kstats.py $O/prof_c$c 2>/dev/null | cut -c1-400)"
done
