#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on the C2 bench + ablation timings
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
P="rocprofv3 --kernel-trace --output-format csv"
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --net-groups 1 --dns-groups 2 > gpurun_out/pmc_abl_ctr.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --net-groups 3 --dns-groups 2 > gpurun_out/pmc_abl_card.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --net-groups 9 --dns-groups 2 > gpurun_out/pmc_abl_top.log 2>&1 &&
timeout -k 10 300 $P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/pmc1 -o c2 -- $B > gpurun_out/pmc1.log 2>&1 &&
timeout -k 10 300 $P --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc2 -o c2 -- $B > gpurun_out/pmc2.log 2>&1 &&
timeout -k 10 300 $P --pmc FETCH_SIZE -d gpurun_out/pmc3 -o c2 -- $B > gpurun_out/pmc3.log 2>&1 &&
timeout -k 10 300 $P --pmc WRITE_SIZE -d gpurun_out/pmc4 -o c2 -- $B > gpurun_out/pmc4.log 2>&1 &&
timeout -k 10 300 $P --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum -d gpurun_out/pmc5 -o c2 -- $B > gpurun_out/pmc5.log 2>&1
echo "chain exit $?"
