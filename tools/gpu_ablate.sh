#!/bin/bash
# attribute kernel time to metric groups (net bits: 1 counters, 2 cardinality, 8 top_ips; dns bits as pvgpu.h)
# usage: gpu_ablate.sh   -> gpurun_out/abl_*.log  + a C4 rocprofv3 kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 $B --config 3 --net-groups 1 --dns-groups 2 > gpurun_out/abl_c3_ctr.log 2>&1 &&
timeout -k 10 200 $B --config 3 --net-groups 1 --dns-groups 3 > gpurun_out/abl_c3_card.log 2>&1 &&
timeout -k 10 200 $B --config 3 --net-groups 1 --dns-groups 66 > gpurun_out/abl_c3_qn.log 2>&1 &&
timeout -k 10 200 $B --config 3 --net-groups 1 --dns-groups 258 > gpurun_out/abl_c3_port.log 2>&1 &&
timeout -k 10 200 $B --config 3 --net-groups 1 --dns-groups 18 > gpurun_out/abl_c3_xact.log 2>&1 &&
timeout -k 10 200 $B --config 3 --net-groups 1 --dns-groups 6 > gpurun_out/abl_c3_q.log 2>&1 &&
timeout -k 10 200 $B --config 3 > gpurun_out/abl_c3_default.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --config 4 --records 4000000 > gpurun_out/abl_c4_prof.log 2>&1
echo "chain exit $?"
