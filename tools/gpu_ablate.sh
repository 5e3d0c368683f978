#!/bin/bash
# attribute kernel time to metric groups (net bits: 1 counters, 2 cardinality, 8 top_ips; dns bits as pvgpu.h)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 $B --read-ceiling > gpurun_out/abl_default.log 2>&1 &&
timeout -k 10 200 $B --net-groups 1 --dns-groups 2 > gpurun_out/abl_counters.log 2>&1 &&
timeout -k 10 200 $B --net-groups 3 --dns-groups 2 > gpurun_out/abl_card.log 2>&1 &&
timeout -k 10 200 $B --net-groups 9 --dns-groups 2 > gpurun_out/abl_topips.log 2>&1 &&
timeout -k 10 200 $B --config 3 --records 10000000 > gpurun_out/abl_c3.log 2>&1 &&
timeout -k 10 200 $B --config 4 --records 4000000 > gpurun_out/abl_c4.log 2>&1
echo "chain exit $?"
