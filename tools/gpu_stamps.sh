#!/bin/bash
# per-phase cycle stamps of the tile loop (diagnostic build pktvisor_amd/variants/libpvgpu_stamps.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PVGPU_LIB=pktvisor_amd/variants/libpvgpu_stamps.so PV_STAMPS=1
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 200 $B --config 2 > gpurun_out/stamps_c2.log 2>&1 &&
PV_DEBUG_STAGES=1 timeout -k 10 200 $B --config 2 > gpurun_out/stamps_c2s1.log 2>&1 &&
timeout -k 10 200 $B --config 3 > gpurun_out/stamps_c3.log 2>&1 &&
timeout -k 10 200 $B --config 4 --records 4000000 > gpurun_out/stamps_c4.log 2>&1
echo "exit $?"
