#!/bin/bash
# Net-pass phase stamps (variants/libpvgpu_stamps.so) on C2 and C4, plus the iteration check
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-x}
O=gpurun_out/it_$T
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
( export PVGPU_LIB=pktvisor_amd/variants/libpvgpu_stamps.so PV_STAMPS=1; timeout -k 10 200 $B > $O/stamps_c2.log 2>&1 && timeout -k 10 200 $B --config 4 --records 4000000 > $O/stamps_c4.log 2>&1 )
