#!/bin/bash
# staging-floor experiments: each variant library in stage-only mode (PV_DEBUG_STAGES=1) on C2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/exp_${1:-x}
mkdir -p $O
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for lib in pktvisor_amd/libpvgpu.so pktvisor_amd/variants/libpvgpu_*.so; do
  v=$(basename $lib .so)
  ( export PVGPU_LIB=$lib PV_DEBUG_STAGES=1; timeout -k 10 120 $B > $O/${v}_s1.log 2>&1 ) || exit 1
  ( export PVGPU_LIB=$lib; timeout -k 10 120 $B > $O/${v}_full.log 2>&1 ) || exit 1
done
echo done
