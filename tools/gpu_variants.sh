#!/bin/bash
# time kernel variants (pktvisor_amd/variants/libpvgpu_*.so) on C2/C3/C4 + staging-only
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/var_${1:-x}
mkdir -p $O
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
for lib in pktvisor_amd/libpvgpu.so pktvisor_amd/variants/libpvgpu_*.so; do
  v=$(basename $lib .so)
  export PVGPU_LIB=$lib
  PV_DEBUG_STAGES=1 timeout -k 10 200 $B --config 2 > $O/${v}_c2s1.log 2>&1 || exit 1
  for cfg in 2 3; do
    timeout -k 10 200 $B --config $cfg > $O/${v}_c$cfg.log 2>&1 || exit 1
  done
  timeout -k 10 200 $B --config 4 --records 4000000 > $O/${v}_c4.log 2>&1 || exit 1
done
echo done
