#!/bin/bash
# time kernel variants (pktvisor_amd/variants/libpvgpu_*.so) on C2/C3/C4 (kernel-trace stats)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/var_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
R="rocprofv3 --kernel-trace --stats --output-format csv"
for lib in pktvisor_amd/libpvgpu.so pktvisor_amd/variants/libpvgpu_*.so; do
  v=$(basename $lib .so)
  export PVGPU_LIB=$lib
  timeout -k 10 200 $R -d $O/${v}_c2 -o k -- $B --config 2 > $O/${v}_c2.log 2>&1 || exit 1
  timeout -k 10 200 $R -d $O/${v}_c3 -o k -- $B --config 3 > $O/${v}_c3.log 2>&1 || exit 1
  timeout -k 10 200 $R -d $O/${v}_c4 -o k -- $B --config 4 --records 4000000 > $O/${v}_c4.log 2>&1 || exit 1
done
echo done
