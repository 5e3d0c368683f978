#!/bin/bash
# C3 / C4 kernel stats of each pktvisor_amd/variants/libpvgpu_*.so (bench lines + rocprofv3)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/v3_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
cd /tmp
for lib in $R/pktvisor_amd/variants/libpvgpu_*.so; do
  v=$(basename $lib .so)
  export PVGPU_LIB=$lib
  for c in 3 4; do
    timeout -k 10 200 $B --config $c > $O/${v}_bench_c$c.json 2> $O/${v}_bench_c$c.err || exit 1
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o c$c -- $B --config $c > /dev/null 2>&1 || exit 1
  done
done
echo "chain exit 0"
