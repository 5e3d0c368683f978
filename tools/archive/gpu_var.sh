#!/bin/bash
# A/B of Net-pass variants: kernel stats of C2/C3/C4 benches per (library, PV_NET_KERNEL)
# pair. VARS="name:lib:kernel ..." (lib "-" = pktvisor_amd/libpvgpu.so, kernel "-" = default)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_${TAG:-var}; mkdir -p $O
export TMPDIR=/tmp
for spec in ${VARS:-base:-:-}; do
  IFS=: read v lib kern <<< "$spec"
  L=$PWD/pktvisor_amd/libpvgpu.so; [ "$lib" != - ] && L=$PWD/pktvisor_amd/variants/libpvgpu_$lib.so
  K=""; [ "$kern" != - ] && K=$kern
  for c in ${CFGS:-2 3 4}; do
    (cd /tmp && PVGPU_LIB=$L PV_NET_KERNEL=$K timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/${v}_c$c -o k -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c > $GRAFT_REPO_ROOT/$O/${v}_c$c.log 2>&1) || { tail $O/${v}_c$c.log; exit 1; }
    python3 tools/kstats.py $O/${v}_c$c | cut -c1-150
  done
done
