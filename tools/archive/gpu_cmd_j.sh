#!/bin/bash
# ring-parser / top-N phase stamps (tst variants) and bench + kernel stats of the product and the
# 8-parser ring layout on C2 / C4
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_j
mkdir -p $O
export TMPDIR=/tmp
for v in tst r8tst; do
  np=4; [ $v = r8tst ] && np=8
  PV_RING_NP=$np PVGPU_LIB=$PWD/pktvisor_amd/variants/libpvgpu_$v.so PV_TSTAMPS=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/$v.log 2>&1 || exit 1
  echo $v; grep pv_tstamps $O/$v.log | tail -2
done
TAG=r4j CFGS="2 4" VARS="base:-:- r8:r8:-" bash tools/gpu_var.sh
