#!/bin/bash
# top-N combine / merge phase cycles (-DPV_TSTAMPS build) on C2, C3, C4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4_u; mkdir -p $O
for c in 2 3 4; do
  PV_TSTAMPS=1 PVGPU_LIB=$PWD/pktvisor_amd/variants/libpvgpu_tst.so timeout -k 10 240 python3 bench.py --config $c --steps 5 \
    --warmup 2 --no-cpu-baseline --no-e2e > $O/c$c.log 2>&1 || { tail -5 $O/c$c.log; exit 1; }
  echo "c$c"; grep pv_tstamps $O/c$c.log | tail -2 | cut -c1-300
done
