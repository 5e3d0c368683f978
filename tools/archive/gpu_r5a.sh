#!/bin/bash
# Round 5 probe: per-phase cycles of the top-N combine / merge (-DPV_TSTAMPS build) on C2-C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5a; mkdir -p $O
for c in 2 3 4; do
  PVGPU_LIB=$PWD/pktvisor_amd/variants/libpvgpu_tst.so PV_TSTAMPS=1 timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/tst_c$c.log 2>&1 || { tail -20 $O/tst_c$c.log; exit 1; }
  grep pv_tstamps $O/tst_c$c.log | tail -2
done
