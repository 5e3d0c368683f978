#!/bin/bash
# Round 5: top-N combine / merge phase times (-DPV_TSTAMPS build, PV_TSTAMPS=1: mean cycles per
# workgroup per phase) on C2 / C3 / C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5z}; mkdir -p $O
export TMPDIR=/tmp
for cfg in 2 3 4; do
  PV_TSTAMPS=1 PVGPU_LIB=$R/pktvisor_amd/variants/libpvgpu_tst.so timeout -k 10 300 python3 -u bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > $O/c$cfg.log 2>&1 || { tail -5 $O/c$cfg.log; exit 1; }
  echo "C$cfg: $(grep 'pv_tstamps combine' $O/c$cfg.log | tail -1)"
done
echo done
