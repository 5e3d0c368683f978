#!/bin/bash
# Round 6: non-temporal stores for the step's large writers (merge write-back default; IP log and
# combine list as variants) on the depth-3 unconditional-load Net pass; kernel stats per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6f}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
run() { # name cfg lib env...
  local n=$1 c=$2 lib=$3; shift 3
  env "$@" PVGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"], d["ms_per_step_median"])')"
}
prof() { # name cfg lib
  (cd /tmp && PVGPU_LIB=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1 -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $2 > $O/prof_$1.log 2>&1) || { tail -20 $O/prof_$1.log; exit 1; }
  echo "$1 $(python3 tools/kstats.py $O/prof_$1 2>/dev/null | cut -c1-250)"
}
L=$R/pktvisor_amd/libpvgpu.so
for c in 2 3 4; do
  run c${c}_main $c $L PV_X=0
  run c${c}_m0 $c $V/libpvgpu_m0.so PV_X=0
  run c${c}_mi $c $V/libpvgpu_mi.so PV_X=0
  run c${c}_mc $c $V/libpvgpu_mc.so PV_X=0
done
prof c2_main 2 $L
prof c2_m0 2 $V/libpvgpu_m0.so
prof c2_mi 2 $V/libpvgpu_mi.so
prof c2_mc 2 $V/libpvgpu_mc.so
echo done
