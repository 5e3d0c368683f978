#!/bin/bash
# Round 6: the Net pass's pipeline depth and unconditional loads (variants d3, u2, u3) against the
# default, one and two workgroups per CU; C3/C4 for each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6e}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
run() { # name cfg lib env...
  local n=$1 c=$2 lib=$3; shift 3
  env "$@" PVGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"])')"
}
L=$R/pktvisor_amd/libpvgpu.so
for c in 2 3 4; do
  run c${c}_base $c $L PV_X=0
  run c${c}_d3 $c $V/libpvgpu_d3.so PV_X=0
  run c${c}_u2 $c $V/libpvgpu_u2.so PV_X=0
  run c${c}_u3 $c $V/libpvgpu_u3.so PV_X=0
done
run c2_u2_g4r2 2 $V/libpvgpu_u2.so PV_NET_WGCU=4 PV_REG_WGCU=2
run c2_u3_g4r2 2 $V/libpvgpu_u3.so PV_NET_WGCU=4 PV_REG_WGCU=2
run c2_base_again 2 $L PV_X=0
echo done
