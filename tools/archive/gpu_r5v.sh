#!/bin/bash
# Round 5: bytes in flight of the register-window Net pass, C2: pipeline depth 2 vs 3, one or two
# workgroups per CU, 4 or 8 waves, at lean level 1 (loads only) and in full; the plain-read ceiling.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5v}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
run() { # name lib env...
  local n=$1 lib=$2; shift 2
  env "$@" PVGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e $XARGS > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"], d.get("read_ceiling_gbs"))')"
}
XARGS=--read-ceiling run lean1_d2_wg1 $V/libpvgpu_lean1.so PV_REG_WGCU=1
XARGS= 
run lean1_d3_wg1 $V/libpvgpu_lean1d3.so PV_REG_WGCU=1
run lean1_d2_wg2 $V/libpvgpu_lean1.so PV_REG_WGCU=2
run lean1_d3_wg2 $V/libpvgpu_lean1d3.so PV_REG_WGCU=2
run lean1_d2_w8 $V/libpvgpu_lean1.so PV_REG_WAVES=8
run full_d2_wg1 $R/pktvisor_amd/libpvgpu.so PV_REG_WGCU=1
run full_d3_wg1 $V/libpvgpu_d3.so PV_REG_WGCU=1
run full_d3_wg2 $V/libpvgpu_d3.so PV_REG_WGCU=2
echo done
