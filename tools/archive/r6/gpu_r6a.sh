#!/bin/bash
# Round 6: the Net pass at two workgroups per CU with a balanced range walk. Round 5's "wg2"
# runs gave 512 Net-pass workgroups 768 grid ranges (3 per CU), so half of them walked two ranges
# and half one; here the grid's ranges per CU are a multiple of the Net pass's workgroups per CU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6a}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
run() { # name lib env...
  local n=$1 lib=$2; shift 2
  env "$@" PVGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py --config ${CFG:-2} --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"])')"
}
L=$R/pktvisor_amd/libpvgpu.so
run full_g3_r1 $L PV_NET_WGCU=3 PV_REG_WGCU=1
run full_g4_r2 $L PV_NET_WGCU=4 PV_REG_WGCU=2
run full_g2_r2 $L PV_NET_WGCU=2 PV_REG_WGCU=2
run full_g3_r3 $L PV_NET_WGCU=3 PV_REG_WGCU=3
run full_g4_r4 $L PV_NET_WGCU=4 PV_REG_WGCU=4
run lean1_g3_r1 $V/libpvgpu_lean1.so PV_NET_WGCU=3 PV_REG_WGCU=1
run lean1_g4_r2 $V/libpvgpu_lean1.so PV_NET_WGCU=4 PV_REG_WGCU=2
run lean1_g2_r2 $V/libpvgpu_lean1.so PV_NET_WGCU=2 PV_REG_WGCU=2
run lean1_g3_r3 $V/libpvgpu_lean1.so PV_NET_WGCU=3 PV_REG_WGCU=3
CFG=3 run c3_default $L PV_X=0
CFG=3 run c3_g4_r2 $L PV_NET_WGCU=4 PV_REG_WGCU=2
CFG=4 run c4_default $L PV_X=0
CFG=4 run c4_g4_r2 $L PV_NET_WGCU=4 PV_REG_WGCU=2
echo done
