#!/bin/bash
# Round 6: the register pass without its general-path call (no scratch, 101 VGPRs; ablation build,
# C2 has no general-path record) at one and two workgroups per CU; the sharded-merge tests on the
# edge-chain change.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6h}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
run() { # name cfg lib env...
  local n=$1 c=$2 lib=$3; shift 3
  env "$@" PVGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"], d["ms_per_step_median"])')"
}
L=$R/pktvisor_amd/libpvgpu.so
run c2_main 2 $L PV_X=0
run c2_noslow 2 $V/libpvgpu_noslow.so PV_X=0
run c2_noslow_g4r2 2 $V/libpvgpu_noslow.so PV_NET_WGCU=4 PV_REG_WGCU=2
run c2_noslow_g2r2 2 $V/libpvgpu_noslow.so PV_NET_WGCU=2 PV_REG_WGCU=2
run c2_noslow_g3r3 2 $V/libpvgpu_noslow.so PV_NET_WGCU=3 PV_REG_WGCU=3
run c2_main_g4r2 2 $L PV_NET_WGCU=4 PV_REG_WGCU=2
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_windows.py tests/test_gpu_dns2_sharded.py tests/test_gpu_dist.py tests/test_gpu_rccl.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
