#!/bin/bash
# Round 6: the register pass with its general-path records deferred to pv_net_slow_list: bench
# C2-C4, then the parity tests that hold general-path records (fixtures, edge mix, variants, TCP).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6i}; mkdir -p $O
export TMPDIR=/tmp
run() { # name cfg env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"], d["ms_per_step_median"])')"
}
run c2 2 PV_X=0
run c3 3 PV_X=0
run c4 4 PV_X=0
run c2_g4r2 2 PV_NET_WGCU=4 PV_REG_WGCU=2
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_net_variants.py tests/test_gpu_tcp.py tests/test_gpu_bpf.py tests/test_gpu_net2.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
