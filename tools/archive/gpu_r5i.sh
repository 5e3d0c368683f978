#!/bin/bash
# Round 5: span-load Net pass (PV_NET_KERNEL=sp) against the default on C2-C4, parity with it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5i}; mkdir -p $O
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config ${CFG:-2} --no-cpu-baseline --no-e2e > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; return 1; }
  echo "$name $(tail -1 $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
}
run c2_default PV_X=0 && run c2_sp PV_NET_KERNEL=sp && run c2_sbd PV_NET_KERNEL=sbd || exit 1
CFG=3 run c3_sp PV_NET_KERNEL=sp && CFG=3 run c3_sbd PV_NET_KERNEL=sbd && CFG=4 run c4_sp PV_NET_KERNEL=sp || exit 1
PV_NET_KERNEL=sp timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py \
  > $O/tests_sp.log 2>&1 || { tail -40 $O/tests_sp.log; exit 1; }
tail -2 $O/tests_sp.log
echo done
