#!/bin/bash
# Round 5: hot-address counting in the register Net pass (default on, PV_HOT=0 off) and the top-N
# combine shape (512 threads over a 4096-entry table, two workgroups per CU): parity tests with
# both on, then C2 / C3 / C4 kernel statistics per setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5y}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_hot.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_topn_bound.py tests/test_gpu_windows.py > $O/tests_hot.log 2>&1
trc=$?
tail -1 $O/tests_hot.log; grep -E "^(FAILED|ERROR)" $O/tests_hot.log | head -20
[ $trc -le 1 ] || exit 1
PVGPU_LIB=$V/libpvgpu_cb512.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_topn_bound.py > $O/tests_cb512.log 2>&1
trc=$?
tail -1 $O/tests_cb512.log; grep -E "^(FAILED|ERROR)" $O/tests_cb512.log | head -20
[ $trc -le 1 ] || exit 1
cd /tmp
run() { # name cfg lib env...
  local n=$1 cfg=$2 lib=$3; shift 3
  env "$@" PVGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $R/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  f=$(find $O/$n -name '*kernel_stats.csv' | head -1); cp "$f" $O/${n}_stats.csv
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])') $(grep -E 'pv_topn_(combine|merge)"' $O/${n}_stats.csv | cut -d, -f1,4 | tr '\n' ' ')"
}
for cfg in 2 3 4; do
  run c${cfg}_hot $cfg $R/pktvisor_amd/libpvgpu.so
  run c${cfg}_nohot $cfg $R/pktvisor_amd/libpvgpu.so PV_HOT=0
  run c${cfg}_cb512 $cfg $V/libpvgpu_cb512.so
  run c${cfg}_cb512_g6 $cfg $V/libpvgpu_cb512.so PV_NET_WGCU=6
done
echo done
