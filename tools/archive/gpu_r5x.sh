#!/bin/bash
# Round 5: top-N combine shape: 1024-thread workgroups over an 8192-entry LDS table (default, one
# workgroup per CU) vs 512 threads over 4096 entries (two per CU), grid of 3 or 6 ranges per CU;
# parity tests under the 512/4096 build, then C2 / C3 / C4 kernel statistics per setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5x}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
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
  run c${cfg}_base $cfg $R/pktvisor_amd/libpvgpu.so
  run c${cfg}_cb512 $cfg $V/libpvgpu_cb512.so
  run c${cfg}_cb512_g6 $cfg $V/libpvgpu_cb512.so PV_NET_WGCU=6
  run c${cfg}_cb512k8 $cfg $V/libpvgpu_cb512k8.so
done
echo done
