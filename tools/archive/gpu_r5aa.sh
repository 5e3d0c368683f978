#!/bin/bash
# Round 5: top-N combine counting regions as entries are created (PV_CB_FUSE) and the merge's
# write-back with all of a thread's count reads in one round trip (PV_MG_WB=8) vs the previous
# build (old variant): parity tests, C2 / C3 / C4 kernel statistics, combine / merge phase times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5aa}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_topn_bound.py tests/test_gpu_windows.py tests/test_gpu_net2.py tests/test_gpu_dist.py > $O/tests.log 2>&1
trc=$?
tail -1 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head -20
[ $trc -le 1 ] || exit 1
cd /tmp
run() { # name cfg lib env...
  local n=$1 cfg=$2 lib=$3; shift 3
  env "$@" PVGPU_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $R/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  f=$(find $O/$n -name '*kernel_stats.csv' | head -1); cp "$f" $O/${n}_stats.csv
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])') $(grep -E 'pv_topn_(combine|merge)"' $O/${n}_stats.csv | cut -d, -f1,4 | tr '\n' ' ')"
}
for cfg in 2 3 4; do
  run c${cfg}_new $cfg $R/pktvisor_amd/libpvgpu.so
  run c${cfg}_old $cfg $V/libpvgpu_old.so
done
cd $R
for cfg in 2 3; do
  PV_TSTAMPS=1 PVGPU_LIB=$V/libpvgpu_tst.so timeout -k 10 300 python3 -u bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > $O/tst_c$cfg.log 2>&1 || { tail -5 $O/tst_c$cfg.log; exit 1; }
  echo "C$cfg: $(grep 'pv_tstamps combine' $O/tst_c$cfg.log | tail -1)"
done
echo done
