#!/bin/bash
# Round 5: the combine's list write with 8 cursor reservations in flight per thread (PV_CB_OB=8,
# default) vs one at a time (ob1 variant): top-N parity tests, alternating C2 / C3 / C4 bench lines,
# combine phase timers.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5nn}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_topn_bound.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py > $O/tests.log 2>&1
trc=$?
tail -1 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head -20
[ $trc -le 1 ] || exit 1
for cfg in 2 3 4; do
for k in 1 2; do
  for v in ob8 ob1; do
    L=$R/pktvisor_amd/libpvgpu.so; [ $v = ob1 ] && L=$V/libpvgpu_ob1.so
    PVGPU_LIB=$L timeout -k 10 400 python3 -u bench.py --config $cfg --no-e2e --no-cpu-baseline > $O/c${cfg}_${v}_$k.log 2>&1 || { tail -20 $O/c${cfg}_${v}_$k.log; exit 1; }
    echo "C$cfg $v: $(grep '^{' $O/c${cfg}_${v}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_step_median"])')"
  done
done
done
for cfg in 2 3; do
  PV_TSTAMPS=1 PVGPU_LIB=$V/libpvgpu_tst.so timeout -k 10 300 python3 -u bench.py --config $cfg --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > $O/tst_c$cfg.log 2>&1 || { tail -5 $O/tst_c$cfg.log; exit 1; }
  echo "C$cfg: $(grep 'pv_tstamps combine' $O/tst_c$cfg.log | tail -1)"
done
echo done
