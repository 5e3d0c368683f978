#!/bin/bash
# Round 5: merge v2 + two-pass IPv4 CPC, combine fan-in A/B (PV_CB_FAN 1/2/3) on C2-C4, stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5c}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_topn_bound.py tests/test_gpu_fullsize.py tests/test_gpu_windows.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 1 2 3; do for c in 2 3 4; do
  PV_CB_FAN=$f timeout -k 10 300 python3 -u bench.py --config $c --no-cpu-baseline --no-e2e > $O/bench_c${c}_f$f.log 2>&1 || { tail -20 $O/bench_c${c}_f$f.log; exit 1; }
  echo "fan $f c$c $(tail -1 $O/bench_c${c}_f$f.log | cut -c100-190)"
done; done
for f in 1 3; do for c in 2 3 4; do
  PV_CB_FAN=$f PVGPU_LIB=$PWD/pktvisor_amd/variants/libpvgpu_tst.so PV_TSTAMPS=1 timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/tst_c${c}_f$f.log 2>&1 || { tail -20 $O/tst_c${c}_f$f.log; exit 1; }
  echo "fan $f c$c $(grep 'pv_tstamps combine' $O/tst_c${c}_f$f.log | tail -1)"
done; done
for f in 1 3; do
(cd /tmp && PV_CB_FAN=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c2_f$f -o k -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 2 > $GRAFT_REPO_ROOT/$O/prof_c2_f$f.log 2>&1) || { tail -20 $O/prof_c2_f$f.log; exit 1; }
python3 tools/kstats.py $O/prof_c2_f$f 2>/dev/null | cut -c1-200
done
step done
