#!/bin/bash
# Round 5: full GPU suite + C2-C4 bench + stamps + C2/C3 kernel stats on the current tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5d}; mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 2 3 4; do
  timeout -k 10 300 python3 -u bench.py --config $c --no-cpu-baseline --no-e2e > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  echo "c$c $(tail -1 $O/bench_c$c.log | cut -c100-190)"
done
for c in 2 3 4; do
  PVGPU_LIB=$PWD/pktvisor_amd/variants/libpvgpu_tst.so PV_TSTAMPS=1 timeout -k 10 300 python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/tst_c$c.log 2>&1 || { tail -20 $O/tst_c$c.log; exit 1; }
  echo "c$c $(grep 'pv_tstamps combine' $O/tst_c$c.log | tail -1)"
done
for c in 2 3 4; do
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c$c -o k -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c > $GRAFT_REPO_ROOT/$O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
python3 tools/kstats.py $O/prof_c$c 2>/dev/null | cut -c1-250
done
step done
