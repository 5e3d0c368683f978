#!/bin/bash
# Round 5: Net-pass store modes (PV_NET_KERNEL=sb|nt|sbnt) on C2 / C3 with full-size parity, and
# the world-8 merge with the binary-search selection.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5h}; mkdir -p $O
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config ${CFG:-2} --no-cpu-baseline --no-e2e > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; return 1; }
  echo "$name $(tail -1 $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["kernel_ms"])')"
}
for m in default sb nt sbnt; do run c2_$m PV_NET_KERNEL=$m || exit 1; done
for m in default sb sbd; do CFG=3 run c3_$m PV_NET_KERNEL=$m || exit 1; done
run c2_sbd PV_NET_KERNEL=sbd || exit 1
PV_NET_KERNEL=sbd timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  > $O/tests_sb.log 2>&1 || { tail -40 $O/tests_sb.log; exit 1; }
tail -2 $O/tests_sb.log
timeout -k 10 900 python3 -u tools/merge_world8.py --records 100000000 > $O/merge_world8.log 2>&1 || { tail -30 $O/merge_world8.log; exit 1; }
grep merge_world8 $O/merge_world8.log
echo done
