#!/bin/bash
# Round 6: pipelined Net chunks (each chunk's combine on a second stream beside the next chunk's
# parse): parity suites, then C2-C4 A/B against PV_NET_CHUNKS=1 and a kernel trace of C2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6s}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_fullsize.py tests/test_gpu_bench_shape.py tests/test_gpu_windows.py tests/test_gpu_net_variants.py tests/test_gpu_topn_bound.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { # name cfg env...
  local n=$1 c=$2; shift 2
  local x=""; [ $c != 2 ] && x="--reset-each-step"
  env "$@" timeout -k 10 300 python3 -u bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-e2e $x > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], r.get("launches_per_step"), d["ms_per_step"], d["ms_per_step_median"])')"
}
for k in 1 2; do
  run c2_pipe_$k 2 PV_X=1
  run c2_flat_$k 2 PV_NET_CHUNKS=1
done
run c3_pipe 3 PV_X=1
run c3_flat 3 PV_NET_CHUNKS=1
run c4_pipe 4 PV_X=1
run c4_flat 4 PV_NET_CHUNKS=1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 2 > $O/prof_c2.log 2>&1) || { tail -20 $O/prof_c2.log; exit 1; }
echo "c2 $(python3 tools/kstats.py $O/prof_c2 2>/dev/null | cut -c1-400)"
