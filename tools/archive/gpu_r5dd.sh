#!/bin/bash
# Round 5: parameter blocks uploaded through kernel arguments (pv_store_blob) instead of copies:
# the whole GPU suite, bench C2 / C3 / C4, a C2 kernel trace (gaps between the step's kernels).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5dd}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
trc=$?
tail -1 $O/gpu_tests.log; grep -E "^(FAILED|ERROR)" $O/gpu_tests.log | head -20
[ $trc -le 1 ] || exit 1
for c in 2 3 4; do
  F="--no-e2e"; [ $c = 2 ] && F=""
  timeout -k 10 400 python3 -u bench.py --config $c $F > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  grep '^{' $O/bench_c$c.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["config"]["workload"][:3], d["value"], d["ms_per_step"], d["ms_per_step_median"], r["kernel_ms"], r["frac"], d["cpu_baseline"]["value"])'
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 2 > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
[ $trc -eq 0 ] || exit 1
echo done
