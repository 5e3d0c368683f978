#!/bin/bash
# Round 5: Net-pass dispatch stamps only on sampled batches (pv_set_kernel_timing; bench: every
# 4th timed step): tests, bench C2-C5, C2 kernel statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5ll}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_contract.py tests/test_gpu_boundary.py tests/test_gpu_net_variants.py > $O/tests.log 2>&1
trc=$?
tail -1 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head -20
[ $trc -le 1 ] || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for c in 2 3 4; do
  F="--no-e2e"; [ $c = 2 ] && F=""
  timeout -k 10 400 python3 -u bench.py --config $c $F > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  grep '^{' $O/bench_c$c.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["config"]["workload"][:3], d["value"], d["ms_per_step"], d["ms_per_step_median"], r["kernel_ms"], r["frac"], r["kernel_ms_sample"], d["cpu_baseline"]["value"])'
done
timeout -k 10 600 python3 -u bench.py --config 5 --steps 2 --warmup 1 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | cut -c1-250
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 2 > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
python3 $R/tools/kstats.py $O/prof_c2 2>/dev/null | cut -c1-300
echo done
