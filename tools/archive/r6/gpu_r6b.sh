#!/bin/bash
# Round 6: net_probe ladder (the register-window load pattern grown toward the product's skeleton,
# on the generator's C2 records and on ring_probe's constant bytes, with and without dirty caches);
# the read-time-merge bench step; the merged-window refusal and the bench-shape parity tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6b}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 tools/net_probe > $O/net_probe.log 2>&1 || { tail -20 $O/net_probe.log; exit 1; }
cat $O/net_probe.log
for c in 2 3 4; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  echo "c$c accumulate: $(grep '^{' $O/bench_c$c.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"], d["ms_per_step_median"])')"
  timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --reset-each-step > $O/bench_c${c}_reset.log 2>&1 || { tail -20 $O/bench_c${c}_reset.log; exit 1; }
  echo "c$c reset: $(grep '^{' $O/bench_c${c}_reset.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"], d["ms_per_step_median"])')"
done
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_rccl.py tests/test_gpu_dist.py tests/test_gpu_bench_shape.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -8 $O/tests.log
echo done
