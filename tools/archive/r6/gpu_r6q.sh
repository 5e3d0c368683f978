#!/bin/bash
# Round 6: 56-bit transaction sort keys: the tests that pair transactions (parity, KATs, DNS v2,
# sharded, TCP, windows, full-size C4), then C4 kernel stats and bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6q}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_dns2.py tests/test_gpu_dns2_sharded.py tests/test_gpu_dist.py tests/test_gpu_tcp.py tests/test_gpu_windows.py tests/test_gpu_deep_sampling.py "tests/test_gpu_bench_shape.py::test_bench_step_full_size[4]" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
c=4
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $c --reset-each-step > $O/prof_c$c.log 2>&1) || { tail -20 $O/prof_c$c.log; exit 1; }
echo "c$c $(python3 tools/kstats.py $O/prof_c$c 2>/dev/null | cut -c1-400)"
timeout -k 10 300 python3 -u bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-e2e --reset-each-step > $O/c$c.log 2>&1 || { tail -5 $O/c$c.log; exit 1; }
echo "c$c: $(grep '^{' $O/c$c.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median"])')"
