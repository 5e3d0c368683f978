#!/bin/bash
# Iteration check: top-N / parity GPU tests, then C2/C3/C4 bench lines and rocprofv3
# kernel stats (csv) of each, into gpurun_out/i3_<tag>/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/i3_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
T="${2:-tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_topn_bound.py tests/test_gpu_net2.py tests/test_gpu_dns2.py}"
B="python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
timeout -k 10 600 python3 -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 200 $B > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 200 $B --config 3 > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 200 $B --config 4 > $O/bench_c4.json 2> $O/bench_c4.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c2 -- $B > /dev/null 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- $B --config 3 > /dev/null 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c4 -- $B --config 4 > /dev/null 2>&1
rc=$?
echo "chain exit $rc"
exit $rc
