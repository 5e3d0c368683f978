#!/bin/bash
# Round-2 (second session) evidence on the final tree: the GPU suite, smoke(), the default
# bench line (as the driver runs it), rocprofv3 kernel-trace stats of the C2/C3/C4 benches,
# and the C2 / C3 PMC passes (one counter group per run: tools/gpu_pmc.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/r2s2_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-e2e"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/bench_torchrun1.log 2>&1 &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o k -- $B > $O/prof_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o k -- $B --config 3 > $O/prof_c3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o k -- $B --config 4 > $O/prof_c4.log 2>&1 &&
cd $R && OUT=gpurun_out/r2s2_${1:-x}/pmc CFGS="2 3" bash tools/gpu_pmc.sh > $O/pmc.log 2>&1
rc=$?
echo "chain exit $rc"
exit $rc
