#!/bin/bash
# GPU parity suite on the main build, then kernel stats of every variant (tools/gpu_variants.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-x}
mkdir -p gpurun_out/var_$T
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/var_$T/gpu_tests.log 2>&1 &&
bash tools/gpu_variants.sh $T
