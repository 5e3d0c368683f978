#!/bin/bash
# A/B of the lean Net pass: register windows (default) vs LDS ring, grids of 2/3 workgroups per CU
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_kat.py tests/test_gpu_tcp.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_reg_tests.log 2>&1 || { tail -30 gpurun_out/r3_reg_tests.log; exit 1; }
tail -2 gpurun_out/r3_reg_tests.log
TAG=reg VARS="reg:-:- ring:-:fast reg4:reg4:-" bash tools/gpu_var.sh || exit 1
for w in 2 4; do PV_NET_WGCU=$w TAG=reg_w$w VARS="reg:-:-" CFGS="2 3" bash tools/gpu_var.sh || exit 1; done
