#!/bin/bash
# Register-window Net pass on C2 at one workgroup per CU: lean levels (2 parse/counters,
# 3 + histogram, 4 + IP log; the full pass is the library), pipeline depth 3 and the
# register cap of one wave per SIMD; then the library's C3 / C4 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=reg3 VARS="base:-:- l2:l2:- l3:l3:- l4:l4:- d3w1:d3w1:- d2w1:d2w1:-" CFGS=2 bash tools/gpu_var.sh || exit 1
TAG=reg3 VARS="base:-:-" CFGS="3 4" bash tools/gpu_var.sh
