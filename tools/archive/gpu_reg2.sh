#!/bin/bash
# Register-window Net pass sweep on C2: pipeline depth, waves per SIMD, workgroups per CU, and
# the lean levels (1 loads only, 2 + parse/counters, 3 + histogram, 4 + IP log)
set -o pipefail
cd $GRAFT_REPO_ROOT
for spec in "base:-:-:0" "base:-:-:2" "d2w2:d2w2:-:1" "d2w2:d2w2:-:2" "d3w2:d3w2:-:1" "d3w2:d3w2:-:2" "d3w3:d3w3:-:0" "d3w3:d3w3:-:2" \
            "l1:l1:-:2" "l2:l2:-:2" "l3:l3:-:2" "l4:l4:-:2" "l1:l1:-:1" "ring:-:fast:0"; do
  IFS=: read v lib kern w <<< "$spec"
  if [ "$w" = 0 ]; then unset PV_NET_WGCU; else export PV_NET_WGCU=$w; fi
  TAG=reg2_w$w VARS="$v:$lib:$kern" CFGS=2 bash tools/gpu_var.sh || exit 1
done
