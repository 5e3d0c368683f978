#!/bin/bash
# ring Net pass layouts on C2 (kernel stats): 4 parsers + 4 producers (product build) vs 8 + 8
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r4n CFGS="2" VARS="ring4:-:ring ring8:r81:ring" bash tools/gpu_var.sh
