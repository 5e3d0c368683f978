#!/bin/bash
# DNS-pass attribution (runtime knobs) on C3, then the bucketed key-cache probe A/B on C2/C3/C4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_dnsknob.sh && TAG=r4bkt CFGS="2 3 4" VARS="base:-:- bkt:bkt:-" bash tools/gpu_var.sh
