#!/bin/bash
# DNS-pass attribution by runtime knobs on C3, then the round-4 evidence (smoke, benches, kernel stats)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export GRAFT_REPO_ROOT=$(pwd)
bash tools/gpu_dnsknob.sh && bash tools/gpu_cmd_ev1.sh
