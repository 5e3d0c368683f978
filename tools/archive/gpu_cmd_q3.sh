#!/bin/bash
# PMC passes (HBM bytes, waves, LDS conflicts) for C2 and C3 on the current tree, folded per kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export GRAFT_REPO_ROOT=$(pwd)
O=gpurun_out/r4_q3
mkdir -p $O
OUT=$O/pmc CFGS="${CFGS:-2 3}" bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
for c in ${CFGS:-2 3}; do python3 tools/pmc_summary.py $O/pmc $c > $O/pmc_c$c.json; done
python3 tools/pmc_bench.py $O/pmc_c2.json 2 10000000 "$(python3 -c 'import json;d=json.load(open("'$O'/pmc_c2.json"));print([k for k in d["kernels"] if k.startswith("pv_net_kernel")][0])')" "C2 10M x 64 B" > $O/pmc_c2_10000000.json
tail -3 $O/pmc.log
