#!/bin/bash
# PMC passes for C2, C3, C4 (tools/gpu_pmc.sh) folded per kernel and per bench config, then the C5 line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export GRAFT_REPO_ROOT=$(pwd)
O=gpurun_out/r4_t; mkdir -p $O
OUT=$O/pmc CFGS="2 3 4" bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
for c in 2 3 4; do python3 tools/pmc_summary.py $O/pmc $c > $O/pmc_c$c.json; done
for c in 2 3 4; do
  k=$(python3 -c "import json;d=json.load(open('$O/pmc_c$c.json'));print([k for k in d['kernels'] if k.startswith('pv_net_kernel')][0])")
  python3 tools/pmc_bench.py $O/pmc_c$c.json $c 10000000 $k "C$c 10M records" > $O/pmc_c${c}_10000000.json
done
tail -2 $O/pmc.log
bash tools/gpu_cmd_ev2.sh
