#!/bin/bash
# PMC passes of the C2 step (product library): instruction mix and HBM bytes per kernel
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_k
mkdir -p $O
OUT=$O/pmc CFGS="2" bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc 2 > $O/pmc_c2.json
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/r4_k/pmc_c2.json"))["kernels"]
for k,m in sorted(d.items()):
    print(k, {x: round(m[x]) if isinstance(m[x], float) and m[x] > 100 else round(m[x],3) for x in ("SQ_INSTS_VALU","SQ_INSTS_SALU","SQ_INSTS_LDS","SQ_INSTS_VMEM_RD","SQ_INSTS_VMEM_WR","SQ_WAVES","fetch_bytes_x2","write_bytes","frac_active_valu","frac_wait_any","lds_bank_conflict_frac") if x in m})
PY
