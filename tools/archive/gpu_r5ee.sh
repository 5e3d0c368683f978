#!/bin/bash
# Round 5: C3 / C4 kernel traces (the step's kernel order and the gaps between them).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5ee}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for c in 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof_c$c -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 6 --warmup 2 --config $c > $O/prof_c$c.log 2>&1 || { tail -20 $O/prof_c$c.log; exit 1; }
done
echo done
