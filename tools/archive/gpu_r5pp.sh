#!/bin/bash
# Round 5: the per-step state merge for the bench's C2 shape (10M records per rank) at world 2
# and 8, ranks sharing one GPU over gloo (tools/merge_world8.py --config 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5pp}; mkdir -p $O
export TMPDIR=/tmp
for w in 2 8; do
  timeout -k 10 600 python3 -u tools/merge_world8.py --config 2 --world $w --records $((w * 10000000)) > $O/merge_c2_w$w.log 2>&1 || { tail -30 $O/merge_c2_w$w.log; exit 1; }
  grep '"tool"' $O/merge_c2_w$w.log | cut -c1-900
done
echo done
