#!/bin/bash
# A/B: the tree in ab_r1/ (an earlier commit, built) and the current tree, same box, same command
set -o pipefail
mkdir -p gpurun_out/ab
for c in ${CFGS:-2}; do
for i in 1 2; do
  for t in ab_r1 .; do
    (cd $t && timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e) > gpurun_out/ab/$( [ $t = . ] && echo cur || echo base)_c${c}_$i.json 2>gpurun_out/ab/err.log || exit 1
  done
done
done
for f in gpurun_out/ab/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', d['ms_per_step'], d['roofline']['kernel_ms'])"; done
