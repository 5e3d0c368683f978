#!/bin/bash
# A/B of the Net pass: the round-1 tree (ab_r1/) and the current tree, same box, same command
set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do
  for t in ab_r1 .; do
    (cd $t && timeout -k 10 300 python bench.py --config ${CFG:-2} --steps 20 --warmup 3 --no-cpu-baseline --no-e2e) > gpurun_out/ab/$(basename $t)_$i.json 2>gpurun_out/ab/err.log || exit 1
  done
done
