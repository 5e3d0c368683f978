#!/bin/bash
# Round 6 evidence A: the bench lines at HEAD (C2 as the driver runs it, with the CPU baseline and
# the end-to-end rates; C3 / C4 with a reset each step; C5 from host memory), then the world-8
# state merge (gloo, ranks sharing the GPU) on C5 and C2 shards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6final}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 1; }
grep '^{' $O/bench_c2.log | tail -1 | cut -c1-300
for c in 3 4; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 40 --warmup 3 --no-e2e --reset-each-step > $O/bench_c$c.log 2>&1 || { tail -5 $O/bench_c$c.log; exit 1; }
  grep '^{' $O/bench_c$c.log | tail -1 | cut -c1-200
done
timeout -k 10 400 python3 -u bench.py --config 5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log | tail -1 | cut -c1-200
timeout -k 10 400 python3 -u tools/merge_world8.py --world 8 --config 2 --records 80000000 > $O/merge_c2_w8.log 2>&1 || { tail -20 $O/merge_c2_w8.log; exit 1; }
tail -n 1 $O/merge_c2_w8.log | cut -c1-300
timeout -k 10 500 python3 -u tools/merge_world8.py --world 8 > $O/merge_world8.log 2>&1 || { tail -20 $O/merge_world8.log; exit 1; }
tail -n 1 $O/merge_world8.log | cut -c1-300
echo done
