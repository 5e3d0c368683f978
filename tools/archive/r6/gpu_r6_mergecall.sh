#!/bin/bash
# pv_topn_merge without device calls (probe build: the direct path and the name fallback compiled
# out) against the product build: C2 / C3 bench lines and rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r6mergecall; mkdir -p $O
export TMPDIR=/tmp
for v in main mnocall; do
  if [ $v = main ]; then L=$R/pktvisor_amd/libpvgpu.so; else L=$R/pktvisor_amd/variants/libpvgpu_$v.so; fi
  PVGPU_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 100 --no-e2e --no-cpu-baseline > $O/bench_c2_$v.log 2>&1 || { tail -5 $O/bench_c2_$v.log; exit 1; }
  echo "$v c2 $(grep '^{' $O/bench_c2_$v.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  PVGPU_LIB=$L timeout -k 10 300 python3 -u bench.py --config 3 --steps 30 --warmup 3 --no-e2e --no-cpu-baseline --reset-each-step > $O/bench_c3_$v.log 2>&1 || { tail -5 $O/bench_c3_$v.log; exit 1; }
  echo "$v c3 $(grep '^{' $O/bench_c3_$v.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  for c in 2 3; do
    PVGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c${c}_$v -o k -- python3 -u bench.py --config $c --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --reset-each-step > $O/prof_c${c}_$v.log 2>&1 || { tail -5 $O/prof_c${c}_$v.log; exit 1; }
    f=$(find $O/prof_c${c}_$v -name '*kernel_stats.csv' | head -1); cp $f $O/c${c}_kernel_stats_$v.csv
    grep -E 'pv_topn_merge|pv_topn_combine' $O/c${c}_kernel_stats_$v.csv | cut -d, -f1-5
  done
done
