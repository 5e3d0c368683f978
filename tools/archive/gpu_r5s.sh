#!/bin/bash
# Round 5: the span-load Net pass (PV_NET_KERNEL=span) against the register-window pass: parity
# tests under span, then C2 / C3 / C4 bench lines for both, and a kernel-trace of each on C2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5s}; mkdir -p $O
export TMPDIR=/tmp
PV_NET_KERNEL=span timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_tcp.py > $O/tests_span.log 2>&1
trc=$?
tail -1 $O/tests_span.log; grep -E "^(FAILED|ERROR)" $O/tests_span.log | head -20
[ $trc -le 1 ] || exit 1
for cfg in 2 3 4; do
  for k in reg span; do
    if [ $k = span ]; then export PV_NET_KERNEL=span; else unset PV_NET_KERNEL; fi
    timeout -k 10 300 python3 -u bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/c${cfg}_$k.log 2>&1 || { tail -5 $O/c${cfg}_$k.log; exit 1; }
    echo "C$cfg $k: $(tail -1 $O/c${cfg}_$k.log | cut -c1-330)"
  done
done
unset PV_NET_KERNEL
cd /tmp
for k in reg span; do
  if [ $k = span ]; then export PV_NET_KERNEL=span; else unset PV_NET_KERNEL; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$k -o run -- python3 $R/bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/prof_$k.log 2>&1 || { tail -5 $O/prof_$k.log; exit 1; }
  f=$(find $O/prof_$k -name '*kernel_stats.csv' | head -1); cp "$f" $O/c2_stats_$k.csv
  grep -E "pv_net|pv_dns_kernel\"|pv_topn" $O/c2_stats_$k.csv | cut -d, -f1-6
done
echo done
