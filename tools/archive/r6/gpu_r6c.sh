#!/bin/bash
# Round 6: net_probe with the writer-wave and reordered-store rungs; rocprofv3 kernel stats of the
# C2 bench with the product and with its loads-only build (no dispatch stamps in the way).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6c}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 tools/net_probe > $O/net_probe.log 2>&1 || { tail -20 $O/net_probe.log; exit 1; }
cat $O/net_probe.log
for v in full lean1; do
  L=$R/pktvisor_amd/libpvgpu.so; [ $v = lean1 ] && L=$R/pktvisor_amd/variants/libpvgpu_lean1.so
  (cd /tmp && PVGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 2 > $O/prof_$v.log 2>&1) || { tail -20 $O/prof_$v.log; exit 1; }
  python3 tools/kstats.py $O/prof_$v 2>/dev/null | cut -c1-300
done
echo done
