#!/bin/bash
# Round 5: merge (PV_MG_U2=2) and names (PV_NWIN=128) tuning builds against the default: kernel
# stats on C2-C4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5l}; mkdir -p $O
export TMPDIR=/tmp
prof() {  # name config lib
  (cd /tmp && PVGPU_LIB=$3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1 -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config $2 > $O/prof_$1.log 2>&1) || { tail -20 $O/prof_$1.log; return 1; }
  echo "$1 $(python3 $R/tools/kstats.py $O/prof_$1 2>/dev/null | cut -c1-220)"
}
for c in 2 3 4; do
  prof base_c$c $c $R/pktvisor_amd/libpvgpu.so || exit 1
  prof mgu2_c$c $c $R/pktvisor_amd/variants/libpvgpu_mgu2.so || exit 1
  [ $c = 2 ] || prof nwin128_c$c $c $R/pktvisor_amd/variants/libpvgpu_nwin128.so || exit 1
done
echo done
