#!/bin/bash
# Round 6: same-box A/B of the Net pass's general path: deferred to pv_net_slow_list (HEAD) vs the
# out-of-line call in the loop (variant inline), C2 interleaved twice; kernel stats of HEAD; the
# state merge at world 8 (gloo, ranks sharing the GPU) for the C5 stream and C2 shards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6k}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
run() { # name cfg lib
  local n=$1 c=$2 lib=$3; shift 3
  PVGPU_LIB=$lib timeout -k 10 300 python3 -u bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-e2e > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel"], r["kernel_ms"], r["frac"], d["ms_per_step"], d["ms_per_step_median"])')"
}
for k in 1 2; do
  run c2_head_$k 2 $R/pktvisor_amd/libpvgpu.so
  run c2_inline_$k 2 $V/libpvgpu_inline.so
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o k -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 2 > $O/prof_c2.log 2>&1) || { tail -20 $O/prof_c2.log; exit 1; }
echo "head $(python3 tools/kstats.py $O/prof_c2 2>/dev/null | cut -c1-300)"
timeout -k 10 400 python3 -u tools/merge_world8.py --world 8 --config 2 --records 80000000 > $O/merge_c2_w8.log 2>&1 || { tail -20 $O/merge_c2_w8.log; exit 1; }
tail -1 $O/merge_c2_w8.log
timeout -k 10 500 python3 -u tools/merge_world8.py --world 8 > $O/merge_world8.log 2>&1 || { tail -20 $O/merge_world8.log; exit 1; }
tail -1 $O/merge_world8.log
echo done
