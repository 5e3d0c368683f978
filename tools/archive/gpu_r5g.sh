#!/bin/bash
# Round 5: the exact TCP LRU mode and the value-buffer tests (TCP / window subsets of the GPU
# suite), then the Net pass's lean-level attribution at one and two workgroups per CU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R5_DIR:-r5g}; mkdir -p $O
export TMPDIR=/tmp
[ -n "$NOTESTS" ] || timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tcp.py tests/test_gpu_tcp_limit.py tests/test_gpu_kat.py tests/test_gpu_bpf.py tests/test_gpu_windows.py \
  > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
[ -n "$NOTESTS" ] || tail -3 $O/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --config ${CFG:-2} --no-cpu-baseline --no-e2e > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; return 1; }
  echo "$name $(tail -1 $O/bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["kernel_ms"])')"
}
for L in 1 2 3 4; do
  run lean${L}_wg1 PVGPU_LIB=pktvisor_amd/variants/libpvgpu_lean$L.so || exit 1
  run lean${L}_wg2 PVGPU_LIB=pktvisor_amd/variants/libpvgpu_lean$L.so PV_NET_WGCU=2 || exit 1
done
run full_wg1 PV_X=0 && run full_wg2 PV_NET_WGCU=2 || exit 1
# C3: the DNS pass without Murmur blocks (what moving the qname CPC coupon off the per-message path could save)
CFG=3 run c3_base PV_X=0 && CFG=3 run c3_nomm PVGPU_LIB=pktvisor_amd/variants/libpvgpu_nomm.so || exit 1
(cd /tmp && PVGPU_LIB=$GRAFT_REPO_ROOT/pktvisor_amd/variants/libpvgpu_nomm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c3nomm -o k -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 10 --config 3 > $GRAFT_REPO_ROOT/$O/prof_c3nomm.log 2>&1) || exit 1
python3 tools/kstats.py $O/prof_c3nomm 2>/dev/null | cut -c1-200
echo done
