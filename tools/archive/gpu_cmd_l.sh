#!/bin/bash
# reg_tc Net pass + merge DMA prefetch: parity subset, C2 bench, kernel stats, phase stamps
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_m
mkdir -p $O
TESTS="tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_topn_bound.py tests/test_gpu_dns2.py" BENCH="2" PROF="2 3 4" bash tools/gpu_r4.sh m || exit 1
PVGPU_LIB=$PWD/pktvisor_amd/variants/libpvgpu_tst.so PV_TSTAMPS=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/tst.log 2>&1 || exit 1
grep pv_tstamps $O/tst.log | tail -1
export TMPDIR=/tmp
(cd /tmp && PV_NET_KERNEL=ring timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ring_c2 -o k -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 10 > $GRAFT_REPO_ROOT/$O/ring_c2.log 2>&1) || exit 1
python3 tools/kstats.py $O/ring_c2
