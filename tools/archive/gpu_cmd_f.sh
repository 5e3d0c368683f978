TESTS="tests/test_gpu_concurrency.py tests/test_afpacket_ring.py" bash tools/gpu_r4.sh f
cd $GRAFT_REPO_ROOT
for v in tst tstnoip; do
  PVGPU_LIB=$PWD/pktvisor_amd/variants/libpvgpu_$v.so PV_TSTAMPS=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > gpurun_out/r4_f/tst_$v.log 2>&1 || exit 1
  grep pv_tstamps gpurun_out/r4_f/tst_$v.log | tail -2
done
