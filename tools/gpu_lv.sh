mkdir -p gpurun_out/r3_lv
timeout -k 10 120 ./tools/stream_probe > gpurun_out/r3_lv/probe.log 2>&1; cat gpurun_out/r3_lv/probe.log
CFGS=2 TAG=lv VARS="full:-:- l1:l1:- l2:l2:- l3:l3:- l4:l4:-" bash tools/gpu_var.sh || exit 1
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS --kernel-include-regex "pv_net.*" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_lv/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM --kernel-include-regex "pv_net.*" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_lv/pmc2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > /dev/null 2>&1
echo pmc $?
