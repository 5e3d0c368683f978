#!/bin/bash
# Net-pass phase stamps (variant built with -DPV_STAMPS): mean cycles per wave per phase
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/stamps_${1:-x}
mkdir -p $O
export PVGPU_LIB=pktvisor_amd/variants/libpvgpu_st.so PV_STAMPS=1
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B > $O/c2.log 2>&1 &&
(export PV_DEBUG_STAGES=1; timeout -k 10 200 $B > $O/c2_s1.log 2>&1) &&
(export PV_DEBUG_STAGES=2; timeout -k 10 200 $B > $O/c2_s2.log 2>&1) &&
timeout -k 10 200 $B --config 4 --records 4000000 > $O/c4.log 2>&1
echo "chain exit $?"
