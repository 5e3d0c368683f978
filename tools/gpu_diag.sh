#!/bin/bash
# Diagnose the torch HIP runtime on the box: device counts from torch and from libpvgpu.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
env | grep -E "HIP|ROCR|HSA|GPU|CUDA" | sort
timeout -k 10 120 python3 -c "
import torch
print('torch', torch.__version__, 'hip', torch.version.hip)
print('device_count', torch.cuda.device_count())
try:
    torch.cuda.init(); print('torch init ok', torch.cuda.get_device_name(0))
except Exception as e:
    print('torch init failed:', e)
" 2>&1 | tail -8
timeout -k 10 120 python3 -c "
import pktvisor_amd as pa
print('pv device_count', pa.device_count())
" 2>&1 | tail -3
timeout -k 10 60 python3 -c "
import pktvisor_amd as pa
print('pv first:', pa.device_count())
import torch
try:
    torch.cuda.init(); print('torch init after pv ok')
except Exception as e:
    print('torch init after pv failed:', e)
" 2>&1 | tail -3
