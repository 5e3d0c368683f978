#!/bin/bash
# bench C2 + rocprofv3 kernel stats of C2/C3/C4 (tools/gpu_r3.sh without tests or PMC)
CFGS="2 3 4" bash tools/gpu_r3.sh ${PTAG:-t8}
