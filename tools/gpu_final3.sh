#!/bin/bash
# Round-3 evidence: bench + rocprofv3 kernel stats of C2/C3/C4 and the PMC passes (HBM bytes,
# LDS, instruction mix) of the same three workloads, each under its own time limit.
PMC=1 PMC_CFGS="${PMC_CFGS:-2 3 4}" CFGS="2 3 4" bash tools/gpu_r3.sh ${PTAG:-final}
