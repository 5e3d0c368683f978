#!/bin/bash
# logical grid 3 vs 4 workgroups per CU on C2/C3/C4 kernel stats (tools/gpu_wgab.sh)
CFGS="2 3 4" bash tools/gpu_wgab.sh ${WTAG:-wg2} "3 4"
