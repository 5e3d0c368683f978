#!/bin/bash
# one line per variant dir of a gpu_iter run: ms/step and the main kernels' mean ms
D=$1; shift
for c in "$@"; do printf "%-9s " $c; grep -o '"ms_per_step": [0-9.]*' $D/$c.log | tr '\n' ' '
grep -E '^"(pv_[a-z_]+)"' $D/$c/k_kernel_stats.csv | awk -F, '$4>20000 {gsub("\"","",$1); printf "%s=%.3f ", $1, $4/1e6}'; echo; done
