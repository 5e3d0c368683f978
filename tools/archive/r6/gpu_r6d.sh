#!/bin/bash
# Round 6: is the IP-log store's cost the HBM write or the store instruction? (net_probe: plain read
# with a 1:20 write, the log to an L2-resident target, non-temporal record loads / log stores)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R6_DIR:-r6d}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 tools/net_probe > $O/net_probe.log 2>&1 || { tail -20 $O/net_probe.log; exit 1; }
cat $O/net_probe.log
