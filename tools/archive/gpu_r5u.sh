#!/bin/bash
# Round 5: load-pattern ceiling of the span pass vs the register-window pass (lean variants:
# 1 = loads + word XOR, 2 = + fast-path parse), C2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5u}; mkdir -p $O
export TMPDIR=/tmp
for v in 1 2; do
  for k in reg span; do
    if [ $k = span ]; then export PV_NET_KERNEL=span; else unset PV_NET_KERNEL; fi
    PVGPU_LIB=$R/pktvisor_amd/variants/libpvgpu_lean$v.so timeout -k 10 300 python3 -u bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/lean${v}_$k.log 2>&1 || { tail -5 $O/lean${v}_$k.log; exit 1; }
    echo "lean$v $k: $(grep '^{' $O/lean${v}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
  done
done
echo done
