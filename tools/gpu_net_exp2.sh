#!/bin/bash
# Net-pass variants: parity subset with each variant library, then kernel time on C2 / C4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/netexp2
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
show() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$1', d['ms_per_step'], r.get('kernel_ms_median'), r['frac'])"; }
for lib in pktvisor_amd/variants/libpvgpu_*.so; do
  v=$(basename $lib .so)
  PVGPU_LIB=$lib timeout -k 10 300 python3 -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "synthetic or fixture or edge" > $O/${v}_par.log 2>&1 || { echo "$v parity FAIL"; tail -5 $O/${v}_par.log; exit 1; }
  tail -1 $O/${v}_par.log
done
for c in ${CFGS:-2 4 3}; do
  for lib in pktvisor_amd/libpvgpu.so pktvisor_amd/variants/libpvgpu_*.so; do
    v=$(basename $lib .so)
    PVGPU_LIB=$lib timeout -k 10 200 $B --config $c > $O/${v}_c$c.json 2>$O/err.log || exit 1
    show $O/${v}_c$c.json
  done
done
