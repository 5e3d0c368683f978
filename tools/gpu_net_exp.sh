#!/bin/bash
# Net-pass experiments: kernel time (bench's HIP-event median) per library variant and per
# PV_DEBUG_STAGES knob (1 staging only, 64 no histogram, 128 no IP log)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/netexp
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
show() { python3 -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$1', d['ms_per_step'], r.get('kernel_ms'), r.get('kernel_ms_median'), r['frac'])"; }
for c in ${CFGS:-2 4}; do
  for lib in pktvisor_amd/libpvgpu.so pktvisor_amd/variants/libpvgpu_*.so; do
    v=$(basename $lib .so)
    PVGPU_LIB=$lib timeout -k 10 200 $B --config $c > $O/${v}_c$c.json 2>$O/err.log || exit 1
    show $O/${v}_c$c.json
  done
done
for d in ${KNOBS:-1 64 128 192}; do
  PV_DEBUG_STAGES=$d timeout -k 10 200 $B --config 2 > $O/dbg${d}_c2.json 2>$O/err.log || exit 1
  show $O/dbg${d}_c2.json
done
