#!/bin/bash
# Round 5: transaction sort with 10 key bits per onesweep pass (7 passes over the 63 key bits) vs
# rocPRIM's default (8 bits, 8 passes): transaction parity tests under the variant, C4 / C3 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5jj}; mkdir -p $O
export TMPDIR=/tmp
V=$R/pktvisor_amd/variants
PVGPU_LIB=$V/libpvgpu_sort10.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_windows.py tests/test_gpu_tcp.py > $O/tests.log 2>&1
trc=$?
tail -1 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head -20
[ $trc -le 1 ] || exit 1
for cfg in 4 3; do
for k in 1 2; do
  for v in base sort10; do
    L=$R/pktvisor_amd/libpvgpu.so; [ $v = sort10 ] && L=$V/libpvgpu_sort10.so
    PVGPU_LIB=$L timeout -k 10 400 python3 -u bench.py --config $cfg --no-e2e --no-cpu-baseline > $O/c${cfg}_${v}_$k.log 2>&1 || { tail -20 $O/c${cfg}_${v}_$k.log; exit 1; }
    echo "C$cfg $v: $(grep '^{' $O/c${cfg}_${v}_$k.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_step_median"])')"
  done
done
done
echo done
