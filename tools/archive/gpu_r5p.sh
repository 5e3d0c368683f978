#!/bin/bash
# Round 5: period shifts in non-monotone batches (window / TCP / parity tests), the C5 ingest chunk
# size A/B, the TA / TCP counters of the C2 Net pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${R5_DIR:-r5p}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_windows.py tests/test_gpu_tcp.py tests/test_gpu_parity.py tests/test_gpu_deep_sampling.py tests/test_gpu_dnstap.py \
  > $O/tests.log 2>&1
trc=$?
tail -1 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head -20
[ $trc -le 1 ] || exit 1
for mb in 64 128 256; do
  PV_INGEST_CHUNK_MB=$mb timeout -k 10 600 python3 -u bench.py --config 5 --steps 2 --warmup 1 > $O/c5_chunk$mb.log 2>&1 || { tail -5 $O/c5_chunk$mb.log; continue; }
  echo "chunk $mb: $(tail -1 $O/c5_chunk$mb.log | cut -c1-260)"
done
R5_DIR=r5n bash tools/archive/gpu_r5n.sh
echo done
