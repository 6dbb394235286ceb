#!/bin/bash
# whitted / simple / multi_hit throughput one frame per launch and with frames in flight, plus the
# whitted parity tests (round 3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/shade_batch}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_whitted.py -m gpu -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for F in 1 4 8; do
    timeout -k 10 300 python tools/shade_bench.py --occ 0 --frames 16 --frames-per-launch $F 2>&1 | grep -v amdgpu.ids \
      | tee -a $OUT/shade.jsonl; rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
  done
done
