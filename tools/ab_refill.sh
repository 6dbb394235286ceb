#!/bin/bash
# AO refill threshold (VRH_OPT_REFILL_MIN) around the default 32, C3 / C4, 20 and 1 frames per launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/refill}; mkdir -p $OUT
V='[{"name":"refill 32"},{"name":"refill 20","refill_min":20},{"name":"refill 24","refill_min":24},{"name":"refill 28","refill_min":28},{"name":"refill 32 again","refill_min":32}]'
for rep in 1 2 3; do
  for s in hf1M hf10M; do
    for B in 20 1; do
      echo "== $s batch $B rep $rep" | tee -a $OUT/ab.log
      VRH_AB="$V" VRH_AB_BATCH=$B timeout -k 10 300 python tools/ab_variants.py $s 3 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.log
      rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
    done
  done
done
