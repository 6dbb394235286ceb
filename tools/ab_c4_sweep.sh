#!/bin/bash
# C4 (hf10M AO, 20 frames per launch) launch-option sweep on the current build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/c4_sweep}; mkdir -p $OUT
V='[{"name":"default"},{"name":"stack 16","stack_cap":16},{"name":"stack 24","stack_cap":24},{"name":"refill 24","refill_min":24},{"name":"refill 40","refill_min":40},{"name":"block 128","block_threads":128},{"name":"block 256","block_threads":256}]'
for rep in 1 2; do
  for s in ${SCENES:-hf10M hf1M}; do
    echo "== $s rep $rep" | tee -a $OUT/ab.log
    VRH_AB="$V" VRH_AB_BATCH=20 timeout -k 10 400 python tools/ab_variants.py $s 3 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.log
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
  done
done
