#!/bin/bash
# descent cap for the primaries of the fused AO kernel (the 4-wide AO descents ignore it), C3 / C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/dcap}; mkdir -p $OUT
V='[{"name":"default"},{"name":"dcap 8","descent_cap":8},{"name":"dcap 16","descent_cap":16},{"name":"dcap 4","descent_cap":4},{"name":"default again"}]'
for rep in 1 2; do
  for s in hf10M hf1M; do
    for B in 20 1; do
      echo "== $s batch $B rep $rep" | tee -a $OUT/ab.log
      VRH_AB="$V" VRH_AB_BATCH=$B timeout -k 10 300 python tools/ab_variants.py $s 3 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.log
      rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
    done
  done
done
