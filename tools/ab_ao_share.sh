#!/bin/bash
# AO tail sharing (VRH_OPT_AO_SHARE): parity tests, then one-frame and 20-frame launches of the
# round-3 head library (libvrh_head.so) against this build with sharing off / on, hf1M and hf10M.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/ao_share}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ao_share.py tests/test_gpu_ao_cut.py -m gpu -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for s in ${SCENES:-hf1M hf10M}; do
    for B in ${BATCHES:-1 20}; do
      echo "== head $s batch $B rep $rep" | tee -a $OUT/ab.log
      VRH_LIB=visionaray_amd/_lib/libvrh_head.so VRH_AB='[{"name":"default"}]' VRH_AB_BATCH=$B timeout -k 10 300 \
        python tools/ab_variants.py $s 3 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.log; rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
      echo "== cur $s batch $B rep $rep" | tee -a $OUT/ab.log
      VRH_AB='[{"name":"default"},{"name":"share","ao_share":1}]' VRH_AB_BATCH=$B timeout -k 10 300 \
        python tools/ab_variants.py $s 3 2>&1 | grep -v amdgpu.ids | tee -a $OUT/ab.log; rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
    done
  done
done
