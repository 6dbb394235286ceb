#!/bin/bash
# Same-box A/B of library builds x launch variants, no test suite (run the GPU tests separately).
#   LIBS="cur leafpipe"   builds: cur = _lib/libvrh.so, x = _lib/libvrh_x.so (make variant NAME=x)
#   SCENES="hf10M hf1M"   scenes (AO kernel unless KERNEL=primary)
#   VRH_AB=[...]          launch variants (tools/ab_variants.py), ROUNDS rounds each, REPS process reps
# Every step has its own time limit; a fatal exit stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export VRH_AB=${VRH_AB:-'[{"name":"default"}]'}
for rep in $(seq 1 ${REPS:-2}); do
  for s in ${SCENES:-hf10M hf1M}; do
    for v in ${LIBS:-cur}; do
      if [ "$v" = cur ]; then lib=visionaray_amd/_lib/libvrh.so; else lib=visionaray_amd/_lib/libvrh_$v.so; fi
      echo "== $v $s rep $rep"
      VRH_LIB=$lib VRH_AB_KERNEL=${KERNEL:-ao} VRH_AB_BATCH=${BATCH:-20} timeout -k 10 300 \
        python tools/ab_variants.py $s ${ROUNDS:-3} 2>&1 | grep -v amdgpu.ids
      rc=${PIPESTATUS[0]}
      [ $rc -eq 0 ] || { echo "fatal rc=$rc"; exit $rc; }
    done
  done
done
exit 0
