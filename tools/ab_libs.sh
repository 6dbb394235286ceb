#!/bin/bash
# Same-box A/B of several builds of libvrh (LIBS="a b c" -> visionaray_amd/_lib/libvrh_<x>.so;
# "cur" = libvrh.so): GPU parity tests on the current library first, then the default launch of
# every build on hf1M AO, hf1M primary and sph1M primary, builds interleaved by process, 2 reps.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; echo pytest=$rc
case $rc in 124|134|137|139) exit $rc;; esac
[ $rc -eq 0 ] || exit $rc
export VRH_AB=${VRH_AB:-'[{"name":"default"}]'}
for rep in 1 2; do
  for v in ${LIBS:-prev cur}; do
    if [ "$v" = cur ]; then lib=visionaray_amd/_lib/libvrh.so; else lib=visionaray_amd/_lib/libvrh_$v.so; fi
    echo "== $v rep $rep"
    VRH_LIB=$lib timeout -k 10 300 python tools/ab_variants.py hf1M 3 || exit $?
    VRH_LIB=$lib VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M 3 || exit $?
    VRH_LIB=$lib VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py sph1M 3 || exit $?
  done
done
[ -n "$DIAG" ] && { timeout -k 10 300 python tools/simd_diag.py || exit $?; }
exit 0
