#!/bin/bash
# GPU A/B session: parity tests first, then launch variants of one library (tools/ab_variants.py,
# VRH_AB overrides the variant list), then the SIMD-utilisation diagnostics of both schedules.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; echo pytest=$rc
case $rc in 124|134|137|139) exit $rc;; esac
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_variants.py hf1M ${ROUNDS:-4} || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M ${ROUNDS:-4} || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py sph1M ${ROUNDS:-4} || exit $?
[ -n "$HF10M" ] && { timeout -k 10 300 python tools/ab_variants.py hf10M 2 || exit $?; }
for s in 3 4; do VRH_AO_SCHEDULE=$s timeout -k 10 300 python tools/simd_diag.py || exit $?; done
exit 0
