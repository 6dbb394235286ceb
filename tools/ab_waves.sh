#!/bin/bash
# A/B of the unified kernel's register budget (VRH_OPT_WAVES_PER_SIMD 5 / 6 / 8 / none) and of the
# scalar fetch of wave-uniform pairs (VRH_OPT_SCALAR_FETCH), same process, interleaved rounds:
# hf1M AO, hf1M primary, hf10M AO, sph1M primary.  The schedule parity tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_schedules.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_sched.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sched.log; echo "pytest rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
export VRH_AB='[{"name": "default (6)"}, {"name": "5 waves/SIMD", "waves_per_simd": 5}, {"name": "8 waves/SIMD", "waves_per_simd": 8}, {"name": "no VGPR cap", "waves_per_simd": 1}, {"name": "scalar fetch off", "scalar_fetch": 2}, {"name": "5 waves, scalar off", "waves_per_simd": 5, "scalar_fetch": 2}]'
timeout -k 10 200 python tools/ab_variants.py hf1M 5 2>&1 | grep -v amdgpu.ids | tail -8 || exit 1
VRH_AB_KERNEL=primary timeout -k 10 200 python tools/ab_variants.py hf1M 5 2>&1 | grep -v amdgpu.ids | tail -8 || exit 1
timeout -k 10 200 python tools/ab_variants.py hf10M 3 2>&1 | grep -v amdgpu.ids | tail -8 || exit 1
timeout -k 10 200 python tools/ab_variants.py sph1M 3 2>&1 | grep -v amdgpu.ids | tail -8
