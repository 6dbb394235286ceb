#!/bin/bash
# Needs a build with the cooperative fetch compiled in: make -C visionaray_amd variant NAME=coop DEFS=-DVRH_COOP=1, then run with VRH_LIB=visionaray_amd/_lib/libvrh_coop.so (the default build has it off).
# A/B of the cooperative pair fetch (VRH_OPT_COOP_FETCH) against the per-lane fetch, same process,
# interleaved rounds: hf1M AO, hf1M primary, hf10M AO.  The full GPU test suite first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
export VRH_AB='[{"name": "default"}, {"name": "coop", "coop_fetch": 1}, {"name": "coop+pop", "coop_fetch": 1, "pop_on_miss": 1}]'
timeout -k 10 200 python tools/ab_variants.py hf1M 3 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
VRH_AB_KERNEL=primary timeout -k 10 200 python tools/ab_variants.py hf1M 3 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
timeout -k 10 200 python tools/ab_variants.py hf10M 2 2>&1 | grep -v amdgpu.ids | tail -4
