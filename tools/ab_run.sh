#!/bin/bash
# GPU A/B session: parity tests first, then launch variants (tools/ab_variants.py)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; echo pytest=$rc
case $rc in 124|134|137|139) exit $rc;; esac
export VRH_AB=${VRH_AB:-'[{"name":"unified occ1 fast"},{"name":"unified occ6 fast","waves_per_simd":6},{"name":"unified occ8 fast","waves_per_simd":8},{"name":"unified b256 fast","block_threads":256}]'}
timeout -k 10 300 python tools/ab_variants.py hf1M 5 || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M 5 || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py sph1M 5 || exit $?
timeout -k 10 300 python tools/ab_variants.py hf10M 3 || exit $?
