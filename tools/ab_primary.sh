#!/bin/bash
# A/B of launch knobs for primary visibility (hf1M closest-hit, sph1M item loop) at 32 frames per
# launch, same process, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export VRH_AB_BATCH=32
export VRH_AB='[{"name": "default"}, {"name": "5 waves/SIMD", "waves_per_simd": 5}, {"name": "8 waves/SIMD", "waves_per_simd": 8}, {"name": "scalar fetch off", "scalar_fetch": 2}, {"name": "descent cap 8", "descent_cap": 8}, {"name": "pop on miss", "pop_on_miss": 1}, {"name": "global queue", "xcd_queues": 2}]'
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M 4 2>&1 | grep -v amdgpu.ids | tail -9 || exit 1
export VRH_AB='[{"name": "default (item loop)"}, {"name": "item refill 8", "refill_min": 8}, {"name": "item refill 32", "refill_min": 32}, {"name": "step loop", "ao_schedule": 3}, {"name": "vote loop", "ao_schedule": 5}, {"name": "item 8 waves", "waves_per_simd": 8}, {"name": "item 5 waves", "waves_per_simd": 5}]'
timeout -k 10 300 python tools/ab_variants.py sph1M 4 2>&1 | grep -v amdgpu.ids | tail -9
