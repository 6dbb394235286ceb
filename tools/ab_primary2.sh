#!/bin/bash
# Second A/B round for primary visibility at 32 frames per launch: pop on miss / descent cap on the
# step loop (hf1M), refill threshold of the item loop (sph1M); also hf1M AO with pop on miss.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export VRH_AB_BATCH=32
export VRH_AB='[{"name": "default"}, {"name": "pop on miss", "pop_on_miss": 1}, {"name": "pop + cap 8", "pop_on_miss": 1, "descent_cap": 8}, {"name": "pop + cap 16", "pop_on_miss": 1, "descent_cap": 16}]'
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M 6 2>&1 | grep -v amdgpu.ids | tail -5 || exit 1
timeout -k 10 300 python tools/ab_variants.py hf1M 4 2>&1 | grep -v amdgpu.ids | tail -5 || exit 1
export VRH_AB='[{"name": "default (item, refill 16)"}, {"name": "refill 24", "refill_min": 24}, {"name": "refill 32", "refill_min": 32}, {"name": "refill 48", "refill_min": 48}, {"name": "refill 64", "refill_min": 64}, {"name": "vote", "ao_schedule": 5}, {"name": "vote refill 32", "ao_schedule": 5, "refill_min": 32}]'
timeout -k 10 300 python tools/ab_variants.py sph1M 6 2>&1 | grep -v amdgpu.ids | tail -8
