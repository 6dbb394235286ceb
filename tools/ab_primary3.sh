#!/bin/bash
# Third A/B round: descent cap sweep with pop on miss, hf1M primary, 32 frames per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export VRH_AB_BATCH=32
export VRH_AB='[{"name": "default"}, {"name": "pop", "pop_on_miss": 1}, {"name": "pop + cap 4", "pop_on_miss": 1, "descent_cap": 4}, {"name": "pop + cap 6", "pop_on_miss": 1, "descent_cap": 6}, {"name": "pop + cap 8", "pop_on_miss": 1, "descent_cap": 8}, {"name": "pop + cap 10", "pop_on_miss": 1, "descent_cap": 10}, {"name": "pop + cap 12", "pop_on_miss": 1, "descent_cap": 12}, {"name": "cap 8", "descent_cap": 8}]'
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M 6 2>&1 | grep -v amdgpu.ids | tail -9 || exit 1
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf10M 3 2>&1 | grep -v amdgpu.ids | tail -9
