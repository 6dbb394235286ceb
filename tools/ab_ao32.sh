#!/bin/bash
# A/B of step-loop knobs for AO (hf1M C3, hf10M C4) at 32 frames per launch, same process,
# interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export VRH_AB_BATCH=32
export VRH_AB='[{"name": "default"}, {"name": "pop", "pop_on_miss": 1}, {"name": "cap 16", "descent_cap": 16}, {"name": "cap 32", "descent_cap": 32}, {"name": "pop + cap 32", "pop_on_miss": 1, "descent_cap": 32}, {"name": "refill 24", "refill_min": 24}, {"name": "refill 40", "refill_min": 40}]'
timeout -k 10 300 python tools/ab_variants.py hf10M 3 2>&1 | grep -v amdgpu.ids | tail -8 || exit 1
timeout -k 10 300 python tools/ab_variants.py hf1M 4 2>&1 | grep -v amdgpu.ids | tail -8
