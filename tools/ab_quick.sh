#!/bin/bash
# Quick A/B with the variants in VRH_AB (no tests): hf1M AO, hf1M primary (PRIMARY=1),
# sph1M primary (SPH=1), hf10M AO (HF10M=1).
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_variants.py hf1M ${ROUNDS:-4} || exit $?
[ -n "$PRIMARY" ] && { VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M ${ROUNDS:-4} || exit $?; }
[ -n "$SPH" ] && { VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py sph1M ${ROUNDS:-4} || exit $?; }
[ -n "$HF10M" ] && { timeout -k 10 300 python tools/ab_variants.py hf10M 2 || exit $?; }
exit 0
