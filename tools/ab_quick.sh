#!/bin/bash
# Quick A/B on hf1M AO (and hf10M AO if HF10M=1) with the variants in VRH_AB; no tests.
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_variants.py hf1M ${ROUNDS:-4} || exit $?
[ -n "$HF10M" ] && { timeout -k 10 300 python tools/ab_variants.py hf10M 2 || exit $?; }
exit 0
