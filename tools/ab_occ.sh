#!/bin/bash
mkdir -p gpurun_out
export VRH_AB='[{"name":"bpc 22 (max)"},{"name":"bpc 16","blocks_per_cu":16},{"name":"bpc 11","blocks_per_cu":11},{"name":"bpc 6","blocks_per_cu":6},{"name":"b256 bpc 5","block_threads":256,"blocks_per_cu":5},{"name":"b256 bpc 3","block_threads":256,"blocks_per_cu":3}]'
timeout -k 10 300 python tools/ab_variants.py hf1M 3 || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M 3 || exit $?
