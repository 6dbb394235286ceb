#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; echo pytest=$rc
case $rc in 124|134|137|139) exit $rc;; esac
export VRH_AB='[{"name":"xcd q, bpc max"},{"name":"global q, bpc max","xcd_queues":2},{"name":"xcd q, bpc 11","blocks_per_cu":11},{"name":"global q, bpc 11","xcd_queues":2,"blocks_per_cu":11},{"name":"xcd q, bpc 16","blocks_per_cu":16}]'
timeout -k 10 300 python tools/ab_variants.py hf1M 4 || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M 4 || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py sph1M 4 || exit $?
timeout -k 10 300 python tools/ab_variants.py hf10M 3 || exit $?
