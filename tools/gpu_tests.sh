#!/bin/bash
# GPU test suite only (optionally a -k filter in K)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log; echo pytest=$rc; exit $rc
