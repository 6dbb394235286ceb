#!/bin/bash
# GPU: shading-related tests (whitted, shading, multi-hit, OBJ, C++ drop-ins) + shading-kernel throughput
mkdir -p gpurun_out
K="whitted or shading or multi_hit or obj or cpp" bash tools/gpu_tests.sh || exit $?
timeout -k 10 400 python -u tools/shade_bench.py > gpurun_out/shade_bench.jsonl 2> gpurun_out/shade_bench.err; rc=$?
cat gpurun_out/shade_bench.jsonl; exit $rc
