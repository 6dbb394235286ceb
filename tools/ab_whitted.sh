#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out/whit
timeout -k 10 300 python -u -m pytest tests/test_gpu_whitted.py tests/test_gpu_shading.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/whit/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/whit/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
 for lib in head cur; do
  if [ $lib = cur ]; then L=visionaray_amd/_lib/libvrh.so; else L=visionaray_amd/_lib/libvrh_$lib.so; fi
  echo "== $lib rep $rep"
  VRH_LIB=$L timeout -k 10 200 python tools/shade_bench.py --variants '[{"waves_per_simd":0},{"waves_per_simd":5}]' 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/whit/bench_$lib.jsonl; rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
 done
done
