#!/bin/bash
# Same-box A/B: libvrh.so vs a build without the cooperative fetch compiled in (VRH_COOP=0,
# visionaray_amd/_lib/variant_nocoop.so): shading kernels, hf1M AO and primary; 2 interleaved reps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export VRH_AB='[{"name": "default"}]' VRH_AB_BATCH=32
for rep in 1 2; do
  for v in cur nocoop; do
    if [ $v = cur ]; then lib=visionaray_amd/_lib/libvrh.so; else lib=visionaray_amd/_lib/variant_nocoop.so; fi
    VRH_LIB=$lib timeout -k 10 200 python tools/shade_bench.py --frames 30 --variants '[{}]' 2>&1 | grep '^{' | sed "s/^/$v /" || exit 1
    VRH_LIB=$lib timeout -k 10 200 python tools/ab_variants.py hf1M 3 2>&1 | grep '^default' | sed "s/^/$v ao /" || exit 1
    VRH_LIB=$lib VRH_AB_KERNEL=primary timeout -k 10 200 python tools/ab_variants.py hf1M 3 2>&1 | grep '^default' | sed "s/^/$v primary /" || exit 1
  done
done
