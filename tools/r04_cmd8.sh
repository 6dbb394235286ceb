#!/bin/bash
# round-4 GPU call: the counting kernel's L1 access model by load kind (C3, C4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04k
for s in hf1M hf10M; do
  timeout -k 10 300 python tools/count_variants.py $s > gpurun_out/r04k/count_$s.log 2>&1 || exit 1
  grep name gpurun_out/r04k/count_$s.log
done
