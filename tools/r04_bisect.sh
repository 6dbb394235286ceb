#!/bin/bash
# same-box A/B of kernel build variants (one change reverted each) on hf10M, static and orbiting camera
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04
export VRH_AB=${VRH_AB:-'[{"name":"default"},{"name":"band","xcd_queues":3}]'}
for o in ${ORBITS:-0.5 0}; do
  VRH_AB_ORBIT=$o LIBS="${LIBS:-r03 oall cur oput odiv owid ospill}" SCENES="${SCENES:-hf10M}" REPS=${REPS:-2} ROUNDS=3 \
    bash tools/ab_builds.sh > gpurun_out/r04/bisect_o$o.log 2>&1 || exit 1
done
