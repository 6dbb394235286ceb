#!/bin/bash
# round-4 GPU call: launch options re-swept under the cluster order (same build): AO refill threshold,
# cluster width; C3 / C4, static and orbiting camera
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04s
V='[{"name":"default"},{"name":"refill16","refill_min":16},{"name":"refill20","refill_min":20},{"name":"refill24","refill_min":24},{"name":"refill28","refill_min":28},{"name":"refill32","refill_min":32},{"name":"refill40","refill_min":40},{"name":"cl4","cluster_tiles":4},{"name":"cl16","cluster_tiles":16}]'
for o in 0 0.5; do
  VRH_AB="$V" VRH_AB_ORBIT=$o LIBS="cur" SCENES="hf10M hf1M" REPS=1 ROUNDS=4 bash tools/ab_builds.sh > gpurun_out/r04s/opts_o$o.log 2>&1 || exit 1
  echo "== orbit $o"; grep -v "parity\|^orbit\|^scene" gpurun_out/r04s/opts_o$o.log
done
