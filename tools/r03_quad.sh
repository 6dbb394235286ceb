#!/bin/bash
# 4-wide record order A/B: breadth-first (libvrh.so) vs depth-first sibling groups (libvrh_qdfs.so),
# C3 / C4 at 20 frames per launch and C4 at 1, alternating libraries (one process each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_quad}; mkdir -p $OUT
L=visionaray_amd/_lib
run() { # name lib scene batch rounds
  VRH_LIB=$L/$2 VRH_AB="[{\"name\":\"$1\"}]" VRH_AB_BATCH=$4 timeout -k 10 300 python tools/ab_variants.py $3 $5 >> $OUT/$3_f$4.log 2>&1 || exit 1
  tail -1 $OUT/$3_f$4.log
}
for rep in 1 2; do
  run bfs libvrh.so hf10M 20 3 && run dfs libvrh_qdfs.so hf10M 20 3 &&
  run bfs libvrh.so hf1M 20 3 && run dfs libvrh_qdfs.so hf1M 20 3 || exit 1
done
run bfs libvrh.so hf10M 1 5 && run dfs libvrh_qdfs.so hf10M 1 5
grep -h parity $OUT/*.log | sort | uniq -c
