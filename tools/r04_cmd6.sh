#!/bin/bash
# round-4 GPU call: LDS cut records -- where the slowdown comes from: HEAD, no records compiled in,
# 1 / 2 / 3 records per parity (LDS per wave 7.3 / 7.5 / 7.8 / 8.0 KB), C3 / C4 static camera
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04r
VRH_AB_ORBIT=0 LIBS="head nocrec crec1 crec2 cur" SCENES="hf10M hf1M" REPS=2 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/r04r/recs.log 2>&1 || exit 1
awk '/^== /{h=$2" "$3" "$5} /^default/{print h, $0} /grid/{print "   ", $0}' gpurun_out/r04r/recs.log
