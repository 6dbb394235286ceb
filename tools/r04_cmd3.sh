#!/bin/bash
# round-4 GPU call: lane layout (VRH_OPT_QUAD_REFILL) and block-shared hand-out (VRH_OPT_GROUP_UNITS):
# parity, counting-kernel access model per variant, same-build timing A/B (static and orbiting camera),
# and this build against HEAD's
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04q
VC='[{"name":"default"},{"name":"q1","quad_refill":1},{"name":"q2","quad_refill":2},{"name":"q3","quad_refill":3}]'
V='[{"name":"default"},{"name":"q1","quad_refill":1},{"name":"q3","quad_refill":3},{"name":"b256","block_threads":256},{"name":"g256","block_threads":256,"group_units":20},{"name":"g256q3","block_threads":256,"group_units":20,"quad_refill":3},{"name":"g192","block_threads":192,"group_units":20},{"name":"g128","block_threads":128,"group_units":20}]'
OUT=gpurun_out/r04q K='schedules or batch' STEPS='tests' tools/r04_session.sh || exit 1
for s in hf1M hf10M; do
  VRH_AB="$VC" timeout -k 10 300 python tools/count_variants.py $s > gpurun_out/r04q/count_$s.log 2>&1 || exit 1
  grep name gpurun_out/r04q/count_$s.log
done
OUT=gpurun_out/r04q VRH_AB="$V" STEPS=ab ABTAIL=10 tools/r04_session.sh || exit 1
VRH_AB_ORBIT=0 LIBS="head cur" SCENES="hf10M hf1M" REPS=2 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/r04q/head_vs_cur.log 2>&1 || exit 1
grep -h "^default\|==" gpurun_out/r04q/head_vs_cur.log
