#!/bin/bash
# round-4 GPU call: LDS copies of the AO cut entries' records (VRH_OPT_AO_CUT_RECORDS): parity, same-build
# A/B (on / off) and this build against HEAD's library, C3 / C4, static and orbiting camera
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04r
OUT=gpurun_out/r04r K='schedules or batch or parity or ao_cut or fuzz or group' STEPS='tests' tools/r04_session.sh || exit 1
V='[{"name":"crec_on"},{"name":"crec_off","ao_cut_records":2}]'
for o in 0 0.5; do
  VRH_AB="$V" VRH_AB_ORBIT=$o LIBS="cur" SCENES="hf10M hf1M" REPS=2 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/r04r/crec_o$o.log 2>&1 || exit 1
  VRH_AB_ORBIT=$o LIBS="head cur" SCENES="hf10M hf1M" REPS=2 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/r04r/head_o$o.log 2>&1 || exit 1
done
for o in 0 0.5; do echo "== orbit $o"; awk '/^== /{h=$2" "$3" "$5} /^crec|^default/{print h, $0}' gpurun_out/r04r/crec_o$o.log gpurun_out/r04r/head_o$o.log; done
