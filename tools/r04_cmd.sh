#!/bin/bash
# round-4 GPU call: GPU tests (K filter), library A/B (round-3 library vs this tree) on C3 / C4 with a
# static and an orbiting camera, user / reference-kernel benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04
STEPS='tests' tools/r04_session.sh && \
tools/r04_user.sh && \
VRH_AB_ORBIT=0 LIBS="r03 cur" SCENES="hf10M hf1M" REPS=2 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/r04/ab_builds_o0.log 2>&1 && \
VRH_AB_ORBIT=0.5 LIBS="r03 cur" SCENES="hf10M hf1M" REPS=2 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/r04/ab_builds_o05.log 2>&1 && \
VRH_AB='[{"name":"default"},{"name":"band","xcd_queues":3},{"name":"cluster8","xcd_queues":4,"cluster_tiles":8},{"name":"strips","xcd_queues":1}]' KERNEL=primary SCENES="hf10M hf1M" STEPS=ab TAG=_primary tools/r04_session.sh
