#!/bin/bash
# round-4 GPU call: full GPU tests on the reverted kernels, then block size of the AO batch launches
# (64 vs 128 vs 256 threads, same build) on C3 / C4 with a static and an orbiting camera, 3 repetitions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04b
OUT=gpurun_out/r04b STEPS='tests' tools/r04_session.sh || exit 1
V='[{"name":"b64"},{"name":"b128","block_threads":128},{"name":"b256","block_threads":256}]'
for o in 0 0.5; do
  VRH_AB="$V" VRH_AB_ORBIT=$o LIBS="cur" SCENES="hf10M hf1M" REPS=3 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/r04b/block_o$o.log 2>&1 || exit 1
done
for o in 0 0.5; do echo "== orbit $o"; awk '/^== /{h=$2" "$3" "$5} /^b64|^b128|^b256/{print h, $0}' gpurun_out/r04b/block_o$o.log; done
