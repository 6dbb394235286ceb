#!/bin/bash
# round-4 GPU call: user-kernel tests (any_hit entry cut), user / reference-kernel benches with and
# without the cut, one-GPU shard scaling at the driver's shape (20 frames per launch) for C3 and C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04 gpurun_out/r04/shard
K=${K:-'user_kernels or ref_kernels'} STEPS='tests' tools/r04_session.sh && \
tools/r04_user.sh && \
for s in hf1M hf10M; do
  timeout -k 10 300 python tools/shard_scaling.py $s 5 ao 20 > gpurun_out/r04/shard/shard_${s}_f20.log 2>&1 || exit 1
  tail -5 gpurun_out/r04/shard/shard_${s}_f20.log | cut -c1-200
done
