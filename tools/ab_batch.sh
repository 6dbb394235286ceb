#!/bin/bash
# Frames in flight: GPU test suite (incl. tests/test_gpu_batch.py), then shard scaling on one GPU
# for F = 1, 2, 4, 8 frames per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > gpurun_out/ab/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/ab/$name.log | tail -${TAILN:-6}; echo "$name rc=$rc"; if fatal $rc; then exit $rc; fi; }
TAILN=4 step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
for F in ${FS:-1 2 4 8}; do TAILN=5 step shard_F$F 300 python tools/shard_scaling.py ${SCENE:-hf1M} 6 ao $F; done
exit 0
