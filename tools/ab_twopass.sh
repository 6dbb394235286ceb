#!/bin/bash
# Two-pass AO vs the fused step loop: parity under the two-pass schedules, then shard scaling
# (one GPU, every shard k of N) with a kernel trace of the two-pass passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > gpurun_out/ab/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/ab/$name.log | tail -${TAILN:-6}; echo "$name rc=$rc"; if fatal $rc; then exit $rc; fi; }
TAILN=3 step pytest_twopass 300 python -u -m pytest tests/test_gpu_schedules.py -k two_pass -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
VRH_AO_SCHEDULE=6 TAILN=5 step shard_twopass 200 python tools/shard_scaling.py hf1M 10 ao
VRH_AO_SCHEDULE=6 TAILN=1 step trace_twopass 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/trace -o run -- python3 tools/shard_scaling.py hf1M 10 ao
exit 0
