#!/bin/bash
# Round-4 close of the user-kernel path: GPU tests, then the user-kernel throughput (tools/r04_user.sh)
# of the shipped programs with the cluster hand-out (VRH_USER_CLUSTER = 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04_user_final; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit $rc
BINS='build/tests/user_kernels build/tests/uk_share build/tests/uk_cut oracle/_ref/ref_kernels oracle/_ref/ref_kernels_share' \
  FS='1 32' REPS=2 OUT=$OUT bash tools/r04_user.sh
