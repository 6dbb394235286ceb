#!/bin/bash
# Shared any-hit walk (VRH_USER_ANYHIT_SHARE) on the user-kernel path: the user-kernel parity tests with
# the shared build, then the AO lambda (C3) throughput of the default and shared builds, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/user_share}; mkdir -p $OUT
VRH_USER_BIN=build/tests/uk_share timeout -k 10 300 python -u -m pytest tests/test_gpu_user_kernels.py -m gpu -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $OUT/pytest_share.log 2>&1; rc=$?; tail -3 $OUT/pytest_share.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT BINS="${BINS:-user_kernels uk_share}" bash tools/r03_user.sh
