#!/bin/bash
# User-kernel (AO lambda, C3) throughput of hip_kernels.h build variants, alternating, twice:
# user_kernels (default), uk_noscalar (VRH_USER_SCALAR_FETCH=0), uk_w5 / uk_w6 (VRH_USER_WAVES),
# uk_w5_noscalar, user_kernels_binary (VRH_USER_BINARY_ANYHIT=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/r03_user}; mkdir -p $OUT
for rep in 1 2; do
  for b in ${BINS:-user_kernels uk_noscalar uk_w5 uk_w5_noscalar uk_w6 user_kernels_binary}; do
    [ -x build/tests/$b ] || continue
    for F in 1 32; do
      L=20; [ $F = 32 ] && L=4
      r=$(timeout -k 10 120 build/tests/$b bench 708 1920 1080 /tmp $L $F | head -1) || exit 1
      echo "$b F=$F $r" | tee -a $OUT/user.log
    done
  done
done
