#!/bin/bash
# User-kernel throughput on C3 (hf1M grid 708, 1920x1080, primary + 8 AO rays per hit pixel): the
# restated AO lambda (build/tests/user_kernels: F = 1 the Appendix-A sample set, F > 1 the
# random_sampler lambda) and ao/main.cpp's own kernel through the reference's headers
# (oracle/_ref/ref_kernels), one frame per launch and F frames in flight, alternating, REPS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=${OUT:-gpurun_out/r04/user}; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for F in ${FS:-1 32}; do
    L=20; [ $F -gt 1 ] && L=4
    for b in ${BINS:-build/tests/user_kernels build/tests/uk_nocut oracle/_ref/ref_kernels oracle/_ref/ref_kernels_nocut}; do
      [ -x $b ] || continue
      case $b in
        *ref_kernels*) r=$(timeout -k 10 120 $b bench hf1M 1920 1080 $L $F) ;;
        *) r=$(timeout -k 10 120 $b bench 708 1920 1080 /tmp $L $F) ;;
      esac
      rc=$?; [ $rc = 0 ] || { echo "$b rc=$rc"; exit $rc; }
      echo "$(basename $b) F=$F $(echo "$r" | grep frame_ms_median)" | tee -a $OUT/user.log
    done
  done
done
