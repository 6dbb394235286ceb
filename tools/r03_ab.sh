#!/bin/bash
# Round-3 A/B session: the round-2 library (libvrh_head.so, built from 9a6edd7's sources) against the
# current one at 1 and 20 frames per launch, the user-kernel throughput (4-wide any-hit walk vs the
# binary walk, one frame vs frames in flight), the default bench line and the GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_ab}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -${TAIL:-7} $OUT/$name.log | cut -c1-300; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  return 0
}
L=visionaray_amd/_lib
if [ -z "$SKIP_AB" ]; then
VRH_LIB=$L/libvrh_head.so VRH_AB='[{"name":"round-2 lib"}]' VRH_AB_BATCH=20 step head_f20 200 python tools/ab_variants.py hf1M 5
VRH_AB='[{"name":"current"}]' VRH_AB_BATCH=20 step cur_f20 200 python tools/ab_variants.py hf1M 5
VRH_LIB=$L/libvrh_head.so VRH_AB='[{"name":"round-2 lib"}]' VRH_AB_BATCH=1 step head_f1 200 python tools/ab_variants.py hf1M 5
VRH_AB='[{"name":"current"}]' VRH_AB_BATCH=1 step cur_f1 200 python tools/ab_variants.py hf1M 5
fi
if [ -z "$SKIP_USER" ]; then
step user_wide 120 build/tests/user_kernels bench 708 1920 1080 /tmp 20
step user_binary 120 build/tests/user_kernels_binary bench 708 1920 1080 /tmp 20
step user_wide_f32 120 build/tests/user_kernels bench 708 1920 1080 /tmp 4 32
fi
[ -z "$SKIP_BENCH" ] && step bench_default 400 python bench.py
TAIL=4 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
exit 0
