#!/bin/bash
# AO tail stealing A/B against the round-2 library (libvrh_head.so) and the library without the
# stash code (libvrh_nosteal.so): register spills of the step loop vs the tail it removes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_steal2}
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
VRH_LIB=$L/libvrh_head.so VRH_AB='[{"name":"head"}]' VRH_AB_BATCH=20 step head_f20 200 python tools/ab_variants.py hf1M 5
VRH_LIB=$L/libvrh_head.so VRH_AB='[{"name":"head"}]' VRH_AB_BATCH=1 step head_f1 200 python tools/ab_variants.py hf1M 5
VRH_LIB=$L/libvrh_nosteal.so VRH_AB='[{"name":"nosteal lib","ao_steal":2}]' VRH_AB_BATCH=20 step nosteal_f20 200 python tools/ab_variants.py hf1M 5
VRH_LIB=$L/libvrh_nosteal.so VRH_AB='[{"name":"nosteal lib","ao_steal":2}]' VRH_AB_BATCH=1 step nosteal_f1 200 python tools/ab_variants.py hf1M 5
VRH_AB='[{"name":"steal on"},{"name":"steal off","ao_steal":2}]' VRH_AB_BATCH=20 step steal_f20 200 python tools/ab_variants.py hf1M 5
VRH_AB='[{"name":"steal on"},{"name":"steal off","ao_steal":2},{"name":"steal x2","ao_steal":32},{"name":"steal x0.5","ao_steal":8}]' VRH_AB_BATCH=1 step steal_f1 300 python tools/ab_variants.py hf1M 5
VRH_AB='[{"name":"steal on"},{"name":"steal off","ao_steal":2}]' VRH_AB_BATCH=1 step steal_f1_hf10M 300 python tools/ab_variants.py hf10M 3
step timeline 200 python tools/wave_timeline.py hf1M 1 20
step bench_default 400 python bench.py
TAIL=4 step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
exit 0
