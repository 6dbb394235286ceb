#!/bin/bash
# AO tail stealing A/B (VRH_OPT_AO_STEAL): GPU tests, one-frame and 20-frame launches with the stash
# on / off, the launch timeline, the sharded rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_steal}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -${TAIL:-12} $OUT/$name.log | cut -c1-300; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  [ "$STOP_ON_FAIL" = 1 ] && [ $rc != 0 ] && exit $rc
  return 0
}
AB='[{"name":"steal on"},{"name":"steal off","ao_steal":2},{"name":"steal x2","ao_steal":32},{"name":"steal x0.5","ao_steal":8}]'
STOP_ON_FAIL=1 TAIL=6 step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
VRH_AB="$AB" VRH_AB_BATCH=1 step ab_f1_hf1M 300 python tools/ab_variants.py hf1M 5
VRH_AB="$AB" VRH_AB_BATCH=1 step ab_f1_hf10M 300 python tools/ab_variants.py hf10M 3
VRH_AB='[{"name":"steal on"},{"name":"steal off","ao_steal":2}]' VRH_AB_BATCH=20 step ab_f20_hf1M 300 python tools/ab_variants.py hf1M 5
step timeline 300 python tools/wave_timeline.py hf1M 1 20
step bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step bench_shards8 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --shards 8
exit 0
