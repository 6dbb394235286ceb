#!/bin/bash
# Round-4 GPU session steps.  STEPS (default "tests ab"):
#   tests    GPU tests selected by K (a pytest -k expression; all GPU tests when empty)
#   ab       same-box A/B of launch variants (VRH_AB json) on SCENES, static camera and ORBIT deg/frame
#   bench    the driver's command on C3 and C4 (--steps 20 --warmup 5)
#   smoke    __graft_entry__.smoke()
# Every GPU step has its own time limit; after a fault / abort / timeout nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04}
STEPS=${STEPS:-tests ab}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -${TAIL:-3} $OUT/$name.log | cut -c1-300; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  [ $rc = 0 ] || exit $rc
}
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  TAIL=8 step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${K:+-k "$K"}
fi
if has smoke; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if has ab; then
  for s in ${SCENES:-hf10M hf1M}; do
    for orbit in ${ORBITS:-0 0.5}; do
      TAIL=${ABTAIL:-8} VRH_AB_ORBIT=$orbit VRH_AB_BATCH=${BATCH:-20} VRH_AB_KERNEL=${KERNEL:-ao} \
        step ab_${s}_o${orbit}${TAG} 400 python tools/ab_variants.py $s ${ROUNDS:-3}
    done
  done
fi
if has bench; then
  step bench_c3 600 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
  step bench_c4 600 python3 bench.py --scene hf10M --steps 20 --warmup 5 --no-cpu-baseline
fi
exit 0
