#!/bin/bash
# Round-3 measurement session: the driver's bench command (defaults), C4, the one-GPU render-group
# rehearsal (--shards 8 / 3) against the unsharded line, the shading kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_measure}; mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -1 $OUT/$name.log | cut -c1-400; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  return 0
}
step bench 400 python bench.py
step bench_c4 300 python bench.py --scene hf10M --no-cpu-baseline
step bench_shards8 300 python bench.py --shards 8 --no-cpu-baseline
step bench_shards3 300 python bench.py --shards 3 --no-cpu-baseline
step bench_c2 200 python bench.py --kernel primary --no-cpu-baseline
step bench_c5 200 python bench.py --scene sph1M --no-cpu-baseline
step shade 300 python tools/shade_bench.py --occ 0 --frames 10
exit 0
