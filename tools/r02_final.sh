#!/bin/bash
# tools/r02_final.sh -- the closing round-2 session on the committed tree: tools/r02_session.sh (GPU
# tests, smoke, the driver's bench command, PMC passes at 20 and 32 frames per launch, kernel trace;
# the L1 roof is not re-measured) and bench.py on C2 / C4 / C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export OUT=${OUT:-gpurun_out/r02_final} SKIP_MICRO=1
bash tools/r02_session.sh || exit $?
for s in "hf1M --kernel primary" "hf10M" "sph1M"; do
  n=$(echo $s | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --scene $s --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "bench $s failed"; exit 1; }
  cut -c1-160 $OUT/bench_$n.json
done
# the moving-camera leg (eye orbiting 0.5 deg per frame) on C3 and C4
for s in "hf1M" "hf10M"; do
  timeout -k 10 300 python bench.py --scene $s --steps 20 --warmup 5 --no-cpu-baseline --single-frames 0 --moving-camera 0.5 > $OUT/bench_moving_$s.json 2> $OUT/bench_moving_$s.err || { echo "bench moving $s failed"; exit 1; }
  cut -c1-160 $OUT/bench_moving_$s.json
done
exit 0
