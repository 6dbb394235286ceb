#!/bin/bash
# Round-3 closing session on the final kernel sources.  STEPS (default "tests c3"):
#   tests  pytest -m gpu + smoke
#   c3     PMC passes of the driver's command shape (C3, 20 frames per launch) -> pmc_traffic_F20.json
#          (into profiles/ of this box copy too, so the bench line that follows reports achieved /
#          frac / traffic), the driver's command itself, and its rocprofv3 kernel trace
#   c4     the same passes for C4 (hf10M, 20 frames per launch) + L2 / TD passes, its bench line;
#          C2 and C5 bench lines
#   f32    the same PMC passes for the no-argument command (64 frames, 32 per launch), C3 and C4, and
#          their bench lines
# Every GPU step has its own time limit; after a fault / abort / timeout nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_close}
STEPS=${STEPS:-tests c3}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -${TAIL:-2} $OUT/$name.log | cut -c1-300; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  [ $rc = 0 ] || exit $rc
}
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
passes() {  # dir, command...
  local d=$1; shift
  step $(basename $d)_tcp 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD --output-format csv -d $d/pmc_bench_tcp -o run -- "$@"
  step $(basename $d)_hbm 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/pmc_bench_hbm -o run -- "$@"
  step $(basename $d)_wr 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/pmc_bench_wr -o run -- "$@"
}
Q="--no-cpu-baseline --single-frames 0 --moving-camera 0"
if has tests; then
  TAIL=6 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if has c3; then
  passes $OUT/c3_f20 python3 bench.py --steps 20 --warmup 5 $Q
  python3 tools/pmc_bench.py $OUT/c3_f20 $OUT/pmc_traffic_F20.json hf1M ao 20 "python3 bench.py --steps 20 --warmup 5 $Q" && cp $OUT/pmc_traffic_F20.json profiles/
  step bench 600 python3 bench.py --steps 20 --warmup 5
  cp $OUT/bench.log $OUT/bench_line.json
  step trace_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bench -o run -- python3 bench.py --steps 20 --warmup 5
fi
if has c4; then
  passes $OUT/c4_f20 python3 bench.py --scene hf10M --steps 20 --warmup 5 $Q
  step c4_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/c4_f20/mem/tcc -o run -- python3 bench.py --scene hf10M --steps 20 --warmup 5 $Q
  step c4_td 300 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/c4_f20/mem/td -o run -- python3 bench.py --scene hf10M --steps 20 --warmup 5 $Q
  python3 tools/pmc_bench.py $OUT/c4_f20 $OUT/pmc_traffic_F20_hf10M.json hf10M ao 20 "python3 bench.py --scene hf10M --steps 20 --warmup 5 $Q" && cp $OUT/pmc_traffic_F20_hf10M.json profiles/
  step bench_c4 600 python3 bench.py --scene hf10M --steps 20 --warmup 5 --no-cpu-baseline
  step bench_c2 600 python3 bench.py --scene hf1M --kernel primary --steps 20 --warmup 5 --no-cpu-baseline
  step bench_c5 600 python3 bench.py --scene sph1M --steps 20 --warmup 5 --no-cpu-baseline
fi
if has f32; then
  # the no-argument bench command (--steps 64 --warmup 32: two launches of 32 frames)
  passes $OUT/c3_f32 python3 bench.py --steps 64 --warmup 32 $Q
  python3 tools/pmc_bench.py $OUT/c3_f32 $OUT/pmc_traffic_F32.json hf1M ao 32 "python3 bench.py --steps 64 --warmup 32 $Q" && cp $OUT/pmc_traffic_F32.json profiles/
  passes $OUT/c4_f32 python3 bench.py --scene hf10M --steps 64 --warmup 32 $Q
  python3 tools/pmc_bench.py $OUT/c4_f32 $OUT/pmc_traffic_F32_hf10M.json hf10M ao 32 "python3 bench.py --scene hf10M --steps 64 --warmup 32 $Q" && cp $OUT/pmc_traffic_F32_hf10M.json profiles/
  step bench_f32 600 python3 bench.py
  step bench_c4_f32 600 python3 bench.py --scene hf10M --no-cpu-baseline
fi
exit 0
