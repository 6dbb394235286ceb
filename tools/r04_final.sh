#!/bin/bash
# Round-4 closing session on the final kernel sources (their hash goes into every
# profiles/pmc_traffic_*.json; bench.py reports achieved / frac / traffic only for a matching pass).
# STEPS (default "tests pmc3 pmc4 bench trace"):
#   tests   pytest -m gpu + smoke
#   pmc3    C3 PMC passes at the driver's shape (F = 20) and the no-argument command (F = 32)
#   pmc4    the same for C4, plus the L2 / TD memory-path passes at F = 20
#   bench   the driver's command on C3 (with the CPU baseline), C4, C2, C5 and the no-argument command
#   trace   rocprofv3 kernel trace of the driver's command
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04_final}
STEPS=${STEPS:-tests pmc3 pmc4 bench trace}
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
mem() {  # dir, command...
  local d=$1; shift
  step $(basename $d)_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $d/mem/tcc -o run -- "$@"
  step $(basename $d)_td 300 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d $d/mem/td -o run -- "$@"
}
Q="--no-cpu-baseline --single-frames 0 --moving-camera 0"
if has tests; then
  TAIL=4 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if has pmc3; then
  passes $OUT/c3_f20 python3 bench.py --steps 20 --warmup 5 $Q
  python3 tools/pmc_bench.py $OUT/c3_f20 $OUT/pmc_traffic_F20.json hf1M ao 20 "python3 bench.py --steps 20 --warmup 5 $Q" && cp $OUT/pmc_traffic_F20.json profiles/
  passes $OUT/c3_f32 python3 bench.py --steps 64 --warmup 32 $Q
  python3 tools/pmc_bench.py $OUT/c3_f32 $OUT/pmc_traffic_F32.json hf1M ao 32 "python3 bench.py --steps 64 --warmup 32 $Q" && cp $OUT/pmc_traffic_F32.json profiles/
fi
if has pmc4; then
  passes $OUT/c4_f20 python3 bench.py --scene hf10M --steps 20 --warmup 5 $Q
  python3 tools/pmc_bench.py $OUT/c4_f20 $OUT/pmc_traffic_F20_hf10M.json hf10M ao 20 "python3 bench.py --scene hf10M --steps 20 --warmup 5 $Q" && cp $OUT/pmc_traffic_F20_hf10M.json profiles/
  mem $OUT/c4_f20 python3 bench.py --scene hf10M --steps 20 --warmup 5 $Q
  passes $OUT/c4_f32 python3 bench.py --scene hf10M --steps 64 --warmup 32 $Q
  python3 tools/pmc_bench.py $OUT/c4_f32 $OUT/pmc_traffic_F32_hf10M.json hf10M ao 32 "python3 bench.py --scene hf10M --steps 64 --warmup 32 $Q" && cp $OUT/pmc_traffic_F32_hf10M.json profiles/
fi
if has bench; then
  step bench 600 python3 bench.py --steps 20 --warmup 5
  step bench_c4 600 python3 bench.py --scene hf10M --steps 20 --warmup 5 --no-cpu-baseline
  step bench_c2 600 python3 bench.py --scene hf1M --kernel primary --steps 20 --warmup 5 --no-cpu-baseline
  step bench_c5 600 python3 bench.py --scene sph1M --steps 20 --warmup 5 --no-cpu-baseline
  step bench_f32 600 python3 bench.py --no-cpu-baseline
  step bench_shards8 600 python3 bench.py --steps 20 --warmup 5 --shards 8 --no-cpu-baseline
fi
if has trace; then
  step trace_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bench -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
fi
exit 0
