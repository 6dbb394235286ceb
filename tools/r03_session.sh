#!/bin/bash
# tools/r03_session.sh -- a round-3 GPU session.  Steps are chosen by the STEPS variable (space
# separated, default all):
#   tests   pytest -m gpu + smoke
#   bench   the driver's command (C3, --steps 20 --warmup 5) and C2 / C4 / C5 with the same shape
#   cpusweep  the reference tiled_sched CPU baseline at 16 / 64 / 128 / 256 threads (CPU only)
#   pmc     PMC passes of `bench.py --scene $PMC_SCENE --steps 20 --warmup 5` (tools/pmc_bench.py layout
#           + the memory-path passes of tools/profile_mem.sh) and its kernel trace
#   trace   rocprofv3 kernel trace of the driver's command
# Every GPU step has its own time limit; after a fault / abort / timeout nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03}
STEPS=${STEPS:-tests bench cpusweep pmc trace}
PMC_SCENE=${PMC_SCENE:-hf10M}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -${TAIL:-3} $OUT/$name.log | cut -c1-400; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  return 0
}
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
BENCH="--steps 20 --warmup 5"
if has tests; then
  TAIL=12 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if has bench; then
  step bench 600 python bench.py $BENCH
  for s in "hf1M --kernel primary" "hf10M" "sph1M"; do
    n=$(echo $s | cut -d' ' -f1)$(echo "$s" | grep -q primary && echo _primary)
    step bench_$n 600 python bench.py --scene $s $BENCH --no-cpu-baseline
  done
fi
if has cpusweep; then
  for t in 16 64 128 256; do
    step cpu_t$t 120 oracle/_ref/vsnray_ref_bench bench hf1M $t 3 1920 1080 8
  done
fi
if has pmc; then
  P="python3 bench.py --scene $PMC_SCENE $BENCH --no-cpu-baseline --single-frames 0"
  d=$OUT/pmc_${PMC_SCENE}
  step pmc_tcp 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD --output-format csv -d $d/pmc_bench_tcp -o run -- $P
  step pmc_hbm 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/pmc_bench_hbm -o run -- $P
  step pmc_wr 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/pmc_bench_wr -o run -- $P
  step pmc_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $d/mem/tcc -o run -- $P
  step pmc_td 600 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d $d/mem/td -o run -- $P
  step pmc_ta 600 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --output-format csv -d $d/mem/ta -o run -- $P
  step pmc_l1 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d $d/mem/tcp -o run -- $P
  step pmc_l1b 600 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD --output-format csv -d $d/mem/tcp2 -o run -- $P
  step trace_pmc_scene 600 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- $P
fi
if has trace; then
  step trace_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bench -o run -- python3 bench.py $BENCH
fi
exit 0
