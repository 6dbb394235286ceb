#!/bin/bash
# tools/r02_session.sh -- round-2 GPU session: GPU tests, smoke, the driver's bench command, the
# L1 roof microbenchmark (+ its PMC pass), a PMC pass and a kernel trace of the bench command.
# Every GPU step has its own time limit; after a fault / abort / timeout nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r02}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -${TAIL:-4} $OUT/$name.log; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  return 0
}
BENCH="--steps 20 --warmup 5"
if [ -z "$SKIP_TESTS" ]; then
  TAIL=30 step pytest_gpu 1200 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py $BENCH
if [ -z "$SKIP_MICRO" ]; then
  step l1_roof 300 tools/micro/l1_roof 16 20 2048
  step l1_roof_64 300 tools/micro/l1_roof 64 20 2048
  step pmc_l1_roof 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD --output-format csv -d $OUT/pmc_l1_roof -o run -- tools/micro/l1_roof 16 20 512
fi
if [ -z "$SKIP_PMC" ]; then
  # the driver's command (--steps 20: F = 20) and the default one (--steps 64: F = 32)
  for B in "$BENCH" ""; do
    d=$OUT/pmc_F$( [ -n "$B" ] && echo 20 || echo 32 )
    step $(basename $d)_tcp 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD --output-format csv -d $d/pmc_bench_tcp -o run -- python3 bench.py $B --no-cpu-baseline
    step $(basename $d)_hbm 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/pmc_bench_hbm -o run -- python3 bench.py $B --no-cpu-baseline
    step $(basename $d)_wr 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/pmc_bench_wr -o run -- python3 bench.py $B --no-cpu-baseline
  done
fi
step trace_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bench -o run -- python3 bench.py $BENCH
exit 0
