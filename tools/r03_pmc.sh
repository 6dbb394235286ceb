#!/bin/bash
# Round-3 closing PMC + trace session on the final kernel sources (their hash goes into every
# profiles/pmc_traffic_*.json, bench.py checks it):
#   C3 hf1M at 32 frames per launch (the driver's default bench command, --steps 64) and at 20
#   (--steps 20); C4 hf10M at 32 frames per launch with the memory-path passes (profiles/r03_c4/after);
#   the rocprofv3 kernel trace of the driver's default command.
# One counter pass per rocprofv3 run (block limits: tools/profile_pmc.sh), each under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r03_pmc}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -2 $OUT/$name.log | cut -c1-300; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  [ $rc = 0 ] || exit $rc
}
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
  step $(basename $d)_ta 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --output-format csv -d $d/mem/ta -o run -- "$@"
  step $(basename $d)_l1 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d $d/mem/tcp -o run -- "$@"
  step $(basename $d)_l1b 300 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD --output-format csv -d $d/mem/tcp2 -o run -- "$@"
}
Q="--no-cpu-baseline --single-frames 0 --moving-camera 0"
[ -z "$SKIP_C3" ] && passes $OUT/c3_f32 python3 bench.py --steps 64 --warmup 32 $Q
[ -z "$SKIP_C3" ] && passes $OUT/c3_f20 python3 bench.py --steps 20 --warmup 5 $Q
[ -z "$SKIP_C4" ] && passes $OUT/c4_f32 python3 bench.py --scene hf10M --steps 64 --warmup 32 $Q
[ -z "$SKIP_C4" ] && mem $OUT/c4_f32 python3 bench.py --scene hf10M --steps 64 --warmup 32 $Q
[ -z "$SKIP_TRACE" ] && step trace_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bench -o run -- python3 bench.py
exit 0
