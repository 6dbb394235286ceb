#!/bin/bash
# rocprofv3 counter passes on the vector-memory path (TA address unit, TD data unit, TCP L1,
# SQ VMEM levels) over tools/frame_driver.py; one counter group per pass, no tracing domains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
SCENE=${SCENE:-hf1M}; FRAMES=${FRAMES:-4}; KIND=${KIND:-ao}; BATCH=${BATCH:-32}; OUTD=${OUTD:-gpurun_out/pmc_mem}
mkdir -p $OUTD
run() {  # name, counters...
  local name=$1; shift
  echo "== pass $name: $*"
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d $OUTD/$name -o run -- python3 tools/frame_driver.py $SCENE $FRAMES $KIND $BATCH > $OUTD/$name.log 2>&1
  local rc=$?; tail -2 $OUTD/$name.log; echo "rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
}
run vmem SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM
run ta TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE
run td TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
run ta2 TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum
run tcp2 TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
run vmem2 SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_BUSY_CU_CYCLES
exit 0
