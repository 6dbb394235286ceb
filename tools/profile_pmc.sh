#!/bin/bash
# rocprofv3 counter passes over tools/frame_driver.py (one counter group per pass, never combined
# with tracing domains).  Output under $OUTD/<pass>/ ; the summary is built by
# tools/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
SCENE=${SCENE:-hf1M}; FRAMES=${FRAMES:-4}; KIND=${KIND:-ao}; BATCH=${BATCH:-32}   # launches x frames per launch
OUTD=${OUTD:-gpurun_out/pmc}
mkdir -p $OUTD
rocprofv3 -L > $OUTD/counters_list.txt 2>&1 || true
run() {  # name, counters...
  local name=$1; shift
  echo "== pass $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUTD/$name -o run -- python3 tools/frame_driver.py $SCENE $FRAMES $KIND $BATCH > $OUTD/$name.log 2>&1
  local rc=$?; tail -2 $OUTD/$name.log; echo "rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
}
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUTD/trace -o run -- python3 tools/frame_driver.py $SCENE $FRAMES $KIND $BATCH > $OUTD/trace.log 2>&1 || exit $?
tail -1 $OUTD/trace.log
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM
run tcc TCC_HIT_sum TCC_MISS_sum
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
exit 0
