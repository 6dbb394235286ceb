#!/bin/bash
# rocprofv3 counter passes over tools/frame_driver.py (one counter group per pass, never combined
# with tracing domains).  Output under gpurun_out/pmc/<pass>/ ; the summary is built by
# tools/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
SCENE=${SCENE:-hf1M}; FRAMES=${FRAMES:-4}; KIND=${KIND:-ao}; BATCH=${BATCH:-32}   # launches x frames per launch
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run() {  # name, counters...
  local name=$1; shift
  echo "== pass $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o run -- python3 tools/frame_driver.py $SCENE $FRAMES $KIND $BATCH > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; tail -2 gpurun_out/pmc/$name.log; echo "rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
}
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/trace -o run -- python3 tools/frame_driver.py $SCENE $FRAMES $KIND $BATCH > gpurun_out/pmc/trace.log 2>&1 || exit $?
tail -1 gpurun_out/pmc/trace.log
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM
run tcc TCC_HIT_sum TCC_MISS_sum
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
exit 0
