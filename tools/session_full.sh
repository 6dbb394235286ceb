#!/bin/bash
# Full measurement session: GPU tests, smoke, PMC passes (PMC=0 skips them), bench (default = C3)
# + other configs, rocprof kernel trace of the bench command.  Each GPU step has its own
# time limit; a fatal status (timeout, abort, segfault) ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2} | cut -c1-1200; echo "$name rc=$rc"; if fatal $rc; then exit $rc; fi; }
TAILN=4 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
# PMC passes first: their summaries (written into this copy's profiles/) are what bench.py reads
# for roofline.traffic / measured_limiter of the same workload
if [ "${PMC:-1}" != 0 ]; then
  TAILN=20 step pmc 900 bash tools/profile_pmc.sh
  TAILN=20 step pmc_mem 900 bash tools/profile_mem.sh
  python3 tools/pmc_summary.py gpurun_out/pmc profiles/pmc_traffic.json hf1M ao 32 > /dev/null || exit 1
  python3 tools/pmc_mem_summary.py gpurun_out/pmc_mem profiles/pmc_mem.json hf1M ao 32 > /dev/null || exit 1
fi
step bench 600 python bench.py
step bench_c2 300 python bench.py --kernel primary --no-cpu-baseline
step bench_c4 300 python bench.py --scene hf10M --no-cpu-baseline
step bench_c5 300 python bench.py --scene sph1M --no-cpu-baseline
TAILN=1 step rocprof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline
exit 0
