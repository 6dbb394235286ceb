#!/bin/bash
# tools/gpu_check.sh -- one GPU-box session: GPU tests, smoke, short bench (+ optional rocprof).
# Every GPU step has its own time limit; after a fault/abort/timeout nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }

echo "== pytest -m gpu"
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if fatal $rc; then echo "fatal pytest exit; stopping"; exit $rc; fi

echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -5 gpurun_out/smoke.log; echo "smoke rc=$rc"
if fatal $rc; then exit $rc; fi

echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; echo "bench rc=$rc"
if fatal $rc; then exit $rc; fi

if [ -n "$PROFILE" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; tail -3 gpurun_out/prof.log; echo "rocprof rc=$rc"
fi
exit 0
