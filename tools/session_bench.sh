#!/bin/bash
# Bench session: default bench (N=1, frames in flight 8), F=1 for comparison, the N>1 code path
# rehearsed with 2 ranks on this one GPU (gloo-staged gather), and a rocprofv3 kernel trace of the
# default bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2} | cut -c1-1500; echo "$name rc=$rc"; if fatal $rc; then exit $rc; fi; }
step bench 600 python bench.py
step bench_f1 300 python bench.py --frames-in-flight 1 --no-cpu-baseline
step bench_c4 300 python bench.py --scene hf10M --no-cpu-baseline --steps 16
step bench_g2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 16 --warmup 8 --dist-backend gloo
TAILN=1 step rocprof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline
exit 0
