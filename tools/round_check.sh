#!/bin/bash
# GPU session: full GPU test suite, 1-GPU bench, 2-rank gloo rehearsal of the sharded bench.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; echo pytest=$rc
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1; rc=$?; tail -1 gpurun_out/bench1.log | cut -c1-300; echo bench=$rc
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 2 --dist-backend gloo > gpurun_out/bench2.log 2>&1; echo rc=$?; tail -1 gpurun_out/bench2.log | cut -c1-400
