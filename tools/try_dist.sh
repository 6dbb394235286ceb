#!/bin/bash
mkdir -p gpurun_out
echo skip tests

timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench1.log 2>&1; tail -1 gpurun_out/bench1.log | cut -c1-200
echo "== torchrun 2 ranks on one GPU"
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo > gpurun_out/bench2.log 2>&1; echo rc=$?; tail -5 gpurun_out/bench2.log | cut -c1-400
