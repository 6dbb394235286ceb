mkdir -p gpurun_out
K=obj bash tools/gpu_tests.sh && timeout -k 10 300 python tools/obj_bench.py --grid 1000 --gpu > gpurun_out/obj_bench.json 2> gpurun_out/obj_bench.err; rc=$?; cat gpurun_out/obj_bench.json; exit $rc
