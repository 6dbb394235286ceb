set -e
D=gpurun_out/s11
T="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"
TD="TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
Q="--steps 20 --warmup 5 --no-cpu-baseline --single-frames 0 --moving-camera 0 --no-user-kernel --no-verify"
mkdir -p $D
timeout -k 10 120 rocprofv3 --pmc $T --output-format csv -d $D/lam_tcp -o run -- build/tests/user_kernels bench 708 1920 1080 /tmp 4 32 > $D/lam_tcp.log 2>&1
timeout -k 10 120 rocprofv3 --pmc $TD --output-format csv -d $D/lam_td -o run -- build/tests/user_kernels bench 708 1920 1080 /tmp 4 32 > $D/lam_td.log 2>&1
timeout -k 10 200 rocprofv3 --pmc $T --output-format csv -d $D/c3_tcp -o run -- python3 bench.py $Q > $D/c3_tcp.log 2>&1
timeout -k 10 200 rocprofv3 --pmc $TD --output-format csv -d $D/c3_td -o run -- python3 bench.py $Q > $D/c3_td.log 2>&1
echo done
