# user-kernel throughput on hf10M (BVH 26 deep: the launch-sized stack) and hf1M, two builds alternating
set -e
for rep in 1 2; do
  for b in user_kernels uk_prev; do
    echo "hf10M $b $(timeout -k 10 300 build/tests/$b bench 2236 1920 1080 /tmp 3 32 | grep frame_ms)"
    echo "hf1M $b $(timeout -k 10 120 build/tests/$b bench 708 1920 1080 /tmp 4 32 | grep frame_ms)"
  done
done
