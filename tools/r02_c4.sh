#!/bin/bash
# C4 (hf10M primary + 8 AO, one GPU) before / after the round-2 AO defaults: PMC traffic and
# memory-path passes at 8 frames per launch (as the round-1 memory-path passes), then bench.py on C2, C4, C5.
# "before" = the round-1 AO settings (ao_gate off, binary any-hit records, no pop on miss).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02_c4
mkdir -p $O
for v in after before; do
  if [ $v = before ]; then export VRH_AO_GATE=2 VRH_WIDE_ANYHIT=2 VRH_POP_ON_MISS=2; else unset VRH_AO_GATE VRH_WIDE_ANYHIT VRH_POP_ON_MISS; fi
  SCENE=hf10M FRAMES=2 BATCH=8 OUTD=$O/$v bash tools/profile_pmc.sh || exit $?
  SCENE=hf10M FRAMES=2 BATCH=8 OUTD=$O/${v}_mem bash tools/profile_mem.sh || exit $?
done
unset VRH_AO_GATE VRH_WIDE_ANYHIT VRH_POP_ON_MISS
for s in "hf1M --kernel primary" "hf10M" "sph1M"; do
  n=$(echo $s | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --scene $s --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$n.log 2>&1 || { echo "bench $s failed"; exit 1; }
  tail -1 $O/bench_$n.log | cut -c1-200
done
exit 0
