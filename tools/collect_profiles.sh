#!/bin/bash
# Copy the results of tools/session_full.sh (gpurun_out/) into profiles/<name>/ and refresh the
# PMC summaries bench.py reads (profiles/pmc_traffic.json, profiles/pmc_mem.json).
#   bash tools/collect_profiles.sh r01_final_v3
cd "$(dirname "$0")/.." || exit 1
name=${1:?usage: collect_profiles.sh <name>}
D=profiles/$name
rm -rf "$D" && mkdir -p "$D/pmc" "$D/pmc_mem"
for f in bench bench_c2 bench_c4 bench_c5; do grep '^{' gpurun_out/$f.log | tail -1 > "$D/$f.json"; done
cp gpurun_out/prof/run_kernel_stats.csv "$D/bench_kernel_stats.csv"
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log "$D/"
for p in fetch write sq1 sq2 tcc lds; do cp gpurun_out/pmc/$p/run_counter_collection.csv "$D/pmc/$p.csv"; done
for p in vmem ta td ta2 tcp tcp2 vmem2; do
  [ -f gpurun_out/pmc_mem/$p/run_counter_collection.csv ] && cp gpurun_out/pmc_mem/$p/run_counter_collection.csv "$D/pmc_mem/$p.csv"
done
python3 tools/pmc_summary.py gpurun_out/pmc profiles/pmc_traffic.json hf1M ao 32 > /dev/null
python3 tools/pmc_mem_summary.py gpurun_out/pmc_mem profiles/pmc_mem.json hf1M ao 32 > /dev/null
python3 - "$D" <<'EOF'
import csv, sys
d = sys.argv[1]
rows = sorted(csv.DictReader(open('gpurun_out/prof/run_kernel_trace.csv')), key=lambda r: int(r['Start_Timestamp']))
with open(d + '/bench_launches.txt', 'w') as f:
    f.write("# every traversal launch of `python bench.py --no-cpu-baseline` under rocprofv3 --kernel-trace, in order\n")
    f.write("# (count pass, reference frame on the item loop, warm-up launches, a buffer-priming launch, the timed F-frame launches)\n")
    for r in rows:
        if 'render' in r['Kernel_Name']:
            f.write("%9.3f ms  %s\n" % ((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, r['Kernel_Name']))
EOF
echo "collected into $D"
