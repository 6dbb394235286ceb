"""Mean per-dispatch value of every counter in a rocprofv3 --pmc output tree, render kernels only.

    python tools/pmc_table.py gpurun_out/pmc_mem
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_mem"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if "render" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k:40s} {sum(v) / len(v):16.6g}   (n={len(v)})")
