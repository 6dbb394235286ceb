"""Summarise rocprofv3 --pmc passes of tools/profile_pmc.sh into profiles/<name>.json.

HBM traffic per launch of the traversal kernel = FETCH_SIZE + WRITE_SIZE (kB -> bytes), with the
gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE counts 128-B read requests at 64 B
(TCC_EA0_RDREQ x 64), so the read side is doubled; WRITE_SIZE is taken as is.  FETCH_SIZE counts
L2 misses towards the fabric, Infinity-Cache hits included, so it is an upper bound on DRAM bytes.

    python tools/pmc_summary.py gpurun_out/pmc profiles/pmc_traffic.json scene kernel [frames per launch]
"""
import csv
import json
import os
import sys
from collections import defaultdict


def load(d, name):
    p = os.path.join(d, name, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    agg = defaultdict(list)
    for r in csv.DictReader(open(p)):
        if "render" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    scene = sys.argv[3] if len(sys.argv) > 3 else "hf1M"
    kernel = sys.argv[4] if len(sys.argv) > 4 else "ao"
    fpl = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    c = {}
    for name in ("fetch", "write", "sq1", "sq2", "tcc", "lds"):
        c.update(load(d, name))
    res = {"scene": scene, "kernel": kernel, "gpus": 1, "frames_per_launch": fpl, "counters_per_dispatch": c}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        read = c["FETCH_SIZE"] * 1024 * 2
        write = c["WRITE_SIZE"] * 1024
        res["hbm_read_bytes_per_launch"] = read
        res["hbm_write_bytes_per_launch"] = write
        res["hbm_bytes_per_launch"] = read + write
        res["correction"] = "FETCH_SIZE x 1024 x 2 (gfx950 128-B requests tallied at 64 B) + WRITE_SIZE x 1024"
    if "TCC_HIT_sum" in c:
        res["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "SQ_WAVE_CYCLES" in c:
        res["wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        res["wait_inst_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
        res["active_inst_frac"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_dispatch"}))


if __name__ == "__main__":
    main()
