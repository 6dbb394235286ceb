#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes over the bench command into profiles/pmc_traffic_F<F>.json
(one file per frames-per-launch value F; bench.py reads the one of its own F).

    python tools/pmc_bench.py <session dir> [out.json] [scene] [kernel] [frames per launch] [command]

<session dir> holds one sub-directory per counter pass (tools/session.sh pmc:<cfg>: pmc_bench_tcp =
TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD, pmc_bench_hbm =
FETCH_SIZE, pmc_bench_wr = WRITE_SIZE).  Only the dispatches of the timed kernel are used: the
frames-in-flight instantiation render_unified_kernel<..., BATCH = true> (its launches all have the
same frame count), averaged per launch.

HBM traffic per launch = FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024 (MI355X_MICROARCH.md §HBM: on
gfx950 FETCH_SIZE tallies 128-B read requests at 64 B; FETCH_SIZE counts L2 misses towards the
fabric, Infinity-Cache hits included, so it bounds DRAM bytes from above).
"""
import csv
import json
import os
import sys
from collections import defaultdict


def batched(name):
    """render_unified_kernel<KIND, AO, COUNT, OCC, EPI, LIST, BATCH[, SPILL]> with BATCH = true."""
    if "render_unified_kernel<" not in name:
        return False
    args = [a.strip() for a in name.split("render_unified_kernel<", 1)[1].split(">", 1)[0].split(",")]
    return len(args) >= 7 and args[6] == "true"


def per_launch(d):
    p = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}, None
    disp = defaultdict(dict)
    name = None
    for r in csv.DictReader(open(p)):
        if not batched(r["Kernel_Name"]):
            continue
        name = r["Kernel_Name"]
        disp[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    agg = defaultdict(list)
    for c in disp.values():
        for k, v in c.items():
            agg[k].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}, name


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
    scene = sys.argv[3] if len(sys.argv) > 3 else "hf1M"
    kernel = sys.argv[4] if len(sys.argv) > 4 else "ao"
    fpl = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    cmd = sys.argv[6] if len(sys.argv) > 6 else "python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline"
    c, name = {}, None
    for sub in ("pmc_bench_tcp", "pmc_bench_hbm", "pmc_bench_wr"):
        v, n = per_launch(os.path.join(d, sub))
        c.update(v)
        name = name or n
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from visionaray_amd.buildinfo import kernel_source_sha256
    res = {"scene": scene, "kernel": kernel, "gpus": 1, "frames_per_launch": fpl, "kernel_name": name,
           "command": cmd, "counters_per_launch": c, "kernel_source_sha256": kernel_source_sha256()}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        read = c["FETCH_SIZE"] * 1024 * 2
        write = c["WRITE_SIZE"] * 1024
        res["hbm_read_bytes_per_launch"] = read
        res["hbm_write_bytes_per_launch"] = write
        res["hbm_bytes_per_launch"] = read + write
        res["correction"] = "FETCH_SIZE x 1024 x 2 (gfx950 128-B requests tallied at 64 B) + WRITE_SIZE x 1024"
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
        res["l1_requests_per_launch"] = c["TCP_TOTAL_CACHE_ACCESSES_sum"]
        res["l1_requests_per_vmem_load"] = c["TCP_TOTAL_CACHE_ACCESSES_sum"] / c["SQ_INSTS_VMEM_RD"]
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs; TD_TD_BUSY_sum over the 256 CUs
        cycles = c["GRBM_GUI_ACTIVE"] / 8.0
        res["td_busy_frac"] = c["TD_TD_BUSY_sum"] / 256.0 / cycles
        res["kernel_cycles"] = cycles
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}))


if __name__ == "__main__":
    main()
