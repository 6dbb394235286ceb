"""Summarise tools/profile_mem.sh passes (vector-memory path) into profiles/<name>.json: busy
fractions of the TA (address) and TD (data) units, L1 accesses per wave-level load, L1 -> L2 miss
rate and L2 read latency, per launch of the traversal kernel.

    python tools/pmc_mem_summary.py gpurun_out/pmc_mem profiles/pmc_mem.json [scene kernel frames-per-launch]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_bench import batched  # noqa: E402


def counting(name):
    """render_unified_kernel<KIND, AO, COUNT, ...> with COUNT = true (bench.py's untimed counting pass)."""
    args = [a.strip() for a in name.split("render_unified_kernel<", 1)[1].split(">", 1)[0].split(",")]
    return len(args) > 2 and args[2] == "true"


def main():
    d, out = sys.argv[1], sys.argv[2]
    scene = sys.argv[3] if len(sys.argv) > 3 else "hf1M"
    kernel = sys.argv[4] if len(sys.argv) > 4 else "ao"
    fpl = int(sys.argv[5]) if len(sys.argv) > 5 else 8
    rows = []
    for name in sorted(os.listdir(d)):
        p = os.path.join(d, name, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        rows += [r for r in csv.DictReader(open(p)) if "render_unified_kernel" in r["Kernel_Name"]
                 and not counting(r["Kernel_Name"])]             # the traversal kernel, not the counting pass
    # over bench.py's command: only the frames-in-flight launches (the timed shape), as tools/pmc_bench.py
    if any(batched(r["Kernel_Name"]) for r in rows):
        rows = [r for r in rows if batched(r["Kernel_Name"])]
    agg = defaultdict(list)
    for r in rows:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: sum(v) / len(v) for k, v in agg.items()}
    cus = 256
    cycles = c["GRBM_GUI_ACTIVE"] / 8            # GRBM_GUI_ACTIVE is summed over the 8 XCDs
    res = {
        "scene": scene, "kernel": kernel, "gpus": 1, "frames_per_launch": fpl,
        "counters_per_dispatch": c,
        "kernel_cycles": cycles,
        "ta_busy_frac": c["TA_TA_BUSY_sum"] / (cus * cycles),
        "td_busy_frac": c["TD_TD_BUSY_sum"] / (cus * cycles),
        "l1_accesses_per_vmem_instr": c["TCP_TOTAL_CACHE_ACCESSES_sum"] / c["SQ_INSTS_VMEM_RD"],
        "l1_to_l2_reads_per_access": c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"],
        "l2_read_latency_cycles": c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"],
        "td_stalled_on_l1_frac": (c["TD_TC_STALL_sum"] / c["TD_TD_BUSY_sum"]) if "TD_TC_STALL_sum" in c else None,
        "l2_hit_frac": (c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])) if "TCC_HIT_sum" in c else None,
        "l1_pending_stall_frac": (c["TCP_PENDING_STALL_CYCLES_sum"] / (cus * cycles))
                                 if "TCP_PENDING_STALL_CYCLES_sum" in c else None,
        "note": "TA/TD busy = fraction of kernel cycles the vector-memory address / data units of the 256 CUs "
                "are busy; td_stalled_on_l1 = share of the TD busy cycles spent waiting for the L1 (TCP); "
                "l1_pending_stall = fraction of cycles the L1 stalls on outstanding misses",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_dispatch"}, indent=1))


if __name__ == "__main__":
    main()
