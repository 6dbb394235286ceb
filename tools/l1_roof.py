#!/usr/bin/env python3
"""Turn the L1 roof microbenchmark's outputs into profiles/l1_roof.json (read by bench.py).

    python tools/l1_roof.py <l1_roof.log> <pmc run_counter_collection.csv> [out.json]

l1_roof.log: the JSON lines of tools/micro/l1_roof (timed without a profiler); the CSV: the same
binary under rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
SQ_INSTS_VMEM_RD (each mode = one warm-up dispatch + one timed dispatch, in mode order).

Per mode: L1 requests (TCP_TOTAL_CACHE_ACCESSES) per wave-level load, TD cycles per load, and the
request rate of the unprofiled run = wave loads/s x requests per load.  The roof of the traversal
kernel's access shape -- per-lane dependent 16-B loads of 64-B records, one chain per lane -- is
the highest request rate of the per-lane / pair / quad modes; bench.py prices it in GB/s of
16-B requests (one TCP access is one lane's 16-B piece for these shapes).
"""
import csv
import json
import sys
from collections import defaultdict

REQ_BYTES = 16
SHAPE_MODES = ("per-lane", "pair", "quad")     # the kernel's shape: one record per lane or shared by 2 / 4 lanes


def main():
    log, pmc = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/l1_roof.json"
    timed = [json.loads(l) for l in open(log) if l.startswith("{")]
    disp = defaultdict(dict)
    for r in csv.DictReader(open(pmc)):
        if not r["Kernel_Name"].startswith("chase"):
            continue
        disp[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(disp)
    modes = {}
    for i, t in enumerate(timed):
        c = disp[ids[2 * i + 1]]                       # the timed dispatch of mode i
        loads = c["SQ_INSTS_VMEM_RD"]
        per = c["TCP_TOTAL_CACHE_ACCESSES_sum"] / loads
        modes[t["mode"]] = {
            "wave_loads_per_s": t["wave_loads_per_s"],
            "tcp_accesses_per_load": round(per, 3),
            "td_cycles_per_load": round(c["TD_TD_BUSY_sum"] / loads, 3),
            "requests_per_s": t["wave_loads_per_s"] * per,
            "requests_per_cu_cycle": round(t["wave_loads_per_s"] * per / t["cus"] / (t["clock_mhz"] * 1e6), 4),
        }
    best = max(SHAPE_MODES, key=lambda m: modes[m]["requests_per_s"])
    peak = modes[best]["requests_per_s"]
    res = {
        "peak_requests_per_s": peak,
        "peak_gbs": round(peak * REQ_BYTES / 1e9, 1),
        "peak_mode": best,
        "request_bytes": REQ_BYTES,
        "table_mb": timed[0]["table_mb"], "waves_per_cu": timed[0]["waves_per_cu"],
        "modes": modes,
        "source": f"tools/micro/l1_roof.hip ({timed[0]['table_mb']} MB table, {timed[0]['waves_per_cu']} waves/CU) "
                  "timed + rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum SQ_INSTS_VMEM_RD",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: res[k] for k in ("peak_gbs", "peak_mode", "peak_requests_per_s")}))


if __name__ == "__main__":
    main()
