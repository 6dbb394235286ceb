#!/usr/bin/env python3
"""Summarise one rocprofv3 SQ counter pass (SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU) of the traversal kernel: the
frames-in-flight render_unified_kernel (built-in, default) or user_render (match=user_render).

    python tools/pmc_sq.py <pass dir> <out.json> <what> <frames per launch> <rays per frame> [match]

Per launch and per frame; the lane utilisation of the VALU work = SQ_THREAD_CYCLES_VALU (thread-cycles)
over 64 x SQ_ACTIVE_INST_VALU (wave-cycles), VALU wave-instructions per ray, the wave-cycle share spent
issuing VALU (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES) and waiting on an instruction dependency
(SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES), resident waves.
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_bench import batched  # noqa: E402


def main():
    d, out, what, fpl, rpf = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), float(sys.argv[5])
    match = sys.argv[6] if len(sys.argv) > 6 else None
    disp = defaultdict(dict)
    name = None
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = r["Kernel_Name"]
        if not (match in k if match else batched(k)):
            continue
        name = k
        disp[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    agg = defaultdict(list)
    for c in disp.values():
        for k, v in c.items():
            agg[k].append(v)
    c = {k: sum(v) / len(v) for k, v in agg.items()}
    rays = rpf * fpl
    res = {"what": what, "kernel_name": name, "frames_per_launch": fpl, "rays_per_launch": rays,
           "counters_per_launch": c,
           "lane_utilisation_valu": c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]),
           "valu_insts_per_ray": c["SQ_INSTS_VALU"] / rays,
           "salu_insts_per_ray": c["SQ_INSTS_SALU"] / rays,
           "valu_issue_share": c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"],
           "wait_inst_share": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
           "waves_per_launch": c["SQ_WAVES"]}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from visionaray_amd.buildinfo import kernel_source_sha256, user_kernel_source_sha256
    res["kernel_source_sha256"] = kernel_source_sha256()
    res["user_kernel_source_sha256"] = user_kernel_source_sha256()
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}))


if __name__ == "__main__":
    main()
