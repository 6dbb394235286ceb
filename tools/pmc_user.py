#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes over a user-kernel program (hip_kernels.h user_render dispatches)
into profiles/pmc_user_<name>.json: per-launch counters, the vector-L1 request rate against the
kernel's own hipEvent-free trace time, and the split that says what holds the kernel.

    python tools/pmc_user.py <session dir> <out.json> <program> <frames per launch> [trace dir]

<session dir> holds one sub-directory per pass (pmc_tcp, pmc_hbm, pmc_wr, pmc_sq); the optional
trace dir a rocprofv3 --kernel-trace --stats run of the same command (mean dispatch duration).
Only dispatches whose kernel name contains "user_render" count; launches are averaged.

Derived (all per launch):
  l1_requests (TCP_TOTAL_CACHE_ACCESSES), TD busy fraction (TD_TD_BUSY / 256 CUs / GRBM_GUI_ACTIVE/8),
  HBM bytes (FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024, the gfx950 correction of bench's passes),
  VALU issue share (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: cycles a wave issues VALU work over its
  resident cycles), VALU instructions per wave, resident waves per launch.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_launch(d, match="user_render"):
    p = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}, None
    disp = defaultdict(dict)
    name = None
    for r in csv.DictReader(open(p)):
        if match not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        disp[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    agg = defaultdict(list)
    for c in disp.values():
        for k, v in c.items():
            agg[k].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}, name


def trace_ms(d, match="user_render"):
    p = os.path.join(d, "run_kernel_stats.csv")
    if not os.path.exists(p):
        return None
    for r in csv.DictReader(open(p)):
        if match in r["Name"]:
            return float(r["AverageNs"]) / 1e6
    return None


def main():
    d, out, prog, fpl = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    tdir = sys.argv[5] if len(sys.argv) > 5 else None
    c, name = {}, None
    for sub in sorted(os.listdir(d)):
        if os.path.isdir(os.path.join(d, sub)) and sub.startswith("pmc_"):
            v, n = per_launch(os.path.join(d, sub))
            c.update(v)
            name = name or n
    res = {"program": prog, "frames_per_launch": fpl, "kernel_name": name, "counters_per_launch": c}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from visionaray_amd.buildinfo import kernel_source_sha256, user_kernel_source_sha256
    res["kernel_source_sha256"] = kernel_source_sha256()
    res["user_kernel_source_sha256"] = user_kernel_source_sha256()
    ms = trace_ms(tdir) if tdir else None
    res["trace_ms_per_launch"] = ms
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
        res["l1_requests_per_launch"] = c["TCP_TOTAL_CACHE_ACCESSES_sum"]
        if c.get("SQ_INSTS_VMEM_RD"):
            res["l1_requests_per_vmem_load"] = c["TCP_TOTAL_CACHE_ACCESSES_sum"] / c["SQ_INSTS_VMEM_RD"]
    if "TD_TD_BUSY_sum" in c and "GRBM_GUI_ACTIVE" in c:
        cycles = c["GRBM_GUI_ACTIVE"] / 8.0
        res["kernel_cycles"] = cycles
        res["td_busy_frac"] = c["TD_TD_BUSY_sum"] / 256.0 / cycles
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        res["hbm_bytes_per_launch"] = c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024
    if c.get("SQ_WAVE_CYCLES"):
        if "SQ_ACTIVE_INST_VALU" in c:
            res["valu_issue_share"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
        if "SQ_ACTIVE_INST_VMEM" in c:
            res["vmem_issue_share"] = c["SQ_ACTIVE_INST_VMEM"] / c["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_INST_ANY" in c:
            res["wait_inst_share"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_WAVES"):
        res["waves_per_launch"] = c["SQ_WAVES"]
        if "SQ_INSTS_VALU" in c:
            res["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
    if ms and "l1_requests_per_launch" in res:
        res["l1_request_gbs"] = res["l1_requests_per_launch"] * 16 / (ms * 1e-3) / 1e9
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}))


if __name__ == "__main__":
    main()
