#!/usr/bin/env python3
"""Table of the traversal kernels' resource usage from `make asm` (-Rpass-analysis=kernel-resource-usage).

    python tools/resource_usage.py [visionaray_amd/_lib/asm/resource-usage.txt] [filter]
One line per render_unified_kernel instance: template arguments <KIND, AO, COUNT, OCC, EPI, LIST, BATCH,
SPILL, SAMPLED, SHARE>, VGPRs, VGPR spills, scratch bytes per lane, SGPRs, SGPR spills, occupancy.
"""
import re
import subprocess
import sys


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return out[:len(names)]


def parse(path):
    recs, cur = [], None
    for ln in open(path):
        m = re.search(r"remark: Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            recs.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\]| \[waves/SIMD\]| \[bytes/block\])?: (\S+) \[", ln)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return recs


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "visionaray_amd/_lib/asm/resource-usage.txt"
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    recs = parse(path)
    dm = demangle([r["name"] for r in recs])
    for r, d in zip(recs, dm):
        if "render_unified_kernel" not in d or filt not in d:
            continue
        args = d.split("render_unified_kernel<", 1)[1].split(">", 1)[0]
        print(f"<{args}>  VGPR {r.get('VGPRs')} spill {r.get('VGPRs Spill')} scratch {r.get('ScratchSize')} "
              f"SGPR {r.get('TotalSGPRs')} sspill {r.get('SGPRs Spill')} occ {r.get('Occupancy')}")


if __name__ == "__main__":
    main()
