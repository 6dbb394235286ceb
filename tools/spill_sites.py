#!/usr/bin/env python3
"""Scratch spill / reload sites of one kernel instance in `make asm` output, with a few lines of context.

    python tools/spill_sites.py <mangled-name-substring> [context lines] [asm file]
"""
import sys

key = sys.argv[1]
ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 6
path = sys.argv[3] if len(sys.argv) > 3 else "visionaray_amd/_lib/asm/vrh_kernels.s"
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(key) and l.split(";")[0].rstrip().endswith(":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
sites = [i for i, l in enumerate(body) if "scratch_" in l]
print(f"{lines[start]} {len(body)} lines, {len(sites)} scratch ops")
for i in sites:
    print(f"---- {i}")
    for l in body[max(0, i - ctx):i + 2]:
        if l.strip() and not l.strip().startswith(";"):
            print("   ", l.rstrip()[:120])
