#!/usr/bin/env python3
"""Per-library, per-variant table of an ab_builds.sh log: median of the per-rep mean ms and the best min ms.

    python tools/ab_table.py <log> [<log> ...]
"""
import re
import statistics
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    cur = None
    res = defaultdict(lambda: defaultdict(list))
    scene = None
    for ln in open(path):
        m = re.match(r"== (\S+) (\S+) rep (\d+)", ln)
        if m:
            cur, scene = m.group(1), m.group(2)
            continue
        p = ln.split()
        if cur and len(p) >= 5 and all(re.match(r"^[0-9.]+$", x) for x in p[-4:]) and not ln.startswith("variant"):
            name = " ".join(p[:-4])
            res[cur][name].append((float(p[-4]), float(p[-3])))
    print(f"{path} ({scene})")
    base = None
    for lib, vs in res.items():
        for name, vals in vs.items():
            mean = statistics.median(v[0] for v in vals)
            mn = min(v[1] for v in vals)
            if base is None:
                base = (mean, mn)
            print(f"  {lib:10s} {name:16s} mean {mean:.4f} ms ({(base[0] / mean - 1) * 100:+.1f} %)  "
                  f"min {mn:.4f} ms ({(base[1] / mn - 1) * 100:+.1f} %)  n={len(vals)}")
