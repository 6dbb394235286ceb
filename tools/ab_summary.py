"""Summarise tools/ab_variants.py logs: per (scene, frames per launch, variant) the mean of the
per-round means and the best per-round minimum over all repetitions.

    python tools/ab_summary.py gpurun_out/refill/ab.log
Section headers are the "== <scene> batch <F> rep <r>" (or "== <lib> <scene> rep <r>") lines the
A/B scripts print; variant rows are ab_variants.py's table rows.
"""
import collections
import re
import sys


def main(path):
    cur = None
    res = collections.defaultdict(list)
    for line in open(path):
        if line.startswith("=="):
            cur = re.sub(r"\s*rep \d+\s*$", "", line[2:].strip())
            continue
        m = re.match(r"(\S.*?)\s{2,}([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s*$", line)
        if m and cur and m.group(1) != "variant":
            res[(cur, m.group(1))].append((float(m.group(2)), float(m.group(3))))
    for (sec, var), v in sorted(res.items()):
        means = [a for a, _ in v]
        print(f"{sec:28s} {var:24s} mean {sum(means) / len(means):8.4f} ms  best min {min(b for _, b in v):8.4f} ms  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
