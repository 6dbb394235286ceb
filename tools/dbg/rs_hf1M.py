"""Diagnostic: where does the reference-header AO kernel miss hits at hf1M?"""
import os, subprocess, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O
g = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
ref = np.load(os.path.join(ROOT, "tests/golden/rs_hf1M_f1.npz"))
out = "/tmp/rsd"; os.makedirs(out, exist_ok=True)
for name, cmd in (("ref_kernels", [os.path.join(ROOT, "oracle/_ref/ref_kernels"), "ao", "hf1M", "1920", "1080", out, "1"]),):
    subprocess.run(cmd, check=True, timeout=120)
    c = np.fromfile(out + "/color.bin", np.float32).reshape(-1, 4)
    t = np.fromfile(out + "/t.bin", np.float32)
    hit = ~np.all(c == np.array([0.1, 0.2, 0.3, 1.0], np.float32), axis=1)
    rh = ref["ao_count"] != 255
    bad = np.nonzero(hit != rh)[0]
    print(name, "hits", hit.sum(), "ref", rh.sum(), "mismatch", len(bad), "gpu-miss-ref-hit", int((rh & ~hit).sum()))
    print("first bad pixels (x, y):", [(int(p % 1920), int(p // 1920)) for p in bad[:40]])
    print("colour of bad:", c[bad[:5]], "t:", t[bad[:5]])
ud = "/tmp/ukd"; os.makedirs(ud, exist_ok=True)
subprocess.run([os.path.join(ROOT, "build/tests/user_kernels"), "ao", "708", "1920", "1080", ud, "0"], check=True, timeout=120)
pid = np.fromfile(ud + "/prim_id.bin", np.uint32)
print("user_kernels standalone hf1M primid hash ok:", O.fnv1a(pid) == g["hf1M"]["primid_hash"], "hits", int((pid != 0xFFFFFFFF).sum()), "ref", g["hf1M"]["hits"])
