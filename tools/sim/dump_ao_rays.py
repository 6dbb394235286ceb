"""Dump the AO lambda's any_hit rays of sampled 8x8 tiles (C3: hf1M, 1920x1080) for tools/sim/oca_sim.c.

    python tools/sim/dump_ao_rays.py OUTDIR [tiles]

Primary hits come from the oracle (plain-C restatement, CPU); AO directions from the built-in counter
sampler (vrh_device.h ao_direction), so the rays are the built-in AO kernel's for frame 0 (not bit-exact
here -- this is a workload model for a schedule simulation, not a parity tool).  Writes:
  nodes.bin  (BVH_NODE_DTYPE), tris.bin (leaf-ordered TRIANGLE_DTYPE), rays.bin: per (tile, sample)
  64 records of 8 float32 (valid, ox, oy, oz, dx, dy, dz, max_t)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from oracle import oracle as O  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

out = sys.argv[1]
ntiles = int(sys.argv[2]) if len(sys.argv) > 2 else 400
os.makedirs(out, exist_ok=True)
name = "hf1M"
prims = scenes.primitives(name)
bvh = va.build_index_bvh(prims)
bvh.nodes.tofile(os.path.join(out, "nodes.bin"))
prims[bvh.indices].tofile(os.path.join(out, "tris.bin"))
nrm = scenes.normals_for(prims)
cam, W, H = scenes.scene_camera(name)
b = cam.basis(W, H)
eye, cu, cv, cw = (np.array(list(getattr(b, k)), np.float32) for k in ("eye", "cam_u", "cam_v", "cam_w"))
prim = O.render(O.make_scene(name), O.scene_camera(name), mode=O.VO_MODE_PRIMARY, threads=8)
pid = prim["prim_id"].reshape(H, W)
tt = prim["t"].reshape(H, W)
rng = np.random.default_rng(1)
tx, ty = W // 8, H // 8
cand = [(i, j) for j in range(ty) for i in range(tx) if (pid[j * 8:j * 8 + 8, i * 8:i * 8 + 8] != 0xFFFFFFFF).any()]
sel = [cand[k] for k in rng.choice(len(cand), size=min(ntiles, len(cand)), replace=False)]


def wang(a):
    a = (a ^ np.uint32(61)) ^ (a >> np.uint32(16))
    a = a + (a << np.uint32(3))
    a = a ^ (a >> np.uint32(4))
    a = a * np.uint32(0x27d4eb2d)
    return a ^ (a >> np.uint32(15))


def u01(k):
    return (wang(np.uint32(k)) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


recs = np.zeros((len(sel), 8, 64, 8), np.float32)
with np.errstate(over="ignore"):
    for n, (i, j) in enumerate(sel):
        for ly in range(8):
            for lx in range(8):
                x, y = i * 8 + lx, j * 8 + ly
                if pid[y, x] == 0xFFFFFFFF:
                    continue
                u = np.float32(2.0) * (np.float32(x) + np.float32(0.5)) / np.float32(W) - np.float32(1.0)
                v = np.float32(2.0) * (np.float32(y) + np.float32(0.5)) / np.float32(H) - np.float32(1.0)
                d = cu * u + cv * v + cw
                d = d / np.sqrt(np.dot(d, d))
                p = eye + d * tt[y, x]
                nn = nrm[pid[y, x]][:3].astype(np.float32)
                if abs(nn[0]) > abs(nn[1]):
                    bv = np.array([-nn[2], 0.0, nn[0]], np.float32)
                else:
                    bv = np.array([0.0, nn[2], -nn[1]], np.float32)
                bv = bv / np.sqrt(np.dot(bv, bv))
                bu = np.cross(bv, nn)
                pix = y * W + x
                for s in range(8):
                    sx = sy = 0.0
                    for k in range(16):
                        c = ((pix * 8 + s) * 16 + k) * 2
                        xa = 2.0 * u01(c) - 1.0
                        ya = 2.0 * u01(c + 1) - 1.0
                        if xa * xa + ya * ya < 1.0:
                            sx, sy = xa, ya
                            break
                    sz = np.sqrt(max(0.0, 1.0 - sx * sx - sy * sy))
                    dd = sx * bu + sy * bv + sz * nn
                    dd = dd / np.sqrt(np.dot(dd, dd))
                    o = p + dd * np.float32(1e-3)
                    recs[n, s, ly * 8 + lx] = (1.0, o[0], o[1], o[2], dd[0], dd[1], dd[2], 0.1)
recs.tofile(os.path.join(out, "rays.bin"))
print(f"{len(sel)} tiles, {int(recs[..., 0].sum())} AO rays, {len(bvh.nodes)} nodes -> {out}")
