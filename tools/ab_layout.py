"""Same-process A/B of the pair-record layout (VRH_OPT_PAIR_LAYOUT, read at scene upload): builder
order vs depth-first line pairing, interleaved rounds, 32 frames per launch, with a parity check.

    python tools/ab_layout.py [scene] [rounds] [ao|primary]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
kind = sys.argv[3] if len(sys.argv) > 3 else "ao"
F = 32
prims = scenes.primitives(scene)
host = va.build_index_bvh(prims)
ctx = va.Context(0)
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
rt = va.hip_buffer_rt(ctx, W, H * F)
devs, res, outs = {}, {}, {}
for lay in (2, 1):
    ctx.set_option("pair_layout", lay)
    devs[lay] = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
    res[lay] = []
ctx.set_option("pair_layout", 0)
for rnd in range(rounds):
    for lay, dev in devs.items():
        kern = va.ao_kernel(dev) if kind == "ao" else va.closest_hit_kernel(dev)
        ctx.stats_reset()
        for _ in range(3):
            va.render_batch(ctx, dev, rt, [basis] * F, kern)
        a = ctx.accum_stats()
        res[lay].append(a["kernel_ms_min"] / F)
        if rnd == 0:
            o = rt.download()
            outs[lay] = (o["prim_id"][:W * H].copy(), o["t"][:W * H].copy(), o.get("occ", np.zeros(1))[:W * H].copy())
same = all(np.array_equal(x, y) for x, y in zip(outs[1], outs[2]))
for lay in (2, 1):
    print(f"{scene} {kind} layout {'builder order' if lay == 2 else 'line pairing '}: min {min(res[lay]):.4f} ms/frame "
          f"median {float(np.median(res[lay])):.4f}", flush=True)
print(f"identical frames: {same}", flush=True)
