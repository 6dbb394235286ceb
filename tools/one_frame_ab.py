"""One-frame launches (the hip_sched::frame shape) of a scene under launch-option variants: median
kernel ms over --frames synchronous frames per variant, alternating variants, --reps rounds.

    python tools/one_frame_ab.py [scene[:ao|primary]] [frames] [reps] [variant ...]
A variant is `name=opt:val,opt:val` (or `default`).
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene, _, kind = (sys.argv[1] if len(sys.argv) > 1 else "sph1M").partition(":")   # scene[:ao|primary]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 20
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
variants = {}
for v in (sys.argv[4:] or ["default"]):
    name, _, opts = v.partition("=")
    variants[name] = [(o.split(":")[0], int(o.split(":")[1])) for o in opts.split(",") if o]
prims = scenes.primitives(scene)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
kind = kind or ("ao" if scene.startswith("hf") else "primary")
kern = va.ao_kernel(dev) if kind == "ao" else va.closest_hit_kernel(dev)
rt = va.hip_buffer_rt(ctx, W, H)
res = {k: [] for k in variants}
fn = 1
for rep in range(reps):
    for name, opts in variants.items():
        for o, val in opts:
            ctx.set_option(o, val)
        va.render(ctx, dev, rt, basis, kern, None, frame_num=fn)
        fn += 1
        ms = []
        for _ in range(frames):
            va.render(ctx, dev, rt, basis, kern, None, frame_num=fn)
            fn += 1
            ms.append(ctx.last_frame_stats()["kernel_ms"])
        res[name].append(statistics.median(ms))
        for o, _ in opts:
            ctx.set_option(o, 0)
rays = ctx.last_frame_stats()["rays"]
out = {k: {"kernel_ms": [round(x, 4) for x in v], "mrays": round(rays / min(v) / 1e3, 1)} for k, v in res.items()}
print(json.dumps({"scene": scene, "kernel": kind, "frames": frames, "reps": reps, "variants": out}))
