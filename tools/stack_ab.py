"""Same-box A/B of the AO kernel's LDS stack capacity (VRH_OPT_STACK_CAP) at the driver's shape
(20 frames per launch): per cap, the mean kernel ms per frame over --launches launches, and with
rocprofv3 --pmc the wave-level vector loads per launch (the load-count model).  Entries beyond the cap
go to the global overflow block -- buffer loads / stores, i.e. vector memory instructions -- so a deep
BVH (hf10M: depth 26) pays loads for what a larger LDS part would keep on chip, at fewer waves per CU.

    python tools/stack_ab.py [scene] [caps, comma-separated; 0 = auto] [launches]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf10M"
caps = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "0,20,24,28").split(",")]
launches = int(sys.argv[3]) if len(sys.argv) > 3 else 10
F = 20
prims = scenes.primitives(scene)
host = va.build_index_bvh(prims)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
kern = va.ao_kernel(dev)
rt = va.hip_buffer_rt(ctx, W, H * F)
out = {"scene": scene, "depth": int(host.max_depth), "frames_per_launch": F, "launches": launches, "caps": {}}
fn = 1
for cap in caps:
    ctx.set_option("stack_cap", cap)
    for _ in range(3):                                   # warm-up (and clock ramp)
        va.render_batch(ctx, dev, rt, [basis] * F, kern, None, frame_num=fn)
        fn += F
    ctx.sync()
    ctx.stats_reset()
    for _ in range(launches):
        va.render_batch(ctx, dev, rt, [basis] * F, kern, None, frame_num=fn)
        fn += F
    ctx.sync()
    a = ctx.accum_stats()
    out["caps"][cap] = {"ms_per_frame": round(a["kernel_ms_total"] / a["timed_frames"] / F, 4),
                        "mrays": round(a["rays"] / a["kernel_ms_total"] / 1e3, 1)}
    print(f"stack_cap {cap}: {out['caps'][cap]}", flush=True)
ctx.set_option("stack_cap", 0)
print(json.dumps(out))
