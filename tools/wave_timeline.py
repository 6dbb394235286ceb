"""Launch timeline of the traversal kernel from per-wave start / end stamps (VRH_OPT_WAVE_TIMES):
where a one-frame launch loses time against frames in flight -- the ramp-up (wave start spread)
and the tail (last wave end vs the median).

    python tools/wave_timeline.py [scene] [frames per launch ...]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
batches = [int(x) for x in sys.argv[2:]] or [1, 4, 20]
prims = scenes.primitives(scene)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
kern = va.ao_kernel(dev) if scene.startswith("hf") else va.closest_hit_kernel(dev)
frame = 1
for F in batches:
    rt = va.hip_buffer_rt(ctx, W, H * F)
    for rep in range(3):
        ctx.set_option("wave_times", 1 if rep == 2 else 0)
        va.render_batch(ctx, dev, rt, [basis] * F, kern, frame_num=frame)
        frame += F
    st = ctx.last_frame_stats()
    t = ctx.wave_times()
    start, end = t[:, 0], t[:, 1]
    q = lambda a, p: float(np.percentile(a, p))  # noqa: E731
    print(json.dumps({"scene": scene, "frames_per_launch": F, "kernel_ms": round(st["kernel_ms"], 4),
                      "waves": int(len(t)), "start_p50_ms": round(q(start, 50), 4), "start_max_ms": round(q(start, 100), 4),
                      "end_min_ms": round(q(end, 0), 4), "end_p10_ms": round(q(end, 10), 4), "end_p50_ms": round(q(end, 50), 4),
                      "end_p90_ms": round(q(end, 90), 4), "end_max_ms": round(q(end, 100), 4),
                      "busy_frac": round(float((end - start).sum() / (len(t) * end.max())), 4)}), flush=True)
