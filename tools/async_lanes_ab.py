"""Asynchronous frames (VRH_OPT_ASYNC_FRAMES) with 2, 3 and 4 frame lanes: --frames back-to-back
hip_sched::frame calls into one shared target, one sync, the rate over the hipEvent span (bench.py's
single_frame_async shape), alternating the lane counts for --reps rounds; synchronous frames beside.

    python tools/async_lanes_ab.py [scene[:ao|primary]] [frames] [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene, _, kind = (sys.argv[1] if len(sys.argv) > 1 else "sph1M").partition(":")
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
kind = kind or ("ao" if scene.startswith("hf") else "primary")
prims = scenes.primitives(scene)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
kern = va.ao_kernel(dev) if kind == "ao" else va.closest_hit_kernel(dev)
rt = va.hip_buffer_rt(ctx, W, H)
sched = va.hip_sched(ctx)
res = {}
fn = 1
for rep in range(reps):
    for lanes in (0, 2, 3, 4):
        ctx.set_option("async_frames", lanes)
        for _ in range(max(lanes, 1)):                      # warm-up: every lane, scratch allocated
            sched.frame(kern, va.make_sched_params(cam, rt), frame_num=fn)
            fn += 1
        ctx.sync()
        ctx.stats_reset()
        for _ in range(frames):
            sched.frame(kern, va.make_sched_params(cam, rt), frame_num=fn)
            fn += 1
        ctx.sync()
        a = ctx.accum_stats()
        ms = a["span_ms"] if lanes else a["kernel_ms_total"]
        res.setdefault(lanes, []).append(round(a["rays"] / ms / 1e3, 1))
        ctx.set_option("async_frames", 0)
print(json.dumps({"scene": scene, "kernel": kind, "frames": frames, "reps": reps,
                  "mrays_by_lanes": {("sync" if k == 0 else str(k)): v for k, v in res.items()}}))
