"""Render K frames of one workload (no CPU baseline, no torch) -- the command profiled by rocprofv3.

    python tools/frame_driver.py [scene] [launches] [ao|primary] [frames per launch]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
kind = sys.argv[3] if len(sys.argv) > 3 else ("ao" if scene.startswith("hf") else "primary")
F = int(sys.argv[4]) if len(sys.argv) > 4 else 1
prims = scenes.primitives(scene)
host = va.build_index_bvh(prims)
ctx = va.Context(0)
for opt in ("waves_per_simd", "block_threads", "exact_minmax", "xcd_queues", "ao_schedule", "wide_anyhit",
            "refill_min", "descent_cap", "ao_gate", "pop_on_miss"):
    v = os.environ.get("VRH_" + opt.upper())
    if v is not None:
        ctx.set_option(opt, int(v))
dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
kern = va.ao_kernel(dev) if kind == "ao" else va.closest_hit_kernel(dev)
rt = va.hip_buffer_rt(ctx, W, H * F)
ctx.stats_reset()
for _ in range(frames):
    va.render_batch(ctx, dev, rt, [basis] * F, kern)
a = ctx.accum_stats()
print(f"{scene} {kind} launches {a['frames']} x {F} frames, mean kernel ms per launch "
      f"{a['kernel_ms_total'] / a['timed_frames']:.4f} Mrays/s {a['rays'] / a['kernel_ms_total'] / 1e3:.1f}")
