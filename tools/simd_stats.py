"""SIMD utilisation of the traversal kernel from the counting variant (VRH_KERNEL_COUNT_TESTS):
lanes busy per refilling-loop step, active lanes per descent / leaf iteration, wave-uniform descents.

    python tools/simd_stats.py [scene] [ao|primary]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
kind = sys.argv[2] if len(sys.argv) > 2 else "ao"
prims = scenes.primitives(scene)
ctx = va.Context(0)
for opt in ("ao_gate", "wide_anyhit", "pop_on_miss", "descent_cap", "refill_min"):
    v = os.environ.get("VRH_" + opt.upper())
    if v is not None:
        ctx.set_option(opt, int(v))
dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
rt = va.hip_buffer_rt(ctx, W, H)
kern = (va.ao_kernel if kind == "ao" else va.closest_hit_kernel)(dev, count_tests=True)
va.render(ctx, dev, rt, cam.basis(W, H), kern, None, frame_num=0)
s = ctx.last_frame_stats()
out = {"scene": scene, "kernel": kind, "rays": s["rays"],
       "lanes_busy_per_step": s["busy_lane_steps"] / max(s["wave_steps"], 1),
       "active_lanes_per_descent_iter": (s["box_tests"] / 2) / max(s["wave_box_iters"], 1),
       "active_lanes_per_leaf_iter": s["prim_tests"] / max(s["wave_prim_iters"], 1),
       "uniform_descent_frac": s["wave_box_uniform_iters"] / max(s["wave_box_iters"], 1),
       "wave_steps_per_ray": s["wave_steps"] / s["rays"], "vmem_instrs_per_ray": s["vmem_instrs"] / s["rays"],
       "box_tests_per_ray": s["box_tests"] / s["rays"], "prim_tests_per_ray": s["prim_tests"] / s["rays"]}
print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}))
