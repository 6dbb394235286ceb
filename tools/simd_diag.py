"""SIMD utilisation of the traversal kernel (counting variant, VRH_KERNEL_COUNT_TESTS).

    python tools/simd_diag.py [scene ...]
Prints, per scene and kernel: rays, box / primitive tests per ray, and the fraction of the wave's
64 lanes doing useful work in the refilling loop (busy lanes), in the node-descent loop and in the
leaf loop.  Written to gpurun_out/simd_diag.log as well.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
log = open(os.path.join(ROOT, "gpurun_out", "simd_diag.log"), "a", buffering=1)


def say(*a):
    print(*a, flush=True)
    print(*a, file=log, flush=True)


ctx = va.Context(0)
if os.environ.get("VRH_AO_SCHEDULE"):
    ctx.set_option("ao_schedule", int(os.environ["VRH_AO_SCHEDULE"]))
for name in sys.argv[1:] or ["hf1M", "sph1M"]:
    prims = scenes.primitives(name)
    host = va.build_index_bvh(prims)
    dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
    cam, W, H = scenes.scene_camera(name)
    rt = va.hip_buffer_rt(ctx, W, H)
    kinds = [("primary", va.closest_hit_kernel(dev, count_tests=True))]
    if prims.dtype == va.TRIANGLE_DTYPE:
        kinds.append(("ao", va.ao_kernel(dev, count_tests=True)))
    for kname, k in kinds:
        va.render(ctx, dev, rt, cam.basis(W, H), k)
        s = ctx.last_frame_stats()
        rays = s["rays"]
        ws = max(s["wave_steps"], 1)
        say(f"{name:6s} {kname:7s} rays {rays} box/ray {s['box_tests'] / rays:.2f} prim/ray {s['prim_tests'] / rays:.2f} "
            f"| wave steps {ws} busy-lane util {s['busy_lane_steps'] / (64 * ws):.3f} "
            f"descent util {s['box_tests'] / 2 / max(64 * s['wave_box_iters'], 1):.3f} "
            f"leaf util {s['prim_tests'] / max(64 * s['wave_prim_iters'], 1):.3f} "
            f"| per wave step: descent iters {s['wave_box_iters'] / ws:.2f} leaf iters {s['wave_prim_iters'] / ws:.2f} "
            f"| one-node (uniform) descent iters {s['wave_box_uniform_iters'] / max(s['wave_box_iters'], 1):.3f}")
