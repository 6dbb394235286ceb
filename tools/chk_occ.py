"""Diagnostic: the launch configuration (grid, stack) and kernel time of a 20-frame primary batch on a
scene, built the way bench.py builds it (python tools/chk_occ.py sph1M)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sph1M"
prims = scenes.primitives(name)
host = va.build_index_bvh(prims)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(name)
basis = cam.basis(W, H)
kern = va.closest_hit_kernel(dev)
for flags in (None, "all"):
    rt = va.hip_buffer_rt(ctx, W, H * 20) if flags is None else va.hip_buffer_rt(ctx, W, H * 20, flags=va._capi.VRH_RT_ALL)
    for it in range(3):
        ctx.stats_reset()
        va.render_batch(ctx, dev, rt, [basis] * 20, kern, None, frame_num=1 + 20 * it)
        a = ctx.accum_stats()
        st = ctx.last_frame_stats()
        print(flags, "grid", st["grid_blocks"], "x", st["block_threads"], "stack", st["stack_depth"],
              "ms/frame", round(a["kernel_ms_total"] / a["timed_frames"] / 20, 4), flush=True)
    rt.close()
