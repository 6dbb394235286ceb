import os, sys, time
sys.path.insert(0, "/root/repo")
import visionaray_amd as va
from visionaray_amd import scenes
prims = scenes.primitives("hf1M"); host = va.build_index_bvh(prims)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
cam, W, H = scenes.scene_camera("hf1M"); basis = cam.basis(W, H)
k = va.ao_kernel(dev)
def one(rt, label):
    ctx.stats_reset(); va.render(ctx, dev, rt, basis, k); a = ctx.accum_stats()
    print(f"{label:40s} {a['kernel_ms_total']:.3f} ms", flush=True)
rt0 = va.hip_buffer_rt(ctx, W, H); one(rt0, "first render, fresh rt"); one(rt0, "second render same rt")
rt1 = va.hip_buffer_rt(ctx, W, H); one(rt1, "fresh rt #2")
rt2 = va.hip_buffer_rt(ctx, W, H); rt2.clear_color_buffer((0,0,0,0)); ctx.sync(); one(rt2, "fresh rt after clear_color_buffer")
rt3 = va.hip_buffer_rt(ctx, W, 8 * H); ctx.stats_reset(); va.render_batch(ctx, dev, rt3, [basis]*8, k); a=ctx.accum_stats(); print("fresh 8-frame rt batch", a['kernel_ms_total'])
ctx.stats_reset(); va.render_batch(ctx, dev, rt3, [basis]*8, k); a=ctx.accum_stats(); print("second 8-frame batch", a['kernel_ms_total'])
