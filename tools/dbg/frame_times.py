import sys, os
sys.path.insert(0, os.getcwd())
import visionaray_amd as va
from visionaray_amd import scenes
prims = scenes.primitives("hf1M")
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
cam, W, H = scenes.scene_camera("hf1M")
basis = cam.basis(W, H)
kern = va.ao_kernel(dev)
rt = va.hip_buffer_rt(ctx, W, H)
res = []
for fn in list(range(0, 40)) + [64, 96, 128, 3, 0, 0, 32]:
    va.render(ctx, dev, rt, basis, kern, frame_num=fn)
    ctx.sync()
    st = ctx.last_frame_stats()
    res.append((fn, round(st["kernel_ms"], 3), st["rays"]))
print(res)
