"""Render every kernel variant once on small scenes, logging progress line by line (GPU debug aid)."""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

log = open(os.path.join(ROOT, "gpurun_out", "debug.log"), "a", buffering=1)


def say(*a):
    print(*a, file=log, flush=True)
    print(*a, flush=True)


faulthandler.dump_traceback_later(60, repeat=True, file=log)
ctx = va.Context(0)
say("ctx ok", va.device_count())
for name, W, H in [("hf64", 64, 32), ("sph5000", 64, 32), ("hf64", 160, 90), ("sph5000", 256, 144), ("sph1M", 1920, 1080)]:
    prims = scenes.primitives(name)
    b = va.build_index_bvh(prims)
    dev = va.hip_index_bvh(ctx, b, scenes.normals_for(prims))
    say(name, "uploaded", dev.info)
    cam, _, _ = scenes.scene_camera(name, W, H)
    for kname in ("primary", "ao"):
        if kname == "ao" and prims.dtype != va.TRIANGLE_DTYPE:
            continue
        for count in (False, True):
            k = va.closest_hit_kernel(dev, count_tests=count) if kname == "primary" else va.ao_kernel(dev, count_tests=count)
            rt = va.hip_buffer_rt(ctx, W, H)
            t0 = time.time()
            va.render(ctx, dev, rt, cam.basis(W, H), k)
            say(" launched", name, W, H, kname, count)
            st = ctx.last_frame_stats()
            out = rt.download()
            say("  done %.3fs" % (time.time() - t0), st, "hits", int((out["prim_id"] != 0xFFFFFFFF).sum()))
faulthandler.cancel_dump_traceback_later()
say("all variants ok")
