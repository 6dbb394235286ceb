"""AO stash diagnostics of one-frame launches (VRH_OPT_WAVE_TIMES = 2): where the tail goes.
    python tools/steal_diag.py [scene] [steal option ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
opts = [int(x) for x in sys.argv[2:]] or [0]
prims = scenes.primitives(scene)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
kern = va.ao_kernel(dev)
rt = va.hip_buffer_rt(ctx, W, H)
frame = 1
q = lambda a, p: round(float(np.nanpercentile(a, p)), 4) if np.isfinite(a).any() else None  # noqa: E731
for o in opts:
    ctx.set_option("ao_steal", o)
    for rep in range(3):
        ctx.set_option("wave_times", 2 if rep == 2 else 0)
        va.render(ctx, dev, rt, basis, kern, frame_num=frame)
        frame += 1
    st = ctx.last_frame_stats()
    t, d = ctx.steal_diag()
    rec = {"scene": scene, "ao_steal": o, "kernel_ms": round(st["kernel_ms"], 4), "waves": int(len(t)),
           "end_p0_p50_p100": [q(t[:, 1], 0), q(t[:, 1], 50), q(t[:, 1], 100)],
           "claims_total": int(d[:, 0].sum()), "steps_p50_max": [q(d[:, 1], 50), q(d[:, 1], 100)], "publishes": int(d[:, 2].sum()),
           "records_published": int(d[:, 6].sum()), "first_claim_p0_p50_p100": [q(d[:, 7], 0), q(d[:, 7], 50), q(d[:, 7], 100)],
           "queue_dry_p0_p50_p100": [q(d[:, 3], 0), q(d[:, 3], 50), q(d[:, 3], 100)],
           "fin_seen_p0_p50_p100": [q(d[:, 4], 0), q(d[:, 4], 50), q(d[:, 4], 100)],
           "last_claim_p50_p100": [q(d[:, 5], 50), q(d[:, 5], 100)],
           "claims_per_wave_max": int(d[:, 0].max())}
    print(json.dumps(rec), flush=True)
