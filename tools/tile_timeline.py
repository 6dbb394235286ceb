"""Where a one-frame launch's tail comes from: the tile timeline of the counting AO kernel
(VRH_OPT_WAVE_TIMES = 2, vrh_get_tile_times: per 8x8 tile hand-out, primaries done, pixels written).
    python tools/tile_timeline.py [scene] [frame]
Prints one JSON line: durations of the tiles and their phases, the tiles that end last (their image
rows, when they were handed out, how long they ran) and the per-row-band mean durations."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
frame = int(sys.argv[2]) if len(sys.argv) > 2 else 1
prims = scenes.primitives(scene)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
kern = va.ao_kernel(dev, count_tests=True)
rt = va.hip_buffer_rt(ctx, W, H)
for rep in range(3):
    ctx.set_option("wave_times", 2 if rep == 2 else 0)
    va.render(ctx, dev, rt, basis, kern, frame_num=frame + rep)
st = ctx.last_frame_stats()
t = ctx.tile_times()
w = ctx.wave_times()
tx = (W + 7) // 8
ty = np.arange(len(t)) // tx
dur = t[:, 2] - t[:, 0]
prim = t[:, 1] - t[:, 0]
ao = t[:, 2] - t[:, 1]
q = lambda a, p: round(float(np.percentile(a, p)), 4)  # noqa: E731
end = t[:, 2].max()
last = np.argsort(t[:, 2])[-64:]                      # the 64 tiles written last
bands = np.array_split(np.arange(ty.max() + 1), 10)
pid = rt.download()["prim_id"].reshape(H, W)
hit_rows = [round(float((pid[b[0] * 8:(b[-1] + 1) * 8] != 0xFFFFFFFF).mean()), 3) for b in bands]
rec = {"scene": scene, "kernel_ms": round(st["kernel_ms"], 4), "tiles": int(len(t)),
       "last_handout_ms": round(float(t[:, 0].max()), 4), "last_written_ms": round(float(end), 4),
       "wave_end_p0_p50_p100": [q(w[:, 1], 0), q(w[:, 1], 50), q(w[:, 1], 100)],
       "tile_ms_p50_p90_p99_max": [q(dur, 50), q(dur, 90), q(dur, 99), q(dur, 100)],
       "primary_phase_ms_p50_p99_max": [q(prim, 50), q(prim, 99), q(prim, 100)],
       "ao_phase_ms_p50_p99_max": [q(ao, 50), q(ao, 99), q(ao, 100)],
       "last64_tiles": {"rows_p0_p50_p100": [int(ty[last].min()), int(np.median(ty[last])), int(ty[last].max())],
                        "handout_ms_p0_p50_p100": [q(t[last, 0], 0), q(t[last, 0], 50), q(t[last, 0], 100)],
                        "tile_ms_p0_p50_p100": [q(dur[last], 0), q(dur[last], 50), q(dur[last], 100)],
                        "primary_ms_p50_max": [q(prim[last], 50), q(prim[last], 100)],
                        "ao_ms_p50_max": [q(ao[last], 50), q(ao[last], 100)]},
       "band_mean_tile_ms": [round(float(dur[np.isin(ty, b)].mean()), 4) for b in bands],
       "band_hit_frac": hit_rows,
       "handed_after_90pct_of_launch": int((t[:, 0] > 0.9 * end).sum()),
       "rays": int(st["rays"]), "wave_steps": int(st["wave_steps"]), "busy_lane_steps": int(st["busy_lane_steps"])}
print(json.dumps(rec), flush=True)
