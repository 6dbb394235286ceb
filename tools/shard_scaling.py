"""Per-GPU cost of an N-way image-tile shard, measured on ONE GPU: for N = 1, 2, 4, 8 render every
shard k of N (packed, as bench.py's ranks do) and record its mean kernel time.  The slowest shard
bounds the N-GPU frame (plus the gather / un-interleave, which one GPU cannot measure).

    python tools/shard_scaling.py [scene] [frames] [ao|primary] [frames in flight]
With frames in flight F > 1 every launch renders F frames (vrh_render_batch); times are per frame.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import _capi, scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
kind = sys.argv[3] if len(sys.argv) > 3 else ("ao" if scene.startswith("hf") else "primary")
F = int(sys.argv[4]) if len(sys.argv) > 4 else 1
prims = scenes.primitives(scene)
host = va.build_index_bvh(prims)
ctx = va.Context(0)
for opt in ("waves_per_simd", "block_threads", "exact_minmax", "xcd_queues", "ao_schedule", "wide_anyhit",
            "refill_min", "descent_cap"):
    v = os.environ.get("VRH_" + opt.upper())
    if v is not None:
        ctx.set_option(opt, int(v))
dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
kern = va.ao_kernel(dev) if kind == "ao" else va.closest_hit_kernel(dev)
from visionaray_amd.buildinfo import kernel_source_sha256  # noqa: E402
out = {"scene": scene, "kind": kind, "frames": frames, "frames_in_flight": F, "per_n": {},
       "kernel_source_sha256": kernel_source_sha256()}
base = None
for n in (1, 2, 4, 8):
    rows = _capi.VRH_BAND_ROWS * va.shard_bands(H, 0, n)
    rt = va.hip_buffer_rt(ctx, W, rows * F)
    ms = []
    rays = []
    for k in range(n):
        shard = _capi.vrh_shard(k, n, 1, 0) if n > 1 else None
        va.render_batch(ctx, dev, rt, [basis] * F, kern, shard)        # warm-up
        ctx.sync()
        ctx.stats_reset()
        for _ in range(frames):
            va.render_batch(ctx, dev, rt, [basis] * F, kern, shard)
        ctx.sync()
        a = ctx.accum_stats()
        ms.append(a["kernel_ms_total"] / a["timed_frames"] / F)
        rays.append(a["rays"] / a["timed_frames"] / F)
    rt.close()
    worst = max(ms)
    if base is None:
        base = worst
    out["per_n"][n] = {"shard_ms": [round(x, 4) for x in ms], "max_ms": round(worst, 4),
                       "rays": [int(r) for r in rays], "kernel_speedup": round(base / worst, 3),
                       "kernel_efficiency": round(base / worst / n, 3)}
    print(f"F={F} N={n}: shard kernel ms {['%.4f' % x for x in ms]} max {worst:.4f} "
          f"speedup {base / worst:.2f}x eff {base / worst / n:.3f}", flush=True)
print(json.dumps(out))
