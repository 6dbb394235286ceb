"""A/B launch variants of the traversal kernel in ONE process, interleaved rounds (guide §5.4 rule 24).

    python tools/ab_variants.py [scene] [rounds]
Each variant is also checked bit-exactly (prim_id / occ / colour hashes) against tests/golden.
VRH_AB_BATCH = frames per launch (default 20, as the driver's bench command); times are per frame.
Frame numbers advance with every frame (distinct AO samples); the parity check renders frame 0.
VRH_AB_ORBIT = degrees the camera orbits the scene centre per frame (default 0: every frame of a
launch shares the camera, as bench.py's frames do); with it, no two frames of a launch trace the
same primary rays.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
VARIANTS = json.loads(os.environ.get("VRH_AB", "null")) or [
    {"name": "default"},
    {"name": "refill 2", "refill_min": 2},
    {"name": "refill 4", "refill_min": 4},
    {"name": "refill 8", "refill_min": 8},
    {"name": "refill 16", "refill_min": 16},
    {"name": "refill 24", "refill_min": 24},
]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
log = open(os.path.join(ROOT, "gpurun_out", f"ab_{scene}.log"), "a", buffering=1)


def say(*a):
    print(*a, flush=True)
    print(*a, file=log, flush=True)


golden = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
g = golden.get(scene)
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402  (hash helper only)

prims = scenes.primitives(scene)
host = va.build_index_bvh(prims)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
ORBIT = float(os.environ.get("VRH_AB_ORBIT", "0"))


def frame_bases(first, n):
    """Camera of frames first..first+n-1: the scene camera orbited ORBIT degrees per frame about +y."""
    if ORBIT == 0.0:
        return [basis] * n
    return scenes.orbit_bases(scene, ORBIT, first + n, W, H)[first:]


ao = prims.dtype == va.TRIANGLE_DTYPE and os.environ.get("VRH_AB_KERNEL", "ao") == "ao"
kern = va.ao_kernel(dev) if ao else va.closest_hit_kernel(dev)
F = int(os.environ.get("VRH_AB_BATCH", "20"))
rt = va.hip_buffer_rt(ctx, W, H * F)
say(f"orbit {ORBIT} deg/frame, {F} frames per launch")
say(f"scene {scene} {len(prims)} prims depth {host.max_depth} ao={ao} wide records {dev.info['wide_records']} "
    f"(depth {dev.info['wide_depth']})")
# the options the variants set (reset to 0 = auto between variants); a library without one of them
# (an older build, VRH_LIB) is then only asked for the ones its variants use
OPTIONS = sorted({k for v in VARIANTS for k in v if k != "name"})
res = {v["name"]: [] for v in VARIANTS}
bases = [frame_bases(1 + k * F, F) for k in range(3)]     # the same camera path for every variant
one = va.hip_buffer_rt(ctx, W, H)
frame = 1
for rnd in range(rounds):
    for v in VARIANTS:
        for o in OPTIONS:
            ctx.set_option(o, v.get(o, 0))
        ctx.stats_reset()
        for _ in range(3):                       # distinct frame numbers: every frame its own AO samples
            va.render_batch(ctx, dev, rt, bases[_], kern, frame_num=frame)
            frame += F
        a = ctx.accum_stats()
        st = ctx.last_frame_stats()
        ms = a["kernel_ms_min"] / F
        res[v["name"]].append((a["kernel_ms_total"] / a["timed_frames"] / F, ms, a["rays"] / a["frames"] / F))
        if rnd == 0 and g is not None:
            va.render(ctx, dev, one, basis, kern, frame_num=0)      # the parity frame
            out = one.download()
            ok = (O.fnv1a(out["prim_id"]) == g["primid_hash"] and O.fnv1a(out["t"]) == g["t_hash"]
                  and (not ao or (O.fnv1a(out["occ"]) == g["occ_hash"] and O.fnv1a(out["color"]) == g["color_hash"])))
            say(f"  {v['name']:24s} grid {st['grid_blocks']} x {st['block_threads']} stack {st['stack_depth']} "
                f"parity {'OK' if ok else 'MISMATCH'}")
say(f"{'variant':26s} {'mean ms':>9s} {'min ms':>9s} {'Mrays/s(min)':>13s} {'Mrays/s(mean)':>14s}")
for name, vals in res.items():
    mean = float(np.median([x[0] for x in vals]))
    mn = float(np.min([x[1] for x in vals]))
    rays = vals[0][2]
    say(f"{name:26s} {mean:9.4f} {mn:9.4f} {rays / mn / 1e3:13.1f} {rays / mean / 1e3:14.1f}")
