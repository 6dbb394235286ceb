"""Counting-kernel statistics (VRH_KERNEL_COUNT_TESTS) of launch variants, one frame each:
SIMD utilisation and the vector-L1 access model (4-lane-group accesses, ideal grouping).

    VRH_AB='[{"name": "default"}, {"name": "q1", "quad_refill": 1}]' python tools/count_variants.py [scene]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "hf1M"
variants = json.loads(os.environ.get("VRH_AB", '[{"name": "default"}]'))
prims = scenes.primitives(scene)
host = va.build_index_bvh(prims)
ctx = va.Context(0)
dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
cam, W, H = scenes.scene_camera(scene)
basis = cam.basis(W, H)
rt = va.hip_buffer_rt(ctx, W, H)
kern = va.ao_kernel(dev, count_tests=True)
opts = sorted({k for v in variants for k in v if k != "name"})
for v in variants:
    for o in opts:
        ctx.set_option(o, v.get(o, 0))
    va.render(ctx, dev, rt, basis, kern, None, frame_num=1)
    s = ctx.last_frame_stats()
    out = {"name": v["name"], "scene": scene, "rays": s["rays"],
           "lane_util": round(s["busy_lane_steps"] / max(1, 64 * s["wave_steps"]), 4),
           "vmem_instrs": s["vmem_instrs"], "group4_accesses": s["l1_group_accesses"],
           "ideal_accesses": s["l1_ideal_accesses"],
           "group4_per_instr": round(s["l1_group_accesses"] / max(1, s["vmem_instrs"]), 3),
           "group4_by_kind": dict(zip(("prims", "quads", "pairs", "normals", "stores"), list(s["l1_group_by_kind"]))),
           "box_tests_per_ray": round(s["box_tests"] / max(1, s["rays"]), 3),
           "prim_tests_per_ray": round(s["prim_tests"] / max(1, s["rays"]), 3)}
    print(json.dumps(out), flush=True)
