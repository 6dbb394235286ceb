"""GPU: randomized sweep of the reference's pixel samplers (sched_common.h:160-300, 440-720) against
the oracle: uniform, jittered, jittered_blend and ssaa<2,4,8> frames of random triangle / sphere
scenes and cameras (tests/test_gpu_fuzz.py), primary or AO, random frame numbers, blended onto a
random initial target through vrh_render_sampled -- prim id, t and colour bit-exact.
"""
import os
import sys

import numpy as np
import pytest

import visionaray_amd as va

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_fuzz import _camera, _ocam, _scene  # noqa: E402

pytestmark = pytest.mark.gpu
SAMPLERS = {"uniform": va.pixel_sampler.uniform_type, "jittered": va.pixel_sampler.jittered_type,
            "jittered_blend": va.pixel_sampler.jittered_blend_type, "ssaa2": va.pixel_sampler.ssaa_type(2),
            "ssaa4": va.pixel_sampler.ssaa_type(4), "ssaa8": va.pixel_sampler.ssaa_type(8)}
NAMES = sorted(SAMPLERS)


@pytest.mark.parametrize("seed", list(range(18)))
def test_random_sampler_frames_vs_oracle(ctx, oracle_mod, seed):
    O = oracle_mod
    rng = np.random.default_rng(7000 + seed)
    kind = "sph" if seed % 3 == 2 else "tri"
    prims = _scene(rng, kind)
    bvh = va.build_index_bvh(prims)
    nrm = va.face_normals(prims) if kind == "tri" else None
    dev = va.hip_index_bvh(ctx, bvh, nrm)
    osc = O.Scene(f"smp{seed}", O.VO_TRI if kind == "tri" else O.VO_SPHERE, prims, bvh.nodes, bvh.indices, nrm,
                  bvh.max_depth)
    W, H = int(rng.integers(9, 100)), int(rng.integers(7, 70))
    basis = _camera(rng, W, H).basis(W, H)
    sampler = NAMES[seed % len(NAMES)]
    ao = kind == "tri"
    frame = int(rng.integers(1, 30))                   # jittered_blend weights 1 / frame_num
    init = tuple(float(np.float32(x)) for x in rng.uniform(0.0, 1.0, 4))
    kern = va.ao_kernel(dev) if ao else va.closest_hit_kernel(dev)
    ref = O.render_sampled(osc, _ocam(basis, W, H), sampler, init=init, mode=O.VO_MODE_AO if ao else O.VO_MODE_PRIMARY,
                           frame_num=frame)
    rt = va.hip_buffer_rt(ctx, W, H)
    rt.clear_color_buffer(init)
    va.render_sampled(ctx, dev, rt, basis, kern, SAMPLERS[sampler], frame_num=frame)
    ctx.sync()
    out = rt.download()
    assert np.array_equal(out["prim_id"], ref["prim_id"]), int((out["prim_id"] != ref["prim_id"]).sum())
    assert np.array_equal(out["t"].view(np.uint32), ref["t"].view(np.uint32))
    bad = int((out["color"].view(np.uint32) != ref["color"].view(np.uint32)).any(axis=1).sum())
    assert bad == 0, f"{sampler}: {bad} pixels' colour differ"
