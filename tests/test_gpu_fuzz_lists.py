"""GPU: randomized sweep of BVH-ref lists and scissor boxes against the oracle.

Each case splits a random triangle scene of tests/test_gpu_fuzz.py into 2-4 BVHs (prim_id mod k),
joins them with vrh_scene_list_create (the reference's closest_hit / any_hit over [begin, end) of
BVH refs, traverse_linear.inl:76-141) and renders primary or AO frames through hip_sched::frame
with a random scissor box (cuda_sched.inl:71), random frame number, sample count and radius.  Every
pixel inside the box must be bit-identical to the oracle's list traversal.
"""
import os
import sys

import numpy as np
import pytest

import visionaray_amd as va

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_fuzz import _camera, _ocam, _scene  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", list(range(16)))
def test_random_lists_and_scissors_vs_oracle(ctx, oracle_mod, seed):
    O = oracle_mod
    rng = np.random.default_rng(9000 + seed)
    prims = _scene(rng, "tri")
    normals = va.face_normals(prims)
    k = int(rng.integers(2, 5))
    parts = [prims[prims["prim_id"] % k == j] for j in range(k)]
    parts = [p for p in parts if len(p)]
    osc, members = [], []
    for j, p in enumerate(parts):
        b = va.build_index_bvh(p)
        osc.append(O.Scene(f"list{seed}", O.VO_TRI, p, b.nodes, b.indices, normals if j == 0 else None, b.max_depth))
        members.append(va.hip_index_bvh(ctx, b))
    lst = va.hip_index_bvh.scene_list(ctx, members, normals)
    W, H = int(rng.integers(9, 120)), int(rng.integers(7, 80))
    cam = _camera(rng, W, H)
    ocam = _ocam(cam.basis(W, H), W, H)
    x0, x1 = sorted(int(v) for v in rng.integers(0, W + 1, 2))
    y0, y1 = sorted(int(v) for v in rng.integers(0, H + 1, 2))
    x1, y1 = max(x1, x0 + 1), max(y1, y0 + 1)
    ao = seed % 2 == 0
    samples, radius = int(rng.integers(1, 9)), float(np.float32(10.0 ** rng.uniform(-2.0, 0.0)))
    frame = int(rng.integers(0, 20))
    kern = va.ao_kernel(lst, samples=samples, radius=radius) if ao else va.closest_hit_kernel(lst)
    ref = O.render(osc, ocam, mode=O.VO_MODE_AO if ao else O.VO_MODE_PRIMARY, samples=samples, radius=radius,
                   frame_num=frame, scissor=(x0, y0, x1, y1))
    rt = va.hip_buffer_rt(ctx, W, H)
    sp = va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt)
    sp.scissor_box = (x0, y0, x1, y1)
    va.hip_sched(ctx).frame(kern, sp, frame_num=frame)
    got = rt.download()
    ys, xs = np.mgrid[0:H, 0:W]
    inside = ((xs >= x0) & (xs < x1) & (ys >= y0) & (ys < y1)).reshape(-1)
    assert inside.any()
    for key in ("prim_id", "t", "occ", "color"):
        a, b = got[key][inside], ref[key][inside]
        if a.dtype.kind == "f":
            a, b = a.view(np.uint32), b.view(np.uint32)
        assert np.array_equal(a, b), f"{key}: {int((a != b).any(axis=-1).sum() if a.ndim > 1 else (a != b).sum())} pixels differ"
    lst.close()
    for m in members:
        m.close()
