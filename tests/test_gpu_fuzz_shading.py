"""GPU: randomized sweep of the shading kernels (simple::kernel, whitted::kernel, multi_hit<N>)
against the oracle, on the random triangle scenes and cameras of tests/test_gpu_fuzz.py.

Materials by geom_id (prim % 3), the oracle's shade / whitted light sets, per-face or per-vertex
normals, random bounce counts and hit-list sizes.  Bar as for the fixed fixtures: hits and t (and
multi_hit's lists) bit-exact, radiance within the north star's 1e-5 relative tolerance (device
powf), misses bit-exact.
"""
import os
import sys

import numpy as np
import pytest

import visionaray_amd as va

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_fuzz import _camera, _ocam, _scene  # noqa: E402

pytestmark = pytest.mark.gpu
RTOL = 1e-5


@pytest.mark.parametrize("seed", list(range(18)))
def test_random_scenes_shading_vs_oracle(ctx, oracle_mod, seed):
    O = oracle_mod
    rng = np.random.default_rng(5000 + seed)
    prims = _scene(rng, "tri")
    prims["geom_id"] = np.arange(len(prims), dtype=np.uint32) % 3
    bvh = va.build_index_bvh(prims)
    fn = va.face_normals(prims)
    vn = O.vertex_normals(fn)
    dev = va.hip_index_bvh(ctx, bvh, fn)
    dev.set_vertex_normals(vn)
    osc = O.Scene(f"shade{seed}", O.VO_TRI, prims, bvh.nodes, bvh.indices, fn, bvh.max_depth, vn)
    W, H = int(rng.integers(9, 120)), int(rng.integers(7, 80))
    basis = _camera(rng, W, H).basis(W, H)
    ocam = _ocam(basis, W, H)
    kind = ("simple", "whitted", "multi")[seed % 3]
    vertex = rng.random() < 0.5
    binding = va.normals_per_vertex_binding if vertex else va.normals_per_face_binding
    obinding = O.VO_NORMALS_PER_VERTEX if vertex else O.VO_NORMALS_PER_FACE
    rt = va.hip_buffer_rt(ctx, W, H)
    if kind == "simple":
        m, lt, amb, bg = O.shade_spec()
        sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
        va.render(ctx, dev, rt, basis, va.simple_kernel(dev, sh, binding=binding, bg=bg, ambient=amb))
        ref = O.render_simple(osc, ocam, obinding)
    elif kind == "whitted":
        m, lt, amb, bg = O.whitted_spec()
        sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
        bounces = int(rng.integers(1, 6))
        va.render(ctx, dev, rt, basis, va.whitted_kernel(dev, sh, binding=binding, bg=bg, ambient=amb,
                                                         num_bounces=bounces, epsilon=1e-3))
        ref = O.render_whitted(osc, ocam, obinding, num_bounces=bounces, eps=1e-3)
    else:
        m, lt, amb, bg = O.shade_spec()
        sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
        n = int(rng.integers(1, 17))
        rt.alloc_multi_hit(n)
        va.render(ctx, dev, rt, basis, va.multi_hit_kernel(dev, sh, max_hits=n, binding=binding))
        ref = O.render_multi(osc, ocam, obinding, max_hits=n)
    out = rt.download()
    if kind == "multi":
        out.update(rt.download_multi_hit())
        assert np.array_equal(out["mh_prim_id"], ref["mh_prim_id"])
        assert np.array_equal(out["mh_t"].view(np.uint32), ref["mh_t"].view(np.uint32))
        np.testing.assert_allclose(out["color"], ref["color"], rtol=RTOL, atol=1e-7)
        return
    assert np.array_equal(out["prim_id"], ref["prim_id"])
    assert np.array_equal(out["t"].view(np.uint32), ref["t"].view(np.uint32))
    miss = out["prim_id"] == 0xFFFFFFFF
    assert np.array_equal(out["color"][miss].view(np.uint32), ref["color"][miss].view(np.uint32))
    np.testing.assert_allclose(out["color"], ref["color"], rtol=RTOL, atol=1e-7)
