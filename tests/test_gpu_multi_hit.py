"""GPU: multi_hit<N> against the reference's own frames.

Fixtures (tests/golden/multi_*.npz) come from the reference harness's "multi" mode: per pixel the
reference's multi_hit<16> hit list (prim id + t, sorted by insert_sorted) and the colour of the
multi_hit example kernel.  Bar: hit lists bit-exact; colour within the north star's 1e-5 relative
tolerance (device powf).  hfstack32x24 stacks 24 terrain layers, so lists fill to the cap of 16.
"""
import os
import sys

import numpy as np
import pytest

import ctypes as C

import visionaray_amd as va
from visionaray_amd import _capi

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_shading import RTOL  # noqa: E402

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ["multi_cornell12_face", "multi_hfstack32x24_face", "multi_hfstack32x24_vertex"]


def product_scene(ctx, O, name):
    _, prims = O.gen_prims(name)          # the fixture's primitives (hfstack is a test-only scene)
    prims = prims.view(va.TRIANGLE_DTYPE).copy()
    prims["geom_id"] = np.arange(len(prims), dtype=np.uint32) % 3
    bvh = va.build_index_bvh(prims)
    fn = va.face_normals(prims)
    dev = va.hip_index_bvh(ctx, bvh, fn)
    dev.set_vertex_normals(O.vertex_normals(fn))
    return dev


def camera_of(O, name, W, H):
    """vrh_camera from the oracle's basis (bit-identical to the product camera, test_capi)."""
    eye, u, v, w, _, _ = O.scene_camera(name, W, H)
    F3 = C.c_float * 3
    return _capi.vrh_camera(F3(*eye), F3(*u), F3(*v), F3(*w), W, H)


def render_multi(ctx, O, dev, name, W, H, binding, max_hits=16):
    m, lt, amb, bg = O.shade_spec()
    sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
    k = va.multi_hit_kernel(dev, sh, max_hits=max_hits, binding=binding)
    rt = va.hip_buffer_rt(ctx, W, H)
    rt.alloc_multi_hit(max_hits)
    va.render(ctx, dev, rt, camera_of(O, name, W, H), k)
    out = rt.download()
    out.update(rt.download_multi_hit())
    return out, ctx.last_frame_stats()


@pytest.mark.parametrize("case", CASES)
def test_multi_hit_matches_reference(ctx, golden, oracle_mod, case):
    O = oracle_mod
    g = golden[case]
    name, W, H = g["scene"], g["W"], g["H"]
    binding = va.normals_per_vertex_binding if g["binding"] == "vertex" else va.normals_per_face_binding
    dev = product_scene(ctx, O, name)
    out, st = render_multi(ctx, O, dev, name, W, H, binding)
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    assert np.array_equal(out["mh_prim_id"], ref["mh_prim_id"]), \
        f"{(out['mh_prim_id'] != ref['mh_prim_id']).any(1).sum()} pixels' hit lists differ"
    assert np.array_equal(out["mh_t"].view(np.uint32), ref["mh_t"].view(np.uint32))
    assert int((out["mh_prim_id"] != 0xFFFFFFFF).sum()) == g["hits"]
    np.testing.assert_allclose(out["color"], ref["color"], rtol=RTOL, atol=1e-7)
    # the frame's prim id / t are the lists' first entries
    assert np.array_equal(out["prim_id"], ref["mh_prim_id"][:, 0])


@pytest.mark.parametrize("n", [1, 3, 7])
def test_multi_hit_prefix_property(ctx, oracle_mod, n):
    """multi_hit<n> keeps the n closest hits: its lists equal the first n entries of the reference's
    multi_hit<16> lists (same sort, ties after earlier ones) -- checked against the oracle."""
    O = oracle_mod
    name, W, H = "hfstack32x24", 96, 54
    dev = product_scene(ctx, O, name)
    out, _ = render_multi(ctx, O, dev, name, W, H, va.normals_per_face_binding, max_hits=n)
    sc = O.make_shade_scene(name)
    ref = O.render_multi(sc, O.scene_camera(name, W, H), O.VO_NORMALS_PER_FACE, max_hits=n)
    assert np.array_equal(out["mh_prim_id"], ref["mh_prim_id"])
    assert np.array_equal(out["mh_t"].view(np.uint32), ref["mh_t"].view(np.uint32))
    np.testing.assert_allclose(out["color"], ref["color"], rtol=RTOL, atol=1e-7)


def test_multi_hit_argument_checks(ctx, oracle_mod):
    O = oracle_mod
    dev = product_scene(ctx, O, "hfstack32x2")
    m, lt, _, _ = O.shade_spec()
    sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
    rt = va.hip_buffer_rt(ctx, 16, 16)
    cam = camera_of(O, "hfstack32x2", 16, 16)
    with pytest.raises(va.VrhError):          # no hit-list buffers
        va.render(ctx, dev, rt, cam, va.multi_hit_kernel(dev, sh, max_hits=4))
    rt.alloc_multi_hit(4)
    with pytest.raises(va.VrhError):          # N mismatch
        va.render(ctx, dev, rt, cam, va.multi_hit_kernel(dev, sh, max_hits=5))
    with pytest.raises(va.VrhError):
        rt.alloc_multi_hit(17)
