"""GPU: the built-in whitted::kernel against the reference's own frames.

The reference harness (oracle/ref_harness.cpp "whitted") renders whitted::kernel through the
reference's make_kernel_params with plastic materials by geom_id and three point lights
(oracle.whitted_spec); tests/golden/whitted_*.npz hold its colour frames, and the oracle restates
it bit-exactly (tests/test_oracle.py).  On the GPU every pixel's primary hit is bit-exact and the
radiance -- a sum over up to num_bounces bounces of ambient + unshadowed lights, each shadow ray an
any-hit traversal -- is within the north star's 1e-5 relative tolerance (device powf).
"""
import os

import numpy as np
import pytest

import sys

import visionaray_amd as va

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_multi_hit import camera_of, product_scene  # noqa: E402

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
RTOL = 1e-5
CASES = ["whitted_cornell12_face", "whitted_cornell12_vertex", "whitted_hfstack32x24_face", "whitted_hf64_vertex"]


def render_whitted(ctx, O, dev, name, W, H, binding, bounces, eps):
    m, lt, amb, bg = O.whitted_spec()
    sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
    k = va.whitted_kernel(dev, sh, binding=binding, bg=bg, ambient=amb, num_bounces=bounces, epsilon=eps)
    rt = va.hip_buffer_rt(ctx, W, H)
    va.render(ctx, dev, rt, camera_of(O, name, W, H), k)
    return rt.download()


@pytest.mark.parametrize("case", CASES)
def test_whitted_kernel_matches_reference(ctx, golden, oracle_mod, case):
    O = oracle_mod
    g = golden[case]
    name, W, H = g["scene"], g["W"], g["H"]
    binding = va.normals_per_vertex_binding if g["binding"] == "vertex" else va.normals_per_face_binding
    dev = product_scene(ctx, O, name)
    out = render_whitted(ctx, O, dev, name, W, H, binding, g["bounces"], g["eps"])
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))["color"]
    # primary hits bit-exact against the oracle's closest hit of the same scene
    osc = O.make_shade_scene(name)
    oref = O.render(osc, O.scene_camera(name, W, H), mode=O.VO_MODE_PRIMARY)
    assert np.array_equal(out["prim_id"], oref["prim_id"])
    assert np.array_equal(out["t"].view(np.uint32), oref["t"].view(np.uint32))
    miss = out["prim_id"] == 0xFFFFFFFF
    assert np.array_equal(out["color"][miss].view(np.uint32), ref[miss].view(np.uint32))
    np.testing.assert_allclose(out["color"], ref, rtol=RTOL, atol=0.0)
    exact = float(np.mean(np.all(out["color"] == ref, axis=1)))
    assert exact > 0.3, f"only {exact:.3f} of the pixels are bit-identical"


def test_whitted_kernel_full_frame_hf1M(ctx, golden, oracle_mod):
    O = oracle_mod
    g = golden["whitted_hf1M_face"]
    dev = product_scene(ctx, O, "hf1M")
    out = render_whitted(ctx, O, dev, "hf1M", 1920, 1080, va.normals_per_face_binding, g["bounces"], g["eps"])
    ref = np.load(os.path.join(HERE, "golden", "whitted_hf1M_face.npz"))
    np.testing.assert_allclose(out["color"][ref["pixels"]], ref["color"], rtol=RTOL, atol=0.0)
    assert O.fnv1a(out["prim_id"]) == golden["hf1M"]["primid_hash"]
    st = ctx.last_frame_stats()
    assert st["rays"] > 1920 * 1080                           # shadow + reflection rays were traced


def test_whitted_zero_bounces_is_black(ctx, oracle_mod):
    """num_bounces 0: the loop never runs -- hits are (0, 0, 0, 1), misses the background."""
    O = oracle_mod
    dev = product_scene(ctx, O, "cornell12")
    out = render_whitted(ctx, O, dev, "cornell12", 64, 64, va.normals_per_face_binding, 0, 1e-3)
    hit = out["prim_id"] != 0xFFFFFFFF
    assert hit.any()
    assert np.array_equal(out["color"][hit], np.tile([0.0, 0.0, 0.0, 1.0], (int(hit.sum()), 1)).astype(np.float32))


@pytest.mark.parametrize("occ", [0, 1])
def test_whitted_frames_in_flight_equal_single_frames(ctx, oracle_mod, occ):
    """whitted::kernel with three frames in one launch (vrh_render_batch, as hip_sched::frames): every
    frame bit-identical to its own single-frame render -- at the default 5 waves/SIMD (the bounce
    surface in LDS after the stack) and at 4 (waves_per_simd 1)."""
    O = oracle_mod
    name, W, H = "hfstack32x24", 96, 64
    dev = product_scene(ctx, O, name)
    m, lt, amb, bg = O.whitted_spec()
    sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
    k = va.whitted_kernel(dev, sh, bg=bg, ambient=amb, num_bounces=4, epsilon=1e-3)
    cam = camera_of(O, name, W, H)
    ctx.set_option("waves_per_simd", occ)
    try:
        one = va.hip_buffer_rt(ctx, W, H)
        va.render(ctx, dev, one, cam, k)
        single = one.download()
        three = va.hip_buffer_rt(ctx, W, 3 * H)
        va.render_batch(ctx, dev, three, [cam] * 3, k)
        got = three.download()
    finally:
        ctx.set_option("waves_per_simd", 0)
    assert (single["prim_id"] != 0xFFFFFFFF).any()
    n = W * H
    for f in range(3):
        for key in ("prim_id", "t", "color"):
            a, b = got[key][f * n:(f + 1) * n], single[key]
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (f, key)
