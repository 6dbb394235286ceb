"""GPU: the built-in simple::kernel against the reference's own frames.

The reference harness (oracle/ref_harness.cpp "shade") renders simple::kernel with plastic
materials by geom_id and two point lights through the reference's make_kernel_params; the
fixtures in tests/golden/shade_*.npz hold its colour frames.  Bar: every pixel's hit (prim id, t)
bit-exact (checked against the oracle); radiance within the north star's 1e-5 relative tolerance
(the device powf may differ from the host libm's in the last bit; everything else is IEEE-exact
in the reference's operation order).
"""
import os

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import _capi, scenes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
RTOL = 1e-5
CASES = ["shade_cornell12_face", "shade_cornell12_vertex", "shade_hf64_face", "shade_hf64_vertex"]


def shade_scene(ctx, O, name):
    """Product-side scene of the shading fixtures: geom_id = prim index % 3, face + vertex normals."""
    prims = scenes.primitives(name)
    prims["geom_id"] = np.arange(len(prims), dtype=np.uint32) % 3
    bvh = va.build_index_bvh(prims)
    fn = va.face_normals(prims)
    dev = va.hip_index_bvh(ctx, bvh, fn)
    dev.set_vertex_normals(O.vertex_normals(fn))
    return prims, bvh, dev


def render_simple(ctx, O, dev, name, W, H, binding):
    m, lt, amb, bg = O.shade_spec()
    sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
    k = va.simple_kernel(dev, sh, binding=binding, bg=bg, ambient=amb)
    cam, _, _ = scenes.scene_camera(name, W, H)
    rt = va.hip_buffer_rt(ctx, W, H)
    va.hip_sched(ctx).frame(k, va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt))
    return rt.download()


@pytest.mark.parametrize("case", CASES)
def test_simple_kernel_matches_reference(ctx, golden, oracle_mod, case):
    O = oracle_mod
    g = golden[case]
    name, W, H = g["scene"], g["W"], g["H"]
    binding = va.normals_per_vertex_binding if g["binding"] == "vertex" else va.normals_per_face_binding
    _, _, dev = shade_scene(ctx, O, name)
    out = render_simple(ctx, O, dev, name, W, H, binding)
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))["color"]
    # hits: bit-exact against the oracle's closest hit of the same scene
    osc = O.make_shade_scene(name)
    ocam = O.scene_camera(name, W, H)
    oref = O.render_simple(osc, ocam, O.VO_NORMALS_PER_VERTEX if g["binding"] == "vertex" else O.VO_NORMALS_PER_FACE)
    assert np.array_equal(oref["color"].view(np.uint32), ref.view(np.uint32))      # the oracle pin
    assert np.array_equal(out["prim_id"], oref["prim_id"])
    assert np.array_equal(out["t"].view(np.uint32), oref["t"].view(np.uint32))
    miss = out["prim_id"] == 0xFFFFFFFF
    assert np.array_equal(out["color"][miss].view(np.uint32), ref[miss].view(np.uint32))
    np.testing.assert_allclose(out["color"], ref, rtol=RTOL, atol=0.0)
    exact = float(np.mean(np.all(out["color"] == ref, axis=1)))
    assert exact > 0.5, f"only {exact:.3f} of the pixels are bit-identical"


def test_simple_kernel_full_frame_hf1M(ctx, golden, oracle_mod):
    O = oracle_mod
    g = golden["shade_hf1M_vertex"]
    _, _, dev = shade_scene(ctx, O, "hf1M")
    out = render_simple(ctx, O, dev, "hf1M", 1920, 1080, va.normals_per_vertex_binding)
    ref = np.load(os.path.join(HERE, "golden", "shade_hf1M_vertex.npz"))
    pix = ref["pixels"]
    np.testing.assert_allclose(out["color"][pix], ref["color"], rtol=RTOL, atol=0.0)
    assert O.fnv1a(out["prim_id"]) == golden["hf1M"]["primid_hash"]     # geom_ids do not change the hits


def test_simple_kernel_argument_checks(ctx, oracle_mod):
    O = oracle_mod
    prims = scenes.primitives("hf64")
    prims["geom_id"] = 5                                  # no material 5
    bvh = va.build_index_bvh(prims)
    dev = va.hip_index_bvh(ctx, bvh, va.face_normals(prims))
    m, lt, amb, bg = O.shade_spec()
    sh = va.shading(ctx, m.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
    cam, _, _ = scenes.scene_camera("hf64", 32, 18)
    rt = va.hip_buffer_rt(ctx, 32, 18)
    with pytest.raises(va.VrhError):
        va.hip_sched(ctx).frame(va.simple_kernel(dev, sh), va.make_sched_params(cam, rt))
    prims["geom_id"] = 0
    dev2 = va.hip_index_bvh(ctx, va.build_index_bvh(prims), va.face_normals(prims))
    with pytest.raises(va.VrhError):                      # per-vertex binding without vertex normals
        va.hip_sched(ctx).frame(va.simple_kernel(dev2, sh, binding=va.normals_per_vertex_binding),
                                va.make_sched_params(cam, rt))
    sph = va.make_spheres([[0, 0, 0]], [1.0])
    sdev = va.hip_index_bvh(ctx, va.build_index_bvh(sph))
    with pytest.raises(va.VrhError) as e:
        va.hip_sched(ctx).frame(va.simple_kernel(sdev, sh), va.make_sched_params(cam, rt))
    assert e.value.code == _capi.VRH_ERR_UNSUPPORTED
