"""GPU: the mask intersector (vrh_hit_mask) against the reference.

The reference harness (oracle/ref_harness.cpp "mask") renders the AO workload through closest_hit /
any_hit with a basic_intersector that clears hr.hit where a byte mask over the hit's texture
coordinate says so -- the intersector example's mask_intersector with its heart given as data.
Bar: every pixel bit-exact (prim id, t, AO mask, colour) for the AO kernel under every schedule
option and in batched / sharded launches; the shading kernels with a mask match the oracle's hits
bit for bit and its radiance within 1e-5 (device powf).
"""
import os
import sys

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import _capi, scenes

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_gpu_parity as base  # noqa: E402
import test_gpu_shading as shading_tests  # noqa: E402

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ["mask_hf200_320x180", "mask_hf64_160x90"]
RTOL = 1e-5


def case_inputs(golden, case):
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    tc = scenes.planar_tex_coords(scenes.primitives(g["scene"]))
    return g, ref, tc, ref["mask"]


def render_masked(ctx, g, tc, mask, batch=1, shard=None):
    _, dev = base.device_scene(ctx, g["scene"])
    m = va.hit_mask(ctx, tc, mask)
    kern = va.with_hit_mask(va.ao_kernel(dev), m)
    cam, _, _ = scenes.scene_camera(g["scene"], g["W"], g["H"])
    W, H = g["W"], g["H"]
    rows = _capi.VRH_BAND_ROWS * va.shard_bands(H, shard.index, shard.count) if shard is not None else H
    rt = va.hip_buffer_rt(ctx, W, rows * batch)
    rt.clear_color_buffer((0, 0, 0, 0))
    va.render_batch(ctx, dev, rt, [cam.basis(W, H)] * batch, kern, shard)
    out = rt.download()
    stats = ctx.last_frame_stats()
    rt.close()
    m.close()
    return out, stats


def assert_equal_frame(out, ref, sl=slice(None)):
    assert np.array_equal(out["prim_id"][sl], ref["prim_id"]), f"{(out['prim_id'][sl] != ref['prim_id']).sum()} ids differ"
    assert np.array_equal(out["t"][sl].view(np.uint32), ref["t"].view(np.uint32))
    assert np.array_equal(out["occ"][sl], ref["occ"])
    assert np.array_equal(out["color"][sl].view(np.uint32), ref["color"].view(np.uint32))


@pytest.mark.parametrize("case", CASES)
def test_mask_intersector_matches_reference(ctx, golden, case):
    g, ref, tc, mask = case_inputs(golden, case)
    out, stats = render_masked(ctx, g, tc, mask)
    assert_equal_frame(out, ref)
    assert stats["hits"] == g["hits"]
    assert stats["rays"] == g["W"] * g["H"] + g["ao_rays"]


@pytest.mark.parametrize("opts", [{"refill_min": 1}, {"xcd_queues": 2}, {"wide_anyhit": 1},
                                  {"exact_minmax": 1}, {"descent_cap": 2}])
def test_mask_under_every_option(ctx, golden, opts):
    g, ref, tc, mask = case_inputs(golden, "mask_hf200_320x180")
    for k, v in opts.items():
        ctx.set_option(k, v)
    try:
        out, _ = render_masked(ctx, g, tc, mask)
    finally:
        for k in opts:
            ctx.set_option(k, 0)
    assert_equal_frame(out, ref)


def test_mask_in_batched_and_sharded_launches(ctx, golden):
    g, ref, tc, mask = case_inputs(golden, "mask_hf200_320x180")
    W, H = g["W"], g["H"]
    out, _ = render_masked(ctx, g, tc, mask, batch=3)
    assert_equal_frame(out, ref, slice(0, W * H))
    # frames 1 and 2 of the launch have frame numbers 1 and 2 (their own AO samples): same hits
    for f in (1, 2):
        sl = slice(f * W * H, (f + 1) * W * H)
        assert np.array_equal(out["prim_id"][sl], ref["prim_id"])
        assert np.array_equal(out["t"][sl].view(np.uint32), ref["t"].view(np.uint32))
    # 3 packed shards, 2 frames each, un-interleaved on the host
    from visionaray_amd import multigpu
    parts = []
    for k in range(3):
        o, _ = render_masked(ctx, g, tc, mask, batch=2, shard=_capi.vrh_shard(k, 3, 1, 0))
        rows = multigpu.rows_max(H, 3)
        n = (o["prim_id"].shape[0] // 2)
        pid = np.full(rows * W, 0xFFFFFFFF, np.uint32)
        pid[:n] = o["prim_id"][n:]                                  # frame 1 of the batch
        parts.append(pid)
    wire = multigpu.wire_layout(_capi.VRH_RT_PRIM_ID, W, H, 1, 3)
    gathered = np.stack([p.view(np.uint8) for p in parts])
    full = multigpu.unshard(gathered, wire, _capi.VRH_RT_PRIM_ID, W, H, 3, 0)["prim_id"]
    assert np.array_equal(full, ref["prim_id"])


def test_mask_has_no_effect_on_spheres(ctx):
    W, H = 128, 72
    a, _ = base.render(ctx, "sph5000", W, H, ao=False)
    _, dev = base.device_scene(ctx, "sph5000")
    m = va.hit_mask(ctx, np.zeros((3 * 5000, 2), np.float32), np.zeros((2, 2), np.uint8))
    kern = va.with_hit_mask(va.closest_hit_kernel(dev), m)
    cam, _, _ = scenes.scene_camera("sph5000", W, H)
    rt = va.hip_buffer_rt(ctx, W, H)
    va.render(ctx, dev, rt, cam.basis(W, H), kern)
    b = rt.download()
    assert np.array_equal(a["prim_id"], b["prim_id"])
    assert np.array_equal(a["t"].view(np.uint32), b["t"].view(np.uint32))


def test_mask_all_zero_hides_every_triangle(ctx):
    W, H = 96, 54
    _, dev = base.device_scene(ctx, "hf64")
    tc = scenes.planar_tex_coords(scenes.primitives("hf64"))
    m = va.hit_mask(ctx, tc, np.zeros((4, 4), np.uint8))
    kern = va.with_hit_mask(va.ao_kernel(dev), m)
    cam, _, _ = scenes.scene_camera("hf64", W, H)
    rt = va.hip_buffer_rt(ctx, W, H)
    va.render(ctx, dev, rt, cam.basis(W, H), kern)
    out = rt.download()
    assert (out["prim_id"] == 0xFFFFFFFF).all() and (out["occ"] == 0).all()


def test_mask_arguments_are_checked(ctx):
    _, dev = base.device_scene(ctx, "hf64")
    with pytest.raises(va.VrhError):
        va.hit_mask(ctx, np.zeros((4, 2), np.float32), np.ones((2, 2), np.uint8))      # not 3 per triangle
    short = va.hit_mask(ctx, np.zeros((3, 2), np.float32), np.ones((2, 2), np.uint8))  # one triangle only
    kern = va.with_hit_mask(va.ao_kernel(dev), short)
    cam, _, _ = scenes.scene_camera("hf64", 32, 18)
    rt = va.hip_buffer_rt(ctx, 32, 18)
    with pytest.raises(va.VrhError):
        va.render(ctx, dev, rt, cam.basis(32, 18), kern)


@pytest.mark.parametrize("kind", ["simple", "whitted", "multi"])
def test_shading_kernels_with_mask_match_oracle(ctx, oracle_mod, kind):
    O = oracle_mod
    name, W, H = "hf64", 160, 90
    _, _, dev = shading_tests.shade_scene(ctx, O, name)
    tc = scenes.planar_tex_coords(scenes.primitives(name))
    mask = scenes.heart_mask(41)
    m = va.hit_mask(ctx, tc, mask)
    osc = O.make_shade_scene(name)
    ocam = O.scene_camera(name, W, H)
    cam, _, _ = scenes.scene_camera(name, W, H)
    binding = va.normals_per_vertex_binding
    ob = O.VO_NORMALS_PER_VERTEX
    if kind == "simple":
        mt, lt, amb, bg = O.shade_spec()
        sh = va.shading(ctx, mt.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
        k = va.simple_kernel(dev, sh, binding=binding, bg=bg, ambient=amb)
        ref = O.render_simple(osc, ocam, ob, hit_mask=(tc, mask))
    elif kind == "whitted":
        mt, lt, amb, bg = O.whitted_spec()
        sh = va.shading(ctx, mt.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
        k = va.whitted_kernel(dev, sh, binding=binding, bg=bg, ambient=amb, num_bounces=4, epsilon=1e-3)
        ref = O.render_whitted(osc, ocam, ob, num_bounces=4, eps=1e-3, hit_mask=(tc, mask))
    else:
        mt, lt, amb, bg = O.shade_spec()
        sh = va.shading(ctx, mt.view(va.PLASTIC_DTYPE), lt.view(va.POINT_LIGHT_DTYPE))
        k = va.multi_hit_kernel(dev, sh, max_hits=8, binding=binding, bg=bg)
        ref = O.render_multi(osc, ocam, ob, max_hits=8, hit_mask=(tc, mask))
    va.with_hit_mask(k, m)
    rt = va.hip_buffer_rt(ctx, W, H)
    if kind == "multi":
        rt.alloc_multi_hit(8)
    va.hip_sched(ctx).frame(k, va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt))
    out = rt.download()
    if kind == "multi":
        mh = rt.download_multi_hit()
        assert np.array_equal(mh["mh_prim_id"], ref["mh_prim_id"])
        assert np.array_equal(mh["mh_t"].view(np.uint32), ref["mh_t"].view(np.uint32))
    else:
        assert np.array_equal(out["prim_id"], ref["prim_id"])
        assert np.array_equal(out["t"].view(np.uint32), ref["t"].view(np.uint32))
    np.testing.assert_allclose(out["color"], ref["color"], rtol=RTOL, atol=0.0)
    # the mask changed the frame
    plain = O.render_simple(osc, ocam, ob) if kind != "multi" else None
    if plain is not None:
        assert not np.array_equal(plain["prim_id"], ref["prim_id"])
