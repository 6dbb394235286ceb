"""GPU: AO tail sharing (VRH_OPT_AO_SHARE) leaves every AO frame bit-identical.

With the option, one-frame AO launches run blocks of 4 waves; once the tile queues are dry a wave
hands its last tile's AO rays out through an LDS counter that idle sibling waves claim from, and
their occlusion bits land in the owner's masks (vrh_kernels.hip step 3b).  Which wave traces a ray
does not change the ray, so every frame must equal the oracle's (the C restatement of
ao/main.cpp:183-246) -- also with the stack overflow block, with the AO cut off, and on every
frame number.
"""
import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import scenes

pytestmark = pytest.mark.gpu

NAME, W, H = "hf200", 320, 180


@pytest.fixture(scope="module")
def scene(ctx, oracle_mod):
    prims = scenes.primitives(NAME)
    dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
    cam, _, _ = scenes.scene_camera(NAME, W, H)
    return dev, cam, oracle_mod.make_scene(NAME)


def _check(got, ref):
    for k in ("prim_id", "occ"):
        assert np.array_equal(got[k], ref[k]), f"{k}: {int((got[k] != ref[k]).sum())} pixels differ"
    for k in ("t", "color"):
        assert np.array_equal(got[k].view(np.uint32), ref[k].view(np.uint32)), k


@pytest.mark.parametrize("stack,cut,frame", [(0, 0, 0), (0, 2, 0), (12, 0, 0), (0, 0, 5), (12, 0, 3)])
def test_ao_share_matches_oracle(ctx, oracle_mod, scene, stack, cut, frame):
    O = oracle_mod
    dev, cam, osc = scene
    ref = O.render(osc, O.scene_camera(NAME, W, H), mode=O.VO_MODE_AO, frame_num=frame)
    ctx.set_option("ao_share", 1)
    ctx.set_option("stack_cap", stack)
    ctx.set_option("ao_cut", cut)
    try:
        for _ in range(3):                       # the split between waves varies run to run
            rt = va.hip_buffer_rt(ctx, W, H)
            va.hip_sched(ctx).frame(va.ao_kernel(dev), va.make_sched_params(cam, rt), frame_num=frame)
            _check(rt.download(), ref)
    finally:
        ctx.set_option("ao_share", 0)
        ctx.set_option("stack_cap", 0)
        ctx.set_option("ao_cut", 0)


def test_ao_share_full_frame_hf1M(ctx, golden, oracle_mod):
    """C3's frame 0 with tail sharing: the reference's hashes."""
    g = golden["hf1M"]
    prims = scenes.primitives("hf1M")
    dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
    cam, W1, H1 = scenes.scene_camera("hf1M")
    ctx.set_option("ao_share", 1)
    try:
        rt = va.hip_buffer_rt(ctx, W1, H1)
        va.hip_sched(ctx).frame(va.ao_kernel(dev), va.make_sched_params(cam, rt))
        got = rt.download()
    finally:
        ctx.set_option("ao_share", 0)
    assert oracle_mod.fnv1a(got["prim_id"]) == g["primid_hash"]
    assert oracle_mod.fnv1a(got["occ"]) == g["occ_hash"]
    assert oracle_mod.fnv1a(got["color"]) == g["color_hash"]


def test_ao_share_option_range(ctx):
    with pytest.raises(Exception):
        ctx.set_option("ao_share", 3)


def test_ao_share_keeps_block_size_where_no_share_instance(ctx, scene):
    """Sharing exists only for one-frame AO launches at 5 waves / SIMD: a batched AO launch or a primary
    launch with the option set runs the plain instance at its usual 64-thread block, and a one-frame AO
    launch runs 4-wave blocks (the kernel selection decides, vrh_kernels.hip render_share_available)."""
    dev, cam, _ = scene
    basis = cam.basis(W, H)
    ctx.set_option("ao_share", 1)
    try:
        rt = va.hip_buffer_rt(ctx, W, 2 * H)
        va.render_batch(ctx, dev, rt, [basis, basis], va.ao_kernel(dev), None, frame_num=1)
        assert ctx.last_frame_stats()["block_threads"] == 64
        rt.close()
        rt = va.hip_buffer_rt(ctx, W, H)
        va.render(ctx, dev, rt, basis, va.closest_hit_kernel(dev), None)
        assert ctx.last_frame_stats()["block_threads"] == 64
        va.render(ctx, dev, rt, basis, va.ao_kernel(dev), None)
        assert ctx.last_frame_stats()["block_threads"] == 256
        rt.close()
    finally:
        ctx.set_option("ao_share", 0)
