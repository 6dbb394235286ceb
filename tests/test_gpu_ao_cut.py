"""GPU: the AO entry cut (VRH_OPT_AO_CUT) leaves every AO frame bit-identical.

A tile's AO rays start at a cut of the 4-wide any-hit tree whose boxes meet the tile's AO reach
(vrh_kernels.hip ao_cut_build).  The cut's depth depends on the AO radius relative to the scene:
tiny radii cut deep, radii larger than the scene keep the root's children.  Every radius is checked
against the oracle (the C restatement of ao/main.cpp:183-246), with the cut on (default) and off,
in one-frame launches and with frames in flight.
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
    assert dev.info["wide_records"] > 0
    cam, _, _ = scenes.scene_camera(NAME, W, H)
    return dev, cam, oracle_mod.make_scene(NAME)


def _check(got, ref, n=None):
    for k in ("prim_id", "occ"):
        a, b = got[k], ref[k]
        assert np.array_equal(a[:n] if n else a, b), k
    for k in ("t", "color"):
        a, b = got[k].view(np.uint32), ref[k].view(np.uint32)
        assert np.array_equal(a[:n] if n else a, b), k


@pytest.mark.parametrize("radius", [0.002, 0.03, 0.1, 0.6, 8.0])
@pytest.mark.parametrize("cut", [0, 2, 3])
@pytest.mark.parametrize("stack", [0, 12])
def test_ao_cut_matches_oracle(ctx, oracle_mod, scene, radius, cut, stack):
    """stack 12: an LDS stack of 12 entries, shallower than the BVH, so the overflow-block (spilling)
    kernel instances run -- with the cut (cutN + 4 <= 12) and without it."""
    O = oracle_mod
    dev, cam, osc = scene
    if stack:
        assert dev.info["max_depth"] > stack
    ref = O.render(osc, O.scene_camera(NAME, W, H), mode=O.VO_MODE_AO, radius=radius)
    ctx.set_option("ao_cut", cut)
    ctx.set_option("stack_cap", stack)
    try:
        rt = va.hip_buffer_rt(ctx, W, H)
        va.hip_sched(ctx).frame(va.ao_kernel(dev, radius=radius), va.make_sched_params(cam, rt))
        _check(rt.download(), ref)
        # frames in flight: frame 0 of a 3-frame launch is the parity frame
        basis = cam.basis(W, H)
        rtb = va.hip_buffer_rt(ctx, W, H * 3)
        va.render_batch(ctx, dev, rtb, [basis] * 3, va.ao_kernel(dev, radius=radius), frame_num=0)
        _check(rtb.download(), ref, W * H)
    finally:
        ctx.set_option("ao_cut", 0)
        ctx.set_option("stack_cap", 0)


def test_ao_cut_option_range(ctx):
    with pytest.raises(Exception):
        ctx.set_option("ao_cut", 4)
