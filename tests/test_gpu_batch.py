"""GPU: frames in flight (vrh_render_batch) -- every frame of a batched launch is bit-identical to
the same frame rendered alone by vrh_render, for each kernel, traversal schedule and packed shard.

A batch interleaves the frames' tiles in the work queues (vrh.h), so a wave moves from one frame's
tile to another's; these tests pin that the per-frame cameras, frame numbers (frame f of a launch
has frame number frame_num + f: its own AO samples) and output rows never mix.  Frames use distinct
cameras (the eye moved along a small orbit), so a swapped camera or row is visible.
"""
import os
import sys

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import _capi, scenes

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_gpu_parity as base  # noqa: E402

pytestmark = pytest.mark.gpu


def frame_cameras(name, W, H, n):
    """n bases of the scene camera with the eye rotated about +y by 3 degrees per frame."""
    cam, _, _ = scenes.scene_camera(name, W, H)
    ex, ey, ez = cam.eye
    out = []
    for f in range(n):
        a = np.radians(3.0 * f)
        c = va.camera()
        c.perspective(cam.fovy, cam.aspect, cam.z_near, cam.z_far)
        c.look_at((float(ex * np.cos(a) + ez * np.sin(a)), ey, float(-ex * np.sin(a) + ez * np.cos(a))),
                  cam.center, cam.up)
        out.append(c.basis(W, H))
    return out


def kernel_for(dev, kind):
    return va.ao_kernel(dev) if kind == "ao" else va.closest_hit_kernel(dev)


def single(ctx, dev, W, rows, basis, kern, shard=None, frame_num=0):
    rt = va.hip_buffer_rt(ctx, W, rows)
    rt.clear_color_buffer((0, 0, 0, 0))
    va.render(ctx, dev, rt, basis, kern, shard, frame_num=frame_num)
    out = rt.download()
    rt.close()
    return out


def check_batch(ctx, name, W, H, kind, n, shard=None, frame_num=11):
    _, dev = base.device_scene(ctx, name)
    kern = kernel_for(dev, kind)
    bases = frame_cameras(name, W, H, n)
    rows = _capi.VRH_BAND_ROWS * va.shard_bands(H, shard.index, shard.count) if shard is not None and shard.packed else H
    rt = va.hip_buffer_rt(ctx, W, n * rows)
    rt.clear_color_buffer((0, 0, 0, 0))
    va.render_batch(ctx, dev, rt, bases, kern, shard, frame_num=frame_num)
    got = rt.download()
    stats = ctx.last_frame_stats()
    rt.close()
    rays = 0
    for f in range(n):
        ref = single(ctx, dev, W, rows, bases[f], kern, shard, frame_num=frame_num + f)
        rays += ctx.last_frame_stats()["rays"]
        sl = slice(f * rows * W, (f + 1) * rows * W)
        for k in ("prim_id", "occ"):
            assert np.array_equal(got[k][sl], ref[k]), f"frame {f}: {k} differs"
        for k in ("t", "color"):
            assert np.array_equal(got[k][sl].view(np.uint32), ref[k].view(np.uint32)), f"frame {f}: {k} bits differ"
    assert stats["rays"] == rays
    # the frames really differ (distinct cameras)
    if n > 1:
        assert not np.array_equal(got["prim_id"][:rows * W], got["prim_id"][rows * W:2 * rows * W])


@pytest.mark.parametrize("n", [1, 2, 3, 8, 17, 32])
@pytest.mark.parametrize("kind", ["ao", "primary"])
def test_batch_frames_equal_single_frames(ctx, kind, n):
    check_batch(ctx, "hf200", 320, 180, kind, n)


@pytest.mark.parametrize("n", [2, 5])
def test_batch_spheres(ctx, n):
    check_batch(ctx, "sph5000", 256, 144, "primary", n)


@pytest.mark.parametrize("opts", [{"ao_schedule": 3}, {"refill_min": 1}, {"xcd_queues": 2}, {"xcd_queues": 1},
                                  {"wide_anyhit": 1}, {"xcd_queues": 4}, {"xcd_queues": 4, "cluster_tiles": 3},
                                  {"xcd_queues": 4, "cluster_tiles": 1}, {"xcd_queues": 4, "cluster_tiles": 1024},
                                  {"block_threads": 256}, {"block_threads": 192, "cluster_tiles": 3}])
def test_batch_under_other_schedules(ctx, opts):
    for k, v in opts.items():
        ctx.set_option(k, v)
    try:
        check_batch(ctx, "hf200", 320, 180, "ao", 3)
        check_batch(ctx, "sph5000", 256, 144, "primary", 2)
    finally:
        for k in opts:
            ctx.set_option(k, 0)


@pytest.mark.parametrize("count,index,n", [(3, 0, 4), (3, 2, 4), (8, 5, 4), (8, 7, 32)])
def test_batch_packed_shards(ctx, count, index, n):
    check_batch(ctx, "hf200", 320, 180, "ao", n, shard=_capi.vrh_shard(index, count, 1, 0))


@pytest.mark.parametrize("count,index,n", [(3, 1, 5), (8, 7, 20)])
def test_batch_packed_shards_cluster_order(ctx, count, index, n):
    ctx.set_option("xcd_queues", 4)
    ctx.set_option("cluster_tiles", 7)
    try:
        check_batch(ctx, "hf200", 320, 180, "ao", n, shard=_capi.vrh_shard(index, count, 1, 0))
    finally:
        for o in ("xcd_queues", "cluster_tiles"):
            ctx.set_option(o, 0)


def test_batch_arguments_are_checked(ctx):
    _, dev = base.device_scene(ctx, "hf64")
    kern = va.ao_kernel(dev)
    bases = frame_cameras("hf64", 160, 90, 2)
    rt = va.hip_buffer_rt(ctx, 160, 90)          # one frame's rows for a 2-frame batch
    with pytest.raises(va.VrhError):
        va.render_batch(ctx, dev, rt, bases, kern)
    rt.close()
    rt = va.hip_buffer_rt(ctx, 160, 90 * (_capi.VRH_MAX_BATCH + 1))
    with pytest.raises(va.VrhError):
        va.render_batch(ctx, dev, rt, bases[:1] * (_capi.VRH_MAX_BATCH + 1), kern)
    rt.close()
    odd = frame_cameras("hf64", 160, 80, 1)[0]
    rt = va.hip_buffer_rt(ctx, 160, 180)
    with pytest.raises(va.VrhError):
        va.render_batch(ctx, dev, rt, [bases[0], odd], kern)
    rt.close()


def test_removed_hand_out_options_are_refused(ctx):
    """Round 4's quad-coherent and block-shared hand-outs measured slower and were removed: 0 is
    accepted, anything else is VRH_ERR_UNSUPPORTED (profiles/r04/ab/lane_layout/)."""
    for opt in (_capi.VRH_OPT_QUAD_REFILL, _capi.VRH_OPT_GROUP_UNITS):
        ctx.set_option(opt, 0)
        with pytest.raises(_capi.VrhError) as e:
            ctx.set_option(opt, 1)
        assert e.value.code == _capi.VRH_ERR_UNSUPPORTED


def test_option_values_out_of_range_rejected(ctx):
    """Negative and too large option values are refused at vrh_ctx_set_option, before they can reach a
    kernel as wrapped uint32 values (a negative cluster size could make cluster x frames 0)."""
    for opt, bad in (("cluster_tiles", -1), ("cluster_tiles", -2**31), ("cluster_tiles", 1025), ("refill_min", -3)):
        with pytest.raises(_capi.VrhError) as e:
            ctx.set_option(opt, bad)
        assert e.value.code == _capi.VRH_ERR_INVALID
    ctx.set_option("cluster_tiles", 0)
    ctx.set_option("refill_min", 0)


# every option with its accepted range (vrh_runtime.hip k_option_ranges) and the values inside it that
# are refused as removed / unsupported
OPTION_RANGES = {
    "block_threads": (0, 256), "stack_cap": (0, 640), "blocks_per_cu": (0, 32), "refill_min": (0, 64),
    "descent_cap": (0, 1024), "cluster_tiles": (0, 1024), "wide_anyhit": (0, 2), "pop_on_miss": (0, 2),
    "scalar_fetch": (0, 2), "pair_layout": (0, 2), "ao_gate": (0, 2), "ao_share": (0, 2), "ao_cut": (0, 3),
    "xcd_queues": (0, 4), "wave_times": (0, 2), "exact_minmax": (0, 1), "async_frames": (0, 4),
    "waves_per_simd": (0, 8), "ao_schedule": (0, 4), "coop_fetch": (0, 2), "quad_refill": (0, 1),
    "group_units": (0, 1), _capi.VRH_OPT_AO_STEAL: (0, 2),
}


@pytest.mark.parametrize("opt", list(OPTION_RANGES), ids=str)
def test_every_option_range_checked(ctx, opt):
    """Each vrh_ctx_set_option value is checked against its option's own range on the int64 before it
    is narrowed: negatives (-1, INT32_MIN, INT64_MIN), one below and one above the range and 2^32 (which
    would wrap to 0) are VRH_ERR_INVALID; both edges of the range are accepted (or refused as
    removed / not a valid setting -- never wrapped)."""
    lo, hi = OPTION_RANGES[opt]
    for bad in {-1, -2**31, -2**63, lo - 1, hi + 1, 2**32, 2**31}:
        with pytest.raises(_capi.VrhError) as e:
            ctx.set_option(opt, bad)
        assert e.value.code == _capi.VRH_ERR_INVALID, (opt, bad)
    for edge in (lo, hi):
        try:
            ctx.set_option(opt, edge)
        except _capi.VrhError as e:          # e.g. waves_per_simd 8 is fine, ao_schedule 4 was removed
            assert e.code in (_capi.VRH_ERR_UNSUPPORTED, _capi.VRH_ERR_INVALID), (opt, edge)
    ctx.set_option(opt, 0)                   # back to automatic


def test_block_threads_above_launch_bounds_rejected(ctx):
    """The traversal kernels are compiled for <= 256 threads per block; a larger block is refused at
    vrh_ctx_set_option instead of failing the launch."""
    for bad in (320, 512, 100):
        with pytest.raises(_capi.VrhError):
            ctx.set_option("block_threads", bad)
    ctx.set_option("block_threads", 256)
    ctx.set_option("block_threads", 0)
