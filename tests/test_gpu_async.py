"""GPU: asynchronous frames (VRH_OPT_ASYNC_FRAMES) -- cuda_sched's issue model
(cuda_sched.inl:306-320: frame() returns once the kernel is issued; gpu_buffer_rt::end_frame is a
no-op, gpu_buffer_rt.inl:84-86) with the frames overlapping on the context's frame lanes (2-4).

The bar is the synchronous path's result: a sequence of frames, clears, downloads and pixel-sampler
passes run with the option on must leave every target -- and every intermediate download -- bit for
bit as the same sequence does one synchronous frame at a time.  That covers the write order of 2, 3
and 4 lanes on one target (the scratch-target copy, pending until something needs it, dropped when a later
frame supersedes it), blending samplers that read the target, scissor boxes, shading kernels (which
wait instead of using scratch), and the joins of the context stream.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import _capi, scenes

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_gpu_parity as base  # noqa: E402
from test_gpu_batch import frame_cameras  # noqa: E402

pytestmark = pytest.mark.gpu

NAME, W, H = "hf200", 320, 180


def _bits(out):
    return {k: v.view(np.uint8).copy() for k, v in out.items()}


def _same(a, b, what):
    assert a.keys() == b.keys(), what
    for k in a:
        assert np.array_equal(a[k], b[k]), f"{what}: {k} differs in {int((a[k] != b[k]).reshape(len(a[k]), -1).any(1).sum())} rows"


@pytest.fixture(scope="module")
def scene(ctx):
    _, dev = base.device_scene(ctx, NAME)
    return dev


def _shading(ctx, dev):
    n = dev.info["max_geom_id"] + 1
    mats = np.concatenate([np.atleast_1d(va.plastic(cd=(0.2 + 0.6 * (i % 3) / 2, 0.5, 0.7), ks=0.3, exp=8.0))
                           for i in range(n)])
    lights = np.concatenate([np.atleast_1d(va.point_light((0.0, 8.0, 0.0))),
                             np.atleast_1d(va.point_light((5.0, 3.0, -4.0), cl=(0.6, 0.5, 0.4)))])
    return va.shading(ctx, mats, lights)


LANES = [2]     # frame lanes of the asynchronous run (the `lanes` fixture sets it per test)


@pytest.fixture(params=[2, 3, 4], autouse=True)
def lanes(request):
    """Every sequence with 2, 3 and 4 frame lanes (VRH_OPT_ASYNC_FRAMES = the lane count): the write
    order of any number of lanes on one target must give the synchronous bits."""
    LANES[0] = request.param
    return request.param


def run_sequence(ctx, dev, ops, n_targets, async_on):
    """Run `ops` with asynchronous frames on or off; return every target's final contents and the
    downloads the sequence asked for on the way."""
    ctx.set_option("async_frames", LANES[0] if async_on else 0)
    cams = frame_cameras(NAME, W, H, 6)
    sh = _shading(ctx, dev)
    kernels = {"ao": va.ao_kernel(dev), "primary": va.closest_hit_kernel(dev),
               "simple": va.simple_kernel(dev, sh), "whitted": va.whitted_kernel(dev, sh, num_bounces=2)}
    rts = [va.hip_buffer_rt(ctx, W, H) for _ in range(n_targets)]
    for rt in rts:
        rt.clear_color_buffer((0.25, 0.5, 0.75, 1.0))
    sched = va.hip_sched(ctx)
    seen = []
    try:
        for op in ops:
            if op[0] == "frame":
                _, ti, kind, ci, fnum, sampler, box = op
                base_cam, _, _ = scenes.scene_camera(NAME, W, H)
                sp = va.make_sched_params(sampler, base_cam, rts[ti])
                if box is not None:
                    sp.scissor_box = box
                # the frame's own camera basis: the bases of frame_cameras orbit the scene
                sp.cam = _basis_camera(cams[ci])
                sched.frame(kernels[kind], sp, frame_num=fnum)
            elif op[0] == "clear":
                rts[op[1]].clear_color_buffer(op[2])
            elif op[0] == "download":
                seen.append(_bits(rts[op[1]].download()))
        finals = [_bits(rt.download()) for rt in rts]
    finally:
        ctx.set_option("async_frames", 0)
        for rt in rts:
            rt.close()
    return finals, seen


class _basis_camera:
    """A camera whose basis() is a fixed vrh_camera (frame_cameras' orbit), for make_sched_params."""

    def __init__(self, basis):
        self._b = basis

    def basis(self, w, h):
        b = _capi.vrh_camera()
        ctypes.memmove(ctypes.byref(b), ctypes.byref(self._b), ctypes.sizeof(b))
        return b


def check_sequence(ctx, dev, ops, n_targets):
    ref_final, ref_seen = run_sequence(ctx, dev, ops, n_targets, False)
    got_final, got_seen = run_sequence(ctx, dev, ops, n_targets, True)
    for i, (a, b) in enumerate(zip(got_seen, ref_seen)):
        _same(a, b, f"download {i}")
    for i, (a, b) in enumerate(zip(got_final, ref_final)):
        _same(a, b, f"target {i}")


U = va.pixel_sampler.uniform_type
J = va.pixel_sampler.jittered_type
JB = va.pixel_sampler.jittered_blend_type


@pytest.mark.parametrize("kind", ["ao", "primary"])
def test_shared_target_back_to_back(ctx, scene, kind):
    """Ten frames into one target (distinct cameras and frame numbers): the target holds the last one."""
    ops = [("frame", 0, kind, i % 6, 3 + i, U, None) for i in range(10)]
    check_sequence(ctx, scene, ops, 1)


def test_two_targets_alternating(ctx, scene):
    ops = [("frame", i % 2, "ao", i % 6, 1 + i, U, None) for i in range(9)]
    check_sequence(ctx, scene, ops, 2)


def test_each_frame_its_own_target_equals_single_renders(ctx, scene):
    """Every frame of a back-to-back sequence equals its own synchronous render."""
    ops = [("frame", i, "ao" if i % 3 else "primary", i % 6, 7 + i, U, None) for i in range(6)]
    check_sequence(ctx, scene, ops, 6)


def test_scissor_boxes_on_a_shared_target(ctx, scene):
    """Pixels outside a frame's box keep the earlier frames' (or the clear's) values: the scratch copy
    moves exactly the box."""
    boxes = [(0, 0, W, H), (13, 7, 200, 150), (100, 40, W, 170), None, (0, 90, 160, H), (31, 0, 32, H)]
    ops = [("frame", 0, "ao" if i % 2 else "primary", i, 2 + i, U, boxes[i]) for i in range(6)]
    check_sequence(ctx, scene, ops, 1)


def test_superseded_scratch_copies(ctx, scene):
    """A frame that goes through the scratch target leaves its copy pending: a later primary / AO frame
    into the same target over at least the same box drops it (that frame's pixels are never seen), any
    other frame, a download or a frame on the same lane for another target issues it first.  Mixed:
    full frames superseding each other, a smaller box (no cover), primary after AO and back, a second
    target in between (the lanes' scratch targets reused), a download mid-sequence."""
    full, half = None, (0, 0, W, 90)
    ops = [("frame", 0, "ao", 0, 1, U, full), ("frame", 0, "primary", 1, 2, U, full),
           ("frame", 0, "ao", 2, 3, U, (20, 20, 300, 160)), ("frame", 0, "ao", 3, 4, U, full),
           ("frame", 1, "primary", 4, 5, U, full), ("frame", 0, "primary", 5, 6, U, full),
           ("frame", 1, "ao", 0, 7, U, full), ("frame", 0, "ao", 1, 8, U, full), ("download", 0),
           ("frame", 0, "ao", 2, 9, U, full), ("frame", 0, "primary", 3, 10, U, half),
           ("frame", 0, "ao", 4, 11, U, full), ("frame", 1, "ao", 5, 12, U, half), ("frame", 0, "ao", 0, 13, U, full)]
    check_sequence(ctx, scene, ops, 2)


def test_target_freed_with_a_pending_copy(ctx, scene):
    """A target closed while its last frame's copy is pending: the copy is dropped (nobody can read
    it) and the context goes on with another target."""
    dev = scene
    cam, _, _ = scenes.scene_camera(NAME, W, H)
    k = va.ao_kernel(dev)
    sched = va.hip_sched(ctx)
    ref = va.hip_buffer_rt(ctx, W, H)
    try:
        sched.frame(k, va.make_sched_params(U, cam, ref), frame_num=4)
        want = _bits(ref.download())
    finally:
        ref.close()
    ctx.set_option("async_frames", 1)
    try:
        a = va.hip_buffer_rt(ctx, W, H)
        for f in range(3):
            sched.frame(k, va.make_sched_params(U, cam, a), frame_num=1 + f)
        a.close()
        b = va.hip_buffer_rt(ctx, W, H)
        for f in range(3):
            sched.frame(k, va.make_sched_params(U, cam, b), frame_num=2 + f)
        got = _bits(b.download())
        b.close()
    finally:
        ctx.set_option("async_frames", 0)
    _same(got, want, "target after a freed target's pending copy")


def test_blending_and_jittered_samplers(ctx, scene):
    """jittered_blend reads the target (the lane waits for the other lane's frame); jittered does not
    (scratch target).  Blend weights depend on frame_num, as in the reference's AO viewer."""
    ops = [("frame", 0, "ao", 0, 1, JB, None), ("frame", 0, "ao", 0, 2, JB, None), ("frame", 0, "ao", 0, 3, JB, None),
           ("frame", 0, "primary", 1, 4, J, None), ("frame", 0, "ao", 2, 5, J, None), ("frame", 0, "ao", 2, 6, JB, None)]
    check_sequence(ctx, scene, ops, 1)


def test_ssaa_passes(ctx, scene):
    ops = [("frame", 0, "ao", 1, 1, va.pixel_sampler.ssaa_type(4), None), ("frame", 0, "primary", 2, 2, U, None),
           ("frame", 0, "ao", 3, 3, va.pixel_sampler.ssaa_type(2), None)]
    check_sequence(ctx, scene, ops, 1)


def test_clears_and_downloads_between_frames(ctx, scene):
    """A clear or a download joins the lanes: it sees every frame issued before it, and the frames
    after it see the clear."""
    ops = [("frame", 0, "ao", 0, 1, U, None), ("frame", 0, "ao", 1, 2, U, (0, 0, 160, 90)), ("download", 0),
           ("clear", 0, (1.0, 0.0, 0.0, 1.0)), ("frame", 0, "primary", 2, 3, U, (50, 50, 250, 120)),
           ("frame", 1, "ao", 3, 4, U, None), ("download", 0), ("frame", 0, "ao", 4, 5, U, (0, 100, W, H)),
           ("clear", 1, (0.0, 1.0, 0.0, 1.0)), ("frame", 1, "primary", 5, 6, U, (10, 10, 20, 20))]
    check_sequence(ctx, scene, ops, 2)


def test_shading_kernels_wait_for_the_other_lane(ctx, scene):
    """simple / whitted frames have no scratch path: a frame into a target the other lane writes waits."""
    ops = [("frame", 0, "simple", 0, 1, U, None), ("frame", 0, "ao", 1, 2, U, (0, 0, 200, 100)),
           ("frame", 0, "whitted", 2, 3, U, None), ("frame", 0, "simple", 3, 4, U, (60, 20, 300, 170)),
           ("frame", 1, "whitted", 4, 5, U, None), ("frame", 0, "primary", 5, 6, U, None)]
    check_sequence(ctx, scene, ops, 2)


def test_stats_count_every_async_frame(ctx, scene):
    dev = scene
    cam, _, _ = scenes.scene_camera(NAME, W, H)
    rt = va.hip_buffer_rt(ctx, W, H)
    k = va.ao_kernel(dev)
    sched = va.hip_sched(ctx)
    ctx.set_option("async_frames", 1)
    try:
        sched.frame(k, va.make_sched_params(cam, rt), frame_num=1)
        rays_one = ctx.last_frame_stats()["rays"]
        ctx.stats_reset()
        for i in range(7):
            sched.frame(k, va.make_sched_params(cam, rt), frame_num=1)
        acc = ctx.accum_stats()
    finally:
        ctx.set_option("async_frames", 0)
        rt.close()
    assert acc["frames"] == 7 and acc["timed_frames"] == 7
    assert acc["rays"] == 7 * rays_one
    assert 0.0 < acc["span_ms"] <= acc["kernel_ms_total"] + 1e-3


def test_user_stream_work_after_async_frames(ctx, scene):
    """vrh_ctx_get_stream joins the lanes: torch work issued on the returned stream after async frames
    reads their pixels (a target wrapping a torch tensor, copied on that stream)."""
    import torch
    dev = scene
    cam, _, _ = scenes.scene_camera(NAME, W, H)
    ref = va.hip_buffer_rt(ctx, W, H)
    k = va.ao_kernel(dev)
    va.hip_sched(ctx).frame(k, va.make_sched_params(cam, ref), frame_num=9)
    want = ref.download()["prim_id"]
    ref.close()
    pid = torch.full((W * H,), -7, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    rt = va.hip_buffer_rt(ctx, W, H, wrap=(0, pid.data_ptr(), 0, 0))
    ctx.set_option("async_frames", 1)
    try:
        for i in range(4):
            va.hip_sched(ctx).frame(k, va.make_sched_params(cam, rt), frame_num=6 + i)
        dev_i, stream = ctypes.c_int(), ctypes.c_void_p()
        _capi.check("vrh_ctx_get_stream", ctx.handle, ctypes.byref(dev_i), ctypes.byref(stream))
        s = torch.cuda.ExternalStream(stream.value, device=torch.device("cuda", dev_i.value))
        with torch.cuda.stream(s):
            out = pid.clone()
        s.synchronize()
        got = out.cpu().numpy().view(np.uint32)
    finally:
        ctx.set_option("async_frames", 0)
        rt.close()
    assert np.array_equal(got, want)


def test_lane_count_changed_between_frames(ctx, scene, lanes):
    """Changing the number of frame lanes while frames are in flight first joins every lane: frames
    issued on 4 lanes, then on 2, then on 3, into one shared target and a second target, leave the
    synchronous run's bits."""
    if lanes != 2:
        pytest.skip("one run is enough: the lane counts are switched inside the test")
    dev = scene
    cams = frame_cameras(NAME, W, H, 6)
    k = va.ao_kernel(dev)
    sched = va.hip_sched(ctx)
    plan = [(4, 0), (4, 1), (4, 0), (2, 0), (2, 1), (3, 0), (3, 0), (3, 1), (4, 0)]

    def run(async_on):
        rts = [va.hip_buffer_rt(ctx, W, H) for _ in range(2)]
        try:
            for i, (n, ti) in enumerate(plan):
                ctx.set_option("async_frames", n if async_on else 0)
                base_cam, _, _ = scenes.scene_camera(NAME, W, H)
                sp = va.make_sched_params(U, base_cam, rts[ti])
                sp.cam = _basis_camera(cams[i % 6])
                sched.frame(k, sp, frame_num=20 + i)
            return [_bits(rt.download()) for rt in rts]
        finally:
            ctx.set_option("async_frames", 0)
            for rt in rts:
                rt.close()

    want, got = run(False), run(True)
    for i, (a, b) in enumerate(zip(got, want)):
        _same(a, b, f"target {i}")


def test_async_option_range(ctx):
    """0 = off, 1 = on with the default lanes, 2..4 = that many lanes; anything else is refused."""
    for bad in (5, -1, 2**32):
        with pytest.raises(_capi.VrhError):
            ctx.set_option("async_frames", bad)
    for ok in (1, 2, 3, 4, 0):
        ctx.set_option("async_frames", ok)


def test_full_frame_hf1M_async_shared_target(ctx, golden, oracle_mod):
    """C3 at 1080p: four back-to-back frames into one target, the last one frame 0 -- the reference's
    hashes; the same into two targets, their last frames 0 and 3."""
    prims = scenes.primitives("hf1M")
    dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
    cam, W1, H1 = scenes.scene_camera("hf1M")
    k = va.ao_kernel(dev)
    sched = va.hip_sched(ctx)
    ctx.set_option("async_frames", 1)
    try:
        rt = va.hip_buffer_rt(ctx, W1, H1)
        for fnum in (5, 2, 7, 0):
            sched.frame(k, va.make_sched_params(cam, rt), frame_num=fnum)
        got = rt.download()
        rt2 = [va.hip_buffer_rt(ctx, W1, H1) for _ in range(2)]
        for i, fnum in enumerate((1, 4, 9, 8, 0, 3)):
            sched.frame(k, va.make_sched_params(cam, rt2[i % 2]), frame_num=fnum)
        got2 = [r.download() for r in rt2]
    finally:
        ctx.set_option("async_frames", 0)
    O = oracle_mod
    for out, g in ((got, golden["hf1M"]), (got2[0], golden["hf1M"]), (got2[1], golden["frame3_hf1M"])):
        assert O.fnv1a(out["prim_id"]) == g["primid_hash"]
        assert O.fnv1a(out["occ"]) == g["occ_hash"]
        assert O.fnv1a(out["color"]) == g["color_hash"]
