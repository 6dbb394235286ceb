"""GPU: the reference's pixel samplers (pixel_sampler::jittered / jittered_blend / ssaa_type<2, 4, 8>,
sched_common.h:160-300 and 440-720) through vrh_render_sampled and hip_sched.frame, bit for bit
against the reference harness's `sampler` frames (tests/golden/sampler_*: colour blended onto a
target filled with (0.25, 0.5, 0.75, 1), the last sample's prim id and t) -- with the pinhole
camera and with view / projection matrices (vrh_render_view, tests/golden/matrix_*)."""
import os

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import scenes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
INIT = (0.25, 0.5, 0.75, 1.0)
CASES = ["sampler_uniform_hf64_ao", "sampler_jittered_hf64_ao", "sampler_jittered_blend_hf64_ao",
         "sampler_ssaa2_hf64_ao", "sampler_ssaa4_hf64_ao", "sampler_ssaa8_hf64_ao",
         "sampler_ssaa8_sph5000_primary", "sampler_jittered_blend_sph5000_primary"]
SAMPLERS = {"uniform": va.pixel_sampler.uniform_type, "jittered": va.pixel_sampler.jittered_type,
            "jittered_blend": va.pixel_sampler.jittered_blend_type, "ssaa2": va.pixel_sampler.ssaa_type(2),
            "ssaa4": va.pixel_sampler.ssaa_type(4), "ssaa8": va.pixel_sampler.ssaa_type(8)}
_dev = {}


def _scene(ctx, name):
    if name not in _dev:
        prims = scenes.primitives(name)
        _dev[name] = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
    return _dev[name]


def _check(out, ref):
    assert np.array_equal(out["prim_id"], ref["prim_id"]), int((out["prim_id"] != ref["prim_id"]).sum())
    assert np.array_equal(out["t"].view(np.uint32), ref["t"].view(np.uint32)), int((out["t"] != ref["t"]).sum())
    bad = int((out["color"].view(np.uint32) != ref["color"].view(np.uint32)).any(axis=1).sum())
    assert bad == 0, f"{bad} pixels' colour differ from the reference"


@pytest.mark.parametrize("case", CASES)
def test_sampler_frame_matches_reference(ctx, golden, case):
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    dev = _scene(ctx, g["scene"])
    cam, _, _ = scenes.scene_camera(g["scene"], g["W"], g["H"])
    kern = va.ao_kernel(dev) if g["kernel"] == "ao" else va.closest_hit_kernel(dev)
    rt = va.hip_buffer_rt(ctx, g["W"], g["H"])
    rt.clear_color_buffer(INIT)
    va.render_sampled(ctx, dev, rt, cam.basis(g["W"], g["H"]), kern, SAMPLERS[g["sampler"]], frame_num=g["frame"])
    ctx.sync()
    _check(rt.download(), ref)
    rt.close()


@pytest.mark.parametrize("case", ["sampler_jittered_blend_hf64_ao", "sampler_ssaa4_hf64_ao"])
def test_sampler_through_hip_sched(ctx, golden, case):
    """make_sched_params(pixel_sampler::..., cam, rt) + hip_sched.frame, as the reference AO example drives it."""
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    dev = _scene(ctx, g["scene"])
    cam, _, _ = scenes.scene_camera(g["scene"], g["W"], g["H"])
    rt = va.hip_buffer_rt(ctx, g["W"], g["H"])
    rt.clear_color_buffer(INIT)
    sched = va.hip_sched(ctx)
    sched.frame(va.ao_kernel(dev), va.make_sched_params(SAMPLERS[g["sampler"]], cam, rt), frame_num=g["frame"])
    _check(rt.download(), ref)
    rt.close()


def test_progressive_jittered_blend_converges_and_shading_is_refused(ctx):
    """Frames 1..4 of jittered_blend average their samples (frame 1 overwrites: a = 1); shading
    kernels refuse the non-uniform samplers."""
    dev = _scene(ctx, "hf64")
    W, H = 160, 90
    cam, _, _ = scenes.scene_camera("hf64", W, H)
    basis = cam.basis(W, H)
    kern = va.ao_kernel(dev)
    rt = va.hip_buffer_rt(ctx, W, H)
    rt.clear_color_buffer((9.0, 9.0, 9.0, 9.0))
    frames = []
    one = va.hip_buffer_rt(ctx, W, H)
    for n in range(1, 5):
        va.render_sampled(ctx, dev, rt, basis, kern, va.pixel_sampler.jittered_blend_type, frame_num=n)
        va.render_sampled(ctx, dev, one, basis, kern, va.pixel_sampler.jittered_type, frame_num=n)
        frames.append(one.download()["color"])
    acc = frames[0].copy()
    for n in range(2, 5):
        a = np.float32(1.0) / np.float32(n)
        acc = (frames[n - 1] * a + acc * (np.float32(1.0) - a)).astype(np.float32)
    assert np.array_equal(rt.download()["color"].view(np.uint32), acc.view(np.uint32))
    sh = va.shading(ctx, [va.plastic(cd=(0.8, 0.3, 0.2))], [va.point_light((1.0, 2.0, 1.0))])
    with pytest.raises(va.VrhError):
        va.render_sampled(ctx, dev, rt, basis, va.simple_kernel(dev, sh), va.pixel_sampler.ssaa_type(4))
    rt.close()
    one.close()


MATRIX_CASES = ["matrix_uniform_hf64_ao", "matrix_ssaa4_hf64_ao", "matrix_jittered_blend_sph5000_primary",
                "matrix_uniform_hf200_ao"]


@pytest.mark.parametrize("case", MATRIX_CASES)
def test_matrix_camera_matches_reference(ctx, golden, case):
    """make_sched_params(sampler, view_matrix, proj_matrix, rt) (scheduler.h:197-212): the host inverse
    and the matrix primary rays (sched_common.h:152-176), alone and under the samplers."""
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    dev = _scene(ctx, g["scene"])
    kern = va.ao_kernel(dev) if g["kernel"] == "ao" else va.closest_hit_kernel(dev)
    rt = va.hip_buffer_rt(ctx, g["W"], g["H"])
    rt.clear_color_buffer(INIT)
    vc = va.view_camera(ref["view"], ref["proj"], g["W"], g["H"])
    va.render_view(ctx, dev, rt, vc, kern, SAMPLERS[g["sampler"]], frame_num=g["frame"])
    ctx.sync()
    _check(rt.download(), ref)
    rt.close()


@pytest.mark.parametrize("case", ["matrix_uniform_hf64_ao", "matrix_jittered_blend_sph5000_primary"])
def test_matrix_camera_through_hip_sched(ctx, golden, case):
    """hip_sched.frame(kernel, make_sched_params(sampler, view, proj, rt)); 4x4 [row, col] matrices
    give the same frame as the column-major 16-vectors; a scissor box leaves the outside untouched."""
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    dev = _scene(ctx, g["scene"])
    kern = va.ao_kernel(dev) if g["kernel"] == "ao" else va.closest_hit_kernel(dev)
    rt = va.hip_buffer_rt(ctx, g["W"], g["H"])
    rt.clear_color_buffer(INIT)
    view = ref["view"].reshape(4, 4).T          # [row, col]
    proj = ref["proj"].reshape(4, 4).T
    sched = va.hip_sched(ctx)
    sched.frame(kern, va.make_sched_params(SAMPLERS[g["sampler"]], view, proj, rt), frame_num=g["frame"])
    _check(rt.download(), ref)
    # scissor: only pixels x0 <= x < x1, y0 <= y < y1 are rendered
    W, H = g["W"], g["H"]
    box = (W // 4, H // 3, W // 2 + 7, H - 5)
    rt.clear_color_buffer(INIT)
    sp = va.make_sched_params(SAMPLERS[g["sampler"]], view, proj, rt)
    sp.scissor_box = box
    sched.frame(kern, sp, frame_num=g["frame"])
    col = rt.download()["color"].reshape(H, W, 4)
    refc = ref["color"].reshape(H, W, 4)
    inside = np.zeros((H, W), bool)
    inside[box[1]:box[3], box[0]:box[2]] = True
    assert np.array_equal(col[inside].view(np.uint32), refc[inside].view(np.uint32))
    assert np.all(col[~inside] == np.asarray(INIT, np.float32))
    rt.close()


def test_matrix_camera_refuses_shading_kernels(ctx):
    dev = _scene(ctx, "hf64")
    rt = va.hip_buffer_rt(ctx, 64, 32)
    sh = va.shading(ctx, [va.plastic(cd=(0.8, 0.3, 0.2))], [va.point_light((1.0, 2.0, 1.0))])
    vc = va.view_camera(np.eye(4), np.eye(4), 64, 32)
    with pytest.raises(va.VrhError):
        va.render_view(ctx, dev, rt, vc, va.simple_kernel(dev, sh))
    rt.close()
