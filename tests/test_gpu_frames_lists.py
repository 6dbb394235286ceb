"""GPU: frame numbers (the AO sampler offset), frames in flight with distinct frame numbers, BVH-ref
lists and the scissor box -- the HIP path through the C-ABI against fixtures the reference harness
produced (tests/golden/make_golden.py --frames / --list) and against the oracle.

Bar: bit-exact prim ids, t bits, list indices (via the oracle), AO masks and colour bits.
"""
import os

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import _capi, scenes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

_cache = {}


def device_scene(ctx, name):
    if name not in _cache:
        prims = scenes.primitives(name)
        b = va.build_index_bvh(prims)
        _cache[name] = (b, va.hip_index_bvh(ctx, b, scenes.normals_for(prims)))
    return _cache[name]


def render_ao(ctx, name, W, H, frame_num=0, scissor=None, scene=None, clear=(0.0, 0.0, 0.0, 0.0)):
    dev = scene if scene is not None else device_scene(ctx, name)[1]
    cam, _, _ = scenes.scene_camera(name, W, H)
    rt = va.hip_buffer_rt(ctx, W, H)
    rt.clear_color_buffer(clear)
    sp = va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt)
    sp.scissor_box = scissor
    va.hip_sched(ctx).frame(va.ao_kernel(dev), sp, frame_num=frame_num)
    out = rt.download()
    rt.close()
    return out


def assert_same(out, ref, keys=("prim_id", "t", "occ", "color")):
    for k in keys:
        a, b = out[k], ref[k]
        if a.dtype.kind == "f":
            a, b = a.view(np.uint32), b.view(np.uint32)
        assert np.array_equal(a, b), f"{k}: {(a != b).sum()} values differ"


@pytest.mark.parametrize("case", ["frame7_hf64_160x90", "frame1_hf200_320x180"])
def test_frame_number_matches_reference(ctx, golden, case):
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    out = render_ao(ctx, g["scene"], g["W"], g["H"], frame_num=g["frame"])
    assert_same(out, ref)
    assert ctx.last_frame_stats()["rays"] == g["W"] * g["H"] + g["ao_rays"]


def test_frame_number_full_size_hashes(ctx, golden, oracle_mod):
    g = golden["frame3_hf1M"]
    ref = np.load(os.path.join(HERE, "golden", "frame3_hf1M.npz"))
    out = render_ao(ctx, "hf1M", 1920, 1080, frame_num=3)
    pix = ref["pixels"]
    assert_same({k: v[pix] for k, v in out.items()}, ref)
    O = oracle_mod
    assert O.fnv1a(out["occ"]) == g["occ_hash"]
    assert O.fnv1a(out["color"]) == g["color_hash"]
    assert O.fnv1a(out["prim_id"]) == g["primid_hash"]


def test_batch_frames_carry_consecutive_frame_numbers(ctx):
    """vrh_render_batch: frame f of a launch has frame number frame_num + f and equals its own
    vrh_render -- the frames in flight the bench times are distinct frames."""
    name, W, H, base, F = "hf200", 320, 180, 5, 4
    host, dev = device_scene(ctx, name)
    cam, _, _ = scenes.scene_camera(name, W, H)
    basis = cam.basis(W, H)
    kern = va.ao_kernel(dev)
    rt = va.hip_buffer_rt(ctx, W, H * F)
    va.render_batch(ctx, dev, rt, [basis] * F, kern, None, frame_num=base)
    batch = rt.download()
    n = W * H
    occs = []
    for f in range(F):
        one = va.hip_buffer_rt(ctx, W, H)
        va.render(ctx, dev, one, basis, kern, None, frame_num=base + f)
        single = one.download()
        assert_same({k: v[f * n:(f + 1) * n] for k, v in batch.items()}, single)
        occs.append(single["occ"])
    assert all(not np.array_equal(occs[0], o) for o in occs[1:]), "frames of a batch must differ"


def list_scene(ctx, ref, scene_name):
    """The two BVHs of a list fixture uploaded and joined by vrh_scene_list_create."""
    prims_all = scenes.primitives(scene_name)
    normals = scenes.normals_for(prims_all)
    members = []
    for k in (0, 1):
        prims = ref[f"bvh{k}_prims"].view(va.TRIANGLE_DTYPE)
        nodes = ref[f"bvh{k}_nodes"].view(va.BVH_NODE_DTYPE)
        host = va.index_bvh(prims, nodes, ref[f"bvh{k}_indices"], 0)
        members.append(va.hip_index_bvh(ctx, host))
    lst = va.hip_index_bvh.scene_list(ctx, members, normals)
    for m in members:
        m.close()             # the list owns copies of the members' arrays
    return lst


@pytest.mark.parametrize("case", ["list_hf64_160x90", "list_hf200_320x180", "list_cornell12_128"])
def test_bvh_list_with_scissor_matches_reference(ctx, golden, case):
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    lst = list_scene(ctx, ref, g["scene"])
    assert lst.info["num_bvhs"] == 2
    out = render_ao(ctx, g["scene"], g["W"], g["H"], frame_num=g["frame"], scissor=tuple(g["scissor"]), scene=lst)
    assert_same(out, ref)
    assert ctx.last_frame_stats()["hits"] == g["hits"]
    lst.close()


def test_bvh_list_primary_and_three_members_vs_oracle(ctx, oracle_mod):
    """Three BVHs over one terrain (prim_id mod 3), primary closest hit and AO, every pixel against
    the oracle's list traversal; a one-member list equals the plain scene."""
    O = oracle_mod
    name, W, H = "hf64", 160, 90
    kind, prims_all = O.gen_prims(name)
    normals = O.face_normals(prims_all)
    parts = [prims_all[prims_all["prim_id"] % 3 == k] for k in range(3)]
    osc, dev_members = [], []
    for k, p in enumerate(parts):
        nodes, idx, depth = O.build_bvh(p, O.VO_TRI)
        osc.append(O.Scene(name, O.VO_TRI, p, nodes, idx, normals if k == 0 else None, depth))
        host = va.index_bvh(p.view(va.TRIANGLE_DTYPE), nodes.view(va.BVH_NODE_DTYPE), idx, depth)
        dev_members.append(va.hip_index_bvh(ctx, host))
    lst = va.hip_index_bvh.scene_list(ctx, dev_members, normals)
    cam = O.scene_camera(name, W, H)
    vcam, _, _ = scenes.scene_camera(name, W, H)
    for mode, kern in ((O.VO_MODE_PRIMARY, va.closest_hit_kernel(lst)), (O.VO_MODE_AO, va.ao_kernel(lst))):
        ref = O.render(osc, cam, mode=mode, frame_num=2)
        rt = va.hip_buffer_rt(ctx, W, H)
        va.hip_sched(ctx).frame(kern, va.make_sched_params(va.pixel_sampler.uniform_type, vcam, rt), frame_num=2)
        assert_same(rt.download(), ref)
    # a one-entry list traverses exactly like the scene itself
    one = va.hip_index_bvh.scene_list(ctx, dev_members[:1], normals)
    ref = O.render(osc[:1], cam, mode=O.VO_MODE_AO)
    rt = va.hip_buffer_rt(ctx, W, H)
    va.hip_sched(ctx).frame(va.ao_kernel(one), va.make_sched_params(va.pixel_sampler.uniform_type, vcam, rt))
    assert_same(rt.download(), ref)


def test_scissor_leaves_outside_pixels_untouched(ctx, oracle_mod):
    O = oracle_mod
    name, W, H = "hf64", 160, 90
    clear = (0.25, 0.5, 0.75, 1.0)
    out = render_ao(ctx, name, W, H, scissor=(150, 80, 400, 400), clear=clear)   # edges past the image clamp
    inside = np.zeros((H, W), bool)
    inside[80:, 150:] = True
    col = out["color"].reshape(H, W, 4)
    assert (col[~inside] == np.array(clear, np.float32)).all()
    assert (out["prim_id"].reshape(H, W)[~inside] == 0xFFFFFFFF).all()
    sc = O.make_scene(name)
    ref = O.render(sc, O.scene_camera(name, W, H), mode=O.VO_MODE_AO)
    assert np.array_equal(out["prim_id"].reshape(H, W)[inside], ref["prim_id"].reshape(H, W)[inside])
    assert np.array_equal(out["occ"].reshape(H, W)[inside], ref["occ"].reshape(H, W)[inside])
    # an empty box renders nothing
    out = render_ao(ctx, name, W, H, scissor=(40, 40, 40, 90), clear=clear)
    assert (out["prim_id"] == 0xFFFFFFFF).all()


def test_occlusion_target_with_more_than_8_samples(ctx):
    """An occlusion byte holds 8 sample bits: a kernel asked to write masks of 9 samples into one is
    rejected; by default such a kernel leaves the buffer untouched (VRH_KERNEL_NO_OCC) and its colour
    equals a render into a target without the buffer."""
    host, dev = device_scene(ctx, "hf64")
    cam, _, _ = scenes.scene_camera("hf64", 160, 90)
    rt = va.hip_buffer_rt(ctx, 160, 90)
    sp = va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt)
    with pytest.raises(_capi.VrhError):
        va.hip_sched(ctx).frame(va.ao_kernel(dev, samples=9, occ=True), sp)
    before = rt.download()["occ"].copy()
    va.hip_sched(ctx).frame(va.ao_kernel(dev, samples=16), sp)
    out = rt.download()
    assert np.array_equal(out["occ"], before)
    rt2 = va.hip_buffer_rt(ctx, 160, 90, flags=_capi.VRH_RT_COLOR | _capi.VRH_RT_PRIM_ID)
    va.hip_sched(ctx).frame(va.ao_kernel(dev, samples=16), va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt2))
    out2 = rt2.download()
    assert np.array_equal(out["color"].view(np.uint32), out2["color"].view(np.uint32))
    assert np.array_equal(out["prim_id"], out2["prim_id"])
    # 16-sample grey levels: 1 - k/16, and some k odd (a level an 8-sample kernel cannot produce)
    k = (1.0 - np.unique(out2["color"][out2["prim_id"] != 0xFFFFFFFF][:, 0]).astype(np.float64)) * 16
    assert np.array_equal(k, np.round(k)) and (np.round(k) % 2 == 1).any()
