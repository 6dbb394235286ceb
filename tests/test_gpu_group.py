"""GPU: multi-GPU render groups (vrh_group_* / vrh_render_sharded) on the one-GPU box.

A one-rank group renders S > 1 image-tile shards on this GPU and runs the whole exchange of the
N-GPU path -- packed shard renders, one ncclSend / ncclRecv pair per shard over RCCL (here rank 0
sending to itself), the un-interleave on the root -- so the code bench.py runs at N > 1 runs here;
only the peer index of each send / receive differs.  Bar: the gathered frame is bit-identical to the
one-GPU frame and, for hf10M 1080p AO in 8 shards, its hashes equal the reference's own.
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


@pytest.fixture(scope="module")
def group(ctx):
    g = va.render_group(ctx, 1, 0, va.render_group.unique_id())     # ncclCommInitRank, one rank
    yield g
    g.close()


def single_frames(ctx, dev, kern, basis, W, H, frames, frame_num):
    out = []
    for f in range(frames):
        rt = va.hip_buffer_rt(ctx, W, H)
        va.render(ctx, dev, rt, basis, kern, None, frame_num=frame_num + f)
        out.append(rt.download())
        rt.close()
    return out


def sharded(ctx, group, dev, kern, basis, W, H, frames, frame_num, shards, fields):
    dst = va.hip_buffer_rt(ctx, W, H * frames)
    dst.clear_color_buffer((0, 0, 0, 0))
    group.render(dev, kern, dst, [basis] * frames, frame_num=frame_num, shards=shards, fields=fields)
    group.sync()
    out = dst.download()
    dst.close()
    return out


def test_hf10M_ao_in_8_shards_equals_reference_hashes(ctx, group, golden, oracle_mod):
    g = golden["hf10M"]
    host, dev = device_scene(ctx, "hf10M")
    cam, W, H = scenes.scene_camera("hf10M")
    fields = _capi.VRH_RT_COLOR | _capi.VRH_RT_PRIM_ID | _capi.VRH_RT_OCC | _capi.VRH_RT_T
    out = sharded(ctx, group, dev, va.ao_kernel(dev), cam.basis(W, H), W, H, 1, 0, 8, fields)
    O = oracle_mod
    assert O.fnv1a(out["prim_id"]) == g["primid_hash"]
    assert O.fnv1a(out["t"]) == g["t_hash"]
    assert O.fnv1a(out["occ"]) == g["occ_hash"]
    assert O.fnv1a(out["color"]) == g["color_hash"]


def test_hf10M_ao_colour_only_in_8_shards_equals_reference_hash(ctx, group, golden, oracle_mod):
    """bench.py's N > 1 gather: a colour-only target, one code byte per pixel on the wire."""
    host, dev = device_scene(ctx, "hf10M")
    cam, W, H = scenes.scene_camera("hf10M")
    dst = va.hip_buffer_rt(ctx, W, H, flags=_capi.VRH_RT_COLOR)
    group.render(dev, va.ao_kernel(dev), dst, [cam.basis(W, H)], shards=8, fields=_capi.VRH_RT_COLOR)
    group.sync()
    out = dst.download()
    dst.close()
    assert set(out) == {"color"}
    assert oracle_mod.fnv1a(out["color"]) == golden["hf10M"]["color_hash"]


@pytest.mark.parametrize("kind,samples,shards,frames", [("ao", 8, 3, 2), ("ao", 3, 8, 1), ("ao", 5, 135, 1),
                                                        ("primary", 0, 5, 2)])
def test_colour_code_wire_equals_single_gpu_colour(ctx, group, kind, samples, shards, frames):
    """Colour-only gathers re-derive the built-in colour from hit + occluded-sample count (any
    sample count up to 8, and primary visibility)."""
    host, dev = device_scene(ctx, "hf200")
    W, H = 320, 180
    cam, _, _ = scenes.scene_camera("hf200", W, H)
    basis = cam.basis(W, H)
    kern = va.ao_kernel(dev, samples=samples) if kind == "ao" else va.closest_hit_kernel(dev)
    dst = va.hip_buffer_rt(ctx, W, H * frames, flags=_capi.VRH_RT_COLOR)
    group.render(dev, kern, dst, [basis] * frames, frame_num=11, shards=shards, fields=_capi.VRH_RT_COLOR)
    group.sync()
    out = dst.download()
    dst.close()
    n = W * H
    for f, ref in enumerate(single_frames(ctx, dev, kern, basis, W, H, frames, 11)):
        assert np.array_equal(out["color"][f * n:(f + 1) * n].view(np.uint32), ref["color"].view(np.uint32)), f


@pytest.mark.parametrize("fields", ["color", "color+prim_id"])
@pytest.mark.parametrize("samples", [8, 5])
def test_no_occ_kernel_through_group(ctx, group, fields, samples):
    """An AO kernel that leaves the occlusion target out (ao_kernel(occ=False), VRH_KERNEL_NO_OCC)
    through the group: the wire's occlusion bytes (code byte / colour re-derivation) are the group's
    own staging data, so the gathered colour still equals the one-GPU frame."""
    host, dev = device_scene(ctx, "hf200")
    W, H = 320, 180
    cam, _, _ = scenes.scene_camera("hf200", W, H)
    basis = cam.basis(W, H)
    f = _capi.VRH_RT_COLOR | (_capi.VRH_RT_PRIM_ID if fields == "color+prim_id" else 0)
    dst = va.hip_buffer_rt(ctx, W, H * 2, flags=f)
    group.render(dev, va.ao_kernel(dev, samples=samples, occ=False), dst, [basis] * 2, frame_num=4, shards=3, fields=f)
    group.sync()
    out = dst.download()
    dst.close()
    n = W * H
    for k, ref in enumerate(single_frames(ctx, dev, va.ao_kernel(dev, samples=samples), basis, W, H, 2, 4)):
        assert np.array_equal(out["color"][k * n:(k + 1) * n].view(np.uint32), ref["color"].view(np.uint32)), k
        if "prim_id" in out:
            assert np.array_equal(out["prim_id"][k * n:(k + 1) * n], ref["prim_id"]), k


@pytest.mark.parametrize("shards,frames", [(2, 1), (3, 4), (8, 2), (135, 1)])
def test_sharded_frames_equal_single_gpu_frames(ctx, group, shards, frames):
    """Frames in flight through the group (frame numbers 7, 8, ...), every buffer gathered."""
    host, dev = device_scene(ctx, "hf200")
    W, H = 320, 180
    cam, _, _ = scenes.scene_camera("hf200", W, H)
    basis = cam.basis(W, H)
    kern = va.ao_kernel(dev)
    out = sharded(ctx, group, dev, kern, basis, W, H, frames, 7, shards, _capi.VRH_RT_ALL)
    n = W * H
    for f, ref in enumerate(single_frames(ctx, dev, kern, basis, W, H, frames, 7)):
        for k in ("prim_id", "t", "occ", "color"):
            assert np.array_equal(out[k][f * n:(f + 1) * n].view(np.uint8), ref[k].view(np.uint8)), (k, f)


def test_sharded_primary_spheres_and_shading_colour(ctx, group):
    """Sphere primary visibility (colour re-derived from prim ids) and simple::kernel (RGBA32F
    colour on the wire) through the group."""
    host, dev = device_scene(ctx, "sph5000")
    W, H = 256, 144
    cam, _, _ = scenes.scene_camera("sph5000", W, H)
    basis = cam.basis(W, H)
    kern = va.closest_hit_kernel(dev)
    out = sharded(ctx, group, dev, kern, basis, W, H, 1, 0, 5, _capi.VRH_RT_COLOR | _capi.VRH_RT_PRIM_ID)
    ref = single_frames(ctx, dev, kern, basis, W, H, 1, 0)[0]
    assert np.array_equal(out["prim_id"], ref["prim_id"])
    assert np.array_equal(out["color"].view(np.uint32), ref["color"].view(np.uint32))

    host, dev = device_scene(ctx, "hf64")
    W, H = 160, 90
    cam, _, _ = scenes.scene_camera("hf64", W, H)
    basis = cam.basis(W, H)
    mats = [va.plastic(cd=(0.8, 0.3, 0.2), ks=0.4, cs=(1, 1, 1), exp=32.0)]
    lights = [va.point_light((1.0, 2.0, 1.0))]
    sh = va.shading(ctx, mats, lights)
    kern = va.simple_kernel(dev, sh)
    out = sharded(ctx, group, dev, kern, basis, W, H, 1, 0, 3, _capi.VRH_RT_COLOR)
    ref = single_frames(ctx, dev, kern, basis, W, H, 1, 0)[0]
    assert np.array_equal(out["color"].view(np.uint32), ref["color"].view(np.uint32))


def test_group_scissor_and_local_group(ctx):
    """vrh_group_create_local (ncclCommInitAll over the visible device) and a scissor box: pixels
    outside the box stay as the root's target was cleared."""
    (g,) = va.render_group.local([ctx])
    host, dev = device_scene(ctx, "hf64")
    W, H = 160, 90
    cam, _, _ = scenes.scene_camera("hf64", W, H)
    basis = cam.basis(W, H)
    basis.scissor[:] = [10, 20, 150, 61]
    kern = va.ao_kernel(dev)
    dst = va.hip_buffer_rt(ctx, W, H)
    dst.clear_color_buffer((0.5, 0.5, 0.5, 1.0))
    g.render(dev, kern, dst, [basis], shards=4)
    g.sync()
    out = dst.download()
    rt = va.hip_buffer_rt(ctx, W, H)
    rt.clear_color_buffer((0.5, 0.5, 0.5, 1.0))
    va.render(ctx, dev, rt, basis, kern, None)
    ref = rt.download()
    for k in ("prim_id", "occ", "color"):
        assert np.array_equal(out[k].view(np.uint8), ref[k].view(np.uint8)), k
    inside = np.zeros((H, W), bool)
    inside[20:61, 10:150] = True
    assert (out["prim_id"].reshape(H, W)[~inside] == 0xFFFFFFFF).all()
    g.close()


def test_colour_code_wire_with_scissor_box(ctx, group):
    """Colour-only gather (1 B per pixel) with a scissor box: pixels inside equal the one-GPU frame,
    pixels outside keep the root target's clear colour."""
    host, dev = device_scene(ctx, "hf200")
    W, H = 320, 180
    cam, _, _ = scenes.scene_camera("hf200", W, H)
    basis = cam.basis(W, H)
    basis.scissor[:] = [17, 9, 301, 150]
    kern = va.ao_kernel(dev)
    clear = (0.25, 0.5, 0.75, 1.0)
    dst = va.hip_buffer_rt(ctx, W, H, flags=_capi.VRH_RT_COLOR)
    dst.clear_color_buffer(clear)
    group.render(dev, kern, dst, [basis], frame_num=5, shards=6, fields=_capi.VRH_RT_COLOR)
    group.sync()
    out = dst.download()["color"].reshape(H, W, 4)
    dst.close()
    rt = va.hip_buffer_rt(ctx, W, H)
    rt.clear_color_buffer(clear)
    va.render(ctx, dev, rt, basis, kern, None, frame_num=5)
    ref = rt.download()["color"].reshape(H, W, 4)
    rt.close()
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    inside = np.zeros((H, W), bool)
    inside[9:150, 17:301] = True
    assert (out[~inside] == np.float32(clear)).all()


def test_group_argument_errors(ctx, group):
    host, dev = device_scene(ctx, "hf64")
    cam, _, _ = scenes.scene_camera("hf64", 160, 90)
    basis = cam.basis(160, 90)
    small = va.hip_buffer_rt(ctx, 160, 45)
    with pytest.raises(va.VrhError):          # the root's target must be W x (H * frames)
        group.render(dev, va.ao_kernel(dev), small, [basis])
    with pytest.raises(va.VrhError):          # AO masks of more than 8 samples do not fit a byte
        group.render(dev, va.ao_kernel(dev, samples=12), va.hip_buffer_rt(ctx, 160, 90), [basis],
                     fields=_capi.VRH_RT_OCC)


def _frame(ctx, dev, kern, basis, W, H):
    rt = va.hip_buffer_rt(ctx, W, H)
    va.render(ctx, dev, rt, basis, kern, None, frame_num=2)
    out = rt.download()
    rt.close()
    return out


def _same(a, b):
    for k in ("prim_id", "occ"):
        assert np.array_equal(a[k], b[k]), k
    for k in ("t", "color"):
        assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k


def test_broadcast_scene_replicas_render_identically(ctx, group, golden, oracle_mod):
    """vrh_group_broadcast_scene (SURVEY.md §8e scene replication: ncclBroadcast from rank 0, here a
    one-rank group broadcasting into a new scene): every scene kind -- uploaded triangles with the
    4-wide records, spheres, a two-BVH list, a GPU-built scene with its reference-layout tree,
    vertex normals for the shading kernels -- renders bit for bit as the original; hf10M's replica
    reproduces the reference hashes."""
    W, H = 320, 180
    host, dev = device_scene(ctx, "hf200")
    cam, _, _ = scenes.scene_camera("hf200", W, H)
    basis = cam.basis(W, H)
    rep = group.broadcast_scene(dev)
    assert rep.handle.value != dev.handle.value
    assert rep.info == dev.info
    _same(_frame(ctx, rep, va.ao_kernel(rep), basis, W, H), _frame(ctx, dev, va.ao_kernel(dev), basis, W, H))
    rep.close()

    host, sdev = device_scene(ctx, "sph5000")
    scam, _, _ = scenes.scene_camera("sph5000", W, H)
    rep = group.broadcast_scene(sdev)
    _same(_frame(ctx, rep, va.closest_hit_kernel(rep), scam.basis(W, H), W, H),
          _frame(ctx, sdev, va.closest_hit_kernel(sdev), scam.basis(W, H), W, H))
    rep.close()

    # a list of two BVHs (prim ids split by parity), AO
    prims = scenes.primitives("hf200")
    halves = [va.hip_index_bvh(ctx, va.build_index_bvh(prims[prims["prim_id"] % 2 == p])) for p in (0, 1)]
    lst = va.hip_index_bvh.scene_list(ctx, halves, scenes.normals_for(prims))
    rep = group.broadcast_scene(lst)
    assert rep.info["num_bvhs"] == 2
    _same(_frame(ctx, rep, va.ao_kernel(rep), basis, W, H), _frame(ctx, lst, va.ao_kernel(lst), basis, W, H))
    rep.close()

    # GPU-built scene: the replica keeps the device tree (download_bvh) and renders the same
    gb = va.hip_index_bvh.gpu_build(ctx, prims, scenes.normals_for(prims))
    rep = group.broadcast_scene(gb)
    n0, i0 = gb.download_bvh()
    n1, i1 = rep.download_bvh()
    assert n0.tobytes() == n1.tobytes() and np.array_equal(i0, i1)
    _same(_frame(ctx, rep, va.ao_kernel(rep), basis, W, H), _frame(ctx, gb, va.ao_kernel(gb), basis, W, H))
    rep.close()

    # vertex normals: simple::kernel with per-vertex shading normals on the replica
    O = oracle_mod
    sprims = scenes.primitives("hf64")
    fn = va.face_normals(sprims)
    vdev = va.hip_index_bvh(ctx, va.build_index_bvh(sprims), fn)
    vdev.set_vertex_normals(O.vertex_normals(fn))
    rep = group.broadcast_scene(vdev)
    assert rep.info["vertex_normals"] == 1
    sh = va.shading(ctx, [va.plastic(cd=(0.8, 0.3, 0.2), ks=0.4, cs=(1, 1, 1), exp=32.0)], [va.point_light((1.0, 2.0, 1.0))])
    vcam, _, _ = scenes.scene_camera("hf64", 160, 90)
    kv = [va.simple_kernel(d, sh, binding=va.normals_per_vertex_binding) for d in (rep, vdev)]
    _same(_frame(ctx, rep, kv[0], vcam.basis(160, 90), 160, 90), _frame(ctx, vdev, kv[1], vcam.basis(160, 90), 160, 90))
    rep.close()

    # hf10M: the replica renders the reference's frame
    g = golden["hf10M"]
    host, big = device_scene(ctx, "hf10M")
    bcam, BW, BH = scenes.scene_camera("hf10M")
    rep = group.broadcast_scene(big)
    out = _frame_num0(ctx, rep, BW, BH, bcam.basis(BW, BH))
    O = oracle_mod
    assert O.fnv1a(out["prim_id"]) == g["primid_hash"]
    assert O.fnv1a(out["occ"]) == g["occ_hash"]
    assert O.fnv1a(out["color"]) == g["color_hash"]
    rep.close()


def _frame_num0(ctx, dev, W, H, basis):
    rt = va.hip_buffer_rt(ctx, W, H)
    va.render(ctx, dev, rt, basis, va.ao_kernel(dev), None, frame_num=0)
    out = rt.download()
    rt.close()
    return out


def test_broadcast_scene_local_group_and_errors(ctx):
    """One process driving the group (vrh_group_create_local): the same call with every member;
    rank 0 must pass its scene."""
    (g,) = va.render_group.local([ctx])
    host, dev = device_scene(ctx, "hf64")
    W, H = 160, 90
    cam, _, _ = scenes.scene_camera("hf64", W, H)
    (rep,) = va.broadcast_scene([g], dev)
    _same(_frame(ctx, rep, va.ao_kernel(rep), cam.basis(W, H), W, H),
          _frame(ctx, dev, va.ao_kernel(dev), cam.basis(W, H), W, H))
    rep.close()
    with pytest.raises(va.VrhError):
        va.broadcast_scene([g], None)
    g.close()
