"""GPU: the HIP traversal path (through the C-ABI) against the reference outputs and the oracle.

Bar: bit-exact on integer hit ids, t bits, occlusion masks and colour bits; the
whole-frame hashes of the 1080p configs equal the hashes the reference itself produced.
"""
import os

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import _capi, scenes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FULL_CASES = ["cornell12", "hf64_160x90", "hf200_320x180", "sph5000_256x144"]

_scene_cache = {}


def device_scene(ctx, name):
    if name not in _scene_cache:
        prims = scenes.primitives(name)
        b = va.build_index_bvh(prims)
        _scene_cache[name] = (b, va.hip_index_bvh(ctx, b, scenes.normals_for(prims)))
    return _scene_cache[name]


def render(ctx, name, W, H, ao=None, samples=8, shard=None, packed=False):
    host, dev = device_scene(ctx, name)
    if ao is None:
        ao = host.prim_kind == va._capi.VRH_PRIM_TRI64
    cam, _, _ = scenes.scene_camera(name, W, H)
    kern = va.ao_kernel(dev, samples=samples) if ao else va.closest_hit_kernel(dev)
    if shard is None:
        # an occlusion target holds one bit per sample in a byte (vrh.h): more samples, no masks
        flags = _capi.VRH_RT_ALL if samples <= 8 else _capi.VRH_RT_ALL & ~_capi.VRH_RT_OCC
        rt = va.hip_buffer_rt(ctx, W, H, flags=flags)
        va.hip_sched(ctx).frame(kern, va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt))
    else:
        rows = va._capi.VRH_BAND_ROWS * va.shard_bands(H, shard[0], shard[1]) if packed else H
        rt = va.hip_buffer_rt(ctx, W, max(rows, 1))
        rt.clear_color_buffer((0, 0, 0, 0))
        va.hip_sched(ctx).frame(kern, va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt, image_size=(W, H)),
                                shard=(shard[0], shard[1], packed))
    out = rt.download()
    stats = ctx.last_frame_stats()
    rt.close()
    return out, stats


@pytest.mark.parametrize("case", FULL_CASES)
def test_every_pixel_matches_reference(ctx, golden, case):
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    out, stats = render(ctx, g["scene"], g["W"], g["H"])
    assert np.array_equal(out["prim_id"], ref["prim_id"]), f"{(out['prim_id'] != ref['prim_id']).sum()} prim ids differ"
    assert np.array_equal(out["t"].view(np.uint32), ref["t"].view(np.uint32)), "t bits differ"
    assert np.array_equal(out["occ"], ref["occ"]), f"{(out['occ'] != ref['occ']).sum()} AO masks differ"
    assert np.array_equal(out["color"].view(np.uint32), ref["color"].view(np.uint32)), "colour bits differ"
    assert stats["hits"] == g["hits"]
    assert stats["rays"] == g["W"] * g["H"] + g["ao_rays"]


@pytest.mark.parametrize("case", ["hf1M", "sph1M", "hf10M"])
def test_full_frame_hashes_match_reference(ctx, golden, oracle_mod, case):
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    out, stats = render(ctx, g["scene"], g["W"], g["H"])
    pix = ref["pixels"]
    assert np.array_equal(out["prim_id"][pix], ref["prim_id"])
    assert np.array_equal(out["t"][pix].view(np.uint32), ref["t"].view(np.uint32))
    assert np.array_equal(out["occ"][pix], ref["occ"])
    O = oracle_mod
    assert O.fnv1a(out["prim_id"]) == g["primid_hash"]
    assert O.fnv1a(out["t"]) == g["t_hash"]
    assert O.fnv1a(out["occ"]) == g["occ_hash"]
    assert O.fnv1a(out["color"]) == g["color_hash"]
    assert stats["hits"] == g["hits"]
    assert stats["rays"] == g["W"] * g["H"] + g["ao_rays"]


def test_primary_kernel_matches_reference_hits(ctx, golden, oracle_mod):
    g = golden["hf1M"]
    out, stats = render(ctx, "hf1M", 1920, 1080, ao=False)
    assert oracle_mod.fnv1a(out["prim_id"]) == g["primid_hash"]
    assert oracle_mod.fnv1a(out["t"]) == g["t_hash"]
    assert stats["rays"] == 1920 * 1080


@pytest.mark.parametrize("count", [2, 3, 8])
def test_packed_shards_gather_to_identical_image(ctx, count):
    """N packed shards rendered on one GPU, 'gathered' and un-interleaved on the device: both the
    full-colour gather and the compressed one (prim id + AO mask, colour re-derived) reproduce the
    single-GPU frame bit for bit."""
    name, W, H = "hf200", 320, 180
    full, _ = render(ctx, name, W, H)
    rows = _capi.VRH_BAND_ROWS * va.shard_bands(H, 0, count)
    n = rows * W
    gathered_c = np.zeros((count, n, 4), np.float32)
    gathered_p = np.full((count, n), 0xFFFFFFFF, np.uint32)
    gathered_o = np.zeros((count, n), np.uint8)
    total_rays = 0
    for gi in range(count):
        out, st = render(ctx, name, W, H, shard=(gi, count), packed=True)
        m = out["prim_id"].shape[0]
        gathered_c[gi, :m] = out["color"]
        gathered_p[gi, :m] = out["prim_id"]
        gathered_o[gi, :m] = out["occ"]
        total_rays += st["rays"]
    assert total_rays == W * H + 8 * int((full["prim_id"] != 0xFFFFFFFF).sum())
    flags = _capi.VRH_RT_COLOR | _capi.VRH_RT_PRIM_ID | _capi.VRH_RT_OCC
    src = va.hip_buffer_rt(ctx, W, count * rows, flags=flags)
    src.upload(color=gathered_c.reshape(-1, 4), prim_id=gathered_p.reshape(-1), occ=gathered_o.reshape(-1))
    cptr, pptr, _, optr = src.device_buffers()
    # (1) full colour gathered
    dst = va.hip_buffer_rt(ctx, W, H, flags=flags)
    va.unshard(ctx, W, H, count, dst, color_ptr=cptr, prim_id_ptr=pptr, occ_ptr=optr)
    got = dst.download(t=False)
    assert np.array_equal(got["prim_id"], full["prim_id"])
    assert np.array_equal(got["occ"], full["occ"])
    assert np.array_equal(got["color"].view(np.uint32), full["color"].view(np.uint32))
    # (2) compressed: 5 B/pixel in ONE buffer per shard [prim ids | masks], colour re-derived
    comb = np.zeros((count, 5 * n), np.uint8)
    comb[:, :4 * n] = gathered_p.view(np.uint8).reshape(count, 4 * n)
    comb[:, 4 * n:] = gathered_o
    cbuf = va.hip_buffer_rt(ctx, W, count * rows * 5 // 4 + 1, flags=_capi.VRH_RT_PRIM_ID)
    padded = np.zeros(cbuf.w * cbuf.h * 4, np.uint8)
    padded[:comb.size] = comb.reshape(-1)
    cbuf.upload(prim_id=padded.view(np.uint32))
    _, base, _, _ = cbuf.device_buffers()
    dst2 = va.hip_buffer_rt(ctx, W, H, flags=flags)
    kern = va.ao_kernel(device_scene(ctx, name)[1])
    va.unshard(ctx, W, H, count, dst2, prim_id_ptr=base, occ_ptr=base + 4 * n, shard_stride_bytes=5 * n, kernel=kern)
    got2 = dst2.download(t=False)
    assert np.array_equal(got2["prim_id"], full["prim_id"])
    assert np.array_equal(got2["occ"], full["occ"])
    assert np.array_equal(got2["color"].view(np.uint32), full["color"].view(np.uint32))


def test_unpacked_shards_compose(ctx):
    name, W, H = "hf64", 160, 90
    full, _ = render(ctx, name, W, H)
    acc = np.full(W * H, 0xFFFFFFFF, np.uint32)
    for gi in range(3):
        out, _ = render(ctx, name, W, H, shard=(gi, 3), packed=False)
        rows = np.arange(H)
        mine = ((rows // _capi.VRH_BAND_ROWS) % 3) == gi
        m = np.repeat(mine, W)
        acc[m] = out["prim_id"][m]
    assert np.array_equal(acc, full["prim_id"])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_soups_vs_oracle(ctx, oracle_mod, seed):
    """Random triangle soups (with many shared-edge ties) and odd image sizes vs the oracle."""
    O = oracle_mod
    rng = np.random.default_rng(seed)
    n = [50, 3000, 40000][seed]
    # a jittered grid of quads: shared edges everywhere -> closest-hit ties resolved by traversal order
    g = int(np.sqrt(n / 2)) + 1
    xs = np.linspace(-1, 1, g + 1, dtype=np.float32)
    X, Z = np.meshgrid(xs, xs)
    Y = (rng.uniform(-0.05, 0.05, X.shape)).astype(np.float32)
    P = np.stack([X, Y, Z], -1)
    a, b, c, e = P[:-1, :-1].reshape(-1, 3), P[:-1, 1:].reshape(-1, 3), P[1:, 1:].reshape(-1, 3), P[1:, :-1].reshape(-1, 3)
    v1 = np.concatenate([a, a]); e1 = np.concatenate([b - a, c - a]); e2 = np.concatenate([c - a, e - a])
    tris = va.make_triangles(v1, e1, e2)
    W, H = [(33, 17), (97, 64), (211, 131)][seed]
    bvh = va.build_index_bvh(tris)
    nrm = va.face_normals(tris)
    dev = va.hip_index_bvh(ctx, bvh, nrm)
    cam = va.camera()
    cam.perspective(0.8, np.float32(W) / np.float32(H), 0.001, 1000.0)
    cam.look_at((0.3, 1.2, 1.1), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0))
    rt = va.hip_buffer_rt(ctx, W, H)
    va.hip_sched(ctx).frame(va.ao_kernel(dev, samples=8, radius=0.2), va.make_sched_params(cam, rt))
    got = rt.download()
    basis = cam.basis(W, H)
    ocam = (np.array(basis.eye[:], np.float32), np.array(basis.cam_u[:], np.float32),
            np.array(basis.cam_v[:], np.float32), np.array(basis.cam_w[:], np.float32), W, H)
    osc = O.Scene("soup", O.VO_TRI, tris, bvh.nodes, bvh.indices, nrm, bvh.max_depth)
    ref = O.render(osc, ocam, mode=O.VO_MODE_AO, radius=0.2)
    assert np.array_equal(got["prim_id"], ref["prim_id"])
    assert np.array_equal(got["t"].view(np.uint32), ref["t"].view(np.uint32))
    assert np.array_equal(got["occ"], ref["occ"])
    assert np.array_equal(got["color"].view(np.uint32), ref["color"].view(np.uint32))


def test_edge_cases_single_leaf_zero_dir_components_and_inside_sphere(ctx, oracle_mod):
    O = oracle_mod
    # single triangle: the root is a leaf
    tris = va.make_triangles([[-1, -1, 0]], [[2, 0, 0]], [[0, 2, 0]])
    bvh = va.build_index_bvh(tris)
    assert len(bvh.nodes) == 1
    dev = va.hip_index_bvh(ctx, bvh, va.face_normals(tris))
    for (W, H) in ((1, 1), (17, 13)):
        cam = va.camera()
        cam.perspective(0.5, np.float32(W) / np.float32(H), 0.001, 1000.0)
        cam.look_at((0.0, 0.0, 2.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0))  # axis-aligned: dir.x = dir.y = 0 at centre
        rt = va.hip_buffer_rt(ctx, W, H)
        va.hip_sched(ctx).frame(va.ao_kernel(dev), va.make_sched_params(cam, rt))
        got = rt.download()
        b = cam.basis(W, H)
        ocam = tuple(np.array(x[:], np.float32) for x in (b.eye, b.cam_u, b.cam_v, b.cam_w)) + (W, H)
        ref = O.render(O.Scene("t", O.VO_TRI, tris, bvh.nodes, bvh.indices, va.face_normals(tris), 0), ocam)
        assert np.array_equal(got["prim_id"], ref["prim_id"]) and np.array_equal(got["t"].view(np.uint32), ref["t"].view(np.uint32))
        assert np.array_equal(got["color"].view(np.uint32), ref["color"].view(np.uint32))
    # camera inside a sphere: t < 0 root rejected (no second root), i.e. the enclosing sphere is a miss
    sph = va.make_spheres([[0, 0, 0], [0, 0, -3]], [1.0, 0.5])
    sb = va.build_index_bvh(sph)
    sdev = va.hip_index_bvh(ctx, sb)
    cam = va.camera()
    cam.perspective(0.6, 1.0, 0.001, 1000.0)
    cam.look_at((0.0, 0.0, 0.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0))
    rt = va.hip_buffer_rt(ctx, 32, 32)
    va.hip_sched(ctx).frame(va.closest_hit_kernel(sdev), va.make_sched_params(cam, rt))
    got = rt.download()
    b = cam.basis(32, 32)
    ocam = tuple(np.array(x[:], np.float32) for x in (b.eye, b.cam_u, b.cam_v, b.cam_w)) + (32, 32)
    ref = O.render(O.Scene("s", O.VO_SPHERE, sph, sb.nodes, sb.indices, None, 0), ocam, mode=O.VO_MODE_PRIMARY)
    assert np.array_equal(got["prim_id"], ref["prim_id"]) and np.array_equal(got["t"].view(np.uint32), ref["t"].view(np.uint32))


def comb_bvh(n):
    """Hand-built 'comb' index BVH of depth n-1 over n triangles along x (valid reference layout):
    inner node at level k has children (leaf: triangle k, inner: level k+1)."""
    xs = np.arange(n, dtype=np.float32) * 0.5
    tris = va.make_triangles(np.stack([xs, np.zeros(n), np.zeros(n)], 1), np.tile([[0.0, 0.4, 0.0]], (n, 1)),
                             np.tile([[0.0, 0.0, 0.4]], (n, 1)))
    nodes = np.zeros(2 * n - 1, va.BVH_NODE_DTYPE)

    def box(lo, hi):
        return [xs[lo], 0.0, 0.0], [xs[hi - 1], 0.4, 0.4]

    inner = 0                       # node index of the inner node for level k
    for k in range(n - 1):
        c = 2 * k + 1
        nodes[inner]["bbox_min"], nodes[inner]["bbox_max"] = box(k, n)
        nodes[inner]["first"], nodes[inner]["num_prims"] = c, 0
        nodes[c]["bbox_min"], nodes[c]["bbox_max"] = box(k, k + 1)
        nodes[c]["first"], nodes[c]["num_prims"] = k, 1
        inner = c + 1
    nodes[inner]["bbox_min"], nodes[inner]["bbox_max"] = box(n - 1, n)
    nodes[inner]["first"], nodes[inner]["num_prims"] = n - 1, 1
    return tris, va.index_bvh(tris, nodes, np.arange(n, dtype=np.uint32), n - 1)


@pytest.mark.parametrize("n", [20, 50, 90, 1000])
def test_deep_trees_overflow_stack_and_rejection(ctx, oracle_mod, n):
    O = oracle_mod
    tris, bvh = comb_bvh(n)
    dev = va.hip_index_bvh(ctx, bvh, va.face_normals(tris))
    assert dev.info["max_depth"] == n - 1
    W, H = 64, 8
    cam = va.camera()
    cam.perspective(1.0, np.float32(W) / np.float32(H), 0.001, 1000.0)
    cam.look_at((-1.0, 0.2, 0.2), (1.0, 0.2, 0.2), (0.0, 1.0, 0.0))
    rt = va.hip_buffer_rt(ctx, W, H)
    if n - 1 > 640:
        # > 160 KiB of stack per 64-lane block: kernels that keep the whole stack in LDS (the
        # counting variant here) reject the BVH; the default AO kernel continues its stack in the
        # global overflow block and renders it exactly (below)
        with pytest.raises(va.VrhError) as e:
            va.hip_sched(ctx).frame(va.ao_kernel(dev, count_tests=True), va.make_sched_params(cam, rt))
        assert e.value.code == _capi.VRH_ERR_UNSUPPORTED
    va.hip_sched(ctx).frame(va.ao_kernel(dev), va.make_sched_params(cam, rt))
    assert ctx.last_frame_stats()["stack_depth"] >= n - 1
    got = rt.download()
    b = cam.basis(W, H)
    ocam = tuple(np.array(x[:], np.float32) for x in (b.eye, b.cam_u, b.cam_v, b.cam_w)) + (W, H)
    ref = O.render(O.Scene("comb", O.VO_TRI, tris, bvh.nodes, bvh.indices, va.face_normals(tris), n - 1), ocam)
    assert (ref["prim_id"] != 0xFFFFFFFF).any()
    assert np.array_equal(got["prim_id"], ref["prim_id"])
    assert np.array_equal(got["t"].view(np.uint32), ref["t"].view(np.uint32))
    assert np.array_equal(got["occ"], ref["occ"])


@pytest.mark.parametrize("samples", [1, 3, 32])
def test_ao_sample_counts(ctx, oracle_mod, samples):
    O = oracle_mod
    name, W, H = "hf64", 160, 90
    out, st = render(ctx, name, W, H, samples=samples)
    sc = O.make_scene(name)
    ref = O.render(sc, O.scene_camera(name, W, H), mode=O.VO_MODE_AO, samples=samples)
    if samples <= 8:
        assert np.array_equal(out["occ"], ref["occ"].astype(np.uint8))
    assert np.array_equal(out["color"].view(np.uint32), ref["color"].view(np.uint32))
    assert st["rays"] == ref["rays"]


def test_background_store_and_clear(ctx):
    """render_target.cpp:19-111 plumbing analogue: misses store the kernel's background exactly."""
    tris = va.make_triangles([[10, 10, 10]], [[0.1, 0, 0]], [[0, 0.1, 0]])
    dev = va.hip_index_bvh(ctx, va.build_index_bvh(tris), va.face_normals(tris))
    cam = va.camera()
    cam.perspective(0.5, 1.0, 0.001, 1000.0)
    cam.look_at((0.0, 0.0, 2.0), (0.0, 0.0, 0.0))
    rt = va.hip_buffer_rt(ctx, 16, 16)
    rt.clear_color_buffer((0.5, 0.5, 0.5, 0.5))
    assert np.all(rt.color() == np.float32(0.5))
    va.hip_sched(ctx).frame(va.ao_kernel(dev, bg=(0.4, 0.4, 0.4, 0.4)), va.make_sched_params(cam, rt))
    got = rt.download()
    assert np.all(got["color"] == np.float32(0.4))
    assert np.all(got["prim_id"] == 0xFFFFFFFF) and np.all(got["t"] == -1.0) and np.all(got["occ"] == 0)


def test_invalid_arguments_are_reported(ctx):
    prims = scenes.primitives("hf64")
    b = va.build_index_bvh(prims)
    bad = va.index_bvh(prims, b.nodes.copy(), b.indices.copy(), b.max_depth)
    bad.indices[3] = len(prims) + 5
    with pytest.raises(va.VrhError) as e:
        va.hip_index_bvh(ctx, bad)
    assert e.value.code == _capi.VRH_ERR_INVALID
    dev = va.hip_index_bvh(ctx, b)             # no normals
    cam, W, H = scenes.scene_camera("hf64", 64, 32)
    rt = va.hip_buffer_rt(ctx, W, H)
    with pytest.raises(va.VrhError):
        va.hip_sched(ctx).frame(va.ao_kernel(dev), va.make_sched_params(cam, rt))   # AO needs normals
    rt2 = va.hip_buffer_rt(ctx, W + 1, H)
    with pytest.raises(va.VrhError):
        va.render(ctx, dev, rt2, cam.basis(W, H), va.closest_hit_kernel(dev))     # size mismatch
