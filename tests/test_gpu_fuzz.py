"""GPU: randomized parity sweep against the oracle (the C restatement of the reference traversal).

Every case draws, from its seed, a scene the fixed fixtures do not cover -- isolated triangles whose
sizes span three decades (some sliver, some nearly degenerate), or spheres of mixed radii, possibly
overlapping -- a camera (outside or inside the scene, at random distance and direction), an image
size (odd sizes, partial 8x8 tiles), the kernel (primary, or AO with a random sample count and
radius) and a frame number, and renders it through the C-ABI both one frame per launch and as frames
in flight (three frames of one launch, each with its own camera and frame number) -- some cases with
the LDS stack cut to 8 entries (the overflow-block instances) or with AO tail sharing on.  Every
pixel's prim id, t, AO mask and colour must be bit-identical to the oracle's.
"""
import numpy as np
import pytest

import visionaray_amd as va

pytestmark = pytest.mark.gpu

SEEDS = list(range(48))


def _scene(rng, kind):
    if kind == "tri":
        n = int(rng.integers(1, 6000))
        c = rng.uniform(-1.0, 1.0, (n, 3))
        size = 10.0 ** rng.uniform(-3.0, -0.5, (n, 1))
        e1 = rng.standard_normal((n, 3)) * size
        e2 = rng.standard_normal((n, 3)) * size
        sliver = rng.random(n) < 0.05                        # nearly degenerate: e2 ~ parallel to e1
        e2[sliver] = e1[sliver] * rng.uniform(0.5, 2.0, (int(sliver.sum()), 1)) + 1e-6 * rng.standard_normal((int(sliver.sum()), 3))
        return va.make_triangles(c - 0.5 * (e1 + e2), e1, e2)
    n = int(rng.integers(1, 4000))
    return va.make_spheres(rng.uniform(-1.0, 1.0, (n, 3)), (10.0 ** rng.uniform(-3.0, -0.7, n)).astype(np.float32))


def _camera(rng, W, H):
    cam = va.camera()
    cam.perspective(float(rng.uniform(0.3, 1.6)), np.float32(W) / np.float32(H), 0.001, 1000.0)
    if rng.random() < 0.25:
        eye = rng.uniform(-0.5, 0.5, 3)                      # inside the scene
    else:
        d = rng.standard_normal(3)
        eye = d / np.linalg.norm(d) * rng.uniform(1.5, 6.0)
    center = rng.uniform(-0.3, 0.3, 3)
    cam.look_at(tuple(float(x) for x in eye), tuple(float(x) for x in center), (0.0, 1.0, 0.0))
    return cam


def _ocam(basis, W, H):
    return (np.array(basis.eye[:], np.float32), np.array(basis.cam_u[:], np.float32),
            np.array(basis.cam_v[:], np.float32), np.array(basis.cam_w[:], np.float32), W, H)


def _same(got, ref, n0=0, n=None):
    sl = slice(n0, None if n is None else n0 + n)
    for k in ("prim_id", "occ"):
        assert np.array_equal(got[k][sl], ref[k]), f"{k}: {int((got[k][sl] != ref[k]).sum())} pixels differ"
    for k in ("t", "color"):
        a, b = got[k][sl].view(np.uint32), ref[k].view(np.uint32)
        assert np.array_equal(a, b), f"{k}: {int((a != b).any(axis=-1).sum() if a.ndim > 1 else (a != b).sum())} pixels differ"


@pytest.mark.parametrize("seed", SEEDS)
def test_random_scenes_cameras_and_kernels_vs_oracle(ctx, oracle_mod, seed):
    O = oracle_mod
    rng = np.random.default_rng(1000 + seed)
    kind = "sph" if seed % 4 == 3 else "tri"        # 8 AO cases, 4 triangle and 4 sphere primary cases
    prims = _scene(rng, kind)
    bvh = va.build_index_bvh(prims)
    nrm = va.face_normals(prims) if kind == "tri" else None
    dev = va.hip_index_bvh(ctx, bvh, nrm)
    W, H = int(rng.integers(9, 140)), int(rng.integers(7, 90))
    ao = kind == "tri" and seed % 4 != 2
    samples, radius = int(rng.integers(1, 9)), float(np.float32(10.0 ** rng.uniform(-2.0, 0.0)))
    kern = va.ao_kernel(dev, samples=samples, radius=radius) if ao else va.closest_hit_kernel(dev)
    osc = O.Scene(f"fuzz{seed}", O.VO_TRI if kind == "tri" else O.VO_SPHERE, prims, bvh.nodes, bvh.indices, nrm,
                  bvh.max_depth)
    mode = O.VO_MODE_AO if ao else O.VO_MODE_PRIMARY
    frame0 = int(rng.integers(0, 50))
    cams = [_camera(rng, W, H) for _ in range(3)]
    bases = [c.basis(W, H) for c in cams]
    refs = [O.render(osc, _ocam(b, W, H), mode=mode, samples=samples, radius=radius, frame_num=frame0 + f)
            for f, b in enumerate(bases)]
    opts = {}
    if seed % 5 == 4 and bvh.max_depth > 8:
        opts["stack_cap"] = 8                                # deeper entries in the overflow block
    if ao and seed % 7 == 6:
        opts["ao_share"] = 1
    for k, v in opts.items():
        ctx.set_option(k, v)
    try:
        # one frame per launch
        rt = va.hip_buffer_rt(ctx, W, H)
        va.hip_sched(ctx).frame(kern, va.make_sched_params(cams[0], rt), frame_num=frame0)
        _same(rt.download(), refs[0])
        # frames in flight: three cameras, frame numbers frame0 .. frame0 + 2, in one launch
        rtb = va.hip_buffer_rt(ctx, W, 3 * H)
        va.render_batch(ctx, dev, rtb, bases, kern, frame_num=frame0)
        got = rtb.download()
        for f in range(3):
            _same(got, refs[f], f * W * H, W * H)
    finally:
        for k in opts:
            ctx.set_option(k, 0)
