"""CPU: the C-ABI library (libvrh.so) loads, exports every symbol include/vrh.h declares, and its host
components (binned-SAH builder, scene generators, camera basis) are bit-identical to the oracle.
No device compute here -- the build container has no GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import _capi, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "vrh.h")).read()
    return sorted(set(re.findall(r"VRH_API\s+[\w\s\*]+?\b(vrh_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    names = declared_symbols()
    assert len(names) >= 25
    lib = _capi.lib()
    for n in names:
        assert hasattr(lib, n), f"libvrh.so does not export {n}"
    assert set(names) == set(_capi.SIGNATURES), "python binding signatures out of sync with include/vrh.h"
    assert b"gfx950" in lib.vrh_version()


def test_library_contains_gfx950_code_object():
    data = open(_capi.LIB_PATH, "rb").read()
    assert b"gfx950" in data and b"render_unified_kernel" in data and b"unshard_kernel" in data


@pytest.mark.parametrize("name", ["cornell12", "hf64", "hf200", "sph5000", "hf1M", "sph1M"])
def test_scene_generators_and_builder_match_oracle(oracle_mod, name):
    O = oracle_mod
    prims = scenes.primitives(name)
    kind, oprims = O.gen_prims(name)
    assert prims.tobytes() == oprims.tobytes()
    b = va.build_index_bvh(prims)
    on, oi, od = O.build_bvh(oprims, kind)
    assert b.nodes.tobytes() == on.tobytes()
    assert np.array_equal(b.indices, oi)
    assert b.max_depth == od
    if kind == O.VO_TRI:
        assert va.face_normals(prims).tobytes() == O.face_normals(oprims).tobytes()


@pytest.mark.parametrize("case", ["hf1M", "sph1M", "hf10M"])
def test_parallel_builder_matches_reference_hashes_full_size(oracle_mod, golden, case):
    """The product builder (subtrees of >= 32K refs on parallel threads) reproduces the reference
    builder's node and index arrays at full size (hashes recorded from the reference)."""
    g = golden[case]
    b = va.build_index_bvh(scenes.primitives(g["scene"]))
    assert oracle_mod.fnv1a(b.nodes) == g["bvh_hash"] and oracle_mod.fnv1a(b.indices) == g["idx_hash"]
    assert len(b.nodes) == g["nodes"] and b.max_depth == g["max_depth"]


def _soup(rng, n, spread=1.0):
    v1 = rng.uniform(-spread, spread, (n, 3)).astype(np.float32)
    e1 = rng.uniform(-0.2, 0.2, (n, 3)).astype(np.float32)
    e2 = rng.uniform(-0.2, 0.2, (n, 3)).astype(np.float32)
    return va.make_triangles(v1, e1, e2)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 17, 1000, 20000, 150000])
def test_builder_random_soups_identical(oracle_mod, n):
    O = oracle_mod
    rng = np.random.default_rng(n)
    tris = _soup(rng, n)
    b = va.build_index_bvh(tris)
    on, oi, _ = O.build_bvh(tris, O.VO_TRI)
    assert b.nodes.tobytes() == on.tobytes() and np.array_equal(b.indices, oi)


def test_parallel_builder_clustered_and_duplicate_inputs(oracle_mod):
    """Inputs large enough to split on parallel threads (>= 32K refs per forked range) whose
    subtrees differ a lot in size: tight clusters, many identical centroids, a long thin strip."""
    O = oracle_mod
    rng = np.random.default_rng(11)
    centres = rng.uniform(-4, 4, (6, 3))
    pts = np.concatenate([c + rng.normal(0, 0.01 * (k + 1), (20000 * (k + 1), 3)) for k, c in enumerate(centres)])
    dup = np.repeat(rng.uniform(-1, 1, (500, 3)), 80, axis=0)
    strip = np.stack([np.linspace(-50, 50, 60000), np.zeros(60000), np.zeros(60000)], 1)
    for v in (pts, dup, strip):
        v = v.astype(np.float32)
        tris = va.make_triangles(v, np.full_like(v, 0.01), np.tile(np.float32([[0.01, -0.01, 0.005]]), (len(v), 1)))
        b = va.build_index_bvh(tris)
        on, oi, od = O.build_bvh(tris, O.VO_TRI)
        assert b.nodes.tobytes() == on.tobytes() and np.array_equal(b.indices, oi) and b.max_depth == od


def test_builder_degenerate_inputs_identical(oracle_mod):
    O = oracle_mod
    # identical centroids (no split possible -> one big leaf), collinear, and quantised coordinates
    same = va.make_triangles(np.zeros((40, 3)), np.ones((40, 3)) * 0.1, np.ones((40, 3)) * -0.1)
    line = va.make_triangles(np.stack([np.arange(64), np.zeros(64), np.zeros(64)], 1) * 0.25,
                             np.full((64, 3), 0.05), np.full((64, 3), -0.05))
    rng = np.random.default_rng(7)
    quant = va.make_triangles(np.round(rng.uniform(-1, 1, (3000, 3)) * 4) / 4, np.full((3000, 3), 0.1),
                              np.tile([[0.1, -0.1, 0.0]], (3000, 1)))
    for tris in (same, line, quant):
        b = va.build_index_bvh(tris)
        on, oi, _ = O.build_bvh(tris, O.VO_TRI)
        assert b.nodes.tobytes() == on.tobytes() and np.array_equal(b.indices, oi)
    b = va.build_index_bvh(same)
    assert len(b.nodes) == 1 and b.nodes[0]["num_prims"] == 40


def test_builder_spheres_identical(oracle_mod):
    O = oracle_mod
    rng = np.random.default_rng(3)
    s = va.make_spheres(rng.uniform(-1, 1, (5000, 3)), rng.uniform(0.001, 0.05, 5000))
    b = va.build_index_bvh(s)
    on, oi, _ = O.build_bvh(s, O.VO_SPHERE)
    assert b.nodes.tobytes() == on.tobytes() and np.array_equal(b.indices, oi)


def test_camera_basis_bits(golden):
    for case in ("cornell12", "hf1M", "sph1M"):
        g = golden[case]
        cam, W, H = scenes.scene_camera(g["scene"], g["W"], g["H"])
        b = cam.basis(W, H)
        for got, want in ((b.cam_u, g["cam_u"]), (b.cam_v, g["cam_v"]), (b.cam_w, g["cam_w"])):
            assert ["%08x" % x for x in np.array(got[:], np.float32).view(np.uint32)] == want


def test_shard_band_arithmetic():
    for H in (1, 15, 16, 17, 1080, 512):
        bands = (H + 7) // 8
        for N in (1, 2, 3, 4, 8):
            got = [va.shard_bands(H, g, N) for g in range(N)]
            assert sum(got) == bands
            assert got == [len(range(g, bands, N)) for g in range(N)]


def test_error_paths_without_device():
    lib = _capi.lib()
    # invalid arguments are reported, not crashed on
    assert lib.vrh_build_bvh(None, 0, 0, None, None, None, None) == _capi.VRH_ERR_INVALID
    assert b"vrh_build_bvh" in lib.vrh_last_error()
    with pytest.raises(va.VrhError):
        _capi.check("vrh_gen_heightfield", 0, None)
    with pytest.raises(ValueError):
        va.build_index_bvh(np.zeros(0, va.TRIANGLE_DTYPE))
    if va.device_count() == 0:
        h = C.c_void_p()
        assert lib.vrh_ctx_create(0, C.byref(h)) == _capi.VRH_ERR_NO_DEVICE
        assert not h.value


def test_unsupported_primitive_dtype():
    with pytest.raises(TypeError):
        va.build_index_bvh(np.zeros(4, np.float32))


@pytest.mark.parametrize("name", ["cornell12", "hf64", "hf200", "sph5000", "hf1M", "sph1M"])
def test_sah_cost_matches_reference(golden, name):
    """vrh_bvh_sah_cost (statistics.h:30-73) of the product-built tree == the reference's own value, bit for bit."""
    b = va.build_index_bvh(scenes.primitives(name))
    c = np.float32(va.sah_cost(b.nodes)).view(np.uint32)
    assert "%08x" % int(c) == golden["sah_cost_bits"][name]


def test_kernel_source_hash_identifies_the_build(tmp_path):
    """bench.py reports a committed PMC pass only for the kernel sources it was measured on
    (visionaray_amd/buildinfo.py): the hash covers every kernel source and changes with any of them."""
    import os
    from visionaray_amd import buildinfo
    files = buildinfo.kernel_sources()
    assert all(os.path.exists(p) for p in files)
    assert any(p.endswith("vrh_kernels.hip") for p in files) and any(p.endswith("vrh_device.h") for p in files)
    h = buildinfo.kernel_source_sha256()
    assert len(h) == 64 and h == buildinfo.kernel_source_sha256()
    orig = buildinfo.kernel_sources
    extra = tmp_path / "x.h"
    extra.write_text("// x\n")
    try:
        buildinfo.kernel_sources = lambda: orig() + [str(extra)]
        assert buildinfo.kernel_source_sha256() != h
    finally:
        buildinfo.kernel_sources = orig


def test_user_kernel_source_hash_covers_the_user_kernel_headers():
    """The user-kernel PMC passes (profiles/pmc_user_*.json, pmc_sq_lambda.json) are reported only for
    the sources they were measured on: libvrh's kernel sources plus the device headers the user programs
    are compiled from and the bench's user-kernel program."""
    import os
    from visionaray_amd import buildinfo
    files = buildinfo.user_kernel_sources()
    assert all(os.path.exists(p) for p in files)
    for name in ("hip_kernels.h", "hip_backend.h", "vrh_device.h", "user_kernels.hip", "vrh_kernels.hip"):
        assert any(os.path.basename(p) == name for p in files), name
    h = buildinfo.user_kernel_source_sha256()
    assert len(h) == 64 and h != buildinfo.kernel_source_sha256()
