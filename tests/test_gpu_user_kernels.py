"""User kernels and custom intersectors (include/visionaray_hip/hip_kernels.h):
a device lambda handed to hip_sched::frame, traversing the device BVH with closest_hit / any_hit and
a basic_intersector subclass, reproduces the reference's own frames bit for bit.

tests/cpp/user_kernels.hip (built by visionaray_amd/Makefile `cpp_tests`) renders:
  * ao    -- the reference harness's AO kernel as a user lambda, default intersector
             (fixtures: hf200_320x180 frame 0, frame1_hf200_320x180);
  * mask  -- the same kernel with a byte-mask basic_intersector (fixtures: mask_* from the harness's
             mask_intersector);
  * heart -- closest hit with the intersector example's procedural cut-out, written in the example's
             width-generic style (unpack / simd::mask_type_t / Mask(bool[N]) / pow), against the
             reference harness's "heart" mode (fixtures: heart_*);
  * list  -- the AO kernel over a list of two BVH refs with a scissor box (fixtures: list_*);
  * isect -- the mask case with the intersector passed in the sched params (kernel(isect, r, x, y)).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.environ.get("VRH_USER_BIN") or os.path.join(ROOT, "build", "tests", "user_kernels")
GOLDEN = os.path.join(ROOT, "tests", "golden")
GRID = {"hf64": 64, "hf200": 200}


DEFER_BIN = os.path.join(ROOT, "build", "tests", "uk_defer")
VARIANTS = {"direct": None, "defer": DEFER_BIN}


@pytest.fixture(params=list(VARIANTS))
def ukbin(request, monkeypatch):
    """Every user-kernel case twice: the default build, and the build with deferred any_hit calls
    (hip_kernels.h VRH_USER_DEFER=1: record, trace the tile's any_hit rays as one pool, replay), whose
    frames must be the same bits."""
    b = VARIANTS[request.param] or BIN
    assert os.path.exists(b), "run __graft_entry__.build() (make -C visionaray_amd cpp_tests)"
    monkeypatch.setattr(sys.modules[__name__], "BIN", b)
    return b


def _run(tmp_path, mode, scene, W, H, *extra):
    out = tmp_path / mode
    out.mkdir()
    subprocess.run([BIN, mode, str(GRID[scene]), str(W), str(H), str(out), *map(str, extra)], check=True,
                   capture_output=True, text=True, timeout=120)
    return {"prim_id": np.fromfile(out / "prim_id.bin", np.uint32), "t": np.fromfile(out / "t.bin", np.float32),
            "occ": np.fromfile(out / "occ.bin", np.uint8),
            "color": np.fromfile(out / "color.bin", np.float32).reshape(-1, 4)}


def _check_hashes(oracle_mod, got, g, keys):
    for k, hk in keys:
        assert oracle_mod.fnv1a(got[k]) == g[hk], f"{k}: FNV-1a hash differs from the reference's frame"


@pytest.mark.gpu
@pytest.mark.parametrize("case,frame", [("hf200_320x180", 0), ("frame1_hf200_320x180", 1)])
def test_user_ao_kernel_matches_reference(tmp_path, golden, oracle_mod, case, frame, ukbin):
    g = golden[case]
    got = _run(tmp_path, "ao", g["scene"], g["W"], g["H"], frame)
    _check_hashes(oracle_mod, got, g, [("prim_id", "primid_hash"), ("t", "t_hash"), ("occ", "occ_hash"),
                                       ("color", "color_hash")])


SHARE_BIN = os.path.join(ROOT, "build", "tests", "uk_share")


@pytest.mark.gpu
@pytest.mark.parametrize("case,frame", [("hf200_320x180", 0), ("frame1_hf200_320x180", 1)])
def test_user_ao_kernel_shared_anyhit_matches_reference(tmp_path, golden, oracle_mod, case, frame, monkeypatch):
    """VRH_USER_ANYHIT_SHARE=1: idle lanes walk subtrees of other lanes' any-hit rays; every ray's
    hit / miss -- so every AO mask and colour -- is still the reference's."""
    assert os.path.exists(SHARE_BIN), "run __graft_entry__.build() (make -C visionaray_amd cpp_tests)"
    monkeypatch.setattr(sys.modules[__name__], "BIN", SHARE_BIN)
    g = golden[case]
    got = _run(tmp_path, "ao", g["scene"], g["W"], g["H"], frame)
    _check_hashes(oracle_mod, got, g, [("prim_id", "primid_hash"), ("t", "t_hash"), ("occ", "occ_hash"),
                                       ("color", "color_hash")])


CUT_BIN = os.path.join(ROOT, "build", "tests", "uk_cut")
OCA_BIN = os.path.join(ROOT, "build", "tests", "uk_oca")


@pytest.mark.gpu
@pytest.mark.parametrize("grid,W,H,frame,radius", [(200, 320, 180, 0, 0.1), (200, 320, 180, 5, 0.4),
                                                   (708, 1920, 1080, 2, 0.1), (64, 160, 90, 1, 2.0)])
def test_anyhit_entry_cut_returns_reference_order_records(tmp_path, grid, W, H, frame, radius):
    """The opt-in any_hit entry cut (hip_kernels.h VRH_USER_ANYHIT_CUT=1, user_cut_entry: a skeleton of
    the BVH's top in LDS, chains skipped only where boxes nest) walks the same leaves in the same order
    as the walk from the root: every any_hit call of the AO lambda returns the same hit RECORD (prim id
    and t of the first hit found), not only the same hit / miss -- against the default build.  So do
    the deferred build and the ordered cooperative walk (VRH_USER_ANYHIT_ORDERED=1: lanes share the
    calls' work, every segment keyed by its place in the ray's walk order)."""
    for b in (CUT_BIN, DEFER_BIN, OCA_BIN):
        assert os.path.exists(b), "run __graft_entry__.build() (make -C visionaray_amd cpp_tests)"
    outs = []
    for b in (CUT_BIN, DEFER_BIN, OCA_BIN, BIN):
        d = tmp_path / os.path.basename(b)
        d.mkdir()
        subprocess.run([b, "anyrec", str(grid), str(W), str(H), str(d), str(frame), str(radius)], check=True,
                       capture_output=True, text=True, timeout=120)
        outs.append(np.fromfile(d / "color.bin", np.float32).reshape(-1, 4))
    ref = outs[-1]
    assert float((ref[:, 1] > 0).mean()) > 0.01, "the case must have occluded AO rays"
    # the deferred build (VRH_USER_DEFER=1) traces the same calls in a pool, in the same walk order:
    # the same records too
    for name, got in zip(("entry cut", "deferred", "ordered cooperative walk"), outs[:3]):
        bad = np.flatnonzero(np.any(got.view(np.uint32) != ref.view(np.uint32), axis=1))
        assert bad.size == 0, f"{name}: {bad.size} pixels' any_hit records differ, first {bad[:8].tolist()}"


@pytest.mark.gpu
@pytest.mark.parametrize("grid,W,H,frame,radius", [(200, 320, 180, 0, 0.1), (708, 1920, 1080, 4, 0.1),
                                                   (64, 160, 90, 2, 0.5)])
def test_deferred_replay_with_more_calls_than_recorded(tmp_path, grid, W, H, frame, radius):
    """A kernel whose later any_hit calls depend on earlier answers (the `chain` mode: a hit adds two
    more calls): the record phase of VRH_USER_DEFER sees only the first call per sample (answered "no
    hit" until the trace), the replay makes up to three.  The calls past each lane's recorded count run
    directly -- the log slots there belong to an earlier tile -- so every record equals the direct build's."""
    outs = []
    for b in (BIN, DEFER_BIN):
        assert os.path.exists(b), "run __graft_entry__.build() (make -C visionaray_amd cpp_tests)"
        d = tmp_path / os.path.basename(b)
        d.mkdir()
        subprocess.run([b, "chain", str(grid), str(W), str(H), str(d), str(frame), str(radius)], check=True,
                       capture_output=True, text=True, timeout=120)
        outs.append(np.fromfile(d / "color.bin", np.float32).reshape(-1, 4))
    direct, deferred = outs
    calls = direct[:, 1]
    assert float((calls > 4).mean()) > 0.01, "the case must have pixels whose replay makes extra calls"
    bad = np.flatnonzero(np.any(deferred.view(np.uint32) != direct.view(np.uint32), axis=1))
    assert bad.size == 0, f"deferred: {bad.size} pixels differ, first {bad[:8].tolist()}"


@pytest.mark.gpu
@pytest.mark.parametrize("n,W,H,frame,radius", [(20000, 320, 180, 3, 0.3), (8000, 160, 90, 1, 0.8),
                                                 (1000000, 96, 54, 2, 0.05)])
def test_user_kernel_on_spheres_closest_hit_and_deferred_records(tmp_path, oracle_mod, n, W, H, frame, radius):
    """closest_hit / any_hit over a sphere BVH (basic_sphere<float>, vrh_gen_spheres) in a user lambda:
    every pixel's closest hit (prim id, t) equals the oracle's primary render of the same scene and
    camera, and the deferred build (VRH_USER_DEFER=1, its trace on the sphere path) returns the direct
    build's any_hit RECORDS for 8 rays per hit.  1M spheres: a BVH 26 levels deep, deeper than the
    short LDS stack (VRH_USER_LDS_STACK), so the launch gives the whole stack."""
    outs = []
    for b in (BIN, DEFER_BIN):
        assert os.path.exists(b), "run __graft_entry__.build() (make -C visionaray_amd cpp_tests)"
        d = tmp_path / os.path.basename(b)
        d.mkdir()
        subprocess.run([b, "sphrec", "64", str(W), str(H), str(d), str(frame), str(radius), str(n)], check=True,
                       capture_output=True, text=True, timeout=120)
        outs.append(np.fromfile(d / "color.bin", np.float32).reshape(-1, 4))
    direct, deferred = outs
    bad = np.flatnonzero(np.any(deferred.view(np.uint32) != direct.view(np.uint32), axis=1))
    assert bad.size == 0, f"deferred: {bad.size} pixels differ, first {bad[:8].tolist()}"
    pid = direct[:, 2].view(np.uint32)
    hit = pid != 0xFFFFFFFF
    assert hit.mean() > 0.02 and float((direct[hit, 1] > 0).mean()) > 0.01, "the case must have hits and occluded rays"
    O = oracle_mod
    ref = O.render(O.make_scene(f"sph{n}"), O.scene_camera(f"sph{n}", W, H), mode=O.VO_MODE_PRIMARY)
    assert np.array_equal(pid, ref["prim_id"]), f"{int((pid != ref['prim_id']).sum())} pixels' closest hit differs from the oracle"
    assert np.array_equal(direct[hit, 3].view(np.uint32), ref["t"][hit].view(np.uint32)), "closest-hit t"


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["mask_hf200_320x180", "mask_hf64_160x90"])
def test_user_mask_intersector_matches_reference(tmp_path, golden, oracle_mod, case, ukbin):
    g = golden[case]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    mpath = tmp_path / "mask.bin"
    ref["mask"].astype(np.uint8).tofile(mpath)
    got = _run(tmp_path, "mask", g["scene"], g["W"], g["H"], mpath, g["mask_size"])
    for k in ("prim_id", "occ"):
        assert np.array_equal(got[k], ref[k]), f"{k}: {int((got[k] != ref[k]).sum())} pixels differ"
    for k in ("t", "color"):
        assert np.array_equal(got[k].view(np.uint32), ref[k].view(np.uint32)), k
    _check_hashes(oracle_mod, got, g, [("prim_id", "primid_hash"), ("t", "t_hash"), ("occ", "occ_hash"),
                                       ("color", "color_hash")])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["jittered", "jittered_blend", "ssaa2", "ssaa4", "ssaa8"])
def test_user_kernel_pixel_samplers_match_reference(tmp_path, golden, kind, ukbin):
    """make_sched_params(pixel_sampler::<kind>, cam, rt) with a user kernel: the reference harness's
    sampler frames (colour blended onto the same initial target, the last sample's prim id)."""
    case = f"sampler_{kind}_hf64_ao"
    g = golden[case]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    out = tmp_path / "s"
    out.mkdir()
    subprocess.run([BIN, "sampler", str(GRID[g["scene"]]), str(g["W"]), str(g["H"]), str(out), kind, str(g["frame"])],
                   check=True, capture_output=True, text=True, timeout=120)
    pid = np.fromfile(out / "sampler_prim_id.bin", np.uint32)
    color = np.fromfile(out / "sampler_color.bin", np.float32).reshape(-1, 4)
    assert np.array_equal(pid, ref["prim_id"])
    assert np.array_equal(color.view(np.uint32), ref["color"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["matrix_uniform_hf64_ao", "matrix_ssaa4_hf64_ao"])
def test_user_kernel_camera_matrices_match_reference(tmp_path, golden, case, ukbin):
    """make_sched_params(sampler, view_matrix, proj_matrix, rt) with a user kernel: the reference
    harness's matrix-camera frames (sched_common.h:152-176)."""
    g = golden[case]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    out = tmp_path / "m"
    out.mkdir()
    mpath = tmp_path / "mats.bin"
    np.concatenate([ref["view"], ref["proj"]]).astype(np.float32).tofile(mpath)
    subprocess.run([BIN, "sampler", str(GRID[g["scene"]]), str(g["W"]), str(g["H"]), str(out), g["sampler"],
                    str(g["frame"]), str(mpath)], check=True, capture_output=True, text=True, timeout=120)
    pid = np.fromfile(out / "sampler_prim_id.bin", np.uint32)
    color = np.fromfile(out / "sampler_color.bin", np.float32).reshape(-1, 4)
    assert np.array_equal(pid, ref["prim_id"])
    assert np.array_equal(color.view(np.uint32), ref["color"].view(np.uint32))


@pytest.mark.gpu
def test_user_kernel_with_intersector_in_sched_params(tmp_path, golden, oracle_mod, ukbin):
    """make_sched_params(sampler, cam, rt, isect) (scheduler.h:177-193): hip_sched calls the kernel as
    kernel(isect, r, x, y) (sched_common.h:786-818) -- the mask frames again."""
    case = "mask_hf200_320x180"
    g = golden[case]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    mpath = tmp_path / "mask.bin"
    ref["mask"].astype(np.uint8).tofile(mpath)
    got = _run(tmp_path, "isect", g["scene"], g["W"], g["H"], mpath, g["mask_size"])
    for k in ("prim_id", "occ"):
        assert np.array_equal(got[k], ref[k]), f"{k}: {int((got[k] != ref[k]).sum())} pixels differ"
    _check_hashes(oracle_mod, got, g, [("prim_id", "primid_hash"), ("t", "t_hash"), ("occ", "occ_hash"),
                                       ("color", "color_hash")])


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["heart_hf64_160x90", "heart_hf200_320x180"])
def test_user_heart_intersector_matches_reference(tmp_path, golden, case, ukbin):
    g = golden[case]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    got = _run(tmp_path, "heart", g["scene"], g["W"], g["H"])
    diff = int((got["prim_id"] != ref["prim_id"]).sum())
    assert diff == 0, f"{diff} pixels' prim id differ from the reference"
    assert np.array_equal(got["t"].view(np.uint32), ref["t"].view(np.uint32))
    assert int((got["prim_id"] != 0xFFFFFFFF).sum()) == g["hits"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["list_hf64_160x90", "list_hf200_320x180"])
def test_user_kernel_over_bvh_list_with_scissor_matches_reference(tmp_path, golden, oracle_mod, case, ukbin):
    """closest_hit / any_hit over a list of two BVH refs (traverse_linear.inl:76-141) in a user lambda,
    with the scissor box honoured by the user-kernel launch (cuda_sched.inl:71)."""
    g = golden[case]
    got = _run(tmp_path, "list", g["scene"], g["W"], g["H"], *g["scissor"], g["frame"])
    _check_hashes(oracle_mod, got, g, [("prim_id", "primid_hash"), ("t", "t_hash"), ("occ", "occ_hash"),
                                       ("color", "color_hash")])


@pytest.mark.gpu
@pytest.mark.parametrize("scene,W,H,nf", [("hf64", 160, 90, 3), ("hf200", 333, 181, 3), ("hf64", 160, 90, 8),
                                          ("hf200", 333, 181, 32)])
def test_user_kernel_frames_in_flight_equal_single_frames(tmp_path, scene, W, H, nf, ukbin):
    """hip_sched::frames with a user kernel (one persistent launch, nf cameras, frame numbers
    f0 .. f0 + nf - 1) equals nf frame() calls bit for bit, and the frames differ (ragged width and
    height: partial tiles at the right and bottom edges)."""
    r = subprocess.run([BIN, "frames", str(GRID[scene]), str(W), str(H), str(tmp_path), "7", str(nf)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert '"frames_ok":true' in r.stdout and '"distinct":true' in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("scene,W,H,frame", [("hf64", 160, 90, 0), ("hf200", 333, 181, 3)])
def test_user_kernel_lanes_on_different_bvhs(tmp_path, scene, W, H, frame, ukbin):
    """closest_hit / any_hit calls in which the lanes of a wave walk different BVHs (chosen per pixel)
    give the records the same calls give when every lane walks the same BVH: the scalar-cache fetches
    of wave-uniform records must not take one lane's BVH for another's (their roots share an index)."""
    r = subprocess.run([BIN, "divbvh", str(GRID[scene]), str(W), str(H), str(tmp_path), str(frame)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert '"same":true' in r.stdout and '"same_hits":true' in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("binary", ["uk_share", "uk_oca", "uk_cut"])
def test_any_hit_variants_with_lanes_on_different_bvhs(tmp_path, binary):
    """The opt-in any_hit walks with the lanes of a wave on different BVHs: the shared walk (whose
    lanes take over each other's subtrees) falls back to per-lane walks and keeps every hit / miss
    answer (which hit it reports may differ by design); the ordered walk and the entry cut keep the
    records too."""
    b = os.path.join(ROOT, "build", "tests", binary)
    assert os.path.exists(b), "make -C visionaray_amd cpp_tests"
    r = subprocess.run([b, "divbvh", "200", "333", "181", str(tmp_path), "3"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert '"same_hits":true' in r.stdout
    if binary != "uk_share":
        assert '"same":true' in r.stdout


def test_user_kernel_header_needs_hipcc(tmp_path):
    """hip_kernels.h is device code: a host compiler gets a clear error, not a silent host path."""
    src = tmp_path / "host.cpp"
    src.write_text("#include <visionaray_hip/hip_kernels.h>\nint main() { return 0; }\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "compile this translation unit with hipcc" in r.stderr


def test_user_kernel_program_is_built():
    """build() compiled the user-kernel programs for gfx950 (they travel to the GPU box with the tree)."""
    for b in (BIN, DEFER_BIN, SHARE_BIN, CUT_BIN, OCA_BIN):
        assert os.path.exists(b), f"{b}: run __graft_entry__.build() (make -C visionaray_amd cpp_tests)"


@pytest.mark.gpu
def test_user_kernel_launch_takes_short_stacks_and_six_waves():
    """The AO lambda's launch on hf1M (a BVH 20 levels deep): 24 LDS stack entries per thread and the
    6-wave instance, 24 one-wave blocks per CU (hip_kernels.h launch_user_render; the bench line's
    user_kernel.launch) -- LDS, not registers, had held the user kernels under 5 waves per SIMD."""
    r = subprocess.run([BIN, "bench", "708", "1920", "1080", "/tmp", "1", "32"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    rec = next(json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{") and "frame_ms_median" in ln)
    assert rec["launch"]["stack_entries"] == 24
    assert rec["launch"]["waves_target"] == 6 and rec["launch"]["blocks_per_cu"] == 24
