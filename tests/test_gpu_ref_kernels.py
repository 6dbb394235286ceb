"""A Visionaray program written for cuda_sched runs on hip_sched with the reference's OWN kernel code
(include/visionaray_hip/reference.h + hip_kernels.h; tests/cpp/ref_kernels.hip, built by
oracle/Makefile into oracle/_ref/ref_kernels because it compiles the reference's headers).

What runs on the GPU is the reference's code -- closest_hit / any_hit / multi_hit (traverse_linear.inl),
the intersectors and hit records, get_normal / get_surface, random_sampler<float>,
cosine_sample_hemisphere, simple::kernel, whitted::kernel -- over the device BVH, whose walk is libvrh's
with the reference's leaf step.  Fixtures come from the reference itself:

  * rs_*       : the AO example's kernel (ao/main.cpp:183-246) verbatim, run by the reference harness
                 (`rsampler` mode, built by clang++ so that the two samp.next() arguments pair the draws
                 as hipcc does) with the per-pixel seeds hip_sched gives a random_sampler
                 (cuda_hash(frame * W * H + y * W + x), cuda_sched.inl:20-45 with the clock replaced);
  * shade_* / whitted_* / multi_* : the harness's simple::kernel / whitted::kernel / multi_hit<16> frames.

Bars: the sampler's draws, every closest-hit t and every pixel's AO count (occluded samples) bit-exact --
cosine_sample_hemisphere's (sampling.h:61-71) float sin / cos are the host library's on the device too
(detail/vrh_libm.h; round 3 used the device's own cosf / sinf and matched 99.9 % of the pixels); shaded
radiance within the north star's 1e-5 relative (device powf), hit lists bit-exact.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "ref_kernels")
GOLDEN = os.path.join(ROOT, "tests", "golden")
BG = np.array([0.1, 0.2, 0.3, 1.0], np.float32)

needs_bin = pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/ref_kernels is built in the build container")


def _use(monkeypatch, variant):
    """run the tests' program as the build `variant` (oracle/Makefile: ref_kernels_<variant>)"""
    b = BIN + "_" + variant
    assert os.path.exists(b), f"oracle/Makefile builds {os.path.basename(b)} next to ref_kernels"
    monkeypatch.setattr(sys.modules[__name__], "BIN", b)


def _run(tmp_path, mode, scene, W, H, *extra):
    out = tmp_path / mode
    out.mkdir()
    subprocess.run([BIN, mode, scene, str(W), str(H), str(out), *map(str, extra)], check=True,
                   capture_output=True, text=True, timeout=120)
    return {"color": np.fromfile(out / "color.bin", np.float32).reshape(-1, 4),
            "t": np.fromfile(out / "t.bin", np.float32), "dir": out}


@pytest.mark.gpu
@needs_bin
@pytest.mark.parametrize("case", ["rs_hf64_160x90_f0", "rs_hf200_320x180_f3", "rs_hf1M_f1"])
def test_random_sampler_draws_bit_exact(tmp_path, golden, oracle_mod, case):
    """kernel(R, random_sampler<S>& samp): draws 0, 1, 2 and 15 of every pixel's sampler equal the
    reference CPU sampler's (std::default_random_engine + uniform_real_distribution<float>)."""
    g = golden[case]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    got = _run(tmp_path, "draws", g["scene"], g["W"], g["H"], g["frame"])["color"]
    assert np.array_equal(got[ref["pixels"]].view(np.uint32), ref["draws"].view(np.uint32))
    assert oracle_mod.fnv1a(got) == g["draws_hash"]


@pytest.mark.gpu
@needs_bin
@pytest.mark.parametrize("case", ["rs_hf64_160x90_f0", "rs_hf200_320x180_f3", "rs_hf1M_f1"])
@pytest.mark.parametrize("variant", ["direct", "share", "defer"])
def test_reference_ao_kernel_on_hip_sched(tmp_path, golden, oracle_mod, case, variant, monkeypatch):
    """ao/main.cpp's kernel, compiled from the reference's headers by hipcc: hits, t and every pixel's
    AO count bit-exact.  share: the build with the shared any-hit walk (VRH_USER_ANYHIT_SHARE=1,
    oracle/_ref/ref_kernels_share); defer: deferred any_hit calls (VRH_USER_DEFER=1, record / trace /
    replay, oracle/_ref/ref_kernels_defer)."""
    if variant != "direct":
        _use(monkeypatch, variant)
    g = golden[case]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    out = _run(tmp_path, "ao", g["scene"], g["W"], g["H"], g["frame"])
    color, t = out["color"], out["t"]
    hit = ~np.all(color == BG, axis=1)
    assert int(hit.sum()) == g["hits"]
    assert np.array_equal(hit, ref["ao_count"] != 255)
    t_ref_layout = np.where(hit, t, np.float32(-1.0)).astype(np.float32)
    assert oracle_mod.fnv1a(t_ref_layout) == g["t_hash"], "closest-hit t differs from the reference"
    k = np.where(hit, np.rint((1.0 - color[:, 0]) * 8.0), 255).astype(np.uint8)
    # every pixel's occluded-sample count is the reference's: the device sin / cos of
    # cosine_sample_hemisphere are the host library's (detail/vrh_libm.h)
    bad = np.flatnonzero(k != ref["ao_count"])
    assert bad.size == 0, f"AO count differs on {bad.size} pixels, first {bad[:8].tolist()}"
    assert int(k[hit].astype(np.int64).sum()) == g["occluded_samples"]


UK_BIN = os.path.join(ROOT, "build", "tests", "user_kernels")
GRID = {"hf64": 64, "hf200": 200, "hf1M": 708}


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["rs_hf64_160x90_f0", "rs_hf1M_f1"])
@pytest.mark.parametrize("prog", ["user_kernels", "uk_defer"])
def test_standalone_random_sampler_and_ao_kernel(tmp_path, golden, oracle_mod, case, prog):
    """Without the reference headers (hip_kernels.h + standalone.h): the restated random_sampler<float>
    draws bit-exact, the AO example's kernel with the restated cosine_sample_hemisphere on the same bar
    as the reference-header build (every AO count exact); uk_defer: deferred any_hit calls."""
    UK_BIN = os.path.join(ROOT, "build", "tests", prog)
    g = golden[case]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    d = tmp_path / "d"
    d.mkdir()
    args = [str(GRID[g["scene"]]), str(g["W"]), str(g["H"]), str(d), str(g["frame"])]
    subprocess.run([UK_BIN, "draws", *args], check=True, capture_output=True, timeout=120)
    draws = np.fromfile(d / "color.bin", np.float32).reshape(-1, 4)
    assert oracle_mod.fnv1a(draws) == g["draws_hash"]
    subprocess.run([UK_BIN, "rsao", *args], check=True, capture_output=True, timeout=120)
    color = np.fromfile(d / "color.bin", np.float32).reshape(-1, 4)
    t = np.fromfile(d / "t.bin", np.float32)
    hit = ~np.all(color == BG, axis=1)
    assert np.array_equal(hit, ref["ao_count"] != 255)
    assert oracle_mod.fnv1a(np.where(hit, t, np.float32(-1.0)).astype(np.float32)) == g["t_hash"]
    k = np.where(hit, np.rint((1.0 - color[:, 0]) * 8.0), 255).astype(np.uint8)
    assert np.array_equal(k, ref["ao_count"])


@pytest.mark.gpu
@needs_bin
@pytest.mark.parametrize("case,mode", [("shade_hf64_face", "shade"), ("shade_hf64_vertex", "shade"),
                                       ("shade_cornell12_face", "shade"), ("shade_cornell12_vertex", "shade"),
                                       ("whitted_hf64_vertex", "whitted"), ("whitted_cornell12_face", "whitted"),
                                       ("whitted_hfstack32x24_face", "whitted")])
@pytest.mark.parametrize("variant", ["direct", "defer"])
def test_reference_shading_kernels_on_hip_sched(tmp_path, golden, case, mode, variant, monkeypatch):
    """simple::kernel / whitted::kernel (the reference's own code, kernels.h make_kernel_params over
    device refs, materials and lights) against the reference's frames: misses bit-exact, radiance
    within 1e-5 relative.  defer: the shadow rays deferred and the bounces replayed (VRH_USER_DEFER=1)."""
    if variant != "direct":
        _use(monkeypatch, variant)
    g = golden[case]
    extra = [g["binding"]] + ([g["bounces"], g["eps"]] if mode == "whitted" else [])
    got = _run(tmp_path, mode, g["scene"], g["W"], g["H"], *extra)["color"]
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))["color"]
    miss = np.all(ref == BG, axis=1)
    assert np.array_equal(got[miss].view(np.uint32), ref[miss].view(np.uint32))
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=0.0)


@pytest.mark.gpu
@needs_bin
@pytest.mark.parametrize("case", ["multi_hfstack32x24_face", "multi_hfstack32x24_vertex", "multi_cornell12_face"])
@pytest.mark.parametrize("variant", ["direct", "defer"])
def test_reference_multi_hit_on_hip_sched(tmp_path, golden, case, variant, monkeypatch):
    """multi_hit<16>(ray, refs) through the reference's traverse / insert_sorted on the device BVH: hit
    lists bit-exact; the multi_hit example's compositing within 1e-5 (defer: multi_hit is never
    deferred, the build must still give the same lists)."""
    if variant != "direct":
        _use(monkeypatch, variant)
    g = golden[case]
    out = _run(tmp_path, "multi", g["scene"], g["W"], g["H"], g["binding"])
    ref = np.load(os.path.join(GOLDEN, case + ".npz"))
    pid = np.fromfile(out["dir"] / "mh_prim_id.bin", np.uint32).reshape(-1, 16)
    mt = np.fromfile(out["dir"] / "mh_t.bin", np.float32).reshape(-1, 16)
    assert np.array_equal(pid, ref["mh_prim_id"]), f"{(pid != ref['mh_prim_id']).any(1).sum()} pixels' lists differ"
    assert np.array_equal(mt.view(np.uint32), ref["mh_t"].view(np.uint32))
    assert int((pid != 0xFFFFFFFF).sum()) == g["hits"]
    np.testing.assert_allclose(out["color"], ref["color"], rtol=1e-5, atol=1e-7)


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="reference headers absent")
def test_reference_headers_compile_for_the_device(tmp_path):
    """reference.h makes the reference headers device code: a hipcc -fsyntax-only of a kernel using
    random_sampler / cosine_sample_hemisphere / closest_hit over hip_index_bvh refs succeeds, and the
    header refuses a host compiler."""
    src = tmp_path / "k.hip"
    src.write_text(
        "#include <visionaray_hip/reference.h>\n#include <visionaray_hip/hip_kernels.h>\n"
        "using namespace visionaray;\n"
        "__global__ void k(hip_bvh_ref_t<basic_triangle<3, float>> const* b, float* o) {\n"
        "  random_sampler<float> s(7u); auto d = cosine_sample_hemisphere(s.next(), s.next());\n"
        "  basic_ray<float> r(vec3(0.0f), d); auto h = closest_hit(r, b, b + 1); o[0] = h.t;\n"
        "  auto a = any_hit(r, b, b + 1, 0.5f); o[1] = a.hit ? 1.0f : 0.0f;\n"
        "  auto m = multi_hit<4>(r, b, b + 1); o[2] = m[3].t; }\n")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-w",
                    "-I/root/reference/include", "-I", os.path.join(ROOT, "include"), str(src)], check=True)
    host = tmp_path / "h.cpp"
    host.write_text("#include <visionaray_hip/reference.h>\nint main() { return 0; }\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I/root/reference/include", "-I",
                        os.path.join(ROOT, "include"), str(host)], capture_output=True, text=True)
    assert r.returncode != 0 and "compile this translation unit with hipcc" in r.stderr
