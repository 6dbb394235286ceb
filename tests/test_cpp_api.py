"""The C++ drop-in layer (include/visionaray_hip): compiles standalone and against the reference's
own headers; on the GPU the C++ programs reproduce the reference's frames bit for bit."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AO_HIP = os.path.join(ROOT, "build", "examples", "ao_hip")
AO_MULTI = os.path.join(ROOT, "build", "examples", "ao_multi_gpu")
DROPIN = os.path.join(ROOT, "oracle", "_ref", "dropin_ref_api")


@pytest.mark.parametrize("example", ["ao_hip.cpp", "ao_multi_gpu.cpp"])
def test_cpp_headers_compile_standalone(tmp_path, example):
    src = os.path.join(ROOT, "examples", example)
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), src],
                   check=True)


def test_builtin_kernel_required(tmp_path):
    """hip_sched::frame rejects an arbitrary lambda at compile time (a callable cannot cross the C ABI)."""
    src = tmp_path / "bad.cpp"
    src.write_text('#include <visionaray_hip/standalone.h>\nusing namespace visionaray;\n'
                   'int main(){ hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt; camera c; hip_sched<ray> s;\n'
                   '  s.frame([](int){ return 0; }, make_sched_params(c, rt)); }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "built-in kernels" in r.stderr


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="reference headers absent")
def test_cpp_drop_in_compiles_against_reference_headers():
    src = os.path.join(ROOT, "tests", "cpp", "drop_in_reference_api.cpp")
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-w", "-I/root/reference/include",
                    "-I", os.path.join(ROOT, "include"), src], check=True)


def _run(binary, *args):
    r = subprocess.run([binary, *map(str, args)], check=True, capture_output=True, text=True, timeout=300)
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("case,grid", [("hf200_320x180", 200), ("hf1M", 708)])
def test_cpp_example_matches_reference(golden, case, grid):
    g = golden[case]
    out = _run(AO_HIP, grid, g["W"], g["H"], 2)
    for k in ("primid_hash", "t_hash", "occ_hash", "color_hash"):
        assert out[k] == g[k], k
    assert out["rays"] == g["W"] * g["H"] + g["ao_rays"]


@pytest.mark.gpu
@pytest.mark.parametrize("case,grid,shards", [("hf200_320x180", 200, 0), ("hf200_320x180", 200, 3), ("hf1M", 708, 8)])
def test_cpp_multi_gpu_example_matches_reference(golden, case, grid, shards):
    """examples/ao_multi_gpu.cpp: a render group over every visible GPU (one on the test box, so
    `shards` > 1 makes the one GPU render several shards and run the RCCL exchange with itself)."""
    g = golden[case]
    out = _run(AO_MULTI, grid, g["W"], g["H"], 2, shards)
    assert out["matches_one_gpu"]
    for k in ("primid_hash", "t_hash", "occ_hash", "color_hash"):
        assert out[k] == g[k], k


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN), reason="drop-in binary is built in the build container only")
def test_reference_api_program_on_hip_backend(golden):
    g = golden["hf200_320x180"]
    out = _run(DROPIN, 200, g["W"], g["H"])
    for k in ("primid_hash", "t_hash", "occ_hash", "color_hash"):
        assert out[k] == g[k], k
    assert out["batch_ok"], "hip_sched::frames: a frame of the batch differs from its own frame()"
    # make_sched_params(pixel_sampler::jittered_blend_type / ssaa_type<4>, cam, rt): the reference harness's frames
    assert out["sampler_jittered_blend_color_hash"] == golden["sampler_jittered_blend_hf200_ao"]["color_hash"]
    assert out["sampler_ssaa4_color_hash"] == golden["sampler_ssaa4_hf200_ao"]["color_hash"]
    # make_sched_params(pixel_sampler::uniform_type, cam.get_view_matrix(), cam.get_proj_matrix(), rt)
    assert out["matrix_color_hash"] == golden["matrix_uniform_hf200_ao"]["color_hash"]
    # make_hip_ao_kernel(bvh, bg, 16) into a hip_buffer_rt (which has an occlusion byte): renders
    assert out["ao16_color_hash"] != "0000000000000000"
    assert out["matrix_t_hash"] == golden["matrix_uniform_hf200_ao"]["t_hash"]


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN), reason="drop-in binary is built in the build container only")
def test_reference_api_program_with_mask_intersector(golden, tmp_path):
    """hip_hit_mask + with_intersector on the reference's own triangles and camera reproduce the
    reference's mask-intersector frame (harness `mask` mode) bit for bit."""
    import numpy as np
    g = golden["mask_hf200_320x180"]
    mask = np.load(os.path.join(ROOT, "tests", "golden", "mask_hf200_320x180.npz"))["mask"]
    mpath = tmp_path / "mask.bin"
    mask.tofile(mpath)
    out = _run(DROPIN, 200, g["W"], g["H"], mpath, mask.shape[0])
    for k in ("primid_hash", "t_hash", "occ_hash", "color_hash"):
        assert out["mask_" + k] == g[k], k


DROPIN_SHADE = os.path.join(ROOT, "oracle", "_ref", "dropin_simple_kernel")


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="reference headers absent")
def test_cpp_shading_drop_in_compiles_against_reference_headers():
    src = os.path.join(ROOT, "tests", "cpp", "drop_in_simple_kernel.cpp")
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-w", "-I/root/reference/include",
                    "-I", os.path.join(ROOT, "include"), src], check=True)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN_SHADE), reason="drop-in binary is built in the build container only")
@pytest.mark.parametrize("binding", ["face", "vertex"])
def test_reference_shading_objects_on_hip_backend(golden, tmp_path, binding):
    """The reference's plastic<float> / point_light<float> objects through hip_shading +
    make_hip_simple_kernel reproduce the reference's simple::kernel frame (radiance within 1e-5)."""
    import numpy as np
    g = golden["shade_hf64_" + binding]
    out_bin = tmp_path / "color.bin"
    _run(DROPIN_SHADE, 64, g["W"], g["H"], binding, out_bin)
    got = np.fromfile(out_bin, np.float32).reshape(-1, 4)
    ref = np.load(os.path.join(ROOT, "tests", "golden", "shade_hf64_%s.npz" % binding))["color"]
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=0.0)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN_SHADE), reason="drop-in binary is built in the build container only")
def test_reference_whitted_objects_on_hip_backend(golden, tmp_path):
    """make_hip_whitted_kernel with the reference's own material / light objects reproduces the
    reference's whitted::kernel frame (radiance within 1e-5)."""
    import numpy as np
    g = golden["whitted_hf64_vertex"]
    out_bin = tmp_path / "color.bin"
    _run(DROPIN_SHADE, 64, g["W"], g["H"], "vertex", out_bin, "whitted", g["bounces"], g["eps"])
    got = np.fromfile(out_bin, np.float32).reshape(-1, 4)
    ref = np.load(os.path.join(ROOT, "tests", "golden", "whitted_hf64_vertex.npz"))["color"]
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=0.0)
