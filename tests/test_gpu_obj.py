"""GPU: a scene read from a Wavefront OBJ file rendered end to end.

OBJ text -> vrh_obj_load -> host SAH BVH -> hip_index_bvh (+ the model's geometric normals and, for
the per-vertex binding, its shading normals) -> simple::kernel with the model's MTL materials.
Checked against the oracle on the same file: oracle/obj_oracle.py's restatement of load_obj, the C
oracle's BVH build and its simple::kernel.  Bar as in test_gpu_shading.py: hits bit-exact, radiance
within 1e-5 relative (device powf).
"""
import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import scenes
from oracle import obj_oracle as oo

pytestmark = pytest.mark.gpu
RTOL = 1e-5
EYE, CENTER, UP = (0.3, 1.1, 1.6), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0)


@pytest.fixture(scope="module")
def terrain(tmp_path_factory):
    d = tmp_path_factory.mktemp("obj")
    obj, mtl = scenes.terrain_obj(160)
    (d / "terrain.obj").write_text(obj)
    (d / "terrain.mtl").write_text(mtl)
    return str(d / "terrain.obj")


def _cameras(O, W, H):
    fovy = np.float32(45.0) * np.float32(va.DEGREES_TO_RADIANS)
    aspect = np.float32(W) / np.float32(H)
    cam = va.camera()
    cam.perspective(float(fovy), float(aspect), 0.001, 1000.0)
    cam.look_at(EYE, CENTER, UP)
    u, v, w = O.camera_basis(EYE, CENTER, UP, float(fovy), float(aspect))
    return cam, (np.array(EYE, np.float32), u, v, w, W, H)


@pytest.mark.parametrize("binding", ["face", "vertex"])
def test_obj_scene_simple_kernel(ctx, oracle_mod, terrain, binding):
    O = oracle_mod
    W, H = 256, 160
    m = va.load_obj(terrain)
    ref = oo.load_obj(terrain)
    assert m.primitives.tobytes() == ref["primitives"].tobytes()
    assert m.has_vertex_normals() and m.num_degenerate > 0 and len(m.materials) == 3

    # product: libvrh all the way
    bvh = va.build_index_bvh(m.primitives)
    dev = va.hip_index_bvh(ctx, bvh, m.geometric_normals)
    dev.set_vertex_normals(m.shading_normals)
    _, lt, amb, bg = O.shade_spec()
    sh = va.shading(ctx, m.materials, lt.view(va.POINT_LIGHT_DTYPE))
    vb = va.normals_per_vertex_binding if binding == "vertex" else va.normals_per_face_binding
    cam, ocam = _cameras(O, W, H)
    rt = va.hip_buffer_rt(ctx, W, H)
    va.hip_sched(ctx).frame(va.simple_kernel(dev, sh, binding=vb, bg=bg, ambient=amb),
                            va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt))
    out = rt.download()

    # oracle: restated loader + C oracle BVH / shading on the same file
    prims = ref["primitives"].view(O.TRI_DTYPE)
    nodes, idx, depth = O.build_bvh(prims, O.VO_TRI)
    fn = O.face_normals(prims)
    assert fn.tobytes() == m.geometric_normals.tobytes()          # normalize(cross(e1, e2)) both ways
    osc = O.Scene("terrain", O.VO_TRI, prims, nodes, idx, fn, depth, ref["shading_normals"])
    oref = O.render(osc, ocam, mode=O.VO_MODE_SIMPLE, materials=ref["materials"].view(O.PLASTIC_DTYPE),
                    lights=lt, ambient=amb, bg=bg,
                    binding=O.VO_NORMALS_PER_VERTEX if binding == "vertex" else O.VO_NORMALS_PER_FACE)

    hit = oref["prim_id"] != 0xFFFFFFFF
    assert hit.mean() > 0.5
    assert np.array_equal(out["prim_id"], oref["prim_id"])
    assert np.array_equal(out["t"].view(np.uint32), oref["t"].view(np.uint32))
    assert np.array_equal(out["color"][~hit].view(np.uint32), oref["color"][~hit].view(np.uint32))
    np.testing.assert_allclose(out["color"], oref["color"], rtol=RTOL, atol=0.0)
    # every material of the file shows up
    geom = m.primitives["geom_id"][out["prim_id"][hit]]
    assert set(np.unique(geom).tolist()) == {0, 1, 2}


def test_cpp_viewer_path_on_obj(ctx, oracle_mod, terrain, tmp_path):
    """tests/cpp/drop_in_obj_model.cpp (standalone model, compiled here): load_obj -> gpu_build ->
    simple::kernel with the file's materials; same frame as the Python path on the same GPU tree."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "visionaray_amd", "_lib")
    exe = tmp_path / "objview"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "cpp", "drop_in_obj_model.cpp"), "-o", str(exe), "-L", lib, "-lvrh",
                    "-Wl,-rpath," + lib], check=True)
    out_file = tmp_path / "frame.bin"
    subprocess.run([str(exe), terrain, str(out_file)], check=True, capture_output=True, timeout=300)
    W, H = 256, 160
    raw = np.fromfile(out_file, np.uint32)
    color = raw[:4 * W * H].view(np.float32).reshape(-1, 4)
    prim = raw[4 * W * H:]

    m = va.load_obj(terrain)
    dev = va.hip_index_bvh.gpu_build(ctx, m.primitives, m.geometric_normals)
    dev.set_vertex_normals(m.shading_normals)
    lt = va.point_light((0.5, 2.0, 1.5))
    sh = va.shading(ctx, m.materials, lt)
    cam, _ = _cameras(oracle_mod, W, H)
    rt = va.hip_buffer_rt(ctx, W, H)
    va.hip_sched(ctx).frame(va.simple_kernel(dev, sh, binding=va.normals_per_vertex_binding, bg=(0.1, 0.2, 0.3, 1.0),
                                             ambient=(0.4, 0.4, 0.4, 0.5)),
                            va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt))
    out = rt.download()
    assert (prim != 0xFFFFFFFF).mean() > 0.5
    assert np.array_equal(prim, out["prim_id"])
    assert np.array_equal(color.view(np.uint32), out["color"].view(np.uint32))
