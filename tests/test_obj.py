"""Wavefront OBJ input: libvrh's vrh_obj_load against the restatement in
oracle/obj_oracle.py and against the reference loader's documented behaviour.

The reference loader (src/common/obj_loader.cpp) needs Boost.Spirit, which this image lacks, so it
cannot be run here: parity is unpinned against the reference binary and rests on (1) bit-exact
agreement of two independent restatements (hand-written C++ descent vs. PEG combinators composed
like obj_grammar.cpp) on hand-written fixtures and on seeded random OBJ text full of grammar corner
cases, and (2) hand-derived expectations of the reference's semantics, one test per rule.
Host-only code: no GPU needed.
"""
import os
import random
import subprocess

import numpy as np
import pytest

import visionaray_amd as va
from oracle import obj_oracle as oo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "obj")
FIXTURES = sorted(f for f in os.listdir(FIX) if f.endswith(".obj"))
ARRAYS = ("primitives", "geometric_normals", "shading_normals", "tex_coords", "materials", "bbox")
SCALARS = ("material_names", "textures", "num_degenerate", "num_unknown_materials", "num_missing_files")


def assert_same(m, ref):
    for k in ARRAYS:
        a, b = getattr(m, k), ref[k]
        assert a.shape == b.shape, (k, a.shape, b.shape)
        assert a.tobytes() == b.tobytes(), k
    for k in SCALARS:
        assert getattr(m, k) == ref[k], k


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_matches_restatement(name):
    path = os.path.join(FIX, name)
    assert_same(va.load_obj(path), oo.load_obj(path))


def test_cube_semantics():
    m = va.load_obj(os.path.join(FIX, "cube.obj"))
    # 6 quads -> 12 fan triangles, prim_id in face order, geom_id = material added by each usemtl
    assert m.primitives["prim_id"].tolist() == list(range(12))
    assert m.primitives["geom_id"].tolist() == [0] * 4 + [1] * 4 + [2] * 4
    # every `usemtl` of a known material appends one (red twice)
    assert m.material_names == ["red", "white", "red"]
    red, white = m.materials[0], m.materials[1]
    assert red["ca"].tolist() == pytest.approx([0.1, 0.0, 0.0]) and red["exp"] == 20.0
    assert red["cd"].tolist() == pytest.approx([0.8, 0.1, 0.1]) and red["cs"].tolist() == [0.5, 0.5, 0.5]
    assert (red["ka"], red["kd"], red["ks"]) == (1.0, 1.0, 1.0)
    # white: only Kd set -> make_default_material's Ka 0.2 / Ks 0.1 / Ns 32
    assert white["ca"].tolist() == pytest.approx([0.2] * 3) and white["cs"].tolist() == pytest.approx([0.1] * 3)
    assert white["exp"] == 32.0 and m.textures[1] == "textures/white.png"
    # first fan triangle of face 1 (1 4 3 2): v1 = v1, e1 = v4 - v1, e2 = v3 - v1
    t = m.primitives[0]
    assert t["v1"][:3].tolist() == [-1, -1, -1] and t["e1"][:3].tolist() == [0, 2, 0]
    assert t["e2"][:3].tolist() == [2, 2, 0]
    # all corners carry vn -> per-vertex normals; all corners of the first 4 faces carry vt
    assert m.has_vertex_normals()
    assert m.shading_normals[:6, :3].tolist() == [[0, 0, -1]] * 6
    assert np.allclose(np.abs(m.geometric_normals[:, :3]).sum(1), 1.0)
    assert m.bbox.tolist() == [[-1, -1, -1], [1, 1, 1]]
    # 8 triangles with vt (24 entries), then the reference's padding loop adds nothing (i = 24 >= 12)
    assert len(m.tex_coords) == 24


def test_quirks_semantics():
    m = va.load_obj(os.path.join(FIX, "quirks.obj"))
    # "v1 0 0" is a vertex; a 5-number `v` line is skipped; "f 1 2" and a face with a trailing
    # comment are skipped; the fan (2 3 4 1 2) closes with a degenerate triangle
    assert len(m.primitives) == 8 and m.num_degenerate == 1
    assert m.primitives["v1"][0, :3].tolist() == [1, 0, 0]
    assert m.primitives["v1"][5, :3].tolist() == [0, 1, 0]
    # faces before the first usemtl: geom_id 0; `usemtl shiny` (without the trailing blanks of the
    # newmtl name) is unknown and keeps geom_id; `usemtl dup` -> 1
    assert m.primitives["geom_id"].tolist() == [0] * 7 + [1]
    assert m.material_names == ["shiny   ", "dup"] and m.num_unknown_materials == 1
    shiny, dup = m.materials
    # "Kd 0.1 0.2 0.3 0.4" fails the rule after the attribute was written (Spirit writes in place)
    assert shiny["cd"].tolist() == pytest.approx([0.1, 0.2, 0.3])
    assert shiny["ca"].tolist() == [1, 1, 1] and shiny["exp"] == 64
    # a repeated newmtl keeps the first entry; "Ns 8 9" writes 8 before failing
    assert dup["cd"].tolist() == [0.5] * 3 and dup["ca"].tolist() == pytest.approx([0.3] * 3) and dup["exp"] == 8
    # vt on all corners of one triangle only -> 3 entries + the padding loop (i = 3 .. 7, 3 each)
    assert len(m.tex_coords) == 3 + 5 * 3
    assert m.tex_coords[:3].tolist() == [[0.5, 0.25], [0.75, 1.0], [0.5, 0.25]]
    # vn on all corners of one triangle only: 3 shading normals, not per-vertex
    assert len(m.shading_normals) == 3 and not m.has_vertex_normals()
    assert m.shading_normals[1, :3].view(np.uint32).tolist() == [0x3F800000, 0, 0x80000000]
    assert m.bbox.tolist() == [[0, 0, 0], [1.5, 2.5, 3.5]]


def test_crlf_negative_indices_and_last_line():
    m = va.load_obj(os.path.join(FIX, "crlf_negative.obj"))
    # f -4 -3 -2 | f 1 2 2 (degenerate) | f -3 -1 -2 | usemtl missing | f 1 2 4 | f 1 3 4 (no eol: skipped)
    assert m.primitives["prim_id"].tolist() == [0, 1, 2] and m.num_degenerate == 1
    assert m.primitives["e1"][:, :3].tolist() == [[1, 0, 0], [0, 1, 0], [1, 0, 0]]
    assert m.primitives["e2"][:, :3].tolist() == [[0, 1, 0], [-1, 1, 0], [1, 1, 0]]
    assert m.num_unknown_materials == 1
    # no material ever added: one default material (make_default_material) for geom_id 0
    assert len(m.materials) == 1 and m.materials[0]["exp"] == 32.0 and m.material_names == [""]


def test_no_mtllib_default_material():
    m = va.load_obj(os.path.join(FIX, "nomtl.obj"))
    assert m.primitives["geom_id"].tolist() == [0, 0]
    d = m.materials[0]
    assert d["ca"].tolist() == pytest.approx([0.2] * 3) and d["cd"].tolist() == pytest.approx([0.8] * 3)
    assert d["cs"].tolist() == pytest.approx([0.1] * 3) and (d["ka"], d["kd"], d["ks"], d["exp"]) == (1, 1, 1, 32)
    # e2 x e1 order flips the second triangle's geometric normal
    assert m.geometric_normals[:, :3].tolist() == [[0, 0, 1], [0, 0, -1]]


def test_empty_model(tmp_path):
    p = tmp_path / "empty.obj"
    p.write_text("# nothing\nv 0 0 0\n")
    m = va.load_obj(p)
    assert len(m.primitives) == 0 and len(m.materials) == 1 and len(m.tex_coords) == 0
    fmax = np.finfo(np.float32).max
    assert m.bbox.tolist() == [[fmax] * 3, [-fmax] * 3]          # aabb::invalidate
    assert_same(m, oo.load_obj(str(p)))


def test_missing_mtllib_is_a_warning(tmp_path):
    p = tmp_path / "m.obj"
    p.write_text("mtllib nothere.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl a\nf 1 2 3\n")
    m = va.load_obj(p)
    assert m.num_missing_files == 1 and m.num_unknown_materials == 1 and len(m.primitives) == 1


@pytest.mark.parametrize("text", ["v 0 0 0\nv 1 0 0\nf 1 2 3\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n",
                                  "v 0 0 0\nv 1 0 0\nv 0 1 0\nf -4 1 2\n",
                                  "v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf 1//1 2//1 3//2\n"])
def test_out_of_range_indices_fail_loudly(tmp_path, text):
    """The reference indexes out of bounds there (undefined); the loader reports VRH_ERR_INVALID."""
    p = tmp_path / "bad.obj"
    p.write_text(text)
    with pytest.raises(va.VrhError) as e:
        va.load_obj(p)
    assert e.value.code == 1 and "out of range" in str(e.value)
    with pytest.raises(oo.ObjError):
        oo.load_obj(str(p))


def test_unreadable_file_fails():
    with pytest.raises(va.VrhError) as e:
        va.load_obj("/nonexistent/file.obj")
    assert e.value.code == 1


# ---- seeded random OBJ text: both restatements must agree bit for bit -------------------------

SAFE_ODD = ["1.", ".5", "-.25", "+2", "1e2", "0.0", "-0", "3.25E-1", "-1.5e+1"]
BAD = ["1e", "x", "7.5.5", "--1", "."]


def _num(rng, safe=True):
    r = rng.random()
    if r < 0.5:
        return f"{rng.uniform(-10, 10):.{rng.randint(0, 5)}f}"
    if r < 0.7:
        return str(rng.randint(-9, 9))
    if r < 0.8:
        return f"{rng.uniform(-1, 1):.3e}"
    if r < 0.99 or safe:
        return rng.choice(SAFE_ODD)
    return rng.choice(BAD)


def _idx(rng, n, bad_rate):
    if rng.random() < bad_rate:
        return rng.choice(["0", str(n + 1), str(-n - 1)])
    k = rng.randint(1, n)
    return str(k if rng.random() < 0.7 else k - n - 1)


def random_obj(rng, lines=400, bad_rate=0.0):
    """OBJ text mixing valid lines (counted, so face indices stay in range) with lines the grammar
    rejects (wrong arity, malformed numbers, comments, unknown keywords)."""
    nv = nt = nn = 0
    out = ["mtllib rand.mtl"]
    nl = rng.choice(["\n", "\r\n"])
    for _ in range(lines):
        r = rng.random()
        blank = rng.choice(["", " ", "\t", "  "])
        valid = rng.random() < 0.9
        if r < 0.35:
            if valid:
                out.append(blank + rng.choice(["v ", "v", "v\t"]) + " ".join(_num(rng) for _ in range(rng.choice([3, 3, 4, 6]))))
                nv += 1
            else:
                k = rng.choice([2, 5, 7, 3])
                out.append(blank + "v " + " ".join(_num(rng, safe=False) if k == 3 else _num(rng) for _ in range(k))
                           + (" x" if k == 3 else ""))
        elif r < 0.42:
            if valid:
                out.append(blank + "vt " + " ".join(_num(rng) for _ in range(rng.choice([2, 2, 3]))))
                nt += 1
            else:
                out.append(blank + "vt " + " ".join(_num(rng) for _ in range(rng.choice([1, 4]))))
        elif r < 0.5:
            if valid:
                out.append(blank + "vn " + " ".join(_num(rng) for _ in range(3)))
                nn += 1
            else:
                out.append(blank + "vn " + " ".join(_num(rng) for _ in range(rng.choice([2, 4]))))
        elif r < 0.85 and nv >= 1:
            corners = []
            form = rng.choice(["v", "v/t", "v//n", "v/t/n", "mix"])
            for _ in range(rng.choice([3, 3, 4, 5, 6, 2])):
                f = form if form != "mix" else rng.choice(["v", "v/t", "v//n", "v/t/n"])
                vi = _idx(rng, nv, bad_rate)
                ti = _idx(rng, nt, bad_rate) if nt else None
                ni = _idx(rng, nn, bad_rate) if nn else None
                if f == "v/t" and ti:
                    corners.append(f"{vi}/{ti}")
                elif f == "v//n" and ni:
                    corners.append(f"{vi}//{ni}")
                elif f == "v/t/n" and ti and ni:
                    corners.append(f"{vi}/{ti}/{ni}")
                else:
                    corners.append(vi)
            tail = rng.choice(["", "", "", " ", " # c", "\t"])
            out.append(blank + "f " + " ".join(corners) + tail)
        elif r < 0.9:
            out.append(blank + "usemtl " + rng.choice(["m0", "m1", "m2", "nope", "m1 "]))
        elif r < 0.95:
            out.append(rng.choice(["# comment", "", "g grp", "s 1", "o obj", "vp 1 2", "foo bar"]))
        else:
            # repeats of one vertex make degenerate triangles likely
            out.append("v 0 0 0")
            nv += 1
    return nl.join(out) + (nl if rng.random() < 0.8 else "")


def random_mtl(rng):
    out = []
    for name in ("m0", "m1", "m2", "m1"):
        out.append(f"newmtl {name}")
        for key in rng.sample(["Ka", "Kd", "Ks", "Ke", "Ns", "map_Kd", "illum", "Ni"], rng.randint(0, 6)):
            if key in ("Ka", "Kd", "Ks", "Ke"):
                out.append(f"{key} " + " ".join(_num(rng) for _ in range(rng.choice([3, 3, 3, 2, 4]))))
            elif key == "Ns":
                out.append("Ns " + " ".join(_num(rng) for _ in range(rng.choice([1, 1, 2]))))
            elif key == "map_Kd":
                out.append("map_Kd tex/" + name + ".png")
            else:
                out.append(f"{key} 2")
    return "\n".join(out) + "\n"


@pytest.mark.parametrize("seed", range(16))
def test_random_obj_text_matches_restatement(tmp_path, seed):
    rng = random.Random(seed)
    (tmp_path / "rand.mtl").write_text(random_mtl(rng))
    p = tmp_path / "rand.obj"
    p.write_bytes(random_obj(rng, lines=600).encode())
    ref = oo.load_obj(str(p))
    m = va.load_obj(p)
    assert_same(m, ref)
    assert len(m.primitives) > 50 and len(m.materials) > 1


@pytest.mark.parametrize("seed", range(4))
def test_random_obj_bad_indices_fail_in_both(tmp_path, seed):
    rng = random.Random(1000 + seed)
    (tmp_path / "rand.mtl").write_text(random_mtl(rng))
    p = tmp_path / "rand.obj"
    p.write_bytes(random_obj(rng, bad_rate=0.02).encode())
    with pytest.raises(oo.ObjError):
        oo.load_obj(str(p))
    with pytest.raises(va.VrhError):
        va.load_obj(p)


# ---- C++ drop-in: visionaray_hip/obj_loader.h filling a model -----------------------------------

def _dump(binary, path):
    import json
    r = subprocess.run([binary, str(path)], check=True, capture_output=True, text=True, timeout=60)
    return json.loads(r.stdout)


def _check_dump(d, m):
    u = lambda a: a.view(np.uint32)
    ids = np.array(d["ids"], np.uint32).reshape(-1, 2)
    assert ids[:, 0].tolist() == m.primitives["geom_id"].tolist()
    assert ids[:, 1].tolist() == m.primitives["prim_id"].tolist()
    for k in ("v1", "e1", "e2"):
        assert d[k] == u(np.ascontiguousarray(m.primitives[k][:, :3])).ravel().tolist(), k
    assert d["shading_normals"] == u(np.ascontiguousarray(m.shading_normals[:, :3])).ravel().tolist()
    assert d["geometric_normals"] == u(np.ascontiguousarray(m.geometric_normals[:, :3])).ravel().tolist()
    assert d["tex_coords"] == u(m.tex_coords).ravel().tolist()
    assert d["materials"] == m.materials.view(np.uint32).ravel().tolist()
    assert d["bbox"] == u(m.bbox).ravel().tolist()


def _build(tmp_path, name, extra):
    exe = tmp_path / name
    lib = os.path.join(ROOT, "visionaray_amd", "_lib")
    subprocess.run(["g++", "-std=c++17", "-O1", *extra, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "drop_in_obj_model.cpp"), "-o", str(exe), "-L", lib, "-lvrh",
                    "-Wl,-rpath," + lib], check=True)
    return exe


@pytest.mark.parametrize("name", FIXTURES)
def test_cpp_obj_loader_standalone_model(tmp_path, name):
    exe = _build(tmp_path, "sa", ["-Wall", "-Werror"])
    _check_dump(_dump(exe, os.path.join(FIX, name)), va.load_obj(os.path.join(FIX, name)))


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/common"), reason="reference sources absent")
def test_cpp_obj_loader_fills_reference_model(tmp_path):
    """The reference's own model class (src/common/model.h, plastic<float> materials) filled by the
    drop-in header: same arrays as the C ABI returns."""
    exe = _build(tmp_path, "rf", ["-w", "-DREFERENCE_MODEL", "-I/root/reference/src", "-I/root/reference/include"])
    for name in FIXTURES:
        _check_dump(_dump(exe, os.path.join(FIX, name)), va.load_obj(os.path.join(FIX, name)))
    assert _dump(exe, tmp_path / "missing.obj") == {"error": 1}
