"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes binding of the plain-C restatement in oracle/vrh_oracle.c (the parity checker) plus helpers
that drive the reference harness oracle/_ref/vsnray_ref.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module; the product path (visionaray_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libvrh_oracle.so")
REF_BIN = os.path.join(HERE, "_ref", "vsnray_ref")
REF_BENCH_BIN = os.path.join(HERE, "_ref", "vsnray_ref_bench")

TRI_DTYPE = np.dtype([("geom_id", "<u4"), ("prim_id", "<u4"), ("pad", "<u4", 2),
                      ("v1", "<f4", 4), ("e1", "<f4", 4), ("e2", "<f4", 4)])
SPHERE_DTYPE = np.dtype([("geom_id", "<u4"), ("prim_id", "<u4"), ("pad", "<u4", 2),
                         ("center", "<f4", 4), ("radius", "<f4"), ("pad2", "<f4", 3)])
NODE_DTYPE = np.dtype([("bmin", "<f4", 3), ("first", "<u4"), ("bmax", "<f4", 3), ("num_prims", "<u4")])
assert TRI_DTYPE.itemsize == 64 and SPHERE_DTYPE.itemsize == 48 and NODE_DTYPE.itemsize == 32

VO_TRI, VO_SPHERE = 0, 1
VO_MODE_PRIMARY, VO_MODE_AO, VO_MODE_SIMPLE, VO_MODE_MULTI_HIT, VO_MODE_WHITTED = 0, 1, 2, 3, 4
VO_NORMALS_PER_FACE, VO_NORMALS_PER_VERTEX = 0, 1
VO_SAMPLER_UNIFORM, VO_SAMPLER_JITTERED, VO_SAMPLER_JITTERED_BLEND, VO_SAMPLER_SSAA = 0, 1, 2, 3
SAMPLERS = {"uniform": (0, 0), "jittered": (1, 0), "jittered_blend": (2, 0), "ssaa2": (3, 2), "ssaa4": (3, 4),
            "ssaa8": (3, 8)}
# plastic<float> / point_light<float> parameter records (vrh_oracle.h vo_plastic / vo_point_light)
PLASTIC_DTYPE = np.dtype([("ca", "<f4", 3), ("ka", "<f4"), ("cd", "<f4", 3), ("kd", "<f4"), ("cs", "<f4", 3),
                          ("ks", "<f4"), ("exp", "<f4")])
POINT_LIGHT_DTYPE = np.dtype([("position", "<f4", 3), ("cl", "<f4", 3), ("kl", "<f4"), ("constant_att", "<f4"),
                              ("linear_att", "<f4"), ("quadratic_att", "<f4")])


class _Bvh(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("num_nodes", C.c_size_t),
                ("indices", C.c_void_p), ("num_indices", C.c_size_t), ("max_depth", C.c_uint)]


class _Counters(C.Structure):
    _fields_ = [("box_tests", C.c_uint64), ("prim_tests", C.c_uint64)]


class _HitMask(C.Structure):
    _fields_ = [("tc", C.c_void_p), ("mask", C.c_void_p), ("w", C.c_int), ("h", C.c_int)]


class _Scene(C.Structure):
    pass


_Scene._fields_ = [("nodes", C.c_void_p), ("indices", C.c_void_p), ("prims", C.c_void_p),
                   ("kind", C.c_int), ("normals", C.c_void_p), ("vertex_normals", C.c_void_p),
                   ("hit_mask", C.c_void_p), ("next", C.POINTER(_Scene))]


class _Camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("cam_u", C.c_float * 3), ("cam_v", C.c_float * 3),
                ("cam_w", C.c_float * 3), ("width", C.c_int), ("height", C.c_int),
                ("scissor", C.c_uint * 4), ("inv_view", C.c_void_p), ("inv_proj", C.c_void_p)]


class _Kernel(C.Structure):
    _fields_ = [("mode", C.c_int), ("samples", C.c_int), ("radius", C.c_float), ("eps", C.c_float),
                ("bg", C.c_float * 4), ("materials", C.c_void_p), ("num_materials", C.c_int),
                ("lights", C.c_void_p), ("num_lights", C.c_int), ("ambient", C.c_float * 4),
                ("normal_binding", C.c_int), ("max_hits", C.c_int), ("num_bounces", C.c_int),
                ("frame_num", C.c_uint32)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, sz = C.c_void_p, C.c_size_t
        L.vo_gen_cornell.argtypes = [vp]; L.vo_gen_cornell.restype = sz
        L.vo_gen_heightfield.argtypes = [C.c_int, vp]; L.vo_gen_heightfield.restype = None
        L.vo_gen_spheres.argtypes = [C.c_int, vp]; L.vo_gen_spheres.restype = None
        L.vo_face_normals.argtypes = [vp, sz, vp]; L.vo_face_normals.restype = None
        L.vo_build.argtypes = [vp, sz, C.c_int, C.POINTER(_Bvh)]; L.vo_build.restype = C.c_int
        L.vo_bvh_free.argtypes = [C.POINTER(_Bvh)]; L.vo_bvh_free.restype = None
        L.vo_camera_basis.argtypes = [C.POINTER(C.c_float)] * 3 + [C.c_float, C.c_float] + [C.POINTER(C.c_float)] * 3
        L.vo_camera_basis.restype = None
        L.vo_render_rows.argtypes = [C.POINTER(_Scene), C.POINTER(_Camera), C.POINTER(_Kernel), C.c_int, C.c_int,
                                     vp, vp, vp, vp, vp, C.c_int, C.POINTER(_Counters)]
        L.vo_render_rows.restype = C.c_uint64
        L.vo_render_pixels.argtypes = [C.POINTER(_Scene), C.POINTER(_Camera), C.POINTER(_Kernel), vp, sz,
                                       vp, vp, vp, vp, C.c_int]
        L.vo_render_pixels.restype = C.c_uint64
        L.vo_render_sampled.argtypes = [C.POINTER(_Scene), C.POINTER(_Camera), C.POINTER(_Kernel), C.c_int, C.c_int,
                                        vp, vp, vp, C.c_int]
        L.vo_render_sampled.restype = C.c_int
        L.vo_inverse4.argtypes = [vp, vp]; L.vo_inverse4.restype = None
        L.vo_fnv1a.argtypes = [vp, sz, C.c_uint64]; L.vo_fnv1a.restype = C.c_uint64
        L.vo_vertex_normals.argtypes = [vp, sz, vp]; L.vo_vertex_normals.restype = None
        L.vo_render_multi.argtypes = [C.POINTER(_Scene), C.POINTER(_Camera), C.POINTER(_Kernel), vp, vp, vp, C.c_int]
        L.vo_render_multi.restype = C.c_uint64
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ---- scenes ------------------------------------------------------------

SCENES = {
    # name: (kind, param, eye, W, H)
    "cornell12": (VO_TRI, 0, (0.0, 0.0, 3.4), 512, 512),
    "hf1M": (VO_TRI, 708, (0.0, 0.9, 1.4), 1920, 1080),
    "hf10M": (VO_TRI, 2236, (0.0, 0.9, 1.4), 1920, 1080),
    "sph1M": (VO_SPHERE, 1000000, (0.0, 0.0, 3.5), 1920, 1080),
}


def scene_spec(name):
    if name in SCENES:
        return SCENES[name]
    if name.startswith("hfstack"):
        return (VO_TRI, int(name[7:].split("x")[0]), (0.0, 0.9, 1.4), 1920, 1080)
    if name.startswith("hf"):
        return (VO_TRI, int(name[2:]), (0.0, 0.9, 1.4), 1920, 1080)
    if name.startswith("sph"):
        return (VO_SPHERE, int(name[3:]), (0.0, 0.0, 3.5), 1920, 1080)
    raise KeyError(name)


def gen_prims(name):
    kind, param, _, _, _ = scene_spec(name)
    L = lib()
    if name.startswith("hfstack"):
        # K copies of hf<G>, layer k shifted down by 0.03 * k (ref_harness.cpp make_hfstack)
        layers = int(name.split("x")[1])
        _, one = gen_prims("hf%d" % param)
        out = np.concatenate([one] * layers)
        for k in range(layers):
            blk = out[k * len(one):(k + 1) * len(one)]
            blk["v1"][:, 1] = blk["v1"][:, 1] - np.float32(0.03) * np.float32(k)
            blk["prim_id"] = np.arange(k * len(one), (k + 1) * len(one), dtype=np.uint32)
        return kind, out
    if kind == VO_TRI:
        if param == 0:
            a = np.zeros(12, TRI_DTYPE)
            L.vo_gen_cornell(_p(a))
        else:
            a = np.zeros(2 * param * param, TRI_DTYPE)
            L.vo_gen_heightfield(param, _p(a))
    else:
        a = np.zeros(param, SPHERE_DTYPE)
        L.vo_gen_spheres(param, _p(a))
    return kind, a


def face_normals(tris):
    out = np.zeros((len(tris), 4), np.float32)
    lib().vo_face_normals(_p(tris), len(tris), _p(out))
    return out


def build_bvh(prims, kind):
    b = _Bvh()
    rc = lib().vo_build(_p(prims), len(prims), kind, C.byref(b))
    if rc != 0:
        raise RuntimeError("vo_build failed")
    nodes = np.ctypeslib.as_array(C.cast(b.nodes, C.POINTER(C.c_uint32)), (b.num_nodes * 8,)).copy().view(NODE_DTYPE)
    idx = np.ctypeslib.as_array(C.cast(b.indices, C.POINTER(C.c_uint32)), (b.num_indices,)).copy()
    depth = b.max_depth
    lib().vo_bvh_free(C.byref(b))
    return nodes, idx, depth


def camera_basis(eye, center, up, fovy, aspect):
    f3 = C.c_float * 3
    u, v, w = f3(), f3(), f3()
    lib().vo_camera_basis(f3(*eye), f3(*center), f3(*up), C.c_float(fovy), C.c_float(aspect), u, v, w)
    return (np.array(u[:], np.float32), np.array(v[:], np.float32), np.array(w[:], np.float32))


def scene_camera(name, W=None, H=None):
    """camera::perspective(45 deg, W/H) + look_at(eye, 0, +y), basis as simple_sched computes it."""
    _, _, eye, W0, H0 = scene_spec(name)
    W = W or W0
    H = H or H0
    fovy = np.float32(45.0) * np.float32(1.74532925199432957692369076849e-02)
    aspect = np.float32(W) / np.float32(H)
    u, v, w = camera_basis(eye, (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), float(fovy), float(aspect))
    return np.array(eye, np.float32), u, v, w, W, H


@dataclass
class Scene:
    name: str
    kind: int
    prims: np.ndarray
    nodes: np.ndarray
    indices: np.ndarray
    normals: np.ndarray | None
    max_depth: int
    vertex_normals: np.ndarray | None = None


def make_scene(name):
    kind, prims = gen_prims(name)
    nodes, idx, depth = build_bvh(prims, kind)
    normals = face_normals(prims) if kind == VO_TRI else None
    return Scene(name, kind, prims, nodes, idx, normals, depth)


def _structs(scene, cam, mode, samples=8, radius=0.1, eps=1e-3, bg=(0.1, 0.2, 0.3, 1.0), materials=None,
             lights=None, ambient=(0.0, 0.0, 0.0, 0.0), binding=VO_NORMALS_PER_FACE, max_hits=0, num_bounces=0,
             hit_mask=None, frame_num=0, scissor=None):
    """scene: a Scene, or a list of Scenes = a BVH-ref list (normals of the first entry, indexed
    by prim_id over the whole list); scissor: (x0, y0, x1, y1) as cuda_sched reads it."""
    hm = None
    if hit_mask is not None:
        tc, mask = hit_mask
        tc = np.ascontiguousarray(tc, np.float32)
        mask = np.ascontiguousarray(mask, np.uint8)
        hm = _HitMask(_p(tc).value, _p(mask).value, mask.shape[1], mask.shape[0])
    members = list(scene) if isinstance(scene, (list, tuple)) else [scene]
    chain = []
    for m in reversed(members):
        nxt = C.pointer(chain[-1]) if chain else None
        chain.append(_Scene(_p(m.nodes).value, _p(m.indices).value, _p(m.prims).value, m.kind,
                            _p(m.normals).value if m.normals is not None else None,
                            _p(m.vertex_normals).value if m.vertex_normals is not None else None,
                            C.cast(C.pointer(hm), C.c_void_p).value if hm is not None else None, nxt))
    s = chain[-1]
    eye, u, v, w, W, H = cam
    c = _Camera((C.c_float * 3)(*eye), (C.c_float * 3)(*u), (C.c_float * 3)(*v), (C.c_float * 3)(*w), W, H,
                (C.c_uint * 4)(*(scissor or (0, 0, 0, 0))))
    k = _Kernel(mode, samples, radius, eps, (C.c_float * 4)(*bg),
                _p(materials).value if materials is not None else None, 0 if materials is None else len(materials),
                _p(lights).value if lights is not None else None, 0 if lights is None else len(lights),
                (C.c_float * 4)(*ambient), binding, max_hits, num_bounces, frame_num)
    _structs.keep = (materials, lights, hm, hit_mask and (tc, mask), chain, members)
    return s, c, k


def render(scene, cam, mode=VO_MODE_AO, rows=None, threads=0, **kw):
    """Full-image (or row range) oracle frame. Returns dict of arrays sized W*H."""
    _, _, _, _, W, H = cam
    y0, y1 = rows if rows else (0, H)
    out = {
        "color": np.zeros((H * W, 4), np.float32),
        "prim_id": np.full(H * W, 0xFFFFFFFF, np.uint32),
        "t": np.full(H * W, -1.0, np.float32),
        "occ": np.zeros(H * W, np.uint8),
        "list_index": np.full(H * W, 0xFFFFFFFF, np.uint32),
    }
    s, c, k = _structs(scene, cam, mode, **kw)
    cnt = _Counters()
    rays = lib().vo_render_rows(C.byref(s), C.byref(c), C.byref(k), y0, y1, _p(out["color"]), _p(out["prim_id"]),
                                _p(out["t"]), _p(out["occ"]), _p(out["list_index"]), threads, C.byref(cnt))
    out["rays"] = int(rays)
    out["box_tests"] = int(cnt.box_tests)
    out["prim_tests"] = int(cnt.prim_tests)
    return out


def inverse4(m):
    """matrix4.inl:209-244 inverse of a column-major 4x4 float matrix (16 floats)."""
    m = np.ascontiguousarray(m, np.float32).reshape(16)
    out = np.zeros(16, np.float32)
    lib().vo_inverse4(_p(m), _p(out))
    return out


def render_sampled(scene, cam, sampler, init=(0.25, 0.5, 0.75, 1.0), mode=VO_MODE_AO, threads=0, matrices=None,
                   **kw):
    """A frame through one of the reference's pixel samplers (SAMPLERS: uniform, jittered,
    jittered_blend, ssaa2/4/8) onto a target filled with `init`: colour + the last sample's prim id.
    matrices=(view, proj): the camera as matrices (column-major 4x4), inverted as the scheduler does."""
    _, _, _, _, W, H = cam
    kind, count = SAMPLERS[sampler]
    out = {"color": np.tile(np.asarray(init, np.float32), (H * W, 1)), "prim_id": np.full(H * W, 0xFFFFFFFF, np.uint32),
           "t": np.full(H * W, -1.0, np.float32)}
    s, c, k = _structs(scene, cam, mode, **kw)
    if matrices is not None:
        iv, ip = inverse4(matrices[0]), inverse4(matrices[1])
        c.inv_view, c.inv_proj = _p(iv).value, _p(ip).value
        render_sampled.keep = (iv, ip)
    rc = lib().vo_render_sampled(C.byref(s), C.byref(c), C.byref(k), kind, count, _p(out["color"]), _p(out["prim_id"]),
                                 _p(out["t"]), threads)
    if rc != 0:
        raise ValueError("render_sampled: bad sampler")
    return out


def render_pixels(scene, cam, pixels, mode=VO_MODE_AO, threads=0, **kw):
    pixels = np.ascontiguousarray(pixels, np.uint32)
    n = len(pixels)
    out = {
        "color": np.zeros((n, 4), np.float32),
        "prim_id": np.zeros(n, np.uint32),
        "t": np.zeros(n, np.float32),
        "occ": np.zeros(n, np.uint8),
    }
    s, c, k = _structs(scene, cam, mode, **kw)
    out["rays"] = int(lib().vo_render_pixels(C.byref(s), C.byref(c), C.byref(k), _p(pixels), n, _p(out["color"]),
                                             _p(out["prim_id"]), _p(out["t"]), _p(out["occ"]), threads))
    return out


# ---- simple::kernel shading spec (mirrors shade_spec() in oracle/ref_harness.cpp) -----------------

def shade_spec():
    """Three plastic materials (by geom_id), two point lights, ambient, background."""
    m = np.zeros(3, PLASTIC_DTYPE)
    m[0] = ((0.2, 0.2, 0.2), 1.0, (0.8, 0.3, 0.2), 1.0, (1.0, 1.0, 1.0), 0.4, 32.0)
    m[1] = ((0.1, 0.1, 0.1), 0.5, (0.2, 0.7, 0.3), 0.9, (0.9, 0.9, 0.9), 0.2, 8.0)
    m[2] = ((0.05, 0.05, 0.1), 1.0, (0.3, 0.3, 0.9), 0.7, (1.0, 0.8, 0.6), 0.6, 64.5)
    lt = np.zeros(2, POINT_LIGHT_DTYPE)
    lt[0] = ((0.5, 2.0, 1.5), (1.0, 1.0, 1.0), 1.0, 1.0, 0.0, 0.0)
    lt[1] = ((-1.5, 1.0, 0.5), (1.0, 0.8, 0.6), 0.7, 1.0, 0.1, 0.05)
    return m, lt, (0.4, 0.4, 0.4, 0.5), (0.1, 0.2, 0.3, 1.0)


def vertex_normals(face_nrm):
    """Deterministic per-vertex normals (3 per triangle, float4 rows) for the shading tests."""
    face_nrm = np.ascontiguousarray(face_nrm, np.float32)
    out = np.zeros((len(face_nrm) * 3, 4), np.float32)
    lib().vo_vertex_normals(_p(face_nrm), len(face_nrm), _p(out))
    return out


def make_shade_scene(name):
    """Triangle scene of the shading tests: geom_id = prim index % 3, face + vertex normals."""
    kind, prims = gen_prims(name)
    assert kind == VO_TRI
    prims["geom_id"] = np.arange(len(prims), dtype=np.uint32) % 3
    nodes, idx, depth = build_bvh(prims, kind)
    fn = face_normals(prims)
    return Scene(name, kind, prims, nodes, idx, fn, depth, vertex_normals(fn))


def render_simple(scene, cam, binding, rows=None, threads=0, hit_mask=None):
    m, lt, amb, bg = shade_spec()
    return render(scene, cam, mode=VO_MODE_SIMPLE, rows=rows, threads=threads, materials=m, lights=lt,
                  ambient=amb, bg=bg, binding=binding, hit_mask=hit_mask)


def whitted_spec():
    """shade_spec() plus a third light inside the scenes (so shadows fall inside the Cornell box)."""
    m, lt, amb, bg = shade_spec()
    l3 = np.zeros(3, POINT_LIGHT_DTYPE)
    l3[:2] = lt
    l3[2] = ((0.2, 0.6, 0.3), (0.9, 0.9, 1.0), 0.8, 1.0, 0.2, 0.1)
    return m, l3, amb, bg


def render_whitted(scene, cam, binding, num_bounces=4, eps=1e-3, rows=None, threads=0, hit_mask=None):
    m, lt, amb, bg = whitted_spec()
    return render(scene, cam, mode=VO_MODE_WHITTED, rows=rows, threads=threads, materials=m, lights=lt,
                  ambient=amb, bg=bg, binding=binding, num_bounces=num_bounces, eps=eps, hit_mask=hit_mask)


def render_multi(scene, cam, binding, max_hits=16, threads=0, hit_mask=None):
    """multi_hit<max_hits> frame: hit lists (W*H, max_hits) + the multi_hit example's colour."""
    m, lt, amb, bg = shade_spec()
    _, _, _, _, W, H = cam
    out = {"color": np.zeros((H * W, 4), np.float32),
           "mh_prim_id": np.full((H * W, max_hits), 0xFFFFFFFF, np.uint32),
           "mh_t": np.full((H * W, max_hits), -1.0, np.float32)}
    s, c, k = _structs(scene, cam, VO_MODE_MULTI_HIT, materials=m, lights=lt, ambient=amb, bg=bg, binding=binding,
                       max_hits=max_hits, hit_mask=hit_mask)
    lib().vo_render_multi(C.byref(s), C.byref(c), C.byref(k), _p(out["color"]), _p(out["mh_prim_id"]),
                          _p(out["mh_t"]), threads)
    return out


def ref_multi(name, outdir, binding, W=None, H=None):
    args = [REF_BIN, "multi", name, outdir, "vertex" if binding == VO_NORMALS_PER_VERTEX else "face"]
    args += [str(W), str(H)] if W else []
    r = subprocess.run(args, check=True, capture_output=True, text=True)
    return json.loads(r.stdout.strip().splitlines()[-1])


def ref_shade(name, outdir, binding, W=None, H=None):
    args = [REF_BIN, "shade", name, outdir, "vertex" if binding == VO_NORMALS_PER_VERTEX else "face"]
    args += [str(W), str(H)] if W else []
    r = subprocess.run(args, check=True, capture_output=True, text=True)
    return json.loads(r.stdout.strip().splitlines()[-1])


def fnv1a(arr):
    a = np.ascontiguousarray(arr)
    return "%016x" % lib().vo_fnv1a(_p(a), a.nbytes, 0)


# ---- reference harness (oracle/_ref) -----------------------------------------------------------

def ref_available():
    return os.path.exists(REF_BIN)


def ref_golden(name, outdir, W=None, H=None):
    args = [REF_BIN, "golden", name, outdir] + ([str(W), str(H)] if W else [])
    r = subprocess.run(args, check=True, capture_output=True, text=True)
    return json.loads(r.stdout.strip().splitlines()[-1])


def ref_bench(name, threads, frames, W=None, H=None, samples=None, timeout=600):
    args = [REF_BENCH_BIN, "bench", name, str(threads), str(frames)]
    if W:
        args += [str(W), str(H)]
        if samples is not None:
            args += [str(samples)]
    r = subprocess.run(args, check=True, capture_output=True, text=True, timeout=timeout)
    return json.loads(r.stdout.strip().splitlines()[-1])
