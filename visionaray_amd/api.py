"""Host-side mirror of Visionaray's scheduler / render-target / BVH interface for the HIP backend.

Names and argument meaning follow the reference so code (and tests) read like Visionaray's own:

    bvh   = build_index_bvh(prims)                          # build<index_bvh<P>>(prims, n)      build.inl:165-178
    ctx   = Context(0)                                      # one per GPU (HIP device + stream)
    dbvh  = hip_index_bvh(ctx, bvh, normals)                # cuda_index_bvh<P>(host_bvh)         bvh.h:344-350
    rt    = hip_buffer_rt(ctx, w, h)                        # gpu_buffer_rt<PF_RGBA32F, ...>     gpu_buffer_rt.h:19-51
    cam   = camera(); cam.perspective(...); cam.look_at(eye, center, up)          camera.inl:10-57
    sched = hip_sched(ctx)                                  # cuda_sched<R>                       cuda_sched.h:25-40
    sched.frame(ao_kernel(dbvh), make_sched_params(pixel_sampler.uniform_type, cam, rt))

Every device call goes through libvrh.so (include/vrh.h).  There is no CPU fallback in this module.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _capi as capi

# reference binary layouts
TRIANGLE_DTYPE = np.dtype([("geom_id", "<u4"), ("prim_id", "<u4"), ("pad", "<u4", 2),
                           ("v1", "<f4", 4), ("e1", "<f4", 4), ("e2", "<f4", 4)])
SPHERE_DTYPE = np.dtype([("geom_id", "<u4"), ("prim_id", "<u4"), ("pad", "<u4", 2),
                         ("center", "<f4", 4), ("radius", "<f4"), ("pad2", "<f4", 3)])
BVH_NODE_DTYPE = np.dtype([("bbox_min", "<f4", 3), ("first", "<u4"), ("bbox_max", "<f4", 3), ("num_prims", "<u4")])


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _kind_of(prims):
    if prims.dtype == TRIANGLE_DTYPE:
        return capi.VRH_PRIM_TRI64
    if prims.dtype == SPHERE_DTYPE:
        return capi.VRH_PRIM_SPHERE48
    raise TypeError(f"unsupported primitive dtype {prims.dtype}; use TRIANGLE_DTYPE or SPHERE_DTYPE")


# ---- primitives -------------------------------------------------------------------------------

def make_triangles(v1, e1, e2, prim_id=None, geom_id=None):
    """basic_triangle<3,float> array from (N,3) vertex / edge arrays."""
    v1, e1, e2 = (np.asarray(a, np.float32).reshape(-1, 3) for a in (v1, e1, e2))
    n = len(v1)
    t = np.zeros(n, TRIANGLE_DTYPE)
    t["v1"][:, :3], t["e1"][:, :3], t["e2"][:, :3] = v1, e1, e2
    t["prim_id"] = np.arange(n, dtype=np.uint32) if prim_id is None else prim_id
    t["geom_id"] = 0 if geom_id is None else geom_id
    return t


def make_spheres(center, radius, prim_id=None, geom_id=None):
    """basic_sphere<float> array."""
    center = np.asarray(center, np.float32).reshape(-1, 3)
    n = len(center)
    s = np.zeros(n, SPHERE_DTYPE)
    s["center"][:, :3] = center
    s["radius"] = radius
    s["prim_id"] = np.arange(n, dtype=np.uint32) if prim_id is None else prim_id
    s["geom_id"] = 0 if geom_id is None else geom_id
    return s


def face_normals(tris):
    """normalize(cross(e1, e2)) per triangle (get_normal normals_per_face_binding input)."""
    out = np.zeros((len(tris), 4), np.float32)
    capi.check("vrh_face_normals", _p(np.ascontiguousarray(tris)), len(tris), _p(out))
    return out


# ---- host BVH ---------------------------------------------------------------------------------

class index_bvh:
    """Host index BVH (index_bvh_t, bvh.h:317-403): prims + nodes + indices, reference layouts."""

    def __init__(self, prims, nodes, indices, max_depth):
        self.prims = prims
        self.nodes = nodes
        self.indices = indices
        self.max_depth = max_depth
        self.prim_kind = _kind_of(prims)

    def num_nodes(self):
        return len(self.nodes)

    def num_primitives(self):
        return len(self.prims)


def build_index_bvh(prims):
    """build<index_bvh<P>>(prims, n) -- binned SAH, tree-identical to the reference builder."""
    prims = np.ascontiguousarray(prims)
    n = len(prims)
    if n == 0:
        raise ValueError("build_index_bvh: no primitives")
    kind = _kind_of(prims)
    nodes = np.zeros(max(2 * n, 1), BVH_NODE_DTYPE)
    idx = np.zeros(n, np.uint32)
    nn, depth = C.c_uint32(0), C.c_uint32(0)
    capi.check("vrh_build_bvh", _p(prims), n, kind, _p(nodes), C.byref(nn), _p(idx), C.byref(depth))
    return index_bvh(prims, nodes[: nn.value].copy(), idx, depth.value)


# ---- camera -----------------------------------------------------------------------------------

class camera:
    """camera (camera.h:46-95): perspective() + look_at(); basis computed as simple_sched does."""

    def __init__(self):
        self.fovy = float(np.float32(45.0) * np.float32(math.pi / 180.0))
        self.aspect = 1.0
        self.z_near, self.z_far = 0.001, 1000.0
        self.eye = (0.0, 0.0, 1.0)
        self.center = (0.0, 0.0, 0.0)
        self.up = (0.0, 1.0, 0.0)

    def perspective(self, fovy, aspect, z_near, z_far):
        self.fovy, self.aspect, self.z_near, self.z_far = float(fovy), float(aspect), float(z_near), float(z_far)

    def look_at(self, eye, center, up=(0.0, 1.0, 0.0)):
        self.eye, self.center, self.up = tuple(eye), tuple(center), tuple(up)

    def basis(self, width, height):
        f3 = C.c_float * 3
        out = capi.vrh_camera()
        capi.check("vrh_make_camera", f3(*self.eye), f3(*self.center), f3(*self.up), C.c_float(self.fovy),
                   C.c_float(self.aspect), width, height, C.byref(out))
        return out


DEGREES_TO_RADIANS = float(np.float32(1.74532925199432957692369076849e-02))


# ---- device objects ---------------------------------------------------------------------------

class Context:
    """One HIP device + stream (vrh_ctx).  stream: optional raw hipStream_t (int) to launch on."""

    def __init__(self, device=0, stream=None):
        h = C.c_void_p()
        if stream is None:
            capi.check("vrh_ctx_create", int(device), C.byref(h))
        else:
            capi.check("vrh_ctx_create_on_stream", int(device), C.c_void_p(stream), C.byref(h))
        self.handle = h
        self.device = device
        self.async_frames = False

    def sync(self):
        capi.check("vrh_sync", self.handle)

    def set_option(self, option, value):
        """Launch tuning (vrh_ctx_set_option): block threads, stack cap, AO schedule, blocks/CU."""
        names = {"block_threads": capi.VRH_OPT_BLOCK_THREADS, "stack_cap": capi.VRH_OPT_STACK_CAP,
                 "ao_schedule": capi.VRH_OPT_AO_SCHEDULE, "blocks_per_cu": capi.VRH_OPT_BLOCKS_PER_CU,
                 "waves_per_simd": capi.VRH_OPT_WAVES_PER_SIMD, "exact_minmax": capi.VRH_OPT_EXACT_MINMAX,
                 "xcd_queues": capi.VRH_OPT_XCD_QUEUES, "refill_min": capi.VRH_OPT_REFILL_MIN,
                 "wide_anyhit": capi.VRH_OPT_WIDE_ANYHIT,
                 "descent_cap": capi.VRH_OPT_DESCENT_CAP, "pop_on_miss": capi.VRH_OPT_POP_ON_MISS,
                 "coop_fetch": capi.VRH_OPT_COOP_FETCH, "scalar_fetch": capi.VRH_OPT_SCALAR_FETCH,
                 "pair_layout": capi.VRH_OPT_PAIR_LAYOUT, "ao_gate": capi.VRH_OPT_AO_GATE, "ao_cut": capi.VRH_OPT_AO_CUT, "wave_times": capi.VRH_OPT_WAVE_TIMES,
                 "ao_share": capi.VRH_OPT_AO_SHARE, "cluster_tiles": capi.VRH_OPT_CLUSTER_TILES,
                 "quad_refill": capi.VRH_OPT_QUAD_REFILL, "group_units": capi.VRH_OPT_GROUP_UNITS,
                 "async_frames": capi.VRH_OPT_ASYNC_FRAMES}
        opt = names.get(option, option)
        capi.check("vrh_ctx_set_option", self.handle, opt, int(value))
        if opt == capi.VRH_OPT_ASYNC_FRAMES:
            # cuda_sched's issue model: hip_sched.frame returns without waiting (end_frame no-op)
            self.async_frames = bool(value)

    def last_frame_stats(self):
        s = capi.vrh_frame_stats()
        capi.check("vrh_last_frame_stats", self.handle, C.byref(s))
        return {k: (list(getattr(s, k)) if isinstance(getattr(s, k), C.Array) else getattr(s, k)) for k, _ in s._fields_}

    def wave_times(self):
        """(start, end) of every wave of the last launch in ms from the launch's first start, or
        None (VRH_OPT_WAVE_TIMES off).  Diagnostic of the launch's ramp-up and tail."""
        import numpy as np
        n, rate = C.c_uint64(), C.c_double()
        capi.check("vrh_get_wave_times", self.handle, None, 0, C.byref(n), C.byref(rate))
        if n.value == 0:
            return None
        buf = np.zeros(2 * n.value, np.uint64)
        capi.check("vrh_get_wave_times", self.handle, buf.ctypes.data_as(C.c_void_p), buf.size, C.byref(n), None)
        t = buf.reshape(-1, 2).astype(np.float64)
        return (t - t[:, 0].min()) / rate.value

    def tile_times(self):
        """(hand-out, primaries done, pixels written) of every tile of the last counting one-frame AO
        launch (VRH_OPT_WAVE_TIMES = 2) in ms from the first hand-out, or None."""
        import numpy as np
        n, rate = C.c_uint64(), C.c_double()
        capi.check("vrh_get_wave_times", self.handle, None, 0, C.byref(C.c_uint64()), C.byref(rate))
        capi.check("vrh_get_tile_times", self.handle, None, 0, C.byref(n))
        if n.value == 0:
            return None
        buf = np.zeros(3 * n.value, np.uint64)
        capi.check("vrh_get_tile_times", self.handle, buf.ctypes.data_as(C.c_void_p), buf.size, C.byref(n))
        t = buf.reshape(-1, 3).astype(np.float64)
        return (t - t[:, 0][t[:, 0] > 0].min()) / rate.value

    def stats_reset(self):
        capi.check("vrh_stats_reset", self.handle)

    def accum_stats(self):
        s = capi.vrh_accum_stats()
        capi.check("vrh_get_accum_stats", self.handle, C.byref(s))
        return {k: (list(getattr(s, k)) if isinstance(getattr(s, k), C.Array) else getattr(s, k)) for k, _ in s._fields_}

    def close(self):
        if self.handle:
            capi.lib().vrh_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count():
    n = C.c_int(0)
    rc = capi.lib().vrh_device_count(C.byref(n))
    return n.value if rc == 0 else 0


class hip_index_bvh:
    """Device-resident index BVH: the cuda_index_bvh<P>(host_bvh) copy-constructor analogue."""

    def __init__(self, ctx, host_bvh, normals=None):
        self.ctx = ctx
        h = C.c_void_p()
        nrm = None if normals is None else np.ascontiguousarray(normals, np.float32)
        if nrm is not None and nrm.shape != (len(host_bvh.prims), 4):
            raise ValueError("normals must be (num_prims, 4) float32")
        capi.check("vrh_scene_upload", ctx.handle, _p(host_bvh.nodes), len(host_bvh.nodes), _p(host_bvh.prims),
                   len(host_bvh.prims), host_bvh.prim_kind, _p(host_bvh.indices), len(host_bvh.indices),
                   _p(nrm), C.byref(h))
        self.handle = h
        self._refresh_info()

    def _refresh_info(self):
        info = capi.vrh_scene_info()
        capi.check("vrh_scene_get_info", self.handle, C.byref(info))
        self.info = {k: getattr(info, k) for k, _ in info._fields_}

    def set_vertex_normals(self, normals):
        """normals_per_vertex_binding array: (3 * num prim ids, 3 or 4) float32, row 3*prim_id + k."""
        n = np.asarray(normals, np.float32)
        if n.ndim != 2 or n.shape[1] not in (3, 4):
            raise ValueError("vertex normals must be (3 * prims, 3|4) float32")
        if n.shape[1] == 3:
            n = np.concatenate([n, np.zeros((len(n), 1), np.float32)], 1)
        n = np.ascontiguousarray(n)
        capi.check("vrh_scene_set_vertex_normals", self.handle, _p(n), len(n))
        self._refresh_info()

    @classmethod
    def gpu_build(cls, ctx, prims, normals=None, max_leaf=4):
        """vrh_scene_build: a linear BVH built on the GPU straight into a device scene (no host
        build or re-layout); the tree differs from build<index_bvh<P>> (see vrh.h)."""
        self = cls.__new__(cls)
        self.ctx = ctx
        prims = np.ascontiguousarray(prims)
        kind = capi.VRH_PRIM_TRI64 if prims.dtype == TRIANGLE_DTYPE else capi.VRH_PRIM_SPHERE48
        nrm = None if normals is None else np.ascontiguousarray(normals, np.float32)
        h = C.c_void_p()
        desc = capi.vrh_build_desc(capi.VRH_BUILD_LBVH, max_leaf)
        capi.check("vrh_scene_build", ctx.handle, _p(prims), len(prims), kind, _p(nrm), C.byref(desc), C.byref(h))
        self.handle = h
        self._refresh_info()
        return self

    @classmethod
    def scene_list(cls, ctx, members, normals=None):
        """vrh_scene_list_create: a list of BVHs rendered as one scene -- closest_hit / any_hit over
        [begin, end) of bvh_refs (traverse_linear.inl:76-141).  normals: (>= max prim_id + 1, 4)
        float32 indexed by prim_id (AO)."""
        self = cls.__new__(cls)
        self.ctx = ctx
        nrm = None if normals is None else np.ascontiguousarray(normals, np.float32)
        arr = (C.c_void_p * len(members))(*[m.handle.value for m in members])
        h = C.c_void_p()
        capi.check("vrh_scene_list_create", ctx.handle, arr, len(members), _p(nrm), 0 if nrm is None else len(nrm),
                   C.byref(h))
        self.handle = h
        self._refresh_info()
        return self

    def download_bvh(self):
        """(nodes, indices) of a GPU-built scene in the reference layout (BVH_NODE_DTYPE, uint32)."""
        n = C.c_uint32(0)
        capi.check("vrh_scene_download_bvh", self.ctx.handle, self.handle, None, C.byref(n), None)
        nodes = np.zeros(n.value, BVH_NODE_DTYPE)
        idx = np.zeros(self.info["num_indices"], np.uint32)
        capi.check("vrh_scene_download_bvh", self.ctx.handle, self.handle, _p(nodes), C.byref(n), _p(idx))
        return nodes, idx

    def close(self):
        if self.handle:
            capi.lib().vrh_scene_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class hip_buffer_rt:
    """gpu_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> plus the integer side buffers used for parity.

    wrap=(color_ptr, prim_id_ptr, t_ptr, occ_ptr) borrows caller device memory (e.g. torch tensors).
    """

    def __init__(self, ctx, width, height, flags=capi.VRH_RT_ALL, wrap=None):
        self.ctx = ctx
        self.handle = None
        self.flags = flags
        self._wrap = wrap
        self.resize(width, height)

    def resize(self, width, height):
        self.close()
        h = C.c_void_p()
        if self._wrap is None:
            capi.check("vrh_rt_alloc", self.ctx.handle, width, height, self.flags, C.byref(h))
        else:
            c, p, t, o = (C.c_void_p(x) if x else None for x in self._wrap)
            capi.check("vrh_rt_wrap", self.ctx.handle, width, height, c, p, t, o, C.byref(h))
        self.handle = h
        self.w, self.h = width, height

    def width(self):
        return self.w

    def height(self):
        return self.h

    def clear_color_buffer(self, color=(0.0, 0.0, 0.0, 0.0)):
        capi.check("vrh_rt_clear", self.ctx.handle, self.handle, (C.c_float * 4)(*color))

    def begin_frame(self):
        pass

    def end_frame(self):
        """Blocks until the frame is done (so hip_sched::frame is synchronous like tiled_sched) -- unless
        the context issues frames asynchronously (set_option("async_frames", 1)): then, like
        gpu_buffer_rt::end_frame (gpu_buffer_rt.inl:84-86), it returns at once and download() waits."""
        if not self.ctx.async_frames:
            self.ctx.sync()

    def device_buffers(self):
        bufs = [C.c_void_p() for _ in range(4)]
        capi.check("vrh_rt_get_buffers", self.handle, *[C.byref(b) for b in bufs])
        return tuple(b.value for b in bufs)

    def alloc_multi_hit(self, max_hits):
        """Hit-list side buffers of multi_hit<max_hits> (W * H * max_hits prim ids and t)."""
        capi.check("vrh_rt_alloc_multi_hit", self.ctx.handle, self.handle, max_hits)
        self.max_hits = max_hits

    def download_multi_hit(self):
        n = self.w * self.h * self.max_hits
        pid = np.empty(n, np.uint32)
        t = np.empty(n, np.float32)
        capi.check("vrh_rt_download_multi_hit", self.ctx.handle, self.handle, _p(pid), _p(t))
        return {"mh_prim_id": pid.reshape(-1, self.max_hits), "mh_t": t.reshape(-1, self.max_hits)}

    def download(self, color=True, prim_id=True, t=True, occ=True):
        n = self.w * self.h
        has = self.device_buffers()
        out = {}
        if color and has[0]:
            out["color"] = np.zeros((n, 4), np.float32)
        if prim_id and has[1]:
            out["prim_id"] = np.zeros(n, np.uint32)
        if t and has[2]:
            out["t"] = np.zeros(n, np.float32)
        if occ and has[3]:
            out["occ"] = np.zeros(n, np.uint8)
        capi.check("vrh_rt_download", self.ctx.handle, self.handle, _p(out.get("color")), _p(out.get("prim_id")),
                   _p(out.get("t")), _p(out.get("occ")))
        return out

    def upload(self, color=None, prim_id=None, t=None, occ=None):
        arrs = [None if a is None else np.ascontiguousarray(a) for a in (color, prim_id, t, occ)]
        n = self.w * self.h
        for a, per in zip(arrs, (16, 4, 4, 1)):
            if a is not None and a.nbytes != n * per:
                raise ValueError("upload: array size does not match the render target")
        capi.check("vrh_rt_upload", self.ctx.handle, self.handle, *[_p(a) for a in arrs])

    def color(self):
        return self.download(prim_id=False, t=False, occ=False)["color"]

    def close(self):
        if self.handle:
            capi.lib().vrh_rt_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- scheduler ----------------------------------------------------------------------------------

class pixel_sampler:
    """pixel_sampler::* (sched_common.h:34-50): the sampler of make_sched_params."""
    class uniform_type:
        kind, count = 0, 0

    class jittered_type:
        kind, count = 1, 0

    class jittered_blend_type:
        kind, count = 2, 0

    class ssaa2_type:
        kind, count = 3, 2

    class ssaa4_type:
        kind, count = 3, 4

    class ssaa8_type:
        kind, count = 3, 8

    @staticmethod
    def ssaa_type(n):
        """pixel_sampler::ssaa_type<N> for N in 1 (= uniform), 2, 4, 8."""
        types = {1: pixel_sampler.uniform_type, 2: pixel_sampler.ssaa2_type, 4: pixel_sampler.ssaa4_type,
                 8: pixel_sampler.ssaa8_type}
        if n not in types:
            raise ValueError("ssaa_type<N>: N is 1, 2, 4 or 8")
        return types[n]


def _matrix4(m):
    """matrix<4, 4, float> in its memory order (column-major, m[col * 4 + row]): a flat 16-vector is
    taken as that order, a 4x4 array as m[row, col]."""
    a = np.asarray(m, dtype=np.float32)
    if a.shape == (4, 4):
        return np.ascontiguousarray(a.T).ravel()
    if a.size != 16:
        raise ValueError("a camera matrix has 4 x 4 entries")
    return np.ascontiguousarray(a.ravel())


class sched_params:
    """sched_params (scheduler.h:53-96): a camera, or view / projection matrices (has_camera_matrices),
    the render target, the pixel sampler and the scissor box."""

    def __init__(self, cam, rt, sampler=pixel_sampler.uniform_type, image_size=None, view_matrix=None,
                 proj_matrix=None):
        if not hasattr(sampler, "kind"):
            raise TypeError("sched_params: the sampler is one of the pixel_sampler types")
        self.sampler = sampler
        self.cam = cam          # stored by value in the reference (scheduler.h:72)
        self.rt = rt            # by reference (scheduler.h:73)
        # the matrix form (scheduler.h:76-96), column-major float32[16], or None
        self.view_matrix = None if view_matrix is None else _matrix4(view_matrix)
        self.proj_matrix = None if proj_matrix is None else _matrix4(proj_matrix)
        # scissor_box (scheduler.h:25-31, default recti(0, 0, w, h) at :175): x, y and the EXCLUSIVE
        # right / bottom edges w, h, as cuda_sched.inl:71 reads them; None = the whole image
        self.scissor_box = None
        # full image size; differs from the rt size only for a packed image-tile shard
        self.image_size = tuple(image_size) if image_size else (rt.width(), rt.height())


def make_sched_params(*args, image_size=None):
    """make_sched_params([pixel_sampler], camera, rt) or make_sched_params([pixel_sampler], view_matrix,
    proj_matrix, rt) -- scheduler.h:164-242."""
    sampler = pixel_sampler.uniform_type
    if args and hasattr(args[0], "kind"):
        sampler, args = args[0], args[1:]
    if len(args) == 2:
        cam, rt = args
        return sched_params(cam, rt, sampler, image_size)
    if len(args) == 3:
        view, proj, rt = args
        return sched_params(None, rt, sampler, image_size, view_matrix=view, proj_matrix=proj)
    raise TypeError("make_sched_params([sampler,] camera, render_target) or ([sampler,] view, proj, render_target)")


class _builtin_kernel:
    def __init__(self, bvh, kind, samples, radius, eps, bg, count_tests=False):
        self.bvh = bvh
        self.desc = capi.vrh_kernel_desc(kind, samples, radius, eps, (C.c_float * 4)(*bg),
                                         capi.VRH_KERNEL_COUNT_TESTS if count_tests else 0)


def closest_hit_kernel(bvh, bg=(0.1, 0.2, 0.3, 1.0), count_tests=False):
    """Primary visibility: closest_hit(ray, bvhs) (traverse_linear.inl:286-329); colour = hit ? 1 : bg."""
    return _builtin_kernel(bvh, capi.VRH_KERNEL_PRIMARY, 0, 0.0, 0.0, bg, count_tests)


def ao_kernel(bvh, samples=8, radius=0.1, eps=1e-3, bg=(0.1, 0.2, 0.3, 1.0), count_tests=False, occ=None):
    """ao/main.cpp:183-246 (closest hit + `samples` any_hit rays, radius), Appendix-A sampler.
    occ: write the target's occlusion-mask buffer (None: when samples <= 8 -- one bit per sample in a
    byte; with more samples the buffer is left untouched, VRH_KERNEL_NO_OCC)."""
    k = _builtin_kernel(bvh, capi.VRH_KERNEL_AO, samples, radius, eps, bg, count_tests)
    if (samples > 8) if occ is None else not occ:
        k.desc.flags |= capi.VRH_KERNEL_NO_OCC
    return k


# ---- mask intersector ------------------------------------------------------

class hit_mask:
    """The intersector example's mask_intersector (examples/intersector/main.cpp:251-330: a
    basic_intersector whose operator()(ray, tri) clears hr.hit where a mask over the hit's texture
    coordinate says so) as data: tex_coords (3 x (u, v) per prim_id, float32) and a (H, W) uint8
    mask; vrh.h vrh_hit_mask_create states the lookup.  Attach with with_hit_mask(kernel, mask)."""

    def __init__(self, ctx, tex_coords, mask):
        self.ctx = ctx
        self.tex_coords = np.ascontiguousarray(tex_coords, np.float32).reshape(-1, 2)
        self.mask = np.ascontiguousarray(mask, np.uint8)
        if self.mask.ndim != 2:
            raise ValueError("hit_mask: mask must be (H, W)")
        h = C.c_void_p()
        capi.check("vrh_hit_mask_create", ctx.handle, _p(self.tex_coords), len(self.tex_coords), _p(self.mask),
                   self.mask.shape[1], self.mask.shape[0], C.byref(h))
        self.handle = h

    def close(self):
        if self.handle:
            capi.lib().vrh_hit_mask_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def with_hit_mask(kernel, mask):
    """closest_hit / any_hit with the mask intersector for every ray of `kernel` (the reference's
    closest_hit(ray, begin, end, intersector) / any_hit(..., intersector), traverse_linear.inl:232-329)."""
    kernel.desc.hit_mask = mask.handle if mask is not None else None
    kernel.hit_mask = mask
    return kernel


# ---- shading ----------------------------------------------------------------

PLASTIC_DTYPE = np.dtype([("ca", "<f4", 3), ("ka", "<f4"), ("cd", "<f4", 3), ("kd", "<f4"), ("cs", "<f4", 3),
                          ("ks", "<f4"), ("exp", "<f4")])
POINT_LIGHT_DTYPE = np.dtype([("position", "<f4", 3), ("cl", "<f4", 3), ("kl", "<f4"), ("constant_att", "<f4"),
                              ("linear_att", "<f4"), ("quadratic_att", "<f4")])
normals_per_face_binding = capi.VRH_NORMALS_PER_FACE
normals_per_vertex_binding = capi.VRH_NORMALS_PER_VERTEX


def plastic(ca=(0.0, 0.0, 0.0), ka=1.0, cd=(0.8, 0.8, 0.8), kd=1.0, cs=(0.0, 0.0, 0.0), ks=0.0, exp=1.0):
    """One plastic<float> material record (material.h:267-323 setters: set_ca/ka/cd/kd/cs/ks/specular_exp)."""
    m = np.zeros((), PLASTIC_DTYPE)
    m["ca"], m["ka"], m["cd"], m["kd"], m["cs"], m["ks"], m["exp"] = ca, ka, cd, kd, cs, ks, exp
    return m


def point_light(position, cl=(1.0, 1.0, 1.0), kl=1.0, constant_att=1.0, linear_att=0.0, quadratic_att=0.0):
    """One point_light<float> record (point_light.h:18-66; attenuation defaults 1, 0, 0)."""
    l_ = np.zeros((), POINT_LIGHT_DTYPE)
    l_["position"], l_["cl"], l_["kl"] = position, cl, kl
    l_["constant_att"], l_["linear_att"], l_["quadratic_att"] = constant_att, linear_att, quadratic_att
    return l_


class shading:
    """Device materials (plastic, indexed by geom_id) + point lights: the materials / lights
    arguments of make_kernel_params (kernels.h:357-389), copied to the GPU once."""

    def __init__(self, ctx, materials, lights):
        self.ctx = ctx
        self.materials = np.ascontiguousarray(np.atleast_1d(materials), PLASTIC_DTYPE)
        self.lights = np.ascontiguousarray(np.atleast_1d(lights), POINT_LIGHT_DTYPE)
        h = C.c_void_p()
        capi.check("vrh_shading_create", ctx.handle, _p(self.materials), len(self.materials),
                   _p(self.lights) if len(self.lights) else None, len(self.lights), C.byref(h))
        self.handle = h

    def close(self):
        if self.handle:
            capi.lib().vrh_shading_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class model:
    """Scene read from a Wavefront OBJ file: the reference's `model` (src/common/model.h:20-49).

    primitives         TRIANGLE_DTYPE, prim_id = kept-triangle order, geom_id = `usemtl` material
    shading_normals    (M, 4) float32, three per triangle whose corners all carry `vn`
    geometric_normals  (N, 4) float32, normalize(cross(e1, e2)) -- the per-face normals
    tex_coords         (K, 2) float32, incl. the reference's dummy padding
    materials          PLASTIC_DTYPE (ca = Ka, cd = Kd, cs = Ks, ka = kd = ks = 1, exp = Ns)
    material_names / textures   `usemtl` name and map_Kd path per material ("" for padding)
    bbox               (2, 3) float32 [min, max]
    """

    def has_vertex_normals(self):
        return len(self.shading_normals) == 3 * len(self.primitives) and len(self.primitives) > 0


def load_obj(filename):
    """load_obj(filename, model&) (src/common/obj_loader.cpp:299-527) through libvrh's parser."""
    h = C.c_void_p()
    capi.check("vrh_obj_load", str(filename).encode(), C.byref(h))
    try:
        info = capi.vrh_obj_info()
        capi.check("vrh_obj_get_info", h, C.byref(info))
        m = model()
        m.primitives = np.zeros(info.num_triangles, TRIANGLE_DTYPE)
        m.geometric_normals = np.zeros((info.num_triangles, 4), np.float32)
        m.shading_normals = np.zeros((info.num_shading_normals, 4), np.float32)
        m.tex_coords = np.zeros((info.num_tex_coords, 2), np.float32)
        m.materials = np.zeros(info.num_materials, PLASTIC_DTYPE)
        capi.check("vrh_obj_get_data", h, _p(m.primitives), _p(m.geometric_normals), _p(m.shading_normals),
                   _p(m.tex_coords), _p(m.materials))
        m.material_names = [capi.lib().vrh_obj_material_name(h, i).decode() for i in range(info.num_materials)]
        m.textures = [capi.lib().vrh_obj_material_texture(h, i).decode() for i in range(info.num_materials)]
        m.bbox = np.array([list(info.bbox_min), list(info.bbox_max)], np.float32)
        m.num_degenerate = info.num_degenerate
        m.num_unknown_materials = info.num_unknown_materials
        m.num_missing_files = info.num_missing_files
        return m
    finally:
        capi.lib().vrh_obj_free(h)


def sah_cost(nodes, ci=1.2, cl=0.0, cp=1.0):
    """sah_cost(bvh) (detail/bvh/statistics.h:30-73) of a reference-layout node array."""
    nodes = np.ascontiguousarray(nodes, BVH_NODE_DTYPE)
    out = C.c_float()
    capi.check("vrh_bvh_sah_cost", _p(nodes), len(nodes), ci, cl, cp, C.byref(out))
    return float(out.value)


def simple_kernel(bvh, shade, binding=normals_per_face_binding, bg=(0.0, 0.0, 0.0, 0.0),
                  ambient=(0.0, 0.0, 0.0, 0.0), count_tests=False):
    """simple::kernel (detail/simple.inl:19-83) over make_kernel_params(binding, prims, normals,
    materials, lights, bounces, eps, bg, ambient): closest hit, ambient + plastic::shade per light."""
    k = _builtin_kernel(bvh, capi.VRH_KERNEL_SIMPLE, 0, 0.0, 0.0, bg, count_tests)
    k.desc.normal_binding = binding
    k.desc.ambient = (C.c_float * 4)(*ambient)
    k.desc.shading = shade.handle
    k.shade = shade          # keep the device arrays alive
    return k


def multi_hit_kernel(bvh, shade, max_hits=16, binding=normals_per_vertex_binding, bg=(0.0, 0.0, 0.0, 0.0),
                     count_tests=False):
    """multi_hit<max_hits> (traverse_linear.inl:333-380): the max_hits closest hits per pixel into
    the render target's hit lists (hip_buffer_rt.alloc_multi_hit) and the colour of the multi_hit
    example kernel (examples/multi_hit/main.cpp:166-235: first light, alpha 0.3, front to back)."""
    k = simple_kernel(bvh, shade, binding=binding, bg=bg, count_tests=count_tests)
    k.desc.kind = capi.VRH_KERNEL_MULTI_HIT
    k.desc.max_hits = max_hits
    return k


def whitted_kernel(bvh, shade, binding=normals_per_face_binding, bg=(0.0, 0.0, 0.0, 0.0),
                   ambient=(0.0, 0.0, 0.0, 0.0), num_bounces=4, epsilon=1e-3, count_tests=False):
    """whitted::kernel (detail/whitted.inl:186-277) over make_kernel_params(binding, prims, normals,
    materials, lights, num_bounces, epsilon, bg, ambient): simple::kernel's shading with an any-hit
    shadow ray per light and the plastic reflection (kr 0.1) for num_bounces loop iterations."""
    k = simple_kernel(bvh, shade, binding=binding, bg=bg, ambient=ambient, count_tests=count_tests)
    k.desc.kind = capi.VRH_KERNEL_WHITTED
    k.desc.num_bounces = num_bounces
    k.desc.eps = epsilon
    return k


class hip_sched:
    """hip_sched<R>: drop-in for cuda_sched<R> (cuda_sched.h:25-40).

    frame() = rt.begin_frame() -> vrh_render -> rt.end_frame().  By default the scheduler issues frames
    as cuda_sched does (cuda_sched.inl:306-320: frame() enqueues and returns, gpu_buffer_rt::end_frame
    is a no-op, gpu_buffer_rt.inl:84-86): it turns on its context's asynchronous frames, back-to-back
    frames overlap their launch tails on the context's frame lanes, and rt.download() / ctx.sync() wait
    for them (VRH_OPT_ASYNC_FRAMES).  hip_sched(ctx, async_frames=False) keeps frame() synchronous (it
    returns when the frame is done, like tiled_sched).  shard=(index, count, packed) renders only that
    image-tile shard.
    """

    def __init__(self, ctx, async_frames=True):
        self.ctx = ctx
        ctx.set_option("async_frames", 1 if async_frames else 0)

    def frame(self, kernel, sparams, frame_num=0, shard=None, sync=True):
        if not isinstance(kernel, _builtin_kernel):
            raise TypeError("hip_sched runs built-in kernels only (closest_hit / ao / simple / multi_hit / whitted): an arbitrary "
                            "callable cannot cross the C ABI")
        rt = sparams.rt
        sampler = getattr(sparams, "sampler", pixel_sampler.uniform_type)
        if getattr(sparams, "view_matrix", None) is not None:
            # camera matrices (sched_common.h:152-176): vrh_render_view, whole image
            if shard is not None:
                raise ValueError("hip_sched::frame: camera matrices render the whole image")
            vc = view_camera(sparams.view_matrix, sparams.proj_matrix, *sparams.image_size)
            if sparams.scissor_box is not None:
                vc.scissor[:] = [int(v) for v in sparams.scissor_box]
            rt.begin_frame()
            render_view(self.ctx, kernel.bvh, rt, vc, kernel, sampler, frame_num)
            if sync:
                rt.end_frame()
            return
        cam = sparams.cam.basis(*sparams.image_size)
        if sparams.scissor_box is not None:
            cam.scissor[:] = [int(v) for v in sparams.scissor_box]
        sh = None
        if shard is not None:
            sh = capi.vrh_shard(shard[0], shard[1], 1 if shard[2] else 0, 0)
        rt.begin_frame()
        if sampler.kind != pixel_sampler.uniform_type.kind:
            # jittered / jittered_blend / ssaa<N> (sched_common.h:160-300, 440-720)
            if sh is not None:
                raise ValueError("hip_sched::frame: pixel samplers other than uniform render the whole image")
            ps = capi.vrh_pixel_sampler(sampler.kind, sampler.count)
            capi.check("vrh_render_sampled", self.ctx.handle, kernel.bvh.handle, rt.handle, C.byref(cam),
                       C.byref(kernel.desc), C.byref(ps), frame_num)
        else:
            capi.check("vrh_render", self.ctx.handle, kernel.bvh.handle, rt.handle, C.byref(cam), C.byref(kernel.desc),
                       C.byref(sh) if sh is not None else None, frame_num)
        if sync:
            rt.end_frame()


def render(ctx, bvh, rt, cam_basis, kernel, shard=None, frame_num=0):
    """Low-level frame with an explicit vrh_camera (full-image size) and optional vrh_shard."""
    capi.check("vrh_render", ctx.handle, bvh.handle, rt.handle, C.byref(cam_basis), C.byref(kernel.desc),
               C.byref(shard) if shard is not None else None, frame_num)


def render_sampled(ctx, bvh, rt, cam_basis, kernel, sampler, frame_num=0):
    """vrh_render_sampled: one frame through a pixel sampler (a pixel_sampler type)."""
    ps = capi.vrh_pixel_sampler(sampler.kind, sampler.count)
    capi.check("vrh_render_sampled", ctx.handle, bvh.handle, rt.handle, C.byref(cam_basis), C.byref(kernel.desc),
               C.byref(ps), frame_num)


def view_camera(view, proj, width, height):
    """vrh_view_camera of view / projection matrices (column-major 16-vectors or 4x4 [row, col])."""
    vc = capi.vrh_view_camera()
    vc.view[:] = [float(x) for x in _matrix4(view)]
    vc.proj[:] = [float(x) for x in _matrix4(proj)]
    vc.width, vc.height = int(width), int(height)
    return vc


def render_view(ctx, bvh, rt, view_cam, kernel, sampler=pixel_sampler.uniform_type, frame_num=0):
    """vrh_render_view: one frame from camera matrices (a vrh_view_camera) through a pixel sampler."""
    ps = capi.vrh_pixel_sampler(sampler.kind, sampler.count)
    capi.check("vrh_render_view", ctx.handle, bvh.handle, rt.handle, C.byref(view_cam), C.byref(kernel.desc),
               C.byref(ps), frame_num)


def matrix_inverse(m):
    """vrh_matrix_inverse: the host inverse vrh_render_view applies (matrix4.inl:209-244)."""
    a = _matrix4(m)
    out = np.empty(16, np.float32)
    capi.lib().vrh_matrix_inverse(a.ctypes.data, out.ctypes.data)
    return out


def render_batch(ctx, bvh, rt, cam_bases, kernel, shard=None, frame_num=0):
    """vrh_render_batch: len(cam_bases) frames in one persistent launch (frames in flight); frame f
    lands in rows [f * R, (f + 1) * R) of rt (R = image height, or rt height / frames when packed)
    and has frame number frame_num + f."""
    n = len(cam_bases)
    cams = (capi.vrh_camera * n)(*cam_bases)
    capi.check("vrh_render_batch", ctx.handle, bvh.handle, rt.handle, cams, n, C.byref(kernel.desc),
               C.byref(shard) if shard is not None else None, frame_num)


def shard_bands(height, index, count):
    return capi.lib().vrh_shard_bands(height, index, count)


def unshard(ctx, width, height, count, dst_rt, color_ptr=0, prim_id_ptr=0, occ_ptr=0, shard_stride_bytes=0,
            kernel=None):
    """vrh_unshard: gathered packed shards -> full render target (device pointers).  Without a
    gathered colour the colour is re-derived from prim ids + AO masks with `kernel`."""
    vp = lambda p: C.c_void_p(p) if p else None  # noqa: E731
    capi.check("vrh_unshard", ctx.handle, width, height, count, vp(color_ptr), vp(prim_id_ptr), vp(occ_ptr),
               int(shard_stride_bytes), C.byref(kernel.desc) if kernel is not None else None, dst_rt.handle)


# ---- multi-GPU render groups (vrh.h vrh_group_*) -------------------------------------

GROUP_ID_BYTES = capi.VRH_GROUP_ID_BYTES


class render_group:
    """One rank's membership of a multi-GPU render group (an RCCL communicator, vrh_group).

    One process per GPU: rank 0 makes an id with render_group.unique_id(), every rank receives it
    (any channel) and constructs render_group(ctx, nranks, rank, uid).  One process driving several
    GPUs: render_group.local([ctx0, ctx1, ...]) returns one member per context; render the frames
    with render_sharded(members, ...).  The exchange is libvrh's (ncclSend / ncclRecv on the
    group's own stream); nothing of it goes through torch."""

    def __init__(self, ctx, nranks, rank, uid, timeout_ms=0):
        """timeout_ms: the deadline of every wait on a peer (join, exchange, sync); 0 = the library's
        VRH_GROUP_TIMEOUT_MS.  A missed deadline aborts the communicator and raises VrhError with
        code VRH_ERR_TIMEOUT instead of hanging (vrh_group_join_timeout)."""
        if len(uid) != GROUP_ID_BYTES:
            raise ValueError("render_group: the id is 128 bytes (vrh_group_id)")
        self.ctx = ctx
        buf = (C.c_char * GROUP_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        capi.check("vrh_group_join_timeout", ctx.handle, nranks, rank, C.cast(buf, C.c_void_p), int(timeout_ms),
                   C.byref(h))
        self.handle = h
        self.nranks, self.rank = nranks, rank

    @staticmethod
    def unique_id():
        buf = (C.c_char * GROUP_ID_BYTES)()
        capi.check("vrh_group_get_id", C.cast(buf, C.c_void_p))
        return bytes(buf.raw)

    @classmethod
    def local(cls, ctxs):
        n = len(ctxs)
        hs = (C.c_void_p * n)()
        capi.check("vrh_group_create_local", n, (C.c_void_p * n)(*[c.handle.value for c in ctxs]), hs)
        out = []
        for i, c in enumerate(ctxs):
            g = cls.__new__(cls)
            g.ctx, g.handle, g.nranks, g.rank = c, C.c_void_p(hs[i]), n, i
            out.append(g)
        return out

    def render(self, scene, kernel, dst_rt, cam_bases, frame_num=0, shards=0, fields=None):
        """vrh_render_sharded for this member alone (one process per GPU)."""
        render_sharded([self], [scene], [kernel], dst_rt, cam_bases, frame_num, shards, fields)

    def broadcast_scene(self, scene=None):
        """vrh_group_broadcast_scene for this member alone (one process per GPU): rank 0 passes its
        hip_index_bvh, the other ranks None; every rank gets a replica on its own context."""
        return broadcast_scene([self], scene)[0]

    def sync(self):
        capi.check("vrh_group_sync", self.handle)

    def set_timeout(self, timeout_ms):
        capi.check("vrh_group_set_timeout", self.handle, int(timeout_ms))

    @property
    def failed(self):
        """True once the group was aborted (an RCCL error or a missed deadline)."""
        return bool(capi.lib().vrh_group_failed(self.handle)) if getattr(self, "handle", None) else False

    def close(self):
        if getattr(self, "handle", None):
            capi.lib().vrh_group_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def broadcast_scene(groups, scene=None):
    """vrh_group_broadcast_scene: rank 0's scene (a hip_index_bvh; None on the other ranks) replicated
    over the group by RCCL broadcasts -- one new hip_index_bvh per member in `groups`, on its context
    (the scene goes to every GPU once, instead of every rank building it)."""
    n = len(groups)
    out = (C.c_void_p * n)()
    capi.check("vrh_group_broadcast_scene", n, (C.c_void_p * n)(*[g.handle.value for g in groups]),
               scene.handle if scene is not None else None, out)
    replicas = []
    for i, g in enumerate(groups):
        r = hip_index_bvh.__new__(hip_index_bvh)
        r.ctx, r.handle = g.ctx, C.c_void_p(out[i])
        r._refresh_info()
        replicas.append(r)
    return replicas


def render_sharded(groups, scenes_, kernels, dst_rt, cam_bases, frame_num=0, shards=0, fields=None):
    """vrh_render_sharded: len(cam_bases) frames over the group; rank 0's dst_rt (W x H * frames)
    receives them in image order (None on the other ranks).  fields: the vrh_rt_flags assembled on
    the root (default: colour + prim id + AO mask, the same on every rank)."""
    n = len(groups)
    nf = len(cam_bases)
    if fields is None:
        fields = capi.VRH_RT_COLOR | capi.VRH_RT_PRIM_ID | capi.VRH_RT_OCC
    gs = (C.c_void_p * n)(*[g.handle.value for g in groups])
    ss = (C.c_void_p * n)(*[s.handle.value for s in scenes_])
    ks = (capi.vrh_kernel_desc * n)(*[k.desc for k in kernels])
    cams = (capi.vrh_camera * nf)(*cam_bases)
    capi.check("vrh_render_sharded", n, gs, ss, ks, dst_rt.handle if dst_rt is not None else None, fields, cams, nf,
               frame_num, shards)
