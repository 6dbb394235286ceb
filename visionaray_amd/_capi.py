"""ctypes binding of libvrh.so (include/vrh.h), the C-ABI of the MI355X traversal backend.

The library is built in-tree (``make -C visionaray_amd`` or ``__graft_entry__.build()``) into
``visionaray_amd/_lib/libvrh.so``.  There is no fallback: if the library is missing or a call fails,
an exception is raised.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VRH_LIB") or os.path.join(_HERE, "_lib", "libvrh.so")

# enums (vrh.h)
VRH_OK, VRH_ERR_INVALID, VRH_ERR_HIP, VRH_ERR_OOM, VRH_ERR_UNSUPPORTED, VRH_ERR_NO_DEVICE, VRH_ERR_TIMEOUT = range(7)
VRH_GROUP_TIMEOUT_MS = 120000
VRH_PRIM_TRI64, VRH_PRIM_SPHERE48 = 0, 1
VRH_KERNEL_PRIMARY, VRH_KERNEL_AO, VRH_KERNEL_SIMPLE, VRH_KERNEL_MULTI_HIT, VRH_KERNEL_WHITTED = 0, 1, 2, 3, 4
VRH_MAX_HITS = 16
VRH_NORMALS_PER_FACE, VRH_NORMALS_PER_VERTEX = 0, 1
VRH_RT_COLOR, VRH_RT_PRIM_ID, VRH_RT_T, VRH_RT_OCC, VRH_RT_ALL = 1, 2, 4, 8, 15


class vrh_camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("cam_u", C.c_float * 3), ("cam_v", C.c_float * 3),
                ("cam_w", C.c_float * 3), ("width", C.c_uint32), ("height", C.c_uint32),
                ("scissor", C.c_uint32 * 4)]


class vrh_kernel_desc(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("samples", C.c_uint32), ("radius", C.c_float), ("eps", C.c_float),
                ("bg", C.c_float * 4), ("flags", C.c_uint32), ("normal_binding", C.c_uint32),
                ("ambient", C.c_float * 4), ("shading", C.c_void_p), ("max_hits", C.c_uint32),
                ("num_bounces", C.c_uint32), ("hit_mask", C.c_void_p)]


class vrh_plastic(C.Structure):
    _fields_ = [("ca", C.c_float * 3), ("ka", C.c_float), ("cd", C.c_float * 3), ("kd", C.c_float),
                ("cs", C.c_float * 3), ("ks", C.c_float), ("exp", C.c_float)]


class vrh_point_light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("cl", C.c_float * 3), ("kl", C.c_float), ("constant_att", C.c_float),
                ("linear_att", C.c_float), ("quadratic_att", C.c_float)]


VRH_KERNEL_COUNT_TESTS = 1
VRH_KERNEL_NO_OCC = 2
VRH_BAND_ROWS = 8
VRH_MAX_BATCH = 32
VRH_OPT_BLOCK_THREADS, VRH_OPT_STACK_CAP, VRH_OPT_AO_SCHEDULE, VRH_OPT_BLOCKS_PER_CU = 1, 2, 3, 4
VRH_OPT_WAVES_PER_SIMD, VRH_OPT_EXACT_MINMAX, VRH_OPT_XCD_QUEUES, VRH_OPT_REFILL_MIN = 5, 6, 7, 8
VRH_OPT_WIDE_ANYHIT, VRH_OPT_DESCENT_CAP, VRH_OPT_POP_ON_MISS, VRH_OPT_COOP_FETCH = 10, 11, 12, 13
VRH_OPT_SCALAR_FETCH, VRH_OPT_PAIR_LAYOUT, VRH_OPT_AO_GATE, VRH_OPT_WAVE_TIMES = 14, 15, 16, 19
VRH_OPT_AO_CUT = 20
VRH_OPT_AO_SHARE = 22
VRH_OPT_CLUSTER_TILES = 23
VRH_OPT_QUAD_REFILL = 24
VRH_OPT_GROUP_UNITS = 25
VRH_OPT_ASYNC_FRAMES = 26
VRH_OPT_AO_STEAL = 21
VRH_MAX_TIMED_FRAMES = 1024
VRH_MAX_SCENE_LIST = 8
VRH_GROUP_ID_BYTES = 128


class vrh_accum_stats(C.Structure):
    _fields_ = [("frames", C.c_uint32), ("timed_frames", C.c_uint32), ("kernel_ms_total", C.c_double),
                ("kernel_ms_min", C.c_double), ("kernel_ms_max", C.c_double), ("rays", C.c_uint64),
                ("hits", C.c_uint64), ("span_ms", C.c_double)]


class vrh_pixel_sampler(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("count", C.c_uint32)]


VRH_SAMPLER_UNIFORM, VRH_SAMPLER_JITTERED, VRH_SAMPLER_JITTERED_BLEND, VRH_SAMPLER_SSAA = 0, 1, 2, 3


class vrh_view_camera(C.Structure):
    _fields_ = [("view", C.c_float * 16), ("proj", C.c_float * 16), ("width", C.c_uint32), ("height", C.c_uint32),
                ("scissor", C.c_uint32 * 4)]


class vrh_shard(C.Structure):
    _fields_ = [("index", C.c_uint32), ("count", C.c_uint32), ("packed", C.c_uint32), ("reserved", C.c_uint32)]


class vrh_frame_stats(C.Structure):
    _fields_ = [("kernel_ms", C.c_float), ("rays", C.c_uint64), ("hits", C.c_uint64), ("box_tests", C.c_uint64),
                ("prim_tests", C.c_uint64), ("launches", C.c_uint32),
                ("grid_blocks", C.c_uint32), ("block_threads", C.c_uint32), ("stack_depth", C.c_uint32),
                ("frames", C.c_uint32),
                ("wave_steps", C.c_uint64), ("busy_lane_steps", C.c_uint64), ("wave_box_iters", C.c_uint64),
                ("wave_prim_iters", C.c_uint64), ("wave_box_uniform_iters", C.c_uint64),
                ("l1_lines", C.c_uint64), ("l1_requests", C.c_uint64), ("vmem_instrs", C.c_uint64),
                ("l1_group_accesses", C.c_uint64), ("l1_ideal_accesses", C.c_uint64),
                ("l1_group_by_kind", C.c_uint64 * 5)]


class vrh_scene_view(C.Structure):
    _fields_ = [("pairs", C.c_void_p), ("prims", C.c_void_p), ("normals", C.c_void_p), ("root", C.c_uint32),
                ("max_depth", C.c_uint32), ("prim_kind", C.c_uint32), ("finite_bounds", C.c_uint32),
                ("num_prims", C.c_uint32), ("quad_depth", C.c_uint32), ("reserved", C.c_uint32 * 2),
                ("quads", C.c_void_p)]


class vrh_scene_info(C.Structure):
    _fields_ = [("num_nodes", C.c_uint32), ("num_prims", C.c_uint32), ("num_indices", C.c_uint32),
                ("prim_kind", C.c_uint32), ("max_depth", C.c_uint32), ("device_bytes", C.c_uint64),
                ("wide_records", C.c_uint32), ("wide_depth", C.c_uint32), ("max_prim_id", C.c_uint32),
                ("max_geom_id", C.c_uint32), ("vertex_normals", C.c_uint32), ("gpu_built", C.c_uint32),
                ("build_ms", C.c_float), ("num_bvhs", C.c_uint32)]


class vrh_build_desc(C.Structure):
    _fields_ = [("method", C.c_uint32), ("max_leaf", C.c_uint32)]


VRH_BUILD_LBVH = 0


class vrh_obj_info(C.Structure):
    _fields_ = [("num_triangles", C.c_uint32), ("num_shading_normals", C.c_uint32),
                ("num_tex_coords", C.c_uint32), ("num_materials", C.c_uint32), ("num_degenerate", C.c_uint32),
                ("num_unknown_materials", C.c_uint32), ("num_missing_files", C.c_uint32),
                ("reserved", C.c_uint32), ("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3)]


class vrh_wire_layout(C.Structure):
    _fields_ = [("prim_id", C.c_uint64), ("occ", C.c_uint64), ("t", C.c_uint64), ("color", C.c_uint64),
                ("code", C.c_uint64), ("shard_bytes", C.c_uint64), ("rows", C.c_uint32), ("derive", C.c_uint32)]


VRH_WIRE_ABSENT = (1 << 64) - 1


class VrhError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed (status {code}): {msg}")
        self.code = code


# every exported symbol of include/vrh.h with its signature: name -> (restype, argtypes)
_vp, _u32, _pf = C.c_void_p, C.c_uint32, C.POINTER(C.c_float)
SIGNATURES = {
    "vrh_make_camera": (C.c_int, [_pf, _pf, _pf, C.c_float, C.c_float, _u32, _u32, C.POINTER(vrh_camera)]),
    "vrh_version": (C.c_char_p, []),
    "vrh_last_error": (C.c_char_p, []),
    "vrh_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "vrh_ctx_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
    "vrh_ctx_create_on_stream": (C.c_int, [C.c_int, _vp, C.POINTER(_vp)]),
    "vrh_ctx_destroy": (C.c_int, [_vp]),
    "vrh_ctx_get_stream": (C.c_int, [_vp, C.POINTER(C.c_int), C.POINTER(C.c_void_p)]),
    "vrh_ctx_set_option": (C.c_int, [_vp, _u32, C.c_int64]),
    "vrh_scene_upload": (C.c_int, [_vp, _vp, _u32, _vp, _u32, _u32, _vp, _u32, _vp, C.POINTER(_vp)]),
    "vrh_scene_get_info": (C.c_int, [_vp, C.POINTER(vrh_scene_info)]),
    "vrh_scene_get_view": (C.c_int, [_vp, C.c_uint32, C.POINTER(vrh_scene_view)]),
    "vrh_get_wave_times": (C.c_int, [_vp, _vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_double)]),
    "vrh_get_tile_times": (C.c_int, [_vp, _vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "vrh_ctx_user_queues": (C.c_int, [_vp, C.POINTER(_vp)]),
    "vrh_scene_list_create": (C.c_int, [_vp, C.POINTER(_vp), _u32, _vp, _u32, C.POINTER(_vp)]),
    "vrh_scene_free": (C.c_int, [_vp]),
    "vrh_scene_set_vertex_normals": (C.c_int, [_vp, _vp, _u32]),
    "vrh_shading_create": (C.c_int, [_vp, _vp, _u32, _vp, _u32, C.POINTER(_vp)]),
    "vrh_shading_free": (C.c_int, [_vp]),
    "vrh_hit_mask_create": (C.c_int, [_vp, _vp, _u32, _vp, _u32, _u32, C.POINTER(_vp)]),
    "vrh_hit_mask_free": (C.c_int, [_vp]),
    "vrh_rt_alloc_multi_hit": (C.c_int, [_vp, _vp, _u32]),
    "vrh_scene_build": (C.c_int, [_vp, _vp, _u32, _u32, _vp, _vp, C.POINTER(_vp)]),
    "vrh_scene_download_bvh": (C.c_int, [_vp, _vp, _vp, C.POINTER(_u32), _vp]),
    "vrh_bvh_sah_cost": (C.c_int, [_vp, _u32, C.c_float, C.c_float, C.c_float, C.POINTER(C.c_float)]),
    "vrh_rt_download_multi_hit": (C.c_int, [_vp, _vp, _vp, _vp]),
    "vrh_rt_alloc": (C.c_int, [_vp, _u32, _u32, _u32, C.POINTER(_vp)]),
    "vrh_rt_wrap": (C.c_int, [_vp, _u32, _u32, _vp, _vp, _vp, _vp, C.POINTER(_vp)]),
    "vrh_rt_get_buffers": (C.c_int, [_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp)]),
    "vrh_rt_clear": (C.c_int, [_vp, _vp, _pf]),
    "vrh_rt_free": (C.c_int, [_vp]),
    "vrh_render": (C.c_int, [_vp, _vp, _vp, C.POINTER(vrh_camera), C.POINTER(vrh_kernel_desc),
                             C.POINTER(vrh_shard), _u32]),
    "vrh_render_batch": (C.c_int, [_vp, _vp, _vp, C.POINTER(vrh_camera), _u32, C.POINTER(vrh_kernel_desc),
                                   C.POINTER(vrh_shard), _u32]),
    "vrh_render_sampled": (C.c_int, [_vp, _vp, _vp, C.POINTER(vrh_camera), C.POINTER(vrh_kernel_desc),
                                     C.POINTER(vrh_pixel_sampler), _u32]),
    "vrh_render_view": (C.c_int, [_vp, _vp, _vp, C.POINTER(vrh_view_camera), C.POINTER(vrh_kernel_desc),
                                  C.POINTER(vrh_pixel_sampler), _u32]),
    "vrh_matrix_inverse": (None, [_vp, _vp]),
    "vrh_sync": (C.c_int, [_vp]),
    "vrh_last_frame_stats": (C.c_int, [_vp, C.POINTER(vrh_frame_stats)]),
    "vrh_stats_reset": (C.c_int, [_vp]),
    "vrh_get_accum_stats": (C.c_int, [_vp, C.POINTER(vrh_accum_stats)]),
    "vrh_rt_download": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "vrh_rt_upload": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "vrh_shard_bands": (C.c_uint32, [_u32, _u32, _u32]),
    "vrh_unshard": (C.c_int, [_vp, _u32, _u32, _u32, _vp, _vp, _vp, C.c_uint64, C.POINTER(vrh_kernel_desc), _vp]),
    "vrh_build_bvh": (C.c_int, [_vp, _u32, _u32, _vp, C.POINTER(_u32), _vp, C.POINTER(_u32)]),
    "vrh_group_get_id": (C.c_int, [C.c_void_p]),
    "vrh_group_join": (C.c_int, [_vp, _u32, _u32, C.c_void_p, C.POINTER(_vp)]),
    "vrh_group_join_timeout": (C.c_int, [_vp, _u32, _u32, C.c_void_p, _u32, C.POINTER(_vp)]),
    "vrh_group_set_timeout": (C.c_int, [_vp, _u32]),
    "vrh_group_failed": (C.c_int, [_vp]),
    "vrh_group_create_local": (C.c_int, [_u32, C.POINTER(_vp), C.POINTER(_vp)]),
    "vrh_group_info": (C.c_int, [_vp, C.POINTER(_u32), C.POINTER(_u32)]),
    "vrh_group_sync": (C.c_int, [_vp]),
    "vrh_group_free": (C.c_int, [_vp]),
    "vrh_group_broadcast_scene": (C.c_int, [_u32, C.POINTER(_vp), _vp, C.POINTER(_vp)]),
    "vrh_render_sharded": (C.c_int, [_u32, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(vrh_kernel_desc), _vp, _u32,
                                     C.POINTER(vrh_camera), _u32, _u32, _u32]),
    "vrh_group_shards_of": (C.c_uint32, [_u32, _u32, _u32, C.POINTER(_u32), _u32]),
    "vrh_group_shard_owner": (C.c_uint32, [_u32, _u32]),
    "vrh_group_wire_layout": (C.c_int, [_u32, C.POINTER(vrh_kernel_desc), _u32, _u32, _u32, _u32,
                                        C.POINTER(vrh_wire_layout)]),
    "vrh_shard_packed_rows": (C.c_int, [_u32, _u32, _u32, C.POINTER(C.c_int32)]),
    "vrh_pack_codes_host": (C.c_int, [_vp, _vp, _vp, C.c_uint64]),
    "vrh_unshard_host": (C.c_int, [_vp, C.POINTER(vrh_wire_layout), _u32, _u32, _u32, _u32, _u32,
                                   C.POINTER(vrh_kernel_desc), _vp, _vp, _vp, _vp]),
    "vrh_gen_heightfield": (C.c_int, [_u32, _vp]),
    "vrh_gen_cornell": (C.c_int, [_vp]),
    "vrh_gen_spheres": (C.c_int, [_u32, _vp]),
    "vrh_face_normals": (C.c_int, [_vp, _u32, _vp]),
    "vrh_obj_load": (C.c_int, [C.c_char_p, C.POINTER(_vp)]),
    "vrh_obj_get_info": (C.c_int, [_vp, C.POINTER(vrh_obj_info)]),
    "vrh_obj_get_data": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "vrh_obj_material_name": (C.c_char_p, [_vp, _u32]),
    "vrh_obj_material_texture": (C.c_char_p, [_vp, _u32]),
    "vrh_obj_free": (C.c_int, [_vp]),
}

_lib = None


def lib():
    """Load libvrh.so (raises if it was not built -- there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C {_HERE}` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("VRH_LIB") and not hasattr(L, name):
                continue            # an older library under A/B (tools/ab_variants.py): what it has
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(fn, *args):
    """Call lib().fn(*args); raise VrhError on a non-zero status."""
    rc = getattr(lib(), fn)(*args)
    if rc != VRH_OK:
        raise VrhError(fn, rc, lib().vrh_last_error().decode(errors="replace"))
    return rc
