"""visionaray_amd -- MI355X-native (gfx950) backend for Visionaray's ray-traversal hot path.

BVH traversal + ray/triangle and ray/sphere intersection as hand-written HIP kernels behind the
C-ABI in include/vrh.h (libvrh.so), with a host API that mirrors the reference's
scheduler / render_target / BVH interface (hip_sched, hip_buffer_rt, hip_index_bvh).
"""
from . import _capi
from .api import (BVH_NODE_DTYPE, DEGREES_TO_RADIANS, PLASTIC_DTYPE, POINT_LIGHT_DTYPE, SPHERE_DTYPE,
                  TRIANGLE_DTYPE, Context, ao_kernel, build_index_bvh, camera, closest_hit_kernel, device_count,
                  face_normals, hip_buffer_rt, hit_mask, with_hit_mask, hip_index_bvh, hip_sched, index_bvh, make_sched_params,
                  load_obj, make_spheres, make_triangles, model, multi_hit_kernel, normals_per_face_binding, normals_per_vertex_binding, pixel_sampler,
                  coop_fetch_available, plastic, point_light, render, render_batch, sah_cost, shading, shard_bands, simple_kernel, unshard, whitted_kernel)
from ._capi import VrhError

__all__ = [
    "BVH_NODE_DTYPE", "DEGREES_TO_RADIANS", "SPHERE_DTYPE", "TRIANGLE_DTYPE", "Context", "VrhError", "ao_kernel",
    "build_index_bvh", "camera", "closest_hit_kernel", "device_count", "face_normals", "hip_buffer_rt",
    "hip_index_bvh", "hip_sched", "index_bvh", "make_sched_params", "make_spheres", "make_triangles",
    "pixel_sampler", "coop_fetch_available", "render", "render_batch", "shard_bands", "unshard", "_capi", "PLASTIC_DTYPE", "POINT_LIGHT_DTYPE",
    "normals_per_face_binding", "normals_per_vertex_binding", "plastic", "point_light", "shading", "simple_kernel",
    "multi_hit_kernel", "sah_cost", "hit_mask", "with_hit_mask", "load_obj", "model", "whitted_kernel",
]
