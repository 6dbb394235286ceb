"""visionaray_amd -- MI355X-native (gfx950) backend for Visionaray's ray-traversal hot path.

BVH traversal + ray/triangle and ray/sphere intersection as hand-written HIP kernels behind the
C-ABI in include/vrh.h (libvrh.so), with a host API that mirrors the reference's
scheduler / render_target / BVH interface (hip_sched, hip_buffer_rt, hip_index_bvh) and the
multi-GPU render groups (render_group, render_sharded: image-tile shards gathered over RCCL).
"""
from . import _capi
from ._capi import VrhError
from .api import (BVH_NODE_DTYPE, DEGREES_TO_RADIANS, GROUP_ID_BYTES, PLASTIC_DTYPE, POINT_LIGHT_DTYPE,
                  SPHERE_DTYPE, TRIANGLE_DTYPE, Context, ao_kernel, broadcast_scene, build_index_bvh, camera, closest_hit_kernel,
                  device_count, face_normals, hip_buffer_rt, hip_index_bvh, hip_sched,
                  hit_mask, index_bvh, load_obj, make_sched_params, make_spheres, make_triangles, matrix_inverse, model,
                  multi_hit_kernel, normals_per_face_binding, normals_per_vertex_binding, pixel_sampler, plastic,
                  point_light, render, render_batch, render_group, render_sampled, render_sharded, render_view, sah_cost, shading,
                  shard_bands, simple_kernel, unshard, view_camera, whitted_kernel, with_hit_mask)

__all__ = [
    "BVH_NODE_DTYPE", "DEGREES_TO_RADIANS", "GROUP_ID_BYTES", "PLASTIC_DTYPE", "POINT_LIGHT_DTYPE", "SPHERE_DTYPE",
    "TRIANGLE_DTYPE", "Context", "VrhError", "_capi", "ao_kernel", "broadcast_scene", "build_index_bvh", "camera", "closest_hit_kernel",
    "device_count", "face_normals", "hip_buffer_rt", "hip_index_bvh", "hip_sched",
    "hit_mask", "index_bvh", "load_obj", "make_sched_params", "make_spheres", "make_triangles", "matrix_inverse", "model",
    "multi_hit_kernel", "normals_per_face_binding", "normals_per_vertex_binding", "pixel_sampler", "plastic",
    "point_light", "render", "render_batch", "render_group", "render_sampled", "render_sharded", "render_view", "sah_cost",
    "shading", "shard_bands", "simple_kernel", "unshard", "view_camera", "whitted_kernel", "with_hit_mask",
]
