/*
 * include/vrh.h -- C-ABI of the MI355X-native Visionaray traversal backend (libvrh.so).
 *
 * This is the drop-in boundary.  Everything above it -- the C++ header API in
 * include/visionaray_hip/ (hip_sched<R>, hip_buffer_rt<CF,DF>, hip_index_bvh<P>) and the Python
 * mirror in visionaray_amd/ -- packs arguments and calls these entry points; everything below it
 * is hand-written HIP for gfx950.  Plain pointers and sizes only; no C++ or torch types.
 *
 * Reference interfaces replaced (file:line in tu500/visionaray v0.1.0):
 *   vrh_scene_upload   <- cuda_index_bvh<P>(host_bvh) copy-ctor       bvh.h:344-350, 443-448; viewer.cpp:791
 *   vrh_rt_alloc/_free <- gpu_buffer_rt<CF,DF>::resize / dtor        gpu_buffer_rt.h:19-51, .inl:14-47
 *   vrh_rt_clear       <- gpu_buffer_rt::clear_color_buffer (thrust::fill) gpu_buffer_rt.inl:49-76
 *   vrh_render         <- cuda_sched<R>::frame(kernel, sparams)      cuda_sched.h:33-34, .inl:160-198, 238-320
 *                         (render<<<grid,block>>> cuda_sched.inl:53-153 -> persistent traversal kernels)
 *   vrh_rt_download    <- gpu_buffer_rt::display_color_buffer D2H   gpu_buffer_rt.inl:90-119
 *   vrh_sync           <- (none: cuda_sched is async) ; called by hip_buffer_rt::end_frame()
 *   vrh_build_bvh      <- build<index_bvh<P>>(prims, n)              detail/bvh/build.inl:165-178 (+ sah.h)
 *   vrh_scene_build    <- build<index_bvh<P>> + cuda_index_bvh copy, on the GPU (linear BVH)
 *   vrh_bvh_sah_cost   <- sah_cost(bvh)                              detail/bvh/statistics.h:30-73
 *   vrh_shading_create <- make_kernel_params(binding, prims, normals, materials, lights, ...)
 *                                                                     kernels.h:357-389 (device copies of
 *                         the material / light arrays, as viewer.cpp:501-523 uploads them)
 *   VRH_KERNEL_SIMPLE  <- simple::kernel<Params>                     detail/simple.inl:19-83
 *   VRH_KERNEL_WHITTED <- whitted::kernel<Params>                    detail/whitted.inl:186-277
 *   vrh_obj_load       <- load_obj(filename, model&)                 src/common/obj_loader.cpp:299-527
 *
 * Status codes: every function returns 0 on success and never throws or longjmps across the ABI;
 * vrh_last_error() gives a thread-local message for the last failure on the calling thread.
 */
#ifndef VRH_H
#define VRH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VRH_API __attribute__((visibility("default")))

typedef struct vrh_ctx   vrh_ctx;    /* one per GPU: device + hipStream_t + events + work counters */
typedef struct vrh_scene vrh_scene;  /* device-resident index BVH (+ face normals)               */
typedef struct vrh_rt    vrh_rt;     /* device render target (colour + side buffers)             */
typedef struct vrh_shading vrh_shading; /* device materials + lights of the shading kernels       */

enum vrh_status {
    VRH_OK = 0,
    VRH_ERR_INVALID = 1,      /* bad argument / shape                                  */
    VRH_ERR_HIP = 2,          /* HIP runtime error (message in vrh_last_error)         */
    VRH_ERR_OOM = 3,          /* device or host allocation failed                      */
    VRH_ERR_UNSUPPORTED = 4,  /* e.g. BVH deeper than the device stack supports        */
    VRH_ERR_NO_DEVICE = 5,    /* no HIP device visible                                 */
    VRH_ERR_TIMEOUT = 6       /* a render-group peer did not answer within the group's deadline: the
                                 communicator was aborted (ncclCommAbort) and the group is failed */
};

/* primitive layouts accepted by vrh_scene_upload / vrh_build_bvh (reference binary layouts,
 * SURVEY.md Appendix C) */
enum vrh_prim_kind {
    VRH_PRIM_TRI64 = 0,       /* basic_triangle<3,float>: geom_id@0 prim_id@4 v1@16 e1@32 e2@48 */
    VRH_PRIM_SPHERE48 = 1     /* basic_sphere<float>:     geom_id@0 prim_id@4 center@16 radius@32 */
};

/* built-in kernels (a C ABI cannot carry an arbitrary C++ lambda; SURVEY.md §7 hard part 6) */
enum vrh_kernel_kind {
    VRH_KERNEL_PRIMARY = 0,   /* closest_hit primary visibility: colour = hit ? 1 : bg     */
    VRH_KERNEL_AO = 1,        /* ao/main.cpp:183-246 with the Appendix-A counter sampler  */
    VRH_KERNEL_SIMPLE = 2,    /* simple::kernel (detail/simple.inl:19-83): closest hit, then
                                 ambient + one plastic::shade per point light, two-sided  */
    VRH_KERNEL_MULTI_HIT = 3, /* multi_hit<N> (traverse_linear.inl:333-380, detail/multi_hit.h):
                                 the N closest hits per pixel (render-target hit lists) and the
                                 front-to-back compositing kernel of examples/multi_hit/main.cpp */
    VRH_KERNEL_WHITTED = 4    /* whitted::kernel (detail/whitted.inl:186-277): simple::kernel's
                                 shading with an any-hit shadow ray per light and plastic
                                 reflections (kr 0.1) for num_bounces iterations; eps is the
                                 scene epsilon (shadow / reflection ray origin offset)       */
};
#define VRH_MAX_HITS 16

enum vrh_normal_binding {
    VRH_NORMALS_PER_FACE = 0,    /* normals_per_face_binding: face normals[prim_id] (upload)  */
    VRH_NORMALS_PER_VERTEX = 1   /* normals_per_vertex_binding: 3 per prim_id, interpolated
                                    with the hit's barycentrics (vrh_scene_set_vertex_normals) */
};

/* plastic<float> (material.h:267-323, detail/material/plastic.inl): ambient ca * ka, lambertian
 * diffuse cd * kd, blinn specular cs * ks with exponent exp.  Indexed by the hit's geom_id. */
typedef struct { float ca[3]; float ka; float cd[3]; float kd; float cs[3]; float ks; float exp; } vrh_plastic;
/* point_light<float> (point_light.h:18-66, detail/point_light.inl): intensity cl * kl with
 * attenuation 1 / (constant + linear * d + quadratic * d * d) */
typedef struct { float position[3]; float cl[3]; float kl; float constant_att, linear_att, quadratic_att; } vrh_point_light;

enum vrh_rt_flags {
    VRH_RT_COLOR = 1u,        /* RGBA32F colour (pixel_access.h:582-604 store)             */
    VRH_RT_PRIM_ID = 2u,      /* u32 closest-hit prim_id, 0xFFFFFFFF on miss               */
    VRH_RT_T = 4u,            /* f32 closest-hit t, -1 on miss                             */
    VRH_RT_OCC = 8u,          /* u8 AO occlusion mask (bit s = sample s occluded)          */
    VRH_RT_ALL = 15u
};

/* Host-computed pinhole basis exactly as simple_sched.inl:61-89 derives it (bit-exact floats),
 * plus the frame's scissor box (sched_params::scissor_box, scheduler.h:25-31; default
 * recti(0, 0, w, h), scheduler.h:175).  As cuda_sched uses it (cuda_sched.inl:71) the box is
 * {x, y, w, h} with w / h the EXCLUSIVE right / bottom edges: pixels x <= px < w, y <= py < h are
 * rendered, every other pixel of the target is left untouched.  All four zero = the whole image. */
typedef struct {
    float    eye[3];
    float    cam_u[3];
    float    cam_v[3];
    float    cam_w[3];
    uint32_t width, height;   /* full image size (primary ray u,v and the AO pixel index use it) */
    uint32_t scissor[4];      /* x, y, w, h (exclusive edges); all zero: whole image             */
} vrh_camera;

typedef struct vrh_hit_mask vrh_hit_mask;   /* see vrh_hit_mask_create                      */

typedef struct {
    uint32_t kind;            /* vrh_kernel_kind                                          */
    uint32_t samples;         /* AO samples per hit pixel (ao/main.cpp default 8, <= 32; a
                                 VRH_RT_OCC target records at most 8: with more, set
                                 VRH_KERNEL_NO_OCC or use a target without the buffer)       */
    float    radius;          /* AO any_hit max_t (default 0.1)                            */
    float    eps;             /* AO origin offset along the sample direction (1e-3); the
                                 whitted kernel's scene epsilon                              */
    float    bg[4];           /* miss colour                                               */
    uint32_t flags;           /* vrh_kernel_flags                                          */
    /* VRH_KERNEL_SIMPLE / MULTI_HIT (make_kernel_params arguments, kernels.h:357-389) */
    uint32_t normal_binding;  /* vrh_normal_binding                                        */
    float    ambient[4];      /* ambient_color (RGBA; rgb scaled by a, spectrum.inl:375)   */
    const vrh_shading* shading;   /* materials + lights (vrh_shading_create)              */
    uint32_t max_hits;        /* VRH_KERNEL_MULTI_HIT: N (1..VRH_MAX_HITS)                  */
    uint32_t num_bounces;     /* VRH_KERNEL_WHITTED: num_bounces (viewer default 4)          */
    const vrh_hit_mask* hit_mask; /* mask intersector for triangles (NULL: none)              */
} vrh_kernel_desc;

enum vrh_kernel_flags {
    VRH_KERNEL_COUNT_TESTS = 1u,  /* instrumented variant: count box / primitive tests (slower;
                                     feeds the algorithmic-bytes roofline)    */
    VRH_KERNEL_NO_OCC = 2u        /* leave the target's VRH_RT_OCC buffer untouched (AO kernels of
                                     more than 8 samples, whose masks do not fit its bytes, render
                                     into a target that has one)                              */
};

/* Image-tile sharding: the image is cut into bands of VRH_BAND_ROWS = 8 rows (one
 * row of 8x8 wave tiles; finer than tiled_sched's 16-row tiles so 1080 rows split over 8 GPUs
 * within 1 %); shard g of N renders bands b with b % N == g.
 * packed = 0: pixels land at their image position in a W x H target.
 * packed = 1: owned bands are stored back to back (band b at local band b / N) in a target of
 *             W x (VRH_BAND_ROWS * vrh_shard_bands(H, g, N)) rows -- the layout gathered over RCCL. */
#define VRH_BAND_ROWS 8
typedef struct {
    uint32_t index, count, packed, reserved;
} vrh_shard;

typedef struct {
    float    kernel_ms;       /* hipEvent time of the traversal launch(es) of the last render */
    uint64_t rays;            /* primary + AO rays traced by the last render                  */
    uint64_t hits;            /* primary hits of the last render                              */
    uint64_t box_tests;       /* ray/box tests (only with VRH_KERNEL_COUNT_TESTS, else 0)     */
    uint64_t prim_tests;      /* ray/primitive tests (only with VRH_KERNEL_COUNT_TESTS)       */
    uint32_t launches;        /* kernel launches in the last render                           */
    uint32_t grid_blocks;
    uint32_t block_threads;
    uint32_t stack_depth;     /* per-lane traversal stack entries used by the variant         */
    uint32_t frames;          /* frames of the last launch (vrh_render_batch)                  */
    /* SIMD utilisation (only with VRH_KERNEL_COUNT_TESTS): wave-level iterations of the refilling
     * loop, lanes busy summed over them, and wave-level iterations of the node-descent and leaf
     * loops (lane-level: box_tests / 2 and prim_tests)                                          */
    uint64_t wave_steps, busy_lane_steps, wave_box_iters, wave_prim_iters;
    uint64_t wave_box_uniform_iters;  /* of wave_box_iters: those whose active lanes all fetch ONE node */
    /* access shape (only with VRH_KERNEL_COUNT_TESTS): over every wave-level vector-memory
     * instruction of the traversal (node pair, primitive and normal loads, output stores), the
     * distinct 128-B lines and the distinct 16-B pieces (merged within a 16-lane quarter) its
     * active lanes touch, and the number of such instructions.  A diagnostic of the lanes'
     * divergence; rocprofv3's TCP_TOTAL_CACHE_ACCESSES counts the hardware's own requests (about
     * 2.2x l1_requests on the AO kernel, profiles/pmc_traffic.json) */
    uint64_t l1_lines, l1_requests, vmem_instrs;
    /* the same instructions under the vector L1's own merging (lanes that want one 16-B piece share
     * an access only inside an aligned group of 4 lanes; tools/micro/l1_roof.hip): l1_group_accesses
     * = the sum over 4-lane groups of the distinct pieces in the group -- the model of
     * TCP_TOTAL_CACHE_ACCESSES -- and l1_ideal_accesses = the sum over distinct pieces of
     * ceil(lanes wanting it / 4), the count if the lanes wanting one piece sat together in groups */
    uint64_t l1_group_accesses, l1_ideal_accesses;
    /* l1_group_accesses by kind: primitives, 4-wide records, binary pair records, AO normals,
     * output stores */
    uint64_t l1_group_by_kind[5];
} vrh_frame_stats;

typedef struct {
    uint32_t num_nodes, num_prims, num_indices, prim_kind;
    uint32_t max_depth;       /* root depth 0; traversal needs <= max_depth stack entries      */
    uint64_t device_bytes;    /* node pairs + leaf-ordered primitives + normals + 4-wide records */
    uint32_t wide_records;    /* 4-wide any-hit records (0: the BVH failed the containment check) */
    uint32_t wide_depth;      /* levels of the 4-wide tree                                      */
    uint32_t max_prim_id;     /* largest prim_id / geom_id of the primitives                    */
    uint32_t max_geom_id;
    uint32_t vertex_normals;  /* per-vertex normals set (vrh_scene_set_vertex_normals)          */
    uint32_t gpu_built;       /* built by vrh_scene_build                                        */
    float    build_ms;        /* vrh_scene_build: device time of the build kernels               */
    uint32_t num_bvhs;        /* BVHs in the scene (> 1: a list, vrh_scene_list_create)          */
} vrh_scene_info;

/* camera::look_at + camera::perspective (camera.inl:10-57) followed by the pinhole basis that
 * simple_sched computes on the host (simple_sched.inl:61-89): f = normalize(eye - center),
 * s = normalize(cross(up, f)), u = cross(f, s), cam_u = s * (tanf(fovy/2) * aspect),
 * cam_v = u * tanf(fovy/2), cam_w = -f.  fovy in radians, aspect = width / height as float. */
VRH_API int vrh_make_camera(const float eye[3], const float center[3], const float up[3], float fovy,
                            float aspect, uint32_t width, uint32_t height, vrh_camera* out);

VRH_API const char* vrh_version(void);
VRH_API const char* vrh_last_error(void);
VRH_API int vrh_device_count(int* count);

/* contexts: one per GPU; hip_stream may be NULL (the context creates its own stream) */
VRH_API int vrh_ctx_create(int hip_device, vrh_ctx** out);
VRH_API int vrh_ctx_create_on_stream(int hip_device, void* hip_stream, vrh_ctx** out);
VRH_API int vrh_ctx_destroy(vrh_ctx* ctx);
/* the context's HIP device and stream (hipStream_t): user kernels (hip_kernels.h) launch on it, so
 * they are ordered with the context's renders, uploads and downloads */
VRH_API int vrh_ctx_get_stream(const vrh_ctx* ctx, int* hip_device, void** hip_stream);

/* launch tuning (per context; 0 = automatic).  Results never depend on these. */
enum vrh_option {
    VRH_OPT_BLOCK_THREADS = 1,   /* threads per block, a multiple of 64 up to 256 (auto: 64)       */
    VRH_OPT_STACK_CAP = 2,       /* traversal stack entries per lane kept in LDS (1..640); entries beyond
                                    them (up to the BVH depth) go to a global overflow block, so
                                    any value is exact.  Primary / AO step loops at their default
                                    register budgets only; other kernels keep the whole stack in
                                    LDS (auto: the depth rounded up to a multiple of 4, lowered in
                                    steps of 4 while LDS rather than registers limits the waves
                                    per CU, and to at most 20 when the BVH is deeper than that) */
    VRH_OPT_AO_SCHEDULE = 3,     /* refilling loop of a wave: 3 = one descend-to-leaf step per
                                    iteration, the only schedule (auto: 3).  Round 1's vote loop,
                                    item-loop AO and two-pass AO were removed (never faster,
                                    profiles/r01/ab*), and in round 2 the primary-visibility item
                                    loop (4, the old sphere default: 6-9 % slower than the step loop,
                                    profiles/r02_ab/ab18_sphere_schedule.log); 4 returns
                                    VRH_ERR_UNSUPPORTED                                             */
    VRH_OPT_BLOCKS_PER_CU = 4,   /* resident blocks per CU for the persistent grid, 1..32 (auto: max) */
    VRH_OPT_WAVES_PER_SIMD = 5,  /* register budget of the unified kernel: 1 (none), 5, 6 or 8 (auto:
                                    AO 6, 5 for test-counting launches and with AO tail sharing;
                                    primary visibility 8 for triangles and for sphere launches of
                                    several frames, 6 for one-frame sphere launches and counting;
                                    pixel-sampler passes and BVH lists AO 5 / primary 6; shading
                                    kernels 1, whitted 5)                                          */
    VRH_OPT_EXACT_MINMAX = 6,    /* 1 = always use the ternary min/max slab test (auto: hardware
                                    min/max where provably identical, see vrh_device.h)           */
    VRH_OPT_XCD_QUEUES = 7,      /* tile queues: 1 = one per XCD (image strips) with stealing,
                                    2 = one global queue, 3 = one per XCD over band-interleaved
                                    (band, frame) units, 4 = one per XCD over image strips in cluster
                                    order (cluster, frame, tile: the frames in flight of a cluster
                                    back to back) (auto: 4 with frames in flight for AO, 3 with frames
                                    in flight for scenes > 256 MB, else 1)                         */
    VRH_OPT_QUAD_REFILL = 24,    /* removed in round 4 (measured slower, profiles/r04/ab/lane_layout/): AO rays
                                    only to fully idle aligned 4-lane groups / 2x2 pixel order;
                                    0 accepted, other values -> VRH_ERR_UNSUPPORTED                */
    VRH_OPT_GROUP_UNITS = 25,    /* removed in round 4 (measured slower): block-shared hand-out of
                                    one tile's frames; 0 accepted, other values -> VRH_ERR_UNSUPPORTED */
    VRH_OPT_CLUSTER_TILES = 23,  /* VRH_OPT_XCD_QUEUES 4: 8x8 tiles per cluster, 1..1024 (auto: 8) */
    VRH_OPT_REFILL_MIN = 8,      /* free lanes (1..64) before finished rays are retired and idle
                                    lanes refilled (auto: AO 24, 28 for scenes above 256 MB)      */
    VRH_OPT_WIDE_ANYHIT = 10,    /* 4-wide node records for any-hit (AO / shadow) rays (step
                                    loop): 1 = on when the BVH passes the containment check, 2 = off
                                    (auto: on for the AO kernel, off for the shading kernels)     */
    VRH_OPT_DESCENT_CAP = 11,    /* step loop: inner visits per step before a lane's descent is
                                    resumed in the next step (1..1024; auto for primary visibility:
                                    6 for spheres, 10 for triangle scenes up to 256 MB, 8 above;
                                    unlimited for AO)                                             */
    VRH_OPT_POP_ON_MISS = 12,    /* step loop: a descent that misses both children pops its stack
                                    and keeps descending in the same step: 1 = on, 2 = off (auto: on) */
    VRH_OPT_COOP_FETCH = 13,     /* removed in round 2 (the cooperative quad fetch measured slower):
                                    0 / 2 accepted, 1 -> VRH_ERR_UNSUPPORTED                     */
    VRH_OPT_SCALAR_FETCH = 14,   /* step loop: a pair record every active lane of a wave wants is
                                    fetched once through the scalar cache: 1 = on, 2 = off (auto: on) */
    VRH_OPT_AO_GATE = 16,        /* AO step loop: a tile's AO rays are handed out only once all its
                                    primaries have finished: 1 = on, 2 = off (auto: on)            */
    VRH_OPT_WAVE_TIMES = 19,     /* 1: the step-loop kernels record every wave's start / end time
                                    (wall_clock64) for vrh_get_wave_times -- a launch-timeline
                                    diagnostic (0 = off, the default); 2: also the tile timeline of
                                    counting one-frame AO launches (vrh_get_tile_times)            */
    VRH_OPT_AO_CUT = 20,         /* AO step loop: any-hit rays start below the top of the 4-wide tree,
                                    at a per-tile cut of at most 8 records whose boxes meet the
                                    tile's AO reach (every hit position +- eps + radius), pushed
                                    so that the entry nearest the tile is popped first: 1 = on,
                                    2 = off, 3 = on with the entries in cut order (auto: on)      */
    VRH_OPT_AO_STEAL = 21,       /* removed in round 3 (the AO tail stash measured slower, DESIGN.md
                                    "Negative results"): 0 / 2 accepted, 1 -> VRH_ERR_UNSUPPORTED  */
    VRH_OPT_AO_SHARE = 22,       /* AO step loop, tail sharing: once the tile queues are dry, a wave's
                                    last tile's AO rays are handed out through an LDS counter that
                                    idle waves of the same block claim from (blocks of 4 waves):
                                    1 = on, 2 = off (auto: off -- measured 2-3 % slower on one-frame
                                    C3 / C4 launches, profiles/r03_ab/ao_share/)                    */
    VRH_OPT_ASYNC_FRAMES = 26,   /* 1: frames are issued like cuda_sched issues them (cuda_sched.inl:306-320,
                                    no synchronisation): they go round robin over the frame lanes of
                                    the context (HIP streams of its own; 2 lanes, or 2..4 given as
                                    the value), so the next frames' waves take the CUs the earlier
                                    frames' launch tails leave idle (changing the lane count first
                                    waits, on the device, for every frame issued so far).
                                    Results are unchanged: a frame into a target that another lane
                                    still writes renders into the lane's scratch target (primary / AO
                                    kernels, one frame, uniform / jittered sampler) and is copied in
                                    issue order, or waits for that lane (every other case); every
                                    entry point that works on the context stream (clears, downloads,
                                    uploads, vrh_sync, vrh_ctx_get_stream, group renders) first waits
                                    for every frame issued so far.  Shard renders stay on the context
                                    stream.  0 = off (the default: frames on the context stream)    */
    VRH_OPT_PAIR_LAYOUT = 15,    /* scene upload (read by vrh_scene_upload): 1 = node pairs in
                                    depth-first preorder, a pair's child-0 pair next to it in one
                                    128-B line; 2 = the builder's order (auto: 2; 1 measured
                                    neutral)                                                      */
};
/* every value is checked against its option's range (the comments above) before it is narrowed:
 * out of range -> VRH_ERR_INVALID, a removed setting -> VRH_ERR_UNSUPPORTED, unknown option ->
 * VRH_ERR_INVALID */
VRH_API int vrh_ctx_set_option(vrh_ctx* ctx, uint32_t option, int64_t value);

/* scene upload: copies the host arrays (reference layouts) into device memory the scene owns.
 * indices may be NULL for a non-index BVH (prims already in leaf order).  face_normals (vec3,
 * 16-B stride, indexed by prim_id) is required for VRH_KERNEL_AO on triangles. */
VRH_API int vrh_scene_upload(vrh_ctx* ctx, const void* nodes, uint32_t num_nodes,
                             const void* prims, uint32_t num_prims, uint32_t prim_kind,
                             const uint32_t* indices, uint32_t num_indices,
                             const void* face_normals, vrh_scene** out);
VRH_API int vrh_scene_get_info(const vrh_scene* scene, vrh_scene_info* info);

/* Device view of BVH `bvh` of a scene (0 for a single BVH; i < num_bvhs for a list) <- the bvh_ref a
 * device BVH hands to kernels (cuda_index_bvh::ref(), bvh.h:344-350, 443-448).  User kernels compiled
 * with hipcc (include/visionaray_hip/hip_kernels.h) traverse it with their own intersectors.  The
 * pointers are device addresses on the scene's context, valid until vrh_scene_free:
 *   pairs : 64-B child-pair records (vrh_device.h layout), prims : leaf-ordered primitives (48-B
 *   triangle / 32-B sphere records with END flags), normals : float4 face normal per prim_id or NULL.
 * root = root link (pair index, or 0x80000000 | first primitive for a one-leaf tree). */
typedef struct {
    const void* pairs;
    const void* prims;
    const void* normals;
    uint32_t root;
    uint32_t max_depth;       /* traversal needs <= max_depth stack entries                     */
    uint32_t prim_kind;       /* vrh_prim_kind                                                   */
    uint32_t finite_bounds;   /* every node bound finite (the hardware min/max slab test is exact) */
    uint32_t num_prims;       /* leaf-ordered primitive records                                  */
    uint32_t quad_depth;      /* levels of the 4-wide records (0: none)                          */
    uint32_t reserved[2];
    const void* quads;        /* 4-wide any-hit records (128 B each, vrh_quad.cpp) of a single-BVH
                                 scene with finite bounds, else NULL: any_hit of a user kernel
                                 descends them (hip_kernels.h walk_quads)                          */
} vrh_scene_view;
VRH_API int vrh_scene_get_view(const vrh_scene* scene, uint32_t bvh, vrh_scene_view* out);

/* A list of BVHs rendered as one scene <- closest_hit / any_hit over [begin, end) of bvh_refs
 * (traverse_linear.inl:76-141, 232-329; the kernels of ao/main.cpp:183 and the viewer pass such a
 * list).  Per ray every BVH is traversed on its own, in list order, with a fresh result and the same
 * max_t, and merged into the running result by update_if(result, hr, is_closer(hr, result, max_t))
 * (strictly closer wins, hit_record.h:54-64); any-hit rays stop at the first BVH with a hit.  The
 * members (single BVHs of one primitive type, same context) are copied into the list, which owns its
 * device memory; the members may be freed afterwards.  face_normals (vec3, 16-B stride, indexed by
 * prim_id, num_normals > every member's largest prim_id) feed AO: the get_normal(normals, hit)
 * array of the kernel.  Primary and AO kernels. */
#define VRH_MAX_SCENE_LIST 8
VRH_API int vrh_scene_list_create(vrh_ctx* ctx, const vrh_scene* const* scenes, uint32_t count,
                                  const void* face_normals, uint32_t num_normals, vrh_scene** out);
VRH_API int vrh_scene_free(vrh_scene* scene);
/* per-vertex normals (vec3, 16-B stride): normals[3 * prim_id + k] for vertex k (v1, v1+e1, v1+e2),
 * the normals_per_vertex_binding array of get_shading_normal.h:64-84 */
VRH_API int vrh_scene_set_vertex_normals(vrh_scene* scene, const void* normals, uint32_t num_normals);

/* materials (plastic, indexed by geom_id) and point lights of VRH_KERNEL_SIMPLE, copied to the
 * device; referenced by vrh_kernel_desc.shading */
VRH_API int vrh_shading_create(vrh_ctx* ctx, const vrh_plastic* materials, uint32_t num_materials,
                               const vrh_point_light* lights, uint32_t num_lights, vrh_shading** out);
VRH_API int vrh_shading_free(vrh_shading* shading);

/* render targets.  vrh_rt_alloc owns its buffers (flags = vrh_rt_flags); vrh_rt_wrap borrows
 * caller device pointers (any may be NULL), e.g. torch tensors used for the RCCL gather. */
VRH_API int vrh_rt_alloc(vrh_ctx* ctx, uint32_t width, uint32_t height, uint32_t flags, vrh_rt** out);
VRH_API int vrh_rt_wrap(vrh_ctx* ctx, uint32_t width, uint32_t height, void* color, uint32_t* prim_id,
                        float* t, uint8_t* occ, vrh_rt** out);
VRH_API int vrh_rt_get_buffers(const vrh_rt* rt, void** color, uint32_t** prim_id, float** t, uint8_t** occ);
VRH_API int vrh_rt_clear(vrh_ctx* ctx, vrh_rt* rt, const float color[4]);
VRH_API int vrh_rt_free(vrh_rt* rt);
/* multi_hit<N> hit lists of a render target: W*H*N prim ids and t, entry [pixel * N + k] is the
 * k-th closest hit (misses: 0xFFFFFFFF / -1) */
VRH_API int vrh_rt_alloc_multi_hit(vrh_ctx* ctx, vrh_rt* rt, uint32_t max_hits);
VRH_API int vrh_rt_download_multi_hit(vrh_ctx* ctx, vrh_rt* rt, uint32_t* prim_ids, float* t);   /* syncs */

/* one frame (asynchronous on the context stream); shard may be NULL (= whole image).
 * frame_num is cuda_sched::frame's frame number (cuda_sched.inl:306-320): the reference reseeds
 * its sampler every frame (cuda_sched.inl:38-45, 79; ao/main.cpp:245 passes ++frame_num).  Here it
 * offsets the deterministic Appendix-A AO sampler: the counter of frame n is
 * ((p*8 + s)*16 + k)*2 + n * 0x9E3779B1 (u32 wrap), so frame 0 is the parity frame and every frame
 * number gives its own AO sample set.  The other built-in kernels draw no random numbers. */
VRH_API int vrh_render(vrh_ctx* ctx, const vrh_scene* scene, vrh_rt* rt, const vrh_camera* cam,
                       const vrh_kernel_desc* kernel, const vrh_shard* shard, uint32_t frame_num);
/* frames in flight: num_frames (1..VRH_MAX_BATCH) frames of one scene and kernel in ONE persistent
 * launch, with frame numbers frame_num, frame_num + 1, ...
 * Frame f renders cams[f] (all of one size) into rows [f * R, (f + 1) * R) of rt, where
 * R = the image height (rt is W x num_frames*H) or, for a packed shard, R = rt height / num_frames.
 * The frames' tiles share the work queues, interleaved tile by tile, so a wave goes on to the next
 * frame's tiles instead of idling while the last tiles of a frame finish; every frame's output is
 * identical to its own vrh_render. */
#define VRH_MAX_BATCH 32
VRH_API int vrh_render_batch(vrh_ctx* ctx, const vrh_scene* scene, vrh_rt* rt, const vrh_camera* cams,
                             uint32_t num_frames, const vrh_kernel_desc* kernel, const vrh_shard* shard,
                             uint32_t frame_num);
VRH_API int vrh_sync(vrh_ctx* ctx);
VRH_API int vrh_last_frame_stats(vrh_ctx* ctx, vrh_frame_stats* stats);   /* syncs */
/* VRH_OPT_WAVE_TIMES: (start, end) clock ticks of every wave of the last launch, 2 * count values
 * into out (capacity values at most); ticks_per_ms = the constant wall clock's rate; syncs */
VRH_API int vrh_get_wave_times(vrh_ctx* ctx, uint64_t* out, uint64_t capacity, uint64_t* count, double* ticks_per_ms);
/* VRH_OPT_WAVE_TIMES = 2: per 8x8 tile of the last counting (VRH_KERNEL_COUNT_TESTS) one-frame AO
 * launch, wall_clock64() at (hand-out, primaries done, pixels written); count = tiles (3 words each) */
VRH_API int vrh_get_tile_times(vrh_ctx* ctx, uint64_t* out, uint64_t capacity, uint64_t* count);

/* Device memory of the context for the user-kernel launches of visionaray_hip/hip_kernels.h: eight
 * tile-queue heads (one per XCD, 64 B apart: VRH_USER_QUEUE_STRIDE words) that the launch zeroes on
 * the context's stream before it starts.  Valid until vrh_ctx_destroy. */
#define VRH_USER_QUEUE_STRIDE 16u
VRH_API int vrh_ctx_user_queues(vrh_ctx* ctx, uint32_t** queues);

/* accumulation over every render since the last vrh_stats_reset (hipEvents per frame, kept in a
 * ring of VRH_MAX_TIMED_FRAMES; frames beyond that are counted in rays/hits but not timed) */
#define VRH_MAX_TIMED_FRAMES 1024
typedef struct {
    uint32_t frames;          /* renders since reset                                      */
    uint32_t timed_frames;    /* renders whose kernel time is in the sums                 */
    double   kernel_ms_total, kernel_ms_min, kernel_ms_max;
    uint64_t rays, hits;
    double   span_ms;         /* first frame's launch start to the last frame's launch end (hipEvents; frames
                                 of overlapping asynchronous launches count once), 0 if not all timed */
} vrh_accum_stats;
VRH_API int vrh_stats_reset(vrh_ctx* ctx);
VRH_API int vrh_get_accum_stats(vrh_ctx* ctx, vrh_accum_stats* out);           /* syncs */

/* Pixel samplers of sched_params (pixel_sampler::*, sched_common.h:160-300 make_primary_rays and
 * :440-720 sample_pixel_impl) for the primary and AO kernels, one frame (`frame_num` as in
 * vrh_render):
 *   UNIFORM        = vrh_render;
 *   JITTERED       the ray through (x + jx, y + jy), colour stored;
 *   JITTERED_BLEND the same ray, colour blended onto the target: c / frame_num + dst (1 - 1 / frame_num)
 *                  (pixel_access.h:1155-1176; the reference AO example's sampler, ao/main.cpp);
 *   SSAA (count 2, 4, 8) the reference's fixed sub-pixel offsets (its 8x table as written, 0.1825
 *                  included): colour 0, then each sample blended with 1 / count, 1, in order.
 * The reference draws the jitter from the scheduler's clock-seeded random_sampler; here the draws of
 * pixel p = y * width + x in frame n are U(c), U(c + 1) with c = p * 2 + 0x632BE5AB + n * 0x68E31DA4
 * and U the Appendix-A hash; jy = U(c) - 0.5, jx = U(c + 1) - 0.5 (the reference's jitter vector takes
 * its two draws in g++'s right-to-left argument order).  The AO samples of every sub-sample are the
 * frame's.  Prim id / t / occ targets hold the last sample's values. */
enum vrh_sampler_kind {
    VRH_SAMPLER_UNIFORM = 0u, VRH_SAMPLER_JITTERED = 1u, VRH_SAMPLER_JITTERED_BLEND = 2u, VRH_SAMPLER_SSAA = 3u
};
typedef struct {
    uint32_t kind;            /* vrh_sampler_kind                                         */
    uint32_t count;           /* VRH_SAMPLER_SSAA: 2, 4 or 8 samples per pixel            */
} vrh_pixel_sampler;
VRH_API int vrh_render_sampled(vrh_ctx* ctx, const vrh_scene* scene, vrh_rt* rt, const vrh_camera* cam,
                               const vrh_kernel_desc* kernel, const vrh_pixel_sampler* sampler, uint32_t frame_num);

/* Camera matrices instead of a pinhole camera: sched_params<Base, MT, RT, PxSamplerT> as
 * make_sched_params(sampler, view_matrix, proj_matrix, rt) builds it (scheduler.h:76-96, :197-212).
 * Both matrices column-major (matrix<4, 4, float>: m[col * 4 + row]).  Their inverses are taken on
 * the host with the reference's cofactor inverse (matrix4.inl:209-244, same float operations), and
 * pixel (x, y) (plus the sampler's offset) gets the ray of sched_common.h:152-176:
 *   u = 2 (x + 0.5) / width - 1, v = 2 (y + 0.5) / height - 1,
 *   o = inv_view (inv_proj (u, v, -1, 1)), d = inv_view (inv_proj (u, v, 1, 1)),
 *   origin = o.xyz / o.w, direction = normalize(d.xyz / d.w - origin).
 * Samplers, frame_num and the scissor box as in vrh_render_sampled / vrh_camera; primary and AO
 * kernels (the others: VRH_ERR_UNSUPPORTED). */
typedef struct {
    float    view[16];        /* view matrix, column-major                                  */
    float    proj[16];        /* projection matrix, column-major                            */
    uint32_t width, height;   /* image size (= the render target's)                         */
    uint32_t scissor[4];      /* x, y, w, h (exclusive edges); all zero: whole image        */
} vrh_view_camera;
VRH_API int vrh_render_view(vrh_ctx* ctx, const vrh_scene* scene, vrh_rt* rt, const vrh_view_camera* cam,
                            const vrh_kernel_desc* kernel, const vrh_pixel_sampler* sampler, uint32_t frame_num);
/* the host inverse vrh_render_view applies (matrix4.inl:209-244 inverse()), for tests */
VRH_API void vrh_matrix_inverse(const float m[16], float out[16]);

/* device -> host copies (any destination may be NULL); synchronous */
VRH_API int vrh_rt_download(vrh_ctx* ctx, vrh_rt* rt, void* color, uint32_t* prim_id, float* t, uint8_t* occ);

/* host -> device copies into a render target (any source may be NULL); synchronous */
VRH_API int vrh_rt_upload(vrh_ctx* ctx, vrh_rt* rt, const void* color, const uint32_t* prim_id, const float* t,
                          const uint8_t* occ);

/* multi-GPU: number of bands shard g of N owns, and the root-side un-interleave of N gathered
 * packed shards into a full target.  Shard g's array starts at base + g * shard_stride_bytes
 * (0 = dense [N][rows][W], rows = VRH_BAND_ROWS * vrh_shard_bands(H, 0, N)) and holds rows x W
 * elements.  gathered_color may be NULL: the colour is then re-derived exactly from the gathered
 * prim ids and AO masks with `kernel` (background on a miss, 1 - k/samples for k occluded samples,
 * ao/main.cpp:234-238; samples <= 8), so 5 B/pixel cross xGMI instead of 20. */
VRH_API uint32_t vrh_shard_bands(uint32_t height, uint32_t index, uint32_t count);
VRH_API int vrh_unshard(vrh_ctx* ctx, uint32_t width, uint32_t height, uint32_t count,
                        const void* gathered_color, const uint32_t* gathered_prim_id,
                        const uint8_t* gathered_occ, uint64_t shard_stride_bytes,
                        const vrh_kernel_desc* kernel, vrh_rt* dst);

/* ---- multi-GPU render groups --------------------------------------------------
 * The image is cut into 8-row bands dealt round-robin to S shards (band b -> shard b % S); shard s
 * is rendered by rank s % N of an N-rank group, packed (vrh_shard.packed), and every shard is
 * gathered to rank 0 over RCCL (ncclSend / ncclRecv, one pair per shard, xGMI point-to-point) and
 * laid back into image order there (vrh_unshard's kernel).  The reference has no multi-GPU path;
 * this lifts tiled_sched's tile distribution (tiled_sched.inl:24-25, 175-224) across devices.
 * A group is one RCCL communicator; a vrh_group is one rank's membership (one context = one GPU):
 *   - one process per GPU: rank 0 calls vrh_group_get_id, hands the id to every rank (any channel,
 *     e.g. torch.distributed / MPI), every rank calls vrh_group_join (collective);
 *   - one process driving every GPU: vrh_group_create_local(ndev, ctxs, out[ndev]).
 * Results are bit-identical to the one-GPU image (the shards partition the pixels; every pixel's
 * arithmetic is unchanged). */
typedef struct vrh_group vrh_group;
typedef struct { char internal[128]; } vrh_group_id;   /* = ncclUniqueId */
VRH_API int vrh_group_get_id(vrh_group_id* id);
VRH_API int vrh_group_join(vrh_ctx* ctx, uint32_t nranks, uint32_t rank, const vrh_group_id* id, vrh_group** out);
/* Failure containment (the first multi-GPU run must fail with an error, not hang):
 * the communicator of a joined group is non-blocking (ncclCommInitRankConfig, blocking = 0).  Every
 * wait on a peer -- the join itself, the enqueue of an exchange or scene broadcast, vrh_group_sync --
 * polls the communicator's state (ncclCommGetAsyncError) and the streams against a deadline of
 * timeout_ms (0: VRH_GROUP_TIMEOUT_MS); on an RCCL error or at the deadline the communicator is
 * aborted (ncclCommAbort), the group is marked failed, and the call returns VRH_ERR_TIMEOUT (or
 * VRH_ERR_HIP for an error) with vrh_last_error set.  Every later call on a failed group returns
 * VRH_ERR_INVALID at once; vrh_group_free releases it without waiting on the peers.  vrh_group_join
 * = vrh_group_join_timeout with timeout_ms 0. */
#define VRH_GROUP_TIMEOUT_MS 120000u
VRH_API int vrh_group_join_timeout(vrh_ctx* ctx, uint32_t nranks, uint32_t rank, const vrh_group_id* id,
                                   uint32_t timeout_ms, vrh_group** out);
/* the deadline of a group's later waits (exchange enqueue, vrh_group_sync, scene broadcast), ms > 0 */
VRH_API int vrh_group_set_timeout(vrh_group* group, uint32_t timeout_ms);
/* 1 if the group failed (aborted after an error or a missed deadline), else 0 */
VRH_API int vrh_group_failed(const vrh_group* group);
VRH_API int vrh_group_create_local(uint32_t ndev, vrh_ctx* const* ctxs, vrh_group** out);
VRH_API int vrh_group_info(const vrh_group* group, uint32_t* nranks, uint32_t* rank);
VRH_API int vrh_group_sync(vrh_group* group);   /* waits for the renders AND the exchange */
VRH_API int vrh_group_free(vrh_group* group);
/* Render num_frames frames (frame numbers frame_num, frame_num + 1, ...) sharded over a group and
 * gather them to rank 0.  groups / scenes / kernels: the n members this caller drives (n = 1 for
 * one process per GPU; every device for vrh_group_create_local), scene i and the kernel's shading /
 * mask objects on group i's context.  Every rank passes the same kernel, fields, cameras, frames
 * and shard count.  dst: rank 0's W x (H * num_frames) target (NULL on the other ranks); fields
 * (vrh_rt_flags) = the buffers assembled there (the same on every rank).  The built-in primary / AO
 * kernels' colour is re-derived on the root (AO samples <= 8): without prim id / AO mask fields
 * one byte per pixel crosses xGMI (0xFF miss, else the number of occluded samples -- the colour
 * depends on nothing else, ao/main.cpp:234-238), with them 4-5 B; shading kernels gather their
 * RGBA32F colour.  shards: S (0 = one per rank;
 * S > N: rank r renders shards r, r + N, ... -- so a one-rank group still runs the whole path).
 * Asynchronous: renders on each context's stream, the exchange and un-interleave on the group's
 * own stream (two staging slots: the next call's renders overlap this call's exchange);
 * vrh_group_sync waits for both. */
/* Scene replication over a group (the scene is broadcast from rank 0 once, instead of
 * every rank building it): rank 0 passes its scene (any kind: uploaded, GPU-built, a list, with
 * vertex normals), the other ranks NULL; out[i] receives, on group i's context, a new scene holding
 * the same device bytes (free it with vrh_scene_free; rank 0's own scene stays its caller's).  One
 * ncclBroadcast per array over the group's communicator (xGMI), after a header with the array
 * sizes.  n / groups as in vrh_render_sharded.  Collective; returns once every replica is complete. */
VRH_API int vrh_group_broadcast_scene(uint32_t n, vrh_group* const* groups, const vrh_scene* root_scene, vrh_scene** out);
VRH_API int vrh_render_sharded(uint32_t n, vrh_group* const* groups, const vrh_scene* const* scenes,
                               const vrh_kernel_desc* kernels, vrh_rt* dst, uint32_t fields,
                               const vrh_camera* cams, uint32_t num_frames, uint32_t frame_num, uint32_t shards);

/* The render-group plan vrh_render_sharded runs, as host functions (no device needed; the same code
 * the group calls -- visionaray_amd/csrc/vrh_plan.h -- so a multi-process test can drive the protocol):
 *   vrh_group_shards_of   : the shards rank `rank` of `nranks` renders, in the order it sends them
 *                           (s = rank, rank + N, ...); returns their count (written up to cap)
 *   vrh_group_shard_owner : the rank the root receives shard s from (it receives s = 0, 1, ... in order)
 *   vrh_group_wire_layout : the bytes of one packed shard of `frames` frames on the wire for a root
 *                           target with buffers `fields` and kernel k (offsets UINT64_MAX: absent)
 *   vrh_shard_packed_rows : image row of every packed row of shard s (-1: padding past the image);
 *                           rows_out holds wire.rows entries
 *   vrh_pack_codes_host   : the one-byte colour code of rendered pixels (0xFF miss, else the number
 *                           of occluded AO samples; occ may be NULL)
 *   vrh_unshard_host      : the root's un-interleave of frame f from S gathered shards (host memory,
 *                           `wire` layout, shard s at gathered + s * wire.shard_bytes) into full-image
 *                           buffers (any may be NULL), colour re-derived as the GPU kernel does */
typedef struct {
    uint64_t prim_id, occ, t, color, code;   /* byte offsets inside a shard (UINT64_MAX: not sent)   */
    uint64_t shard_bytes;                    /* one packed shard, every frame                        */
    uint32_t rows;                           /* packed rows per shard and frame                      */
    uint32_t derive;                         /* the root re-derives the colour (prim ids / codes)    */
} vrh_wire_layout;
VRH_API uint32_t vrh_group_shards_of(uint32_t nranks, uint32_t rank, uint32_t shards, uint32_t* out, uint32_t cap);
VRH_API uint32_t vrh_group_shard_owner(uint32_t nranks, uint32_t shard);
VRH_API int vrh_group_wire_layout(uint32_t fields, const vrh_kernel_desc* k, uint32_t width, uint32_t height,
                                  uint32_t frames, uint32_t shards, vrh_wire_layout* out);
VRH_API int vrh_shard_packed_rows(uint32_t height, uint32_t shard, uint32_t shards, int32_t* rows_out);
VRH_API int vrh_pack_codes_host(const uint32_t* prim_id, const uint8_t* occ, uint8_t* code, uint64_t n);
VRH_API int vrh_unshard_host(const void* gathered, const vrh_wire_layout* wire, uint32_t width, uint32_t height,
                             uint32_t shards, uint32_t frame, uint32_t fields, const vrh_kernel_desc* k,
                             void* color, uint32_t* prim_id, uint8_t* occ, float* t);

/* GPU BVH construction: a linear BVH (Morton order, Karras 2012 hierarchy,
 * leaves of up to max_leaf primitives) built on the device straight into a scene -- no host build,
 * no host re-layout.  The tree differs from build<index_bvh<P>> (binned SAH), so closest-hit ties
 * on shared edges can resolve to another primitive; vrh_bvh_sah_cost measures its quality. */
enum vrh_build_method { VRH_BUILD_LBVH = 0 };
typedef struct {
    uint32_t method;          /* vrh_build_method                                               */
    uint32_t max_leaf;        /* primitives per leaf (1..64; the reference's SAH builder uses 4)  */
} vrh_build_desc;
VRH_API int vrh_scene_build(vrh_ctx* ctx, const void* prims, uint32_t num_prims, uint32_t prim_kind,
                            const void* face_normals, const vrh_build_desc* desc, vrh_scene** out);
/* the scene's tree in the reference layout (bvh_node, index array): nodes_out holds *num_nodes
 * entries on input (NULL: only query the count), indices_out num_prims entries.  Works for
 * uploaded and GPU-built scenes alike. */
VRH_API int vrh_scene_download_bvh(vrh_ctx* ctx, const vrh_scene* scene, void* nodes_out, uint32_t* num_nodes,
                                   uint32_t* indices_out);
/* sah_cost (detail/bvh/statistics.h:30-73): ci * sum A(inner) / A(root) + cl * sum A(leaf) / A(root)
 * + cp * sum A(leaf) * N(leaf) / A(root), in the reference's float arithmetic */
VRH_API int vrh_bvh_sah_cost(const void* nodes, uint32_t num_nodes, float ci, float cl, float cp, float* cost);

/* host binned-SAH builder, tree-identical to build<index_bvh<P>> (build.inl:165-178).
 * nodes_out must hold 2*num_prims nodes (32 B each), indices_out num_prims entries. */
VRH_API int vrh_build_bvh(const void* prims, uint32_t num_prims, uint32_t prim_kind,
                          void* nodes_out, uint32_t* num_nodes_out, uint32_t* indices_out,
                          uint32_t* max_depth_out);

/* Wavefront OBJ input <- load_obj(filename, model&)   obj_loader.cpp:299-527
 * (grammar obj_grammar.cpp:40-77, model model.h:20-49).  The model matches the reference's field by
 * field: triangles in TRI64 layout with prim_id = kept-triangle order and geom_id = last `usemtl`
 * material, degenerate triangles dropped, 3 shading normals / tex coords per triangle whose corners
 * all carry them, geometric normals normalize(cross(e1, e2)), plastic materials from the MTL files
 * (padded with the reference's default material), bbox over v1, v1+e1, v1+e2.  Textures are not
 * loaded (vrh_obj_material_texture gives the map_Kd path).  Errors: unreadable file or a face index
 * outside the data read so far -> VRH_ERR_INVALID (the reference throws / is undefined there). */
typedef struct vrh_obj vrh_obj;
typedef struct {
    uint32_t num_triangles;          /* model::primitives                                        */
    uint32_t num_shading_normals;    /* model::shading_normals (== 3 * num_triangles: per vertex) */
    uint32_t num_tex_coords;         /* model::tex_coords, incl. the reference's dummy padding   */
    uint32_t num_materials;          /* model::materials                                         */
    uint32_t num_degenerate;         /* zero-area triangles rejected (store_triangle :72-80)     */
    uint32_t num_unknown_materials;  /* `usemtl` names not found in any mtllib                   */
    uint32_t num_missing_files;      /* `mtllib` files that do not exist                         */
    uint32_t reserved;
    float bbox_min[3], bbox_max[3];  /* model::bbox (invalid = FLT_MAX / -FLT_MAX when empty)     */
} vrh_obj_info;
VRH_API int vrh_obj_load(const char* filename, vrh_obj** out);
VRH_API int vrh_obj_get_info(const vrh_obj* obj, vrh_obj_info* info);
/* copies out the arrays (NULL pointers skipped): triangles num_triangles TRI64, geometric_normals
 * 4 floats per triangle, shading_normals 4 floats per entry, tex_coords 2 floats per entry,
 * materials num_materials entries */
VRH_API int vrh_obj_get_data(const vrh_obj* obj, void* triangles, float* geometric_normals,
                             float* shading_normals, float* tex_coords, vrh_plastic* materials);
VRH_API const char* vrh_obj_material_name(const vrh_obj* obj, uint32_t index);     /* "" for padding */
VRH_API const char* vrh_obj_material_texture(const vrh_obj* obj, uint32_t index);  /* map_Kd or ""   */
VRH_API int vrh_obj_free(vrh_obj* obj);

/* Mask intersector <- a basic_intersector (intersector.h:24-119) whose
 * operator()(ray, basic_triangle) wraps intersect() and clears hr.hit where a mask over the hit's
 * texture coordinate says so -- the intersector example's mask_intersector
 * (examples/intersector/main.cpp:251-330), with the example's procedural heart test given as data.
 * Per-triangle texture coordinates (3 x vec2 per prim_id, the model's tex_coords layout,
 * get_tex_coord.h:25-38) and a W x H byte mask: a triangle hit at barycentrics (u, v) is kept iff
 *   tc = lerp(tc[3p], tc[3p+1], tc[3p+2], u, v)              (math.h:468-475, operation order kept)
 *   i  = x < W ? u32(x) : W - 1,  x = (tc.x > 0 ? tc.x : 0) * float(W)   (j likewise with H)
 *   mask[j * W + i] != 0.
 * Applied to every triangle hit of every ray of the kernel (closest hit, AO / shadow any hit,
 * multi_hit, the shading kernels), in the leaf test itself -- no extra pass, no indirect call.
 * Spheres are not masked.  Kernels with a mask run the step-loop schedule. */
VRH_API int vrh_hit_mask_create(vrh_ctx* ctx, const float* tex_coords, uint32_t num_tex_coords,
                                const uint8_t* mask, uint32_t mask_width, uint32_t mask_height,
                                vrh_hit_mask** out);
VRH_API int vrh_hit_mask_free(vrh_hit_mask* mask);

/* synthetic scenes of SURVEY.md Appendix A (bench / test inputs) */
VRH_API int vrh_gen_heightfield(uint32_t grid, void* tris_out);        /* 2*grid*grid TRI64   */
VRH_API int vrh_gen_cornell(void* tris_out);                           /* 12 TRI64            */
VRH_API int vrh_gen_spheres(uint32_t n, void* spheres_out);            /* n SPHERE48          */
VRH_API int vrh_face_normals(const void* tris, uint32_t n, float* normals_out); /* 4 floats each */

#ifdef __cplusplus
}
#endif
#endif /* VRH_H */
