/*
 * oracle/vrh_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference hot path (Visionaray v0.1.0), used exclusively as the
 * parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
 * (visionaray_amd/, include/vrh.h) never links, loads or calls anything in oracle/.
 *
 * Pinned against the reference itself: oracle/_ref/vsnray_ref (built by oracle/Makefile from the
 * reference headers where they lie) emits BVHs, per-pixel prim_id / t / AO masks and hashes; the
 * committed fixtures in tests/golden/ carry those results to the GPU box.
 *
 * All binary layouts are the reference's:
 *   vo_tri    64 B : geom_id@0 prim_id@4 v1@16 e1@32 e2@48      (basic_triangle<3,float>)
 *   vo_sphere 48 B : geom_id@0 prim_id@4 center@16 radius@32     (basic_sphere<float>)
 *   vo_node   32 B : bbox_min[3] first_child|first_prim bbox_max[3] num_prims   (bvh.h:52-119)
 */
#ifndef VRH_ORACLE_H
#define VRH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z, pad; } vo_vec3;                         /* vector<3,float>, 16 B */
typedef struct { uint32_t geom_id, prim_id, pad0, pad1; vo_vec3 v1, e1, e2; } vo_tri;
typedef struct { uint32_t geom_id, prim_id, pad0, pad1; vo_vec3 center; float radius, pad2, pad3, pad4; } vo_sphere;
typedef struct { float bmin[3]; uint32_t first; float bmax[3]; uint32_t num_prims; } vo_node;

enum { VO_TRI = 0, VO_SPHERE = 1 };
enum { VO_MODE_PRIMARY = 0, VO_MODE_AO = 1, VO_MODE_SIMPLE = 2, VO_MODE_MULTI_HIT = 3, VO_MODE_WHITTED = 4 };
enum { VO_MAX_HITS = 16 };
enum { VO_NORMALS_PER_FACE = 0, VO_NORMALS_PER_VERTEX = 1 };

/* plastic<float> (material.h:267-323, detail/material/plastic.inl): ambient ca*ka, lambertian
 * diffuse cd*kd, blinn specular cs*ks with exponent exp */
typedef struct { float ca[3]; float ka; float cd[3]; float kd; float cs[3]; float ks; float exp; } vo_plastic;
/* point_light<float> (point_light.h, detail/point_light.inl) */
typedef struct { float position[3]; float cl[3]; float kl; float constant_att, linear_att, quadratic_att; } vo_point_light;

/* ---- synthetic scenes, SURVEY.md Appendix A ---- */
uint32_t vo_wang(uint32_t a);
float    vo_uniform(uint32_t k);
size_t   vo_gen_cornell(vo_tri* out);                                  /* 12 tris */
void     vo_gen_heightfield(int grid, vo_tri* out);                    /* 2*grid*grid tris */
void     vo_gen_spheres(int n, vo_sphere* out);
void     vo_face_normals(const vo_tri* tris, size_t n, vo_vec3* out);  /* normalize(cross(e1,e2)) */

/* ---- binned SAH builder (build.inl:28-178, sah.h:150-763), tree-identical to the reference ---- */
typedef struct {
    vo_node*  nodes;   size_t num_nodes;
    uint32_t* indices; size_t num_indices;
    unsigned  max_depth;
} vo_bvh;
int  vo_build(const void* prims, size_t n, int kind, vo_bvh* out);    /* 0 = ok */
void vo_bvh_free(vo_bvh* b);

/* ---- camera basis, simple_sched.inl:61-89 (tanf from the host libm) ---- */
void vo_camera_basis(const float eye[3], const float center[3], const float up[3],
                     float fovy, float aspect, float out_u[3], float out_v[3], float out_w[3]);

/* ---- traversal: one ray against one index BVH (detail/bvh/intersect.inl:25-134) ---- */
typedef struct {
    int      hit;
    uint32_t prim_id, geom_id, list_index;
    float    t, u, v;
} vo_hit;
typedef struct { uint64_t box_tests, prim_tests; } vo_counters;

vo_hit vo_intersect(const float ori[3], const float dir[3], const vo_node* nodes, const uint32_t* indices,
                    const void* prims, int kind, int any_hit, float max_t, vo_counters* cnt);

/* the intersector example's mask_intersector (examples/intersector/main.cpp:251-330) as data, the
 * product's vrh_hit_mask: a triangle hit keeps hr.hit iff mask[j * w + i] != 0 at the texel of
 * tc = lerp(tc[3p], tc[3p+1], tc[3p+2], u, v) (math.h:468-475), i = x < w ? (u32)x : w - 1 with
 * x = (tc.x > 0 ? tc.x : 0) * (float)w, j likewise */
typedef struct { const float* tc; const uint8_t* mask; int w, h; } vo_hit_mask;
vo_hit vo_intersect_masked(const float ori[3], const float dir[3], const vo_node* nodes, const uint32_t* indices,
                           const void* prims, int kind, int any_hit, float max_t, const vo_hit_mask* mask,
                           vo_counters* cnt);

/* multi_hit<N> (traverse_linear.inl:333-380 -> intersect<MultiHit, N>, detail/multi_hit.h): the N
 * closest hits sorted by t (insert_sorted, algorithm.h:46-75: ties after the existing ones);
 * boxes and primitives are tested against the N-th kept t.  out[N]; returns the hit count. */
int vo_intersect_multi(const float ori[3], const float dir[3], const vo_node* nodes, const uint32_t* indices,
                       const void* prims, int kind, int n, vo_hit* out, vo_counters* cnt);
int vo_intersect_multi_masked(const float ori[3], const float dir[3], const vo_node* nodes, const uint32_t* indices,
                              const void* prims, int kind, int n, vo_hit* out, const vo_hit_mask* mask,
                              vo_counters* cnt);

/* ---- a frame, simple_sched order (row-major), over rows [y0, y1) ---- */
typedef struct vo_scene vo_scene;
struct vo_scene {
    const vo_node* nodes; const uint32_t* indices; const void* prims; int kind;
    const vo_vec3* normals;               /* per prim_id (AO; simple kernel, per-face binding) */
    const vo_vec3* vertex_normals;        /* 3 per prim_id (simple kernel, per-vertex binding) */
    const vo_hit_mask* hit_mask;          /* mask intersector for every ray (NULL: none) */
    /* BVH-ref list (traverse_linear.inl:76-141): the next BVH of the list (NULL: last).  Primary /
     * AO rays traverse every BVH on its own and merge with update_if(result, hr, is_closer(hr,
     * result, max_t)); any hit stops at the first BVH with a hit.  normals / vertex_normals /
     * hit_mask are the first entry's. */
    const vo_scene* next;
};
typedef struct {
    float eye[3], cam_u[3], cam_v[3], cam_w[3];
    int   width, height;
    /* scissor box as cuda_sched reads it (cuda_sched.inl:71): pixels x0 <= x < x1, y0 <= y < y1 are
     * rendered, the others not written; all zero = whole image */
    unsigned scissor[4];
    /* the camera as matrices (sched_params with view / projection matrices, scheduler.h:77-95): the
     * inverses (column-major 4x4, vo_inverse4); NULL = the pinhole basis above */
    const float* inv_view;
    const float* inv_proj;
} vo_camera;
/* matrix4.inl:209-244 inverse of a column-major 4x4 matrix, the reference's cofactor formula */
void vo_inverse4(const float m[16], float out[16]);
typedef struct {
    int   mode;                           /* VO_MODE_PRIMARY | VO_MODE_AO | VO_MODE_SIMPLE */
    int   samples;                        /* AO samples (8) */
    float radius;                         /* AO radius (0.1) */
    float eps;                            /* AO origin offset (1e-3) */
    float bg[4];                          /* miss colour */
    /* simple::kernel (detail/simple.inl:19-83) */
    const vo_plastic* materials; int num_materials;       /* indexed by geom_id */
    const vo_point_light* lights; int num_lights;
    float ambient[4];
    int   normal_binding;                 /* VO_NORMALS_PER_FACE | VO_NORMALS_PER_VERTEX */
    int   max_hits;                       /* VO_MODE_MULTI_HIT: N (<= VO_MAX_HITS) */
    int   num_bounces;                    /* VO_MODE_WHITTED (eps = scene epsilon) */
    /* frame number (cuda_sched::frame's frame_num): the AO sampler counter of frame n is
     * ((p*8 + s)*16 + k)*2 + n * 0x9E3779B1 (u32 wrap); frame 0 = SURVEY.md Appendix A */
    uint32_t frame_num;
} vo_kernel;

/* deterministic per-vertex normals for tests: prim k, vertex j: normalize(n_k + 0.4 * (U(b) - 0.5,
 * U(b+1) - 0.5, U(b+2) - 0.5)) with b = (3k + j) * 3 and n_k the face normal */
void vo_vertex_normals(const vo_vec3* face_normals, size_t n, vo_vec3* out);

/* Any output pointer may be NULL.  Arrays are full-image sized (W*H), indexed y*W+x.
 * threads <= 0: all cores (OpenMP).  Returns rays traced (primary + AO) over the rows. */
uint64_t vo_render_rows(const vo_scene* s, const vo_camera* cam, const vo_kernel* k, int y0, int y1,
                        float* color, uint32_t* prim_id, float* t, uint8_t* occ, uint32_t* list_index,
                        int threads, vo_counters* cnt);

/* VO_MODE_MULTI_HIT frame: per pixel the hit list (mh_prim_id / mh_t: W*H*max_hits, misses
 * 0xFFFFFFFF / -1) and the colour of examples/multi_hit/main.cpp:166-235 (front-to-back
 * compositing of plastic::shade with the first light, alpha 0.3). */
uint64_t vo_render_multi(const vo_scene* s, const vo_camera* cam, const vo_kernel* k, float* color,
                         uint32_t* mh_prim_id, float* mh_t, int threads);

/* Same, for an explicit list of pixel indices (p = y*W + x); outputs are indexed by list position. */
/* pixel samplers: VO_SAMPLER_* kind, count = ssaa samples (2, 4, 8); color is read (blend) and
 * written for the whole image, prim_id = the last sample's hit.  Returns 0, -1 for a bad count. */
enum { VO_SAMPLER_UNIFORM = 0, VO_SAMPLER_JITTERED = 1, VO_SAMPLER_JITTERED_BLEND = 2, VO_SAMPLER_SSAA = 3 };
void vo_sampler_offsets(int kind, int count, unsigned x, unsigned y, unsigned width, uint32_t frame_num,
                        int sub, float* ox, float* oy);
int vo_render_sampled(const vo_scene* s, const vo_camera* cam, const vo_kernel* k, int kind, int count,
                      float* color, uint32_t* prim_id, float* t, int threads);
uint64_t vo_render_pixels(const vo_scene* s, const vo_camera* cam, const vo_kernel* k,
                          const uint32_t* pixels, size_t npix,
                          float* color, uint32_t* prim_id, float* t, uint8_t* occ, int threads);

/* FNV-1a 64 over bytes (hash convention used by tests/golden) */
uint64_t vo_fnv1a(const void* data, size_t n, uint64_t h);

#ifdef __cplusplus
}
#endif
#endif
