/*
 * oracle/vrh_oracle.c -- TEST INFRASTRUCTURE ONLY (see vrh_oracle.h).
 *
 * Plain-C restatement of the reference algorithm for the hot path.  Compiled with
 * -O2 -ffp-contract=off (no FMA contraction: SURVEY.md §7 hard part 1), float arithmetic in
 * exactly the reference's operation order.  Every function cites the reference file:line it
 * restates.  Parity of this file against the reference is checked by tests/test_oracle.py
 * (against oracle/_ref/vsnray_ref when built, and against the committed tests/golden fixtures).
 */
#include "vrh_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------ */
/* math/detail/math.h:48-60  min(x,y) = x<y?x:y, max(x,y) = x<y?y:x  (NaN follows the ternary)   */
static inline float fmin_ref(float x, float y) { return x < y ? x : y; }
static inline float fmax_ref(float x, float y) { return x < y ? y : x; }

typedef struct { float x, y, z; } v3;
static inline v3 mk(float x, float y, float z) { v3 r = { x, y, z }; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 smul(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
/* vector3.inl:291-301 */
static inline v3 cross(v3 u, v3 v) { return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x); }
/* vector3.inl:303-307  (x*x + y*y) + z*z */
static inline float dot(v3 u, v3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
/* vector3.inl:331-336 + math.h:477-481  v * (1/sqrt(dot(v,v))) */
static inline v3 normalize(v3 v) { return muls(v, 1.0f / sqrtf(dot(v, v))); }
static inline v3 ld(const vo_vec3* p) { return mk(p->x, p->y, p->z); }
static inline void st(vo_vec3* p, v3 v) { p->x = v.x; p->y = v.y; p->z = v.z; p->pad = 0.0f; }
static inline float comp(v3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

/* ------------------------------------------------------------------------------------------ */
/* SURVEY.md Appendix A                                                                        */
uint32_t vo_wang(uint32_t a)
{
    a = (a ^ 61u) ^ (a >> 16);
    a = a + (a << 3);
    a = a ^ (a >> 4);
    a = a * 0x27d4eb2du;
    a = a ^ (a >> 15);
    return a;
}

float vo_uniform(uint32_t k) { return (float)(vo_wang(k) >> 8) * (1.0f / 16777216.0f); }

static void set_tri(vo_tri* t, v3 a, v3 b, v3 c, uint32_t prim_id)
{
    memset(t, 0, sizeof(*t));
    t->geom_id = 0;
    t->prim_id = prim_id;
    st(&t->v1, a);
    st(&t->e1, sub(b, a));
    st(&t->e2, sub(c, a));
}

size_t vo_gen_cornell(vo_tri* out)
{
    static const float q[6][4][3] = {
        {{-1,-1,-1},{ 1,-1,-1},{ 1,-1, 1},{-1,-1, 1}},
        {{-1, 1,-1},{-1, 1, 1},{ 1, 1, 1},{ 1, 1,-1}},
        {{-1,-1,-1},{-1, 1,-1},{ 1, 1,-1},{ 1,-1,-1}},
        {{-1,-1,-1},{-1,-1, 1},{-1, 1, 1},{-1, 1,-1}},
        {{ 1,-1,-1},{ 1, 1,-1},{ 1, 1, 1},{ 1,-1, 1}},
        {{-.25f,.99f,-.25f},{-.25f,.99f,.25f},{.25f,.99f,.25f},{.25f,.99f,-.25f}},
    };
    size_t n = 0;
    for (int f = 0; f < 6; ++f) {
        v3 a = mk(q[f][0][0], q[f][0][1], q[f][0][2]);
        v3 b = mk(q[f][1][0], q[f][1][1], q[f][1][2]);
        v3 c = mk(q[f][2][0], q[f][2][1], q[f][2][2]);
        v3 d = mk(q[f][3][0], q[f][3][1], q[f][3][2]);
        set_tri(&out[n], a, b, c, (uint32_t)n); ++n;
        set_tri(&out[n], a, c, d, (uint32_t)n); ++n;
    }
    return n;
}

static v3 hf_vertex(int grid, int i, int j)
{
    float x = -1.0f + 2.0f * (float)i / (float)grid;
    float z = -1.0f + 2.0f * (float)j / (float)grid;
    uint32_t k = (uint32_t)j * (uint32_t)(grid + 1) + (uint32_t)i;
    float y = 0.3f * x * z * (1.0f - x * x) * (1.0f - z * z) + 0.004f * (vo_uniform(k) - 0.5f);
    return mk(x, y, z);
}

void vo_gen_heightfield(int grid, vo_tri* out)
{
    #pragma omp parallel for schedule(static)
    for (int j = 0; j < grid; ++j) {
        for (int i = 0; i < grid; ++i) {
            v3 a = hf_vertex(grid, i, j), b = hf_vertex(grid, i + 1, j);
            v3 c = hf_vertex(grid, i + 1, j + 1), e = hf_vertex(grid, i, j + 1);
            size_t base = (size_t)2 * ((size_t)j * grid + i);
            set_tri(&out[base], a, b, c, (uint32_t)base);
            set_tri(&out[base + 1], a, c, e, (uint32_t)(base + 1));
        }
    }
}

void vo_gen_spheres(int n, vo_sphere* out)
{
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        uint32_t k = 6u * (uint32_t)i;
        vo_sphere* s = &out[i];
        memset(s, 0, sizeof(*s));
        st(&s->center, mk(2.0f * vo_uniform(k) - 1.0f, 2.0f * vo_uniform(k + 1) - 1.0f, 2.0f * vo_uniform(k + 2) - 1.0f));
        s->radius = 0.002f + 0.008f * vo_uniform(k + 3);
        s->prim_id = (uint32_t)i;
        s->geom_id = 0;
    }
}

void vo_face_normals(const vo_tri* tris, size_t n, vo_vec3* out)
{
    #pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)n; ++i)
        st(&out[i], normalize(cross(ld(&tris[i].e1), ld(&tris[i].e2))));
}

/* ------------------------------------------------------------------------------------------ */
/* Builder: build.inl:28-178, sah.h:150-763, math/detail/aabb.inl                              */
typedef struct { v3 mn, mx; } box;

static inline void box_invalidate(box* b)            /* aabb.inl invalidate: max() / lowest() */
{
    b->mn = mk(FLT_MAX, FLT_MAX, FLT_MAX);
    b->mx = mk(-FLT_MAX, -FLT_MAX, -FLT_MAX);
}
static inline void box_insert_v(box* b, v3 v)        /* aabb.inl insert(vec) */
{
    b->mn = mk(fmin_ref(b->mn.x, v.x), fmin_ref(b->mn.y, v.y), fmin_ref(b->mn.z, v.z));
    b->mx = mk(fmax_ref(b->mx.x, v.x), fmax_ref(b->mx.y, v.y), fmax_ref(b->mx.z, v.z));
}
static inline void box_insert_b(box* b, const box* o) /* aabb.inl insert(aabb) */
{
    b->mn = mk(fmin_ref(b->mn.x, o->mn.x), fmin_ref(b->mn.y, o->mn.y), fmin_ref(b->mn.z, o->mn.z));
    b->mx = mk(fmax_ref(b->mx.x, o->mx.x), fmax_ref(b->mx.y, o->mx.y), fmax_ref(b->mx.z, o->mx.z));
}
static inline v3 box_center(const box* b) { return muls(add(b->mx, b->mn), 0.5f); }
static inline v3 box_size(const box* b) { return sub(b->mx, b->mn); }
static inline float safe_hsa(const box* b)           /* aabb.inl safe_half_surface_area */
{
    v3 s = sub(b->mx, b->mn);
    s.x = fmax_ref(0.0f, s.x); s.y = fmax_ref(0.0f, s.y); s.z = fmax_ref(0.0f, s.z);
    return s.x * s.y + s.y * s.z + s.z * s.x;
}

typedef struct { box bounds; int index; } prim_ref;  /* sah.h:155-167 */
typedef struct { box prim_bounds, cent_bounds; int enter, leave; } bin; /* sah.h:193-220 */
typedef struct { box prim_bounds, cent_bounds; int first; } leaf_info;  /* sah.h:270-275 */
enum { NUM_BINS = 16 };

typedef struct {
    prim_ref* refs; size_t nrefs;
    vo_node* nodes; size_t nn, cap_n;
    uint32_t* indices; size_t ni;
    unsigned max_depth;
} builder;

static void bin_merge(bin* lhs, const bin* rhs)      /* sah.h:211-219 */
{
    box_insert_b(&lhs->prim_bounds, &rhs->prim_bounds);
    box_insert_b(&lhs->cent_bounds, &rhs->cent_bounds);
    lhs->enter += rhs->enter;
    lhs->leave += rhs->leave;
}

static void set_node(vo_node* n, const box* b, uint32_t first, uint32_t count)
{
    n->bmin[0] = b->mn.x; n->bmin[1] = b->mn.y; n->bmin[2] = b->mn.z;
    n->bmax[0] = b->mx.x; n->bmax[1] = b->mx.y; n->bmax[2] = b->mx.z;
    n->first = first; n->num_prims = count;
}

static size_t push_node(builder* B)
{
    if (B->nn == B->cap_n) {
        B->cap_n = B->cap_n ? B->cap_n * 2 : 64;
        B->nodes = (vo_node*)realloc(B->nodes, B->cap_n * sizeof(vo_node));
    }
    memset(&B->nodes[B->nn], 0, sizeof(vo_node));
    return B->nn++;
}

/* sah.h:678-762 (object split only: no spatial splits in any config) */
static int sah_split(builder* B, leaf_info childs[2], const leaf_info* leaf, int max_leaf_size)
{
    int leaf_size = (int)(B->nrefs - (size_t)leaf->first);
    if (leaf_size <= max_leaf_size) return 0;

    v3 size = box_size(&leaf->cent_bounds);
    /* vector.inl:811-821 max_index */
    int axis = comp(size, 1) < comp(size, 0) ? 0 : 1;
    axis = comp(size, 2) < comp(size, axis) ? axis : 2;
    if (comp(size, axis) <= 0.0f) return 0;

    /* sah.h:224-268 projection */
    float k0 = comp(leaf->cent_bounds.mn, axis);
    float k1 = (float)NUM_BINS / (comp(leaf->cent_bounds.mx, axis) - k0);

    /* sah.h:387-402 find_object_split */
    bin bins[NUM_BINS];
    for (int i = 0; i < NUM_BINS; ++i) {
        box_invalidate(&bins[i].prim_bounds); box_invalidate(&bins[i].cent_bounds);
        bins[i].enter = bins[i].leave = 0;
    }
    for (size_t r = (size_t)leaf->first; r < B->nrefs; ++r) {
        v3 cen = box_center(&B->refs[r].bounds);
        int bi = (int)(k1 * (comp(cen, axis) - k0));
        if (bi < 0) bi = 0;
        if (bi > NUM_BINS - 1) bi = NUM_BINS - 1;
        bin* b = &bins[bi];
        box_insert_b(&b->prim_bounds, &B->refs[r].bounds);
        box_insert_v(&b->cent_bounds, cen);
        b->enter++; b->leave++;
    }

    /* sah.h:308-367 find_split */
    float hsa_parent = safe_hsa(&leaf->prim_bounds);
    float best_cost = FLT_MAX;
    int best_index = -1;
    bin acc_l[NUM_BINS], acc_r[NUM_BINS];
    acc_l[0] = bins[0];
    for (int i = 1; i < NUM_BINS; ++i) { acc_l[i] = acc_l[i - 1]; bin_merge(&acc_l[i], &bins[i]); }
    acc_r[NUM_BINS - 1] = bins[NUM_BINS - 1];
    for (int i = NUM_BINS - 1; i > 0; --i) {
        acc_r[i - 1] = acc_r[i]; bin_merge(&acc_r[i - 1], &bins[i - 1]);
        const bin* L = &acc_l[i - 1];
        const bin* R = &acc_r[i];
        /* sah.h:279-292 compute_split_cost */
        float cost = 1.0f + (safe_hsa(&L->prim_bounds) / hsa_parent) * (3.0f * (float)L->enter)
                          + (safe_hsa(&R->prim_bounds) / hsa_parent) * (3.0f * (float)R->leave);
        if (cost < best_cost) { best_cost = cost; best_index = i; }
    }
    if (best_index <= 0) return 0; /* unreachable for finite input (reference asserts) */

    /* sah.h:742-747 leaf cost check */
    if (best_cost > 3.0f * (float)leaf_size) return 0;

    const bin* L = &acc_l[best_index - 1];
    const bin* R = &acc_r[best_index];

    /* sah.h:405-424 perform_object_partition, std::partition = libstdc++ bidirectional
     * __partition (stl_algo.h): Hoare-style swaps from both ends */
    childs[0].prim_bounds = L->prim_bounds; childs[0].cent_bounds = L->cent_bounds;
    childs[1].prim_bounds = R->prim_bounds; childs[1].cent_bounds = R->cent_bounds;
    prim_ref* first = B->refs + leaf->first;
    prim_ref* last = B->refs + B->nrefs;
#define PRED(pr) ((int)(k1 * (comp(box_center(&(pr)->bounds), axis) - k0)) < best_index)
    for (;;) {
        for (;;) {
            if (first == last) goto done;
            else if (PRED(first)) ++first;
            else break;
        }
        --last;
        for (;;) {
            if (first == last) goto done;
            else if (!PRED(last)) --last;
            else break;
        }
        { prim_ref tmp = *first; *first = *last; *last = tmp; }
        ++first;
    }
#undef PRED
done:
    childs[0].first = leaf->first;
    childs[1].first = (int)(first - B->refs);
    return 1;
}

/* build.inl:28-81 build_tree_impl: children allocated as an adjacent pair, right subtree first */
static void build_rec(builder* B, size_t index, const leaf_info* leaf, int max_leaf_size, unsigned depth)
{
    if (depth > B->max_depth) B->max_depth = depth;
    leaf_info childs[2];
    if (sah_split(B, childs, leaf, max_leaf_size)) {
        size_t first_child = B->nn;
        set_node(&B->nodes[index], &leaf->prim_bounds, (uint32_t)first_child, 0);
        push_node(B); push_node(B);
        build_rec(B, first_child + 1, &childs[1], max_leaf_size, depth + 1);
        build_rec(B, first_child + 0, &childs[0], max_leaf_size, depth + 1);
    } else {
        /* sah.h:657-672 insert_indices */
        uint32_t first = (uint32_t)B->ni;
        uint32_t count = (uint32_t)(B->nrefs - (size_t)leaf->first);
        for (size_t r = (size_t)leaf->first; r < B->nrefs; ++r) B->indices[B->ni++] = (uint32_t)B->refs[r].index;
        B->nrefs = (size_t)leaf->first;
        set_node(&B->nodes[index], &leaf->prim_bounds, first, count);
    }
}

static box prim_bounds(const void* prims, int kind, size_t i)
{
    box b;
    box_invalidate(&b);
    if (kind == VO_TRI) {                  /* triangle.inl:34-44 */
        const vo_tri* t = (const vo_tri*)prims + i;
        v3 v1 = ld(&t->v1);
        box_insert_v(&b, v1);
        box_insert_v(&b, add(v1, ld(&t->e1)));
        box_insert_v(&b, add(v1, ld(&t->e2)));
    } else {                               /* sphere.inl:29-38: center -/+ radius */
        const vo_sphere* s = (const vo_sphere*)prims + i;
        v3 c = ld(&s->center);
        float r = s->radius;
        box_insert_v(&b, mk(c.x - r, c.y - r, c.z - r));
        box_insert_v(&b, mk(c.x + r, c.y + r, c.z + r));
    }
    return b;
}

int vo_build(const void* prims, size_t n, int kind, vo_bvh* out)
{
    memset(out, 0, sizeof(*out));
    if (n == 0) return 1;
    builder B;
    memset(&B, 0, sizeof(B));
    B.refs = (prim_ref*)malloc(n * sizeof(prim_ref));
    B.indices = (uint32_t*)malloc(n * sizeof(uint32_t));
    B.nrefs = n;
    /* sah.h:171-186 init + sah.h:643-654 */
    leaf_info root;
    box_invalidate(&root.prim_bounds);
    box_invalidate(&root.cent_bounds);
    root.first = 0;
    for (size_t i = 0; i < n; ++i) {
        B.refs[i].bounds = prim_bounds(prims, kind, i);
        B.refs[i].index = (int)i;
        box_insert_b(&root.prim_bounds, &B.refs[i].bounds);
        box_insert_v(&root.cent_bounds, box_center(&B.refs[i].bounds));
    }
    B.cap_n = 2 * (n / 4) + 64;
    B.nodes = (vo_node*)malloc(B.cap_n * sizeof(vo_node));
    push_node(&B);                        /* build.inl:156 root node */
    build_rec(&B, 0, &root, 4, 0);        /* build.inl:137-140 max_leaf_size = 4 */
    free(B.refs);
    out->nodes = B.nodes; out->num_nodes = B.nn;
    out->indices = B.indices; out->num_indices = B.ni;
    out->max_depth = B.max_depth;
    return 0;
}

void vo_bvh_free(vo_bvh* b)
{
    free(b->nodes); free(b->indices);
    memset(b, 0, sizeof(*b));
}

/* ------------------------------------------------------------------------------------------ */
/* simple_sched.inl:61-89 camera basis                                                         */
void vo_camera_basis(const float eye[3], const float center[3], const float up[3],
                     float fovy, float aspect, float ou[3], float ov[3], float ow[3])
{
    v3 e = mk(eye[0], eye[1], eye[2]), c = mk(center[0], center[1], center[2]), u0 = mk(up[0], up[1], up[2]);
    v3 f = normalize(sub(e, c));
    v3 s = normalize(cross(u0, f));
    v3 u = cross(f, s);
    float th = tanf(fovy / 2.0f);
    v3 cu = muls(s, th * aspect);
    v3 cv = muls(u, th);
    v3 cw = mk(-f.x, -f.y, -f.z);
    ou[0] = cu.x; ou[1] = cu.y; ou[2] = cu.z;
    ov[0] = cv.x; ov[1] = cv.y; ov[2] = cv.z;
    ow[0] = cw.x; ow[1] = cw.y; ow[2] = cw.z;
}

/* ------------------------------------------------------------------------------------------ */
/* Traversal                                                                                   */
typedef struct { int hit; float t, u, v; uint32_t prim_id, geom_id; } prim_hit;

/* math/intersect.h:122-179 ray/triangle (Moller-Trumbore, two-sided) */
static inline prim_hit isect_tri(v3 ori, v3 dir, const vo_tri* tri)
{
    prim_hit r; r.hit = 0; r.t = -1.0f; r.u = 0.0f; r.v = 0.0f; r.prim_id = 0; r.geom_id = 0;
    v3 v1 = ld(&tri->v1), e1 = ld(&tri->e1), e2 = ld(&tri->e2);
    v3 s1 = cross(dir, e2);
    float div = dot(s1, e1);
    if (!(div != 0.0f)) return r;
    float inv_div = 1.0f / div;
    v3 d = sub(ori, v1);
    float b1 = dot(d, s1) * inv_div;
    if (!(b1 >= 0.0f && b1 <= 1.0f)) return r;
    v3 s2 = cross(d, e1);
    float b2 = dot(dir, s2) * inv_div;
    if (!(b2 >= 0.0f && b1 + b2 <= 1.0f)) return r;
    r.hit = 1;
    r.prim_id = tri->prim_id; r.geom_id = tri->geom_id;
    r.t = dot(e2, s2) * inv_div;
    r.u = b1; r.v = b2;
    return r;
}

/* math/intersect.h:186-221 ray/sphere */
static inline prim_hit isect_sphere(v3 ori, v3 dir, const vo_sphere* s)
{
    prim_hit r; r.u = 0.0f; r.v = 0.0f;
    v3 o = sub(ori, ld(&s->center));
    float A = dot(dir, dir);
    float B = dot(dir, o) * 2.0f;
    float C = dot(o, o) - s->radius * s->radius;
    float disc = B * B - 4.0f * A * C;
    int valid = disc >= 0.0f;
    float root_disc = valid ? sqrtf(disc) : disc;
    float q = B < 0.0f ? -0.5f * (B - root_disc) : -0.5f * (B + root_disc);
    float t1 = q / A;
    float t2 = C / q;
    r.hit = valid;
    r.prim_id = s->prim_id; r.geom_id = s->geom_id;
    r.t = valid ? (t1 > t2 ? t2 : t1) : -1.0f;
    return r;
}

/* the example's mask test on a triangle hit (vrh_oracle.h vo_hit_mask); hr.hit &= mask */
static inline unsigned mask_texel(float c, int n)
{
    float x = (c > 0.0f ? c : 0.0f) * (float)n;
    return x < (float)n ? (unsigned)x : (unsigned)(n - 1);
}

static inline int mask_keep(const vo_hit_mask* m, uint32_t prim_id, float u, float v)
{
    const float* a = m->tc + 6u * prim_id;       /* 3 x (x, y) per prim_id */
    /* lerp(a, b, c, u, v), math.h:468-475: s2 = c * v; s3 = b * u; s1 = a * (1 - (u + v)); s1 + s2 + s3 */
    float w = 1.0f - (u + v);
    float x = (a[0] * w + a[4] * v) + a[2] * u;
    float y = (a[1] * w + a[5] * v) + a[3] * u;
    return m->mask[mask_texel(y, m->h) * (unsigned)m->w + mask_texel(x, m->w)] != 0;
}

vo_hit vo_intersect(const float ori_[3], const float dir_[3], const vo_node* nodes, const uint32_t* indices,
                    const void* prims, int kind, int any_hit, float max_t, vo_counters* cnt)
{
    return vo_intersect_masked(ori_, dir_, nodes, indices, prims, kind, any_hit, max_t, NULL, cnt);
}

vo_hit vo_intersect_masked(const float ori_[3], const float dir_[3], const vo_node* nodes, const uint32_t* indices,
                           const void* prims, int kind, int any_hit, float max_t, const vo_hit_mask* mask,
                           vo_counters* cnt)
{
    v3 ori = mk(ori_[0], ori_[1], ori_[2]);
    v3 dir = mk(dir_[0], dir_[1], dir_[2]);
    /* hit_record ctor (intersect.h:95-103): hit false, ids 0, t = max(), u = v = 0 */
    vo_hit res; res.hit = 0; res.prim_id = 0; res.geom_id = 0; res.list_index = 0;
    res.t = FLT_MAX; res.u = 0.0f; res.v = 0.0f;
    uint64_t nbox = 0, nprim = 0;

    /* detail/bvh/intersect.inl:60-63; stack sized generously (reference stack<32>, stack.h: at most
     * one entry per tree level is ever live, so 4096 covers any tree this test suite builds) */
    uint32_t stack[4096];
    int sp = 0;
    stack[sp++] = 0;
    v3 inv_dir = mk(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);

    while (sp > 0) {
        const vo_node* node = &nodes[stack[--sp]];
        int terminated = 0;
        while (node->num_prims == 0) {
            const vo_node* ch = &nodes[node->first];
            float tn[2], tf[2]; int hb[2];
            for (int c = 0; c < 2; ++c) {
                /* math/intersect.h:52-70 slab test */
                v3 t1 = mul(sub(mk(ch[c].bmin[0], ch[c].bmin[1], ch[c].bmin[2]), ori), inv_dir);
                v3 t2 = mul(sub(mk(ch[c].bmax[0], ch[c].bmax[1], ch[c].bmax[2]), ori), inv_dir);
                tn[c] = fmax_ref(fmin_ref(t1.x, t2.x), fmax_ref(fmin_ref(t1.y, t2.y), fmin_ref(t1.z, t2.z)));
                tf[c] = fmin_ref(fmax_ref(t1.x, t2.x), fmin_ref(fmax_ref(t1.y, t2.y), fmax_ref(t1.z, t2.z)));
                int h = tf[c] >= tn[c];
                /* update_if.h:60-66,82-88 is_closer(box) */
                hb[c] = h && tn[c] < res.t && tf[c] >= 0.0f && tn[c] < max_t;
            }
            nbox += 2;
            if (hb[0] && hb[1]) {
                unsigned near_addr = (tn[0] < tn[1]) ? 0u : 1u;   /* intersect.inl:86 */
                if (sp == 4096) { res.hit = 0; goto out; }   /* unreachable for depth < 4096 */
                stack[sp++] = node->first + (near_addr ^ 1u);
                node = &nodes[node->first + near_addr];
            } else if (hb[0]) {
                node = &nodes[node->first];
            } else if (hb[1]) {
                node = &nodes[node->first + 1];
            } else {
                terminated = 1;
                break;
            }
        }
        if (terminated) continue;
        for (uint32_t i = node->first; i != node->first + node->num_prims; ++i) {
            prim_hit hr = kind == VO_TRI ? isect_tri(ori, dir, (const vo_tri*)prims + indices[i])
                                         : isect_sphere(ori, dir, (const vo_sphere*)prims + indices[i]);
            ++nprim;
            if (mask && kind == VO_TRI && hr.hit) hr.hit = mask_keep(mask, hr.prim_id, hr.u, hr.v);
            /* update_if.h:48-56,73-79 is_closer + update_if.h:27-37 + hit_record.h:54-64 */
            int closer = hr.hit && hr.t >= 0.0f && hr.t < res.t && hr.t < max_t;
            if (!closer) continue;
            res.hit = 1; res.t = hr.t; res.prim_id = hr.prim_id; res.geom_id = hr.geom_id;
            res.u = hr.u; res.v = hr.v; res.list_index = i;
            if (any_hit) goto out;          /* exit_traversal.h:49-56 */
        }
    }
out:
    if (cnt) { cnt->box_tests += nbox; cnt->prim_tests += nprim; }
    return res;
}

int vo_intersect_multi(const float ori_[3], const float dir_[3], const vo_node* nodes, const uint32_t* indices,
                       const void* prims, int kind, int n, vo_hit* res, vo_counters* cnt)
{
    return vo_intersect_multi_masked(ori_, dir_, nodes, indices, prims, kind, n, res, NULL, cnt);
}

int vo_intersect_multi_masked(const float ori_[3], const float dir_[3], const vo_node* nodes, const uint32_t* indices,
                              const void* prims, int kind, int n, vo_hit* res, const vo_hit_mask* mask,
                              vo_counters* cnt)
{
    v3 ori = mk(ori_[0], ori_[1], ori_[2]);
    v3 dir = mk(dir_[0], dir_[1], dir_[2]);
    for (int k = 0; k < n; ++k) {            /* hit_record ctor: hit false, t = max() */
        res[k].hit = 0; res[k].prim_id = 0; res[k].geom_id = 0; res[k].list_index = 0;
        res[k].t = FLT_MAX; res[k].u = 0.0f; res[k].v = 0.0f;
    }
    uint64_t nbox = 0, nprim = 0;
    uint32_t stack[4096];
    int sp = 0;
    stack[sp++] = 0;
    v3 inv_dir = mk(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
    while (sp > 0) {
        const vo_node* node = &nodes[stack[--sp]];
        int terminated = 0;
        while (node->num_prims == 0) {
            const vo_node* ch = &nodes[node->first];
            float tn[2], tf[2]; int hb[2];
            for (int c = 0; c < 2; ++c) {
                v3 t1 = mul(sub(mk(ch[c].bmin[0], ch[c].bmin[1], ch[c].bmin[2]), ori), inv_dir);
                v3 t2 = mul(sub(mk(ch[c].bmax[0], ch[c].bmax[1], ch[c].bmax[2]), ori), inv_dir);
                tn[c] = fmax_ref(fmin_ref(t1.x, t2.x), fmax_ref(fmin_ref(t1.y, t2.y), fmin_ref(t1.z, t2.z)));
                tf[c] = fmin_ref(fmax_ref(t1.x, t2.x), fmin_ref(fmax_ref(t1.y, t2.y), fmax_ref(t1.z, t2.z)));
                int h = tf[c] >= tn[c];
                /* multi_hit.h:221-244: is_closer against any kept record (max_t = max()) */
                int closer = 0;
                for (int k = 0; k < n && !closer; ++k)
                    closer = h && tn[c] < res[k].t && tf[c] >= 0.0f && tn[c] < FLT_MAX;
                hb[c] = closer;
            }
            nbox += 2;
            if (hb[0] && hb[1]) {
                unsigned near_addr = (tn[0] < tn[1]) ? 0u : 1u;
                if (sp == 4096) goto out;
                stack[sp++] = node->first + (near_addr ^ 1u);
                node = &nodes[node->first + near_addr];
            } else if (hb[0]) {
                node = &nodes[node->first];
            } else if (hb[1]) {
                node = &nodes[node->first + 1];
            } else {
                terminated = 1;
                break;
            }
        }
        if (terminated) continue;
        for (uint32_t i = node->first; i != node->first + node->num_prims; ++i) {
            prim_hit hr = kind == VO_TRI ? isect_tri(ori, dir, (const vo_tri*)prims + indices[i])
                                         : isect_sphere(ori, dir, (const vo_sphere*)prims + indices[i]);
            ++nprim;
            if (mask && kind == VO_TRI && hr.hit) hr.hit = mask_keep(mask, hr.prim_id, hr.u, hr.v);
            int closer = 0;
            for (int k = 0; k < n && !closer; ++k)
                closer = hr.hit && hr.t >= 0.0f && hr.t < res[k].t && hr.t < FLT_MAX;
            if (!closer) continue;
            /* update_if -> insert_sorted(hr, result, is_closer_t) (multi_hit.h:180-189, algorithm.h:46-75) */
            int pos = n;
            for (int k = 0; k < n; ++k)
                if (hr.hit && hr.t >= 0.0f && hr.t < res[k].t) { pos = k; break; }
            if (pos == n) continue;
            for (int k = n - 1; k > pos; --k) res[k] = res[k - 1];
            res[pos].hit = 1; res[pos].t = hr.t; res[pos].prim_id = hr.prim_id; res[pos].geom_id = hr.geom_id;
            res[pos].u = hr.u; res[pos].v = hr.v; res[pos].list_index = i;
        }
    }
out:
    if (cnt) { cnt->box_tests += nbox; cnt->prim_tests += nprim; }
    int hits = 0;
    for (int k = 0; k < n; ++k) hits += res[k].hit;
    return hits;
}

/* ------------------------------------------------------------------------------------------ */
/* Pixel pipeline + kernels                                                                    */

/* sched_common.h:130-150 make_primary_ray_impl (pinhole) for the pixel position (x + ox, y + oy):
 * the uniform sampler (:180-195) passes offset 0, jittered / ssaa (:196-300) their offsets */
static inline float det2(float m00, float m01, float m10, float m11) { return m00 * m11 - m10 * m01; }  /* math.h:493-496 */

void vo_inverse4(const float m[16], float out[16])
{
#define M(r, c) m[(c) * 4 + (r)]
    float s0 = det2(M(0, 0), M(0, 1), M(1, 0), M(1, 1));
    float s1 = det2(M(0, 0), M(0, 2), M(1, 0), M(1, 2));
    float s2 = det2(M(0, 0), M(0, 3), M(1, 0), M(1, 3));
    float s3 = det2(M(0, 1), M(0, 2), M(1, 1), M(1, 2));
    float s4 = det2(M(0, 1), M(0, 3), M(1, 1), M(1, 3));
    float s5 = det2(M(0, 2), M(0, 3), M(1, 2), M(1, 3));
    float c5 = det2(M(2, 2), M(2, 3), M(3, 2), M(3, 3));
    float c4 = det2(M(2, 1), M(2, 3), M(3, 1), M(3, 3));
    float c3 = det2(M(2, 1), M(2, 2), M(3, 1), M(3, 2));
    float c2 = det2(M(2, 0), M(2, 3), M(3, 0), M(3, 3));
    float c1 = det2(M(2, 0), M(2, 2), M(3, 0), M(3, 2));
    float c0 = det2(M(2, 0), M(2, 1), M(3, 0), M(3, 1));
    float det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
    const float r[16] = {   /* the constructor's arguments, column by column */
        (+ M(1, 1) * c5 - M(1, 2) * c4 + M(1, 3) * c3) / det,
        (- M(1, 0) * c5 + M(1, 2) * c2 + M(1, 3) * c1) / det,
        (+ M(1, 0) * c4 - M(1, 1) * c2 + M(1, 3) * c0) / det,
        (- M(1, 0) * c3 + M(1, 1) * c1 + M(1, 2) * c0) / det,
        (- M(0, 1) * c5 + M(0, 2) * c4 - M(0, 3) * c3) / det,
        (+ M(0, 0) * c5 - M(0, 2) * c2 + M(0, 3) * c1) / det,
        (- M(0, 0) * c4 + M(0, 1) * c2 - M(0, 3) * c0) / det,
        (+ M(0, 0) * c3 - M(0, 1) * c1 + M(0, 2) * c0) / det,
        (+ M(3, 1) * s5 - M(3, 2) * s4 + M(3, 3) * s3) / det,
        (- M(3, 0) * s5 + M(3, 2) * s2 - M(3, 3) * s1) / det,
        (+ M(3, 0) * s4 - M(3, 1) * s2 + M(3, 3) * s0) / det,
        (- M(3, 0) * s3 + M(3, 1) * s1 - M(3, 2) * s0) / det,
        (- M(2, 1) * s5 + M(2, 2) * s4 - M(2, 3) * s3) / det,
        (+ M(2, 0) * s5 - M(2, 2) * s2 + M(2, 3) * s1) / det,
        (- M(2, 0) * s4 + M(2, 1) * s2 - M(2, 3) * s0) / det,
        (+ M(2, 0) * s3 - M(2, 1) * s1 + M(2, 2) * s0) / det };
#undef M
    memcpy(out, r, sizeof(r));
}

/* matrix4.inl:171-181 matrix * vector (column-major m[c * 4 + r]) */
static inline void mat_vec(const float* m, const float v[4], float out[4])
{
    for (int r = 0; r < 4; ++r)
        out[r] = m[0 * 4 + r] * v[0] + m[1 * 4 + r] * v[1] + m[2 * 4 + r] * v[2] + m[3 * 4 + r] * v[3];
}

static inline void primary_ray_at(const vo_camera* cam, unsigned x, unsigned y, float ox, float oy, v3* ori, v3* dir)
{
    float fx = (float)x + ox, fy = (float)y + oy;
    float u = 2.0f * (fx + 0.5f) / (float)cam->width - 1.0f;
    float v = 2.0f * (fy + 0.5f) / (float)cam->height - 1.0f;
    if (cam->inv_view) {
        /* sched_common.h:152-176: o = inv_view (inv_proj (u, v, -1, 1)), d likewise at z = +1;
         * ori = o.xyz / o.w, dir = normalize(d.xyz / d.w - ori) */
        const float pn[4] = { u, v, -1.0f, 1.0f }, pf[4] = { u, v, 1.0f, 1.0f };
        float a[4], o[4], b[4], d[4];
        mat_vec(cam->inv_proj, pn, a); mat_vec(cam->inv_view, a, o);
        mat_vec(cam->inv_proj, pf, b); mat_vec(cam->inv_view, b, d);
        *ori = mk(o[0] / o[3], o[1] / o[3], o[2] / o[3]);
        *dir = normalize(sub(mk(d[0] / d[3], d[1] / d[3], d[2] / d[3]), *ori));
        return;
    }
    v3 cu = mk(cam->cam_u[0], cam->cam_u[1], cam->cam_u[2]);
    v3 cv = mk(cam->cam_v[0], cam->cam_v[1], cam->cam_v[2]);
    v3 cw = mk(cam->cam_w[0], cam->cam_w[1], cam->cam_w[2]);
    *ori = mk(cam->eye[0], cam->eye[1], cam->eye[2]);
    *dir = normalize(add(add(muls(cu, u), muls(cv, v)), cw));
}

static inline void primary_ray(const vo_camera* cam, unsigned x, unsigned y, v3* ori, v3* dir)
{
    primary_ray_at(cam, x, y, 0.0f, 0.0f, ori, dir);
}

typedef struct { float color[4]; uint32_t prim_id; float t; uint8_t occ; uint32_t list_index; uint32_t rays; } px_out;

/* closest_hit / any_hit over a list of BVH refs (traverse_linear.inl:76-141): each BVH traversed
 * with a fresh result and the same max_t; hr merged by update_if(result, hr, is_closer(hr, result,
 * max_t)) (update_if.h:27-79, hit_record.h:54-64: strictly closer); exit_traversal<AnyHit> after
 * every merge (exit_traversal.h:49-56) */
static vo_hit trace(const vo_scene* s, const float o[3], const float d[3], int any, float max_t, vo_counters* cnt)
{
    if (!s->next) return vo_intersect_masked(o, d, s->nodes, s->indices, s->prims, s->kind, any, max_t, s->hit_mask, cnt);
    vo_hit res;
    memset(&res, 0, sizeof(res));
    res.t = FLT_MAX;                      /* hit_record ctor: t = numeric_limits<float>::max() */
    for (const vo_scene* b = s; b; b = b->next) {
        vo_hit hr = vo_intersect_masked(o, d, b->nodes, b->indices, b->prims, b->kind, any, max_t, s->hit_mask, cnt);
        if (hr.hit && hr.t >= 0.0f && hr.t < res.t && hr.t < max_t) res = hr;
        if (any && res.hit) break;
    }
    return res;
}
static void shade_simple(const vo_scene* s, const vo_kernel* k, v3 ori, v3 dir, const vo_hit* hr, float out[4]);
static void shade_whitted(const vo_scene* s, const vo_kernel* k, v3 ori, v3 dir, vo_hit hr, float out[4],
                          uint32_t* rays, vo_counters* cnt);

/* ao/main.cpp:183-246 with the deterministic sampler of SURVEY.md Appendix A */
static px_out shade_pixel_at(const vo_scene* s, const vo_camera* cam, const vo_kernel* k, unsigned x, unsigned y,
                             float ox, float oy, vo_counters* cnt)
{
    px_out o;
    memcpy(o.color, k->bg, sizeof(o.color));
    o.prim_id = 0xFFFFFFFFu; o.t = -1.0f; o.occ = 0; o.list_index = 0xFFFFFFFFu; o.rays = 1;
    v3 ori, dir;
    primary_ray_at(cam, x, y, ox, oy, &ori, &dir);
    float fo[3] = { ori.x, ori.y, ori.z }, fd[3] = { dir.x, dir.y, dir.z };
    vo_hit hr = trace(s, fo, fd, 0, FLT_MAX, cnt);
    if (!hr.hit) return o;
    o.prim_id = hr.prim_id; o.t = hr.t; o.list_index = hr.list_index;
    if (k->mode == VO_MODE_SIMPLE) {
        shade_simple(s, k, ori, dir, &hr, o.color);
        return o;
    }
    if (k->mode == VO_MODE_WHITTED) {
        shade_whitted(s, k, ori, dir, hr, o.color, &o.rays, cnt);
        return o;
    }
    if (k->mode != VO_MODE_AO) {
        o.color[0] = o.color[1] = o.color[2] = o.color[3] = 1.0f;
        return o;
    }
    v3 isect_pos = add(ori, muls(dir, hr.t));
    v3 n = ld(&s->normals[hr.prim_id]);                                /* get_normal.h:26-37 */
    /* vector3.inl:357-367 make_orthonormal_basis (w = n) */
    v3 bv = fabsf(n.x) > fabsf(n.y) ? normalize(mk(-n.z, 0.0f, n.x)) : normalize(mk(0.0f, n.z, -n.y));
    v3 bu = cross(bv, n);
    float clr = 1.0f;
    uint32_t p = (uint32_t)y * (uint32_t)cam->width + (uint32_t)x;
    float step = 1.0f / (float)k->samples;
    for (int smp = 0; smp < k->samples; ++smp) {
        float sx = 0.0f, sy = 0.0f;
        for (uint32_t kk = 0; kk < 16; ++kk) {
            uint32_t ctr = ((p * 8u + (uint32_t)smp) * 16u + kk) * 2u + k->frame_num * 0x9E3779B1u;
            float xa = 2.0f * vo_uniform(ctr) - 1.0f;
            float ya = 2.0f * vo_uniform(ctr + 1) - 1.0f;
            if (xa * xa + ya * ya < 1.0f) { sx = xa; sy = ya; break; }
        }
        float sz = sqrtf(fmax_ref(0.0f, 1.0f - sx * sx - sy * sy));
        v3 d = normalize(add(add(smul(sx, bu), smul(sy, bv)), smul(sz, n)));
        v3 ao = add(isect_pos, muls(d, k->eps));
        float ao_o[3] = { ao.x, ao.y, ao.z }, ao_d[3] = { d.x, d.y, d.z };
        vo_hit ar = trace(s, ao_o, ao_d, 1, k->radius, cnt);
        o.rays++;
        if (ar.hit) { clr = clr - step; o.occ |= (uint8_t)(1u << smp); }
    }
    o.color[0] = o.color[1] = o.color[2] = clr;
    o.color[3] = 1.0f;
    return o;
}

static px_out shade_pixel(const vo_scene* s, const vo_camera* cam, const vo_kernel* k, unsigned x, unsigned y,
                          vo_counters* cnt)
{
    return shade_pixel_at(s, cam, k, x, y, 0.0f, 0.0f, cnt);
}

/* get_surface (get_surface.h:336-376, 576-592) of a triangle hit: geometric + shading normal by
 * the normal binding, material by geom_id */
static const vo_plastic* surface(const vo_scene* s, const vo_kernel* k, const vo_hit* hr, v3* gn, v3* sn)
{
    if (k->normal_binding == VO_NORMALS_PER_FACE) {
        *gn = *sn = ld(&s->normals[hr->prim_id]);                       /* get_normal.h:26-37 */
    } else {
        /* get_surface.h:336-376 -> get_normal(hr, primitive(list_index)) (get_normal.h:110-116)
         * and get_shading_normal.h:64-84 with lerp(a,b,c,u,v) (math.h:466-475) */
        const vo_tri* tri = (const vo_tri*)s->prims + s->indices[hr->list_index];
        *gn = normalize(cross(ld(&tri->e1), ld(&tri->e2)));
        v3 n0 = ld(&s->vertex_normals[hr->prim_id * 3u]);
        v3 n1 = ld(&s->vertex_normals[hr->prim_id * 3u + 1u]);
        v3 n2 = ld(&s->vertex_normals[hr->prim_id * 3u + 2u]);
        v3 s2 = muls(n2, hr->v), s3 = muls(n1, hr->u), s1 = muls(n0, 1.0f - (hr->u + hr->v));
        *sn = normalize(add(add(s1, s2), s3));
    }
    return &k->materials[hr->geom_id];
}

/* plastic.inl:13-16 ambient() = ca * ka, times from_rgba(ambient_color) (spectrum.inl:375-378) */
static v3 ambient_term(const vo_kernel* k, const vo_plastic* m)
{
    v3 amb_c = mk(k->ambient[0] * k->ambient[3], k->ambient[1] * k->ambient[3], k->ambient[2] * k->ambient[3]);
    return mul(muls(mk(m->ca[0], m->ca[1], m->ca[2]), m->ka), amb_c);
}

/* plastic::shade (plastic.inl:21-37) for one point light at surface point pos: pi * (lambertian +
 * blinn) * intensity * ndotl */
static v3 plastic_light(const vo_plastic* m, v3 n, v3 view, v3 pos, const vo_point_light* L)
{
    const float PI = 3.14159265358979323846264338328e+00f, INV_PI = 3.18309886183790691216444201928e-01f;
    v3 lpos = mk(L->position[0], L->position[1], L->position[2]);
    v3 wi = normalize(sub(lpos, pos));                                  /* simple.inl:59 */
    v3 wo = view;
    float ndotl = fmax_ref(0.0f, dot(n, wi));                           /* plastic.inl:29 */
    /* brdf.h:36-41 lambertian::f = cd * kd * inv_pi */
    v3 diff = muls(muls(mk(m->cd[0], m->cd[1], m->cd[2]), m->kd), INV_PI);
    /* brdf.h:111-122 blinn::f */
    v3 h = normalize(add(wo, wi));
    float hdotn = fmax_ref(0.0f, dot(h, n));
    v3 spec = muls(mk(m->cs[0], m->cs[1], m->cs[2]), m->ks);
    float sat = fmax_ref(0.0f, fmin_ref(dot(wi, h), 1.0f));              /* math.h:454-457 */
    float p5 = powf(1.0f - sat, 5.0f);
    v3 schlick = add(spec, muls(mk(1.0f - spec.x, 1.0f - spec.y, 1.0f - spec.z), p5));
    float nfactor = (m->exp + 2.0f) / (8.0f * PI);
    v3 bl = muls(muls(schlick, nfactor), powf(hdotn, m->exp));
    /* point_light.inl:12-28 intensity: (cl * kl) * float(1.0 / (c + l*d + q*d*d)) */
    float dist = sqrtf(dot(sub(lpos, pos), sub(lpos, pos)));
    float den = L->constant_att + L->linear_att * dist + L->quadratic_att * dist * dist;
    float att = (float)(1.0 / (double)den);
    v3 I = muls(muls(mk(L->cl[0], L->cl[1], L->cl[2]), L->kl), att);
    return muls(mul(smul(PI, add(diff, bl)), I), ndotl);
}

/* detail/simple.inl:26-79 (simple::kernel) with plastic materials and point lights: ambient term,
 * two-sided shading normal (faceforward), one plastic::shade per light.  Colour of a hit pixel. */
static void shade_simple(const vo_scene* s, const vo_kernel* k, v3 ori, v3 dir, const vo_hit* hr, float out[4])
{
    v3 pos = add(ori, muls(dir, hr->t));                               /* simple.inl:37 */
    v3 gn, sn;
    const vo_plastic* m = surface(s, k, hr, &gn, &sn);
    v3 shaded = ambient_term(k, m);
    v3 view = mk(-dir.x, -dir.y, -dir.z);
    v3 n = dot(gn, view) < 0.0f ? mk(-sn.x, -sn.y, -sn.z) : sn;          /* vector.inl:674-681 */
    for (int li = 0; li < k->num_lights; ++li)
        shaded = add(shaded, plastic_light(m, n, view, pos, &k->lights[li]));   /* simple.inl:63 */
    out[0] = shaded.x; out[1] = shaded.y; out[2] = shaded.z; out[3] = 1.0f;   /* to_rgba */
}

/* detail/whitted.inl:186-277 (whitted::kernel) for a pixel whose primary ray hit (hr): loop while
 * the last closest hit hit, throughput > epsilon and depth++ < num_bounces: ambient, an any-hit
 * shadow ray per light (origin pos + l * eps, max_t = |pos - light|), colour += shaded *
 * throughput, then the plastic bounce (specular_bounce fall-through, whitted.inl:64-77):
 * reflect(view, shading normal) = 2 dot(n, view) n - view with kr = 0.1.  The reflection ray is
 * traced only when the next loop test can pass (its hit is unused otherwise). */
static void shade_whitted(const vo_scene* s, const vo_kernel* k, v3 ori, v3 dir, vo_hit hr, float out[4],
                          uint32_t* rays, vo_counters* cnt)
{
    v3 color = mk(0.0f, 0.0f, 0.0f);
    float thr = 1.0f;
    int depth = 0;
    while (hr.hit && thr > k->eps && depth++ < k->num_bounces) {
        v3 pos = add(ori, muls(dir, hr.t));                            /* whitted.inl:223 */
        v3 gn, sn;
        const vo_plastic* m = surface(s, k, &hr, &gn, &sn);
        v3 shaded = ambient_term(k, m);
        v3 view = mk(-dir.x, -dir.y, -dir.z);
        v3 n = dot(gn, view) < 0.0f ? mk(-sn.x, -sn.y, -sn.z) : sn;      /* faceforward */
        for (int li = 0; li < k->num_lights; ++li) {
            const vo_point_light* L = &k->lights[li];
            v3 lpos = mk(L->position[0], L->position[1], L->position[2]);
            v3 ldir = normalize(sub(lpos, pos));
            v3 so = add(pos, muls(ldir, k->eps));
            float max_t = sqrtf(dot(sub(pos, lpos), sub(pos, lpos)));   /* length(isect_pos - pos) */
            float fo[3] = { so.x, so.y, so.z }, fd[3] = { ldir.x, ldir.y, ldir.z };
            vo_hit sh = vo_intersect_masked(fo, fd, s->nodes, s->indices, s->prims, s->kind, 1, max_t, s->hit_mask, cnt);
            ++*rays;
            /* shaded_clr += select(active, clr, 0) */
            shaded = add(shaded, sh.hit ? mk(0.0f, 0.0f, 0.0f) : plastic_light(m, n, view, pos, L));
        }
        color = add(color, muls(shaded, thr));
        float d2 = 2.0f * dot(sn, view);                               /* vector.inl:683-689 */
        v3 rd = sub(mk(d2 * sn.x, d2 * sn.y, d2 * sn.z), view);
        float thr2 = thr * 0.1f;
        if (!(thr2 > k->eps && depth < k->num_bounces)) break;
        ori = add(pos, muls(rd, k->eps));
        dir = rd;
        float fo[3] = { ori.x, ori.y, ori.z }, fd[3] = { dir.x, dir.y, dir.z };
        hr = vo_intersect_masked(fo, fd, s->nodes, s->indices, s->prims, s->kind, 0, FLT_MAX, s->hit_mask, cnt);
        ++*rays;
        thr = thr2;
    }
    out[0] = color.x; out[1] = color.y; out[2] = color.z; out[3] = 1.0f;     /* to_rgba */
}

/* examples/multi_hit/main.cpp:166-235: for every kept hit (in t order) the surface of
 * get_surface(hit_rec[i], params), plastic::shade with the FIRST light (no ambient), alpha 0.3,
 * front-to-back compositing; colour starts at 0 */
static void shade_multi(const vo_scene* s, const vo_kernel* k, v3 ori, v3 dir, const vo_hit* hits, int n, float out[4])
{
    float acc[4] = { 0.0f, 0.0f, 0.0f, 0.0f };
    for (int i = 0; i < n; ++i) {
        if (!hits[i].hit) break;
        float c[4];
        vo_kernel one = *k;
        one.num_lights = k->num_lights > 0 ? 1 : 0;
        one.ambient[0] = one.ambient[1] = one.ambient[2] = one.ambient[3] = 0.0f;
        shade_simple(s, &one, ori, dir, &hits[i], c);     /* ambient 0: ca*ka*0 = 0, then + shade */
        c[3] = 0.3f;
        c[0] = c[0] * c[3]; c[1] = c[1] * c[3]; c[2] = c[2] * c[3];
        float f = 1.0f - acc[3];
        for (int q = 0; q < 4; ++q) acc[q] = acc[q] + c[q] * f;
    }
    memcpy(out, acc, sizeof(acc));
}

uint64_t vo_render_multi(const vo_scene* s, const vo_camera* cam, const vo_kernel* k, float* color,
                         uint32_t* mh_prim_id, float* mh_t, int threads)
{
    int W = cam->width, H = cam->height, n = k->max_hits;
    if (n < 1 || n > VO_MAX_HITS) return 0;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#else
    threads = 1;
#endif
    #pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            v3 ori, dir;
            primary_ray(cam, (unsigned)x, (unsigned)y, &ori, &dir);
            float fo[3] = { ori.x, ori.y, ori.z }, fd[3] = { dir.x, dir.y, dir.z };
            vo_hit hits[VO_MAX_HITS];
            vo_intersect_multi_masked(fo, fd, s->nodes, s->indices, s->prims, s->kind, n, hits, s->hit_mask, NULL);
            size_t p = (size_t)y * W + x;
            for (int i = 0; i < n; ++i) {
                if (mh_prim_id) mh_prim_id[p * n + i] = hits[i].hit ? hits[i].prim_id : 0xFFFFFFFFu;
                if (mh_t) mh_t[p * n + i] = hits[i].hit ? hits[i].t : -1.0f;
            }
            if (color) shade_multi(s, k, ori, dir, hits, n, color + 4 * p);
        }
    }
    return (uint64_t)W * H;
}

void vo_vertex_normals(const vo_vec3* face_normals, size_t n, vo_vec3* out)
{
    for (size_t k = 0; k < n; ++k) {
        v3 fn = ld(&face_normals[k]);
        for (uint32_t j = 0; j < 3; ++j) {
            uint32_t b = ((uint32_t)k * 3u + j) * 3u;
            v3 p = mk((vo_uniform(b) - 0.5f) * 0.4f, (vo_uniform(b + 1u) - 0.5f) * 0.4f, (vo_uniform(b + 2u) - 0.5f) * 0.4f);
            st(&out[k * 3 + j], normalize(add(fn, p)));
        }
    }
}

uint64_t vo_render_rows(const vo_scene* s, const vo_camera* cam, const vo_kernel* k, int y0, int y1,
                        float* color, uint32_t* prim_id, float* t, uint8_t* occ, uint32_t* list_index,
                        int threads, vo_counters* cnt)
{
    uint64_t rays = 0, nbox = 0, nprim = 0;
    int W = cam->width;
    const unsigned* sb = cam->scissor;
    const int whole = sb[0] == 0 && sb[1] == 0 && sb[2] == 0 && sb[3] == 0;
    const int cx0 = whole ? 0 : (int)sb[0], cy0 = whole ? 0 : (int)sb[1];
    const int cx1 = whole ? W : (int)(sb[2] < (unsigned)W ? sb[2] : (unsigned)W);
    const int cy1 = whole ? cam->height : (int)(sb[3] < (unsigned)cam->height ? sb[3] : (unsigned)cam->height);
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#else
    threads = 1;
#endif
    #pragma omp parallel for schedule(dynamic, 1) num_threads(threads) reduction(+:rays,nbox,nprim)
    for (int y = y0; y < y1; ++y) {
        vo_counters c = { 0, 0 };
        if (y < cy0 || y >= cy1) continue;              /* outside the scissor box: not written */
        for (int x = cx0; x < cx1; ++x) {
            px_out o = shade_pixel(s, cam, k, (unsigned)x, (unsigned)y, &c);
            size_t p = (size_t)y * W + x;
            if (color) memcpy(color + 4 * p, o.color, 16);
            if (prim_id) prim_id[p] = o.prim_id;
            if (t) t[p] = o.t;
            if (occ) occ[p] = o.occ;
            if (list_index) list_index[p] = o.list_index;
            rays += o.rays;
        }
        nbox += c.box_tests; nprim += c.prim_tests;
    }
    if (cnt) { cnt->box_tests += nbox; cnt->prim_tests += nprim; }
    return rays;
}

/* pixel samplers (sched_common.h:196-300 make_primary_rays, :440-720 sample_pixel_impl), pixel by
 * pixel: uniform and jittered store the kernel's colour; jittered_blend blends it onto the target,
 * dst = c * a + dst * (1 - a) with a = 1 / frame_num (pixel_access.h:1155-1176); ssaa<N> stores 0
 * and then blends each of its N fixed-offset samples with a = 1 / N, 1 (the reference's offset
 * tables, including its 8x entry 0.1825).  The jitter draws of pixel p in frame n are U(c) - 0.5,
 * U(c + 1) - 0.5 with c = p * 2 + 0x632BE5AB + n * 0x68E31DA4 (the build's deterministic stand-in
 * for the scheduler's clock-seeded random_sampler; the reference's jitter vector takes them in
 * g++'s argument order: y the first, x the second).  prim_id: the last sample's hit. */
static const float ssaa2[2][2] = { { -0.25f, -0.25f }, { 0.25f, 0.25f } };
static const float ssaa4[4][2] = { { -0.125f, -0.375f }, { 0.375f, -0.125f }, { 0.125f, 0.375f }, { -0.375f, 0.125f } };
static const float ssaa8[8][2] = { { -0.125f, -0.4375f }, { 0.375f, -0.3125f }, { -0.375f, -0.1875f }, { 0.125f, -0.0625f },
                                   { -0.125f, 0.0625f }, { 0.375f, 0.1825f }, { -0.375f, 0.3125f }, { 0.125f, 0.4375f } };

void vo_sampler_offsets(int kind, int count, unsigned x, unsigned y, unsigned width, uint32_t frame_num,
                        int sub, float* ox, float* oy)
{
    *ox = 0.0f; *oy = 0.0f;
    if (kind == VO_SAMPLER_JITTERED || kind == VO_SAMPLER_JITTERED_BLEND) {
        /* vector<2, S> jitter(samp.next() - 0.5, samp.next() - 0.5) (sched_common.h:208): the two
         * draws are constructor arguments, whose evaluation order C++ leaves unspecified; g++ on
         * x86-64 (the reference build here) evaluates them right to left, so y takes the first draw */
        uint32_t c = (y * width + x) * 2u + 0x632BE5ABu + frame_num * 0x68E31DA4u;
        *oy = vo_uniform(c) - 0.5f;
        *ox = vo_uniform(c + 1u) - 0.5f;
    } else if (kind == VO_SAMPLER_SSAA) {
        const float (*t)[2] = count == 2 ? ssaa2 : count == 4 ? ssaa4 : ssaa8;
        *ox = t[sub][0]; *oy = t[sub][1];
    }
}

int vo_render_sampled(const vo_scene* s, const vo_camera* cam, const vo_kernel* k, int kind, int count,
                      float* color, uint32_t* prim_id, float* t, int threads)
{
    if (kind == VO_SAMPLER_SSAA && count != 2 && count != 4 && count != 8) return -1;
    const int n = kind == VO_SAMPLER_SSAA ? count : 1;
    int W = cam->width;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#else
    threads = 1;
#endif
    #pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
    for (int y = 0; y < cam->height; ++y) {
        for (int x = 0; x < W; ++x) {
            size_t p = (size_t)y * W + x;
            float* dst = color + 4 * p;
            if (kind == VO_SAMPLER_SSAA) dst[0] = dst[1] = dst[2] = dst[3] = 0.0f;
            for (int sub = 0; sub < n; ++sub) {
                float ox, oy;
                vo_sampler_offsets(kind, count, (unsigned)x, (unsigned)y, (unsigned)W, k->frame_num, sub, &ox, &oy);
                px_out o = shade_pixel_at(s, cam, k, (unsigned)x, (unsigned)y, ox, oy, NULL);
                prim_id[p] = o.prim_id;
                if (t) t[p] = o.t;
                if (kind == VO_SAMPLER_UNIFORM || kind == VO_SAMPLER_JITTERED) {
                    memcpy(dst, o.color, 16);
                } else {
                    float a = kind == VO_SAMPLER_SSAA ? 1.0f / (float)n : 1.0f / (float)k->frame_num;
                    float b = kind == VO_SAMPLER_SSAA ? 1.0f : 1.0f - a;
                    for (int c = 0; c < 4; ++c) {
                        float sc = o.color[c] * a, dc = dst[c] * b;
                        dst[c] = sc + dc;
                    }
                }
            }
        }
    }
    return 0;
}

uint64_t vo_render_pixels(const vo_scene* s, const vo_camera* cam, const vo_kernel* k,
                          const uint32_t* pixels, size_t npix,
                          float* color, uint32_t* prim_id, float* t, uint8_t* occ, int threads)
{
    uint64_t rays = 0;
    int W = cam->width;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#else
    threads = 1;
#endif
    #pragma omp parallel for schedule(dynamic, 64) num_threads(threads) reduction(+:rays)
    for (long i = 0; i < (long)npix; ++i) {
        unsigned x = pixels[i] % (unsigned)W, y = pixels[i] / (unsigned)W;
        px_out o = shade_pixel(s, cam, k, x, y, NULL);
        if (color) memcpy(color + 4 * i, o.color, 16);
        if (prim_id) prim_id[i] = o.prim_id;
        if (t) t[i] = o.t;
        if (occ) occ[i] = o.occ;
        rays += o.rays;
    }
    return rays;
}

uint64_t vo_fnv1a(const void* data, size_t n, uint64_t h)
{
    const unsigned char* b = (const unsigned char*)data;
    if (h == 0) h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ull; }
    return h;
}
