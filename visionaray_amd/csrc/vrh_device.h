// visionaray_amd/csrc/vrh_device.h -- device-side data layout and traversal for gfx950.
//
// HBM layout (built once at vrh_scene_upload from the reference arrays):
//
//   pairs  : one 64-B record per inner node n, holding BOTH children's boxes and links, stored at
//            index (n.first_child - 1) / 2 (the reference allocates children as adjacent pairs at
//            odd node indices, build.inl:45-50, so this is dense).  Slab-major and child-interleaved,
//            so each float4 feeds two packed-fp32 (child 0, child 1) operand pairs:
//              q0 = c0.min.x c1.min.x c0.min.y c1.min.y    q1 = c0.min.z c1.min.z c0.max.x c1.max.x
//              q2 = c0.max.y c1.max.y c0.max.z c1.max.z    q3 = link0 link1 0 0
//            link = pair index of an inner child, or LEAF_BIT | first_prim for a leaf child.
//            One inner visit = one aligned 64-B read (the reference reads the same 64 B as two
//            32-B bvh_nodes, intersect.inl:76-79).
//   prims  : primitives permuted into leaf order (prims[i] = reference prims[indices[i]]), so the
//            index indirection of index_bvh_ref_t::primitive (bvh.h:226-229) disappears; the last
//            primitive of each leaf carries END_BIT.  triangle = 3 x float4 (48 B):
//              (v1.xyz, e1.x) (e1.yz, e2.xy) (e2.z, prim_id, geom_id, flags)
//            sphere = 2 x float4 (32 B): (center.xyz, radius) (prim_id, geom_id, flags, 0)
//   normals: float4 per prim_id (face normals for AO, get_normal.h:26-37).
//
// Arithmetic is the reference's, operation for operation (compiled with -ffp-contract=off and
// IEEE division/sqrt), so results are bit-identical to the CPU simple_sched path.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#ifndef VRH_PACKED_SLABS
#define VRH_PACKED_SLABS 0   // 1: slab distances with v_pk_add_f32 / v_pk_mul_f32
#endif

namespace vrh {
namespace dev {

constexpr uint32_t LEAF_BIT = 0x80000000u;
constexpr uint32_t END_BIT = 1u;
constexpr int KIND_TRI = 0;
constexpr int KIND_SPHERE = 1;
constexpr float FMAX = 3.402823466e+38f;       // numeric_limits<float>::max(), hit_record ctor

// math/detail/math.h:48-60
__device__ __forceinline__ float tmin(float x, float y) { return x < y ? x : y; }
__device__ __forceinline__ float tmax(float x, float y) { return x < y ? y : x; }

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk3(float x, float y, float z) { return { x, y, z }; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return { a.x + b.x, a.y + b.y, a.z + b.z }; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return { a.x - b.x, a.y - b.y, a.z - b.z }; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return { a.x * b.x, a.y * b.y, a.z * b.z }; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return { a.x * s, a.y * s, a.z * s }; }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return { s * a.x, s * a.y, s * a.z }; }
// vector3.inl:291-307
__device__ __forceinline__ f3 cross(f3 u, f3 v) { return { u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x }; }
__device__ __forceinline__ float dot(f3 u, f3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
// vector3.inl:331-336, math.h:477-481 (rsqrt = 1/sqrt, both IEEE)
__device__ __forceinline__ f3 normalize(f3 v) { return v * (1.0f / __builtin_sqrtf(dot(v, v))); }

struct ray_t { f3 ori, dir, inv; };

typedef float f2 __attribute__((ext_vector_type(2)));   // packed fp32: v_pk_add_f32 / v_pk_mul_f32

// Both children of a pair: math/intersect.h:52-70 slab test + update_if.h:60-66,82-88 box
// is_closer.  The slab distances (b - o) * inv of child 0 and child 1 are computed two at a time
// with packed fp32 adds and multiplies; each half is the same IEEE single operation as the scalar
// expression, so nothing changes numerically.
//
// FAST = false is the reference formulation literally: min/max are the ternaries of
// math/detail/math.h:48-60 (v_cmp + v_cndmask pairs).  FAST = true uses v_min/v_max/v_min3/v_max3.
// The two agree on every comparison outcome whenever no slab distance is NaN: hardware min/max
// then differ from the ternaries only in the sign of a zero result, and signed zeros compare
// equal in every use of tnear/tfar below.  A slab distance (b - o) * inv is NaN only if inv is
// infinite (a zero direction component) or an input is not finite, so FAST is used only for rays
// with finite origin and finite inv over scenes with finite node bounds (checked at upload).
template <bool FAST>
__device__ __forceinline__ void box_pair(float4 q0, float4 q1, float4 q2, const ray_t& r, float best_t,
                                         float max_t, bool& b0, bool& b1, float& tn0, float& tn1)
{
#if VRH_PACKED_SLABS
    const f2 ox = { r.ori.x, r.ori.x }, oy = { r.ori.y, r.ori.y }, oz = { r.ori.z, r.ori.z };
    const f2 ix = { r.inv.x, r.inv.x }, iy = { r.inv.y, r.inv.y }, iz = { r.inv.z, r.inv.z };
    const f2 t1x = (f2{ q0.x, q0.y } - ox) * ix;
    const f2 t1y = (f2{ q0.z, q0.w } - oy) * iy;
    const f2 t1z = (f2{ q1.x, q1.y } - oz) * iz;
    const f2 t2x = (f2{ q1.z, q1.w } - ox) * ix;
    const f2 t2y = (f2{ q2.x, q2.y } - oy) * iy;
    const f2 t2z = (f2{ q2.z, q2.w } - oz) * iz;
#else
    f2 t1x, t1y, t1z, t2x, t2y, t2z;
    t1x.x = (q0.x - r.ori.x) * r.inv.x; t1x.y = (q0.y - r.ori.x) * r.inv.x;
    t1y.x = (q0.z - r.ori.y) * r.inv.y; t1y.y = (q0.w - r.ori.y) * r.inv.y;
    t1z.x = (q1.x - r.ori.z) * r.inv.z; t1z.y = (q1.y - r.ori.z) * r.inv.z;
    t2x.x = (q1.z - r.ori.x) * r.inv.x; t2x.y = (q1.w - r.ori.x) * r.inv.x;
    t2y.x = (q2.x - r.ori.y) * r.inv.y; t2y.y = (q2.y - r.ori.y) * r.inv.y;
    t2z.x = (q2.z - r.ori.z) * r.inv.z; t2z.y = (q2.w - r.ori.z) * r.inv.z;
#endif
    float tf0, tf1;
    if constexpr (FAST)
    {
        tn0 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1x.x, t2x.x), __builtin_fminf(t1y.x, t2y.x)), __builtin_fminf(t1z.x, t2z.x));
        tf0 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t1x.x, t2x.x), __builtin_fmaxf(t1y.x, t2y.x)), __builtin_fmaxf(t1z.x, t2z.x));
        tn1 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1x.y, t2x.y), __builtin_fminf(t1y.y, t2y.y)), __builtin_fminf(t1z.y, t2z.y));
        tf1 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t1x.y, t2x.y), __builtin_fmaxf(t1y.y, t2y.y)), __builtin_fmaxf(t1z.y, t2z.y));
    }
    else
    {
        tn0 = tmax(tmin(t1x.x, t2x.x), tmax(tmin(t1y.x, t2y.x), tmin(t1z.x, t2z.x)));
        tf0 = tmin(tmax(t1x.x, t2x.x), tmin(tmax(t1y.x, t2y.x), tmax(t1z.x, t2z.x)));
        tn1 = tmax(tmin(t1x.y, t2x.y), tmax(tmin(t1y.y, t2y.y), tmin(t1z.y, t2z.y)));
        tf1 = tmin(tmax(t1x.y, t2x.y), tmin(tmax(t1y.y, t2y.y), tmax(t1z.y, t2z.y)));
    }
    b0 = (tf0 >= tn0) & (tn0 < best_t) & (tf0 >= 0.0f) & (tn0 < max_t);
    b1 = (tf1 >= tn1) & (tn1 < best_t) & (tf1 >= 0.0f) & (tn1 < max_t);
}

__device__ __forceinline__ bool finite_ray(const ray_t& r)
{
    return __builtin_isfinite(r.inv.x) && __builtin_isfinite(r.inv.y) && __builtin_isfinite(r.inv.z)
        && __builtin_isfinite(r.ori.x) && __builtin_isfinite(r.ori.y) && __builtin_isfinite(r.ori.z);
}

// math/intersect.h:122-179 ray/triangle (Moller-Trumbore, two-sided, closed edges) without the
// early outs: every quantity is computed exactly as the reference computes it; the reference's
// early returns only skip work whose result it then discards, so the accepted hits and their t are
// identical, and the lanes of a wave do not diverge.
__device__ __forceinline__ bool isect_tri(const ray_t& r, float4 a, float4 b, float4 c, float& t)
{
    f3 v1 = mk3(a.x, a.y, a.z), e1 = mk3(a.w, b.x, b.y), e2 = mk3(b.z, b.w, c.x);
    f3 s1 = cross(r.dir, e2);
    float div = dot(s1, e1);
    float inv_div = 1.0f / div;
    f3 d = r.ori - v1;
    float b1 = dot(d, s1) * inv_div;
    f3 s2 = cross(d, e1);
    float b2 = dot(r.dir, s2) * inv_div;
    t = dot(e2, s2) * inv_div;
    return (div != 0.0f) & (b1 >= 0.0f) & (b1 <= 1.0f) & (b2 >= 0.0f) & (b1 + b2 <= 1.0f);
}

// math/intersect.h:186-221 ray/sphere
__device__ __forceinline__ bool isect_sphere(const ray_t& r, float4 a, float& t)
{
    f3 o = r.ori - mk3(a.x, a.y, a.z);
    float A = dot(r.dir, r.dir);
    float B = dot(r.dir, o) * 2.0f;
    float C = dot(o, o) - a.w * a.w;
    float disc = B * B - 4.0f * A * C;
    bool valid = disc >= 0.0f;
    float root_disc = valid ? __builtin_sqrtf(disc) : disc;
    float q = B < 0.0f ? -0.5f * (B - root_disc) : -0.5f * (B + root_disc);
    float t1 = q / A;
    float t2 = C / q;
    t = valid ? (t1 > t2 ? t2 : t1) : -1.0f;
    return valid;
}

// Per-lane LDS stack, column-major ([entry][lane]) so a wave's pushes/pops hit 64 distinct banks.
// The top is kept as a word offset advanced by the block stride (no multiply per push/pop).
struct lds_stack
{
    uint32_t* mem;        // dynamic LDS base
    uint32_t base;        // this lane's column (word offset of entry 0)
    uint32_t top;         // word offset of the next free entry
    uint32_t stride;      // words between entries = threads per block
    __device__ __forceinline__ void reset() { top = base; }
    __device__ __forceinline__ void push(uint32_t v) { mem[top] = v; top += stride; }
    __device__ __forceinline__ uint32_t pop() { top -= stride; return mem[top]; }
    __device__ __forceinline__ bool empty() const { return top == base; }
};

// Test counts of the counting variant (VRH_KERNEL_COUNT_TESTS).  box / prim are per lane; the
// step fields measure SIMD utilisation: `it_box` / `it_prim` are this lane's descent / leaf loop
// iterations in the current ray_step call, folded by count_wave() into the wave-level totals
// (w_steps outer iterations, w_box / w_prim = iterations the wave executed, i.e. the lane maximum).
struct test_counts
{
    uint32_t box, prim;
    bool aborted;
    uint32_t it_box, it_prim;
    uint64_t w_steps, w_busy, w_box, w_prim;
};

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    return v;
}

// called by every lane of the wave after a step of the busy lanes
__device__ __forceinline__ void count_wave(test_counts& c, bool busy)
{
    c.w_steps += 1;
    c.w_busy += (uint64_t)__popcll(__ballot(busy));
    c.w_box += wave_max(c.it_box);
    c.w_prim += wave_max(c.it_prim);
    c.it_box = 0;
    c.it_prim = 0;
}

// One outer iteration of the reference loop (detail/bvh/intersect.inl:66-130) for EITHER traversal
// type: closest hit (any = false: boxes culled against the running best_t, all primitives of
// reached leaves tested, best_t / best_prim updated by is_closer) or any hit (any = true: best_t
// stays max() until the first accepted hit, which ends the ray, exit_traversal.h:49-56).  Depth
// first, near child first (ties -> child 1, intersect.inl:86), far child pushed, leaf primitives in
// index order; popped nodes are NOT re-culled (the reference does not), which keeps closest-hit
// tie resolution identical.  Lanes of one wave may be in different
// modes and still run the same instruction stream.  Returns 1 = any-hit found, -1 = ray finished
// (stack empty), 0 = continue.
template <int KIND, bool COUNT, bool FAST>
__device__ __forceinline__ int ray_step(const float4* __restrict__ pairs, const float4* __restrict__ prims,
                                        const ray_t& r, float max_t, bool any, lds_stack& st,
                                        float& best_t, uint32_t& best_prim, test_counts& cnt,
                                        uint32_t& steps, uint32_t step_limit)
{
    // the tree was validated at upload (no cycles, links in range), so the descent terminates;
    // the guard below only bounds the number of outer iterations per ray
    if (st.empty()) return -1;
    if (++steps > step_limit) { cnt.aborted = true; return -1; }
    uint32_t link = st.pop();
    while (!(link & LEAF_BIT))
    {
        const float4* p = pairs + 4u * link;
        const float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
        bool b0, b1;
        float tn0, tn1;
        box_pair<FAST>(q0, q1, q2, r, best_t, max_t, b0, b1, tn0, tn1);
        const uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
        if (COUNT) { cnt.box += 2; cnt.it_box += 1; }
        // intersect.inl:84-101 without branches: both hit -> push the far child, descend the near
        // one (near = tn0 < tn1 ? 0 : 1); one hit -> descend it; none -> pop
        const bool both = b0 & b1;
        const bool go0 = both ? (tn0 < tn1) : b0;
        if (both) st.push(go0 ? l1 : l0);
        if (!(b0 | b1)) return st.empty() ? -1 : 0;
        link = go0 ? l0 : l1;
    }
    uint32_t i = link & ~LEAF_BIT;
    for (;;)
    {
        float t;
        bool h;
        uint32_t flags, pid;
        if constexpr (KIND == KIND_TRI)
        {
            const float4* q = prims + 3u * i;
            float4 a = q[0], b = q[1], c = q[2];
            h = isect_tri(r, a, b, c, t);
            pid = __float_as_uint(c.y);
            flags = __float_as_uint(c.w);
        }
        else
        {
            const float4* q = prims + 2u * i;
            float4 a = q[0], b = q[1];
            h = isect_sphere(r, a, t);
            pid = __float_as_uint(b.x);
            flags = __float_as_uint(b.z);
        }
        if (COUNT) { cnt.prim += 1; cnt.it_prim += 1; }
        if (h & (t >= 0.0f) & (t < best_t) & (t < max_t))      // update_if.h:48-56, 73-79
        {
            best_t = t;
            best_prim = pid;
            if (any) return 1;                                   // exit_traversal.h:49-56
        }
        if (flags & END_BIT) break;
        ++i;
    }
    return st.empty() ? -1 : 0;
}

__device__ __forceinline__ ray_t make_ray(f3 ori, f3 dir)
{
    ray_t r;
    r.ori = ori; r.dir = dir;
    r.inv = mk3(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);   // intersect.inl:63
    return r;
}

// SURVEY.md Appendix A counter hash
__device__ __forceinline__ uint32_t wang(uint32_t a)
{
    a = (a ^ 61u) ^ (a >> 16);
    a = a + (a << 3);
    a = a ^ (a >> 4);
    a = a * 0x27d4eb2du;
    return a ^ (a >> 15);
}
__device__ __forceinline__ float uniform01(uint32_t k) { return (float)(wang(k) >> 8) * (1.0f / 16777216.0f); }

// Appendix A Malley sample s of pixel p -> direction in the (u, v, n) basis (ao/main.cpp:218-226)
__device__ __forceinline__ f3 ao_direction(uint32_t p, uint32_t s, f3 bu, f3 bv, f3 n)
{
    float sx = 0.0f, sy = 0.0f;
    for (uint32_t k = 0; k < 16; ++k)
    {
        uint32_t ctr = ((p * 8u + s) * 16u + k) * 2u;
        float xa = 2.0f * uniform01(ctr) - 1.0f;
        float ya = 2.0f * uniform01(ctr + 1u) - 1.0f;
        if (xa * xa + ya * ya < 1.0f) { sx = xa; sy = ya; break; }
    }
    float sz = __builtin_sqrtf(tmax(0.0f, 1.0f - sx * sx - sy * sy));
    return normalize((sx * bu + sy * bv) + sz * n);
}

} // namespace dev
} // namespace vrh
