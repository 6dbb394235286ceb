// visionaray_amd/csrc/vrh_device.h -- device-side data layout and traversal for gfx950.
//
// HBM layout (built once at vrh_scene_upload from the reference arrays):
//
//   pairs  : one 64-B record per inner node n, holding BOTH children's boxes and links, stored at
//            index (n.first_child - 1) / 2 (the reference allocates children as adjacent pairs at
//            odd node indices, build.inl:45-50, so this is dense).  4 x float4:
//              q0 = c0.min.xyz, c0.max.x      q1 = c0.max.yz, c1.min.xy
//              q2 = c1.min.z,   c1.max.xyz    q3 = link0, link1, 0, 0
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

namespace vrh {
namespace dev {

constexpr uint32_t LEAF_BIT = 0x80000000u;
constexpr uint32_t END_BIT = 1u;
constexpr int KIND_TRI = 0;
constexpr int KIND_SPHERE = 1;

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

struct hit_t
{
    float    t, u, v;
    uint32_t prim_id, geom_id, list_index;
    bool     hit;
};

__device__ __forceinline__ hit_t miss_record()
{
    // hit_record ctor, math/intersect.h:95-103
    hit_t h;
    h.t = 3.402823466e+38f; h.u = 0.0f; h.v = 0.0f;
    h.prim_id = 0; h.geom_id = 0; h.list_index = 0; h.hit = false;
    return h;
}

// math/intersect.h:52-70 slab test + update_if.h:60-66,82-88 box is_closer.
//
// FAST = false is the reference formulation literally: min/max are the ternaries of
// math/detail/math.h:48-60 (v_cmp + v_cndmask pairs).  FAST = true uses v_min/v_max/v_min3/v_max3.
// The two agree on every comparison outcome whenever no slab distance is NaN: hardware min/max
// then differ from the ternaries only in the sign of a zero result, and signed zeros compare
// equal in every use of tnear/tfar below.  A slab distance (b - o) * inv is NaN only if inv is
// infinite (a zero direction component) or an input is not finite, so FAST is used only for rays
// with finite origin and finite inv over scenes with finite node bounds (checked at upload).
template <bool FAST>
__device__ __forceinline__ bool box_closer(float lx, float ly, float lz, float hx, float hy, float hz,
                                           const ray_t& r, float best_t, float max_t, float& tnear)
{
    float t1x = (lx - r.ori.x) * r.inv.x, t1y = (ly - r.ori.y) * r.inv.y, t1z = (lz - r.ori.z) * r.inv.z;
    float t2x = (hx - r.ori.x) * r.inv.x, t2y = (hy - r.ori.y) * r.inv.y, t2z = (hz - r.ori.z) * r.inv.z;
    float tn, tf;
    if constexpr (FAST)
    {
        tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1x, t2x), __builtin_fminf(t1y, t2y)), __builtin_fminf(t1z, t2z));
        tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t1x, t2x), __builtin_fmaxf(t1y, t2y)), __builtin_fmaxf(t1z, t2z));
    }
    else
    {
        tn = tmax(tmin(t1x, t2x), tmax(tmin(t1y, t2y), tmin(t1z, t2z)));
        tf = tmin(tmax(t1x, t2x), tmin(tmax(t1y, t2y), tmax(t1z, t2z)));
    }
    tnear = tn;
    return (tf >= tn) & (tn < best_t) & (tf >= 0.0f) & (tn < max_t);
}

__device__ __forceinline__ bool finite_ray(const ray_t& r)
{
    return __builtin_isfinite(r.inv.x) && __builtin_isfinite(r.inv.y) && __builtin_isfinite(r.inv.z)
        && __builtin_isfinite(r.ori.x) && __builtin_isfinite(r.ori.y) && __builtin_isfinite(r.ori.z);
}

// math/intersect.h:122-179 ray/triangle, Moller-Trumbore (two-sided, closed edges)
__device__ __forceinline__ bool isect_tri(const ray_t& r, float4 a, float4 b, float4 c, float& t, float& u, float& v)
{
    f3 v1 = mk3(a.x, a.y, a.z), e1 = mk3(a.w, b.x, b.y), e2 = mk3(b.z, b.w, c.x);
    f3 s1 = cross(r.dir, e2);
    float div = dot(s1, e1);
    if (!(div != 0.0f)) return false;
    float inv_div = 1.0f / div;
    f3 d = r.ori - v1;
    float b1 = dot(d, s1) * inv_div;
    if (!(b1 >= 0.0f && b1 <= 1.0f)) return false;
    f3 s2 = cross(d, e1);
    float b2 = dot(r.dir, s2) * inv_div;
    if (!(b2 >= 0.0f && b1 + b2 <= 1.0f)) return false;
    t = dot(e2, s2) * inv_div;
    u = b1; v = b2;
    return true;
}

// The same test without early outs (math/intersect.h:122-179): every quantity is computed exactly
// as the reference computes it; the reference's early returns only skip work whose result it then
// discards, so the accepted hits and their t are identical.  Avoids divergent branches per lane.
__device__ __forceinline__ bool isect_tri_nb(const ray_t& r, float4 a, float4 b, float4 c, float& t)
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

constexpr int SCHED_ROUNDS = 0;    // AO rays handed out 64 at a time
constexpr int SCHED_REFILL = 1;    // AO rays refilled per lane; primary rays traced first
constexpr int SCHED_UNIFIED = 2;   // primary and AO rays share one refilling loop

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

// detail/bvh/intersect.inl:25-134: depth-first traversal, near child first (ties -> child 1),
// far child pushed, leaf primitives tested in index order, AnyHit exits at the first accepted hit
// (exit_traversal.h:49-56).  Box culling uses the running closest t exactly like the reference;
// popped nodes are NOT re-culled (the reference does not), which keeps tie resolution identical.
struct test_counts { uint32_t box, prim; bool aborted; };

// step_limit bounds the node visits + primitive tests of one ray (a correct traversal never needs
// more than nodes + primitives); a corrupt BVH therefore ends the ray with `aborted` set instead
// of spinning the wave forever.
template <int KIND, bool ANY, bool COUNT, class Stack>
__device__ __forceinline__ hit_t trace(const float4* __restrict__ pairs, const float4* __restrict__ prims,
                                       uint32_t root, const ray_t& r, float max_t, Stack& st, test_counts& cnt,
                                       uint32_t step_limit)
{
    hit_t res = miss_record();
    uint32_t steps = 0;
    st.reset();
    st.push(root);
    while (!st.empty())
    {
        uint32_t link = st.pop();
        while (!(link & LEAF_BIT))
        {
            if (++steps > step_limit) { cnt.aborted = true; return res; }
            const float4* p = pairs + 4u * link;
            float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
            float tn0, tn1;
            bool b0 = box_closer<false>(q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, r, res.t, max_t, tn0);
            bool b1 = box_closer<false>(q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, r, res.t, max_t, tn1);
            uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
            if (COUNT) cnt.box += 2;
            if (b0 && b1)
            {
                bool near0 = tn0 < tn1;          // intersect.inl:86
                st.push(near0 ? l1 : l0);
                link = near0 ? l0 : l1;
            }
            else if (b0) link = l0;
            else if (b1) link = l1;
            else goto next;
        }
        {
            uint32_t i = link & ~LEAF_BIT;
            for (;;)
            {
                uint32_t flags;
                float t, u = 0.0f, v = 0.0f;
                bool h;
                uint32_t pid, gid;
                if constexpr (KIND == KIND_TRI)
                {
                    const float4* q = prims + 3u * i;
                    float4 a = q[0], b = q[1], c = q[2];
                    h = isect_tri(r, a, b, c, t, u, v);
                    pid = __float_as_uint(c.y); gid = __float_as_uint(c.z); flags = __float_as_uint(c.w);
                }
                else
                {
                    const float4* q = prims + 2u * i;
                    float4 a = q[0], b = q[1];
                    h = isect_sphere(r, a, t);
                    pid = __float_as_uint(b.x); gid = __float_as_uint(b.y); flags = __float_as_uint(b.z);
                }
                if (COUNT) cnt.prim += 1;
                // update_if.h:48-56 is_closer, update_if.h:27-37 + hit_record.h:54-64 update
                if (h && t >= 0.0f && t < res.t && t < max_t)
                {
                    res.hit = true; res.t = t; res.u = u; res.v = v;
                    res.prim_id = pid; res.geom_id = gid; res.list_index = i;
                    if (ANY) return res;
                }
                if (flags & END_BIT) break;
                ++i;
                if (++steps > step_limit) { cnt.aborted = true; return res; }
            }
        }
    next:;
    }
    return res;
}

// One outer iteration of the any-hit loop (intersect.inl:67-130 with AnyHit): pop a node, descend
// to a leaf, test its primitives.  The stack holds the rest of the ray's state, so a wave can
// interleave rays (REFILL schedule).  Returns 1 = occluded (first accepted hit, exit_traversal.h:
// 49-56), -1 = missed (stack empty), 0 = continue.  Before the first hit result.t is max(), so the
// set of visited nodes -- and the occlusion bit -- does not depend on how iterations interleave.
template <int KIND, bool COUNT>
__device__ __forceinline__ int anyhit_step(const float4* __restrict__ pairs, const float4* __restrict__ prims,
                                           const ray_t& r, float max_t, lds_stack& st, test_counts& cnt,
                                           uint32_t& steps, uint32_t step_limit)
{
    const float best_t = 3.402823466e+38f;
    if (st.empty()) return -1;
    uint32_t link = st.pop();
    while (!(link & LEAF_BIT))
    {
        if (++steps > step_limit) { cnt.aborted = true; return -1; }
        const float4* p = pairs + 4u * link;
        float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
        float tn0, tn1;
        bool b0 = box_closer<false>(q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, r, best_t, max_t, tn0);
        bool b1 = box_closer<false>(q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, r, best_t, max_t, tn1);
        uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
        if (COUNT) cnt.box += 2;
        if (b0 && b1)
        {
            bool near0 = tn0 < tn1;
            st.push(near0 ? l1 : l0);
            link = near0 ? l0 : l1;
        }
        else if (b0) link = l0;
        else if (b1) link = l1;
        else return st.empty() ? -1 : 0;
    }
    uint32_t i = link & ~LEAF_BIT;
    for (;;)
    {
        float t, u, v;
        bool h;
        uint32_t flags;
        if constexpr (KIND == KIND_TRI)
        {
            const float4* q = prims + 3u * i;
            float4 a = q[0], b = q[1], c = q[2];
            h = isect_tri(r, a, b, c, t, u, v);
            flags = __float_as_uint(c.w);
        }
        else
        {
            const float4* q = prims + 2u * i;
            float4 a = q[0], b = q[1];
            h = isect_sphere(r, a, t);
            flags = __float_as_uint(b.z);
        }
        if (COUNT) cnt.prim += 1;
        if (h && t >= 0.0f && t < best_t && t < max_t) return 1;
        if (flags & END_BIT) break;
        ++i;
        if (++steps > step_limit) { cnt.aborted = true; return -1; }
    }
    return st.empty() ? -1 : 0;
}

// One outer iteration of the reference loop (intersect.inl:67-130) for EITHER traversal type:
// closest hit (any = false: boxes culled against the running best_t, all primitives of reached
// leaves tested, best_t / best_prim updated by is_closer) or any hit (any = true: best_t stays
// max() until the first accepted hit, which ends the ray).  Lanes of one wave may be in different
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
        float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
        float tn0, tn1;
        const bool b0 = box_closer<FAST>(q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, r, best_t, max_t, tn0);
        const bool b1 = box_closer<FAST>(q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, r, best_t, max_t, tn1);
        const uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
        if (COUNT) cnt.box += 2;
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
            h = isect_tri_nb(r, a, b, c, t);
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
        if (COUNT) cnt.prim += 1;
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
