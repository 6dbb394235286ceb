// include/visionaray_hip/detail/vrh_device.h -- device-side data layout and traversal for gfx950
// (libvrh.so's kernels and the user kernels of visionaray_hip/hip_kernels.h share it).
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
#include <type_traits>

#ifndef VRH_SCALAR_UNIFORM
#define VRH_SCALAR_UNIFORM 1   // wave-uniform pair fetches through the scalar cache (ray_step)
#endif
#ifndef VRH_SORTED_PUSH
#define VRH_SORTED_PUSH 1    // the 4-wide any-hit step pushes its other hit entries farthest first (0: in
                             // index order; 1: hf1M +0.7 %, hf10M equal, profiles/r04/ab/sorted_push/)
#endif
#ifndef VRH_PACKED_SLABS
#define VRH_PACKED_SLABS 0   // 1: slab distances with v_pk_add_f32 / v_pk_mul_f32
#endif

namespace vrh {
namespace dev {

constexpr bool SCALAR_UNIFORM = VRH_SCALAR_UNIFORM != 0;
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
__device__ __forceinline__ bool isect_tri(const ray_t& r, float4 a, float4 b, float4 c, float& t, float& u, float& v)
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
    u = b1;
    v = b2;
    return (div != 0.0f) & (b1 >= 0.0f) & (b1 <= 1.0f) & (b2 >= 0.0f) & (b1 + b2 <= 1.0f);
}

__device__ __forceinline__ bool isect_tri(const ray_t& r, float4 a, float4 b, float4 c, float& t)
{
    float u, v;
    return isect_tri(r, a, b, c, t, u, v);
}

// Mask intersector (vrh_hit_mask_create): the intersector example's mask_intersector
// (examples/intersector/main.cpp:251-330) as data.  tc = lerp(tc0, tc1, tc2, u, v) in the order of
// math.h:468-475 (s2 = c v, s3 = b u, s1 = a (1 - (u + v)), (s1 + s2) + s3), then a nearest texel.
struct hit_mask_params
{
    const float2* tc;         // 3 per prim_id
    const uint8_t* mask;      // w x h, row-major; null = no mask
    uint32_t w, h;
};

__device__ __forceinline__ uint32_t mask_texel(float c, uint32_t n)
{
    const float x = (c > 0.0f ? c : 0.0f) * (float)n;      // NaN -> 0
    return x < (float)n ? (uint32_t)x : n - 1u;
}

__device__ __forceinline__ bool mask_keep(const hit_mask_params& m, uint32_t prim_id, float u, float v)
{
    const float2 a = m.tc[3u * prim_id], b = m.tc[3u * prim_id + 1u], c = m.tc[3u * prim_id + 2u];
    const float w = 1.0f - (u + v);
    const float x = (a.x * w + c.x * v) + b.x * u;
    const float y = (a.y * w + c.y * v) + b.y * u;
    return m.mask[mask_texel(y, m.h) * m.w + mask_texel(x, m.w)] != 0;
}

// extra closest-hit state the shading kernels need: barycentrics (hit_record u, v) and the
// leaf-order index of the hit primitive (hit_record_bvh::primitive_list_index)
struct hit_extra { float u, v; uint32_t li; };

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

// Per-lane stack, column-major ([entry][lane]) so a wave's pushes/pops hit 64 distinct LDS banks.
// `used` = entries in use x the block stride (a word offset from the lane's column `base`), so the
// bounds checks compare it with wave-uniform limits only (no per-lane limit register stays live).
// SPILL = true: only the first cap_off / stride entries live in LDS; deeper entries continue, in the
// same column layout, in a global overflow block of the launch (`spill`), so a BVH deeper than the
// LDS part is still exact -- used where LDS, not registers, would limit the waves per CU
// (vrh_render; the check costs 2-4 % where it is not needed, so SPILL = false has none).  The
// overflow block is addressed through a buffer resource (wave-uniform base in SGPRs, 32-bit per-lane
// offset, accesses past the block dropped): no 64-bit per-lane address stays live.
template <bool SPILL>
struct stack_t
{
    uint32_t* mem;        // dynamic LDS base
    uint32_t base;        // this lane's column (word offset of entry 0)
    uint32_t used;        // entries in use x stride
    uint32_t stride;      // words between entries = threads per block
    uint32_t cap_off;     // SPILL: LDS entries x stride (wave-uniform; unused otherwise)
    uint32_t lim_off;     // total entries x stride (LDS + overflow; wave-uniform)
    uint32_t* spill;      // SPILL: this block's overflow block (wave-uniform): the entry at used >= cap_off
                          // lives at word base + used - cap_off of it (addressed as byte offset
                          // 4 (base + used) from a descriptor base 4 cap_off bytes before the block, so
                          // no per-lane base - cap_off is kept)
    __device__ __forceinline__ void init(uint32_t* m, uint32_t column, uint32_t block_stride, uint32_t lds_entries,
                                         uint32_t total_entries, uint32_t* overflow)
    {
        mem = m; base = column; used = 0u; stride = block_stride;
        cap_off = lds_entries * block_stride;
        lim_off = total_entries * block_stride;
        spill = overflow;
    }
    __device__ __forceinline__ void reset() { used = 0u; }
    // k more entries fit
    __device__ __forceinline__ bool room(uint32_t k) const { return used + k * stride <= lim_off; }
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) uint32_t lds_word;
    // the LDS byte address of the lane's entry at `used` (SPILL): one per-lane value serves the LDS access
    // and, past the LDS part, the offset into the overflow block's buffer resource
    __device__ __forceinline__ uint32_t entry_addr() const
    {
        return uint32_t(reinterpret_cast<uintptr_t>((lds_word*)mem)) + (base + used) * 4u;
    }
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t overflow() const
    {
        // gfx9 buffer descriptor word 3 (raw dwords, as composable_kernel's CK_BUFFER_RESOURCE_3RD_DWORD);
        // the base moved back by the LDS part and the LDS base address, as integers (descriptor fields, not
        // C++ pointers), so that entry_addr() is the byte offset; no range check (num_records = max: every
        // offset a lane forms lies in its column of the block)
        const uintptr_t lds0 = uintptr_t(uint32_t(reinterpret_cast<uintptr_t>((lds_word*)mem)));
        return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(spill) - uintptr_t(cap_off) * 4u - lds0),
                                                 0, -1, 0x00020000);
    }
#endif
    __device__ __forceinline__ void push(uint32_t v)
    {
        if constexpr (SPILL)
        {
#if defined(__HIP_DEVICE_COMPILE__)
            const uint32_t a = entry_addr();
            if (__builtin_expect(used < cap_off, 1)) *(lds_word*)uintptr_t(a) = v;
            else __builtin_amdgcn_raw_buffer_store_b32(v, overflow(), int(a), 0, 0);
#endif
        }
        else
            mem[base + used] = v;
        used += stride;
    }
    __device__ __forceinline__ uint32_t pop()
    {
        used -= stride;
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (SPILL)
        {
            const uint32_t a = entry_addr();
            if (__builtin_expect(used >= cap_off, 0)) return __builtin_amdgcn_raw_buffer_load_b32(overflow(), int(a), 0, 0);
            return *(lds_word*)uintptr_t(a);
        }
#endif
        return mem[base + used];
    }
    __device__ __forceinline__ bool empty() const { return used == 0u; }
};
using lds_stack = stack_t<false>;

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
    uint64_t w_uni;           // wave-level descent iterations whose active lanes all fetch one node
    // access shape (counting variant): per wave-level vector-memory instruction of the traversal
    // (node pair, primitive and normal loads, output stores), the distinct 16-B pieces its active
    // lanes request (`reqs`, merged within a 16-lane quarter), the distinct 128-B lines (`lines`) and
    // the instruction count (`vmem`); kept by the wave's first active lane, summed over lanes at the
    // end.  A divergence diagnostic -- the hardware's TCP access count is measured by PMC instead.
    uint64_t reqs, lines, vmem;
    // the vector L1's merging (counting variant): acc4 = distinct pieces per aligned 4-lane group,
    // summed over groups (the hardware's accesses); acc_ideal = per distinct piece ceil(lanes / 4)
    uint64_t acc4, acc_ideal;
    uint64_t acc_kind[5];     // acc4 by load kind (VMEM_*)
};
// kinds of the counted vector-memory instructions
constexpr uint32_t VMEM_PRIM = 0, VMEM_QUAD = 1, VMEM_PAIR = 2, VMEM_NORMAL = 3, VMEM_STORE = 4;

// distinct values of `key` over the active lanes (wave-uniform result)
__device__ __forceinline__ uint32_t distinct_keys(uint64_t key)
{
    uint64_t rem = __ballot(true);
    uint32_t n = 0;
    while (rem)
    {
        const int first = __builtin_ctzll(rem);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, first);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), first);
        rem &= ~__ballot(key == (((uint64_t)hi << 32) | lo));
        ++n;
    }
    return n;
}

// distinct values of `key` within each 16-lane quarter of the wave, summed (wave-uniform result):
// the vector L1 merges the requests of lanes that ask for the same 16-B piece only inside a quarter
// wave (tools/micro/l1_roof.hip: 64 lanes over 4 pieces of one record = 16 TCP accesses, 4 lanes per
// piece = 16, one piece per lane = 64)
__device__ __forceinline__ uint32_t distinct_keys_per_quarter(uint64_t key)
{
    uint64_t rem = __ballot(true);
    uint32_t n = 0;
    while (rem)
    {
        const int first = __builtin_ctzll(rem);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, first);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), first);
        const uint64_t quarter = 0xFFFFull << (first & 48);
        rem &= ~(__ballot(key == (((uint64_t)hi << 32) | lo)) & quarter);
        ++n;
    }
    return n;
}

// distinct values of `key` within each aligned 4-lane group, summed, and sum over distinct values of
// ceil(lanes with it / 4) (wave-uniform results): the vector L1's accesses of a 16-B-per-lane load
// as the lanes sit, and as they would if the lanes wanting one piece sat together
__device__ __forceinline__ void group_accesses(uint64_t key, uint32_t& acc4, uint32_t& ideal)
{
    const uint64_t act = __ballot(true);
    const uint32_t lane = __lane_id();
    // this lane is the first (lowest) active lane of its group with its key
    bool first = true;
#pragma unroll
    for (uint32_t k = 1; k < 4; ++k)
    {
        const uint32_t o = (lane & ~3u) + ((lane + k) & 3u);          // the other lanes of the group
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)key, (int)o), hi = (uint32_t)__shfl((int)(uint32_t)(key >> 32), (int)o);
        const bool same = ((act >> o) & 1ull) && ((((uint64_t)hi << 32) | lo) == key);
        first = first && !(same && o < lane);
    }
    acc4 = (uint32_t)__popcll(__ballot(first));
    uint64_t rem = act;
    uint32_t n = 0;
    while (rem)
    {
        const int f = __builtin_ctzll(rem);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, f);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), f);
        const uint64_t m = __ballot(key == (((uint64_t)hi << 32) | lo)) & act;
        n += ((uint32_t)__popcll(m) + 3u) / 4u;
        rem &= ~m;
    }
    ideal = n;
}

// one wave-level vector-memory instruction whose lanes access `bytes` (<= 16) at `p`: account for it
// in the L1 model (counting variant only; called by the active lanes)
__device__ __forceinline__ void count_vmem(test_counts& c, const void* p, uint32_t times = 1u, uint32_t kind = VMEM_PRIM)
{
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t l = distinct_keys(a >> 7), q = distinct_keys_per_quarter(a >> 4);
    uint32_t g4, gi;
    group_accesses(a >> 4, g4, gi);
    if (__lane_id() == (uint32_t)__builtin_ctzll(__ballot(true)))
    {
        c.lines += (uint64_t)l * times;
        c.reqs += (uint64_t)q * times;
        c.vmem += times;
        c.acc4 += (uint64_t)g4 * times;
        c.acc_ideal += (uint64_t)gi * times;
        c.acc_kind[kind] += (uint64_t)g4 * times;
    }
}

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

constexpr uint32_t QUAD_NONE = 0xFFFFFFFFu;
constexpr uint32_t NO_RESUME = 0xFFFFFFFFu;   // ray_step: no descent to resume

// One entry of a 4-wide any-hit record (vrh_quad.cpp): the box test of update_if.h:60-66 with
// best_t = max() (an any-hit ray has no hit yet while it traverses), hardware min/max (the lane's
// ray is finite, so the slab distances are never NaN).
__device__ __forceinline__ bool quad_entry(float xl, float yl, float zl, float xh, float yh, float zh,
                                           const ray_t& r, float max_t, float& tn)
{
    const float t1x = (xl - r.ori.x) * r.inv.x, t1y = (yl - r.ori.y) * r.inv.y, t1z = (zl - r.ori.z) * r.inv.z;
    const float t2x = (xh - r.ori.x) * r.inv.x, t2y = (yh - r.ori.y) * r.inv.y, t2z = (zh - r.ori.z) * r.inv.z;
    tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t1x, t2x), __builtin_fminf(t1y, t2y)), __builtin_fminf(t1z, t2z));
    const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t1x, t2x), __builtin_fmaxf(t1y, t2y)), __builtin_fmaxf(t1z, t2z));
    return (tf >= tn) & (tn < FMAX) & (tf >= 0.0f) & (tn < max_t);
}

// The leaf of the reference loop (intersect.inl:103-128): every primitive of the leaf `link` in
// index order, is_closer / update_if (update_if.h:27-79), multi_hit insertion, the mask intersector.
// Returns true when an any-hit ray found its hit (exit_traversal.h:49-56).
template <int KIND, bool COUNT, bool UV, class MultiList>
__device__ __forceinline__ bool leaf_loop(const float4* __restrict__ prims, uint32_t link, const ray_t& r, float max_t,
                                          bool any, float& best_t, uint32_t& best_prim, test_counts& cnt,
                                          hit_extra* hx, const MultiList* mh, const hit_mask_params* hm)
{
    uint32_t i = link & ~LEAF_BIT;
    for (;;)
    {
        float t, hu = 0.0f, hv = 0.0f;
        bool h;
        uint32_t flags, pid;
        if constexpr (KIND == KIND_TRI)
        {
            const float4* q = prims + 3u * i;
            float4 a = q[0], b = q[1], c = q[2];
            if (COUNT) { count_vmem(cnt, q); count_vmem(cnt, q + 1); count_vmem(cnt, q + 2); }
            h = isect_tri(r, a, b, c, t, hu, hv);
            pid = __float_as_uint(c.y);
            flags = __float_as_uint(c.w);
        }
        else
        {
            const float4* q = prims + 2u * i;
            float4 a = q[0], b = q[1];
            if (COUNT) { count_vmem(cnt, q); count_vmem(cnt, q + 1); }
            h = isect_sphere(r, a, t);
            pid = __float_as_uint(b.x);
            flags = __float_as_uint(b.z);
        }
        if (COUNT) { cnt.prim += 1; cnt.it_prim += 1; }
        bool closer = h & (t >= 0.0f) & (t < best_t) & (t < max_t);     // update_if.h:48-56, 73-79
        // mask intersector: hr.hit &= mask (a pure test, so applying it only where the hit would be
        // taken equals masking every primitive test)
        if constexpr (KIND == KIND_TRI)
            if (closer && hm != nullptr && hm->mask != nullptr) closer = mask_keep(*hm, pid, hu, hv);
        if (closer)
        {
            if constexpr (!std::is_void<MultiList>::value)
            {
                // multi_hit<N>: is_closer against the kept hits (multi_hit.h:221-244) = t below the
                // N-th kept t (best_t), then insert_sorted; best_t becomes the new N-th t
                best_t = mh->insert(t, pid, i, hu, hv);
            }
            else
            {
                best_t = t;
                best_prim = pid;
                if constexpr (UV) { hx->u = hu; hx->v = hv; hx->li = i; }   // hit_record.h:54-64
                if (any) return true;                            // exit_traversal.h:49-56
            }
        }
        if (flags & END_BIT) break;
        ++i;
    }
    return false;
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
//
// `resume` / `cap`: see the binary descent loop below (cap = ~0u: descend to the leaf in one call).
// `quad` lanes (any-hit rays with a finite ray, scene with 4-wide records) descend the 4-wide
// records instead: the same set of leaves is reached (vrh_quad.cpp), the order does not matter
// for an any-hit result, and the nearest hit entry is descended first.  If a record's hits could
// overflow the stack, the ray restarts on the binary records from `root` (still exact).
// CAPPED = false: an instance without the descent cap (`resume` is never set, `cap` is ignored): the
// kernels whose launches never cap a descent keep no per-lane visit counter
template <int KIND, bool COUNT, bool FAST, bool UV = false, class MultiList = void, bool CAPPED = true, class Stack>
__device__ __forceinline__ int ray_step(const float4* __restrict__ pairs, const float4* __restrict__ prims,
                                        const float4* __restrict__ quads, uint32_t root, bool& quad,
                                        const ray_t& r, float max_t, bool any, Stack& st,
                                        float& best_t, uint32_t& best_prim, test_counts& cnt,
                                        uint32_t& steps, uint32_t step_limit, uint32_t& resume, uint32_t cap,
                                        uint32_t flags, hit_extra* hx = nullptr, const MultiList* mh = nullptr,
                                        const hit_mask_params* hm = nullptr)
{
    // flags (render_params::step_flags): bit 0 pop on miss, bit 1 scalar fetch of wave-uniform pairs
    const bool pop_on_miss = (flags & 1u) != 0u;
    const bool scalar_uniform = SCALAR_UNIFORM && (flags & 2u) != 0u;
    // the tree was validated at upload (no cycles, links in range), so the descent terminates;
    // the guard below only bounds the number of outer iterations per ray
    uint32_t link;
    if (CAPPED && resume != NO_RESUME)
    {
        link = resume;
        resume = NO_RESUME;
    }
    else
    {
        if (st.empty()) return -1;
        if (++steps > step_limit) { cnt.aborted = true; return -1; }
        link = st.pop();
    }
    if (quad)
    {
        while (!(link & LEAF_BIT))
        {
            const float4* p = quads + 8u * link;
            const float4 xl = p[0], yl = p[1], zl = p[2], xh = p[3], yh = p[4], zh = p[5], lk = p[6];
            if (COUNT) count_vmem(cnt, p, 7u, VMEM_QUAD);
            const uint32_t k0 = __float_as_uint(lk.x), k1 = __float_as_uint(lk.y);
            const uint32_t k2 = __float_as_uint(lk.z), k3 = __float_as_uint(lk.w);
            float d0, d1, d2, d3;
            const bool h0 = quad_entry(xl.x, yl.x, zl.x, xh.x, yh.x, zh.x, r, max_t, d0) & (k0 != QUAD_NONE);
            const bool h1 = quad_entry(xl.y, yl.y, zl.y, xh.y, yh.y, zh.y, r, max_t, d1) & (k1 != QUAD_NONE);
            const bool h2 = quad_entry(xl.z, yl.z, zl.z, xh.z, yh.z, zh.z, r, max_t, d2) & (k2 != QUAD_NONE);
            const bool h3 = quad_entry(xl.w, yl.w, zl.w, xh.w, yh.w, zh.w, r, max_t, d3) & (k3 != QUAD_NONE);
            if (COUNT) cnt.box += 4;
            if (!(h0 | h1 | h2 | h3)) return st.empty() ? -1 : 0;
            if (!st.room(3u))
            {
                st.reset();
                st.push(root);
                quad = false;
                return 0;
            }
            // nearest hit entry first (ties -> lower index), the other hits pushed
            d0 = h0 ? d0 : INFINITY; d1 = h1 ? d1 : INFINITY; d2 = h2 ? d2 : INFINITY; d3 = h3 ? d3 : INFINITY;
#if VRH_SORTED_PUSH
            // all hit entries in distance order: a 4-element sorting network, the nearest descended,
            // the others pushed farthest first.  Only the descended entry keeps the old selection's tie
            // rule (equal distances -> the lower index); the order among the pushed entries is not
            // stable for ties (d = [1, 1, 0, 5] pushes index 1 ahead of 0) -- harmless for this
            // boolean any-hit walk, whose result does not depend on the visiting order, but not a
            // first-found hit record order
            float e0 = d0, e1 = d1, e2 = d2, e3 = d3;
            uint32_t c0 = k0, c1 = k1, c2 = k2, c3 = k3;
            auto cx = [](float& a, uint32_t& ka, float& b, uint32_t& kb) {
                const bool sw = b < a;
                const float t = sw ? b : a; b = sw ? a : b; a = t;
                const uint32_t u = sw ? kb : ka; kb = sw ? ka : kb; ka = u;
            };
            cx(e0, c0, e1, c1); cx(e2, c2, e3, c3); cx(e0, c0, e2, c2); cx(e1, c1, e3, c3); cx(e1, c1, e2, c2);
            if (e3 != INFINITY) st.push(c3);
            if (e2 != INFINITY) st.push(c2);
            if (e1 != INFINITY) st.push(c1);
            link = c0;
#else
            const bool a01 = d1 < d0, a23 = d3 < d2;
            const float m01 = a01 ? d1 : d0, m23 = a23 ? d3 : d2;
            const uint32_t j = (m23 < m01) ? (a23 ? 3u : 2u) : (a01 ? 1u : 0u);
            if (h0 & (j != 0u)) st.push(k0);
            if (h1 & (j != 1u)) st.push(k1);
            if (h2 & (j != 2u)) st.push(k2);
            if (h3 & (j != 3u)) st.push(k3);
            link = j == 0u ? k0 : j == 1u ? k1 : j == 2u ? k2 : k3;
#endif
        }
    }
    else for (uint32_t it = cap; !(link & LEAF_BIT); --it)
    {
        // at most `cap` inner visits per call: a lane still descending keeps its node in `resume`
        // and continues next call, so one long descent does not hold the whole wave
        if (CAPPED && it == 0u) { resume = link; return 0; }
        if (COUNT)
        {
            // one node for the whole wave? (counted once, by the first active lane)
            const uint64_t act = __ballot(true);
            const uint32_t lf = (uint32_t)__builtin_amdgcn_readfirstlane((int)link);
            const bool uni = __ballot(link != lf) == 0ull;
            if (uni && __lane_id() == (uint32_t)__builtin_ctzll(act)) cnt.w_uni += 1;
        }
        // The vector-memory data path (TD) is the kernel's busiest unit (profiles/pmc_mem.json), and
        // in about a third of the wave-level descent iterations every active lane fetches the SAME
        // pair (upper tree levels): those fetch it once through the scalar cache instead (s_load on
        // a wave-uniform address, constant address space), the rest per lane (56 of the record's
        // 64 B: two boxes, two links).  Same bytes either way.  (Extending this to waves whose lanes
        // want 2 or 3 distinct pairs -- one scalar load each, selected per lane -- measured 2-10 %
        // slower: profiles/r01/ab_peel/.)
        float4 q0, q1, q2;
        float2 q3;
        typedef const __attribute__((address_space(4))) float cfloat;
        const uint32_t lf = (uint32_t)__builtin_amdgcn_readfirstlane((int)link);
        const uint64_t rest1 = __ballot(link != lf);
        if (scalar_uniform && rest1 == 0ull)
        {
            cfloat* cp = (cfloat*)(const float*)(pairs) + 16u * lf;
            q0 = make_float4(cp[0], cp[1], cp[2], cp[3]);
            q1 = make_float4(cp[4], cp[5], cp[6], cp[7]);
            q2 = make_float4(cp[8], cp[9], cp[10], cp[11]);
            q3 = make_float2(cp[12], cp[13]);
        }
        else
        {
            const float4* p = pairs + 4u * link;
            q0 = p[0]; q1 = p[1]; q2 = p[2];
            q3 = *reinterpret_cast<const float2*>(p + 3);
            if (COUNT) count_vmem(cnt, p, 4u, VMEM_PAIR);      // one 64-B record: 4 loads, one line each
        }
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
        if (!(b0 | b1))
        {
            // pop_on_miss: take the next stack entry and keep descending in this call (the lane's
            // own sequence of operations is unchanged -- it only does in one wave step what it
            // would otherwise do in the next one)
            if (!pop_on_miss || st.empty()) return st.empty() ? -1 : 0;
            if (++steps > step_limit) { cnt.aborted = true; return -1; }
            link = st.pop();
            continue;
        }
        link = go0 ? l0 : l1;
    }
    if (leaf_loop<KIND, COUNT, UV, MultiList>(prims, link, r, max_t, any, best_t, best_prim, cnt, hx, mh, hm)) return 1;
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

// per-frame sampler offset: the reference seeds its sampler anew every frame (cuda_sched.inl:38-45,
// 79; ao/main.cpp passes ++frame_num, :245).  The Appendix-A counter of frame n is shifted by
// n * 0x9E3779B1 (u32 wrap); frame 0 keeps the Appendix-A counter exactly (the parity fixtures).
__host__ __device__ __forceinline__ uint32_t frame_salt(uint32_t frame_num) { return frame_num * 0x9E3779B1u; }

// Appendix A Malley sample s of pixel p -> direction in the (u, v, n) basis (ao/main.cpp:218-226)
__device__ __forceinline__ f3 ao_direction(uint32_t p, uint32_t s, f3 bu, f3 bv, f3 n, uint32_t salt)
{
    float sx = 0.0f, sy = 0.0f;
    for (uint32_t k = 0; k < 16; ++k)
    {
        uint32_t ctr = ((p * 8u + s) * 16u + k) * 2u + salt;
        float xa = 2.0f * uniform01(ctr) - 1.0f;
        float ya = 2.0f * uniform01(ctr + 1u) - 1.0f;
        if (xa * xa + ya * ya < 1.0f) { sx = xa; sy = ya; break; }
    }
    float sz = __builtin_sqrtf(tmax(0.0f, 1.0f - sx * sx - sy * sy));
    return normalize((sx * bu + sy * bv) + sz * n);
}

} // namespace dev
} // namespace vrh
