// include/visionaray_hip/hip_kernels.h -- user kernels and custom intersectors on the GPU.
//
// hip_sched::frame runs the built-in kernels through the C ABI.  A translation unit compiled by
// hipcc that includes this header can also hand it its OWN kernel -- any callable
//
//     result_record<float> kernel(ray r)                    (or (ray, hip_sampler&) / (ray, x, y))
//
// as cuda_sched runs one (cuda_sched.inl:53-153, sched_common.h:78-120): one GPU thread per pixel of
// the scissor box, the reference's pinhole primary ray, the returned colour stored in the render
// target.  Inside, the reference's traversal intrinsics work on the device BVHs:
//
//     closest_hit(ray, begin, end [, isect])     traverse_linear.inl:286-329
//     any_hit(ray, begin, end, max_t [, isect])  traverse_linear.inl:232-283
//
// over a range of hip_bvh_ref (hip_index_bvh::ref(), the bvh_ref of bvh.h:344-350) or of plain
// primitives (basic_triangle<3,float> / basic_sphere<float> arrays in device memory), with the
// default intersector or a basic_intersector subclass (intersector.h:24-119) -- e.g. the
// intersector example's mask_intersector (examples/intersector/main.cpp:251-330) compiles unchanged
// against these types.  The BVH walk is libvrh's (visionaray_hip/detail/vrh_device.h: the 64-B pair
// records, box_pair's slab test, near child first with ties to child 1, far child pushed, leaf
// primitives in index order), with the primitive test handed to the intersector, so the default
// intersector gives the built-in kernels' bits.
//
// Device lambdas capture by value ([=]): they run on the GPU.  The traversal stack lives in LDS
// (VRH_USER_STACK entries per thread); BVHs deeper than that are rejected by hip_bvh_ref checks.
#pragma once

#if !defined(__HIP__)
#error "visionaray_hip/hip_kernels.h is device code: compile this translation unit with hipcc"
#endif

#include <hip/hip_runtime.h>

#include "standalone.h"
#include "detail/vrh_device.h"

#include <array>
#include <cassert>
#include <cfloat>
#include <cstring>
#include <stdexcept>
#include <type_traits>
#include <utility>

#ifndef VRH_USER_STACK
// traversal stack entries per thread (LDS), >= the deepest BVH traversed.  32 = the reference's own
// detail::stack<32> (stack.h:17-51, usable depth 31); 64 entries (round 1) cost a 64-thread block
// 16 KB of LDS, which held a CU to 10 resident waves (2.5 per SIMD) -- 32 lets the registers bound
// it (4 waves per SIMD for the AO kernel)
#define VRH_USER_STACK 32
#endif

namespace visionaray
{

//-------------------------------------------------------------------------------------------------
// SIMD vocabulary at width 1 (math/simd/type_traits.h): the reference's kernels are written for
// float / float4 / float8 alike; one GPU lane is width 1.  mask_type_t<float> is a one-lane mask
// that, like mask4 / mask8, can be built from an array of bools (the intersector example builds
// its mask with Mask(hits) from bool hits[N]).
//

namespace simd
{
struct mask1
{
    bool v = false;
    VRH_FUNC mask1() = default;
    VRH_FUNC mask1(bool b) : v(b) {}
    VRH_FUNC explicit mask1(bool const* p) : v(p[0]) {}
    VRH_FUNC operator bool() const { return v; }
};
template <typename T> struct num_elements { static constexpr int value = 1; };
template <typename T> struct mask_type { using type = mask1; };
template <typename T> using mask_type_t = typename mask_type<T>::type;
template <typename T> struct int_type { using type = int; };
template <typename T> using int_type_t = typename int_type<T>::type;
template <typename T> struct is_simd_vector : std::false_type {};
} // simd

VRH_FUNC inline bool any(bool b) { return b; }
VRH_FUNC inline bool all(bool b) { return b; }
template <typename T> VRH_FUNC inline T select(bool m, T const& a, T const& b) { return m ? a : b; }

// math.h:461-475 lerp(a, b, c, u, v) in the reference's operation order
template <typename T, typename S>
VRH_FUNC inline T lerp(T const& a, T const& b, T const& c, S const& u, S const& v)
{
    auto s2 = c * v;
    auto s3 = b * u;
    auto s1 = a * (S(1.0f) - (u + v));
    return s1 + s2 + s3;
}

// vector3.inl:357-367 make_orthonormal_basis(u, v, w): w is the given normal
template <typename T>
VRH_FUNC inline void make_orthonormal_basis(vector<3, T>& u, vector<3, T>& v, vector<3, T> const& w)
{
    v = std::abs(w.x) > std::abs(w.y) ? normalize(vector<3, T>(-w.z, T(0.0), w.x))
                                      : normalize(vector<3, T>(T(0.0), w.z, -w.y));
    u = cross(v, w);
}

//-------------------------------------------------------------------------------------------------
// hit records (math/intersect.h:87-111, detail/bvh/hit_record.h, result_record.h)
//

template <typename R, typename Base> struct hit_record;

template <typename T>
struct hit_record<basic_ray<T>, primitive<unsigned>>
{
    using scalar_type = T;
    using int_type = int;
    using mask_type = bool;
    VRH_FUNC hit_record() : hit(false), prim_id(0), geom_id(0), t(FLT_MAX), u(0.0f), v(0.0f) {}
    bool hit;
    int prim_id;
    int geom_id;
    T t;
    vector<3, T> isect_pos;
    T u;
    T v;
};

// hit_record_bvh (detail/bvh/hit_record.h:20-64): + the leaf-order index of the hit primitive
template <typename Base>
struct hit_record_bvh : Base
{
    VRH_FUNC hit_record_bvh() = default;
    VRH_FUNC hit_record_bvh(Base const& b, unsigned i) : Base(b), primitive_list_index(i) {}
    unsigned primitive_list_index = 0;
};

template <typename T>
class result_record
{
public:
    using scalar_type = T;
    using color_type = vector<4, T>;
    VRH_FUNC result_record() : hit(false), color(T(0.0)), depth(T(0.0)), isect_pos(T(0.0)) {}
    bool hit;
    color_type color;
    T depth;
    vector<3, T> isect_pos;
};

// width-1 unpack (vector*.inl unpack, hit_record.h:103-130): the one lane
template <typename T>
VRH_FUNC inline std::array<T, 1> unpack(T const& v) { return std::array<T, 1>{ { v } }; }

//-------------------------------------------------------------------------------------------------
// ray / primitive tests (math/intersect.h:122-221): libvrh's arithmetic, the reference's record
//

namespace hip_detail
{
__device__ inline vrh::dev::ray_t dev_ray(basic_ray<float> const& r)
{
    return vrh::dev::make_ray(vrh::dev::mk3(r.ori.x, r.ori.y, r.ori.z), vrh::dev::mk3(r.dir.x, r.dir.y, r.dir.z));
}
} // hip_detail

__device__ inline hit_record<basic_ray<float>, primitive<unsigned>> intersect(basic_ray<float> const& ray,
                                                                               basic_triangle<3, float, unsigned> const& tri)
{
    hit_record<basic_ray<float>, primitive<unsigned>> hr;
    const float4 a = make_float4(tri.v1.x, tri.v1.y, tri.v1.z, tri.e1.x);
    const float4 b = make_float4(tri.e1.y, tri.e1.z, tri.e2.x, tri.e2.y);
    const float4 c = make_float4(tri.e2.z, 0.0f, 0.0f, 0.0f);
    float t, u, v;
    hr.hit = vrh::dev::isect_tri(hip_detail::dev_ray(ray), a, b, c, t, u, v);
    hr.t = -1.0f;
    if (hr.hit)            // the reference fills these only for a hit (intersect.h:172-177)
    {
        hr.prim_id = int(tri.prim_id);
        hr.geom_id = int(tri.geom_id);
        hr.t = t;
        hr.u = u;
        hr.v = v;
    }
    return hr;
}

__device__ inline hit_record<basic_ray<float>, primitive<unsigned>> intersect(basic_ray<float> const& ray,
                                                                               basic_sphere<float, unsigned> const& s)
{
    hit_record<basic_ray<float>, primitive<unsigned>> hr;
    float t;
    hr.hit = vrh::dev::isect_sphere(hip_detail::dev_ray(ray), make_float4(s.center.x, s.center.y, s.center.z, s.radius), t);
    hr.prim_id = int(s.prim_id);
    hr.geom_id = int(s.geom_id);
    hr.t = t;
    return hr;
}

// update_if.h:48-79
template <typename HR>
VRH_FUNC inline bool is_closer(HR const& query, HR const& reference, float max_t)
{
    return query.hit && query.t >= 0.0f && query.t < reference.t && query.t < max_t;
}

//-------------------------------------------------------------------------------------------------
// basic_intersector (intersector.h:24-119): the CRTP base of custom intersectors.  A subclass
// overrides operator()(ray, primitive) for the primitive types it cares about; everything else
// falls back to intersect().
//

template <typename Derived>
struct basic_intersector
{
    template <size_t N>
    using multi_hit_max = std::integral_constant<size_t, N>;

    template <typename R, typename P, typename... Args>
    __device__ auto operator()(R const& ray, P const& prim, Args&&... args)
        -> decltype(intersect(ray, prim, std::forward<Args>(args)...))
    {
        return intersect(ray, prim);
    }
};

struct default_intersector : basic_intersector<default_intersector>
{
};

//-------------------------------------------------------------------------------------------------
// BVH traversal with an intersector: intersect<ClosestHit / AnyHit>(ray, bvh, isect)
// (detail/bvh/intersect.inl:25-134) over libvrh's device layout
//

namespace hip_detail
{
// the leaf primitive i of the device layout, rebuilt as the reference's primitive object
__device__ inline basic_triangle<3, float> leaf_triangle(const float4* prims, uint32_t i, uint32_t& flags)
{
    const float4 a = prims[3u * i], b = prims[3u * i + 1u], c = prims[3u * i + 2u];
    basic_triangle<3, float> t;
    t.v1 = vec3(a.x, a.y, a.z);
    t.e1 = vec3(a.w, b.x, b.y);
    t.e2 = vec3(b.z, b.w, c.x);
    t.prim_id = __float_as_uint(c.y);
    t.geom_id = __float_as_uint(c.z);
    flags = __float_as_uint(c.w);
    return t;
}

__device__ inline basic_sphere<float> leaf_sphere(const float4* prims, uint32_t i, uint32_t& flags)
{
    const float4 a = prims[2u * i], b = prims[2u * i + 1u];
    basic_sphere<float> s;
    s.center = vec3(a.x, a.y, a.z);
    s.radius = a.w;
    s.prim_id = __float_as_uint(b.x);
    s.geom_id = __float_as_uint(b.y);
    flags = __float_as_uint(b.z);
    return s;
}

// the per-thread traversal stack: a column of the block's dynamic LDS (hip_sched's user-kernel
// launch provides VRH_USER_STACK entries per thread)
__device__ inline vrh::dev::lds_stack user_stack()
{
    extern __shared__ uint32_t vrh_user_smem[];
    const uint32_t nthreads = blockDim.x * blockDim.y * blockDim.z;
    const uint32_t tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
    vrh::dev::lds_stack st;
    st.mem = vrh_user_smem;
    st.base = tid;
    st.stride = nthreads;
    st.top = tid;
    st.end = tid + VRH_USER_STACK * nthreads;
    st.lim = st.end;
    st.spill = nullptr;          // checked_ref: the BVH fits the LDS stack
    return st;
}

// the hit record of intersect(ray, primitive) -- and of every intersector built on it
using prim_record = hit_record<basic_ray<float>, primitive<unsigned>>;
using bvh_record = hit_record_bvh<prim_record>;

template <bool Any, bool FAST, typename Isect>
__device__ inline bvh_record traverse_bvh_slab(basic_ray<float> const& ray, vrh_scene_view const& b, Isect& isect, float max_t)
{
    using HR = prim_record;
    hit_record_bvh<HR> result;
    // the LDS stack holds VRH_USER_STACK entries: a deeper BVH (not passed through checked_ref)
    // is not traversed -- a miss, never an out-of-bounds stack write
    if (b.max_depth >= VRH_USER_STACK) return result;
    const vrh::dev::ray_t r = dev_ray(ray);
    const float4* pairs = static_cast<const float4*>(b.pairs);
    const float4* prims = static_cast<const float4*>(b.prims);
    vrh::dev::lds_stack st = user_stack();
    st.push(b.root);
    while (!st.empty())
    {
        uint32_t link = st.pop();
        bool at_leaf = true;
        while (!(link & vrh::dev::LEAF_BIT))
        {
            const float4* p = pairs + 4u * link;
            const float4 q0 = p[0], q1 = p[1], q2 = p[2];
            const float2 q3 = *reinterpret_cast<const float2*>(p + 3);
            bool b0, b1;
            float tn0, tn1;
            vrh::dev::box_pair<FAST>(q0, q1, q2, r, result.t, max_t, b0, b1, tn0, tn1);
            const uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
            if (!(b0 | b1)) { at_leaf = false; break; }                               // pop
            const bool go0 = (b0 & b1) ? (tn0 < tn1) : b0;                             // ties -> child 1
            if (b0 & b1) st.push(go0 ? l1 : l0);
            link = go0 ? l0 : l1;
        }
        if (!at_leaf) continue;
        // the leaf: every primitive in index order, is_closer / update_if (intersect.inl:103-128)
        for (uint32_t i = link & ~vrh::dev::LEAF_BIT;; ++i)
        {
            uint32_t flags;
            HR hr;
            if (b.prim_kind == VRH_PRIM_TRI64) hr = isect(ray, leaf_triangle(prims, i, flags));
            else hr = isect(ray, leaf_sphere(prims, i, flags));
            if (is_closer(hr, static_cast<HR const&>(result), max_t))
            {
                result = hit_record_bvh<HR>(hr, i);
                if (Any) return result;                   // exit_traversal.h:49-56
            }
            if (flags & vrh::dev::END_BIT) break;
        }
    }
    return result;
}

template <bool Any, typename Isect>
__device__ inline bvh_record traverse_bvh(basic_ray<float> const& ray, vrh_scene_view const& b, Isect& isect, float max_t)
{
    // the hardware min/max slab test where it is provably identical (vrh_device.h box_pair)
    if (b.finite_bounds && vrh::dev::finite_ray(dev_ray(ray)))
        return traverse_bvh_slab<Any, true>(ray, b, isect, max_t);
    return traverse_bvh_slab<Any, false>(ray, b, isect, max_t);
}

template <typename It>
using range_value_t = typename std::decay<decltype(*std::declval<It>())>::type;
} // hip_detail

// closest_hit / any_hit over [begin, end) of hip_bvh_ref (traverse_linear.inl:76-141): every BVH on
// its own with the same max_t, merged by update_if(result, hr, is_closer(hr, result, max_t));
// any_hit stops at the first BVH with a hit
template <typename It, typename Isect,
          typename = typename std::enable_if<std::is_same<hip_detail::range_value_t<It>, hip_bvh_ref>::value>::type>
__device__ inline hip_detail::bvh_record closest_hit(basic_ray<float> const& ray, It begin, It end, Isect& isect)
{
    hip_detail::bvh_record result;
    for (It it = begin; it != end; ++it)
    {
        auto hr = hip_detail::traverse_bvh<false>(ray, it->view, isect, FLT_MAX);
        if (is_closer(hr, result, FLT_MAX)) result = hr;
    }
    return result;
}

template <typename It, typename Isect,
          typename = typename std::enable_if<std::is_same<hip_detail::range_value_t<It>, hip_bvh_ref>::value>::type>
__device__ inline hip_detail::bvh_record any_hit(basic_ray<float> const& ray, It begin, It end, float max_t, Isect& isect)
{
    hip_detail::bvh_record result;
    for (It it = begin; it != end; ++it)
    {
        auto hr = hip_detail::traverse_bvh<true>(ray, it->view, isect, max_t);
        if (is_closer(hr, result, max_t)) result = hr;
        if (result.hit) return result;
    }
    return result;
}

// the same over [begin, end) of primitives (traverse_linear.inl:25-62): a linear scan
template <typename It, typename Isect,
          typename = typename std::enable_if<!std::is_same<hip_detail::range_value_t<It>, hip_bvh_ref>::value>::type,
          typename = void>
__device__ inline auto closest_hit(basic_ray<float> const& ray, It begin, It end, Isect& isect)
{
    using HR = decltype(isect(ray, *begin));
    HR result;
    for (It it = begin; it != end; ++it)
    {
        auto hr = isect(ray, *it);
        if (is_closer(hr, result, FLT_MAX)) result = hr;
    }
    return result;
}

template <typename It, typename Isect,
          typename = typename std::enable_if<!std::is_same<hip_detail::range_value_t<It>, hip_bvh_ref>::value>::type,
          typename = void>
__device__ inline auto any_hit(basic_ray<float> const& ray, It begin, It end, float max_t, Isect& isect)
{
    using HR = decltype(isect(ray, *begin));
    HR result;
    for (It it = begin; it != end; ++it)
    {
        auto hr = isect(ray, *it);
        if (is_closer(hr, result, max_t)) { result = hr; return result; }
    }
    return result;
}

// the default intersector (traverse_linear.inl:286-329, 232-283 without an intersector argument)
template <typename It>
__device__ inline auto closest_hit(basic_ray<float> const& ray, It begin, It end)
{
    default_intersector isect;
    return closest_hit(ray, begin, end, isect);
}

template <typename It>
__device__ inline auto any_hit(basic_ray<float> const& ray, It begin, It end, float max_t)
{
    default_intersector isect;
    return any_hit(ray, begin, end, max_t, isect);
}

// get_tex_coord(tex_coords, hr) (get_tex_coord.h:25-38, 128-136): lerp of the hit triangle's
// three tex coords with the hit's barycentrics
template <typename TexCoords, typename HR>
VRH_FUNC inline auto get_tex_coord(TexCoords tex_coords, HR const& hr)
    -> typename std::decay<decltype(tex_coords[0])>::type
{
    return lerp(tex_coords[hr.prim_id * 3], tex_coords[hr.prim_id * 3 + 1], tex_coords[hr.prim_id * 3 + 2], hr.u, hr.v);
}

// get_normal(normals, hr) for normals_per_face_binding (get_normal.h:26-37)
template <typename Normals, typename HR>
VRH_FUNC inline vec3 get_normal(Normals normals, HR const& hr)
{
    return normals[hr.prim_id];
}

//-------------------------------------------------------------------------------------------------
// Samplers.  The reference seeds a random_sampler per pixel from the clock (cuda_sched.inl:38-45,
// 79); here every draw is the SURVEY.md Appendix-A counter hash, so frames are reproducible:
//   hip_sampler::next()        uniform [0, 1) from the counter (pixel, frame number, draw)
//   hip_ao_sample(p, s, frame) the built-in AO kernel's cosine-hemisphere sample s of pixel p
//                              (Malley disk point, z = sqrt(1 - x^2 - y^2)) -- the same sample set
//                              as VRH_KERNEL_AO, so a user AO kernel reproduces its frames.
//

struct hip_sampler
{
    uint32_t ctr;
    __device__ explicit hip_sampler(uint32_t pixel, uint32_t frame_num)
        : ctr(vrh::dev::wang(pixel * 0x9E3779B1u ^ vrh::dev::frame_salt(frame_num + 1u)))
    {
    }
    __device__ float next() { return vrh::dev::uniform01(ctr++); }
};

__device__ inline vec3 hip_ao_sample(uint32_t pixel, uint32_t s, uint32_t frame_num)
{
    // ao_direction's point on the disk (vrh_device.h), before the basis is applied
    float sx = 0.0f, sy = 0.0f;
    const uint32_t salt = vrh::dev::frame_salt(frame_num);
    for (uint32_t k = 0; k < 16; ++k)
    {
        const uint32_t c = ((pixel * 8u + s) * 16u + k) * 2u + salt;
        const float xa = 2.0f * vrh::dev::uniform01(c) - 1.0f;
        const float ya = 2.0f * vrh::dev::uniform01(c + 1u) - 1.0f;
        if (xa * xa + ya * ya < 1.0f) { sx = xa; sy = ya; break; }
    }
    return vec3(sx, sy, __builtin_sqrtf(vrh::dev::tmax(0.0f, 1.0f - sx * sx - sy * sy)));
}

//-------------------------------------------------------------------------------------------------
// The launch: one thread per pixel, 8 x 8 threads (one wave) per block, dynamic LDS for the
// traversal stacks; cuda_sched.inl:53-99 with sample_pixel's uniform store (colour, and the depth
// into the target's t buffer when the result carries one).
//

namespace hip_detail
{
struct user_frame
{
    vrh_camera cam;
    float4* color;
    float* t;
    uint32_t width, height, frame_num;
    uint32_t x0, y0, x1, y1;      // scissor box, exclusive right / bottom edges
    uint32_t matrix_cam;          // sched_params with camera matrices: their inverses (column-major)
    float inv_view[16], inv_proj[16];
};

// the primary ray through image position (fx, fy) (the pixel plus the sampler's offset):
// sched_common.h:130-150 (pinhole basis) or :152-176 (camera matrices), the built-in kernels' arithmetic
__device__ inline basic_ray<float> user_primary_ray(user_frame const& f, float fx, float fy)
{
    const float u = 2.0f * (fx + 0.5f) / (float)f.width - 1.0f;
    const float v = 2.0f * (fy + 0.5f) / (float)f.height - 1.0f;
    if (f.matrix_cam)
    {
        float a[4], b[4], o[4], d[4];
        for (int r = 0; r < 4; ++r)
        {
            a[r] = f.inv_proj[r] * u + f.inv_proj[4 + r] * v + f.inv_proj[8 + r] * -1.0f + f.inv_proj[12 + r] * 1.0f;
            b[r] = f.inv_proj[r] * u + f.inv_proj[4 + r] * v + f.inv_proj[8 + r] * 1.0f + f.inv_proj[12 + r] * 1.0f;
        }
        for (int r = 0; r < 4; ++r)
        {
            o[r] = f.inv_view[r] * a[0] + f.inv_view[4 + r] * a[1] + f.inv_view[8 + r] * a[2] + f.inv_view[12 + r] * a[3];
            d[r] = f.inv_view[r] * b[0] + f.inv_view[4 + r] * b[1] + f.inv_view[8 + r] * b[2] + f.inv_view[12 + r] * b[3];
        }
        const vec3 ori(o[0] / o[3], o[1] / o[3], o[2] / o[3]);
        const vec3 far(d[0] / d[3], d[1] / d[3], d[2] / d[3]);
        return basic_ray<float>(ori, normalize(far - ori));
    }
    const vec3 cu(f.cam.cam_u[0], f.cam.cam_u[1], f.cam.cam_u[2]);
    const vec3 cv(f.cam.cam_v[0], f.cam.cam_v[1], f.cam.cam_v[2]);
    const vec3 cw(f.cam.cam_w[0], f.cam.cam_w[1], f.cam.cam_w[2]);
    const vec3 eye(f.cam.eye[0], f.cam.eye[1], f.cam.eye[2]);
    return basic_ray<float>(eye, normalize((cu * u + cv * v) + cw));
}

// sched_common.h:78-120 invoke_kernel: kernel(r), kernel(r, sampler) or kernel(r, x, y), in that
// order of preference (the int / long / ... tag ranks the overloads)
template <typename K, typename S>
__device__ inline auto invoke_kernel(K& kernel, basic_ray<float> const& r, S&, unsigned, unsigned, int) -> decltype(kernel(r))
{
    return kernel(r);
}
template <typename K, typename S>
__device__ inline auto invoke_kernel(K& kernel, basic_ray<float> const& r, S& samp, unsigned, unsigned, long)
    -> decltype(kernel(r, samp))
{
    return kernel(r, samp);
}
template <typename K, typename S>
__device__ inline auto invoke_kernel(K& kernel, basic_ray<float> const& r, S&, unsigned x, unsigned y, ...)
    -> decltype(kernel(r, x, y))
{
    return kernel(r, x, y);
}

// sched_params with an intersector (scheduler.h:33-45, 177-193: make_sched_params(sampler, cam, rt,
// isect)): the kernel is called as kernel(isect, r ...) (sched_common.h:786-818
// call_kernel_with_intersector); the intersector is copied into the launch (it holds device pointers)
template <typename K, typename I>
struct call_with_intersector
{
    K kernel;
    I isect;

    template <typename... A>
    __device__ auto operator()(A&&... a) -> decltype(kernel(isect, std::forward<A>(a)...))
    {
        return kernel(isect, std::forward<A>(a)...);
    }
};

template <typename T, typename = void> struct has_depth : std::false_type {};
template <typename T> struct has_depth<T, decltype((void)std::declval<T>().depth)> : std::true_type {};

template <typename K, uint32_t SK = VRH_SAMPLER_UNIFORM, uint32_t SN = 1>
__global__ __launch_bounds__(64) void user_render(K kernel, user_frame f)
{
    const uint32_t x = blockIdx.x * 8u + threadIdx.x;
    const uint32_t y = blockIdx.y * 8u + threadIdx.y;
    if (x < f.x0 || y < f.y0 || x >= f.x1 || y >= f.y1) return;
    hip_sampler samp(y * f.width + x, f.frame_num);
    const size_t o = size_t(y) * f.width + x;
    if constexpr (SK == VRH_SAMPLER_UNIFORM)
    {
        // sched_common.h:130-176 make_primary_ray_impl (uniform pixel sampler), as the built-in kernels
        auto res = invoke_kernel(kernel, user_primary_ray(f, (float)x, (float)y), samp, x, y, 0);
        if (f.color) f.color[o] = make_float4(res.color.x, res.color.y, res.color.z, res.color.w);
        if constexpr (has_depth<decltype(res)>::value)
            if (f.t) f.t[o] = res.depth;
    }
    else
    {
        // the jittered / jittered_blend / ssaa<N> samplers (sched_common.h:196-300, 440-720), with the
        // jitter draws and offset tables of vrh.h vrh_pixel_sampler
        auto ray_at = [&](float ox, float oy) { return user_primary_ray(f, (float)x + ox, (float)y + oy); };
        if constexpr (SK == VRH_SAMPLER_SSAA)
        {
            constexpr float off2[2][2] = { { -0.25f, -0.25f }, { 0.25f, 0.25f } };
            constexpr float off4[4][2] = { { -0.125f, -0.375f }, { 0.375f, -0.125f }, { 0.125f, 0.375f }, { -0.375f, 0.125f } };
            constexpr float off8[8][2] = { { -0.125f, -0.4375f }, { 0.375f, -0.3125f }, { -0.375f, -0.1875f }, { 0.125f, -0.0625f },
                                           { -0.125f, 0.0625f }, { 0.375f, 0.1825f }, { -0.375f, 0.3125f }, { 0.125f, 0.4375f } };
            const float a = 1.0f / float(SN);
            float4 d = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll 1
            for (uint32_t i = 0; i < SN; ++i)
            {
                const float ox = SN == 2 ? off2[i][0] : SN == 4 ? off4[i][0] : off8[i][0];
                const float oy = SN == 2 ? off2[i][1] : SN == 4 ? off4[i][1] : off8[i][1];
                auto res = invoke_kernel(kernel, ray_at(ox, oy), samp, x, y, 0);
                d = make_float4(res.color.x * a + d.x * 1.0f, res.color.y * a + d.y * 1.0f,
                                res.color.z * a + d.z * 1.0f, res.color.w * a + d.w * 1.0f);
                if constexpr (has_depth<decltype(res)>::value)
                    if (f.t) f.t[o] = res.depth;
            }
            if (f.color) f.color[o] = d;
        }
        else
        {
            const uint32_t k = (y * f.width + x) * 2u + 0x632BE5ABu + f.frame_num * 0x68E31DA4u;
            const float oy = vrh::dev::uniform01(k) - 0.5f, ox = vrh::dev::uniform01(k + 1u) - 0.5f;
            auto res = invoke_kernel(kernel, ray_at(ox, oy), samp, x, y, 0);
            float4 c = make_float4(res.color.x, res.color.y, res.color.z, res.color.w);
            if constexpr (SK == VRH_SAMPLER_JITTERED_BLEND)
            {
                const float a = 1.0f / float(f.frame_num), b = 1.0f - a;
                if (f.color)
                {
                    const float4 d = f.color[o];
                    c = make_float4(c.x * a + d.x * b, c.y * a + d.y * b, c.z * a + d.z * b, c.w * a + d.w * b);
                }
            }
            if (f.color) f.color[o] = c;
            if constexpr (has_depth<decltype(res)>::value)
                if (f.t) f.t[o] = res.depth;
        }
    }
}
} // hip_detail

namespace hip_detail
{
template <typename K>
struct user_kernels<K, typename std::enable_if<!std::is_same<K, hip_builtin_kernel>::value>::type>
{
    static constexpr bool available = true;

    template <typename SP>
    static void frame(hip_context& ctx, K const& kernel, SP& sparams, unsigned frame_num)
    {
        using PS = sampler_desc<typename sampler_of<SP>::type>;
        static_assert(PS::supported, "hip_sched: the pixel samplers are uniform_type, jittered_type, "
                                     "jittered_blend_type and ssaa_type<2 / 4 / 8>");
        auto& rt = sparams.rt;
        user_frame f{};
        if constexpr (has_camera_matrices<SP>::value)
        {
            // sched_params<Base, MT, RT, PxSamplerT> (scheduler.h:76-96): the host inverses of
            // vrh_render_view (matrix4.inl:209-244)
            f.matrix_cam = 1u;
            vrh_matrix_inverse(sparams.view_matrix.data(), f.inv_view);
            vrh_matrix_inverse(sparams.proj_matrix.data(), f.inv_proj);
        }
        else
        {
            auto const& cam = sparams.cam;
            float eye[3] = { cam.eye().x, cam.eye().y, cam.eye().z };
            float center[3] = { cam.center().x, cam.center().y, cam.center().z };
            float up[3] = { cam.up().x, cam.up().y, cam.up().z };
            check(vrh_make_camera(eye, center, up, cam.fovy(), cam.aspect(), uint32_t(rt.width()), uint32_t(rt.height()),
                                  &f.cam),
                  "vrh_make_camera");
        }
        set_scissor(sparams, f.cam);
        f.width = uint32_t(rt.width());
        f.height = uint32_t(rt.height());
        f.frame_num = frame_num;
        const uint32_t* sc = f.cam.scissor;
        const bool whole = sc[0] == 0 && sc[1] == 0 && sc[2] == 0 && sc[3] == 0;
        f.x0 = whole ? 0u : sc[0];
        f.y0 = whole ? 0u : sc[1];
        f.x1 = whole ? f.width : (sc[2] < f.width ? sc[2] : f.width);
        f.y1 = whole ? f.height : (sc[3] < f.height ? sc[3] : f.height);
        auto ref = rt.ref();
        f.color = reinterpret_cast<float4*>(ref.color);
        f.t = ref.t;
        int dev = 0, prev = 0;
        void* stream = nullptr;
        check(vrh_ctx_get_stream(ctx.get(), &dev, &stream), "vrh_ctx_get_stream");
        if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(dev) != hipSuccess) throw hip_error("hipSetDevice", VRH_ERR_HIP);
        rt.begin_frame();
        hipError_t e = hipSuccess;
        if (f.x1 > f.x0 && f.y1 > f.y0)
        {
            const dim3 grid((f.width + 7u) / 8u, (f.height + 7u) / 8u);
            const size_t lds = size_t(64) * VRH_USER_STACK * sizeof(uint32_t);
            if constexpr (has_sched_intersector<SP>::value)
            {
                using I = typename std::decay<decltype(sparams.intersector)>::type;
                using C = call_with_intersector<K, I>;
                hipLaunchKernelGGL((user_render<C, PS::kind, PS::count>), grid, dim3(8, 8), lds,
                                   static_cast<hipStream_t>(stream), C{ kernel, sparams.intersector }, f);
            }
            else
                hipLaunchKernelGGL((user_render<K, PS::kind, PS::count>), grid, dim3(8, 8), lds,
                                   static_cast<hipStream_t>(stream), kernel, f);
            e = hipGetLastError();
        }
        (void)hipSetDevice(prev);        // the caller's current device is left as it was
        if (e != hipSuccess) throw std::runtime_error(std::string("hip_sched::frame: user kernel launch: ") + hipGetErrorString(e));
        rt.end_frame();
    }
};
} // hip_detail

// the user traversal stack holds VRH_USER_STACK entries: a deeper BVH cannot be traversed (the
// device code then reports a miss); checked_ref rejects it on the host instead
inline hip_bvh_ref checked_ref(hip_bvh_ref r)
{
    if (r.view.max_depth >= VRH_USER_STACK)
        throw hip_error("hip_bvh_ref: BVH deeper than VRH_USER_STACK", VRH_ERR_UNSUPPORTED);
    return r;
}

} // visionaray
