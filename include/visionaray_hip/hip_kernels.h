// include/visionaray_hip/hip_kernels.h -- user kernels and custom intersectors on the GPU.
//
// hip_sched::frame runs the built-in kernels through the C ABI.  A translation unit compiled by
// hipcc that includes this header can also hand it its OWN kernel -- any callable
//
//     result_record<float> kernel(ray r)     (or (ray, random_sampler<float>&) / (ray, x, y))
//
// as cuda_sched runs one (cuda_sched.inl:53-153, sched_common.h:78-120): one GPU thread per pixel of
// the scissor box, the reference's pinhole primary ray, the returned colour stored in the render
// target.  A kernel taking a sampler gets a random_sampler<float> seeded per pixel (below).
// Inside, the reference's traversal intrinsics work on the device BVHs:
//
//     closest_hit(ray, begin, end [, isect])     traverse_linear.inl:286-329
//     any_hit(ray, begin, end, max_t [, isect])  traverse_linear.inl:232-283
//     multi_hit<N>(ray, begin, end [, isect])    traverse_linear.inl:333-380 (reference headers)
//
// over a range of hip_bvh_ref (hip_index_bvh::ref(), the bvh_ref of bvh.h:344-350) or of plain
// primitives (basic_triangle<3,float> / basic_sphere<float> arrays in device memory), with the
// default intersector or a basic_intersector subclass (intersector.h:24-119).
//
// Two vocabularies:
//   * with visionaray_hip/reference.h included first, the REFERENCE'S OWN headers are device code:
//     its types, closest_hit / any_hit / multi_hit, update_if, basic_intersector, get_normal,
//     random_sampler<float>, cosine_sample_hemisphere, kernels<> ...  This header then only adds the
//     device BVH as one more BVH type of the reference's traversal (is_index_bvh<hip_bvh_ref_t<P>>
//     and its intersect<Traversal>(), below): a kernel written for cuda_sched compiles unchanged.
//   * without it, visionaray_hip/standalone.h's minimal restatement of the same names (this header
//     adds the kernel-side ones: hit records, intersect(), basic_intersector, random_sampler<float>,
//     cosine_sample_hemisphere, ...), for programs that do not have the Visionaray headers.
// Either way the BVH walk is libvrh's (visionaray_hip/detail/vrh_device.h: the 64-B pair records,
// box_pair's slab test, near child first with ties to child 1, far child pushed, leaf primitives in
// index order), with the primitive test handed to the intersector, so the default intersector gives
// the built-in kernels' bits.
//
// Device lambdas capture by value ([=]): they run on the GPU.  The traversal stack lives in LDS (at most
// VRH_USER_STACK entries per thread, VRH_USER_LDS_STACK while every BVH the program has taken a ref of
// is shallower; below); BVHs deeper than VRH_USER_STACK are rejected by checked_ref.
#pragma once

#if !defined(__HIP__)
#error "visionaray_hip/hip_kernels.h is device code: compile this translation unit with hipcc"
#endif

#include <hip/hip_runtime.h>

#if defined(VRH_REFERENCE_HEADERS)
#include "hip_backend.h"
#ifndef VRH_FUNC
#define VRH_FUNC __host__ __device__
#endif
#else
#include "standalone.h"
#endif
#include "detail/vrh_device.h"
#include "detail/vrh_libm.h"

#include <array>
#include <atomic>
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
#ifndef VRH_USER_DEFER
#define VRH_USER_DEFER 0          // deferred any_hit calls (below), opt-in
#endif
#ifndef VRH_USER_LDS_STACK
// the stack entries per thread a launch gives in LDS while every BVH the program has taken a ref of
// (hip_index_bvh::ref) is shallower than that; once one is deeper, the depth + 1 it needs (at most
// VRH_USER_STACK).  LDS bounded the waves per CU: 64 lanes x 32 entries are 8 KB per one-wave block,
// and a CU held fewer than 20; with 24 entries (6 KB) a CU holds 26 and the registers bound it (C3,
// the AO lambda: 1.698 -> 1.549 ms per frame at 6 waves / SIMD, ao/main.cpp's kernel 1.662 -> 1.490;
// profiles/r06/user_lds/).  The opt-in walks below that keep their own state in the stack columns
// always take the whole stack.
#if VRH_USER_DEFER || VRH_USER_ANYHIT_CUT || VRH_USER_ANYHIT_SHARE || VRH_USER_ANYHIT_ORDERED
#define VRH_USER_LDS_STACK VRH_USER_STACK
#else
#define VRH_USER_LDS_STACK 24
#endif
#endif
static_assert(VRH_USER_LDS_STACK >= 1 && VRH_USER_LDS_STACK <= VRH_USER_STACK, "VRH_USER_LDS_STACK: 1 .. VRH_USER_STACK");

namespace visionaray
{

namespace hip_detail
{
__device__ inline vrh::dev::ray_t dev_ray(basic_ray<float> const& r)
{
    return vrh::dev::make_ray(vrh::dev::mk3(r.ori.x, r.ori.y, r.ori.z), vrh::dev::mk3(r.dir.x, r.dir.y, r.dir.z));
}
} // hip_detail

#if !defined(VRH_REFERENCE_HEADERS)
// ================================================================================================
// standalone vocabulary (the reference headers define all of this themselves)
// ================================================================================================

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
// random_sampler<float> (random_sampler.h:24-57): std::default_random_engine -- libstdc++'s
// minstd_rand0, x <- 16807 x mod (2^31 - 1), seeded with seed mod (2^31 - 1) (1 for 0) -- under
// std::uniform_real_distribution<float>(0, 1), i.e. generate_canonical<float, 24> (random.tcc:
// one engine call; (x - 1) as float over float(2^31 - 1 + 1) = 2^31; 1.0 clamped to the float below 1)
// times (1 - 0) plus 0.  Bit-identical to the reference's CPU sampler (tests/test_gpu_ref_kernels.py).
//

template <typename T> class random_sampler;

template <>
class random_sampler<float>
{
public:
    using value_type = float;

    VRH_FUNC random_sampler() = default;
    VRH_FUNC random_sampler(unsigned seed) : x_(seed % 2147483647u == 0u ? 1u : seed % 2147483647u) {}

    VRH_FUNC float next()
    {
        x_ = uint32_t((uint64_t(x_) * 16807u) % 2147483647u);
        float r = float(x_ - 1u) / 2147483648.0f;
        if (r >= 1.0f) r = 0.99999994f;             // std::nextafter(1.0f, 0.0f)
        return r * (1.0f - 0.0f) + 0.0f;
    }

private:
    uint32_t x_ = 1u;                               // default_seed
};

// float sin / cos as the host C library computes them (detail/vrh_libm.h restates glibc's sinf / cosf,
// equal to it on every float input), so the samplers below draw the reference CPU run's directions on
// the device too; other types keep std::sin / std::cos
VRH_FUNC inline float libm_cos(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return ::vrh::libm::cosf(x);
#else
    return ::cosf(x);
#endif
}
VRH_FUNC inline float libm_sin(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return ::vrh::libm::sinf(x);
#else
    return ::sinf(x);
#endif
}
template <typename T> VRH_FUNC inline T libm_cos(T x) { return std::cos(x); }
template <typename T> VRH_FUNC inline T libm_sin(T x) { return std::sin(x); }

// sampling.h:49-71 (math/detail/math.h:241 two_pi; max(x, y) = x < y ? y : x)
template <typename T>
VRH_FUNC inline vector<3, T> uniform_sample_hemisphere(T u1, T u2)
{
    auto m = T(1.0) - u1 * u1;
    auto r = std::sqrt(T(0.0) < m ? m : T(0.0));
    auto phi = T(6.28318530717958647692528676656e+00) * u2;
    return vector<3, T>(r * libm_cos(phi), r * libm_sin(phi), u1);
}

template <typename T>
VRH_FUNC inline vector<3, T> cosine_sample_hemisphere(T u1, T u2)
{
    auto r = std::sqrt(u1);
    auto theta = T(6.28318530717958647692528676656e+00) * u2;
    auto x = r * libm_cos(theta);
    auto y = r * libm_sin(theta);
    auto m = T(1.0) - u1;
    auto z = std::sqrt(T(0.0) < m ? m : T(0.0));
    return vector<3, T>(x, y, z);
}

#endif // !VRH_REFERENCE_HEADERS

//-------------------------------------------------------------------------------------------------
// The BVH walk over libvrh's device layout (detail/bvh/intersect.inl:60-134), shared by both
// vocabularies: near child first (ties -> child 1), the far child pushed, a node pair culled against
// the running result's t (cull_t(): is_closer(box, result, max_t), update_if.h:60-88), a leaf's
// primitives handed in index order to `leaf(i)`, which tests and merges one primitive and returns
// true to end the traversal (exit_traversal<AnyHit>).
//

namespace hip_detail
{
// The BVH arrays a user kernel walks are reached through pointers it reads from device memory (the
// hip_bvh_ref range): the compiler cannot tell their address space and emits FLAT loads, which count
// against both vmcnt and lgkmcnt -- every wait for an LDS stack pop then also waits for the record
// fetches in flight, and a triangle's 48 B came out as five loads around one such wait.  They are
// global memory (vrh_scene_view, hipMalloc), so the fetches below say so: global_load_dwordx4.
#ifndef VRH_USER_GLOBAL_LOADS
#define VRH_USER_GLOBAL_LOADS 1
#endif
// (component by component: a whole-struct copy binds the global lvalue to float4's copy constructor,
// a generic reference, and the load is FLAT again)
typedef __attribute__((address_space(1))) const float4 global_float4;
typedef __attribute__((address_space(1))) const float2 global_float2;
__device__ __forceinline__ float4 gld4(const float4* p)
{
#if VRH_USER_GLOBAL_LOADS && defined(__HIP_DEVICE_COMPILE__)
    global_float4* g = (global_float4*)p;
    return make_float4(g->x, g->y, g->z, g->w);
#else
    return *p;
#endif
}
__device__ __forceinline__ float2 gld2(const float2* p)
{
#if VRH_USER_GLOBAL_LOADS && defined(__HIP_DEVICE_COMPILE__)
    global_float2* g = (global_float2*)p;
    return make_float2(g->x, g->y);
#else
    return *p;
#endif
}

// A BVH ref's view (vrh_scene_view, 72 B) is read at every closest_hit / any_hit call.  The ref lives
// in device memory the kernel never writes (a bvh_ref array, ao/main.cpp:171-178), at an address
// every lane of the wave shares: read it then through the scalar cache (s_load) instead of one
// vector load per field and call.  A ref in private or LDS memory (a local copy) is read as usual.
__device__ inline vrh_scene_view uniform_view(vrh_scene_view const& v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const uint64_t a = reinterpret_cast<uint64_t>(&v);
    const uint64_t af = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(a)))))
                      | (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(a >> 32))))) << 32);
    const void* pf = reinterpret_cast<const void*>(af);
    if (__ballot(a != af) == 0ull && (af & 3u) == 0u && !__builtin_amdgcn_is_private(pf) && !__builtin_amdgcn_is_shared(pf))
    {
        typedef const __attribute__((address_space(4))) uint32_t cword;
        cword* cw = (cword*)(pf);
        vrh_scene_view r;
        uint32_t* w = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
        for (uint32_t k = 0; k < uint32_t(sizeof(vrh_scene_view) / 4u); ++k) w[k] = cw[k];
        return r;
    }
#endif
    return v;
}

// p as held by the wave's first active lane, and whether every active lane holds the same p: the
// opt-in walks that keep one BVH's state for the whole wave (the shared any_hit walk, whose lanes take
// over each other's subtrees; the entry cut's skeleton) need every lane on the same BVH.  (The scalar
// fetches of wave-uniform records need no such check: a load through a divergent pointer is compiled
// as a vector load -- tests/cpp/user_kernels.hip divbvh)
template <typename T>
__device__ __forceinline__ const T* first_lane_ptr(const T* p, bool& uniform)
{
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint64_t af = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(a)))))
                      | (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(a >> 32))))) << 32);
    uniform = __ballot(a != af) == 0ull;
    return reinterpret_cast<const T*>(af);
}

// the leaf primitive i of the device layout, rebuilt as a primitive object of type P (the
// reference's basic_triangle<3,float> / basic_sphere<float>, or standalone.h's of the same layout)
template <typename P>
__host__ __device__ inline P leaf_primitive(const float4* prims, uint32_t i, uint32_t& flags)
{
    P p;
#if defined(__HIP_DEVICE_COMPILE__)
    auto ld = [](const float4* q) { return gld4(q); };
#else
    auto ld = [](const float4* q) { return *q; };
#endif
    if constexpr (is_sphere<P>::value)
    {
        const float4 a = ld(prims + 2u * i), b = ld(prims + 2u * i + 1u);
        p.center = decltype(p.center)(a.x, a.y, a.z);
        p.radius = a.w;
        p.prim_id = __float_as_uint(b.x);
        p.geom_id = __float_as_uint(b.y);
        flags = __float_as_uint(b.z);
    }
    else
    {
        const float4 a = ld(prims + 3u * i), b = ld(prims + 3u * i + 1u), c = ld(prims + 3u * i + 2u);
#if defined(__HIP_DEVICE_COMPILE__)
        // the third 16 B as ONE load: its fields are read at different places (e2.z and the flags by the
        // test, prim / geom ids only for a hit), and the compiler would otherwise split it into a dword
        // load now and another after the test -- a per-lane gather costs the TD about the same for 4 B
        // as for 16 B (profiles/l1_roof.json)
        asm volatile("" :: "v"(c.x), "v"(c.y), "v"(c.z), "v"(c.w));
#endif
        p.v1 = decltype(p.v1)(a.x, a.y, a.z);
        p.e1 = decltype(p.e1)(a.w, b.x, b.y);
        p.e2 = decltype(p.e2)(b.z, b.w, c.x);
        p.prim_id = __float_as_uint(c.y);
        p.geom_id = __float_as_uint(c.z);
        flags = __float_as_uint(c.w);
    }
    return p;
}

// the per-thread traversal stack: a column of the block's dynamic LDS.  With VRH_USER_LDS_STACK <
// VRH_USER_STACK the launch gives either many entries per thread (USER_STACK_SIZED); the first LDS
// word then holds that count (user_render writes it) and the columns start after it
constexpr bool USER_STACK_SIZED = VRH_USER_LDS_STACK < VRH_USER_STACK;
constexpr uint32_t USER_LDS_HEADER = USER_STACK_SIZED ? 1u : 0u;
__device__ inline uint32_t user_stack_entries()
{
    extern __shared__ uint32_t vrh_user_smem[];
    if constexpr (USER_STACK_SIZED) return (uint32_t)__builtin_amdgcn_readfirstlane((int)vrh_user_smem[0]);
    return VRH_USER_STACK;
}
__device__ inline vrh::dev::lds_stack user_stack()
{
    extern __shared__ uint32_t vrh_user_smem[];
    const uint32_t nthreads = blockDim.x * blockDim.y * blockDim.z;
    const uint32_t tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
    vrh::dev::lds_stack st;
    const uint32_t n = user_stack_entries();
    st.init(vrh_user_smem + USER_LDS_HEADER, tid, nthreads, n, n, nullptr);   // walk(): the BVH fits
    return st;
}

// A record every active lane of the wave wants (the upper tree levels, for the rays of one 8 x 8
// tile) is fetched once through the scalar cache, as the built-in kernels fetch wave-uniform pairs
// (vrh_device.h ray_step); otherwise per lane.  Same bytes either way.
#ifndef VRH_USER_SCALAR_FETCH
#define VRH_USER_SCALAR_FETCH 1
#endif
typedef const __attribute__((address_space(4))) float user_cfloat;
__device__ inline void fetch_pair(const float4* pairs, uint32_t link, float4& q0, float4& q1, float4& q2, float2& q3)
{
    const uint32_t lf = (uint32_t)__builtin_amdgcn_readfirstlane((int)link);
    if (VRH_USER_SCALAR_FETCH && __ballot(link != lf) == 0ull)
    {
        user_cfloat* cp = (user_cfloat*)(const float*)(pairs) + 16u * lf;
        q0 = make_float4(cp[0], cp[1], cp[2], cp[3]);
        q1 = make_float4(cp[4], cp[5], cp[6], cp[7]);
        q2 = make_float4(cp[8], cp[9], cp[10], cp[11]);
        q3 = make_float2(cp[12], cp[13]);
    }
    else
    {
        const float4* p = pairs + 4u * link;
        q0 = gld4(p); q1 = gld4(p + 1); q2 = gld4(p + 2);
        q3 = gld2(reinterpret_cast<const float2*>(p + 3));
    }
}

__device__ inline void fetch_quad(const float4* quads, uint32_t link, float4 (&q)[7])
{
    const uint32_t lf = (uint32_t)__builtin_amdgcn_readfirstlane((int)link);
    if (VRH_USER_SCALAR_FETCH && __ballot(link != lf) == 0ull)
    {
        user_cfloat* cp = (user_cfloat*)(const float*)(quads) + 32u * lf;
#pragma unroll
        for (int k = 0; k < 7; ++k) q[k] = make_float4(cp[4 * k], cp[4 * k + 1], cp[4 * k + 2], cp[4 * k + 3]);
    }
    else
    {
        const float4* p = quads + 8u * link;
#pragma unroll
        for (int k = 0; k < 7; ++k) q[k] = gld4(p + k);
    }
}

// ---- entry cut of any_hit calls (exact, in the reference's visiting order) ---------------------
// An any-hit ray of a short segment (AO: max_t = the radius) only reaches leaves whose boxes come
// within float error of its segment: its box test passes only where the box meets the segment.  So
// for the segments of a wave, all inside a region R, every subtree whose box does not meet R is a box
// test every one of those rays fails.  The wave keeps, in LDS, a skeleton of the BVH's top for R:
// copies of the pair records (both child boxes, the same bits) from the root down to at most
// UCUT_ENTRIES subtrees that meet R, where
//   * a child whose box does not meet R becomes SKEL_NONE -- the test every contained ray fails;
//   * a record with exactly one child meeting R is skipped into that child's record when the child's
//     box contains both grandchildren's boxes (checked per step): a ray that fails the child's box
//     fails both grandchildren's (the slab test is monotone in the box bounds under round-to-nearest,
//     DESIGN.md section 4), and a ray that passes it visits them next -- with one candidate there is
//     no near / far order to keep.
// A contained ray then walks the skeleton from LDS exactly as it would walk those records from HBM:
// the same box tests on the same bits, near child first, ties to child 1, far child pushed.  It
// visits the same leaves in the same order as the walk from the root, so the hit record an any_hit
// returns is the reference's first-found one (not only its hit / miss).  The skeleton is rebuilt
// (wave-uniform, records through the scalar cache) when more than a quarter of the wave's segments
// leave R; R covers every direction from the segments' origins (o +- max_t |d|) plus 5 % of max_t,
// so the next calls of an AO loop from the same hit points reuse it.  Lanes outside R, and non-finite
// rays, start at the root.
// Opt-in (VRH_USER_ANYHIT_CUT=1): exact, but measured SLOWER on the AO lambda (C3, round 4,
// profiles/r04/user/): 2.06 vs 1.93 ms per frame at 32 frames per launch, 2.33 vs 2.22 one frame per
// launch; ao/main.cpp's own kernel 2.11 vs 1.86 / 2.43 vs 2.19.  In a user kernel the levels above the
// cut are walked by the whole wave together (every lane at the same record: the scalar-cache fetch),
// so the LDS skeleton saves little, while the per-call containment test and the skeleton's LDS reads
// cost on every call.  The built-in AO kernel gains from its cut (+9 %) because its rays start AT the
// cut entries, which an any_hit that must return the reference's first-found record cannot do.
#ifndef VRH_USER_ANYHIT_CUT
#define VRH_USER_ANYHIT_CUT 0
#endif
constexpr uint32_t UCUT_NODES = 8;               // skeleton records
constexpr uint32_t UCUT_ENTRIES = 8;             // subtrees below the skeleton that meet R
constexpr uint32_t SKEL_BIT = 0x40000000u;       // link to skeleton record (link & 0xFF)
constexpr uint32_t SKEL_NONE = 0x7FFFFFFFu;      // a child every contained ray misses
// LDS words after the block's stacks: [0, 1] BVH key, [2] records (0: none), [4..6] R lo, [7..9] R hi,
// [10..15] reduction scratch, [16 + 16 k, 32 + 16 k) record k (the pair layout: q0 q1 q2 links)
constexpr uint32_t UCUT_WORDS = 16u + 16u * UCUT_NODES;

__device__ inline uint32_t* user_cut_area()
{
    extern __shared__ uint32_t vrh_user_smem[];
    return vrh_user_smem + VRH_USER_STACK * 64u;
}

// child c of a pair record (14 words: q0 q1 q2, link0, link1): lo = w[c], w[2 + c], w[4 + c],
// hi = w[6 + c], w[8 + c], w[10 + c]
__device__ inline bool ucut_meets(const float (&w)[14], uint32_t c, const float* lo, const float* hi)
{
    return (w[c] <= hi[0]) & (w[6 + c] >= lo[0]) & (w[2 + c] <= hi[1]) & (w[8 + c] >= lo[1])
         & (w[4 + c] <= hi[2]) & (w[10 + c] >= lo[2]);
}
// both child boxes of record v inside child c's box of record w
__device__ inline bool ucut_contains(const float (&w)[14], uint32_t c, const float (&v)[14])
{
    bool ok = true;
#pragma unroll
    for (uint32_t a = 0; a < 3; ++a)
        ok = ok & (v[2 * a] >= w[2 * a + c]) & (v[2 * a + 1] >= w[2 * a + c])
                & (v[6 + 2 * a] <= w[6 + 2 * a + c]) & (v[6 + 2 * a + 1] <= w[6 + 2 * a + c]);
    return ok;
}
__device__ inline void ucut_load(const float4* pairs, uint32_t p, float (&w)[14])
{
    user_cfloat* cp = (user_cfloat*)(const float*)(pairs) + 16u * (uint32_t)__builtin_amdgcn_readfirstlane((int)p);
#pragma unroll
    for (int k = 0; k < 14; ++k) w[k] = cp[k];
}
// the record to keep for the subtree under pair link p: p, or the record a chain of single-child
// steps leads to (containment checked at every step)
__device__ inline void ucut_compress(const float4* pairs, uint32_t p, const float* lo, const float* hi, float (&w)[14])
{
    ucut_load(pairs, p, w);
#pragma unroll 1
    for (int guard = 0; guard < 64; ++guard)
    {
        const bool m0 = ucut_meets(w, 0, lo, hi), m1 = ucut_meets(w, 1, lo, hi);
        if (m0 == m1) return;
        const uint32_t c = m0 ? 0u : 1u;
        const uint32_t l = __float_as_uint(w[12 + c]);
        if (l & vrh::dev::LEAF_BIT) return;
        float v[14];
        ucut_load(pairs, l, v);
        if (!ucut_contains(w, c, v)) return;
#pragma unroll
        for (int k = 0; k < 14; ++k) w[k] = v[k];
    }
}
// write record w as skeleton record k (by the first active lane); returns its inner children that
// meet R (new entries), links rewritten: outside R -> SKEL_NONE
__device__ inline uint32_t ucut_put(uint32_t* cw, uint32_t k, const float (&w)[14], const float* lo, const float* hi, bool writer)
{
    uint32_t l[2], entries = 0;
#pragma unroll
    for (uint32_t c = 0; c < 2; ++c)
    {
        l[c] = __float_as_uint(w[12 + c]);
        if (!ucut_meets(w, c, lo, hi)) l[c] = SKEL_NONE;
        else if (!(l[c] & vrh::dev::LEAF_BIT)) entries += 1u;
    }
    if (writer)
    {
        float4* r = reinterpret_cast<float4*>(cw + 16u + 16u * k);
        r[0] = make_float4(w[0], w[1], w[2], w[3]);
        r[1] = make_float4(w[4], w[5], w[6], w[7]);
        r[2] = make_float4(w[8], w[9], w[10], w[11]);
        r[3] = make_float4(__uint_as_float(l[0]), __uint_as_float(l[1]), 0.0f, 0.0f);
    }
    return entries;
}
__device__ inline void ucut_sync()
{
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// The link this lane's any-hit walk starts at: skeleton record 0 if its segment lies in the wave's
// R (rebuilt here when needed), else the root.  Called by every lane that calls any_hit.
__device__ inline uint32_t user_cut_entry(vrh_scene_view const& b, vrh::dev::ray_t const& r, float max_t, bool fast)
{
    using namespace vrh::dev;
    uint32_t* cw = user_cut_area();
    float* cf = reinterpret_cast<float*>(cw);
    const uint32_t lane = __lane_id();
    const uint64_t act = __ballot(true);
    const uint32_t first = (uint32_t)__builtin_ctzll(act);
    // the segment {o + t d : 0 <= t <= max_t}, per axis
    const float o[3] = { r.ori.x, r.ori.y, r.ori.z }, d[3] = { r.dir.x, r.dir.y, r.dir.z };
    float slo[3], shi[3];
    bool seg_ok = fast;
#pragma unroll
    for (int a = 0; a < 3; ++a)
    {
        const float t = max_t * d[a];
        slo[a] = o[a] + (t < 0.0f ? t : 0.0f);
        shi[a] = o[a] + (t > 0.0f ? t : 0.0f);
        seg_ok = seg_ok & __builtin_isfinite(slo[a]) & __builtin_isfinite(shi[a]);
    }
    bool same_bvh = false;
    (void)first_lane_ptr(b.pairs, same_bvh);
    if (!same_bvh) return b.root;                    // the skeleton is one BVH's: lanes on others start at the root
    const uint64_t key = (uint64_t)(uintptr_t)b.pairs;
    auto inside = [&]() {
        const bool have = cw[2] != 0u && cw[0] == (uint32_t)key && cw[1] == (uint32_t)(key >> 32);
        return have & seg_ok & (slo[0] >= cf[4]) & (slo[1] >= cf[5]) & (slo[2] >= cf[6])
                    & (shi[0] <= cf[7]) & (shi[1] <= cf[8]) & (shi[2] <= cf[9]);
    };
    bool in = inside();
    const uint64_t out = __ballot(seg_ok & !in);
    const uint32_t nout = (uint32_t)__popcll(out);
    if (nout == 0u || 4u * nout <= (uint32_t)__popcll(act)) return in ? SKEL_BIT : b.root;

    // rebuild: R = every direction from the origins of this call's finite segments, plus slack
    if (lane == first)
    {
        cw[2] = 0u;
        cf[10] = cf[11] = cf[12] = INFINITY;
        cf[13] = cf[14] = cf[15] = -INFINITY;
    }
    ucut_sync();
    if (seg_ok)
    {
        const float reach = max_t * __builtin_sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) * 1.0001f + 0.05f * max_t;
#pragma unroll
        for (int a = 0; a < 3; ++a)
        {
            atomicMin(&cf[10 + a], o[a] - reach);
            atomicMax(&cf[13 + a], o[a] + reach);
        }
    }
    ucut_sync();
    float rlo[3], rhi[3], lo[3], hi[3], mag = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a)
    {
        rlo[a] = cf[10 + a];
        rhi[a] = cf[13 + a];
        mag = fmaxf(mag, fmaxf(fabsf(rlo[a]), fabsf(rhi[a])));
    }
    // R grown by a margin far above a slab test's float error: every box a contained ray passes meets it
    const float m = 1e-4f * (1.0f + mag);
    bool finite = true;
#pragma unroll
    for (int a = 0; a < 3; ++a)
    {
        lo[a] = rlo[a] - m;
        hi[a] = rhi[a] + m;
        finite = finite & __builtin_isfinite(lo[a]) & __builtin_isfinite(hi[a]);
    }
    // (a binary tree over n leaf-ordered primitives has fewer than n pairs: pair links stay below SKEL_BIT)
    if (!finite || (b.root & LEAF_BIT) || b.num_prims >= SKEL_BIT) return b.root;
    // the skeleton, breadth first: record 0 for the root, then entries expanded in order while the
    // records and the entries below them fit
    const float4* pairs = static_cast<const float4*>(b.pairs);
    float w[14];
    ucut_compress(pairs, b.root, lo, hi, w);
    uint32_t n = 1, entries = ucut_put(cw, 0, w, lo, hi, lane == first);
    ucut_sync();
#pragma unroll 1
    for (uint32_t k = 0; k < n && n < UCUT_NODES; ++k)
    {
#pragma unroll 1
        for (uint32_t c = 0; c < 2u && n < UCUT_NODES; ++c)
        {
            const uint32_t g = (uint32_t)__builtin_amdgcn_readfirstlane((int)cw[16u + 16u * k + 12u + c]);
            if ((g & LEAF_BIT) || (g & SKEL_BIT)) continue;            // leaf, outside R, or expanded
            float v[14];
            ucut_compress(pairs, g, lo, hi, v);
            uint32_t e = 0;
            for (uint32_t cc = 0; cc < 2u; ++cc)
                e += (ucut_meets(v, cc, lo, hi) && !(__float_as_uint(v[12 + cc]) & LEAF_BIT)) ? 1u : 0u;
            if (entries - 1u + e > UCUT_ENTRIES) continue;
            ucut_put(cw, n, v, lo, hi, lane == first);
            if (lane == first) cw[16u + 16u * k + 12u + c] = SKEL_BIT | n;
            entries = entries - 1u + e;
            n += 1u;
            ucut_sync();
        }
    }
    if (lane == first)
    {
        cw[0] = (uint32_t)key;
        cw[1] = (uint32_t)(key >> 32);
        cf[4] = rlo[0]; cf[5] = rlo[1]; cf[6] = rlo[2];
        cf[7] = rhi[0]; cf[8] = rhi[1]; cf[9] = rhi[2];
        cw[2] = n;
    }
    ucut_sync();
    in = inside();
    return in ? SKEL_BIT : b.root;
}

// (the pair step as a lambda: the same walk, compiled 1.5 % faster than with the step written out in
// the loop -- C3, AO lambda 1.727 vs 1.754 ms per frame, ao/main.cpp's kernel 1.665 vs 1.690, same box.
// Measured and not kept, profiles/r06/user_walk/: popping on a miss inside the descent loop, +4 %; that
// plus descending past a first leaf while a lane of the wave has none, +15 %; one pair or primitive per
// lane and loop iteration, +13 %.  The nested loops keep a wave's lanes in step: they restart together
// after each leaf phase and share records through the scalar cache)
template <bool FAST, bool CUT = false, typename CullT, typename Leaf>
__device__ inline void walk_slab(vrh_scene_view const& b, vrh::dev::ray_t const& r, float max_t, CullT const& cull_t, Leaf&& leaf,
                                 uint32_t start = 0xFFFFFFFFu)
{
    using vrh::dev::LEAF_BIT;
    const float4* pairs = static_cast<const float4*>(b.pairs);
    auto st = user_stack();
    // the pair record `link`: which children are hit (b0, b1), and whether child 0 is the near one
    auto step = [&](uint32_t link, bool& b0, bool& b1, uint32_t& l0, uint32_t& l1, bool& go0)
    {
        float4 q0, q1, q2;
        float2 q3;
        if (CUT && (link & SKEL_BIT))
        {
            // a skeleton record (user_cut_entry): the pair record's own bits, from LDS
            const float4* nr = reinterpret_cast<const float4*>(user_cut_area() + 16u + 16u * (link & 0xFFu));
            q0 = nr[0]; q1 = nr[1]; q2 = nr[2];
            const float4 l = nr[3];
            q3 = make_float2(l.x, l.y);
        }
        else
            fetch_pair(pairs, link, q0, q1, q2, q3);
        float tn0, tn1;
        vrh::dev::box_pair<FAST>(q0, q1, q2, r, cull_t(), max_t, b0, b1, tn0, tn1);
        l0 = __float_as_uint(q3.x);
        l1 = __float_as_uint(q3.y);
        if (CUT) { b0 = b0 & (l0 != SKEL_NONE); b1 = b1 & (l1 != SKEL_NONE); }      // outside R: missed
        go0 = (b0 & b1) ? (tn0 < tn1) : b0;                                             // ties -> child 1
    };
    st.push(CUT ? start : b.root);
    while (!st.empty())
    {
        uint32_t link = st.pop();
        bool at_leaf = true;
        while (!(link & LEAF_BIT))
        {
            bool b0, b1, go0;
            uint32_t l0, l1;
            step(link, b0, b1, l0, l1, go0);
            if (!(b0 | b1)) { at_leaf = false; break; }                               // pop
            if (b0 & b1) st.push(go0 ? l1 : l0);
            link = go0 ? l0 : l1;
        }
        if (!at_leaf) continue;
        for (uint32_t i = link & ~LEAF_BIT;; ++i)
        {
            uint32_t flags = 0;
            if (leaf(i, flags)) return;
            if (flags & vrh::dev::END_BIT) break;
        }
    }
}

// An any-hit ray over the scene's 4-wide records (vrh_scene_view::quads, vrh_quad.cpp): the records
// hold the grandchildren of every binary node, so a ray reaches exactly the leaves the binary walk
// reaches -- before its first accepted hit an any-hit ray's box tests compare against constants, so
// whether it finds a hit does not depend on the order -- in half the dependent steps, nearest entry
// first (as the built-in AO / shadow rays, vrh_device.h ray_step).  Returns false when a record's hits
// would overflow the stack; the caller then walks the binary records from the root (nothing was
// accepted so far, so the result is unchanged).
template <typename Leaf>
__device__ inline bool walk_quads(vrh_scene_view const& b, vrh::dev::ray_t const& r, float max_t, Leaf&& leaf)
{
    using vrh::dev::QUAD_NONE;
    const float4* quads = static_cast<const float4*>(b.quads);
    auto st = user_stack();
    st.push(0u);
    while (!st.empty())
    {
        uint32_t link = st.pop();
        bool at_leaf = true;
        while (!(link & vrh::dev::LEAF_BIT))
        {
            float4 qr[7];
            fetch_quad(quads, link, qr);
            const float4 xl = qr[0], yl = qr[1], zl = qr[2], xh = qr[3], yh = qr[4], zh = qr[5], lk = qr[6];
            const uint32_t k0 = __float_as_uint(lk.x), k1 = __float_as_uint(lk.y);
            const uint32_t k2 = __float_as_uint(lk.z), k3 = __float_as_uint(lk.w);
            float d0, d1, d2, d3;
            const bool h0 = vrh::dev::quad_entry(xl.x, yl.x, zl.x, xh.x, yh.x, zh.x, r, max_t, d0) & (k0 != QUAD_NONE);
            const bool h1 = vrh::dev::quad_entry(xl.y, yl.y, zl.y, xh.y, yh.y, zh.y, r, max_t, d1) & (k1 != QUAD_NONE);
            const bool h2 = vrh::dev::quad_entry(xl.z, yl.z, zl.z, xh.z, yh.z, zh.z, r, max_t, d2) & (k2 != QUAD_NONE);
            const bool h3 = vrh::dev::quad_entry(xl.w, yl.w, zl.w, xh.w, yh.w, zh.w, r, max_t, d3) & (k3 != QUAD_NONE);
            if (!(h0 | h1 | h2 | h3)) { at_leaf = false; break; }
            if (!st.room(3u)) return false;
            d0 = h0 ? d0 : INFINITY; d1 = h1 ? d1 : INFINITY; d2 = h2 ? d2 : INFINITY; d3 = h3 ? d3 : INFINITY;
            const bool a01 = d1 < d0, a23 = d3 < d2;
            const float m01 = a01 ? d1 : d0, m23 = a23 ? d3 : d2;
            const uint32_t j = (m23 < m01) ? (a23 ? 3u : 2u) : (a01 ? 1u : 0u);
            if (h0 & (j != 0u)) st.push(k0);
            if (h1 & (j != 1u)) st.push(k1);
            if (h2 & (j != 2u)) st.push(k2);
            if (h3 & (j != 3u)) st.push(k3);
            link = j == 0u ? k0 : j == 1u ? k1 : j == 2u ? k2 : k3;
        }
        if (!at_leaf) continue;
        for (uint32_t i = link & ~vrh::dev::LEAF_BIT;; ++i)
        {
            uint32_t flags = 0;
            if (leaf(i, flags)) return true;
            if (flags & vrh::dev::END_BIT) break;
        }
    }
    return true;
}

// the LDS stack holds VRH_USER_STACK entries: a deeper BVH (not passed through checked_ref) is not
// traversed -- a miss, never an out-of-bounds stack write.  The hardware min/max slab test where it is
// provably identical (vrh_device.h box_pair).  ANY: an any-hit walk (the leaf ends it at the first
// accepted hit).  By default it is the binary walk in the reference's order, so the hit record an
// any_hit returns is the reference's first-found one; VRH_USER_BINARY_ANYHIT=0 takes the 4-wide
// records where the scene has them and the ray is finite (the hit / miss answer is the same, WHICH
// hit ends the ray may differ).  Measured on the AO lambda (C3, profiles/r03_ab/user/): the binary
// walk with the scalar fetch of wave-uniform pairs is 2-3 % faster than the 4-wide one.
#ifndef VRH_USER_BINARY_ANYHIT
#define VRH_USER_BINARY_ANYHIT 1
#endif
template <bool ANY = false, typename Ray, typename CullT, typename Leaf>
__device__ inline void walk(vrh_scene_view const& b, Ray const& ray, float max_t, CullT const& cull_t, Leaf&& leaf)
{
    if (b.max_depth >= user_stack_entries()) return;
    const vrh::dev::ray_t r = dev_ray(ray);
    const bool fast = b.finite_bounds && vrh::dev::finite_ray(r);
    if constexpr (ANY && !VRH_USER_BINARY_ANYHIT)
        if (fast && b.quads && walk_quads(b, r, max_t, leaf)) return;
    if constexpr (ANY && VRH_USER_ANYHIT_CUT)
    {
        // the entry cut needs the LDS area user_render provides after the stacks of its 64-thread blocks
        if (blockDim.x * blockDim.y * blockDim.z == 64u)
        {
            const uint32_t start = user_cut_entry(b, r, max_t, fast);
            if (fast) walk_slab<true, true>(b, r, max_t, cull_t, leaf, start);
            else walk_slab<false>(b, r, max_t, cull_t, leaf);
            return;
        }
    }
    if (fast) walk_slab<true>(b, r, max_t, cull_t, leaf);
    else walk_slab<false>(b, r, max_t, cull_t, leaf);
}

// Shared any-hit walk (VRH_USER_ANYHIT_SHARE=1).  A user kernel calls any_hit from one thread per
// pixel, and the wave runs each call until its slowest lane is done: on the AO lambda (C3) 55 % of
// the lane-steps of the any_hit calls are idle lanes waiting (CPU replay of sampled tiles).  Here the
// lanes that called any_hit together share the work: a lane whose ray is done (miss, or another
// lane found its hit) takes the oldest stack entry -- the largest unvisited subtree -- of a lane
// still traversing, with that lane's ray, and walks it; whoever finds a hit for a ray ends it for
// every lane working on it, and the ray's owner receives that lane's hit record.  The hit / miss
// answer is exactly the reference's: before its first accepted hit an any-hit ray's box tests
// compare against constants (best_t = max(), its max_t), so the set of leaves it can reach does not
// depend on the order in which they are visited (the argument of vrh_device.h's 4-wide records).
// WHICH hit a ray reports may differ from the reference's first one in its traversal order (the
// reference's own SIMD packets already report other first hits than its scalar path), so this is
// opt-in.  The stack is a ring of VRH_USER_STACK entries (pops at the top, steals at the bottom);
// a lane never holds more live entries than the BVH is deep (checked_ref).
#ifndef VRH_USER_ANYHIT_SHARE
#define VRH_USER_ANYHIT_SHARE 0
#endif

// position of the n-th set bit (n from 0) of m, for n < popcount(m)
__device__ __forceinline__ uint32_t nth_bit(uint64_t m, uint32_t n)
{
    uint32_t p = 0;
#pragma unroll
    for (uint32_t w = 32; w; w >>= 1)
    {
        const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
        if (n >= c) { n -= c; m >>= w; p += w; }
    }
    return p;
}

// leaf2(ray, max_t, i, flags, rec): test primitive i for `ray` into the record `rec` (update_if),
// true = rec holds the hit that ends the ray
template <bool FAST, typename RT, typename Leaf2>
__device__ inline void walk_shared(vrh_scene_view const& b, vrh::dev::ray_t const& r0, float max_t0, RT& result, Leaf2&& leaf2)
{
    using namespace vrh::dev;
    static_assert(sizeof(RT) % 4 == 0 && std::is_trivially_copyable<RT>::value, "hit record words move between lanes");
    constexpr uint32_t CAP = VRH_USER_STACK, NOTASK = 0xFFFFFFFFu;
    constexpr uint32_t RW = sizeof(RT) / 4;
    // a finished lane's LDS column carries a hit record (RW words) or a stolen entry with its ray (12)
    static_assert(RW <= CAP && CAP >= 12u, "VRH_USER_ANYHIT_SHARE: the stack column must hold a hit record and a ray");
    extern __shared__ uint32_t vrh_user_smem[];
    const float4* pairs = static_cast<const float4*>(b.pairs);
    const uint32_t nthreads = blockDim.x * blockDim.y * blockDim.z;
    const uint32_t tid = threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z);
    const uint32_t lane = __lane_id();
    auto slot = [&](uint32_t k) -> uint32_t& { return vrh_user_smem[tid + (k % CAP) * nthreads]; };
    uint32_t task = lane;                 // the lane whose ray this lane traverses (NOTASK: idle)
    ray_t tr = r0;
    float tmax = max_t0;
    uint32_t bot = 0, top = 0;            // live stack entries [bot, top) of the ring
    slot(top++) = b.root;
    uint64_t found = 0ull;                // lanes whose ray has its hit (wave-uniform)
    for (;;)
    {
        if (task != NOTASK && ((found >> task) & 1ull)) task = NOTASK;
        if (task != NOTASK && top == bot) task = NOTASK;
        const uint64_t busy = __ballot(task != NOTASK);
        if (busy == 0ull) break;
        // 1. idle lanes take the bottom entry of a lane with two or more (k-th idle <- k-th donor):
        //    the donor writes that entry and its ray into the idle lane's LDS column (an idle lane's
        //    stack is empty), which the idle lane then reads -- no cross-lane register traffic
        const uint64_t idle = __ballot(task == NOTASK);
        const uint64_t donors = __ballot(task != NOTASK && top - bot >= 2u);
        if (idle != 0ull && donors != 0ull)
        {
            const uint32_t n = min((uint32_t)__popcll(idle), (uint32_t)__popcll(donors));
            const uint32_t dr = (uint32_t)__popcll(donors & ((1ull << lane) - 1ull));
            if (((donors >> lane) & 1ull) && dr < n)
            {
                uint32_t* c = vrh_user_smem + (tid - lane + nth_bit(idle, dr));
                c[0] = __float_as_uint(tr.ori.x); c[nthreads] = __float_as_uint(tr.ori.y); c[2 * nthreads] = __float_as_uint(tr.ori.z);
                c[3 * nthreads] = __float_as_uint(tr.dir.x); c[4 * nthreads] = __float_as_uint(tr.dir.y); c[5 * nthreads] = __float_as_uint(tr.dir.z);
                c[6 * nthreads] = __float_as_uint(tr.inv.x); c[7 * nthreads] = __float_as_uint(tr.inv.y); c[8 * nthreads] = __float_as_uint(tr.inv.z);
                c[9 * nthreads] = __float_as_uint(tmax); c[10 * nthreads] = task; c[11 * nthreads] = slot(bot++);
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            const uint32_t ir = (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
            if (((idle >> lane) & 1ull) && ir < n)
            {
                const uint32_t* c = vrh_user_smem + tid;
                tr.ori = mk3(__uint_as_float(c[0]), __uint_as_float(c[nthreads]), __uint_as_float(c[2 * nthreads]));
                tr.dir = mk3(__uint_as_float(c[3 * nthreads]), __uint_as_float(c[4 * nthreads]), __uint_as_float(c[5 * nthreads]));
                tr.inv = mk3(__uint_as_float(c[6 * nthreads]), __uint_as_float(c[7 * nthreads]), __uint_as_float(c[8 * nthreads]));
                tmax = __uint_as_float(c[9 * nthreads]);
                task = c[10 * nthreads];
                bot = 11u; top = 12u;                         // the entry is ring slot 11
            }
            __builtin_amdgcn_wave_barrier();
        }
        // 2. one descent (pop, down to a leaf or a miss) and the leaf's primitives
        bool hit = false;
        RT rec;
        if (task != NOTASK)
        {
            uint32_t link = slot(--top);
            bool at_leaf = true;
            while (!(link & LEAF_BIT))
            {
                float4 q0, q1, q2;
                float2 q3;
                fetch_pair(pairs, link, q0, q1, q2, q3);
                bool b0, b1;
                float tn0, tn1;
                box_pair<FAST>(q0, q1, q2, tr, FMAX, tmax, b0, b1, tn0, tn1);
                const uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
                if (!(b0 | b1)) { at_leaf = false; break; }
                const bool go0 = (b0 & b1) ? (tn0 < tn1) : b0;                 // ties -> child 1
                if (b0 & b1) slot(top++) = go0 ? l1 : l0;
                link = go0 ? l0 : l1;
            }
            if (at_leaf)
                for (uint32_t i = link & ~LEAF_BIT;; ++i)
                {
                    uint32_t flags = 0;
                    if (leaf2(tr, tmax, i, flags, rec)) { hit = true; break; }
                    if (flags & END_BIT) break;
                }
        }
        // 3. a hit ends its ray on every lane; the ray's owner takes the record of the lowest lane
        //    that found one in this step
        uint64_t hl = __ballot(hit);
        if (hl != 0ull)
        {
            uint32_t winner = NOTASK;
            while (hl != 0ull)
            {
                const uint32_t l = (uint32_t)__builtin_ctzll(hl);
                hl &= hl - 1ull;
                const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)task, (int)l);
                if (!((found >> o) & 1ull))
                {
                    found |= 1ull << o;
                    if (lane == o) winner = l;
                }
            }
            // the winner's stack is dead (its ray ended): its record goes to the first words of its
            // own LDS column, where the owner reads it
            if (hit)
            {
                uint32_t w[RW];
                __builtin_memcpy(w, &rec, sizeof(RT));
#pragma unroll
                for (uint32_t k = 0; k < RW; ++k) vrh_user_smem[tid + k * nthreads] = w[k];
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            if (winner != NOTASK)
            {
                uint32_t got[RW];
#pragma unroll
                for (uint32_t k = 0; k < RW; ++k) got[k] = vrh_user_smem[tid - lane + winner + k * nthreads];
                __builtin_memcpy(&result, got, sizeof(RT));
            }
            __builtin_amdgcn_wave_barrier();
            if (hit) task = NOTASK;
        }
    }
}

// ---- ordered cooperative any_hit (VRH_USER_ANYHIT_ORDERED, the default) --------------------------
// A user kernel calls any_hit from one lane per pixel; each call runs until its slowest lane is done.
// Here the lanes that entered the call together share the work AND keep the reference's answer: the
// record of the FIRST accepted primitive in the ray's own depth-first order (near child first, ties to
// child 1, leaf primitives in index order; intersect.inl:66-130 with exit_traversal<AnyHit>).
//   * Every place in a ray's walk has a key: the bits of the branches taken at the pairs where both
//     children were hit (0 = the near child, 1 = the far one), MSB first, with an end marker.  Keys of
//     disjoint subtrees compare as integers in the order the walk visits them.
//   * A lane whose ray is done (or that never had one) takes the BOTTOM entry of a lane holding two or
//     more -- or one, while that lane is inside a descent -- with the donor's ray and the entry's key:
//     the bottom entry is the last work of that segment of the walk, so every segment stays a
//     contiguous stretch of the ray's order.
//   * Before an any-hit ray's first accepted primitive its box tests compare against constants (max_t),
//     so the leaves a segment reaches and the order it reaches them in do not depend on who walks it.
//   * A lane that accepts a primitive records (key, primitive) for the ray (LDS atomicMin of the key in
//     the owner's column) and ends its segment; a lane whose next work is later than the ray's best key
//     drops it.  When no lane has work left, the smallest key is the reference's first hit.
// The owner then rebuilds its record by testing that one primitive with its own ray and intersector
// (the test every lane ran is the same arithmetic).  Default intersector and update rule, one BVH of
// at most 2^25 primitives, depth <= VRH_USER_STACK - 4, one-wave blocks of user_render; otherwise the
// walk above.  Descents are cut after OCA_VISITS pair visits per step so that work can move between
// lanes.
// Opt-in (VRH_USER_ANYHIT_ORDERED=1): exact (every any_hit record of the parity suite equals the
// per-lane walk's), but SLOWER.  A schedule simulation of C3's AO calls (tools/sim/oca_sim.c, 3,200
// calls of sampled tiles, scalar fetches of wave-uniform records modelled) puts its wave-level vector
// loads at only 0.89 of the per-lane walk's with 4 visits per step (0.96 with whole descents; a
// perfectly packed wave would need 0.57): the calls' tails have little left to share.  And its lane
// state costs registers: the AO lambda needs 143 VGPRs (3 waves / SIMD) or spills 200 B at 5 waves, so
// C3 ran 2.01 ms per frame against 1.75 (profiles/r06/oca/).
#ifndef VRH_USER_ANYHIT_ORDERED
#define VRH_USER_ANYHIT_ORDERED 0
#endif
#ifndef VRH_OCA_VISITS
#define VRH_OCA_VISITS 4
#endif
constexpr uint32_t OCA_RING = VRH_USER_STACK - 2u;       // stack ring; the column's last two words: best key, prim
constexpr uint32_t OCA_LVL_SHIFT = 25u;                  // entry = link | level << 25
constexpr uint32_t OCA_LINK_MASK = vrh::dev::LEAF_BIT | ((1u << OCA_LVL_SHIFT) - 1u);
constexpr uint32_t OCA_NOKEY = 0xFFFFFFFFu, OCA_NONE = 0xFFFFFFFFu, OCA_IDLE = 0xFFFFFFFFu;
static_assert(VRH_USER_STACK >= 16u, "the ordered any_hit walk moves 14 words through a lane's stack column");

// the key of `len` path bits (len <= 30): the bits left-aligned, then a one
__device__ __forceinline__ uint32_t oca_key(uint32_t path, uint32_t len)
{
    return uint32_t((uint64_t(path) << (32u - len)) | (1ull << (31u - len)));
}

// every active lane calls with the same BVH, which the walk can take (wave-uniform answer)
__device__ __forceinline__ bool oca_wave_usable(vrh_scene_view const& b)
{
    const uint64_t pa = reinterpret_cast<uint64_t>(b.pairs);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane(int(uint32_t(pa)));
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane(int(uint32_t(pa >> 32)));
    const bool ok = VRH_USER_ANYHIT_ORDERED && b.max_depth + 4u <= VRH_USER_STACK && b.num_prims < (1u << OCA_LVL_SHIFT)
                  && blockDim.x * blockDim.y * blockDim.z == 64u && pa == ((uint64_t(hi) << 32) | lo);
    return __ballot(!ok) == 0ull;
}

// test(ray, max_t, i, flags) -> bool: primitive i accepted for that ray (the walk's own leaf test);
// returns the leaf index of this lane's ray's first hit in the reference order, or OCA_NONE
template <bool FAST, typename Test>
__device__ inline uint32_t walk_ordered(vrh_scene_view const& b, vrh::dev::ray_t const& r0, float max_t0, Test&& test)
{
    using namespace vrh::dev;
    extern __shared__ uint32_t vrh_user_smem[];
    constexpr uint32_t N = 64u;                            // one-wave blocks (oca_usable)
    const float4* pairs = static_cast<const float4*>(b.pairs);
    const uint32_t lane = __lane_id();
    uint32_t* col = vrh_user_smem + lane;                  // this lane's column: word k at col[k * N]
    auto slot = [&](uint32_t k) -> uint32_t& { return col[(k % OCA_RING) * N]; };
    col[OCA_RING * N] = OCA_NOKEY;                          // this lane's ray: best key, its primitive
    col[(OCA_RING + 1u) * N] = OCA_NONE;
    uint32_t task = lane;                                   // whose ray this lane walks (OCA_IDLE: none)
    ray_t tr = r0;
    float tmax = max_t0;
    uint32_t path = 0u, plen = 0u;                          // key of the current place
    uint32_t cur = b.root;                                  // node to continue from (OCA_NONE: pop)
    uint32_t bot = 0u, top = 0u;                            // live ring entries [bot, top)
    __builtin_amdgcn_wave_barrier();
    for (;;)
    {
        // 1. work later in its ray's order than the ray's best hit is dropped; no work left: idle
        if (task != OCA_IDLE)
        {
            uint32_t pos = OCA_NOKEY;
            if (cur != OCA_NONE) pos = oca_key(path, plen);
            else if (top != bot)
            {
                const uint32_t lv = (slot(top - 1u) >> OCA_LVL_SHIFT) & 31u;
                pos = oca_key(((path >> (plen - lv)) << 1) | 1u, lv + 1u);
            }
            else task = OCA_IDLE;
            if (task != OCA_IDLE && vrh_user_smem[task + OCA_RING * N] < pos) task = OCA_IDLE;
        }
        const uint64_t busy = __ballot(task != OCA_IDLE);
        if (busy == 0ull) break;
        // 2. idle lanes take bottom entries (k-th idle <- k-th donor), through the idle lane's column
        const uint64_t idle = __ballot(task == OCA_IDLE);
        const uint64_t donors = __ballot(task != OCA_IDLE && (top - bot >= 2u || (cur != OCA_NONE && top != bot)));
        if (idle != 0ull && donors != 0ull)
        {
            const uint32_t n = min((uint32_t)__popcll(idle), (uint32_t)__popcll(donors));
            const uint32_t dr = (uint32_t)__popcll(donors & ((1ull << lane) - 1ull));
            if (((donors >> lane) & 1ull) && dr < n)
            {
                const uint32_t e = slot(bot++);
                const uint32_t lv = (e >> OCA_LVL_SHIFT) & 31u;
                uint32_t* c = vrh_user_smem + nth_bit(idle, dr);
                c[0] = __float_as_uint(tr.ori.x); c[N] = __float_as_uint(tr.ori.y); c[2 * N] = __float_as_uint(tr.ori.z);
                c[3 * N] = __float_as_uint(tr.dir.x); c[4 * N] = __float_as_uint(tr.dir.y); c[5 * N] = __float_as_uint(tr.dir.z);
                c[6 * N] = __float_as_uint(tr.inv.x); c[7 * N] = __float_as_uint(tr.inv.y); c[8 * N] = __float_as_uint(tr.inv.z);
                c[9 * N] = __float_as_uint(tmax); c[10 * N] = task; c[11 * N] = e & OCA_LINK_MASK;
                c[12 * N] = ((path >> (plen - lv)) << 1) | 1u; c[13 * N] = lv + 1u;
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            const uint32_t ir = (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
            if (((idle >> lane) & 1ull) && ir < n)
            {
                tr.ori = mk3(__uint_as_float(col[0]), __uint_as_float(col[N]), __uint_as_float(col[2 * N]));
                tr.dir = mk3(__uint_as_float(col[3 * N]), __uint_as_float(col[4 * N]), __uint_as_float(col[5 * N]));
                tr.inv = mk3(__uint_as_float(col[6 * N]), __uint_as_float(col[7 * N]), __uint_as_float(col[8 * N]));
                tmax = __uint_as_float(col[9 * N]);
                task = col[10 * N];
                cur = col[11 * N];
                path = col[12 * N];
                plen = col[13 * N];
                bot = top = 0u;
            }
            __builtin_amdgcn_wave_barrier();
        }
        // 3. at most VRH_OCA_VISITS pair visits, or the leaf reached
        bool hit = false;
        uint32_t key = 0u, won = OCA_NONE;
        if (task != OCA_IDLE)
        {
            uint32_t link = cur;
            cur = OCA_NONE;
            if (link == OCA_NONE)
            {
                const uint32_t e = slot(--top);
                const uint32_t lv = (e >> OCA_LVL_SHIFT) & 31u;
                link = e & OCA_LINK_MASK;
                path = ((path >> (plen - lv)) << 1) | 1u;
                plen = lv + 1u;
            }
            bool at_leaf = true;
            for (uint32_t k = 0;; ++k)
            {
                if (link & LEAF_BIT) break;
                if (k == VRH_OCA_VISITS) { cur = link; at_leaf = false; break; }
                float4 q0, q1, q2;
                float2 q3;
                fetch_pair(pairs, link, q0, q1, q2, q3);
                bool b0, b1;
                float tn0, tn1;
                box_pair<FAST>(q0, q1, q2, tr, FMAX, tmax, b0, b1, tn0, tn1);
                const uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
                if (!(b0 | b1)) { at_leaf = false; break; }
                const bool go0 = (b0 & b1) ? (tn0 < tn1) : b0;                 // ties -> child 1
                if (b0 & b1)
                {
                    slot(top++) = (go0 ? l1 : l0) | (plen << OCA_LVL_SHIFT);
                    path <<= 1;                                                  // the near side: 0
                    plen += 1u;
                }
                link = go0 ? l0 : l1;
            }
            if (at_leaf)
                for (uint32_t i = link & ~LEAF_BIT;; ++i)
                {
                    uint32_t flags = 0;
                    if (test(tr, tmax, i, flags)) { hit = true; won = i; key = oca_key(path, plen); break; }
                    if (flags & END_BIT) break;
                }
            if (hit)
            {
                atomicMin(&vrh_user_smem[task + OCA_RING * N], key);
                cur = OCA_NONE; bot = top = 0u;
            }
        }
        // 4. the ray's primitive: written by the lane whose key won (keys of distinct leaves differ)
        if (__ballot(hit) != 0ull)
        {
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            if (hit && vrh_user_smem[task + OCA_RING * N] == key) vrh_user_smem[task + (OCA_RING + 1u) * N] = won;
            __builtin_amdgcn_wave_barrier();
            if (hit) task = OCA_IDLE;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    return col[OCA_RING * N] == OCA_NOKEY ? OCA_NONE : col[(OCA_RING + 1u) * N];
}

// ---- deferred any_hit calls (VRH_USER_DEFER=1) --------------------------------------------------
// A user kernel runs one pixel per lane and its any_hit calls one after another, so the wave waits
// for its slowest lane once per call (the AO lambda: eight times per tile, VALU lane utilisation 0.37
// against the built-in kernel's 0.51).  With the option, user_render runs every tile in
// three phases:
//   record  the kernel runs for the tile's pixels; each any_hit call with the default intersector on
//           a single BVH is logged (ray, max_t) into the wave's log and answered "no hit" for now;
//           closest_hit calls run as usual and are logged with the leaf index of their result; nothing
//           is stored into the render target;
//   trace   the wave traces the tile's logged any_hit rays as one pool: a lane whose ray is done takes
//           the next ray of the pool (vrh_device.h ray_step, the binary records in the reference's
//           order -- near child first, ties to child 1, far child pushed, leaf primitives in index
//           order -- so every ray ends on the reference's first-found hit);
//   replay  the kernel runs again from the start with the same sampler seeds; a call that is the
//           logged one bit for bit (the same kind, BVH, origin, direction and max_t) gets the logged
//           answer -- its hit record rebuilt by testing the one recorded leaf primitive with the
//           call's own intersector and update rule -- and any other call runs directly.  The colours
//           are stored.
// The kernel's results are those of running it once: a replayed call returns what the direct call
// would return (the same ray, the same leaf, the same test), and a kernel whose later calls depend on
// earlier answers simply finds them unlogged and runs them directly.  The kernel must be a pure
// function of its ray, sampler and position -- it runs twice per pixel -- which every reference
// kernel is; hence opt-in.  Calls with a custom intersector or update rule, multi_hit, other BVHs
// than the tile's first and calls past VRH_USER_DEFER_SLOTS per pixel run directly.
#ifndef VRH_USER_DEFER
#define VRH_USER_DEFER 0
#endif
#ifndef VRH_USER_DEFER_SLOTS
#define VRH_USER_DEFER_SLOTS 12     // logged calls per pixel (AO: 1 closest + 8 any); more run directly
#endif
// the trace phase's tuning (AO lambda, C3, 32 frames per launch, rates, profiles/r05/defer/): a lane takes
// a new ray once 32 lanes are idle (1: -0.5 %, 48: -2 %, 64: -22 %); pairs wave-uniform over the active
// lanes through the scalar cache, no pop on miss (ray_step flags 2; 3: -4 %, 1: -7 %, 0: -2 %); no descent
// cap (4 / 8 visits: -21 % / -14 %); the pool in call order (pixel order: -16 %); binary records only
// (hit / miss over the 4-wide records first, then a binary re-walk of the hits: -41 %)
constexpr uint32_t DEFER_REFILL = 32u;
constexpr uint32_t DEFER_STEP_FLAGS = 2u;
static_assert(!(VRH_USER_DEFER && VRH_USER_ANYHIT_SHARE), "VRH_USER_DEFER and VRH_USER_ANYHIT_SHARE are alternatives");
constexpr uint32_t DEFER_OFF = 0u, DEFER_RECORD = 1u, DEFER_REPLAY = 2u;
// the last word of a log entry: DTAG_ANY for an any_hit call, DTAG_PENDING until the trace phase has
// answered it, the low bits the leaf index of the hit primitive or DTAG_NONE
constexpr uint32_t DTAG_ANY = 0x80000000u, DTAG_PENDING = 0x40000000u, DTAG_NONE = 0x3FFFFFFFu;
// a wave's log: VRH_USER_DEFER_SLOTS x 64 entries of 32 B ([slot][lane]: ori, dir, max_t, tag); the
// pool (entry indices of the pending any_hit calls, in call order) is in LDS
constexpr uint32_t DEFER_ENTRIES = VRH_USER_DEFER_SLOTS * 64u;
constexpr size_t DEFER_WAVE_BYTES = size_t(DEFER_ENTRIES) * 32u;
// LDS words after the stacks (and the entry-cut area): [0] phase, [1] pool size, [2] BVH set,
// [4, 6) log base, [6, 24) the tile's BVH (vrh_scene_view), [24, 88) calls per lane so far, [88, ...) the pool
// then the pool: 16-bit entry indices, DEFER_ENTRIES / 2 words (10,080 B of LDS per wave with the
// stacks: 16 waves / CU; the pool in the global log instead: -2 %, profiles/r05/defer/)
// then one bit per entry: the trace phase found no hit (a miss leaves the entry's tag pending; only a
// hit writes its leaf index to the log)
// The per-lane call word [24 + lane] counts the calls so far in its low 16 bits; in the replay its high
// 16 bits hold the number of calls the record phase logged.  The replay trusts a log entry only below
// that count: a kernel whose answers change its path can make more calls in the replay than it logged,
// and the slots past the count hold entries of an earlier tile
constexpr uint32_t DEFER_MISS_WORDS = DEFER_ENTRIES / 32u;
constexpr uint32_t DEFER_WORDS = 88u + DEFER_ENTRIES / 2u + DEFER_MISS_WORDS;
__device__ inline uint32_t* defer_miss_bits(uint32_t* a) { return a + 88u + DEFER_ENTRIES / 2u; }
static_assert(DEFER_ENTRIES <= 65536u, "16-bit pool entries");
static_assert(sizeof(vrh_scene_view) <= 18u * 4u, "the LDS copy of the tile's BVH holds 18 words");
enum defer_state : uint32_t { DEFER_RUN = 0u, DEFER_RUN_LOG = 1u, DEFER_PENDING = 2u, DEFER_LOGGED = 3u };
#ifndef VRH_DEFER_PROF
#define VRH_DEFER_PROF 0
#endif
// VRH_DEFER_PROF (diagnostic build): per block, lane 0 sums [0] record [1] trace [2] replay clock
// cycles, [3] tiles, [4] pooled rays, [5] trace-loop iterations, [6] busy lanes summed over those
// iterations, and writes them with DEFER_PROF_MAGIC in [7] to the first 64 B of its log at the end
constexpr unsigned long long DEFER_PROF_MAGIC = 0x5652484445464552ull;

__device__ inline uint32_t* defer_area()
{
    extern __shared__ uint32_t vrh_user_smem[];
    return vrh_user_smem + VRH_USER_STACK * 64u + (VRH_USER_ANYHIT_CUT ? UCUT_WORDS : 0u);
}

__device__ inline float4* defer_log(const uint32_t* a)
{
    return reinterpret_cast<float4*>(uintptr_t(a[4]) | (uintptr_t(a[5]) << 32));
}

struct defer_call
{
    uint32_t state;     // defer_state
    uint32_t entry;     // the call's log entry (slot * 64 + lane)
    uint32_t li;        // DEFER_LOGGED: leaf index of the answer's primitive, or DTAG_NONE
};

__device__ inline bool same_bits(float a, float b) { return __float_as_uint(a) == __float_as_uint(b); }

// what to do with a call of the current phase (any: any_hit, else closest_hit) on BVH v
__device__ inline defer_call defer_begin(vrh_scene_view const& v, basic_ray<float> const& ray, float max_t, bool any)
{
    defer_call d{ DEFER_RUN, 0u, DTAG_NONE };
    uint32_t* a = defer_area();
    const uint32_t phase = a[0];
    if (phase == DEFER_OFF || v.max_depth >= VRH_USER_STACK || v.num_prims >= DTAG_NONE) return d;
    const uint32_t lane = __lane_id();
    if (phase == DEFER_RECORD && a[2] == 0u)
    {
        // the tile's BVH: the first one a call names (the lowest calling lane's)
        if (lane == (uint32_t)__builtin_ctzll(__ballot(true)))
        {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
            for (uint32_t k = 0; k < uint32_t(sizeof(vrh_scene_view) / 4u); ++k) a[6u + k] = w[k];
            a[2] = 1u;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (a[2] == 0u || reinterpret_cast<const vrh_scene_view*>(a + 6)->pairs != v.pairs) return d;
    const uint32_t cw = a[24u + lane];
    const uint32_t c = cw & 0xFFFFu;
    if (c >= VRH_USER_DEFER_SLOTS) return d;
    if (phase == DEFER_REPLAY && c >= (cw >> 16)) return d;      // not logged in this tile's record phase: run it
    a[24u + lane] = cw + 1u;
    d.entry = c * 64u + lane;
    float4* ent = defer_log(a) + 2u * d.entry;
    if (phase == DEFER_RECORD)
    {
        if (!any) { d.state = DEFER_RUN_LOG; return d; }
        ent[0] = make_float4(ray.ori.x, ray.ori.y, ray.ori.z, ray.dir.x);
        ent[1] = make_float4(ray.dir.y, ray.dir.z, max_t, __uint_as_float(DTAG_ANY | DTAG_PENDING));
        // the pool, in call order: the lanes deferring here take consecutive places
        const uint64_t m = __ballot(true);
        const uint32_t n = a[1];
        const uint32_t pos = n + __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        reinterpret_cast<uint16_t*>(a + 88)[pos] = uint16_t(d.entry);
        __builtin_amdgcn_wave_barrier();
        if (lane == (uint32_t)__builtin_ctzll(m)) a[1] = n + uint32_t(__popcll(m));
        __builtin_amdgcn_wave_barrier();
        d.state = DEFER_PENDING;
        return d;
    }
    // replay: the logged call must be this one, bit for bit (reading only the tag while every answer so
    // far equals the record phase's -- the kernel then makes the same calls -- measured 0.8-1.3 % slower)
    const float4 e0 = ent[0], e1 = ent[1];
    uint32_t tag = __float_as_uint(e1.w);
    if (any && (tag & DTAG_PENDING) && (defer_miss_bits(a)[d.entry >> 5] >> (d.entry & 31u) & 1u)) tag = DTAG_ANY | DTAG_NONE;
    if (same_bits(e0.x, ray.ori.x) && same_bits(e0.y, ray.ori.y) && same_bits(e0.z, ray.ori.z) && same_bits(e0.w, ray.dir.x)
        && same_bits(e1.x, ray.dir.y) && same_bits(e1.y, ray.dir.z) && same_bits(e1.z, max_t)
        && (tag & (DTAG_ANY | DTAG_PENDING)) == (any ? DTAG_ANY : 0u))
    {
        d.state = DEFER_LOGGED;
        d.li = tag & DTAG_NONE;
    }
    return d;
}

// record phase: a closest_hit call ran directly and ended on leaf primitive li (DTAG_NONE: no hit)
__device__ inline void defer_log_closest(defer_call const& d, basic_ray<float> const& ray, float max_t, uint32_t li)
{
    float4* ent = defer_log(defer_area()) + 2u * d.entry;
    ent[0] = make_float4(ray.ori.x, ray.ori.y, ray.ori.z, ray.dir.x);
    ent[1] = make_float4(ray.dir.y, ray.dir.z, max_t, __uint_as_float(li));
}

// trace phase: the pool's rays, a lane taking the next one as soon as its ray is done
template <int KIND>
__device__ inline void defer_trace_kind(uint32_t* a, unsigned long long* prof)
{
    using namespace vrh::dev;
    const uint32_t n = a[1];
    const vrh_scene_view& v = *reinterpret_cast<const vrh_scene_view*>(a + 6);
    const float4* pairs = static_cast<const float4*>(v.pairs);
    const float4* prims = static_cast<const float4*>(v.prims);
    const uint32_t root = v.root;
    const bool finite_scene = v.finite_bounds != 0u;
    float4* ent = defer_log(a);
    const uint16_t* pool = reinterpret_cast<const uint16_t*>(a + 88);
    auto st = user_stack();
    constexpr uint32_t IDLE = 0xFFFFFFFFu;
    uint32_t cur = IDLE, next = 0u;
    ray_t r{};
    float max_t = 0.0f, best_t = FMAX;
    uint32_t pid = 0u, resume = NO_RESUME;  // (no descent cap: resume stays unset)
    bool fin = true, quad = false;          // (binary records only: quad stays false)
    hit_extra hx{ 0.0f, 0.0f, 0u };
    test_counts cnt{};
#if VRH_DEFER_PROF
    uint32_t prof_it = 0u, prof_busy = 0u;
#endif
    for (;;)
    {
        const uint64_t idle = __ballot(cur == IDLE);
        if (idle != 0ull && next < n && (uint32_t(__popcll(idle)) >= DEFER_REFILL || idle == ~0ull))
        {
            const uint32_t k = next + __builtin_amdgcn_mbcnt_hi(uint32_t(idle >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(idle), 0u));
            if (cur == IDLE && k < n)
            {
                cur = uint32_t(pool[k]);
                const float4 e0 = ent[2u * cur], e1 = ent[2u * cur + 1u];
                r = make_ray(mk3(e0.x, e0.y, e0.z), mk3(e0.w, e1.x, e1.y));
                max_t = e1.z;
                best_t = FMAX;
                fin = finite_ray(r);
                st.reset();
                st.push(root);
            }
            next += uint32_t(__popcll(idle));
        }
        const bool busy = cur != IDLE;
        const uint64_t active = __ballot(busy);
        if (active == 0ull) break;
#if VRH_DEFER_PROF
        prof_it += 1u;
        prof_busy += uint32_t(__popcll(active));
#endif
        const bool fast = finite_scene && __ballot(busy && !fin) == 0ull;
        if (busy)
        {
            uint32_t steps = 0u;
            const int res = fast ? ray_step<KIND, false, true, true, void, false>(pairs, prims, nullptr, root, quad, r, max_t, true, st,
                                                                               best_t, pid, cnt, steps, 0xFFFFFFFFu, resume,
                                                                               0xFFFFFFFFu, DEFER_STEP_FLAGS, &hx)
                                 : ray_step<KIND, false, false, true, void, false>(pairs, prims, nullptr, root, quad, r, max_t, true, st,
                                                                                best_t, pid, cnt, steps, 0xFFFFFFFFu, resume,
                                                                                0xFFFFFFFFu, DEFER_STEP_FLAGS, &hx);
            if (res != 0)
            {
                if (res == 1) reinterpret_cast<uint32_t*>(ent + 2u * cur + 1u)[3] = DTAG_ANY | hx.li;
                else atomicOr(&defer_miss_bits(a)[cur >> 5], 1u << (cur & 31u));
                cur = IDLE;
            }
        }
    }
#if VRH_DEFER_PROF
    prof[4] += n;
    prof[5] += prof_it;
    prof[6] += prof_busy;
#endif
}

__device__ inline void defer_trace(unsigned long long* prof)
{
    uint32_t* a = defer_area();
    if (a[1] == 0u) return;
    if (reinterpret_cast<const vrh_scene_view*>(a + 6)->prim_kind == VRH_PRIM_TRI64) defer_trace_kind<vrh::dev::KIND_TRI>(a, prof);
    else defer_trace_kind<vrh::dev::KIND_SPHERE>(a, prof);
}

template <typename It>
using range_value_t = typename std::decay<decltype(*std::declval<It>())>::type;
template <typename It>
using is_bvh_ref_range = std::is_base_of<hip_bvh_ref, range_value_t<It>>;
} // hip_detail

template <typename P>
__host__ __device__ inline P hip_bvh_ref_t<P>::primitive(size_t i) const
{
    uint32_t flags;
    return hip_detail::leaf_primitive<P>(static_cast<const float4*>(view.prims), uint32_t(i), flags);
}

#if defined(VRH_REFERENCE_HEADERS)
// ================================================================================================
// The reference's traversal over the device BVH.  hip_bvh_ref_t<P> is one more index BVH for the
// reference's templates: closest_hit / any_hit / multi_hit over [begin, end) of refs run the
// reference's own traverse() (traverse_linear.inl:76-141), which calls the intersector's BVH
// overloads (intersector.h:38-106), which call intersect<Traversal>(ray, ref, isect, max_t, cond)
// below: libvrh's walk with the reference's leaf step -- HR(isect(ray, prim), i), update_cond,
// update_if, exit_traversal<Traversal> (intersect.inl:103-128) -- so the result records, the
// multi-hit insertion and any custom intersector are the reference's code.
// ================================================================================================

template <typename P>
struct is_index_bvh<hip_bvh_ref_t<P>> : std::true_type {};

namespace hip_detail
{
// is_closer(box record, result, max_t) compares the box's tnear with result.t, or for a multi-hit
// array with every entry's t (multi_hit.h: any entry) -- i.e. with the largest
template <typename RT>
__device__ inline float cull_of(RT const& r) { return r.t; }
template <typename HR, size_t N>
__device__ inline float cull_of(array<HR, N> const& r)
{
    float m = r[0].t;
    for (size_t k = 1; k < N; ++k) m = m < r[k].t ? r[k].t : m;
    return m;
}
} // hip_detail

template <
    detail::traversal_type Traversal,
    size_t MultiHitMax = 1,
    typename P,
    typename Intersector,
    typename Cond = is_closer_t
    >
VRH_FUNC inline auto intersect(
        basic_ray<float> const& ray,
        hip_bvh_ref_t<P> const& b,
        Intersector&            isect,
        float                   max_t = numeric_limits<float>::max(),
        Cond                    update_cond = Cond()
        )
    -> typename detail::traversal_result<
            hit_record_bvh<basic_ray<float>, hip_bvh_ref_t<P>, decltype(isect(ray, std::declval<P>()))>,
            Traversal, MultiHitMax>::type
{
    using HR = hit_record_bvh<basic_ray<float>, hip_bvh_ref_t<P>, decltype(isect(ray, std::declval<P>()))>;
    using RT = typename detail::traversal_result<HR, Traversal, MultiHitMax>::type;
    RT result;
    const vrh_scene_view view = hip_detail::uniform_view(b.view);
    const float4* prims = static_cast<const float4*>(view.prims);
    if constexpr (Traversal == detail::AnyHit && VRH_USER_ANYHIT_SHARE)
    {
        // the shared any-hit walk (hip_detail::walk_shared): the same leaf step on the ray being
        // traversed, into the record of this visit -- when every lane of the wave walks the same BVH
        // (a lane takes over another lane's subtrees); otherwise each lane walks its own below
        bool same_bvh = false;
        (void)hip_detail::first_lane_ptr(view.pairs, same_bvh);
        if (same_bvh)
        {
            if (view.max_depth >= VRH_USER_STACK) return result;
            const vrh::dev::ray_t r = hip_detail::dev_ray(ray);
            auto leaf2 = [&](vrh::dev::ray_t const& tr, float tmax, uint32_t i, uint32_t& flags, RT& rec) -> bool
            {
                const basic_ray<float> ray2(vector<3, float>(tr.ori.x, tr.ori.y, tr.ori.z), vector<3, float>(tr.dir.x, tr.dir.y, tr.dir.z));
                const P prim = hip_detail::leaf_primitive<P>(prims, i, flags);
                auto hr = HR(isect(ray2, prim), int(i));
                auto closer = update_cond(hr, rec, tmax);
                if (!any(closer)) return false;
                update_if(rec, hr, closer);
                detail::exit_traversal<Traversal> early_exit;
                return early_exit.check(rec);
            };
            if (view.finite_bounds && __ballot(!vrh::dev::finite_ray(r)) == 0ull)
                hip_detail::walk_shared<true>(view, r, max_t, result, leaf2);
            else
                hip_detail::walk_shared<false>(view, r, max_t, result, leaf2);
            return result;
        }
    }
    // the ordered cooperative walk (hip_detail::walk_ordered): default intersector and update rule
    constexpr bool orderable = VRH_USER_ANYHIT_ORDERED && Traversal == detail::AnyHit && MultiHitMax == 1
                               && std::is_same<Intersector, default_intersector>::value && std::is_same<Cond, is_closer_t>::value;
    if constexpr (orderable)
    {
        if (view.max_depth >= VRH_USER_STACK) return result;
        if (hip_detail::oca_wave_usable(view))
        {
            const vrh::dev::ray_t r = hip_detail::dev_ray(ray);
            auto test = [&](vrh::dev::ray_t const& tr, float tmax, uint32_t i, uint32_t& flags) -> bool
            {
                const basic_ray<float> ray2(vector<3, float>(tr.ori.x, tr.ori.y, tr.ori.z), vector<3, float>(tr.dir.x, tr.dir.y, tr.dir.z));
                const P prim = hip_detail::leaf_primitive<P>(prims, i, flags);
                return any(update_cond(HR(isect(ray2, prim), int(i)), RT(), tmax));
            };
            const uint32_t w = (view.finite_bounds && __ballot(!vrh::dev::finite_ray(r)) == 0ull)
                             ? hip_detail::walk_ordered<true>(view, r, max_t, test) : hip_detail::walk_ordered<false>(view, r, max_t, test);
            if (w != hip_detail::OCA_NONE)
            {
                // the owner's own leaf step on the primitive its ray's walk accepts first
                uint32_t flags = 0;
                const P prim = hip_detail::leaf_primitive<P>(prims, w, flags);
                auto hr = HR(isect(ray, prim), int(w));
                auto closer = update_cond(hr, result, max_t);
                if (any(closer)) update_if(result, hr, closer);
            }
            return result;
        }
    }
    // deferred calls (VRH_USER_DEFER: user_render's record / trace / replay phases): the default
    // intersector and update rule on one primitive type, one hit record
    constexpr bool deferrable = VRH_USER_DEFER && MultiHitMax == 1 && Traversal != detail::MultiHit
                                && std::is_same<Intersector, default_intersector>::value && std::is_same<Cond, is_closer_t>::value;
    hip_detail::defer_call d{ hip_detail::DEFER_RUN, 0u, hip_detail::DTAG_NONE };
    if constexpr (deferrable)
    {
        d = hip_detail::defer_begin(view, ray, max_t, Traversal == detail::AnyHit);
        if (d.state == hip_detail::DEFER_PENDING) return result;     // record phase: answered in the replay
        if (d.state == hip_detail::DEFER_LOGGED)
        {
            if (d.li == hip_detail::DTAG_NONE) return result;
            // the logged answer: the one primitive it names, through the walk's own leaf step
            uint32_t flags = 0;
            const P prim = hip_detail::leaf_primitive<P>(prims, d.li, flags);
            auto hr = HR(isect(ray, prim), int(d.li));
            auto closer = update_cond(hr, result, max_t);
            if (any(closer))
            {
                update_if(result, hr, closer);
                return result;
            }
        }
    }
    uint32_t won = hip_detail::DTAG_NONE;      // the leaf index of the primitive the result holds
    hip_detail::walk<Traversal == detail::AnyHit>(view, ray, max_t, [&]() { return hip_detail::cull_of(result); },
                     [&](uint32_t i, uint32_t& flags) -> bool
                     {
                         const P prim = hip_detail::leaf_primitive<P>(prims, i, flags);
                         auto hr = HR(isect(ray, prim), int(i));
                         auto closer = update_cond(hr, result, max_t);
                         if (!any(closer)) return false;
                         update_if(result, hr, closer);
                         won = i;
                         detail::exit_traversal<Traversal> early_exit;
                         return early_exit.check(result);
                     });
    if constexpr (deferrable)
        if (d.state == hip_detail::DEFER_RUN_LOG) hip_detail::defer_log_closest(d, ray, max_t, won);
    return result;
}

// the default (closest hit) overloads, intersect.inl:140-189
template <typename P, typename Intersector, typename Cond = is_closer_t>
VRH_FUNC inline auto intersect(basic_ray<float> const& ray, hip_bvh_ref_t<P> const& b, Intersector& isect,
                                 Cond update_cond = Cond())
    -> hit_record_bvh<basic_ray<float>, hip_bvh_ref_t<P>, decltype(isect(ray, std::declval<P>()))>
{
    return intersect<detail::ClosestHit>(ray, b, isect, numeric_limits<float>::max(), update_cond);
}

template <typename P>
VRH_FUNC inline auto intersect(basic_ray<float> const& ray, hip_bvh_ref_t<P> const& b)
    -> hit_record_bvh<basic_ray<float>, hip_bvh_ref_t<P>, decltype(intersect(ray, std::declval<P>()))>
{
    default_intersector isect;
    return intersect<detail::ClosestHit>(ray, b, isect, numeric_limits<float>::max(), is_closer_t());
}

#else
// ================================================================================================
// standalone: closest_hit / any_hit over hip_bvh_ref ranges and primitive arrays
// ================================================================================================

namespace hip_detail
{
// the hit record of intersect(ray, primitive) -- and of every intersector built on it
using prim_record = hit_record<basic_ray<float>, primitive<unsigned>>;
using bvh_record = hit_record_bvh<prim_record>;

template <bool Any, typename Isect>
__device__ inline bvh_record traverse_bvh_direct(basic_ray<float> const& ray, vrh_scene_view const& b, Isect& isect, float max_t)
{
    using HR = prim_record;
    bvh_record result;
    const float4* prims = static_cast<const float4*>(b.prims);
    if constexpr (Any && VRH_USER_ANYHIT_SHARE)
    {
        // lanes take over each other's subtrees: only when the wave walks one BVH
        bool same_bvh = false;
        (void)first_lane_ptr(b.pairs, same_bvh);
        if (same_bvh)
        {
            if (b.max_depth >= VRH_USER_STACK) return result;
            const vrh::dev::ray_t r = dev_ray(ray);
            auto leaf2 = [&](vrh::dev::ray_t const& tr, float tmax, uint32_t i, uint32_t& flags, bvh_record& rec) -> bool
            {
                const basic_ray<float> ray2(vec3(tr.ori.x, tr.ori.y, tr.ori.z), vec3(tr.dir.x, tr.dir.y, tr.dir.z));
                HR hr;
                if (b.prim_kind == VRH_PRIM_TRI64) hr = isect(ray2, leaf_primitive<basic_triangle<3, float>>(prims, i, flags));
                else hr = isect(ray2, leaf_primitive<basic_sphere<float>>(prims, i, flags));
                if (!is_closer(hr, static_cast<HR const&>(rec), tmax)) return false;
                rec = bvh_record(hr, i);
                return true;                                      // exit_traversal.h:49-56
            };
            if (b.finite_bounds && __ballot(!vrh::dev::finite_ray(r)) == 0ull) walk_shared<true>(b, r, max_t, result, leaf2);
            else walk_shared<false>(b, r, max_t, result, leaf2);
            return result;
        }
    }
    if constexpr (Any && VRH_USER_ANYHIT_ORDERED && std::is_same<Isect, default_intersector>::value)
    {
        // the ordered cooperative walk (walk_ordered): the reference's first hit, lanes sharing the work
        if (b.max_depth >= VRH_USER_STACK) return result;
        if (oca_wave_usable(b))
        {
            const vrh::dev::ray_t r = dev_ray(ray);
            auto test = [&](vrh::dev::ray_t const& tr, float tmax, uint32_t i, uint32_t& flags) -> bool
            {
                const basic_ray<float> ray2(vec3(tr.ori.x, tr.ori.y, tr.ori.z), vec3(tr.dir.x, tr.dir.y, tr.dir.z));
                HR hr;
                if (b.prim_kind == VRH_PRIM_TRI64) hr = isect(ray2, leaf_primitive<basic_triangle<3, float>>(prims, i, flags));
                else hr = isect(ray2, leaf_primitive<basic_sphere<float>>(prims, i, flags));
                return is_closer(hr, HR(), tmax);
            };
            const uint32_t w = (b.finite_bounds && __ballot(!vrh::dev::finite_ray(r)) == 0ull)
                             ? walk_ordered<true>(b, r, max_t, test) : walk_ordered<false>(b, r, max_t, test);
            if (w != OCA_NONE)
            {
                uint32_t flags = 0;
                HR hr;
                if (b.prim_kind == VRH_PRIM_TRI64) hr = isect(ray, leaf_primitive<basic_triangle<3, float>>(prims, w, flags));
                else hr = isect(ray, leaf_primitive<basic_sphere<float>>(prims, w, flags));
                if (is_closer(hr, static_cast<HR const&>(result), max_t)) result = bvh_record(hr, w);
            }
            return result;
        }
    }
    // the leaf: every primitive in index order, is_closer / update_if (intersect.inl:103-128).  One walk
    // per primitive type, chosen by the (wave-uniform) scene kind, so the leaf step of the walk tests
    // one type of primitive (C3, AO lambda: 1.699 vs 1.721 ms per frame with the kind tested per
    // primitive, 2.045 vs 2.108 at one frame per launch, profiles/r06/user_walk/kind_walks.log)
    auto walk_prims = [&](auto prim_tag)
    {
        using P = decltype(prim_tag);
        walk<Any>(b, ray, max_t, [&]() { return result.t; },
             [&](uint32_t i, uint32_t& flags) -> bool
             {
                 const HR hr = isect(ray, leaf_primitive<P>(prims, i, flags));
                 if (is_closer(hr, static_cast<HR const&>(result), max_t))
                 {
                     result = bvh_record(hr, i);
                     if (Any) return true;                     // exit_traversal.h:49-56
                 }
                 return false;
             });
    };
    if (b.prim_kind == VRH_PRIM_TRI64) walk_prims(basic_triangle<3, float>());
    else walk_prims(basic_sphere<float>());
    return result;
}

template <bool Any, typename Isect>
__device__ inline bvh_record traverse_bvh(basic_ray<float> const& ray, vrh_scene_view const& b, Isect& isect, float max_t)
{
    if constexpr (VRH_USER_DEFER && std::is_same<Isect, default_intersector>::value)
    {
        // deferred calls (user_render's record / trace / replay phases, above)
        const defer_call d = defer_begin(b, ray, max_t, Any);
        if (d.state == DEFER_PENDING) return bvh_record();        // record phase: answered in the replay
        if (d.state == DEFER_LOGGED)
        {
            if (d.li == DTAG_NONE) return bvh_record();
            // the logged answer: the one primitive it names, tested and merged as the walk's leaf does
            const float4* prims = static_cast<const float4*>(b.prims);
            uint32_t flags = 0;
            prim_record hr;
            if (b.prim_kind == VRH_PRIM_TRI64) hr = isect(ray, leaf_primitive<basic_triangle<3, float>>(prims, d.li, flags));
            else hr = isect(ray, leaf_primitive<basic_sphere<float>>(prims, d.li, flags));
            if (is_closer(hr, prim_record(), max_t)) return bvh_record(hr, d.li);
        }
        bvh_record res = traverse_bvh_direct<Any>(ray, b, isect, max_t);
        if (d.state == DEFER_RUN_LOG) defer_log_closest(d, ray, max_t, res.hit ? res.primitive_list_index : DTAG_NONE);
        return res;
    }
    return traverse_bvh_direct<Any>(ray, b, isect, max_t);
}
} // hip_detail

// closest_hit / any_hit over [begin, end) of hip_bvh_ref (traverse_linear.inl:76-141): every BVH on
// its own with the same max_t, merged by update_if(result, hr, is_closer(hr, result, max_t));
// any_hit stops at the first BVH with a hit
template <typename It, typename Isect, typename = typename std::enable_if<hip_detail::is_bvh_ref_range<It>::value>::type>
__device__ inline hip_detail::bvh_record closest_hit(basic_ray<float> const& ray, It begin, It end, Isect& isect)
{
    hip_detail::bvh_record result;
    for (It it = begin; it != end; ++it)
    {
        auto hr = hip_detail::traverse_bvh<false>(ray, hip_detail::uniform_view(it->view), isect, FLT_MAX);
        if (is_closer(hr, result, FLT_MAX)) result = hr;
    }
    return result;
}

template <typename It, typename Isect, typename = typename std::enable_if<hip_detail::is_bvh_ref_range<It>::value>::type>
__device__ inline hip_detail::bvh_record any_hit(basic_ray<float> const& ray, It begin, It end, float max_t, Isect& isect)
{
    hip_detail::bvh_record result;
    for (It it = begin; it != end; ++it)
    {
        auto hr = hip_detail::traverse_bvh<true>(ray, hip_detail::uniform_view(it->view), isect, max_t);
        if (is_closer(hr, result, max_t)) result = hr;
        if (result.hit) return result;
    }
    return result;
}

// the same over [begin, end) of primitives (traverse_linear.inl:25-62): a linear scan
template <typename It, typename Isect, typename = typename std::enable_if<!hip_detail::is_bvh_ref_range<It>::value>::type,
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

template <typename It, typename Isect, typename = typename std::enable_if<!hip_detail::is_bvh_ref_range<It>::value>::type,
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
#endif // VRH_REFERENCE_HEADERS

//-------------------------------------------------------------------------------------------------
// Samplers.  A kernel taking a sampler, kernel(ray, random_sampler<float>& samp), gets the
// reference's random_sampler<float> (random_sampler.h:24-57) seeded per pixel as cuda_sched seeds it
// (cuda_sched.inl:20-45: cuda_hash(tic() + y * w + x)), with the clock tic() replaced by
// frame_num * W * H so that frames are reproducible and the seeds of consecutive frames distinct:
//
//     seed(x, y) = cuda_hash(frame_num * W * H + y * W + x)        (32-bit unsigned arithmetic)
//
// The reference CPU path run with the same seeds draws the same numbers bit for bit
// (oracle/ref_harness.cpp `rsampler`, tests/test_gpu_ref_kernels.py).
//   hip_ao_sample(p, s, frame) is the built-in AO kernel's cosine-hemisphere sample s of pixel p
//   (Malley disk point, z = sqrt(1 - x^2 - y^2)) -- the same sample set as VRH_KERNEL_AO, so a user
//   AO kernel can reproduce the built-in kernel's frames.
//

namespace hip_detail
{
// cuda_sched.inl:27-36 (the integer hash of thrust's monte_carlo example)
__device__ inline unsigned seed_hash(unsigned a)
{
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}

__device__ inline unsigned pixel_seed(unsigned x, unsigned y, unsigned w, unsigned h, unsigned frame_num)
{
    return seed_hash(frame_num * w * h + y * w + x);
}
} // hip_detail

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
// The launch: a persistent grid of one-wave blocks (8 x 8 threads = one 8 x 8 pixel tile, dynamic
// LDS for the traversal stacks) sized to what is resident on the GPU; the waves take tiles from
// eight per-XCD queues (vrh_ctx_user_queues) until every tile of every frame is done -- the tiles of
// a queue are a contiguous strip of each frame (BVH nodes stay in that XCD's L2), a wave drains its
// own XCD's queue first and then the others in turn.  Per pixel it is cuda_sched.inl:53-99 with
// sample_pixel's uniform store (colour, and the depth into the target's t buffer when the result
// carries one).  frames(): several frames per launch (frames in flight), frame f with its own camera
// and frame number into rows [f * H, (f + 1) * H) of the target, so the launch's tail is paid once.
//

namespace hip_detail
{
template <uint32_t NC>
struct user_frames
{
    vrh_camera cam[NC];
    float4* color;
    float* t;
    uint32_t width, height, frame_num, nframes;
    uint32_t x0, y0, x1, y1;      // scissor box, exclusive right / bottom edges
    uint32_t tiles_x, tiles;      // 8 x 8 tiles of the box per row / per frame
    uint32_t* queues;             // vrh_ctx_user_queues: 8 heads, VRH_USER_QUEUE_STRIDE words apart
    uint32_t matrix_cam;          // sched_params with camera matrices: their inverses (column-major)
    float inv_view[16], inv_proj[16];
    char* defer_log;              // VRH_USER_DEFER: DEFER_WAVE_BYTES per block of the grid
    uint32_t stack_entries;       // LDS stack entries per thread of this launch (USER_STACK_SIZED)
};

// the primary ray through image position (fx, fy) (the pixel plus the sampler's offset) of camera c:
// sched_common.h:130-150 (pinhole basis) or :152-176 (camera matrices), the built-in kernels' arithmetic
template <uint32_t NC>
__device__ inline basic_ray<float> user_primary_ray(user_frames<NC> const& f, uint32_t c, float fx, float fy)
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
    vrh_camera const& cam = f.cam[c];
    const vec3 cu(cam.cam_u[0], cam.cam_u[1], cam.cam_u[2]);
    const vec3 cv(cam.cam_v[0], cam.cam_v[1], cam.cam_v[2]);
    const vec3 cw(cam.cam_w[0], cam.cam_w[1], cam.cam_w[2]);
    const vec3 eye(cam.eye[0], cam.eye[1], cam.eye[2]);
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

// pixel (x, y) of frame c of the launch; STORE = false (the record phase of VRH_USER_DEFER) runs the
// kernel without storing its results
template <typename K, uint32_t SK, uint32_t SN, uint32_t NC, bool STORE = true>
__device__ inline void user_pixel(K& kernel, user_frames<NC> const& f, uint32_t c, uint32_t x, uint32_t y)
{
    const uint32_t frame_num = f.frame_num + c;
    random_sampler<float> samp(pixel_seed(x, y, f.width, f.height, frame_num));
    const size_t o = (size_t(c) * f.height + y) * f.width + x;
    if constexpr (SK == VRH_SAMPLER_UNIFORM)
    {
        // sched_common.h:130-176 make_primary_ray_impl (uniform pixel sampler), as the built-in kernels
        auto res = invoke_kernel(kernel, user_primary_ray(f, c, (float)x, (float)y), samp, x, y, 0);
        if (STORE && f.color) f.color[o] = make_float4(res.color.x, res.color.y, res.color.z, res.color.w);
        if constexpr (has_depth<decltype(res)>::value)
            if (STORE && f.t) f.t[o] = res.depth;
    }
    else
    {
        // the jittered / jittered_blend / ssaa<N> samplers (sched_common.h:196-300, 440-720), with the
        // jitter draws and offset tables of vrh.h vrh_pixel_sampler
        auto ray_at = [&](float ox, float oy) { return user_primary_ray(f, c, (float)x + ox, (float)y + oy); };
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
                    if (STORE && f.t) f.t[o] = res.depth;
            }
            if (STORE && f.color) f.color[o] = d;
        }
        else
        {
            const uint32_t k = (y * f.width + x) * 2u + 0x632BE5ABu + frame_num * 0x68E31DA4u;
            const float oy = vrh::dev::uniform01(k) - 0.5f, ox = vrh::dev::uniform01(k + 1u) - 0.5f;
            auto res = invoke_kernel(kernel, ray_at(ox, oy), samp, x, y, 0);
            float4 cl = make_float4(res.color.x, res.color.y, res.color.z, res.color.w);
            if constexpr (SK == VRH_SAMPLER_JITTERED_BLEND)
            {
                const float a = 1.0f / float(frame_num), b = 1.0f - a;
                if (f.color)
                {
                    const float4 d = f.color[o];
                    cl = make_float4(cl.x * a + d.x * b, cl.y * a + d.y * b, cl.z * a + d.z * b, cl.w * a + d.w * b);
                }
            }
            if (STORE && f.color) f.color[o] = cl;
            if constexpr (has_depth<decltype(res)>::value)
                if (STORE && f.t) f.t[o] = res.depth;
        }
    }
}

__device__ inline uint32_t xcc_id()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}

// the persistent loop: queue q hands out strip q (tiles [tiles * q / 8, tiles * (q + 1) / 8)) of
// every frame, in cluster order (VRH_USER_CLUSTER, below) or frame-major; every (frame, tile) is
// handed out exactly once by one of the 8 heads, so
// which XCD a wave runs on changes only speed.  Every wave leaves once all 8 queues are empty.
// VRH_USER_WAVES: waves per SIMD the register allocation targets (0: the compiler's choice)
#if VRH_USER_DEFER && !defined(VRH_USER_WAVES)
// the deferred build's LDS (8 KB of stacks + 2.2 KB of log state per wave) holds a CU to 15 waves, so
// it targets 4 waves per SIMD: without the target the AO lambda drifted to 130-134 VGPRs (3 waves) on
// small source changes -- 1.92 vs 1.65 ms per frame (profiles/r06/defer_regs/)
#define VRH_USER_WAVES 4
#endif
#ifndef VRH_USER_WAVES
#define VRH_USER_WAVES 0
#endif
// VRH_USER_CLUSTER: with several frames per launch, tiles per cluster of the hand-out order (the
// frames of a cluster back to back); 0: frame-major strips.  ao/main.cpp's kernel, C3, 32 frames per
// launch (profiles/r04/user/cluster_ab.log): strips 1.858 ms per frame, clusters of 8 tiles 1.765,
// of 1 tile (a tile's frames back to back) 1.744; 4 / 16 / 64 tiles as 8
#ifndef VRH_USER_CLUSTER
#define VRH_USER_CLUSTER 1u
#endif
#if VRH_USER_WAVES
#define VRH_USER_OCC __attribute__((amdgpu_waves_per_eu(VRH_USER_WAVES)))
#else
#define VRH_USER_OCC
#endif
template <typename K, uint32_t SK, uint32_t SN, uint32_t NC>
__device__ __forceinline__ void user_render_body(K& kernel, user_frames<NC> const& f);

template <typename K, uint32_t SK = VRH_SAMPLER_UNIFORM, uint32_t SN = 1, uint32_t NC = 1>
__global__ __launch_bounds__(64) VRH_USER_OCC void user_render(K kernel, user_frames<NC> f)
{
    user_render_body<K, SK, SN, NC>(kernel, f);
}

// VRH_USER_AUTO_WAVES (default on unless VRH_USER_WAVES or VRH_USER_DEFER is set): the same kernel
// also compiled for a 5-wave register target; the launch takes it when it holds more waves per CU
// and spills at most VRH_USER_AUTO_SCRATCH bytes per lane (the AO lambda: 104 VGPRs = 4 waves, or 96
// with 4 spilled = 5 waves: +4.2 %, profiles/r05/user/; round 6: 64 B, below)
#ifndef VRH_USER_AUTO_WAVES
#define VRH_USER_AUTO_WAVES (VRH_USER_WAVES == 0 && !VRH_USER_DEFER)
#endif
#ifndef VRH_USER_AUTO_SCRATCH
// round 6: the AO lambda with global loads is 96 VGPRs + 48 B of scratch at 5 waves against 114 VGPRs
// at 4: 1.750 vs 1.821 ms per frame (profiles/r06/user_loads/), so up to 64 B
#define VRH_USER_AUTO_SCRATCH 64
#endif
#ifndef VRH_USER_AUTO_SCRATCH6
// the 6-wave instance may spill more: with 24 LDS stack entries the AO lambda at 6 waves (80 VGPRs +
// 108 B of scratch) ran 1.542 ms per frame against 1.607 at 5 (96 + 28 B), ao/main.cpp's kernel at 6
// (80 + 216 B) 1.495 against 1.588 at 5 (96 + 20 B) (profiles/r06/user_lds/)
#define VRH_USER_AUTO_SCRATCH6 256
#endif
#ifndef VRH_USER_MAX_DEVICES
#define VRH_USER_MAX_DEVICES 64     // device ordinals the per-device launch choices are cached for
#endif
#if VRH_USER_AUTO_WAVES
template <typename K, uint32_t SK = VRH_SAMPLER_UNIFORM, uint32_t SN = 1, uint32_t NC = 1>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void user_render_w5(K kernel, user_frames<NC> f)
{
    user_render_body<K, SK, SN, NC>(kernel, f);
}
template <typename K, uint32_t SK = VRH_SAMPLER_UNIFORM, uint32_t SN = 1, uint32_t NC = 1>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void user_render_w6(K kernel, user_frames<NC> f)
{
    user_render_body<K, SK, SN, NC>(kernel, f);
}
#endif

template <typename K, uint32_t SK, uint32_t SN, uint32_t NC>
__device__ __forceinline__ void user_render_body(K& kernel, user_frames<NC> const& f)
{
    const uint32_t lane = threadIdx.y * 8u + threadIdx.x;
    if constexpr (USER_STACK_SIZED)
    {
        extern __shared__ uint32_t vrh_user_smem[];
        if (lane == 0u) vrh_user_smem[0] = f.stack_entries;        // the stack entries this launch gives
        __syncthreads();
    }
    if (VRH_USER_ANYHIT_CUT && lane == 0u) user_cut_area()[2] = 0u;     // no any_hit entry cut yet
    if (VRH_USER_DEFER && lane == 0u) defer_area()[0] = DEFER_OFF;
    unsigned long long prof[8] = {};         // VRH_DEFER_PROF
    (void)prof;
    uint32_t q = xcc_id();
    for (uint32_t tried = 0; tried < 8u; ++tried, q = (q + 1u) & 7u)
    {
        const uint32_t lo = uint32_t((uint64_t(f.tiles) * q) / 8u);
        const uint32_t len = uint32_t((uint64_t(f.tiles) * (q + 1u)) / 8u) - lo;
        const uint32_t n = len * f.nframes;
        for (;;)
        {
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(f.queues + q * VRH_USER_QUEUE_STRIDE, 1u);
            t = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)t, 0));
            if (t >= n) break;
            uint32_t c, tile;
            if (VRH_USER_CLUSTER > 0u && f.nframes > 1u)
            {
                // cluster order: the strip's tiles in clusters of VRH_USER_CLUSTER, the frames of a
                // cluster handed out back to back (the last cluster may be narrower)
                const uint32_t C = VRH_USER_CLUSTER, F = f.nframes;
                const uint32_t cl = t / (C * F);
                const uint32_t r = t - cl * C * F;
                const uint32_t cw = min(C, len - cl * C);
                c = r / cw;
                tile = lo + cl * C + (r - c * cw);
            }
            else
            {
                c = t / len;
                tile = lo + (t - c * len);
            }
            const uint32_t ty = tile / f.tiles_x;
            const uint32_t x = f.x0 + (tile - ty * f.tiles_x) * 8u + threadIdx.x;
            const uint32_t y = f.y0 + ty * 8u + threadIdx.y;
            const bool in = x < f.x1 && y < f.y1;
            if constexpr (VRH_USER_DEFER)
            {
                // record, trace, replay (the deferred any_hit calls, above); one wave per block, so the
                // barriers only order the phases' LDS and global accesses
                uint32_t* da = defer_area();
                da[24u + lane] = 0u;
                for (uint32_t w = lane; w < DEFER_MISS_WORDS; w += 64u) defer_miss_bits(da)[w] = 0u;
                if (lane == 0u)
                {
                    const uintptr_t log = uintptr_t(f.defer_log + size_t(blockIdx.x) * DEFER_WAVE_BYTES);
                    da[0] = DEFER_RECORD; da[1] = 0u; da[2] = 0u;
                    da[4] = uint32_t(log); da[5] = uint32_t(uint64_t(log) >> 32);
                }
                __syncthreads();
#if VRH_DEFER_PROF
                const uint64_t p0 = clock64();
#endif
                if (in) user_pixel<K, SK, SN, NC, false>(kernel, f, c, x, y);
                __threadfence_block();
                __syncthreads();
#if VRH_DEFER_PROF
                const uint64_t p1 = clock64();
#endif
                if (da[2] != 0u) defer_trace(prof);
                __threadfence_block();
                __syncthreads();
#if VRH_DEFER_PROF
                const uint64_t p2 = clock64();
#endif
                da[24u + lane] = (da[24u + lane] & 0xFFFFu) << 16;     // logged calls, and the count from 0
                if (lane == 0u) da[0] = DEFER_REPLAY;
                __syncthreads();
                if (in) user_pixel<K, SK, SN, NC>(kernel, f, c, x, y);
                __syncthreads();
#if VRH_DEFER_PROF
                const uint64_t p3 = clock64();
                prof[0] += p1 - p0;
                prof[1] += p2 - p1;
                prof[2] += p3 - p2;
                prof[3] += 1u;
#endif
            }
            else if (in) user_pixel<K, SK, SN, NC>(kernel, f, c, x, y);
        }
    }
#if VRH_DEFER_PROF
    if (VRH_USER_DEFER && lane == 0u)
    {
        prof[7] = DEFER_PROF_MAGIC;
        unsigned long long* o = reinterpret_cast<unsigned long long*>(f.defer_log + size_t(blockIdx.x) * DEFER_WAVE_BYTES);
        for (int k = 0; k < 8; ++k) o[k] = prof[k];
    }
#endif
}

// at least `bytes` of device memory kept with the context (grown after a device sync: earlier
// launches on the context's stream may still use the old block)
inline char* context_scratch(hip_context& ctx, size_t bytes)
{
    auto& sb = ctx.scratch();
    if (bytes > sb.bytes)
    {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
            throw hip_error("hip_sched: device scratch: device sync", VRH_ERR_HIP);
        sb.mem.reset();
        sb.bytes = 0;
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) throw hip_error("hip_sched: device scratch: hipMalloc", VRH_ERR_OOM);
        sb.mem.reset(p, [dev](void* q) {
            int d0 = 0;
            if (hipGetDevice(&d0) == hipSuccess && hipSetDevice(dev) == hipSuccess)
            {
                (void)hipFree(q);
                (void)hipSetDevice(d0);
            }
        });
        sb.bytes = bytes;
    }
    return static_cast<char*>(sb.mem.get());
}

// what the calling thread's last user-kernel launch chose: the instance's register target (0: the
// compiler's own allocation, else 5 or 6 waves per SIMD), its one-wave blocks per CU, the LDS stack
// entries per thread and the grid (the bench line reports them)
struct user_launch_info
{
    int waves_target = 0;
    int blocks_per_cu = 0;
    uint32_t stack_entries = 0;
    uint32_t grid = 0;
};
inline user_launch_info& last_user_launch()
{
    static thread_local user_launch_info info;
    return info;
}

// launch `kern` over f on the context's stream: the queues zeroed first, then a grid of as many
// one-wave blocks as the GPU holds at once (the kernel's own occupancy), at most one per tile
template <typename K, uint32_t SK, uint32_t SN, uint32_t NC>
inline hipError_t launch_user_render(hip_context& ctx, K const& kernel, user_frames<NC>& f, hipStream_t stream)
{
    static_assert(!USER_STACK_SIZED || !(VRH_USER_DEFER || VRH_USER_ANYHIT_CUT || VRH_USER_ANYHIT_SHARE || VRH_USER_ANYHIT_ORDERED),
                  "the deferred calls, the entry cut and the shared / ordered any_hit walks keep their state in whole LDS stack columns");
    // the stack the deepest BVH the program has taken a ref of needs, at least VRH_USER_LDS_STACK and at
    // most VRH_USER_STACK entries per thread: fewer entries, fewer bytes of LDS per block, more blocks
    if (USER_STACK_SIZED)
    {
        const uint32_t need = user_ref_depth().load(std::memory_order_acquire) + 1u;
        f.stack_entries = need < VRH_USER_LDS_STACK ? VRH_USER_LDS_STACK : need > VRH_USER_STACK ? VRH_USER_STACK : need;
    }
    else
        f.stack_entries = VRH_USER_STACK;
    const size_t lds = (size_t(64) * f.stack_entries + USER_LDS_HEADER + (VRH_USER_ANYHIT_CUT ? UCUT_WORDS : 0u)
                        + (VRH_USER_DEFER ? DEFER_WORDS : 0u)) * sizeof(uint32_t);
    auto fn = user_render<K, SK, SN, NC>;
    check(vrh_ctx_user_queues(ctx.get(), &f.queues), "vrh_ctx_user_queues");
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, lds);
    if (e != hipSuccess) return e;
#if VRH_USER_AUTO_WAVES
    {
        // once per kernel and device: the instance for 5 or 6 waves / SIMD when it holds more waves per CU
        // and spills at most VRH_USER_AUTO_SCRATCH (5) / VRH_USER_AUTO_SCRATCH6 (6) bytes per lane, the
        // one with more waves first.  The answer is cached per device ordinal (devices of different
        // architectures get their own), in atomics: 0 = not asked yet, else (waves << 8) | blocks per CU
        // of the chosen instance.  Two threads asking at once compute the same answer.
        static std::atomic<int> wave_cache[VRH_USER_MAX_DEVICES][VRH_USER_STACK + 1];     // [device][stack entries]
        auto fn5 = user_render_w5<K, SK, SN, NC>;
        auto fn6 = user_render_w6<K, SK, SN, NC>;
        const uint32_t se = f.stack_entries;
        int pick = (dev >= 0 && dev < VRH_USER_MAX_DEVICES) ? wave_cache[dev][se].load(std::memory_order_acquire) : 0;
        if (pick == 0)
        {
            pick = (1 << 8) | per_cu;
            const std::pair<decltype(fn), int> cand[2] = { { fn6, VRH_USER_AUTO_SCRATCH6 }, { fn5, VRH_USER_AUTO_SCRATCH } };
            for (int k = 0; k < 2; ++k)
            {
                hipFuncAttributes a{};
                int n = 0;
                if ((e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(cand[k].first))) != hipSuccess) return e;
                if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, cand[k].first, 64, lds)) != hipSuccess) return e;
                if (n > per_cu && a.localSizeBytes <= size_t(cand[k].second))
                {
                    pick = ((6 - k) << 8) | n;
                    break;
                }
            }
            if (dev >= 0 && dev < VRH_USER_MAX_DEVICES) wave_cache[dev][se].store(pick, std::memory_order_release);
        }
        if ((pick >> 8) == 6) fn = fn6;
        else if ((pick >> 8) == 5) fn = fn5;
        per_cu = pick & 0xFF;
        last_user_launch().waves_target = (pick >> 8) > 1 ? (pick >> 8) : 0;
    }
#endif
    const uint64_t work = uint64_t(f.tiles) * f.nframes;
    const uint64_t resident = uint64_t(cus > 0 ? cus : 1) * uint64_t(per_cu > 0 ? per_cu : 1);
    const uint32_t grid = uint32_t(work < resident ? work : resident);
    auto& info = last_user_launch();
    if (!VRH_USER_AUTO_WAVES) info.waves_target = VRH_USER_WAVES;
    info.blocks_per_cu = per_cu;
    info.stack_entries = f.stack_entries;
    info.grid = grid;
    if (VRH_USER_DEFER) f.defer_log = context_scratch(ctx, size_t(grid) * DEFER_WAVE_BYTES);
    if ((e = hipMemsetAsync(f.queues, 0, 8u * VRH_USER_QUEUE_STRIDE * sizeof(uint32_t), stream)) != hipSuccess) return e;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(8, 8), lds, stream, kernel, f);
    return hipGetLastError();
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
        user_frames<1> f{};
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
                                  &f.cam[0]),
                  "vrh_make_camera");
        }
        set_scissor(sparams, f.cam[0]);
        if constexpr (has_sched_intersector<SP>::value)
        {
            using I = typename std::decay<decltype(sparams.intersector)>::type;
            using C = call_with_intersector<K, I>;
            run<C, PS::kind, PS::count>(ctx, C{ kernel, sparams.intersector }, f, rt, 1u, uint32_t(rt.height()), frame_num);
        }
        else
            run<K, PS::kind, PS::count>(ctx, kernel, f, rt, 1u, uint32_t(rt.height()), frame_num);
    }

    // frames in flight: camera f into rows [f * H, (f + 1) * H) of rt (height = cams.size() * H),
    // frame number frame_num + f; every frame equals its own frame() call
    template <typename Camera, typename RT>
    static void frames(hip_context& ctx, K const& kernel, std::vector<Camera> const& cams, RT& rt, unsigned frame_num)
    {
        if (cams.empty() || cams.size() > VRH_MAX_BATCH || rt.height() % cams.size() != 0)
            throw std::runtime_error("hip_sched::frames: 1..VRH_MAX_BATCH cameras, render target height = frames x image height");
        const uint32_t W = uint32_t(rt.width()), H = uint32_t(rt.height() / cams.size());
        user_frames<VRH_MAX_BATCH> f{};
        for (size_t c = 0; c < cams.size(); ++c)
        {
            auto const& cam = cams[c];
            float eye[3] = { cam.eye().x, cam.eye().y, cam.eye().z };
            float center[3] = { cam.center().x, cam.center().y, cam.center().z };
            float up[3] = { cam.up().x, cam.up().y, cam.up().z };
            check(vrh_make_camera(eye, center, up, cam.fovy(), cam.aspect(), W, H, &f.cam[c]), "vrh_make_camera");
        }
        run<K, VRH_SAMPLER_UNIFORM, 1>(ctx, kernel, f, rt, uint32_t(cams.size()), H, frame_num);
    }

private:
    template <typename KK, uint32_t SK, uint32_t SN, uint32_t NC, typename RT>
    static void run(hip_context& ctx, KK const& kk, user_frames<NC>& f, RT& rt, uint32_t nframes, uint32_t H,
                    unsigned frame_num)
    {
        f.width = uint32_t(rt.width());
        f.height = H;
        f.frame_num = frame_num;
        f.nframes = nframes;
        const uint32_t* sc = f.cam[0].scissor;
        const bool whole = sc[0] == 0 && sc[1] == 0 && sc[2] == 0 && sc[3] == 0;
        f.x0 = whole ? 0u : sc[0];
        f.y0 = whole ? 0u : sc[1];
        f.x1 = whole ? f.width : (sc[2] < f.width ? sc[2] : f.width);
        f.y1 = whole ? f.height : (sc[3] < f.height ? sc[3] : f.height);
        const bool any = f.x1 > f.x0 && f.y1 > f.y0;
        f.tiles_x = any ? (f.x1 - f.x0 + 7u) / 8u : 0u;
        f.tiles = any ? f.tiles_x * ((f.y1 - f.y0 + 7u) / 8u) : 0u;
        auto ref = rt.ref();
        f.color = reinterpret_cast<float4*>(ref.color);
        f.t = ref.t;
        int dev = 0, prev = 0;
        void* stream = nullptr;
        check(vrh_ctx_get_stream(ctx.get(), &dev, &stream), "vrh_ctx_get_stream");
        if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(dev) != hipSuccess) throw hip_error("hipSetDevice", VRH_ERR_HIP);
        rt.begin_frame();
        hipError_t e = hipSuccess;
        if (any) e = launch_user_render<KK, SK, SN, NC>(ctx, kk, f, static_cast<hipStream_t>(stream));
        (void)hipSetDevice(prev);        // the caller's current device is left as it was
        if (e != hipSuccess) throw std::runtime_error(std::string("hip_sched::frame: user kernel launch: ") + hipGetErrorString(e));
        rt.end_frame();
    }
};
} // hip_detail

// the user traversal stack holds VRH_USER_STACK entries: a deeper BVH cannot be traversed (the
// device code then reports a miss); checked_ref rejects it on the host instead
template <typename Ref>
inline Ref checked_ref(Ref r)
{
    if (r.view.max_depth >= VRH_USER_STACK)
        throw hip_error("hip_bvh_ref: BVH deeper than VRH_USER_STACK", VRH_ERR_UNSUPPORTED);
    return r;
}

} // visionaray
