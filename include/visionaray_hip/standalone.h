// include/visionaray_hip/standalone.h -- minimal stand-in for the Visionaray types hip_backend.h
// consumes, for programs that use the HIP backend WITHOUT the Visionaray headers.  Layouts and
// member names follow the reference, so code written against these types
// also compiles against the real ones.  Do not include together with the Visionaray headers.
//
// The math types (vector<N,T>, basic_ray<T>, basic_triangle<3,T>, basic_sphere<T>) are host and
// device code when the translation unit is compiled by hipcc (VRH_FUNC plays the reference's
// VSNRAY_FUNC role, detail/macros.h), so user kernels (visionaray_hip/hip_kernels.h) use the same
// types on the GPU; with g++ they are plain host types.
#pragma once

#if defined(VSNRAY_BVH_H) || defined(VSNRAY_CAMERA_H)
#error "visionaray_hip/standalone.h duplicates Visionaray's own types: include hip_backend.h only"
#endif

#include "hip_backend.h"

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <vector>

#if defined(__HIP__)
#define VRH_FUNC __host__ __device__
#else
#define VRH_FUNC
#endif

namespace visionaray
{

enum pixel_format { PF_UNSPECIFIED = 0, PF_RGBA32F = 12 };   // the reference's values (pixel_format.h:15-60)

//-------------------------------------------------------------------------------------------------
// vector<N, T> (math/vector.h): vec2 / vec3 / vec4 with the reference's member names.  vec3 is
// 16-B aligned: basic_triangle<3,float> is 64 B with v1 at 16, and face
// normal arrays have a 16-B stride.
//

template <size_t Dim, typename T> struct vector;

template <typename T>
struct vector<2, T>
{
    T x = T(0), y = T(0);
    VRH_FUNC vector() = default;
    VRH_FUNC vector(T a, T b) : x(a), y(b) {}
    VRH_FUNC explicit vector(T s) : x(s), y(s) {}
    VRH_FUNC T& operator[](size_t i) { return i == 0 ? x : y; }
    VRH_FUNC T const& operator[](size_t i) const { return i == 0 ? x : y; }
};

template <typename T>
struct alignas(16) vector<3, T>
{
    T x = T(0), y = T(0), z = T(0);
    VRH_FUNC vector() = default;
    VRH_FUNC vector(T a, T b, T c) : x(a), y(b), z(c) {}
    VRH_FUNC explicit vector(T s) : x(s), y(s), z(s) {}
    VRH_FUNC T& operator[](size_t i) { return i == 0 ? x : i == 1 ? y : z; }
    VRH_FUNC T const& operator[](size_t i) const { return i == 0 ? x : i == 1 ? y : z; }
};

template <typename T>
struct alignas(16) vector<4, T>
{
    T x = T(0), y = T(0), z = T(0), w = T(0);
    VRH_FUNC vector() = default;
    VRH_FUNC vector(T a, T b, T c, T d) : x(a), y(b), z(c), w(d) {}
    VRH_FUNC explicit vector(T s) : x(s), y(s), z(s), w(s) {}
    VRH_FUNC vector(vector<3, T> const& v, T d) : x(v.x), y(v.y), z(v.z), w(d) {}
    VRH_FUNC vector<3, T> xyz() const { return vector<3, T>(x, y, z); }
    VRH_FUNC T& operator[](size_t i) { return i == 0 ? x : i == 1 ? y : i == 2 ? z : w; }
    VRH_FUNC T const& operator[](size_t i) const { return i == 0 ? x : i == 1 ? y : i == 2 ? z : w; }
};

using vec2 = vector<2, float>;
using vec3 = vector<3, float>;
using vec4 = vector<4, float>;

// component-wise arithmetic (math/detail/vector*.inl), evaluated component by component
#define VRH_VEC_OP(OP)                                                                                          \
    template <typename T> VRH_FUNC inline vector<2, T> operator OP(vector<2, T> const& a, vector<2, T> const& b) \
    { return vector<2, T>(a.x OP b.x, a.y OP b.y); }                                                            \
    template <typename T> VRH_FUNC inline vector<2, T> operator OP(vector<2, T> const& a, T const& s)            \
    { return vector<2, T>(a.x OP s, a.y OP s); }                                                                \
    template <typename T> VRH_FUNC inline vector<2, T> operator OP(T const& s, vector<2, T> const& a)            \
    { return vector<2, T>(s OP a.x, s OP a.y); }                                                                \
    template <typename T> VRH_FUNC inline vector<3, T> operator OP(vector<3, T> const& a, vector<3, T> const& b) \
    { return vector<3, T>(a.x OP b.x, a.y OP b.y, a.z OP b.z); }                                                \
    template <typename T> VRH_FUNC inline vector<3, T> operator OP(vector<3, T> const& a, T const& s)            \
    { return vector<3, T>(a.x OP s, a.y OP s, a.z OP s); }                                                      \
    template <typename T> VRH_FUNC inline vector<3, T> operator OP(T const& s, vector<3, T> const& a)            \
    { return vector<3, T>(s OP a.x, s OP a.y, s OP a.z); }                                                      \
    template <typename T> VRH_FUNC inline vector<4, T> operator OP(vector<4, T> const& a, vector<4, T> const& b) \
    { return vector<4, T>(a.x OP b.x, a.y OP b.y, a.z OP b.z, a.w OP b.w); }                                    \
    template <typename T> VRH_FUNC inline vector<4, T> operator OP(vector<4, T> const& a, T const& s)            \
    { return vector<4, T>(a.x OP s, a.y OP s, a.z OP s, a.w OP s); }                                            \
    template <typename T> VRH_FUNC inline vector<4, T> operator OP(T const& s, vector<4, T> const& a)            \
    { return vector<4, T>(s OP a.x, s OP a.y, s OP a.z, s OP a.w); }                                            \
    template <size_t N, typename T, typename U> VRH_FUNC inline vector<N, T>& operator OP##=(vector<N, T>& a, U const& b) \
    { a = a OP b; return a; }
VRH_VEC_OP(+)
VRH_VEC_OP(-)
VRH_VEC_OP(*)
VRH_VEC_OP(/)
#undef VRH_VEC_OP

template <typename T> VRH_FUNC inline vector<2, T> operator-(vector<2, T> const& a) { return vector<2, T>(-a.x, -a.y); }
template <typename T> VRH_FUNC inline vector<3, T> operator-(vector<3, T> const& a) { return vector<3, T>(-a.x, -a.y, -a.z); }
template <typename T> VRH_FUNC inline vector<4, T> operator-(vector<4, T> const& a) { return vector<4, T>(-a.x, -a.y, -a.z, -a.w); }

// vector2/3/4.inl: dot sums left to right, cross, length, normalize = v * rsqrt(dot(v, v)) with
// rsqrt(x) = 1 / sqrt(x) (math.h:477-481)
template <typename T> VRH_FUNC inline T dot(vector<2, T> const& u, vector<2, T> const& v) { return u.x * v.x + u.y * v.y; }
template <typename T> VRH_FUNC inline T dot(vector<3, T> const& u, vector<3, T> const& v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
template <typename T> VRH_FUNC inline T dot(vector<4, T> const& u, vector<4, T> const& v)
{
    return u.x * v.x + u.y * v.y + u.z * v.z + u.w * v.w;
}
template <typename T>
VRH_FUNC inline vector<3, T> cross(vector<3, T> const& u, vector<3, T> const& v)
{
    return vector<3, T>(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
template <size_t N, typename T> VRH_FUNC inline T length(vector<N, T> const& v) { return std::sqrt(dot(v, v)); }
template <size_t N, typename T> VRH_FUNC inline vector<N, T> normalize(vector<N, T> const& v)
{
    return v * (T(1.0) / std::sqrt(dot(v, v)));
}

//-------------------------------------------------------------------------------------------------
// rays and primitives (math/ray.h, math/primitive.h, math/triangle.h, math/sphere.h)
//

template <typename T>
struct basic_ray
{
    using scalar_type = T;
    using vec_type = vector<3, T>;
    vector<3, T> ori, dir;
    VRH_FUNC basic_ray() = default;
    VRH_FUNC basic_ray(vector<3, T> const& o, vector<3, T> const& d) : ori(o), dir(d) {}
};
using ray = basic_ray<float>;

template <typename T>
struct primitive
{
    T geom_id = T(0);
    T prim_id = T(0);
};

// basic_triangle<3, float>: geom_id@0 prim_id@4 v1@16 e1@32 e2@48 (64 B; one vertex + two edges)
template <size_t Dim, typename T, typename P = unsigned>
struct basic_triangle : primitive<P>
{
    static_assert(Dim == 3, "basic_triangle<3, T>");
    vector<3, T> v1, e1, e2;
    VRH_FUNC basic_triangle() = default;
    VRH_FUNC basic_triangle(vector<3, T> const& v, vector<3, T> const& a, vector<3, T> const& b) : v1(v), e1(a), e2(b) {}
};

// basic_sphere<float>: geom_id@0 prim_id@4 center@16 radius@32 (48 B)
template <typename T, typename P = unsigned>
struct basic_sphere : primitive<P>
{
    vector<3, T> center;
    T radius = T(0);
    VRH_FUNC basic_sphere() = default;
    VRH_FUNC basic_sphere(vector<3, T> const& c, T r) : center(c), radius(r) {}
};

struct aabb
{
    vec3 min, max;
    aabb() = default;
    aabb(vec3 const& lo, vec3 const& hi) : min(lo), max(hi) {}
};

// normal binding tags (tags.h:44-47)
struct normal_binding {};
struct normals_per_face_binding : normal_binding {};
struct normals_per_vertex_binding : normal_binding {};

// bvh_node (bvh.h:52-119), 32 B
struct alignas(32) bvh_node
{
    float bbox_min[3];
    unsigned first;
    float bbox_max[3];
    unsigned num_prims;
};
static_assert(sizeof(basic_triangle<3, float>) == 64 && sizeof(basic_sphere<float>) == 48 && sizeof(bvh_node) == 32,
              "layouts");

// index_bvh<P> (index_bvh_t, bvh.h:317-403) built by the tree-identical host builder
template <typename P>
class index_bvh
{
public:
    using primitive_type = P;
    index_bvh() = default;
    index_bvh(P const* prims, size_t n) : primitives_(prims, prims + n) {}
    std::vector<P> const& primitives() const { return primitives_; }
    std::vector<bvh_node> const& nodes() const { return nodes_; }
    std::vector<unsigned> const& indices() const { return indices_; }
    std::vector<bvh_node>& nodes() { return nodes_; }
    std::vector<unsigned>& indices() { return indices_; }
    unsigned max_depth = 0;
private:
    std::vector<P> primitives_;
    std::vector<bvh_node> nodes_;
    std::vector<unsigned> indices_;
};

// build<index_bvh<P>>(prims, n) -- build.inl:165-178
template <typename Tree, typename P>
Tree build(P const* prims, size_t n)
{
    Tree t(prims, n);
    t.max_depth = hip_build_index_bvh(prims, n, t.nodes(), t.indices());
    return t;
}

// model (src/common/model.h:20-49) as visionaray_hip/obj_loader.h fills it; materials are the
// C-ABI plastic records (same fields as plastic<float>), textures are not part of it
struct model
{
    using triangle_type = basic_triangle<3, float>;
    using normal_type = vec3;
    using tex_coord_type = vec2;
    using material_type = vrh_plastic;
    std::vector<triangle_type> primitives;
    std::vector<normal_type> shading_normals;
    std::vector<normal_type> geometric_normals;
    std::vector<tex_coord_type> tex_coords;
    std::vector<material_type> materials;
    aabb bbox;
};

namespace constants
{
template <typename T> T degrees_to_radians() { return T(1.74532925199432957692369076849e-02); }
}

// camera (camera.h:46-95): only what the pinhole schedulers read
class camera
{
public:
    void look_at(vec3 const& eye, vec3 const& center, vec3 const& up = vec3(0.0f, 1.0f, 0.0f))
    {
        eye_ = eye; center_ = center; up_ = up;
    }
    void perspective(float fovy, float aspect, float z_near, float z_far)
    {
        fovy_ = fovy; aspect_ = aspect; z_near_ = z_near; z_far_ = z_far;
    }
    vec3 const& eye() const { return eye_; }
    vec3 const& center() const { return center_; }
    vec3 const& up() const { return up_; }
    float fovy() const { return fovy_; }
    float aspect() const { return aspect_; }
private:
    vec3 eye_, center_, up_{ 0.0f, 1.0f, 0.0f };
    float fovy_ = 0.785398f, aspect_ = 1.0f, z_near_ = 0.001f, z_far_ = 1000.0f;
};

// pixel samplers (sched_common.h:34-50)
namespace pixel_sampler
{
struct base_type {};
template <size_t N> struct ssaa_type : base_type {};
using uniform_type = ssaa_type<1>;
struct jittered_type : base_type {};
struct jittered_blend_type : jittered_type {};
}

// recti (math/rectangle.h): x, y, w, h; the scissor box cuda_sched reads (cuda_sched.inl:71)
struct recti
{
    int x = 0, y = 0, w = 0, h = 0;
    recti() = default;
    recti(int a, int b, int c, int d) : x(a), y(b), w(c), h(d) {}
};

// sched_params / make_sched_params (scheduler.h:52-75, 164-242): camera by value, rt by reference,
// scissor box recti(0, 0, w, h) (scheduler.h:175)
template <typename RT, typename PxSamplerT = pixel_sampler::uniform_type>
struct sched_params
{
    using rt_type = RT;
    using pixel_sampler_type = PxSamplerT;

    camera cam;
    RT& rt;
    recti scissor_box;
};

template <typename PxSamplerT, typename RT,
          typename = typename std::enable_if<std::is_base_of<pixel_sampler::base_type, PxSamplerT>::value>::type>
sched_params<RT, PxSamplerT> make_sched_params(PxSamplerT, camera const& cam, RT& rt)
{
    return sched_params<RT, PxSamplerT>{ cam, rt, recti(0, 0, int(rt.width()), int(rt.height())) };
}

// with an intersector (scheduler.h:33-45, 177-193): kernels are called as kernel(isect, r ...)
template <typename RT, typename PxSamplerT, typename Intersector>
struct sched_params_isect : sched_params<RT, PxSamplerT>
{
    using has_intersector = void;
    Intersector& intersector;
};

template <typename PxSamplerT, typename RT, typename Intersector,
          typename = typename std::enable_if<std::is_base_of<pixel_sampler::base_type, PxSamplerT>::value>::type>
sched_params_isect<RT, PxSamplerT, Intersector> make_sched_params(PxSamplerT, camera const& cam, RT& rt, Intersector& isect)
{
    return sched_params_isect<RT, PxSamplerT, Intersector>{ { cam, rt, recti(0, 0, int(rt.width()), int(rt.height())) },
                                                            isect };
}

template <typename RT>
sched_params<RT> make_sched_params(camera const& cam, RT& rt)
{
    return sched_params<RT>{ cam, rt, recti(0, 0, int(rt.width()), int(rt.height())) };
}

// matrix<4, 4, float> (math/matrix.h:75-125): column-major storage, data() = m[col * 4 + row]
template <size_t M, size_t N, typename T> class matrix;
template <>
class matrix<4, 4, float>
{
public:
    matrix() = default;
    explicit matrix(float const* col_major) { for (int i = 0; i < 16; ++i) m_[i] = col_major[i]; }
    static matrix identity()
    {
        matrix r;
        r.m_[0] = r.m_[5] = r.m_[10] = r.m_[15] = 1.0f;
        return r;
    }
    float* data() { return m_; }
    float const* data() const { return m_; }
    float& operator()(int row, int col) { return m_[col * 4 + row]; }
    float operator()(int row, int col) const { return m_[col * 4 + row]; }
private:
    float m_[16] = {};
};
using mat4 = matrix<4, 4, float>;

// sched_params with camera matrices (scheduler.h:76-96, 197-231): view and projection matrix by
// value instead of a camera
template <typename RT, typename PxSamplerT = pixel_sampler::uniform_type>
struct sched_params_matrices
{
    using has_camera_matrices = void;
    using rt_type = RT;
    using pixel_sampler_type = PxSamplerT;

    mat4 view_matrix;
    mat4 proj_matrix;
    RT& rt;
    recti scissor_box;
};

template <typename PxSamplerT, typename RT,
          typename = typename std::enable_if<std::is_base_of<pixel_sampler::base_type, PxSamplerT>::value>::type>
sched_params_matrices<RT, PxSamplerT> make_sched_params(PxSamplerT, mat4 const& view, mat4 const& proj, RT& rt)
{
    return sched_params_matrices<RT, PxSamplerT>{ view, proj, rt, recti(0, 0, int(rt.width()), int(rt.height())) };
}

template <typename RT>
sched_params_matrices<RT> make_sched_params(mat4 const& view, mat4 const& proj, RT& rt)
{
    return sched_params_matrices<RT>{ view, proj, rt, recti(0, 0, int(rt.width()), int(rt.height())) };
}

} // visionaray
