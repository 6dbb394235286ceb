// include/visionaray_hip/standalone.h -- minimal stand-in for the Visionaray types hip_backend.h
// consumes, for programs that use the HIP backend WITHOUT the Visionaray headers.  Layouts and
// member names follow the reference, so code written against these types
// also compiles against the real ones.  Do not include together with the Visionaray headers.
#pragma once

#if defined(VSNRAY_BVH_H) || defined(VSNRAY_CAMERA_H)
#error "visionaray_hip/standalone.h duplicates Visionaray's own types: include hip_backend.h only"
#endif

#include "hip_backend.h"

#include <cmath>
#include <cstdint>
#include <vector>

namespace visionaray
{

enum pixel_format { PF_UNSPECIFIED = 0, PF_RGBA32F = 1 };

struct alignas(16) vec3
{
    float x = 0, y = 0, z = 0;
    vec3() = default;
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
};
struct alignas(16) vec4
{
    float x = 0, y = 0, z = 0, w = 0;
    vec4() = default;
    vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
};

struct vec2
{
    float x = 0, y = 0;
    vec2() = default;
    vec2(float a, float b) : x(a), y(b) {}
};
struct aabb
{
    vec3 min, max;
    aabb() = default;
    aabb(vec3 const& lo, vec3 const& hi) : min(lo), max(hi) {}
};

struct basic_ray_float {};                 // tag standing in for basic_ray<float> (hip_sched<R>)

// normal binding tags (tags.h:44-47)
struct normal_binding {};
struct normals_per_face_binding : normal_binding {};
struct normals_per_vertex_binding : normal_binding {};
using ray = basic_ray_float;

// basic_triangle<3,float>: geom_id@0 prim_id@4 v1@16 e1@32 e2@48 (64 B)
struct alignas(16) basic_triangle
{
    unsigned geom_id = 0, prim_id = 0;
    vec3 v1, e1, e2;
};
// basic_sphere<float>: geom_id@0 prim_id@4 center@16 radius@32 (48 B)
struct alignas(16) basic_sphere
{
    unsigned geom_id = 0, prim_id = 0;
    vec3 center;
    float radius = 0;
};
// bvh_node (bvh.h:52-119), 32 B
struct alignas(32) bvh_node
{
    float bbox_min[3];
    unsigned first;
    float bbox_max[3];
    unsigned num_prims;
};
static_assert(sizeof(basic_triangle) == 64 && sizeof(basic_sphere) == 48 && sizeof(bvh_node) == 32, "layouts");

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
    using triangle_type = basic_triangle;
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

namespace pixel_sampler
{
struct uniform_type {};
}

// sched_params / make_sched_params (scheduler.h:52-75, 164-242): camera by value, rt by reference
template <typename RT>
struct sched_params
{
    camera cam;
    RT& rt;
};

template <typename RT>
sched_params<RT> make_sched_params(pixel_sampler::uniform_type, camera const& cam, RT& rt)
{
    return sched_params<RT>{ cam, rt };
}

template <typename RT>
sched_params<RT> make_sched_params(camera const& cam, RT& rt)
{
    return sched_params<RT>{ cam, rt };
}

} // visionaray
