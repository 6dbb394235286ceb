// visionaray_amd/csrc/vrh_scenes.cpp -- synthetic benchmark scenes.
//
// The reference ships no scene generator (it loads OBJ files through Boost.Spirit, which is out of
// scope); these deterministic, libm-free generators define the BASELINE.json configs.  Float
// arithmetic in the order written, compiled with -ffp-contract=off.

#include "vrh_internal.h"

#include <cmath>
#include <cstring>

namespace vrh {
namespace {

inline uint32_t wang(uint32_t a)
{
    a = (a ^ 61u) ^ (a >> 16);
    a = a + (a << 3);
    a = a ^ (a >> 4);
    a = a * 0x27d4eb2du;
    return a ^ (a >> 15);
}

inline float uniform01(uint32_t k) { return static_cast<float>(wang(k) >> 8) * (1.0f / 16777216.0f); }

struct p3 { float x, y, z; };

inline p3 height_vertex(uint32_t grid, uint32_t i, uint32_t j)
{
    float x = -1.0f + 2.0f * static_cast<float>(i) / static_cast<float>(grid);
    float z = -1.0f + 2.0f * static_cast<float>(j) / static_cast<float>(grid);
    uint32_t k = j * (grid + 1) + i;
    float y = 0.3f * x * z * (1.0f - x * x) * (1.0f - z * z) + 0.004f * (uniform01(k) - 0.5f);
    return { x, y, z };
}

inline void emit_tri(tri64& t, p3 a, p3 b, p3 c, uint32_t id)
{
    std::memset(&t, 0, sizeof(t));
    t.prim_id = id;
    t.v1[0] = a.x; t.v1[1] = a.y; t.v1[2] = a.z;
    t.e1[0] = b.x - a.x; t.e1[1] = b.y - a.y; t.e1[2] = b.z - a.z;
    t.e2[0] = c.x - a.x; t.e2[1] = c.y - a.y; t.e2[2] = c.z - a.z;
}

} // namespace
} // namespace vrh

using namespace vrh;

extern "C" VRH_API int vrh_gen_heightfield(uint32_t grid, void* out)
{
    if (!out || grid == 0) { set_error("vrh_gen_heightfield: bad argument"); return VRH_ERR_INVALID; }
    auto tris = static_cast<tri64*>(out);
    for (int64_t jj = 0; jj < static_cast<int64_t>(grid); ++jj)
    {
        uint32_t j = static_cast<uint32_t>(jj);
        for (uint32_t i = 0; i < grid; ++i)
        {
            p3 a = height_vertex(grid, i, j), b = height_vertex(grid, i + 1, j);
            p3 c = height_vertex(grid, i + 1, j + 1), e = height_vertex(grid, i, j + 1);
            size_t base = size_t(2) * (size_t(j) * grid + i);
            emit_tri(tris[base], a, b, c, static_cast<uint32_t>(base));
            emit_tri(tris[base + 1], a, c, e, static_cast<uint32_t>(base + 1));
        }
    }
    return VRH_OK;
}

extern "C" VRH_API int vrh_gen_cornell(void* out)
{
    if (!out) { set_error("vrh_gen_cornell: null output"); return VRH_ERR_INVALID; }
    static const float quads[6][4][3] = {
        {{-1,-1,-1},{ 1,-1,-1},{ 1,-1, 1},{-1,-1, 1}},   // floor
        {{-1, 1,-1},{-1, 1, 1},{ 1, 1, 1},{ 1, 1,-1}},   // ceiling
        {{-1,-1,-1},{-1, 1,-1},{ 1, 1,-1},{ 1,-1,-1}},   // back
        {{-1,-1,-1},{-1,-1, 1},{-1, 1, 1},{-1, 1,-1}},   // left
        {{ 1,-1,-1},{ 1, 1,-1},{ 1, 1, 1},{ 1,-1, 1}},   // right
        {{-.25f,.99f,-.25f},{-.25f,.99f,.25f},{.25f,.99f,.25f},{.25f,.99f,-.25f}},  // light
    };
    auto tris = static_cast<tri64*>(out);
    uint32_t n = 0;
    for (auto const& q : quads)
    {
        p3 v[4];
        for (int k = 0; k < 4; ++k) v[k] = { q[k][0], q[k][1], q[k][2] };
        emit_tri(tris[n], v[0], v[1], v[2], n); ++n;
        emit_tri(tris[n], v[0], v[2], v[3], n); ++n;
    }
    return VRH_OK;
}

extern "C" VRH_API int vrh_gen_spheres(uint32_t n, void* out)
{
    if (!out) { set_error("vrh_gen_spheres: null output"); return VRH_ERR_INVALID; }
    auto s = static_cast<sphere48*>(out);
    for (int64_t ii = 0; ii < static_cast<int64_t>(n); ++ii)
    {
        uint32_t i = static_cast<uint32_t>(ii), k = 6u * i;
        sphere48& sp = s[i];
        std::memset(&sp, 0, sizeof(sp));
        sp.center[0] = 2.0f * uniform01(k) - 1.0f;
        sp.center[1] = 2.0f * uniform01(k + 1) - 1.0f;
        sp.center[2] = 2.0f * uniform01(k + 2) - 1.0f;
        sp.radius = 0.002f + 0.008f * uniform01(k + 3);
        sp.prim_id = i;
    }
    return VRH_OK;
}

// get_normal.h:26-37 normals_per_face_binding input: normalize(cross(e1, e2)) per triangle
extern "C" VRH_API int vrh_face_normals(const void* in, uint32_t n, float* out)
{
    if (!in || !out) { set_error("vrh_face_normals: null argument"); return VRH_ERR_INVALID; }
    auto tris = static_cast<const tri64*>(in);
    for (int64_t ii = 0; ii < static_cast<int64_t>(n); ++ii)
    {
        const tri64& t = tris[ii];
        float cx = t.e1[1] * t.e2[2] - t.e1[2] * t.e2[1];
        float cy = t.e1[2] * t.e2[0] - t.e1[0] * t.e2[2];
        float cz = t.e1[0] * t.e2[1] - t.e1[1] * t.e2[0];
        float inv = 1.0f / std::sqrt(cx * cx + cy * cy + cz * cz);
        float* o = out + 4 * ii;
        o[0] = cx * inv; o[1] = cy * inv; o[2] = cz * inv; o[3] = 0.0f;
    }
    return VRH_OK;
}

// camera.inl:10-57 + simple_sched.inl:61-89 (host-side basis; tanf from the host libm)
extern "C" VRH_API int vrh_make_camera(const float eye[3], const float center[3], const float up[3], float fovy,
                                       float aspect, uint32_t width, uint32_t height, vrh_camera* out)
{
    if (!eye || !center || !up || !out) { set_error("vrh_make_camera: null argument"); return VRH_ERR_INVALID; }
    auto sub = [](const float* a, const float* b, float* r) { for (int i = 0; i < 3; ++i) r[i] = a[i] - b[i]; };
    auto cross = [](const float* u, const float* v, float* r) {
        r[0] = u[1] * v[2] - u[2] * v[1];
        r[1] = u[2] * v[0] - u[0] * v[2];
        r[2] = u[0] * v[1] - u[1] * v[0];
    };
    auto normalize = [](float* v) {
        float inv = 1.0f / std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        for (int i = 0; i < 3; ++i) v[i] = v[i] * inv;
    };
    float f[3], s[3], u[3];
    sub(eye, center, f);
    normalize(f);
    cross(up, f, s);
    normalize(s);
    cross(f, s, u);
    float th = std::tan(fovy / 2.0f);
    float su = th * aspect;
    for (int i = 0; i < 3; ++i)
    {
        out->eye[i] = eye[i];
        out->cam_u[i] = s[i] * su;
        out->cam_v[i] = u[i] * th;
        out->cam_w[i] = -f[i];
    }
    out->width = width;
    out->height = height;
    for (int i = 0; i < 4; ++i) out->scissor[i] = 0u;   // whole image
    return VRH_OK;
}
