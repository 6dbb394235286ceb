// tests/cpp/drop_in_simple_kernel.cpp -- the shading kernel through the REAL reference API.
//
// Compiled (oracle/Makefile `ref`, build container only) against /root/reference/include and
// include/visionaray_hip/hip_backend.h.  The reference's own plastic<float> / point_light<float>
// objects (material.h, point_light.h), normal binding tags (tags.h) and build<index_bvh<P>> feed
// hip_shading / make_hip_simple_kernel where make_kernel_params + simple::kernel stood
// (kernels.h:357-389, detail/simple.inl:19-83).  Same scene and spec as the reference harness's
// "shade" mode; writes the colour frame to argv[5] (the test compares it with the fixture).
#include <visionaray/math/math.h>
#include <visionaray/bvh.h>
#include <visionaray/camera.h>
#include <visionaray/material.h>
#include <visionaray/pixel_format.h>
#include <visionaray/point_light.h>
#include <visionaray/scheduler.h>
#include <visionaray/tags.h>

#include <visionaray_hip/hip_backend.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using namespace visionaray;

static uint32_t wang(uint32_t a)
{
    a = (a ^ 61u) ^ (a >> 16); a = a + (a << 3); a = a ^ (a >> 4); a = a * 0x27d4eb2du; return a ^ (a >> 15);
}
static float U(uint32_t k) { return float(wang(k) >> 8) * (1.0f / 16777216.0f); }

int main(int argc, char** argv)
{
    if (argc < 6) { fprintf(stderr, "usage: %s grid W H face|vertex out.bin [whitted bounces eps]\n", argv[0]); return 2; }
    const bool whitted = argc > 8 && std::string(argv[6]) == "whitted";
    const unsigned bounces = whitted ? unsigned(atoi(argv[7])) : 0u;
    const float eps = whitted ? float(atof(argv[8])) : 0.0f;
    unsigned grid = unsigned(atoi(argv[1])), W = unsigned(atoi(argv[2])), H = unsigned(atoi(argv[3]));
    bool per_vertex = std::string(argv[4]) == "vertex";
    using tri_t = basic_triangle<3, float>;
    std::vector<tri_t> tris(size_t(2) * grid * grid);
    if (vrh_gen_heightfield(grid, tris.data()) != VRH_OK) return 2;
    for (size_t i = 0; i < tris.size(); ++i) tris[i].geom_id = unsigned(i % 3);
    auto host_bvh = build<index_bvh<tri_t>>(tris.data(), tris.size());
    std::vector<vec3> normals(tris.size()), vnormals(tris.size() * 3);
    for (size_t i = 0; i < tris.size(); ++i) normals[i] = normalize(cross(tris[i].e1, tris[i].e2));
    for (size_t k = 0; k < tris.size(); ++k)
        for (uint32_t j = 0; j < 3; ++j)
        {
            uint32_t b = (uint32_t(k) * 3u + j) * 3u;
            vnormals[k * 3 + j] = normalize(normals[k] + vec3((U(b) - 0.5f) * 0.4f, (U(b + 1) - 0.5f) * 0.4f,
                                                              (U(b + 2) - 0.5f) * 0.4f));
        }

    // the reference's own material / light objects (the spec of oracle/ref_harness.cpp shade_spec)
    std::vector<plastic<float>> materials(3);
    float m[3][13] = { { 0.2f, 0.2f, 0.2f, 1.0f, 0.8f, 0.3f, 0.2f, 1.0f, 1.0f, 1.0f, 1.0f, 0.4f, 32.0f },
                       { 0.1f, 0.1f, 0.1f, 0.5f, 0.2f, 0.7f, 0.3f, 0.9f, 0.9f, 0.9f, 0.9f, 0.2f, 8.0f },
                       { 0.05f, 0.05f, 0.1f, 1.0f, 0.3f, 0.3f, 0.9f, 0.7f, 1.0f, 0.8f, 0.6f, 0.6f, 64.5f } };
    for (int i = 0; i < 3; ++i)
    {
        materials[i].set_ca(from_rgb(vec3(m[i][0], m[i][1], m[i][2]))); materials[i].set_ka(m[i][3]);
        materials[i].set_cd(from_rgb(vec3(m[i][4], m[i][5], m[i][6]))); materials[i].set_kd(m[i][7]);
        materials[i].set_cs(from_rgb(vec3(m[i][8], m[i][9], m[i][10]))); materials[i].set_ks(m[i][11]);
        materials[i].set_specular_exp(m[i][12]);
    }
    std::vector<point_light<float>> lights(2);
    lights[0].set_position(vec3(0.5f, 2.0f, 1.5f)); lights[0].set_cl(vec3(1.0f)); lights[0].set_kl(1.0f);
    lights[1].set_position(vec3(-1.5f, 1.0f, 0.5f)); lights[1].set_cl(vec3(1.0f, 0.8f, 0.6f)); lights[1].set_kl(0.7f);
    lights[1].set_constant_attenuation(1.0f); lights[1].set_linear_attenuation(0.1f);
    lights[1].set_quadratic_attenuation(0.05f);
    if (whitted)
    {
        // whitted_spec: a third light inside the scene
        point_light<float> l2;
        l2.set_position(vec3(0.2f, 0.6f, 0.3f)); l2.set_cl(vec3(0.9f, 0.9f, 1.0f)); l2.set_kl(0.8f);
        l2.set_constant_attenuation(1.0f); l2.set_linear_attenuation(0.2f); l2.set_quadratic_attenuation(0.1f);
        lights.push_back(l2);
    }

    camera cam;
    cam.perspective(45.0f * constants::degrees_to_radians<float>(), W / static_cast<float>(H), 0.001f, 1000.0f);
    cam.look_at(vec3(0.0f, 0.9f, 1.4f), vec3(0.0f), vec3(0.0f, 1.0f, 0.0f));
    try
    {
        hip_index_bvh<tri_t> device_bvh(host_bvh, normals.data());
        if (per_vertex) device_bvh.set_vertex_normals(vnormals);
        hip_shading shading(materials, lights);                          // was: device material / light vectors
        hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
        rt.resize(W, H);
        hip_sched<basic_ray<float>> sched;
        auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);
        vec4 bg(0.1f, 0.2f, 0.3f, 1.0f), ambient(0.4f, 0.4f, 0.4f, 0.5f);
        if (whitted && per_vertex)           // was: whitted::kernel<decltype(kparams)>{kparams}
            sched.frame(make_hip_whitted_kernel(normals_per_vertex_binding{}, device_bvh, shading, bounces, eps, bg,
                                                ambient), sparams);
        else if (whitted)
            sched.frame(make_hip_whitted_kernel(normals_per_face_binding{}, device_bvh, shading, bounces, eps, bg,
                                                ambient), sparams);
        else if (per_vertex)
            sched.frame(make_hip_simple_kernel(normals_per_vertex_binding{}, device_bvh, shading, bg, ambient), sparams);
        else
            sched.frame(make_hip_simple_kernel(normals_per_face_binding{}, device_bvh, shading, bg, ambient), sparams);
        std::vector<float> color(size_t(4) * W * H);
        rt.download(color.data());
        FILE* f = fopen(argv[5], "wb");
        if (!f || fwrite(color.data(), 4, color.size(), f) != color.size()) return 3;
        fclose(f);
        printf("{\"grid\":%u,\"W\":%u,\"H\":%u,\"binding\":\"%s\"}\n", grid, W, H, per_vertex ? "vertex" : "face");
    }
    catch (std::exception const& e)
    {
        fprintf(stderr, "dropin_simple: %s\n", e.what());
        return 1;
    }
    return 0;
}
