// tests/cpp/drop_in_obj_model.cpp -- visionaray_hip/obj_loader.h filling a model, printed as JSON
// (float bit patterns) for tests/test_obj.py.  Built against the reference's own model class
// (src/common/model.h, plastic<float> materials) with -DREFERENCE_MODEL, else standalone.h's.
// With a second argument (standalone build, GPU): the viewer's path on the loaded model --
// hip_index_bvh::gpu_build, per-vertex normals, hip_shading from the model's materials, one
// simple::kernel frame (256 x 160) -- written as RGBA32F + prim_id to that file
// (tests/test_gpu_obj.py compares it with the Python path).
#ifdef REFERENCE_MODEL
#include <common/model.h>
#include <visionaray/material.h>
#include <visionaray/math/math.h>
#else
#include <visionaray_hip/standalone.h>
#endif
#include <visionaray_hip/obj_loader.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

using namespace visionaray;

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

template <typename V>
static void vec3s(const char* name, V const& v)
{
    std::printf("\"%s\": [", name);
    for (size_t i = 0; i < v.size(); ++i)
        std::printf("%s%u, %u, %u", i ? ", " : "", bits(v[i].x), bits(v[i].y), bits(v[i].z));
    std::printf("], ");
}

#ifdef REFERENCE_MODEL
static void mat(plastic<float> const& m, float out[13])
{
    auto ca = m.get_ca().samples(), cd = m.get_cd().samples(), cs = m.get_cs().samples();
    float v[13] = { ca[0], ca[1], ca[2], m.get_ka(), cd[0], cd[1], cd[2], m.get_kd(), cs[0], cs[1], cs[2],
                    m.get_ks(), m.get_specular_exp() };
    std::memcpy(out, v, sizeof(v));
}
#else
static void mat(vrh_plastic const& m, float out[13]) { std::memcpy(out, &m, 13 * sizeof(float)); }
#endif

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    model mod;
    try
    {
        load_obj(argv[1], mod);
    }
    catch (hip_error const& e)
    {
        std::printf("{\"error\": %d}\n", e.status);
        return 0;
    }
#ifndef REFERENCE_MODEL
    if (argc > 2)
    {
        const unsigned W = 256, H = 160;
        try
        {
            auto device_bvh = hip_index_bvh<basic_triangle<3, float>>::gpu_build(mod.primitives, mod.geometric_normals);
            device_bvh.set_vertex_normals(mod.shading_normals);
            std::vector<vrh_point_light> lights(1);
            lights[0] = vrh_point_light{ { 0.5f, 2.0f, 1.5f }, { 1.0f, 1.0f, 1.0f }, 1.0f, 1.0f, 0.0f, 0.0f };
            hip_shading shading(mod.materials, lights);
            hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
            rt.resize(W, H);
            camera cam;
            cam.perspective(45.0f * constants::degrees_to_radians<float>(), W / static_cast<float>(H), 0.001f, 1000.0f);
            cam.look_at(vec3(0.3f, 1.1f, 1.6f), vec3(0.0f, 0.0f, 0.0f), vec3(0.0f, 1.0f, 0.0f));
            hip_sched<ray> sched;
            sched.frame(make_hip_simple_kernel(normals_per_vertex_binding{}, device_bvh, shading,
                                               vec4(0.1f, 0.2f, 0.3f, 1.0f), vec4(0.4f, 0.4f, 0.4f, 0.5f)),
                        make_sched_params(pixel_sampler::uniform_type{}, cam, rt));
            std::vector<float> color(size_t(4) * W * H);
            std::vector<uint32_t> prim(size_t(W) * H);
            rt.download(color.data(), prim.data());
            FILE* f = std::fopen(argv[2], "wb");
            if (!f || std::fwrite(color.data(), 4, color.size(), f) != color.size() ||
                std::fwrite(prim.data(), 4, prim.size(), f) != prim.size())
                return 3;
            std::fclose(f);
        }
        catch (std::exception const& e)
        {
            std::fprintf(stderr, "drop_in_obj_model: %s\n", e.what());
            return 1;
        }
    }
#endif
    std::printf("{\"ids\": [");
    for (size_t i = 0; i < mod.primitives.size(); ++i)
        std::printf("%s%u, %u", i ? ", " : "", mod.primitives[i].geom_id, mod.primitives[i].prim_id);
    std::printf("], ");
    std::vector<vec3> v1, e1, e2;
    for (auto const& t : mod.primitives) { v1.push_back(t.v1); e1.push_back(t.e1); e2.push_back(t.e2); }
    vec3s("v1", v1); vec3s("e1", e1); vec3s("e2", e2);
    vec3s("shading_normals", mod.shading_normals);
    vec3s("geometric_normals", mod.geometric_normals);
    std::printf("\"tex_coords\": [");
    for (size_t i = 0; i < mod.tex_coords.size(); ++i)
        std::printf("%s%u, %u", i ? ", " : "", bits(mod.tex_coords[i].x), bits(mod.tex_coords[i].y));
    std::printf("], \"materials\": [");
    for (size_t i = 0; i < mod.materials.size(); ++i)
    {
        float m[13];
        mat(mod.materials[i], m);
        for (int k = 0; k < 13; ++k) std::printf("%s%u", (i || k) ? ", " : "", bits(m[k]));
    }
    std::printf("], \"bbox\": [%u, %u, %u, %u, %u, %u]}\n", bits(mod.bbox.min.x), bits(mod.bbox.min.y),
                bits(mod.bbox.min.z), bits(mod.bbox.max.x), bits(mod.bbox.max.y), bits(mod.bbox.max.z));
    return 0;
}
