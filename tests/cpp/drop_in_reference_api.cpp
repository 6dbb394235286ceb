// tests/cpp/drop_in_reference_api.cpp -- drop-in check against the REAL reference API.
//
// Compiled (oracle/Makefile `dropin`, build container only) with the reference headers from
// /root/reference/include and include/visionaray_hip/hip_backend.h: the reference's own camera,
// basic_triangle<3,float>, build<index_bvh<P>> (build.inl:165-178), make_sched_params
// (scheduler.h:164-242) and pixel formats drive hip_index_bvh / hip_buffer_rt / hip_sched exactly
// where cuda_index_bvh / gpu_buffer_rt / cuda_sched stood (viewer.cpp:779-791, cuda_sched.h:25-40).
// The binary (oracle/_ref/dropin_ref_api) prints the same JSON as examples/ao_hip.
#include <visionaray/math/math.h>
#include <visionaray/bvh.h>
#include <visionaray/camera.h>
#include <visionaray/pixel_format.h>
#include <visionaray/scheduler.h>

#include <visionaray_hip/hip_backend.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace visionaray;

static uint64_t fnv1a(const void* p, size_t n)
{
    auto b = static_cast<const unsigned char*>(p);
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ull; }
    return h;
}

int main(int argc, char** argv)
{
    unsigned grid = argc > 1 ? unsigned(atoi(argv[1])) : 200;
    unsigned W = argc > 2 ? unsigned(atoi(argv[2])) : 320;
    unsigned H = argc > 3 ? unsigned(atoi(argv[3])) : 180;
    using tri_t = basic_triangle<3, float>;
    std::vector<tri_t> tris(size_t(2) * grid * grid);
    if (vrh_gen_heightfield(grid, tris.data()) != VRH_OK) return 2;

    // the reference's own builder and camera
    auto host_bvh = build<index_bvh<tri_t>>(tris.data(), tris.size());
    std::vector<vec3> normals(tris.size());
    for (size_t i = 0; i < tris.size(); ++i) normals[i] = normalize(cross(tris[i].e1, tris[i].e2));
    camera cam;
    cam.perspective(45.0f * constants::degrees_to_radians<float>(), W / static_cast<float>(H), 0.001f, 1000.0f);
    cam.look_at(vec3(0.0f, 0.9f, 1.4f), vec3(0.0f), vec3(0.0f, 1.0f, 0.0f));

    try
    {
        hip_index_bvh<tri_t> device_bvh(host_bvh, normals.data());       // was: cuda_index_bvh<tri_t>
        hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;                     // was: gpu_buffer_rt<...>
        rt.resize(W, H);
        hip_sched<basic_ray<float>> sched;                                // was: cuda_sched<ray>
        auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);
        sched.frame(make_hip_ao_kernel(device_bvh, vec4(0.1f, 0.2f, 0.3f, 1.0f)), sparams);

        size_t n = size_t(W) * H;
        std::vector<float> color(4 * n), t(n);
        std::vector<uint32_t> pid(n);
        std::vector<uint8_t> occ(n);
        rt.download(color.data(), pid.data(), t.data(), occ.data());
        unsigned long long rays = sched.context().last_frame_stats().rays;

        // frames in flight: three frames (the reference camera, then the eye raised twice) in one
        // launch; each must equal its own frame() call
        std::vector<camera> cams(3, cam);
        cams[1].look_at(vec3(0.0f, 1.0f, 1.4f), vec3(0.0f), vec3(0.0f, 1.0f, 0.0f));
        cams[2].look_at(vec3(0.0f, 1.1f, 1.4f), vec3(0.0f), vec3(0.0f, 1.0f, 0.0f));
        hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt3;
        rt3.resize(W, 3 * H);
        auto kern = make_hip_ao_kernel(device_bvh, vec4(0.1f, 0.2f, 0.3f, 1.0f));
        sched.frames(kern, cams, rt3);
        std::vector<float> color3(12 * n), t3(3 * n);
        std::vector<uint32_t> pid3(3 * n);
        std::vector<uint8_t> occ3(3 * n);
        rt3.download(color3.data(), pid3.data(), t3.data(), occ3.data());
        bool batch_ok = true;
        for (size_t f = 0; f < 3; ++f)
        {
            hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> one;
            one.resize(W, H);
            auto sp = make_sched_params(pixel_sampler::uniform_type{}, cams[f], one);
            sched.frame(kern, sp, unsigned(f));       // frame f of the batch has frame number f
            one.download(color.data(), pid.data(), t.data(), occ.data());
            batch_ok = batch_ok && std::memcmp(color.data(), color3.data() + 4 * f * n, 16 * n) == 0
                && std::memcmp(pid.data(), pid3.data() + f * n, 4 * n) == 0
                && std::memcmp(t.data(), t3.data() + f * n, 4 * n) == 0
                && std::memcmp(occ.data(), occ3.data() + f * n, n) == 0;
        }
        batch_ok = batch_ok && std::memcmp(pid3.data(), pid3.data() + n, 4 * n) != 0;   // distinct cameras
        // the first frame of the batch is the reference camera's frame
        std::memcpy(color.data(), color3.data(), 16 * n);
        std::memcpy(pid.data(), pid3.data(), 4 * n);
        std::memcpy(t.data(), t3.data(), 4 * n);
        std::memcpy(occ.data(), occ3.data(), n);

        // mask intersector (optional argv[4] = mask file, argv[5] = its size n): the AO frame with
        // with_intersector(kernel, hip_hit_mask) over planar (x, z) tex coords of every corner
        unsigned long long mask_hashes[4] = { 0, 0, 0, 0 };
        if (argc > 5)
        {
            unsigned mn = unsigned(atoi(argv[5]));
            std::vector<uint8_t> mask(size_t(mn) * mn);
            FILE* f = fopen(argv[4], "rb");
            if (!f || fread(mask.data(), 1, mask.size(), f) != mask.size()) { if (f) fclose(f); return 3; }
            fclose(f);
            std::vector<vec2> tc(3 * tris.size());
            for (auto const& tri : tris)
            {
                vec3 c[3] = { tri.v1, tri.v1 + tri.e1, tri.v1 + tri.e2 };
                for (int k = 0; k < 3; ++k) tc[3 * tri.prim_id + k] = vec2(c[k].x * 0.5f + 0.5f, c[k].z * 0.5f + 0.5f);
            }
            hip_hit_mask hm(tc, mask.data(), mn, mn);
            hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> mrt;
            mrt.resize(W, H);
            auto msp = make_sched_params(pixel_sampler::uniform_type{}, cam, mrt);
            sched.frame(with_intersector(kern, hm), msp);
            std::vector<float> mc(4 * n), mt(n);
            std::vector<uint32_t> mp(n);
            std::vector<uint8_t> mo(n);
            mrt.download(mc.data(), mp.data(), mt.data(), mo.data());
            mask_hashes[0] = fnv1a(mp.data(), n * 4);
            mask_hashes[1] = fnv1a(mt.data(), n * 4);
            mask_hashes[2] = fnv1a(mo.data(), n);
            mask_hashes[3] = fnv1a(mc.data(), n * 16);
        }
        // the reference AO example's own sampler (ao/main.cpp: pixel_sampler::jittered_blend_type) and
        // 4x SSAA, frame 3, blended onto a target cleared to (0.25, 0.5, 0.75, 1)
        unsigned long long sampler_hashes[2] = { 0, 0 };
        {
            hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> srt;
            srt.resize(W, H);
            std::vector<float> sc(4 * n);
            srt.clear_color_buffer(vec4(0.25f, 0.5f, 0.75f, 1.0f));
            sched.frame(kern, make_sched_params(pixel_sampler::jittered_blend_type{}, cam, srt), 3);
            srt.download(sc.data(), nullptr, nullptr, nullptr);
            sampler_hashes[0] = fnv1a(sc.data(), n * 16);
            srt.clear_color_buffer(vec4(0.25f, 0.5f, 0.75f, 1.0f));
            sched.frame(kern, make_sched_params(pixel_sampler::ssaa_type<4>{}, cam, srt), 3);
            srt.download(sc.data(), nullptr, nullptr, nullptr);
            sampler_hashes[1] = fnv1a(sc.data(), n * 16);
        }
        // the camera as view / projection matrices (make_sched_params(sampler, view, proj, rt),
        // scheduler.h:197-212): the camera's own get_view_matrix() / get_proj_matrix(), frame 0
        unsigned long long matrix_hashes[2] = { 0, 0 };
        {
            hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> vrt;
            vrt.resize(W, H);
            std::vector<float> vc(4 * n), vt(n);
            vrt.clear_color_buffer(vec4(0.25f, 0.5f, 0.75f, 1.0f));
            sched.frame(kern, make_sched_params(pixel_sampler::uniform_type{}, cam.get_view_matrix(), cam.get_proj_matrix(), vrt), 0);
            vrt.download(vc.data(), nullptr, vt.data(), nullptr);
            matrix_hashes[0] = fnv1a(vc.data(), n * 16);
            matrix_hashes[1] = fnv1a(vt.data(), n * 4);
        }
        // AO_Samples = 16 (ao/main.cpp:85, 115 take it from the command line): the frame renders into the
        // same target, whose occlusion byte cannot hold 16 masks and is left as it was
        unsigned long long ao16_hash = 0;
        {
            hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> art;
            art.resize(W, H);
            std::vector<float> ac(4 * n);
            sched.frame(make_hip_ao_kernel(device_bvh, vec4(0.1f, 0.2f, 0.3f, 1.0f), 16), make_sched_params(pixel_sampler::uniform_type{}, cam, art));
            art.download(ac.data(), nullptr, nullptr, nullptr);
            ao16_hash = fnv1a(ac.data(), n * 16);
        }
        printf("{\"ao16_color_hash\":\"%016llx\",", ao16_hash);
        printf("\"sampler_jittered_blend_color_hash\":\"%016llx\",\"sampler_ssaa4_color_hash\":\"%016llx\",",
               sampler_hashes[0], sampler_hashes[1]);
        printf("\"matrix_color_hash\":\"%016llx\",\"matrix_t_hash\":\"%016llx\",", matrix_hashes[0], matrix_hashes[1]);
        printf("\"mask_primid_hash\":\"%016llx\",\"mask_t_hash\":\"%016llx\",\"mask_occ_hash\":\"%016llx\","
               "\"mask_color_hash\":\"%016llx\",", mask_hashes[0], mask_hashes[1], mask_hashes[2], mask_hashes[3]);
        printf("\"grid\":%u,\"W\":%u,\"H\":%u,\"rays\":%llu,\"primid_hash\":\"%016llx\",\"t_hash\":\"%016llx\","
               "\"occ_hash\":\"%016llx\",\"color_hash\":\"%016llx\",\"batch_ok\":%s}\n", grid, W, H, rays,
               (unsigned long long)fnv1a(pid.data(), n * 4), (unsigned long long)fnv1a(t.data(), n * 4),
               (unsigned long long)fnv1a(occ.data(), n), (unsigned long long)fnv1a(color.data(), n * 16),
               batch_ok ? "true" : "false");
    }
    catch (std::exception const& e)
    {
        fprintf(stderr, "dropin: %s\n", e.what());
        return 1;
    }
    return 0;
}
