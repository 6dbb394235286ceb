// examples/ao_hip.cpp -- the reference's ao example (src/examples/ao/main.cpp:183-246) on the HIP
// backend through the C++ drop-in API, headless: build the heightfield scene, build the BVH on the
// host, upload (hip_index_bvh), render one AO frame with hip_sched, print FNV-1a hashes of the
// integer outputs as JSON (compared against tests/golden by tests/test_cpp_api.py).
//
//     ao_hip [grid] [width] [height] [frames] [frame_num]
//
// Every frame is rendered with frame number frame_num (default 0: the parity frame of SURVEY.md
// Appendix A); ao/main.cpp passes ++frame_num instead, which gives every frame its own AO samples.
#include <visionaray_hip/standalone.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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
    unsigned grid = argc > 1 ? unsigned(atoi(argv[1])) : 708;
    unsigned W = argc > 2 ? unsigned(atoi(argv[2])) : 1920;
    unsigned H = argc > 3 ? unsigned(atoi(argv[3])) : 1080;
    int frames = argc > 4 ? atoi(argv[4]) : 1;
    unsigned frame_num = argc > 5 ? unsigned(atoi(argv[5])) : 0u;
    try
    {
        // scene + host BVH: build<index_bvh<P>> (build.inl:165-178)
        std::vector<basic_triangle<3, float>> tris(size_t(2) * grid * grid);
        hip_detail::check(vrh_gen_heightfield(grid, tris.data()), "vrh_gen_heightfield");
        auto host_bvh = build<index_bvh<basic_triangle<3, float>>>(tris.data(), tris.size());
        std::vector<vec4> normals(tris.size());
        hip_detail::check(vrh_face_normals(tris.data(), uint32_t(tris.size()), &normals[0].x), "vrh_face_normals");

        // device objects: cuda_index_bvh -> hip_index_bvh, gpu_buffer_rt -> hip_buffer_rt, cuda_sched -> hip_sched
        hip_index_bvh<basic_triangle<3, float>> device_bvh(host_bvh, normals.data());
        hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
        rt.resize(W, H);

        camera cam;
        float aspect = W / static_cast<float>(H);
        cam.perspective(45.0f * constants::degrees_to_radians<float>(), aspect, 0.001f, 1000.0f);
        cam.look_at(vec3(0.0f, 0.9f, 1.4f), vec3(0.0f, 0.0f, 0.0f), vec3(0.0f, 1.0f, 0.0f));

        hip_sched<ray> sched;
        auto kernel = make_hip_ao_kernel(device_bvh, vec4(0.1f, 0.2f, 0.3f, 1.0f), 8, 0.1f);
        auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);

        double best_ms = 1e30;
        uint64_t rays = 0;
        for (int f = 0; f < frames; ++f)
        {
            auto t0 = std::chrono::steady_clock::now();
            sched.frame(kernel, sparams, frame_num);
            sched.context().sync();                   // frame() only issues the frame (cuda_sched's model)
            auto t1 = std::chrono::steady_clock::now();
            best_ms = std::min(best_ms, std::chrono::duration<double, std::milli>(t1 - t0).count());
            rays = sched.context().last_frame_stats().rays;
        }

        size_t n = size_t(W) * H;
        std::vector<float> color(4 * n), t(n);
        std::vector<uint32_t> pid(n);
        std::vector<uint8_t> occ(n);
        rt.download(color.data(), pid.data(), t.data(), occ.data());
        printf("{\"grid\":%u,\"W\":%u,\"H\":%u,\"max_depth\":%u,\"rays\":%llu,\"frame_ms\":%.4f,"
               "\"primid_hash\":\"%016llx\",\"t_hash\":\"%016llx\",\"occ_hash\":\"%016llx\",\"color_hash\":\"%016llx\"}\n",
               grid, W, H, host_bvh.max_depth, (unsigned long long)rays, best_ms,
               (unsigned long long)fnv1a(pid.data(), n * 4), (unsigned long long)fnv1a(t.data(), n * 4),
               (unsigned long long)fnv1a(occ.data(), n), (unsigned long long)fnv1a(color.data(), n * 16));
    }
    catch (std::exception const& e)
    {
        fprintf(stderr, "ao_hip: %s\n", e.what());
        return 1;
    }
    return 0;
}
