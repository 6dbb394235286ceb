// examples/ao_multi_gpu.cpp -- the reference's ao example (src/examples/ao/main.cpp:183-246) sharded
// across every visible GPU from one process, headless, through the C++ drop-in API:
// a hip_render_group over all devices (vrh_group_create_local: ncclCommInitAll), one BVH replica
// per device (the cuda_index_bvh copy-ctor per device), and hip_sched's group overload, which
// renders each GPU's image-tile shards and gathers them to device 0 over RCCL.  The gathered frame
// is compared with the same frame rendered by device 0 alone, and FNV-1a hashes of the outputs are
// printed as JSON (compared against tests/golden by tests/test_cpp_api.py).
//
//     ao_multi_gpu [grid] [width] [height] [frames] [shards]
//
// frames > 1 renders frame numbers 0, 1, ... (a new AO sample set per frame, as ao/main.cpp's
// ++frame_num); the hashes are those of frame 0.  shards = 0: one per GPU.
#include <visionaray_hip/standalone.h>

#include <chrono>
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
    unsigned grid = argc > 1 ? unsigned(atoi(argv[1])) : 708;
    unsigned W = argc > 2 ? unsigned(atoi(argv[2])) : 1920;
    unsigned H = argc > 3 ? unsigned(atoi(argv[3])) : 1080;
    int frames = argc > 4 ? atoi(argv[4]) : 1;
    unsigned shards = argc > 5 ? unsigned(atoi(argv[5])) : 0u;
    try
    {
        std::vector<basic_triangle<3, float>> tris(size_t(2) * grid * grid);
        hip_detail::check(vrh_gen_heightfield(grid, tris.data()), "vrh_gen_heightfield");
        auto host_bvh = build<index_bvh<basic_triangle<3, float>>>(tris.data(), tris.size());
        std::vector<vec4> normals(tris.size());
        hip_detail::check(vrh_face_normals(tris.data(), uint32_t(tris.size()), &normals[0].x), "vrh_face_normals");

        hip_render_group group;                     // every visible GPU
        // the BVH goes to GPU 0 once and is broadcast from there to every member over RCCL
        hip_index_bvh<basic_triangle<3, float>> root_bvh(host_bvh, normals.data(), group.context(0));
        auto replicas = hip_index_bvh<basic_triangle<3, float>>::broadcast(group, &root_bvh);
        std::vector<hip_builtin_kernel> kernels;
        for (auto const& r : replicas)
            kernels.push_back(make_hip_ao_kernel(r, vec4(0.1f, 0.2f, 0.3f, 1.0f), 8, 0.1f));

        hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt(group.context(0));
        rt.resize(W, H);
        camera cam;
        cam.perspective(45.0f * constants::degrees_to_radians<float>(), W / static_cast<float>(H), 0.001f, 1000.0f);
        cam.look_at(vec3(0.0f, 0.9f, 1.4f), vec3(0.0f, 0.0f, 0.0f), vec3(0.0f, 1.0f, 0.0f));
        auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);

        hip_sched<ray> sched(group, shards);
        size_t n = size_t(W) * H;
        std::vector<float> color(4 * n), t(n);
        std::vector<uint32_t> pid(n);
        std::vector<uint8_t> occ(n);
        double best_ms = 1e30;
        for (int f = frames - 1; f >= 0; --f)       // frame 0 last: its buffers are the ones hashed
        {
            auto t0 = std::chrono::steady_clock::now();
            sched.frame(kernels, sparams, unsigned(f));
            auto t1 = std::chrono::steady_clock::now();
            best_ms = std::min(best_ms, std::chrono::duration<double, std::milli>(t1 - t0).count());
        }
        rt.download(color.data(), pid.data(), t.data(), occ.data());

        // the same frame on device 0 alone
        hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> one(group.context(0));
        one.resize(W, H);
        hip_sched<ray> single(group.context(0));
        single.frame(kernels[0], make_sched_params(pixel_sampler::uniform_type{}, cam, one), 0u);
        std::vector<float> color1(4 * n), t1(n);
        std::vector<uint32_t> pid1(n);
        std::vector<uint8_t> occ1(n);
        one.download(color1.data(), pid1.data(), t1.data(), occ1.data());
        const bool same = std::memcmp(color.data(), color1.data(), 16 * n) == 0 && pid == pid1 && occ == occ1
                          && std::memcmp(t.data(), t1.data(), 4 * n) == 0;

        printf("{\"gpus\":%zu,\"shards\":%u,\"grid\":%u,\"W\":%u,\"H\":%u,\"frame_ms\":%.4f,\"matches_one_gpu\":%s,"
               "\"primid_hash\":\"%016llx\",\"t_hash\":\"%016llx\",\"occ_hash\":\"%016llx\",\"color_hash\":\"%016llx\"}\n",
               group.size(), shards ? shards : unsigned(group.size()), grid, W, H, best_ms, same ? "true" : "false",
               (unsigned long long)fnv1a(pid.data(), n * 4), (unsigned long long)fnv1a(t.data(), n * 4),
               (unsigned long long)fnv1a(occ.data(), n), (unsigned long long)fnv1a(color.data(), n * 16));
        return same ? 0 : 3;
    }
    catch (std::exception const& e)
    {
        fprintf(stderr, "ao_multi_gpu: %s\n", e.what());
        return 1;
    }
}
