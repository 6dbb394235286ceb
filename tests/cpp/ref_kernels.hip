// tests/cpp/ref_kernels.hip -- a Visionaray program written for cuda_sched, ported to hip_sched by
// its include lines and the three backend type names only.  Built by oracle/Makefile (`ref_kernels`,
// it needs the reference's headers) into oracle/_ref/ref_kernels.
//
// Everything a kernel touches is the REFERENCE'S OWN code, made device code by
// visionaray_hip/reference.h: basic_ray / vector / basic_triangle, closest_hit / any_hit /
// multi_hit (traverse_linear.inl), the intersectors, get_normal, make_orthonormal_basis,
// random_sampler<float> and cosine_sample_hemisphere, simple::kernel (detail/simple.inl) with
// plastic<float> and point_light<float>.  What the program brings is the device BVH
// (hip_index_bvh<P>::ref(), traversed by libvrh's walk with the reference's leaf step), the render
// target and the scheduler.
//
//   ref_kernels draws  <grid> <W> <H> <outdir> <frame>          kernel(R, random_sampler<S>&): the
//                                                               sampler's draws 0, 1, 2, 15 as colour
//   ref_kernels ao     <grid> <W> <H> <outdir> <frame> [spp]    the AO kernel of ao/main.cpp:183-246
//                                                               verbatim (+ depth = hit t)
//   ref_kernels simple <grid> <W> <H> <outdir>                  kernel<decltype(make_kernel_params(...))>
//                                                               = simple::kernel (kernels.h:357-389,
//                                                               detail/simple.inl:19-83) over device
//                                                               bvh refs, materials and lights
//   ref_kernels multi  <grid> <W> <H> <outdir>                  multi_hit<16> over the refs: hit count
//                                                               and the first / last hit per pixel
//   ref_kernels bench  <grid> <W> <H> <launches> [F]            AO kernel throughput (median frame,
//                                                               F frames per launch)
//
// Outputs: color.bin (RGBA32F as rendered), t.bin (the depth the kernel returned, where it set one).
#include <visionaray_hip/reference.h>      // was: #include <visionaray/bvh.h> ... <visionaray/traverse.h>
#include <visionaray_hip/hip_kernels.h>    // was: <visionaray/cuda/...>, <visionaray/detail/cuda_sched.h>, <thrust/...>

#include <cstdio>

using namespace visionaray;

using tri_t = basic_triangle<3, float>;
using R = basic_ray<float>;
using S = R::scalar_type;
using C = vector<4, S>;
using V = vector<3, S>;

static void write_file(std::string const& path, const void* p, size_t n)
{
    FILE* f = fopen(path.c_str(), "wb");
    if (!f || fwrite(p, 1, n, f) != n) { fprintf(stderr, "cannot write %s\n", path.c_str()); exit(3); }
    fclose(f);
}

// thrust::device_vector<T>(host) stand-in: the reference keeps kernel inputs in device vectors and
// hands raw pointers to the kernel (multi_hit/main.cpp:289-306)
template <typename T>
static T* device_copy(T const* p, size_t n)
{
    T* d = nullptr;
    if (hipMalloc(&d, n * sizeof(T)) != hipSuccess || hipMemcpy(d, p, n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
    {
        fprintf(stderr, "device copy failed\n");
        exit(4);
    }
    return d;
}

// the heightfield of SURVEY.md Appendix A (as the reference harness generates it)
static uint32_t wang(uint32_t a)
{
    a = (a ^ 61u) ^ (a >> 16);
    a = a + (a << 3);
    a = a ^ (a >> 4);
    a = a * 0x27d4eb2du;
    a = a ^ (a >> 15);
    return a;
}
static float U(uint32_t k) { return float(wang(k) >> 8) * (1.0f / 16777216.0f); }
static vec3 hf_vertex(int grid, int i, int j)
{
    float x = -1.0f + 2.0f * float(i) / float(grid);
    float z = -1.0f + 2.0f * float(j) / float(grid);
    uint32_t k = uint32_t(j) * uint32_t(grid + 1) + uint32_t(i);
    float y = 0.3f * x * z * (1.0f - x * x) * (1.0f - z * z) + 0.004f * (U(k) - 0.5f);
    return vec3(x, y, z);
}
static void heightfield(int grid, aligned_vector<tri_t>& tris)
{
    tris.resize(size_t(2) * grid * grid);
    for (int j = 0; j < grid; ++j)
        for (int i = 0; i < grid; ++i)
        {
            vec3 a = hf_vertex(grid, i, j), b = hf_vertex(grid, i + 1, j), c = hf_vertex(grid, i + 1, j + 1),
                 e = hf_vertex(grid, i, j + 1);
            size_t base = size_t(2) * (size_t(j) * grid + i);
            tri_t& t0 = tris[base];
            t0.v1 = a; t0.e1 = b - a; t0.e2 = c - a; t0.prim_id = unsigned(base); t0.geom_id = 0;
            tri_t& t1 = tris[base + 1];
            t1.v1 = a; t1.e1 = c - a; t1.e2 = e - a; t1.prim_id = unsigned(base + 1); t1.geom_id = 0;
        }
}

// hf<G> | hfstack<G>x<K> (K copies, layer k 0.03 k lower) | cornell12, with the eye of each
static aligned_vector<tri_t> make_scene(std::string const& name, vec3& eye)
{
    aligned_vector<tri_t> tris;
    eye = vec3(0.0f, 0.9f, 1.4f);
    if (name == "cornell12")
    {
        const float q[6][4][3] = {
            {{-1,-1,-1},{ 1,-1,-1},{ 1,-1, 1},{-1,-1, 1}}, {{-1, 1,-1},{-1, 1, 1},{ 1, 1, 1},{ 1, 1,-1}},
            {{-1,-1,-1},{-1, 1,-1},{ 1, 1,-1},{ 1,-1,-1}}, {{-1,-1,-1},{-1,-1, 1},{-1, 1, 1},{-1, 1,-1}},
            {{ 1,-1,-1},{ 1, 1,-1},{ 1, 1, 1},{ 1,-1, 1}},
            {{-.25f,.99f,-.25f},{-.25f,.99f,.25f},{.25f,.99f,.25f},{.25f,.99f,-.25f}} };
        for (int f = 0; f < 6; ++f)
        {
            vec3 a(q[f][0]), b(q[f][1]), c(q[f][2]), d(q[f][3]);
            tri_t t;
            t.geom_id = 0;
            t.v1 = a; t.e1 = b - a; t.e2 = c - a; t.prim_id = unsigned(tris.size()); tris.push_back(t);
            t.v1 = a; t.e1 = c - a; t.e2 = d - a; t.prim_id = unsigned(tris.size()); tris.push_back(t);
        }
        eye = vec3(0.0f, 0.0f, 3.4f);
    }
    else if (name.compare(0, 7, "hfstack") == 0)
    {
        const int grid = atoi(name.c_str() + 7), layers = atoi(strchr(name.c_str(), 'x') + 1);
        aligned_vector<tri_t> one;
        heightfield(grid, one);
        tris.resize(one.size() * layers);
        for (int k = 0; k < layers; ++k)
            for (size_t i = 0; i < one.size(); ++i)
            {
                tri_t t = one[i];
                t.v1.y = t.v1.y - 0.03f * float(k);
                t.prim_id = unsigned(size_t(k) * one.size() + i);
                tris[size_t(k) * one.size() + i] = t;
            }
    }
    else if (name == "hf1M" || name == "hf10M")
        heightfield(name == "hf1M" ? 708 : 2236, tris);          // SURVEY.md Appendix A grid sizes
    else if (name.compare(0, 2, "hf") == 0)
        heightfield(atoi(name.c_str() + 2), tris);
    else
    {
        fprintf(stderr, "unknown scene %s\n", name.c_str());
        exit(2);
    }
    return tris;
}

// the shading spec of the reference harness's shade / whitted / multi modes (oracle/ref_harness.cpp
// make_shade_spec / make_whitted_spec): three plastic materials by geom_id = prim index % 3, point lights
static void shade_spec(bool whitted, aligned_vector<plastic<float>>& materials, aligned_vector<point_light<float>>& lights,
                       vec4& ambient, vec4& bg)
{
    struct { float ca[3], ka, cd[3], kd, cs[3], ks, exp; } m[3] = {
        { { 0.2f, 0.2f, 0.2f }, 1.0f, { 0.8f, 0.3f, 0.2f }, 1.0f, { 1.0f, 1.0f, 1.0f }, 0.4f, 32.0f },
        { { 0.1f, 0.1f, 0.1f }, 0.5f, { 0.2f, 0.7f, 0.3f }, 0.9f, { 0.9f, 0.9f, 0.9f }, 0.2f, 8.0f },
        { { 0.05f, 0.05f, 0.1f }, 1.0f, { 0.3f, 0.3f, 0.9f }, 0.7f, { 1.0f, 0.8f, 0.6f }, 0.6f, 64.5f } };
    for (auto const& d : m)
    {
        plastic<float> p;
        p.set_ca(from_rgb(vec3(d.ca[0], d.ca[1], d.ca[2])));
        p.set_ka(d.ka);
        p.set_cd(from_rgb(vec3(d.cd[0], d.cd[1], d.cd[2])));
        p.set_kd(d.kd);
        p.set_cs(from_rgb(vec3(d.cs[0], d.cs[1], d.cs[2])));
        p.set_ks(d.ks);
        p.set_specular_exp(d.exp);
        materials.push_back(p);
    }
    point_light<float> l0;
    l0.set_position(vec3(0.5f, 2.0f, 1.5f));
    l0.set_cl(vec3(1.0f, 1.0f, 1.0f));
    l0.set_kl(1.0f);
    lights.push_back(l0);
    point_light<float> l1;
    l1.set_position(vec3(-1.5f, 1.0f, 0.5f));
    l1.set_cl(vec3(1.0f, 0.8f, 0.6f));
    l1.set_kl(0.7f);
    l1.set_constant_attenuation(1.0f);
    l1.set_linear_attenuation(0.1f);
    l1.set_quadratic_attenuation(0.05f);
    lights.push_back(l1);
    if (whitted)
    {
        point_light<float> l2;
        l2.set_position(vec3(0.2f, 0.6f, 0.3f));
        l2.set_cl(vec3(0.9f, 0.9f, 1.0f));
        l2.set_kl(0.8f);
        l2.set_constant_attenuation(1.0f);
        l2.set_linear_attenuation(0.2f);
        l2.set_quadratic_attenuation(0.1f);
        lights.push_back(l2);
    }
    ambient = vec4(0.4f, 0.4f, 0.4f, 0.5f);
    bg = vec4(0.1f, 0.2f, 0.3f, 1.0f);
}

int main(int argc, char** argv)
{
    if (argc < 5) { fprintf(stderr, "usage: ref_kernels draws|ao|simple|multi|bench grid W H ...\n"); return 2; }
    const std::string mode = argv[1];
    const std::string scene = argv[2];
    const int W = atoi(argv[3]), H = atoi(argv[4]);
    const std::string outdir = argc > 5 ? argv[5] : ".";

    vec3 eye;
    auto tris = make_scene(scene, eye);
    const bool shading = mode == "shade" || mode == "whitted" || mode == "multi";
    if (shading)
        for (size_t i = 0; i < tris.size(); ++i) tris[i].geom_id = unsigned(i % 3);
    auto host_bvh = build<index_bvh<tri_t>>(tris.data(), tris.size());           // the reference's builder
    aligned_vector<vec3> normals(tris.size());
    for (size_t i = 0; i < tris.size(); ++i) normals[i] = normalize(cross(tris[i].e1, tris[i].e2));

    camera cam;
    cam.perspective(45.0f * constants::degrees_to_radians<float>(), W / static_cast<float>(H), 0.001f, 1000.0f);
    cam.look_at(eye, vec3(0.0f, 0.0f, 0.0f), vec3(0.0f, 1.0f, 0.0f));

    try
    {
        hip_index_bvh<tri_t> device_bvh(host_bvh, normals.data());              // was: cuda_index_bvh<tri_t>
        hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;                             // was: gpu_buffer_rt<...>
        rt.resize(W, H);
        hip_sched<R> sched;                                                        // was: cuda_sched<R>
        auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);

        // thrust::device_vector<bvh_ref> device_primitives; device_primitives.push_back(device_bvh.ref());
        using bvh_ref = decltype(device_bvh.ref());
        bvh_ref ref = checked_ref(device_bvh.ref());
        bvh_ref const* prims_begin = device_copy(&ref, 1);
        bvh_ref const* prims_end = prims_begin + 1;
        vec3 const* device_normals = device_copy(normals.data(), normals.size());
        const vec3 bgcolor(0.1f, 0.2f, 0.3f);

        if (mode == "draws")
        {
            const unsigned frame_num = argc > 6 ? unsigned(strtoul(argv[6], nullptr, 10)) : 0u;
            sched.frame([=] __device__ (R ray, random_sampler<S>& samp) -> result_record<S>
            {
                result_record<S> result;
                S d[16];
                for (int k = 0; k < 16; ++k) d[k] = samp.next();
                result.color = C(d[0], d[1], d[2], d[15]);
                return result;
            }, sparams, frame_num);
        }
        else if (mode == "ao" || mode == "bench")
        {
            const int AO_Samples = mode == "ao" && argc > 7 ? atoi(argv[7]) : 8;
            const S AO_Radius = 0.1f;
            // ao/main.cpp:183-246, the kernel as the reference's AO example writes it
            auto kernel = [=] __device__ (R ray, random_sampler<S>& samp) -> result_record<S>
            {
                result_record<S> result;
                result.color = C(bgcolor, 1.0f);

                auto hit_rec = closest_hit(
                        ray,
                        prims_begin,
                        prims_end
                        );

                result.hit = hit_rec.hit;

                if (any(hit_rec.hit))
                {
                    hit_rec.isect_pos = ray.ori + ray.dir * hit_rec.t;
                    result.isect_pos  = hit_rec.isect_pos;
                    result.depth      = hit_rec.t;                  // (added: the test compares t)

                    C clr(1.0);

                    auto n = get_normal(
                        device_normals,
                        hit_rec,
                        hip_index_bvh<tri_t>::bvh_ref{},      // was: index_bvh<tri_t>{} (a host container)
                        normals_per_face_binding{}
                        );

                    V u;
                    V v;
                    V w = n;
                    make_orthonormal_basis(u, v, w);

                    S radius = AO_Radius;

                    for (int i = 0; i < AO_Samples; ++i)
                    {
                        auto sp = cosine_sample_hemisphere(samp.next(), samp.next());

                        auto dir = normalize( sp.x * u + sp.y * v + sp.z * w );

                        R ao_ray;
                        ao_ray.ori = hit_rec.isect_pos + dir * S(1E-3f);
                        ao_ray.dir = dir;

                        auto ao_rec = any_hit(
                                ao_ray,
                                prims_begin,
                                prims_end,
                                radius
                                );

                        clr = select(
                                ao_rec.hit,
                                clr - S(1.0f / AO_Samples),
                                clr
                                );
                    }

                    result.color      = select( hit_rec.hit, C(clr.xyz(), S(1.0)), result.color );

                }

                return result;
            };
            if (mode == "ao")
            {
                const unsigned frame_num = argc > 6 ? unsigned(strtoul(argv[6], nullptr, 10)) : 0u;
                rt.clear_color_buffer();
                sched.frame(kernel, sparams, frame_num);
            }
            else
            {
                // bench <grid> <W> <H> <launches> [F]: median wall time per frame over `launches`
                // synchronous launches of F frames each (F = 1: one frame() per frame, as cuda_sched is
                // driven; F > 1: hip_sched::frames, frames in flight, distinct sampler seeds per frame)
                const int launches = argc > 5 ? atoi(argv[5]) : 10;
                const int F = argc > 6 ? atoi(argv[6]) : 1;
                hip_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rtF;
                rtF.resize(W, H * unsigned(F));
                std::vector<camera> cams(size_t(F), cam);
                std::vector<double> ms;
                for (int l = 0; l <= launches; ++l)
                {
                    auto t0 = std::chrono::steady_clock::now();
                    if (F == 1) sched.frame(kernel, sparams, unsigned(l));
                    else sched.frames(kernel, cams, rtF, unsigned(l * F));
                    hip_context::default_context()->sync();  // frame() only issues the launch (cuda_sched's model)
                    auto t1 = std::chrono::steady_clock::now();
                    if (l > 0) ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count() / F);
                }
                std::sort(ms.begin(), ms.end());
                printf("{\"mode\":\"bench\",\"kernel\":\"ao/main.cpp (reference headers)\",\"frame_ms_median\":%.4f,"
                       "\"launches\":%d,\"frames_per_launch\":%d}\n", ms[ms.size() / 2], launches, F);
                return 0;
            }
        }
        else if (shading)
        {
            // shade|whitted|multi <scene> <W> <H> <outdir> <face|vertex> [bounces eps]:
            // kernel<decltype(make_kernel_params(...))> over DEVICE pointers, as multi_hit/main.cpp:287-312
            // sets its CUDA kernel up (thrust::raw_pointer_cast of device vectors)
            const bool per_vertex = argc > 6 && std::string(argv[6]) == "vertex";
            const unsigned bounces = argc > 8 ? unsigned(atoi(argv[7])) : (mode == "whitted" ? 4u : 5u);
            const float eps = argc > 8 ? float(atof(argv[8])) : 1e-3f;
            aligned_vector<plastic<float>> materials;
            aligned_vector<point_light<float>> lights;
            vec4 ambient, bg;
            shade_spec(mode == "whitted", materials, lights, ambient, bg);
            // per-vertex normals of the harness: prim k, vertex j = normalize(n_k + 0.4 (U(b) - 0.5, ...)), b = (3k + j) 3
            aligned_vector<vec3> vnormals(tris.size() * 3);
            for (size_t k = 0; k < tris.size(); ++k)
                for (uint32_t j = 0; j < 3; ++j)
                {
                    uint32_t b = (uint32_t(k) * 3u + j) * 3u;
                    vec3 p((U(b) - 0.5f) * 0.4f, (U(b + 1) - 0.5f) * 0.4f, (U(b + 2) - 0.5f) * 0.4f);
                    vnormals[k * 3 + j] = normalize(normals[k] + p);
                }
            vec3 const* device_vnormals = device_copy(vnormals.data(), vnormals.size());
            plastic<float> const* device_materials = device_copy(materials.data(), materials.size());
            point_light<float> const* device_lights = device_copy(lights.data(), lights.size());
            auto run = [&](auto binding, vec3 const* nrm)
            {
                auto kparams = make_kernel_params(binding, prims_begin, prims_end, nrm, device_materials, device_lights,
                                                  device_lights + lights.size(), bounces, eps, bg, ambient);
                if (mode == "simple" || mode == "shade")
                {
                    simple::kernel<decltype(kparams)> kern;
                    kern.params = kparams;
                    sched.frame(kern, sparams);
                }
                else if (mode == "whitted")
                {
                    whitted::kernel<decltype(kparams)> kern;
                    kern.params = kparams;
                    sched.frame(kern, sparams);
                }
                else
                {
                    // multi_hit<16> + the multi_hit example's compositing (examples/multi_hit/main.cpp:166-235,
                    // the harness's run_multi_frame), hit lists into device arrays, kernel form (ray, x, y)
                    constexpr int N = 16;
                    std::vector<uint32_t> hp(size_t(W) * H * N, 0xFFFFFFFFu);
                    std::vector<float> ht(size_t(W) * H * N, -1.0f);
                    uint32_t* mh_pid = device_copy(hp.data(), hp.size());
                    float* mh_t = device_copy(ht.data(), ht.size());
                    const int w = W;
                    sched.frame([=] __device__ (R r, unsigned x, unsigned y) -> result_record<S>
                    {
                        auto const& params = kparams;
                        result_record<S> result;
                        result.color = C(0.0);
                        auto hit_rec = multi_hit<N>(r, params.prims.begin, params.prims.end);
                        size_t p = size_t(y) * w + x;
                        for (int i = 0; i < N; ++i)
                        {
                            if (!hit_rec[i].hit) break;
                            mh_pid[p * N + i] = hit_rec[i].prim_id;
                            mh_t[p * N + i] = hit_rec[i].t;
                        }
                        result.hit = hit_rec[0].hit;
                        result.isect_pos = r.ori + r.dir * hit_rec[0].t;
                        for (size_t i = 0; i < hit_rec.size(); ++i)
                        {
                            if (!hit_rec[i].hit) break;
                            hit_rec[i].isect_pos = r.ori + r.dir * hit_rec[i].t;
                            auto surf = get_surface(hit_rec[i], params);
                            auto view_dir = -r.dir;
                            auto n = surf.shading_normal;
                            n = faceforward(n, view_dir, surf.geometric_normal);
                            auto it = params.lights.begin;
                            auto sr = make_shade_record<decltype(kparams), S>();
                            sr.active = hit_rec[i].hit;
                            sr.isect_pos = hit_rec[i].isect_pos;
                            sr.normal = n;
                            sr.view_dir = view_dir;
                            sr.light_dir = normalize(V(it->position()) - hit_rec[i].isect_pos);
                            sr.light = *it;
                            auto shaded_clr = surf.shade(sr);
                            auto color = to_rgba(shaded_clr);
                            color.w = S(0.3);
                            color.xyz() *= color.w;
                            result.color += select(hit_rec[i].hit, color * (1.0f - result.color.w), C(0.0));
                        }
                        return result;
                    }, sparams);
                    if (hipMemcpy(hp.data(), mh_pid, hp.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
                        hipMemcpy(ht.data(), mh_t, ht.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
                        exit(4);
                    write_file(outdir + "/mh_prim_id.bin", hp.data(), hp.size() * 4);
                    write_file(outdir + "/mh_t.bin", ht.data(), ht.size() * 4);
                }
            };
            if (per_vertex) run(normals_per_vertex_binding{}, device_vnormals);
            else run(normals_per_face_binding{}, device_normals);
        }
        else
            return 2;

        const size_t npx = size_t(W) * H;
        std::vector<float> out(4 * npx), t(npx);
        rt.download(out.data(), nullptr, t.data());
        write_file(outdir + "/color.bin", out.data(), out.size() * 4);
        write_file(outdir + "/t.bin", t.data(), t.size() * 4);
        printf("{\"mode\":\"%s\",\"W\":%d,\"H\":%d}\n", mode.c_str(), W, H);
    }
    catch (std::exception const& e)
    {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
