// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as product).
//
// Drives the *reference* Visionaray headers (compiled in place from /root/reference/include by
// oracle/Makefile; no reference source is copied into this repository) to produce:
//
//   golden <scene> <outdir> [W H]  : reference BVH (build<index_bvh<P>>, build.inl:165-178), the
//                                    scalar simple_sched<basic_ray<float>> frame (simple_sched.inl:
//                                    139-151) of primary closest_hit (traverse_linear.inl:286-329) and
//                                    the parity version of the ao/main.cpp:183-246 kernel (SURVEY.md
//                                    Appendix A), written as raw little-endian arrays + hashes.
//   shade  <scene> <outdir> <face|vertex> [W H]
//                                  : simple::kernel (detail/simple.inl:19-83) through the reference's
//                                    make_kernel_params (kernels.h:357-389), plastic<float> materials
//                                    by geom_id (= prim index % 3) and two point lights (the spec in
//                                    shade_spec() below, mirrored by tests/shading_spec.py), colour
//                                    frame written as color.bin + hash.
//   whitted <scene> <outdir> <face|vertex> [W H] [bounces eps]
//                                  : whitted::kernel (detail/whitted.inl:186-277) through the same
//                                    make_kernel_params, shade_spec + a third light (whitted_spec).
//   multi  <scene> <outdir> <face|vertex> [W H]
//                                  : multi_hit<16> (traverse_linear.inl:333-380) per pixel over the
//                                    shade-mode scene, hit lists (prim_id / t) + the compositing
//                                    kernel of examples/multi_hit/main.cpp:166-235 (restated on the
//                                    reference's get_surface / plastic::shade).
//   rsampler <scene> <outdir> <W> <H> <frame> [samples]
//                                  : ao/main.cpp:183-246 verbatim (random_sampler<float> +
//                                    cosine_sample_hemisphere) with hip_sched's per-pixel seeds
//                                    (built by clang++: vsnray_ref_clang)
//   bench  <scene> <threads> <frames> [W H] [samples]
//                                  : the reference SSE4 CPU path, tiled_sched<basic_ray<simd::float4>>
//                                    (tiled_sched.inl:365-391) running the ao/main.cpp:183-246 kernel
//                                    verbatim in behaviour (random_sampler + cosine_sample_hemisphere),
//                                    timed; prints one JSON line (Mrays/s, rays, cores).
//
// The synthetic scenes follow SURVEY.md Appendix A (libm-free, fixed seeds).  This file is the only
// place that instantiates reference code; outputs land in oracle/_ref/ or a caller-given directory.

#include <visionaray/math/math.h>
#include <visionaray/bvh.h>
#include <visionaray/camera.h>
#include <visionaray/get_normal.h>
#include <visionaray/detail/bvh/statistics.h>
#include <visionaray/kernels.h>
#include <visionaray/material.h>
#include <visionaray/point_light.h>
#include <visionaray/result_record.h>
#include <visionaray/sampling.h>
#include <visionaray/random_sampler.h>
#include <visionaray/scheduler.h>
#include <visionaray/simple_buffer_rt.h>
#include <visionaray/traverse.h>

#include <atomic>
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using namespace visionaray;

using tri_t = basic_triangle<3, float>;
using sph_t = basic_sphere<float>;

//-------------------------------------------------------------------------------------------------
// Appendix A scene generators
//

static inline uint32_t wang(uint32_t a)
{
    a = (a ^ 61u) ^ (a >> 16);
    a = a + (a << 3);
    a = a ^ (a >> 4);
    a = a * 0x27d4eb2du;
    a = a ^ (a >> 15);
    return a;
}

static inline float U(uint32_t k)
{
    return float(wang(k) >> 8) * (1.0f / 16777216.0f);
}

static vec3 hf_vertex(int grid, int i, int j)
{
    float x = -1.0f + 2.0f * float(i) / float(grid);
    float z = -1.0f + 2.0f * float(j) / float(grid);
    uint32_t k = uint32_t(j) * uint32_t(grid + 1) + uint32_t(i);
    float y = 0.3f * x * z * (1.0f - x * x) * (1.0f - z * z) + 0.004f * (U(k) - 0.5f);
    return vec3(x, y, z);
}

static void make_heightfield(int grid, aligned_vector<tri_t>& tris)
{
    tris.resize(size_t(2) * grid * grid);
    std::vector<vec3> row0(grid + 1), row1(grid + 1);
    for (int j = 0; j < grid; ++j)
    {
        for (int i = 0; i <= grid; ++i) { row0[i] = hf_vertex(grid, i, j); row1[i] = hf_vertex(grid, i, j + 1); }
        for (int i = 0; i < grid; ++i)
        {
            vec3 a = row0[i], b = row0[i + 1], c = row1[i + 1], e = row1[i];
            size_t base = size_t(2) * (size_t(j) * grid + i);
            tri_t& t0 = tris[base];
            t0.v1 = a; t0.e1 = b - a; t0.e2 = c - a; t0.prim_id = unsigned(base); t0.geom_id = 0;
            tri_t& t1 = tris[base + 1];
            t1.v1 = a; t1.e1 = c - a; t1.e2 = e - a; t1.prim_id = unsigned(base + 1); t1.geom_id = 0;
        }
    }
}

// hfstack<G>x<K>: K copies of hf<G>, layer k shifted down by 0.03 * k (prim_id = k * n + i): rays
// from above cross many layers (multi-hit tests)
static void make_hfstack(int grid, int layers, aligned_vector<tri_t>& tris)
{
    aligned_vector<tri_t> one;
    make_heightfield(grid, one);
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

static void make_cornell(aligned_vector<tri_t>& tris)
{
    const float q[6][4][3] = {
        {{-1,-1,-1},{ 1,-1,-1},{ 1,-1, 1},{-1,-1, 1}},
        {{-1, 1,-1},{-1, 1, 1},{ 1, 1, 1},{ 1, 1,-1}},
        {{-1,-1,-1},{-1, 1,-1},{ 1, 1,-1},{ 1,-1,-1}},
        {{-1,-1,-1},{-1,-1, 1},{-1, 1, 1},{-1, 1,-1}},
        {{ 1,-1,-1},{ 1, 1,-1},{ 1, 1, 1},{ 1,-1, 1}},
        {{-.25f,.99f,-.25f},{-.25f,.99f,.25f},{.25f,.99f,.25f},{.25f,.99f,-.25f}},
    };
    tris.clear();
    for (int f = 0; f < 6; ++f)
    {
        vec3 a(q[f][0]), b(q[f][1]), c(q[f][2]), d(q[f][3]);
        tri_t t;
        t.geom_id = 0;
        t.v1 = a; t.e1 = b - a; t.e2 = c - a; t.prim_id = unsigned(tris.size()); tris.push_back(t);
        t.v1 = a; t.e1 = c - a; t.e2 = d - a; t.prim_id = unsigned(tris.size()); tris.push_back(t);
    }
}

static void make_spheres(int n, aligned_vector<sph_t>& s)
{
    s.resize(n);
    for (int i = 0; i < n; ++i)
    {
        uint32_t k = uint32_t(6) * uint32_t(i);
        s[i].center = vec3(2.0f * U(k) - 1.0f, 2.0f * U(k + 1) - 1.0f, 2.0f * U(k + 2) - 1.0f);
        s[i].radius = 0.002f + 0.008f * U(k + 3);
        s[i].prim_id = unsigned(i);
        s[i].geom_id = 0;
    }
}

//-------------------------------------------------------------------------------------------------
// Hashing (FNV-1a 64; SURVEY.md Appendix B conventions)
//

struct fnv
{
    uint64_t h = 0xcbf29ce484222325ull;
    void bytes(void const* p, size_t n)
    {
        auto b = static_cast<unsigned char const*>(p);
        for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ull; }
    }
    void u32(uint32_t w) { bytes(&w, 4); }
};

static void write_file(std::string const& path, void const* p, size_t n)
{
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { perror(path.c_str()); exit(2); }
    if (n && fwrite(p, 1, n, f) != n) { perror("fwrite"); exit(2); }
    fclose(f);
}

static uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

//-------------------------------------------------------------------------------------------------
// Scene description
//

struct scene_desc
{
    std::string name;
    bool spheres = false;
    int  grid = 0;        // heightfield grid, 0 = cornell
    int  nspheres = 0;
    int  layers = 0;      // hfstack
    vec3 eye;
    int  W = 1920, H = 1080;
};

static scene_desc lookup(std::string const& name)
{
    scene_desc d;
    d.name = name;
    if (name == "cornell12") { d.grid = 0; d.eye = vec3(0.0f, 0.0f, 3.4f); d.W = 512; d.H = 512; }
    else if (name == "hf1M")  { d.grid = 708;  d.eye = vec3(0.0f, 0.9f, 1.4f); }
    else if (name == "hf10M") { d.grid = 2236; d.eye = vec3(0.0f, 0.9f, 1.4f); }
    else if (name == "sph1M") { d.spheres = true; d.nspheres = 1000000; d.eye = vec3(0.0f, 0.0f, 3.5f); }
    else if (name.compare(0, 7, "hfstack") == 0)
    {
        d.grid = atoi(name.c_str() + 7);
        d.layers = atoi(strchr(name.c_str(), 'x') + 1);
        d.eye = vec3(0.0f, 0.9f, 1.4f);
    }
    else if (name.compare(0, 2, "hf") == 0) { d.grid = atoi(name.c_str() + 2); d.eye = vec3(0.0f, 0.9f, 1.4f); }
    else if (name.compare(0, 3, "sph") == 0) { d.spheres = true; d.nspheres = atoi(name.c_str() + 3); d.eye = vec3(0.0f, 0.0f, 3.5f); }
    else { fprintf(stderr, "unknown scene %s\n", name.c_str()); exit(2); }
    return d;
}

static camera make_camera(scene_desc const& d, int W, int H)
{
    camera cam;
    float aspect = W / static_cast<float>(H);
    cam.perspective(45.0f * constants::degrees_to_radians<float>(), aspect, 0.001f, 1000.0f);
    cam.look_at(d.eye, vec3(0.0f, 0.0f, 0.0f), vec3(0.0f, 1.0f, 0.0f));
    return cam;
}

//-------------------------------------------------------------------------------------------------
// golden: scalar simple_sched frame, primary closest hit + parity AO
//

//-------------------------------------------------------------------------------------------------
// mask: the intersector example's mask_intersector (examples/intersector/main.cpp:251-330) -- a
// basic_intersector (intersector.h:24-119) whose triangle operator() clears hr.hit where a mask over
// the hit's texture coordinate (get_tex_coord.h:25-38 -> lerp, math.h:468-475) says so -- with the
// example's procedural heart replaced by a byte mask (the test's data), looked up at the nearest
// texel exactly as vrh.h vrh_hit_mask_create states
//

struct mask_intersector : basic_intersector<mask_intersector>
{
    using basic_intersector<mask_intersector>::operator();

    template <typename R, typename S>
    auto operator()(R const& ray, basic_triangle<3, S> const& tri) -> decltype( intersect(ray, tri) )
    {
        auto hr = intersect(ray, tri);
        if (!hr.hit) return hr;
        vec2 tc = get_tex_coord(tex_coords, hr, tri);
        hr.hit &= mask[texel(tc.y, h) * unsigned(w) + texel(tc.x, w)] != 0;
        return hr;
    }

    static unsigned texel(float c, int n)
    {
        float x = (c > 0.0f ? c : 0.0f) * float(n);
        return x < float(n) ? unsigned(x) : unsigned(n - 1);
    }

    vec2 const* tex_coords = nullptr;
    uint8_t const* mask = nullptr;
    int w = 0, h = 0;
};

//-------------------------------------------------------------------------------------------------
// heart: the intersector example's procedural cut-out itself (examples/intersector/main.cpp:251-330:
// tc -> (x, y) = 3 tc - 1.5, kept where (x^2 + y^2 - 1)^3 - x^2 y^3 < 0), evaluated per lane.  For
// scalar rays the example's Mask(hits) is bool(bool[1]) -- a pointer, always true -- so the scalar
// reference would cut nothing out; this restates what its SIMD rays compute, one lane at a time.
//

struct heart_intersector : basic_intersector<heart_intersector>
{
    using basic_intersector<heart_intersector>::operator();

    template <typename R, typename S>
    auto operator()(R const& ray, basic_triangle<3, S> const& tri) -> decltype( intersect(ray, tri) )
    {
        auto hr = intersect(ray, tri);
        if (!hr.hit) return hr;
        vec2 tc = get_tex_coord(tex_coords, hr, tri);
        float x = tc.x * 3.0f - 1.5f;
        float y = tc.y * 3.0f - 1.5f;
        hr.hit &= (pow(x * x + y * y - 1.0f, 3.0f) - x * x * y * y * y) < 0.0f;
        return hr;
    }

    vec2 const* tex_coords = nullptr;
};

// the parity AO sampler of SURVEY.md Appendix A, frame n offset by n * 0x9E3779B1 (the build's
// stand-in for the reference's per-frame reseeding, cuda_sched.inl:38-45, 79; frame 0 = Appendix A):
// Malley sample s of pixel p
static vec2 ao_sample(uint32_t p, int smp, uint32_t frame_num)
{
    for (uint32_t k = 0; k < 16; ++k)
    {
        uint32_t ctr = ((p * 8u + uint32_t(smp)) * 16u + k) * 2u + frame_num * 0x9E3779B1u;
        float xa = 2.0f * U(ctr) - 1.0f;
        float ya = 2.0f * U(ctr + 1) - 1.0f;
        if (xa * xa + ya * ya < 1.0f) return vec2(xa, ya);
    }
    return vec2(0.0f, 0.0f);
}

template <typename P, typename Isect = default_intersector>
static int run_golden(scene_desc const& d, aligned_vector<P>& prims, std::vector<vec3> const& normals,
                      std::string const& outdir, int W, int H, bool do_ao, Isect isect = Isect{},
                      uint32_t frame_num = 0)
{
    auto t0 = std::chrono::steady_clock::now();
    auto bvh = build<index_bvh<P>>(prims.data(), prims.size());
    auto t1 = std::chrono::steady_clock::now();

    fnv hn, hi;
    unsigned max_depth = 0;
    for (auto const& n : bvh.nodes()) { uint32_t w[8]; std::memcpy(w, &n, 32); for (int k = 0; k < 8; ++k) hn.u32(w[k]); }
    for (auto i : bvh.indices()) hi.u32(i);
    {
        // tree depth (root depth 0), for stack-size planning
        std::vector<std::pair<unsigned, unsigned>> st{{0u, 0u}};
        while (!st.empty())
        {
            auto e = st.back(); st.pop_back();
            max_depth = std::max(max_depth, e.second);
            auto const& n = bvh.nodes()[e.first];
            if (n.num_prims == 0) { st.push_back({n.first_child, e.second + 1}); st.push_back({n.first_child + 1, e.second + 1}); }
        }
    }
    write_file(outdir + "/nodes.bin", bvh.nodes().data(), bvh.nodes().size() * sizeof(bvh_node));
    write_file(outdir + "/indices.bin", bvh.indices().data(), bvh.indices().size() * 4);
    write_file(outdir + "/prims.bin", prims.data(), prims.size() * sizeof(P));

    camera cam = make_camera(d, W, H);

    // camera basis exactly as simple_sched.inl:61-89 computes it (recorded as bits)
    auto f = normalize(cam.eye() - cam.center());
    auto s = normalize(cross(cam.up(), f));
    auto u = cross(f, s);
    vec3 cam_u = s * float(tan(cam.fovy() / 2.0f) * cam.aspect());
    vec3 cam_v = u * float(tan(cam.fovy() / 2.0f));
    vec3 cam_w = -f;
    vec3 basis[4] = { cam.eye(), cam_u, cam_v, cam_w };
    write_file(outdir + "/camera.bin", basis, sizeof(basis));

    size_t npx = size_t(W) * H;
    std::vector<uint32_t> prim_id(npx, 0xFFFFFFFFu);
    std::vector<float> tval(npx, -1.0f);
    std::vector<uint8_t> occ(npx, 0);
    std::vector<uint32_t> leaf_pos(npx, 0xFFFFFFFFu);

    using bvh_ref = typename index_bvh<P>::bvh_ref;
    std::vector<bvh_ref> bvhs{ bvh.ref() };
    auto prims_begin = bvhs.data();
    auto prims_end = bvhs.data() + bvhs.size();

    simple_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
    rt.resize(W, H);
    auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);
    simple_sched<ray> sched;

    uint64_t ao_rays = 0, ao_occ = 0;
    const vec4 bg(0.1f, 0.2f, 0.3f, 1.0f);

    sched.frame([&](ray r, unsigned x, unsigned y) -> result_record<float>
    {
        result_record<float> result;
        result.color = bg;
        auto hr = closest_hit(r, prims_begin, prims_end, isect);
        result.hit = hr.hit;
        size_t p = size_t(y) * W + x;
        if (!hr.hit) return result;
        prim_id[p] = hr.prim_id;
        tval[p] = hr.t;
        leaf_pos[p] = hr.primitive_list_index;
        if (!do_ao) { result.color = vec4(1.0f); return result; }

        hr.isect_pos = r.ori + r.dir * hr.t;
        vec4 clr(1.0f);
        vec3 n = normals[hr.prim_id];
        vec3 uu, vv, w = n;
        make_orthonormal_basis(uu, vv, w);
        uint8_t mask = 0;
        for (int smp = 0; smp < 8; ++smp)
        {
            vec2 sxy = ao_sample(uint32_t(p), smp, frame_num);
            float sx = sxy.x, sy = sxy.y;
            float sz = sqrt(std::max(0.0f, 1.0f - sx * sx - sy * sy));
            auto dir = normalize(sx * uu + sy * vv + sz * w);
            ray ao;
            ao.ori = hr.isect_pos + dir * 1E-3f;
            ao.dir = dir;
            auto ar = any_hit(ao, prims_begin, prims_end, 0.1f, isect);
            ++ao_rays;
            if (ar.hit) { clr = clr - 1.0f / 8; mask |= uint8_t(1u << smp); ++ao_occ; }
        }
        occ[p] = mask;
        result.color = vec4(clr.xyz(), 1.0f);
        return result;
    }, sparams);
    auto t2 = std::chrono::steady_clock::now();

    write_file(outdir + "/prim_id.bin", prim_id.data(), npx * 4);
    write_file(outdir + "/t.bin", tval.data(), npx * 4);
    write_file(outdir + "/leaf_pos.bin", leaf_pos.data(), npx * 4);
    write_file(outdir + "/color.bin", rt.color(), npx * 16);
    if (do_ao) write_file(outdir + "/occ.bin", occ.data(), npx);

    fnv hp, ht, ho, hc;
    uint64_t hits = 0;
    for (size_t p = 0; p < npx; ++p)
    {
        hp.u32(prim_id[p]); ht.u32(fbits(tval[p])); ho.bytes(&occ[p], 1);
        hits += prim_id[p] != 0xFFFFFFFFu;
    }
    hc.bytes(rt.color(), npx * 16);

    printf("{\"scene\":\"%s\",\"W\":%d,\"H\":%d,\"prims\":%zu,\"nodes\":%zu,\"max_depth\":%u,"
           "\"bvh_hash\":\"%016llx\",\"idx_hash\":\"%016llx\",\"hits\":%llu,\"ao_rays\":%llu,\"ao_occluded\":%llu,"
           "\"primid_hash\":\"%016llx\",\"t_hash\":\"%016llx\",\"occmask_hash\":\"%016llx\",\"color_hash\":\"%016llx\","
           "\"cam_u\":[\"%08x\",\"%08x\",\"%08x\"],\"cam_v\":[\"%08x\",\"%08x\",\"%08x\"],\"cam_w\":[\"%08x\",\"%08x\",\"%08x\"],"
           "\"build_s\":%.3f,\"render_s\":%.3f}\n",
           d.name.c_str(), W, H, prims.size(), bvh.nodes().size(), max_depth,
           (unsigned long long)hn.h, (unsigned long long)hi.h, (unsigned long long)hits,
           (unsigned long long)ao_rays, (unsigned long long)ao_occ,
           (unsigned long long)hp.h, (unsigned long long)ht.h, (unsigned long long)ho.h, (unsigned long long)hc.h,
           fbits(cam_u.x), fbits(cam_u.y), fbits(cam_u.z), fbits(cam_v.x), fbits(cam_v.y), fbits(cam_v.z),
           fbits(cam_w.x), fbits(cam_w.y), fbits(cam_w.z),
           std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count());
    return 0;
}

//-------------------------------------------------------------------------------------------------
// shade: simple::kernel with plastic materials and point lights
//

struct shade_spec
{
    aligned_vector<plastic<float>> materials;
    aligned_vector<point_light<float>> lights;
    vec4 ambient, bg;
};

static shade_spec make_shade_spec()
{
    shade_spec sp;
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
        sp.materials.push_back(p);
    }
    point_light<float> l0;
    l0.set_position(vec3(0.5f, 2.0f, 1.5f));
    l0.set_cl(vec3(1.0f, 1.0f, 1.0f));
    l0.set_kl(1.0f);
    sp.lights.push_back(l0);
    point_light<float> l1;
    l1.set_position(vec3(-1.5f, 1.0f, 0.5f));
    l1.set_cl(vec3(1.0f, 0.8f, 0.6f));
    l1.set_kl(0.7f);
    l1.set_constant_attenuation(1.0f);
    l1.set_linear_attenuation(0.1f);
    l1.set_quadratic_attenuation(0.05f);
    sp.lights.push_back(l1);
    sp.ambient = vec4(0.4f, 0.4f, 0.4f, 0.5f);
    sp.bg = vec4(0.1f, 0.2f, 0.3f, 1.0f);
    return sp;
}

// whitted_spec (tests' oracle.whitted_spec): shade_spec plus a light inside the scenes
static shade_spec make_whitted_spec()
{
    shade_spec sp = make_shade_spec();
    point_light<float> l2;
    l2.set_position(vec3(0.2f, 0.6f, 0.3f));
    l2.set_cl(vec3(0.9f, 0.9f, 1.0f));
    l2.set_kl(0.8f);
    l2.set_constant_attenuation(1.0f);
    l2.set_linear_attenuation(0.2f);
    l2.set_quadratic_attenuation(0.1f);
    sp.lights.push_back(l2);
    return sp;
}

template <template <typename> class Kernel, typename Binding, typename Normals>
static void shade_frame(std::vector<typename index_bvh<tri_t>::bvh_ref> const& bvhs, Normals const* normals,
                        shade_spec const& sp, unsigned bounces, float eps, camera const& cam,
                        simple_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED>& rt)
{
    auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);
    simple_sched<ray> sched;
    auto kp = make_kernel_params(Binding{}, bvhs.data(), bvhs.data() + bvhs.size(), normals, sp.materials.data(),
                                 sp.lights.data(), sp.lights.data() + sp.lights.size(), bounces, eps, sp.bg,
                                 sp.ambient);
    Kernel<decltype(kp)> kern;
    kern.params = kp;
    sched.frame(kern, sparams);
}

static int run_shade(scene_desc const& d, aligned_vector<tri_t>& prims, std::vector<vec3> const& face_normals,
                     std::string const& outdir, bool per_vertex, int W, int H, bool whitted = false,
                     unsigned bounces = 4, float eps = 1e-3f)
{
    for (size_t i = 0; i < prims.size(); ++i) prims[i].geom_id = unsigned(i % 3);
    auto bvh = build<index_bvh<tri_t>>(prims.data(), prims.size());
    using bvh_ref = typename index_bvh<tri_t>::bvh_ref;
    std::vector<bvh_ref> bvhs{ bvh.ref() };
    // per-vertex normals: prim k, vertex j: normalize(n_k + 0.4 * (U(b) - 0.5, ...)), b = (3k + j) * 3
    std::vector<vec3> vnormals(prims.size() * 3);
    for (size_t k = 0; k < prims.size(); ++k)
        for (uint32_t j = 0; j < 3; ++j)
        {
            uint32_t b = (uint32_t(k) * 3u + j) * 3u;
            vec3 p((U(b) - 0.5f) * 0.4f, (U(b + 1) - 0.5f) * 0.4f, (U(b + 2) - 0.5f) * 0.4f);
            vnormals[k * 3 + j] = normalize(face_normals[k] + p);
        }
    shade_spec sp = whitted ? make_whitted_spec() : make_shade_spec();
    camera cam = make_camera(d, W, H);
    simple_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
    rt.resize(W, H);
    if (whitted && per_vertex)
        shade_frame<whitted::kernel, normals_per_vertex_binding>(bvhs, vnormals.data(), sp, bounces, eps, cam, rt);
    else if (whitted)
        shade_frame<whitted::kernel, normals_per_face_binding>(bvhs, face_normals.data(), sp, bounces, eps, cam, rt);
    else if (per_vertex)
        shade_frame<simple::kernel, normals_per_vertex_binding>(bvhs, vnormals.data(), sp, 5u, 1e-3f, cam, rt);
    else
        shade_frame<simple::kernel, normals_per_face_binding>(bvhs, face_normals.data(), sp, 5u, 1e-3f, cam, rt);
    size_t npx = size_t(W) * H;
    write_file(outdir + "/color.bin", rt.color(), npx * 16);
    fnv hc;
    hc.bytes(rt.color(), npx * 16);
    printf("{\"scene\":\"%s\",\"W\":%d,\"H\":%d,\"binding\":\"%s\",\"kernel\":\"%s\",\"bounces\":%u,"
           "\"eps\":%.9g,\"color_hash\":\"%016llx\"}\n",
           d.name.c_str(), W, H, per_vertex ? "vertex" : "face", whitted ? "whitted" : "simple", bounces, eps,
           (unsigned long long)hc.h);
    return 0;
}

//-------------------------------------------------------------------------------------------------
// multi: multi_hit<16> hit lists + the multi_hit example's compositing
//

template <typename Params>
static void run_multi_frame(Params const& params, camera const& cam, int W, int H, std::string const& outdir)
{
    constexpr int N = 16;
    simple_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
    rt.resize(W, H);
    auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);
    simple_sched<ray> sched;
    size_t npx = size_t(W) * H;
    std::vector<uint32_t> mh_pid(npx * N, 0xFFFFFFFFu);
    std::vector<float> mh_t(npx * N, -1.0f);
    sched.frame([&](ray r, unsigned x, unsigned y) -> result_record<float>
    {
        using S = float;
        using C = vector<4, S>;
        using V = vector<3, S>;
        result_record<S> result;
        result.color = C(0.0);
        auto hit_rec = multi_hit<N>(r, params.prims.begin, params.prims.end);
        size_t p = size_t(y) * W + x;
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
            auto sr = make_shade_record<Params, S>();
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
    write_file(outdir + "/color.bin", rt.color(), npx * 16);
    write_file(outdir + "/mh_prim_id.bin", mh_pid.data(), mh_pid.size() * 4);
    write_file(outdir + "/mh_t.bin", mh_t.data(), mh_t.size() * 4);
    fnv hc, hp, ht;
    hc.bytes(rt.color(), npx * 16);
    hp.bytes(mh_pid.data(), mh_pid.size() * 4);
    ht.bytes(mh_t.data(), mh_t.size() * 4);
    size_t hits = 0;
    for (auto v : mh_pid) hits += v != 0xFFFFFFFFu;
    printf("{\"W\":%d,\"H\":%d,\"max_hits\":%d,\"hits\":%zu,\"color_hash\":\"%016llx\","
           "\"mh_primid_hash\":\"%016llx\",\"mh_t_hash\":\"%016llx\"}\n", W, H, N, hits,
           (unsigned long long)hc.h, (unsigned long long)hp.h, (unsigned long long)ht.h);
}

static int run_multi(scene_desc const& d, aligned_vector<tri_t>& prims, std::vector<vec3> const& face_normals,
                     std::string const& outdir, bool per_vertex, int W, int H)
{
    for (size_t i = 0; i < prims.size(); ++i) prims[i].geom_id = unsigned(i % 3);
    auto bvh = build<index_bvh<tri_t>>(prims.data(), prims.size());
    using bvh_ref = typename index_bvh<tri_t>::bvh_ref;
    std::vector<bvh_ref> bvhs{ bvh.ref() };
    std::vector<vec3> vnormals(prims.size() * 3);
    for (size_t k = 0; k < prims.size(); ++k)
        for (uint32_t j = 0; j < 3; ++j)
        {
            uint32_t b = (uint32_t(k) * 3u + j) * 3u;
            vec3 p((U(b) - 0.5f) * 0.4f, (U(b + 1) - 0.5f) * 0.4f, (U(b + 2) - 0.5f) * 0.4f);
            vnormals[k * 3 + j] = normalize(face_normals[k] + p);
        }
    shade_spec sp = make_shade_spec();
    camera cam = make_camera(d, W, H);
    if (per_vertex)
        run_multi_frame(make_kernel_params(normals_per_vertex_binding{}, bvhs.data(), bvhs.data() + bvhs.size(),
                                           vnormals.data(), sp.materials.data(), sp.lights.data(),
                                           sp.lights.data() + sp.lights.size()), cam, W, H, outdir);
    else
        run_multi_frame(make_kernel_params(normals_per_face_binding{}, bvhs.data(), bvhs.data() + bvhs.size(),
                                           face_normals.data(), sp.materials.data(), sp.lights.data(),
                                           sp.lights.data() + sp.lights.size()), cam, W, H, outdir);
    return 0;
}

//-------------------------------------------------------------------------------------------------
// bench: reference SSE4 tiled_sched<ray4> path, ao/main.cpp kernel
//

template <typename P>
static int run_bench(scene_desc const& d, aligned_vector<P>& prims, std::vector<vec3> const& normals,
                     int threads, int frames, int W, int H, int samples)
{
    using R = basic_ray<simd::float4>;
    using S = R::scalar_type;
    using C = vector<4, S>;
    using V = vector<3, S>;

    auto bvh = build<index_bvh<P>>(prims.data(), prims.size());
    camera cam = make_camera(d, W, H);

    using bvh_ref = typename index_bvh<P>::bvh_ref;
    std::vector<bvh_ref> bvhs{ bvh.ref() };
    auto prims_begin = bvhs.data();
    auto prims_end = bvhs.data() + bvhs.size();

    simple_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
    rt.resize(W, H);
    auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);
    tiled_sched<R> sched(threads);
    // tiled_sched can lose the wakeup of a worker that is not waiting yet (tiled_sched.inl:181,386)
    std::this_thread::sleep_for(std::chrono::milliseconds(300));

    std::atomic<uint64_t> rays{0};
    float radius = 0.1f;
    auto kernel = [&](R ray, random_sampler<S>& samp) -> result_record<S>
    {
        result_record<S> result;
        result.color = C(vec4(0.1f, 0.2f, 0.3f, 1.0f));
        auto hit_rec = closest_hit(ray, prims_begin, prims_end);
        result.hit = hit_rec.hit;
        uint64_t local = 4;
        if (samples > 0 && any(hit_rec.hit))
        {
            hit_rec.isect_pos = ray.ori + ray.dir * hit_rec.t;
            C clr(1.0);
            V n;
            if (!d.spheres)
                n = get_normal(normals.data(), hit_rec, index_bvh<tri_t>{}, normals_per_face_binding{});
            else
                n = V(vec3(0.0f, 1.0f, 0.0f));
            V u, v, w = n;
            make_orthonormal_basis(u, v, w);
            alignas(16) float hf[4];
            simd::store(hf, select(hit_rec.hit, S(1.0f), S(0.0f)));
            int nh = int(hf[0] + hf[1] + hf[2] + hf[3]);
            for (int i = 0; i < samples; ++i)
            {
                auto sp = cosine_sample_hemisphere(samp.next(), samp.next());
                auto dir = normalize(sp.x * u + sp.y * v + sp.z * w);
                R ao_ray;
                ao_ray.ori = hit_rec.isect_pos + dir * S(1E-3f);
                ao_ray.dir = dir;
                auto ao_rec = any_hit(ao_ray, prims_begin, prims_end, S(radius));
                clr = select(ao_rec.hit, clr - S(1.0f / samples), clr);
            }
            local += uint64_t(nh) * samples;
            result.color = select(hit_rec.hit, C(clr.xyz(), S(1.0)), result.color);
        }
        rays.fetch_add(local, std::memory_order_relaxed);
        return result;
    };

    sched.frame(kernel, sparams);  // warm-up
    std::vector<double> times;
    uint64_t rays_per_frame = 0;
    for (int f = 0; f < frames; ++f)
    {
        // the same lost wakeup between frames: a worker still leaving the last frame's tile loop
        // misses the next notify_all, and if all of them do, frame() waits forever -- give them
        // time to reach threads_start.wait() (outside the timed region)
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        rays = 0;
        auto t0 = std::chrono::steady_clock::now();
        sched.frame(kernel, sparams);
        auto t1 = std::chrono::steady_clock::now();
        times.push_back(std::chrono::duration<double>(t1 - t0).count());
        rays_per_frame = rays.load();
    }
    std::sort(times.begin(), times.end());
    double med = times[times.size() / 2];
    printf("{\"kind\":\"reference\",\"path\":\"tiled_sched<basic_ray<simd::float4>> -O3 -msse4.1\",\"scene\":\"%s\","
           "\"W\":%d,\"H\":%d,\"samples\":%d,\"threads\":%d,\"frames\":%d,\"rays_per_frame\":%llu,"
           "\"median_s\":%.6f,\"min_s\":%.6f,\"max_s\":%.6f,\"mrays_per_s\":%.3f}\n",
           d.name.c_str(), W, H, samples, threads, frames, (unsigned long long)rays_per_frame, med,
           times.front(), times.back(), rays_per_frame / med / 1e6);
    return 0;
}

//-------------------------------------------------------------------------------------------------

template <typename F>
static int with_scene(scene_desc const& d, F&& f)
{
    if (d.spheres)
    {
        aligned_vector<sph_t> s;
        make_spheres(d.nspheres, s);
        std::vector<vec3> normals;
        return f(s, normals);
    }
    aligned_vector<tri_t> t;
    if (d.grid == 0) make_cornell(t); else if (d.layers) make_hfstack(d.grid, d.layers, t); else make_heightfield(d.grid, t);
    std::vector<vec3> normals(t.size());
    for (size_t i = 0; i < t.size(); ++i) normals[i] = normalize(cross(t[i].e1, t[i].e2));
    return f(t, normals);
}

//-------------------------------------------------------------------------------------------------
// list: closest_hit / any_hit over a LIST of two BVH refs (traverse_linear.inl:76-141) -- the
// scene's triangles split by prim_id parity, each half its own build<index_bvh<P>> -- rendered by
// tiled_sched<ray> (tiled_sched.inl:365-391) with a scissor box (the clip of tiled_sched.inl:
// 244-260): pixels x0 <= x < x1, y0 <= y < y1 (tiled_sched reads recti(x, y, width, height), so
// the box is recti(x0, y0, x1 - x0, y1 - y0); cuda_sched reads the same pixel set from
// recti(x0, y0, x1, y1), cuda_sched.inl:71).  Kernel: the golden primary + parity AO of frame
// `frame_num`.  Pixels outside the box keep the cleared target (colour 0, prim_id ~0, t -1, occ 0).
//

static int run_list(scene_desc const& d, aligned_vector<tri_t> const& all, std::string const& outdir, int W, int H,
                    int const sb[4], uint32_t frame_num)
{
    aligned_vector<tri_t> part[2];
    for (auto const& tri : all) part[tri.prim_id % 2u].push_back(tri);
    std::vector<vec3> normals(all.size());
    for (auto const& tri : all) normals[tri.prim_id] = normalize(cross(tri.e1, tri.e2));
    auto b0 = build<index_bvh<tri_t>>(part[0].data(), part[0].size());
    auto b1 = build<index_bvh<tri_t>>(part[1].data(), part[1].size());
    for (int k = 0; k < 2; ++k)
    {
        auto const& b = k == 0 ? b0 : b1;
        std::string pre = outdir + "/bvh" + std::to_string(k) + "_";
        write_file(pre + "nodes.bin", b.nodes().data(), b.nodes().size() * sizeof(bvh_node));
        write_file(pre + "indices.bin", b.indices().data(), b.indices().size() * 4);
        write_file(pre + "prims.bin", part[k].data(), part[k].size() * sizeof(tri_t));
    }
    using bvh_ref = index_bvh<tri_t>::bvh_ref;
    std::vector<bvh_ref> bvhs{ b0.ref(), b1.ref() };
    auto prims_begin = bvhs.data();
    auto prims_end = bvhs.data() + bvhs.size();

    camera cam = make_camera(d, W, H);
    size_t npx = size_t(W) * H;
    std::vector<uint32_t> prim_id(npx, 0xFFFFFFFFu), leaf_pos(npx, 0xFFFFFFFFu);
    std::vector<float> tval(npx, -1.0f);
    std::vector<uint8_t> occ(npx, 0);
    simple_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
    rt.resize(W, H);
    rt.clear_color_buffer(vec4(0.0f));
    auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);
    sparams.scissor_box = recti(sb[0], sb[1], sb[2] - sb[0], sb[3] - sb[1]);
    const vec4 bg(0.1f, 0.2f, 0.3f, 1.0f);
    std::atomic<uint64_t> ao_rays{0}, ao_occ{0};
    tiled_sched<ray> sched(2);
    // tiled_sched can lose the wakeup of a worker that is not waiting yet (tiled_sched.inl:181,386)
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
    sched.frame([&](ray r, unsigned x, unsigned y) -> result_record<float>
    {
        result_record<float> result;
        result.color = bg;
        auto hr = closest_hit(r, prims_begin, prims_end);
        result.hit = hr.hit;
        size_t p = size_t(y) * W + x;
        if (!hr.hit) return result;
        prim_id[p] = hr.prim_id;
        tval[p] = hr.t;
        leaf_pos[p] = hr.primitive_list_index;
        hr.isect_pos = r.ori + r.dir * hr.t;
        vec4 clr(1.0f);
        vec3 n = normals[hr.prim_id];
        vec3 uu, vv, w = n;
        make_orthonormal_basis(uu, vv, w);
        uint8_t mask = 0;
        for (int smp = 0; smp < 8; ++smp)
        {
            vec2 sxy = ao_sample(uint32_t(p), smp, frame_num);
            float sz = sqrt(std::max(0.0f, 1.0f - sxy.x * sxy.x - sxy.y * sxy.y));
            auto dir = normalize(sxy.x * uu + sxy.y * vv + sz * w);
            ray ao;
            ao.ori = hr.isect_pos + dir * 1E-3f;
            ao.dir = dir;
            auto ar = any_hit(ao, prims_begin, prims_end, 0.1f);
            ++ao_rays;
            if (ar.hit) { clr = clr - 1.0f / 8; mask |= uint8_t(1u << smp); ++ao_occ; }
        }
        occ[p] = mask;
        result.color = vec4(clr.xyz(), 1.0f);
        return result;
    }, sparams, frame_num);

    write_file(outdir + "/prim_id.bin", prim_id.data(), npx * 4);
    write_file(outdir + "/t.bin", tval.data(), npx * 4);
    write_file(outdir + "/leaf_pos.bin", leaf_pos.data(), npx * 4);
    write_file(outdir + "/occ.bin", occ.data(), npx);
    write_file(outdir + "/color.bin", rt.color(), npx * 16);
    fnv hp, ht, ho, hc;
    uint64_t hits = 0;
    for (size_t p = 0; p < npx; ++p)
    {
        hp.u32(prim_id[p]); ht.u32(fbits(tval[p])); ho.bytes(&occ[p], 1);
        hits += prim_id[p] != 0xFFFFFFFFu;
    }
    hc.bytes(rt.color(), npx * 16);
    printf("{\"scene\":\"%s\",\"W\":%d,\"H\":%d,\"scissor\":[%d,%d,%d,%d],\"frame\":%u,\"bvh_nodes\":[%zu,%zu],"
           "\"hits\":%llu,\"ao_rays\":%llu,\"ao_occluded\":%llu,\"primid_hash\":\"%016llx\",\"t_hash\":\"%016llx\","
           "\"occmask_hash\":\"%016llx\",\"color_hash\":\"%016llx\"}\n",
           d.name.c_str(), W, H, sb[0], sb[1], sb[2], sb[3], frame_num, b0.nodes().size(), b1.nodes().size(),
           (unsigned long long)hits, (unsigned long long)ao_rays.load(), (unsigned long long)ao_occ.load(),
           (unsigned long long)hp.h, (unsigned long long)ht.h, (unsigned long long)ho.h, (unsigned long long)hc.h);
    return 0;
}

//-------------------------------------------------------------------------------------------------
// sampler: the reference's pixel samplers (sched_common.h:160-300 make_primary_rays for uniform,
// jittered and ssaa<2/4/8>; :440-720 sample_pixel_impl: store, blend with 1/frame_num, ssaa's
// store-zero-then-blend) driven pixel by pixel as simple_sched does, with the build's deterministic
// stand-in for the scheduler's clock-seeded random_sampler: the jitter draws of pixel p in frame n
// are U(c), U(c + 1) with c = p * 2 + 0x632BE5AB + n * 0x68E31DA4 (the AO samples keep Appendix A).
// The target starts as `init` everywhere (what jittered_blend blends onto).
//

struct det_sampler
{
    uint32_t c;
    float next() { return U(c++); }
};

template <typename P, typename SamplerT, typename MakeRays>
static int run_sampler_impl(scene_desc const& d, aligned_vector<P>& prims, std::vector<vec3> const& normals,
                            std::string const& outdir, int W, int H, bool do_ao, uint32_t frame_num, SamplerT st,
                            MakeRays make_rays)
{
    auto bvh = build<index_bvh<P>>(prims.data(), prims.size());
    camera cam = make_camera(d, W, H);
    auto f = normalize(cam.eye() - cam.center());
    auto s = normalize(cross(cam.up(), f));
    auto u = cross(f, s);
    vec3 cam_u = s * float(tan(cam.fovy() / 2.0f) * cam.aspect());
    vec3 cam_v = u * float(tan(cam.fovy() / 2.0f));
    vec3 cam_w = -f;
    vec3 eye = cam.eye();

    using bvh_ref = typename index_bvh<P>::bvh_ref;
    std::vector<bvh_ref> bvhs{ bvh.ref() };
    auto prims_begin = bvhs.data();
    auto prims_end = bvhs.data() + bvhs.size();
    const vec4 bg(0.1f, 0.2f, 0.3f, 1.0f);
    const vec4 init(0.25f, 0.5f, 0.75f, 1.0f);
    size_t npx = size_t(W) * H;
    std::vector<uint32_t> prim_id(npx, 0xFFFFFFFFu);    // the last sub-sample's hit
    std::vector<float> tval(npx, -1.0f);
    std::vector<vec4> color(npx, init);
    render_target_ref<PF_RGBA32F> rt_ref(color.data(), nullptr, size_t(W), size_t(H));

    auto kernel = [&](ray r, unsigned x, unsigned y) -> result_record<float>
    {
        result_record<float> result;
        result.color = bg;
        auto hr = closest_hit(r, prims_begin, prims_end);
        result.hit = hr.hit;
        size_t p = size_t(y) * W + x;
        prim_id[p] = hr.hit ? hr.prim_id : 0xFFFFFFFFu;
        tval[p] = hr.hit ? hr.t : -1.0f;
        if (!hr.hit) return result;
        if (!do_ao) { result.color = vec4(1.0f); return result; }
        hr.isect_pos = r.ori + r.dir * hr.t;
        vec4 clr(1.0f);
        vec3 n = normals[hr.prim_id];
        vec3 uu, vv, w = n;
        make_orthonormal_basis(uu, vv, w);
        for (int smp = 0; smp < 8; ++smp)
        {
            vec2 sxy = ao_sample(uint32_t(p), smp, frame_num);
            float sx = sxy.x, sy = sxy.y;
            float sz = sqrt(std::max(0.0f, 1.0f - sx * sx - sy * sy));
            auto dir = normalize(sx * uu + sy * vv + sz * w);
            ray ao;
            ao.ori = hr.isect_pos + dir * 1E-3f;
            ao.dir = dir;
            auto ar = any_hit(ao, prims_begin, prims_end, 0.1f);
            if (ar.hit) clr = clr - 1.0f / 8;
        }
        result.color = vec4(clr.xyz(), 1.0f);
        return result;
    };

    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
        {
            det_sampler samp{ uint32_t(y * W + x) * 2u + 0x632BE5ABu + frame_num * 0x68E31DA4u };
            auto rays = make_rays(samp, unsigned(x), unsigned(y), eye, cam_u, cam_v, cam_w);
            visionaray::detail::sample_pixel_impl(kernel, st, rays, samp, frame_num, rt_ref, x, y, W, H);
        }

    write_file(outdir + "/prim_id.bin", prim_id.data(), npx * 4);
    write_file(outdir + "/t.bin", tval.data(), npx * 4);
    write_file(outdir + "/color.bin", color.data(), npx * 16);
    fnv hp, hc;
    for (size_t p = 0; p < npx; ++p) hp.u32(prim_id[p]);
    hc.bytes(color.data(), npx * 16);
    printf("{\"scene\":\"%s\",\"W\":%d,\"H\":%d,\"frame\":%u,\"primid_hash\":\"%016llx\",\"color_hash\":\"%016llx\"}\n",
           d.name.c_str(), W, H, frame_num, (unsigned long long)hp.h, (unsigned long long)hc.h);
    return 0;
}

template <typename P>
static int run_sampler(scene_desc const& d, aligned_vector<P>& prims, std::vector<vec3> const& normals,
                       std::string const& outdir, int W, int H, bool do_ao, std::string const& kind, uint32_t frame_num,
                       bool matrices = false)
{
    // matrices: the camera given as view / projection matrices (sched_params with MT, scheduler.h:77-95),
    // rays from make_primary_ray_impl's matrix form (sched_common.h:152-176) with the inverses the
    // scheduler computes (cuda_sched.inl:228-235, matrix4.inl:209-244); the matrices are written out
    camera mcam = make_camera(d, W, H);
    const mat4 view = mcam.get_view_matrix(), proj = mcam.get_proj_matrix();
    const mat4 inv_view = inverse(view), inv_proj = inverse(proj);
    if (matrices)
    {
        write_file(outdir + "/view.bin", &view, sizeof(view));
        write_file(outdir + "/proj.bin", &proj, sizeof(proj));
    }
    auto rays_of = [&](auto st)
    {
        return [=](det_sampler& samp, unsigned x, unsigned y, vec3 eye, vec3 cu, vec3 cv, vec3 cw)
        {
            if (matrices)
                return visionaray::detail::make_primary_rays(ray{}, st, samp, x, y, size_t(W), size_t(H), view, inv_view,
                                                             proj, inv_proj);
            return visionaray::detail::make_primary_rays(ray{}, st, samp, x, y, size_t(W), size_t(H), eye, cu, cv, cw);
        };
    };
    if (kind == "uniform")        return run_sampler_impl(d, prims, normals, outdir, W, H, do_ao, frame_num, pixel_sampler::uniform_type{}, rays_of(pixel_sampler::uniform_type{}));
    if (kind == "jittered")       return run_sampler_impl(d, prims, normals, outdir, W, H, do_ao, frame_num, pixel_sampler::jittered_type{}, rays_of(pixel_sampler::jittered_type{}));
    if (kind == "jittered_blend") return run_sampler_impl(d, prims, normals, outdir, W, H, do_ao, frame_num, pixel_sampler::jittered_blend_type{}, rays_of(pixel_sampler::jittered_type{}));
    if (kind == "ssaa2")          return run_sampler_impl(d, prims, normals, outdir, W, H, do_ao, frame_num, pixel_sampler::ssaa_type<2>{}, rays_of(pixel_sampler::ssaa_type<2>{}));
    if (kind == "ssaa4")          return run_sampler_impl(d, prims, normals, outdir, W, H, do_ao, frame_num, pixel_sampler::ssaa_type<4>{}, rays_of(pixel_sampler::ssaa_type<4>{}));
    if (kind == "ssaa8")          return run_sampler_impl(d, prims, normals, outdir, W, H, do_ao, frame_num, pixel_sampler::ssaa_type<8>{}, rays_of(pixel_sampler::ssaa_type<8>{}));
    return 2;
}

//-------------------------------------------------------------------------------------------------
// rsampler: the ao/main.cpp:183-246 kernel verbatim -- random_sampler<float> (random_sampler.h:24-57)
// draws, cosine_sample_hemisphere(samp.next(), samp.next()) (sampling.h:61-71), closest_hit /
// any_hit over the bvh_ref list, get_normal(normals, hit, index_bvh<P>{}, normals_per_face_binding{})
// -- with the per-pixel sampler seeded as hip_sched seeds it (visionaray_hip/hip_kernels.h:
// cuda_sched's cuda_hash(tic() + y * w + x), cuda_sched.inl:20-45, with tic() = frame * W * H).
// The pixel loop is simple_sched's (simple_sched.inl:139-151, kernel form (ray, x, y)); the sampler
// is built per pixel from the seed instead of once per frame from the clock.  Also records draws
// 0, 1, 2 and 15 of every pixel's sampler (a copy, before the kernel draws).
// Built for these fixtures by clang++ (oracle/Makefile vsnray_ref_clang): the order in which the two
// samp.next() arguments are evaluated is the compiler's (g++ right to left, clang and hipcc left to
// right), and the GPU side is compiled by hipcc.
//

static unsigned rs_hash(unsigned a)
{
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}

static int run_rsampler(scene_desc const& d, aligned_vector<tri_t>& prims, std::vector<vec3> const& normals,
                        std::string const& outdir, int W, int H, uint32_t frame_num, int AO_Samples)
{
    using R = ray;
    using S = float;
    using C = vec4;
    using V = vec3;
    auto bvh = build<index_bvh<tri_t>>(prims.data(), prims.size());
    camera cam = make_camera(d, W, H);
    using bvh_ref = index_bvh<tri_t>::bvh_ref;
    std::vector<bvh_ref> bvhs{ bvh.ref() };
    auto prims_begin = bvhs.data();
    auto prims_end = bvhs.data() + bvhs.size();
    const vec4 bgcolor(0.1f, 0.2f, 0.3f, 1.0f);
    const S AO_Radius = 0.1f;
    size_t npx = size_t(W) * H;
    std::vector<float> draws(4 * npx), tval(npx, -1.0f);
    simple_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;
    rt.resize(W, H);
    auto sparams = make_sched_params(pixel_sampler::uniform_type{}, cam, rt);
    simple_sched<R> sched;
    sched.frame([&](R ray, unsigned x, unsigned y) -> result_record<S>
    {
        random_sampler<S> samp(rs_hash(frame_num * unsigned(W) * unsigned(H) + y * unsigned(W) + x));
        size_t p = size_t(y) * W + x;
        {
            random_sampler<S> c = samp;
            float dd[16];
            for (int k = 0; k < 16; ++k) dd[k] = c.next();
            draws[4 * p] = dd[0]; draws[4 * p + 1] = dd[1]; draws[4 * p + 2] = dd[2]; draws[4 * p + 3] = dd[15];
        }
        // ao/main.cpp:185-242
        result_record<S> result;
        result.color = C(bgcolor.xyz(), 1.0f);
        auto hit_rec = closest_hit(ray, prims_begin, prims_end);
        result.hit = hit_rec.hit;
        if (any(hit_rec.hit))
        {
            tval[p] = hit_rec.t;
            hit_rec.isect_pos = ray.ori + ray.dir * hit_rec.t;
            result.isect_pos = hit_rec.isect_pos;
            C clr(1.0);
            auto n = get_normal(normals.data(), hit_rec, index_bvh<tri_t>{}, normals_per_face_binding{});
            V u;
            V v;
            V w = n;
            make_orthonormal_basis(u, v, w);
            S radius = AO_Radius;
            for (int i = 0; i < AO_Samples; ++i)
            {
                auto sp = cosine_sample_hemisphere(samp.next(), samp.next());
                auto dir = normalize(sp.x * u + sp.y * v + sp.z * w);
                R ao_ray;
                ao_ray.ori = hit_rec.isect_pos + dir * S(1E-3f);
                ao_ray.dir = dir;
                auto ao_rec = any_hit(ao_ray, prims_begin, prims_end, radius);
                clr = select(ao_rec.hit, clr - S(1.0f / AO_Samples), clr);
            }
            result.color = select(hit_rec.hit, C(clr.xyz(), S(1.0)), result.color);
        }
        return result;
    }, sparams);
    write_file(outdir + "/draws.bin", draws.data(), draws.size() * 4);
    write_file(outdir + "/t.bin", tval.data(), npx * 4);
    write_file(outdir + "/color.bin", rt.color(), npx * 16);
    fnv hd, ht, hc;
    uint64_t hits = 0;
    for (size_t p = 0; p < npx; ++p) { ht.u32(fbits(tval[p])); hits += tval[p] >= 0.0f; }
    hd.bytes(draws.data(), draws.size() * 4);
    hc.bytes(rt.color(), npx * 16);
    printf("{\"scene\":\"%s\",\"W\":%d,\"H\":%d,\"frame\":%u,\"samples\":%d,\"hits\":%llu,\"draws_hash\":\"%016llx\","
           "\"t_hash\":\"%016llx\",\"color_hash\":\"%016llx\"}\n",
           d.name.c_str(), W, H, frame_num, AO_Samples, (unsigned long long)hits, (unsigned long long)hd.h,
           (unsigned long long)ht.h, (unsigned long long)hc.h);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 3)
    {
        fprintf(stderr, "usage: %s golden <scene> <outdir> [W H]\n"
                        "       %s bench <scene> <threads> <frames> [W H] [samples]\n", argv[0], argv[0]);
        return 2;
    }
    std::string mode = argv[1];
    scene_desc d = lookup(argv[2]);
    if (mode == "golden")
    {
        if (argc < 4) return 2;
        std::string outdir = argv[3];
        int W = argc > 5 ? atoi(argv[4]) : d.W;
        int H = argc > 5 ? atoi(argv[5]) : d.H;
        uint32_t frame_num = argc > 6 ? uint32_t(strtoul(argv[6], nullptr, 10)) : 0u;
        return with_scene(d, [&](auto& prims, std::vector<vec3> const& normals)
        {
            return run_golden(d, prims, normals, outdir, W, H, !d.spheres, default_intersector{}, frame_num);
        });
    }
    if (mode == "shade" || mode == "whitted")
    {
        // shade|whitted <scene> <outdir> <face|vertex> [W H] [bounces eps]
        if (argc < 5 || d.spheres) return 2;
        std::string outdir = argv[3];
        bool per_vertex = std::string(argv[4]) == "vertex";
        int W = argc > 6 ? atoi(argv[5]) : d.W;
        int H = argc > 6 ? atoi(argv[6]) : d.H;
        unsigned bounces = argc > 8 ? unsigned(atoi(argv[7])) : 4u;
        float eps = argc > 8 ? float(atof(argv[8])) : 1e-3f;
        aligned_vector<tri_t> t;
        if (d.grid == 0) make_cornell(t); else if (d.layers) make_hfstack(d.grid, d.layers, t); else make_heightfield(d.grid, t);
        std::vector<vec3> normals(t.size());
        for (size_t i = 0; i < t.size(); ++i) normals[i] = normalize(cross(t[i].e1, t[i].e2));
        return run_shade(d, t, normals, outdir, per_vertex, W, H, mode == "whitted", bounces, eps);
    }
    if (mode == "mask")
    {
        // mask <scene> <outdir> <mask.bin> <mask_w> <mask_h> [W H]: golden frame (primary + AO) with
        // the mask intersector; tex coords = planar (x, z) projection of every corner, written to
        // outdir/tex_coords.bin
        if (argc < 7 || d.spheres) return 2;
        std::string outdir = argv[3];
        int mw = atoi(argv[5]), mh = atoi(argv[6]);
        int W = argc > 8 ? atoi(argv[7]) : d.W;
        int H = argc > 8 ? atoi(argv[8]) : d.H;
        std::vector<uint8_t> mask(size_t(mw) * mh);
        FILE* f = fopen(argv[4], "rb");
        if (!f || fread(mask.data(), 1, mask.size(), f) != mask.size()) { if (f) fclose(f); return 3; }
        fclose(f);
        aligned_vector<tri_t> t;
        if (d.grid == 0) make_cornell(t); else if (d.layers) make_hfstack(d.grid, d.layers, t); else make_heightfield(d.grid, t);
        std::vector<vec3> normals(t.size());
        for (size_t i = 0; i < t.size(); ++i) normals[i] = normalize(cross(t[i].e1, t[i].e2));
        // per prim_id: corners v1, v1 + e1, v1 + e2 -> (x * 0.5 + 0.5, z * 0.5 + 0.5)
        std::vector<vec2> tc(3 * t.size());
        for (auto const& tri : t)
        {
            vec3 c[3] = { tri.v1, tri.v1 + tri.e1, tri.v1 + tri.e2 };
            for (int k = 0; k < 3; ++k) tc[3 * tri.prim_id + k] = vec2(c[k].x * 0.5f + 0.5f, c[k].z * 0.5f + 0.5f);
        }
        write_file(outdir + "/tex_coords.bin", tc.data(), tc.size() * sizeof(vec2));
        mask_intersector isect;
        isect.tex_coords = tc.data();
        isect.mask = mask.data();
        isect.w = mw;
        isect.h = mh;
        return run_golden(d, t, normals, outdir, W, H, true, isect);
    }
    if (mode == "heart")
    {
        // heart <scene> <outdir> [W H]: primary closest hit with the procedural heart cut-out over
        // the planar (x, z) tex coords of the mask mode
        if (argc < 4 || d.spheres) return 2;
        std::string outdir = argv[3];
        int W = argc > 5 ? atoi(argv[4]) : d.W;
        int H = argc > 5 ? atoi(argv[5]) : d.H;
        aligned_vector<tri_t> t;
        if (d.grid == 0) make_cornell(t); else if (d.layers) make_hfstack(d.grid, d.layers, t); else make_heightfield(d.grid, t);
        std::vector<vec3> normals(t.size());
        for (size_t i = 0; i < t.size(); ++i) normals[i] = normalize(cross(t[i].e1, t[i].e2));
        std::vector<vec2> tc(3 * t.size());
        for (auto const& tri : t)
        {
            vec3 c[3] = { tri.v1, tri.v1 + tri.e1, tri.v1 + tri.e2 };
            for (int k = 0; k < 3; ++k) tc[3 * tri.prim_id + k] = vec2(c[k].x * 0.5f + 0.5f, c[k].z * 0.5f + 0.5f);
        }
        heart_intersector isect;
        isect.tex_coords = tc.data();
        return run_golden(d, t, normals, outdir, W, H, false, isect);
    }
    if (mode == "list")
    {
        // list <scene> <outdir> <W> <H> <x0> <y0> <x1> <y1> <frame>: BVH-ref lists + scissor box
        if (argc < 11 || d.spheres) return 2;
        std::string outdir = argv[3];
        int W = atoi(argv[4]), H = atoi(argv[5]);
        int sb[4] = { atoi(argv[6]), atoi(argv[7]), atoi(argv[8]), atoi(argv[9]) };
        uint32_t frame_num = uint32_t(strtoul(argv[10], nullptr, 10));
        aligned_vector<tri_t> t;
        if (d.grid == 0) make_cornell(t); else if (d.layers) make_hfstack(d.grid, d.layers, t); else make_heightfield(d.grid, t);
        return run_list(d, t, outdir, W, H, sb, frame_num);
    }
    if (mode == "sah")
    {
        // sah_cost (detail/bvh/statistics.h:30-73) of the reference's own tree
        return with_scene(d, [&](auto& prims, std::vector<vec3> const&)
        {
            using P = typename std::decay<decltype(prims[0])>::type;
            auto bvh = build<index_bvh<P>>(prims.data(), prims.size());
            uint32_t bits;
            float c = sah_cost(bvh);
            std::memcpy(&bits, &c, 4);
            printf("{\"scene\":\"%s\",\"sah_cost\":%.9g,\"sah_cost_bits\":\"%08x\"}\n", d.name.c_str(), c, bits);
            return 0;
        });
    }
    if (mode == "multi")
    {
        if (argc < 5 || d.spheres) return 2;
        std::string outdir = argv[3];
        bool per_vertex = std::string(argv[4]) == "vertex";
        int W = argc > 6 ? atoi(argv[5]) : d.W;
        int H = argc > 6 ? atoi(argv[6]) : d.H;
        aligned_vector<tri_t> t;
        if (d.grid == 0) make_cornell(t); else if (d.layers) make_hfstack(d.grid, d.layers, t); else make_heightfield(d.grid, t);
        std::vector<vec3> normals(t.size());
        for (size_t i = 0; i < t.size(); ++i) normals[i] = normalize(cross(t[i].e1, t[i].e2));
        return run_multi(d, t, normals, outdir, per_vertex, W, H);
    }
    if (mode == "sampler")
    {
        // sampler <scene> <outdir> <uniform|jittered|jittered_blend|ssaa2|ssaa4|ssaa8>[+matrix] <primary|ao> <frame> [W H]
        if (argc < 7) return 2;
        std::string outdir = argv[3], kind = argv[4];
        bool matrices = false;
        if (kind.size() > 7 && kind.substr(kind.size() - 7) == "+matrix") { matrices = true; kind.resize(kind.size() - 7); }
        bool do_ao = std::string(argv[5]) == "ao" && !d.spheres;
        uint32_t frame_num = uint32_t(strtoul(argv[6], nullptr, 10));
        int W = argc > 8 ? atoi(argv[7]) : d.W;
        int H = argc > 8 ? atoi(argv[8]) : d.H;
        return with_scene(d, [&](auto& prims, std::vector<vec3> const& normals)
        {
            return run_sampler(d, prims, normals, outdir, W, H, do_ao, kind, frame_num, matrices);
        });
    }
    if (mode == "rsampler")
    {
        // rsampler <scene> <outdir> <W> <H> <frame> [samples]: the AO example's kernel with per-pixel
        // seeded random_sampler<float> (triangle scenes)
        if (argc < 7 || d.spheres) return 2;
        std::string outdir = argv[3];
        int W = atoi(argv[4]), H = atoi(argv[5]);
        uint32_t frame_num = uint32_t(strtoul(argv[6], nullptr, 10));
        int samples = argc > 7 ? atoi(argv[7]) : 8;
        aligned_vector<tri_t> t;
        if (d.grid == 0) make_cornell(t); else if (d.layers) make_hfstack(d.grid, d.layers, t); else make_heightfield(d.grid, t);
        std::vector<vec3> normals(t.size());
        for (size_t i = 0; i < t.size(); ++i) normals[i] = normalize(cross(t[i].e1, t[i].e2));
        return run_rsampler(d, t, normals, outdir, W, H, frame_num, samples);
    }
    if (mode == "bench")
    {
        int threads = argc > 3 ? atoi(argv[3]) : int(std::thread::hardware_concurrency());
        int frames = argc > 4 ? atoi(argv[4]) : 5;
        int W = argc > 6 ? atoi(argv[5]) : d.W;
        int H = argc > 6 ? atoi(argv[6]) : d.H;
        int samples = argc > 7 ? atoi(argv[7]) : (d.spheres ? 0 : 8);
        return with_scene(d, [&](auto& prims, std::vector<vec3> const& normals)
        {
            return run_bench(d, prims, normals, threads, frames, W, H, samples);
        });
    }
    return 2;
}
