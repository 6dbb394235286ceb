// visionaray_amd/csrc/vrh_shade.h -- built-in shading on top of the traversal.
//
// simple::kernel (detail/simple.inl:19-83) for triangles with plastic<float> materials indexed by
// geom_id and point lights: ambient term, two-sided shading normal, one plastic::shade per light.
// Operation order is the reference's, expression by expression, compiled like the traversal with
// -ffp-contract=off and IEEE division / sqrt; the attenuation division is in double as in
// point_light.inl:20-25.  The one libm call, powf (blinn specular, brdf.h:111-122), is the device
// library's: it can differ from the host libm in the last bit, so radiance is compared with a
// relative tolerance (north star: 1e-5) while hit ids stay bit-exact.
#pragma once

#include "visionaray_hip/detail/vrh_device.h"

namespace vrh {
namespace dev {

// device copies of vrh_plastic / vrh_point_light (include/vrh.h), 4-byte fields
struct plastic_t { float ca[3]; float ka; float cd[3]; float kd; float cs[3]; float ks; float exp; };
struct point_light_t { float position[3]; float cl[3]; float kl; float constant_att, linear_att, quadratic_att; };

struct shade_params
{
    const plastic_t* materials;
    const point_light_t* lights;
    uint32_t num_lights;
    uint32_t per_vertex;          // normals_per_vertex_binding
    const float4* vnormals;       // 3 per prim_id
    float ambient[4];
    float amb[3];                 // ambient[i] * ambient[3], computed on the host (the same IEEE products)
};

__device__ __forceinline__ f3 neg(f3 a) { return mk3(-a.x, -a.y, -a.z); }

struct surface_t { f3 gn, sn; plastic_t m; uint32_t mi; };

// get_surface (get_surface.h:336-376, 576-592) for a triangle hit: normals by binding, material by
// the primitive's geom_id
__device__ inline surface_t get_surface(const shade_params& S, const float4* __restrict__ prims,
                                        const float4* __restrict__ normals, uint32_t prim_id, uint32_t li,
                                        float u, float v)
{
    surface_t sf;
    const float4* q = prims + 3u * li;
    const float4 qb = q[1], qc = q[2];
    sf.mi = __float_as_uint(qc.z);
    sf.m = S.materials[sf.mi];
    if (!S.per_vertex)
    {
        const float4 nn = normals[prim_id];                            // get_normal.h:26-37
        sf.gn = sf.sn = mk3(nn.x, nn.y, nn.z);
    }
    else
    {
        // geometric normal of primitive(list_index) (get_normal.h:110-116), shading normal
        // lerp(n0, n1, n2, u, v) (get_shading_normal.h:64-84, math.h:466-475)
        const float4 qa = q[0];
        const f3 e1 = mk3(qa.w, qb.x, qb.y), e2 = mk3(qb.z, qb.w, qc.x);
        sf.gn = normalize(cross(e1, e2));
        const float4 a = S.vnormals[3u * prim_id], b = S.vnormals[3u * prim_id + 1u], c = S.vnormals[3u * prim_id + 2u];
        const f3 s2 = mk3(c.x, c.y, c.z) * v;
        const f3 s3 = mk3(b.x, b.y, b.z) * u;
        const f3 s1 = mk3(a.x, a.y, a.z) * (1.0f - (u + v));
        sf.sn = normalize((s1 + s2) + s3);
    }
    return sf;
}

// plastic::shade (plastic.inl:21-37) for one point light: pi * (lambertian + blinn) * intensity * ndotl
__device__ inline f3 plastic_shade(const plastic_t& m, f3 n, f3 wo, f3 pos, const point_light_t& L)
{
    constexpr float PI = 3.14159265358979323846264338328e+00f;      // math.h:240 constants::pi
    constexpr float INV_PI = 3.18309886183790691216444201928e-01f;  // math.h:242 constants::inv_pi
    const f3 lpos = mk3(L.position[0], L.position[1], L.position[2]);
    const f3 wi = normalize(lpos - pos);                                // simple.inl:59
    const float ndotl = tmax(0.0f, dot(n, wi));                        // plastic.inl:29
    const f3 cd = (mk3(m.cd[0], m.cd[1], m.cd[2]) * m.kd) * INV_PI;    // lambertian::f, brdf.h:36-41
    // blinn::f, brdf.h:111-122
    const f3 h = normalize(wo + wi);
    const float hdotn = tmax(0.0f, dot(h, n));
    const f3 spec = mk3(m.cs[0], m.cs[1], m.cs[2]) * m.ks;
    const float sat = tmax(0.0f, tmin(dot(wi, h), 1.0f));              // saturate, math.h:454-457
    const float p5 = __builtin_powf(1.0f - sat, 5.0f);
    const f3 schlick = spec + mk3(1.0f - spec.x, 1.0f - spec.y, 1.0f - spec.z) * p5;
    const float nfactor = (m.exp + 2.0f) / (8.0f * PI);
    const f3 bl = (schlick * nfactor) * __builtin_powf(hdotn, m.exp);
    // point_light::intensity, point_light.inl:12-28
    const f3 dv = lpos - pos;
    const float dist = __builtin_sqrtf(dot(dv, dv));
    const float den = L.constant_att + L.linear_att * dist + L.quadratic_att * dist * dist;
    const float att = (float)(1.0 / (double)den);
    const f3 I = (mk3(L.cl[0], L.cl[1], L.cl[2]) * L.kl) * att;
    return ((PI * (cd + bl)) * I) * ndotl;
}

// colour of a closest hit, simple.inl:32-69 (the miss colour is the caller's)
__device__ inline float4 shade_simple(const shade_params& S, const float4* __restrict__ prims,
                                      const float4* __restrict__ normals, const ray_t& r, float t,
                                      uint32_t prim_id, const hit_extra& hx)
{
    const f3 pos = r.ori + r.dir * t;                                  // simple.inl:37
    const surface_t sf = get_surface(S, prims, normals, prim_id, hx.li, hx.u, hx.v);
    // plastic.inl:13-16 ambient() = ca * ka, times from_rgba(ambient_color) (spectrum.inl:375-378)
    const f3 amb = mk3(S.amb[0], S.amb[1], S.amb[2]);
    f3 shaded = (mk3(sf.m.ca[0], sf.m.ca[1], sf.m.ca[2]) * sf.m.ka) * amb;
    const f3 view = neg(r.dir);
    const f3 n = dot(sf.gn, view) < 0.0f ? neg(sf.sn) : sf.sn;       // faceforward, vector.inl:674-681
    for (uint32_t li = 0; li < S.num_lights; ++li)
        shaded = shaded + plastic_shade(sf.m, n, view, pos, S.lights[li]);   // simple.inl:63
    return make_float4(shaded.x, shaded.y, shaded.z, 1.0f);           // to_rgba
}

// whitted::kernel (detail/whitted.inl:186-277) as a per-lane state machine: a closest-hit ray
// (primary or reflection) that hits sets up the surface, then one any-hit shadow ray per light
// (max_t = distance to the light), then the reflection ray of the plastic fall-through bounce
// (reflect(view, shading normal), kr = 0.1, whitted.inl:64-77).  The lane keeps what the loop body
// carries between those rays.  The bounce's surface (isect_pos, two-sided shading normal,
// view_dir, shaded_clr: 12 words) is read only when a ray of the bounce ends, so it lives in LDS
// after the traversal stack ([word][lane], conflict-free), not in registers: the kernel then fits
// 96 VGPRs without spills, 5 waves / SIMD instead of 4 at 124.
struct whitted_lane
{
    f3 color;        // accumulated radiance (`color`)
    float thr;       // throughput
    uint32_t depth;  // loop iterations entered
    uint32_t li;     // light of the shadow ray in flight
    uint32_t mi;     // material (geom_id)
    uint32_t shadow; // 1 while a shadow ray is traced
    float* sm;       // LDS base of the surface words: word k of this lane at sm[base + k * stride]
    uint32_t base, stride;
    __device__ __forceinline__ float& at(uint32_t k) const { return sm[base + k * stride]; }
    __device__ __forceinline__ f3 ld3(uint32_t k) const { return mk3(at(k), at(k + 1u), at(k + 2u)); }
    __device__ __forceinline__ void st3(uint32_t k, f3 v) const { at(k) = v.x; at(k + 1u) = v.y; at(k + 2u) = v.z; }
};
constexpr uint32_t WL_POS = 0, WL_N = 3, WL_VIEW = 6, WL_SHADED = 9, WL_WORDS = 12;   // LDS words per lane

// loop body up to the light loop (whitted.inl:225-233), for a hit at t of ray r
__device__ inline void whitted_surface(const shade_params& S, const float4* __restrict__ prims,
                                       const float4* __restrict__ normals, whitted_lane& w, const ray_t& r, float t,
                                       uint32_t prim_id, const hit_extra& hx)
{
    w.st3(WL_POS, r.ori + r.dir * t);
    const surface_t sf = get_surface(S, prims, normals, prim_id, hx.li, hx.u, hx.v);
    w.mi = sf.mi;
    const f3 amb = mk3(S.amb[0], S.amb[1], S.amb[2]);
    w.st3(WL_SHADED, (mk3(sf.m.ca[0], sf.m.ca[1], sf.m.ca[2]) * sf.m.ka) * amb);
    const f3 view = neg(r.dir);
    w.st3(WL_VIEW, view);
    w.st3(WL_N, dot(sf.gn, view) < 0.0f ? neg(sf.sn) : sf.sn);      // faceforward
    w.li = 0;
}

// specular_bounce(plastic) = reflect(view_dir, shading_normal): 2 * dot(n, i) * n - i
// (vector.inl:683-689, whitted.inl:262) with the un-flipped shading normal sn.  Computed from the
// stored two-sided normal n = +-sn: dot(-sn, v) = -dot(sn, v) and (-d) * (-x) = d * x exactly under
// round-to-nearest, so the result is bit-identical.
__device__ inline f3 whitted_reflect(const whitted_lane& w)
{
    const f3 n = w.ld3(WL_N), view = w.ld3(WL_VIEW);
    const float d2 = 2.0f * dot(n, view);
    return mk3(d2 * n.x, d2 * n.y, d2 * n.z) - view;
}

// shadow ray of light w.li (whitted.inl:237-252): origin pushed along the light direction, any hit
// closer than the light
__device__ inline ray_t whitted_shadow_ray(const shade_params& S, const whitted_lane& w, float eps, float& max_t)
{
    const point_light_t& L = S.lights[w.li];
    const f3 lpos = mk3(L.position[0], L.position[1], L.position[2]);
    const f3 pos = w.ld3(WL_POS);
    const f3 ldir = normalize(lpos - pos);
    const f3 dv = pos - lpos;
    max_t = __builtin_sqrtf(dot(dv, dv));                              // length(isect_pos - position)
    return make_ray(pos + ldir * eps, ldir);
}

// a shadow ray ended: add the light's plastic::shade unless occluded (select(active, clr, 0))
__device__ inline void whitted_light_done(const shade_params& S, whitted_lane& w, bool occluded)
{
    const f3 c = occluded ? mk3(0.0f, 0.0f, 0.0f)
               : plastic_shade(S.materials[w.mi], w.ld3(WL_N), w.ld3(WL_VIEW), w.ld3(WL_POS), S.lights[w.li]);
    w.st3(WL_SHADED, w.ld3(WL_SHADED) + c);
    w.li += 1u;
}

// per-lane sorted hit list of multi_hit<N> in LDS, column-major [field][entry][lane]
struct mh_list
{
    uint32_t* mem;
    uint32_t base;       // lane's word offset of field 0, entry 0
    uint32_t stride;     // words between consecutive entries (= threads per block)
    uint32_t n;          // N
    __device__ __forceinline__ uint32_t& at(uint32_t field, uint32_t k) const { return mem[base + (field * n + k) * stride]; }
    __device__ __forceinline__ float t(uint32_t k) const { return __uint_as_float(at(0, k)); }
    __device__ __forceinline__ void reset() const
    {
        for (uint32_t k = 0; k < n; ++k) { at(0, k) = __float_as_uint(FMAX); at(1, k) = 0xFFFFFFFFu; }
    }
    // insert_sorted (algorithm.h:46-75) with is_closer_t (update_if.h:48-56): the first entry whose
    // t is larger takes the hit, later entries shift down, the last one drops out.  Returns the
    // new N-th t (the culling distance of multi_hit, multi_hit.h:221-244).
    __device__ __forceinline__ float insert(float t_new, uint32_t pid, uint32_t li, float u, float v) const
    {
        uint32_t pos = n - 1u;
        for (uint32_t k = 0; k < n; ++k)
            if (t_new < t(k)) { pos = k; break; }
        for (uint32_t k = n - 1u; k > pos; --k)
            for (uint32_t f = 0; f < 5u; ++f) at(f, k) = at(f, k - 1u);
        at(0, pos) = __float_as_uint(t_new); at(1, pos) = pid; at(2, pos) = li;
        at(3, pos) = __float_as_uint(u); at(4, pos) = __float_as_uint(v);
        return t(n - 1u);
    }
};

// examples/multi_hit/main.cpp:178-235: every kept hit (t order) shaded with the first light,
// alpha 0.3, composited front to back; colour starts at 0
__device__ inline float4 shade_multi(const shade_params& S, const float4* __restrict__ prims,
                                     const float4* __restrict__ normals, const ray_t& r, const mh_list& L)
{
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (uint32_t k = 0; k < L.n; ++k)
    {
        const float t = L.t(k);
        if (!(t < FMAX)) break;
        const f3 pos = r.ori + r.dir * t;
        const surface_t sf = get_surface(S, prims, normals, L.at(1, k), L.at(2, k), __uint_as_float(L.at(3, k)),
                                         __uint_as_float(L.at(4, k)));
        const f3 view = neg(r.dir);
        const f3 n = dot(sf.gn, view) < 0.0f ? neg(sf.sn) : sf.sn;
        f3 c = S.num_lights ? plastic_shade(sf.m, n, view, pos, S.lights[0]) : mk3(0.0f, 0.0f, 0.0f);
        const float a = 0.3f;
        c = c * a;
        const float f = 1.0f - acc.w;
        acc = make_float4(acc.x + c.x * f, acc.y + c.y * f, acc.z + c.z * f, acc.w + a * f);
    }
    return acc;
}

} // namespace dev
} // namespace vrh
