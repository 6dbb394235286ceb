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

#include "vrh_device.h"

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
};

__device__ __forceinline__ f3 neg(f3 a) { return mk3(-a.x, -a.y, -a.z); }

// colour of a closest hit, simple.inl:32-69 (the miss colour is the caller's)
__device__ inline float4 shade_simple(const shade_params& S, const float4* __restrict__ prims,
                                      const float4* __restrict__ normals, const ray_t& r, float t,
                                      uint32_t prim_id, const hit_extra& hx)
{
    constexpr float PI = 3.14159265358979323846264338328e+00f;      // math.h:240 constants::pi
    constexpr float INV_PI = 3.18309886183790691216444201928e-01f;  // math.h:242 constants::inv_pi
    const f3 pos = r.ori + r.dir * t;                                  // simple.inl:37
    const float4* q = prims + 3u * hx.li;
    const float4 qb = q[1], qc = q[2];
    const uint32_t geom_id = __float_as_uint(qc.z);
    f3 gn, sn;
    if (!S.per_vertex)
    {
        const float4 nn = normals[prim_id];                            // get_normal.h:26-37
        gn = sn = mk3(nn.x, nn.y, nn.z);
    }
    else
    {
        // get_surface.h:336-376: geometric normal of primitive(list_index) (get_normal.h:110-116),
        // shading normal lerp(n0, n1, n2, u, v) (get_shading_normal.h:64-84, math.h:466-475)
        const float4 qa = q[0];
        const f3 e1 = mk3(qa.w, qb.x, qb.y), e2 = mk3(qb.z, qb.w, qc.x);
        gn = normalize(cross(e1, e2));
        const float4 a = S.vnormals[3u * prim_id], b = S.vnormals[3u * prim_id + 1u], c = S.vnormals[3u * prim_id + 2u];
        const f3 s2 = mk3(c.x, c.y, c.z) * hx.v;
        const f3 s3 = mk3(b.x, b.y, b.z) * hx.u;
        const f3 s1 = mk3(a.x, a.y, a.z) * (1.0f - (hx.u + hx.v));
        sn = normalize((s1 + s2) + s3);
    }
    const plastic_t m = S.materials[geom_id];
    // plastic.inl:13-16 ambient() = ca * ka, times from_rgba(ambient_color) (spectrum.inl:375-378)
    const f3 amb = mk3(S.ambient[0] * S.ambient[3], S.ambient[1] * S.ambient[3], S.ambient[2] * S.ambient[3]);
    f3 shaded = (mk3(m.ca[0], m.ca[1], m.ca[2]) * m.ka) * amb;
    const f3 view = neg(r.dir);
    const f3 n = dot(gn, view) < 0.0f ? neg(sn) : sn;                 // faceforward, vector.inl:674-681
    const f3 cd = (mk3(m.cd[0], m.cd[1], m.cd[2]) * m.kd) * INV_PI;  // lambertian::f, brdf.h:36-41
    const f3 spec = mk3(m.cs[0], m.cs[1], m.cs[2]) * m.ks;
    const float nfactor = (m.exp + 2.0f) / (8.0f * PI);
    for (uint32_t li = 0; li < S.num_lights; ++li)
    {
        const point_light_t L = S.lights[li];
        const f3 lpos = mk3(L.position[0], L.position[1], L.position[2]);
        const f3 wi = normalize(lpos - pos);                            // simple.inl:59
        const f3 wo = view;
        const float ndotl = tmax(0.0f, dot(n, wi));                    // plastic.inl:29
        // blinn::f, brdf.h:111-122
        const f3 h = normalize(wo + wi);
        const float hdotn = tmax(0.0f, dot(h, n));
        const float sat = tmax(0.0f, tmin(dot(wi, h), 1.0f));          // saturate, math.h:454-457
        const float p5 = __builtin_powf(1.0f - sat, 5.0f);
        const f3 schlick = spec + mk3(1.0f - spec.x, 1.0f - spec.y, 1.0f - spec.z) * p5;
        const f3 bl = (schlick * nfactor) * __builtin_powf(hdotn, m.exp);
        // point_light::intensity, point_light.inl:12-28
        const f3 dv = lpos - pos;
        const float dist = __builtin_sqrtf(dot(dv, dv));
        const float den = L.constant_att + L.linear_att * dist + L.quadratic_att * dist * dist;
        const float att = (float)(1.0 / (double)den);
        const f3 I = (mk3(L.cl[0], L.cl[1], L.cl[2]) * L.kl) * att;
        // plastic::shade, plastic.inl:21-37: pi * (cd + blinn) * intensity * ndotl
        const f3 clr = ((PI * (cd + bl)) * I) * ndotl;
        shaded = shaded + clr;                                          // simple.inl:63
    }
    return make_float4(shaded.x, shaded.y, shaded.z, 1.0f);           // to_rgba
}

} // namespace dev
} // namespace vrh
