// include/visionaray_hip/obj_loader.h -- drop-in for src/common/obj_loader.h (load_obj), without Boost.
//
//   #include <common/model.h>                  // the reference's model (model.h:20-49), or
//   #include <visionaray_hip/standalone.h>     // visionaray::model without the Visionaray headers
//   #include <visionaray_hip/obj_loader.h>     // instead of <common/obj_loader.h>
//
//   visionaray::model mod;
//   visionaray::load_obj(filename, mod);       // obj_loader.cpp:299-527, parsed by libvrh (vrh_obj_load)
//
// Fills mod.primitives, shading_normals, geometric_normals, tex_coords, materials and bbox with what
// the reference's loader stores there (appending, as the reference does).  Textures are not loaded:
// mod.texture_map / textures stay untouched.  Errors throw hip_error (the reference throws from
// boost::iostreams on an unreadable file).
#pragma once

#include "hip_backend.h"

#include <cstdint>
#include <string>
#include <type_traits>
#include <vector>

namespace visionaray
{

namespace hip_detail
{
// vrh_plastic -> the model's material_type: plastic<float> through its setters (material.h:297-316)
// with from_rgb (spectrum.inl:331-369), or a vrh_plastic record as is
inline void assign_material(vrh_plastic& dst, vrh_plastic const& src, void*) { dst = src; }

template <typename M, typename Vec3>
auto assign_material(M& dst, vrh_plastic const& s, Vec3*)
    -> decltype(dst.set_specular_exp(s.exp), void())
{
    dst.set_ca(from_rgb(Vec3(s.ca[0], s.ca[1], s.ca[2])));   // Vec3 makes the call dependent (ADL)
    dst.set_ka(s.ka);
    dst.set_cd(from_rgb(Vec3(s.cd[0], s.cd[1], s.cd[2])));
    dst.set_kd(s.kd);
    dst.set_cs(from_rgb(Vec3(s.cs[0], s.cs[1], s.cs[2])));
    dst.set_ks(s.ks);
    dst.set_specular_exp(s.exp);
}

struct obj_handle
{
    vrh_obj* h = nullptr;
    ~obj_handle() { if (h) vrh_obj_free(h); }
};

struct obj_triangle_record                  // TRI64 (include/vrh.h)
{
    uint32_t geom_id, prim_id, pad[2];
    float v1[4], e1[4], e2[4];
};
} // hip_detail

template <typename Model>
void load_obj(std::string const& filename, Model& mod)
{
    using triangle_type = typename Model::triangle_type;
    using normal_type = typename Model::normal_type;
    using tex_coord_type = typename Model::tex_coord_type;
    using material_type = typename std::decay<decltype(mod.materials[0])>::type;

    hip_detail::obj_handle obj;
    hip_detail::check(vrh_obj_load(filename.c_str(), &obj.h), "vrh_obj_load");
    vrh_obj_info info;
    hip_detail::check(vrh_obj_get_info(obj.h, &info), "vrh_obj_get_info");

    std::vector<hip_detail::obj_triangle_record> tris(info.num_triangles);
    std::vector<float> gn(4 * size_t(info.num_triangles)), sn(4 * size_t(info.num_shading_normals));
    std::vector<float> tc(2 * size_t(info.num_tex_coords));
    std::vector<vrh_plastic> mats(info.num_materials);
    hip_detail::check(vrh_obj_get_data(obj.h, tris.data(), gn.data(), sn.data(), tc.data(), mats.data()),
                      "vrh_obj_get_data");

    for (auto const& r : tris)
    {
        triangle_type t;
        t.v1 = normal_type(r.v1[0], r.v1[1], r.v1[2]);
        t.e1 = normal_type(r.e1[0], r.e1[1], r.e1[2]);
        t.e2 = normal_type(r.e2[0], r.e2[1], r.e2[2]);
        t.prim_id = r.prim_id;
        t.geom_id = r.geom_id;
        mod.primitives.push_back(t);
    }
    for (size_t i = 0; i < info.num_shading_normals; ++i)
        mod.shading_normals.push_back(normal_type(sn[4 * i], sn[4 * i + 1], sn[4 * i + 2]));
    for (size_t i = 0; i < info.num_triangles; ++i)
        mod.geometric_normals.push_back(normal_type(gn[4 * i], gn[4 * i + 1], gn[4 * i + 2]));
    for (size_t i = 0; i < info.num_tex_coords; ++i)
        mod.tex_coords.push_back(tex_coord_type(tc[2 * i], tc[2 * i + 1]));
    for (auto const& p : mats)
    {
        material_type m;
        hip_detail::assign_material(m, p, static_cast<normal_type*>(nullptr));
        mod.materials.push_back(m);
    }
    mod.bbox = decltype(mod.bbox)(normal_type(info.bbox_min[0], info.bbox_min[1], info.bbox_min[2]),
                                  normal_type(info.bbox_max[0], info.bbox_max[1], info.bbox_max[2]));
}

} // visionaray
