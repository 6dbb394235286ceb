// visionaray_amd/csrc/vrh_internal.h -- shared host-side declarations of libvrh.
#pragma once

#include "../../include/vrh.h"

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace vrh {

// Reference binary layouts
struct node32                                     // bvh_node, bvh.h:52-119
{
    float    bmin[3];
    uint32_t first;                               // first_child (inner) | first_prim (leaf)
    float    bmax[3];
    uint32_t num_prims;                           // 0 = inner
};
struct tri64                                      // basic_triangle<3,float>
{
    uint32_t geom_id, prim_id, pad[2];
    float    v1[4], e1[4], e2[4];
};
struct sphere48                                   // basic_sphere<float>
{
    uint32_t geom_id, prim_id, pad[2];
    float    center[4];
    float    radius, pad2[3];
};
static_assert(sizeof(node32) == 32, "node layout");
static_assert(sizeof(tri64) == 64, "triangle layout");
static_assert(sizeof(sphere48) == 48, "sphere layout");

void set_error(const std::string& msg);

constexpr uint32_t QUAD_NONE = 0xFFFFFFFFu;     // unused entry of a 4-wide record

// 4-wide any-hit records from the binary BVH (vrh_quad.cpp); false = the scene keeps the binary
// path (containment or box validity does not hold, or the root is a leaf)
bool build_quads(const node32* nodes, uint32_t num_nodes, std::vector<float>& out, uint32_t& root_link,
                 uint32_t& quad_depth);

int build_bvh(const void* prims, uint32_t n, uint32_t kind, node32* nodes_out, uint32_t* num_nodes_out,
              uint32_t* indices_out, uint32_t* max_depth_out);

} // namespace vrh
