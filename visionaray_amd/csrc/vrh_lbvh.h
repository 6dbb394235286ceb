// visionaray_amd/csrc/vrh_lbvh.h -- GPU BVH construction interface (vrh_lbvh.hip).
#pragma once

#include "vrh_internal.h"

#include <hip/hip_runtime.h>
#include <string>

namespace vrh {

struct lbvh_out
{
    node32* nodes = nullptr;      // device, reference bvh_node layout, num_nodes entries
    uint32_t* indices = nullptr;  // device, index array (sorted original primitive indices)
    float4* pairs = nullptr;      // device pair records (vrh_device.h)
    float4* prims = nullptr;      // device leaf-ordered primitives with END flags
    uint32_t num_nodes = 0, num_pairs = 0, root = 0, max_depth = 0;
    uint32_t max_prim_id = 0, max_geom_id = 0;
    bool finite = true;
    float build_ms = 0.0f;        // device time of the build kernels (after the primitive upload)
};

// builds a linear BVH over host primitives (reference layouts) on the stream's device; on success
// the caller owns every pointer in `out`
int build_lbvh(const void* prims_host, uint32_t n, uint32_t kind, uint32_t max_leaf, hipStream_t stream,
               lbvh_out& out, std::string& err);

} // namespace vrh
