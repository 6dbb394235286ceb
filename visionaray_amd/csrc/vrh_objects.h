// visionaray_amd/csrc/vrh_objects.h -- the opaque objects of the C-ABI (include/vrh.h), shared by
// the runtime (vrh_runtime.hip) and the multi-GPU render groups (vrh_group.hip).
#pragma once

#include "vrh_internal.h"
#include "vrh_kernels.h"

#include <hip/hip_runtime.h>

#include <vector>

struct vrh_ctx
{
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int num_cus = 0;
    // the `written` events of this context's targets that a render group's root wrote (one per target,
    // re-recorded by every unshard): vrh_sync waits for all of them (two groups may write two targets)
    std::vector<hipEvent_t> group_written;
    // device counters (u64), see render_params::counters; [0..7] reset per frame
    unsigned long long* counters = nullptr;
    uint32_t* user_queues = nullptr;            // vrh_ctx_user_queues (8 heads x 64 B)
    unsigned long long* tile_times = nullptr;   // VRH_OPT_WAVE_TIMES = 2 (counting kernels): 3 per tile
    size_t tile_times_n = 0, tile_times_used = 0;
    unsigned long long* wave_times = nullptr;   // VRH_OPT_WAVE_TIMES buffer (2 per resident wave)
    size_t wave_times_n = 0, wave_times_used = 0;
    void* spill = nullptr;          // traversal stack overflow blocks (vrh_render_batch), grown on demand
    size_t spill_bytes = 0;
    // one hipEvent pair per frame since vrh_stats_reset (ring of VRH_MAX_TIMED_FRAMES)
    std::vector<hipEvent_t> ev_start, ev_stop;
    uint32_t frames = 0;
    uint32_t last_slot = 0;
    vrh_frame_stats last{};
    bool have_frame = false;
    // asynchronous frames (VRH_OPT_ASYNC_FRAMES, cuda_sched's issue model, cuda_sched.inl:306-320):
    // frames go round robin over `num_lanes` frame lanes (streams of their own; 2-4, VRH_OPT_ASYNC_FRAMES),
    // so frame k + 1's waves take the CUs that frame k's launch tail leaves idle.  Each lane has its own counter block and stack
    // overflow block; a target written by the other lane is rendered into the lane's scratch target
    // and copied in issue order (vrh_runtime.hip issue_async).  Work on `stream` joins the lanes
    // first (ctx_join): it waits for every frame issued so far.
    struct lane_t
    {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;              // recorded after every frame issued on this lane
        bool used = false;
        unsigned long long* counters = nullptr; // COUNTERS_WORDS words of the counter allocation
        void* spill = nullptr;
        size_t spill_bytes = 0;
        // scratch target (primary / AO frames into a target the other lane still writes)
        float4* color = nullptr;
        uint32_t* prim_id = nullptr;
        float* t = nullptr;
        uint8_t* occ = nullptr;
        size_t pixels = 0;
        // the frame in the scratch target whose copy into `pending_rt` is not issued yet: a later frame
        // into that target writing the same fields over at least the same box drops it (only the last
        // frame's pixels are ever seen), anything else issues it first (ctx_flush_pending)
        vrh_rt* pending_rt = nullptr;
        uint32_t pending_clip[4] = {};
        bool pending_fields[4] = {};      // colour, prim id, t, occlusion
    } lane[vrh::VRH_MAX_FRAME_LANES];
    uint32_t next_lane = 0;
    uint32_t num_lanes = 2;                     // frame lanes in use (VRH_OPT_ASYNC_FRAMES)
    hipEvent_t main_mark = nullptr;             // position of `stream` that an async frame waits for
    mutable uint64_t join_epoch = 0;            // incremented by every join of the lanes into `stream`
    unsigned long long* last_counters = nullptr;    // counter block of the last frame (vrh_last_frame_stats)
    // tuning options (0 = automatic), vrh_ctx_set_option
    int opt_async = 0;
    int opt_block = 0, opt_stack = 0, opt_sched = 0, opt_refill = 0, opt_dcap = 0, opt_bpc = 0, opt_occ = 0, opt_exact_minmax = 0, opt_xcd_queues = 0, opt_wide = 0, opt_pop = 0, opt_scalar = 0, opt_layout = 0, opt_gate = 0, opt_wave_times = 0, opt_cut = 0, opt_share = 0, opt_cluster = 0;
};

struct vrh_scene
{
    vrh_ctx* ctx = nullptr;
    float4* pairs = nullptr;
    float4* prims = nullptr;
    float4* normals = nullptr;
    float4* quads = nullptr;     // 4-wide any-hit records (vrh_quad.cpp), null if the scene has none
    float4* vnormals = nullptr;  // per-vertex normals (3 per prim_id), VRH_NORMALS_PER_VERTEX
    vrh::node32* dnodes = nullptr;    // GPU-built scenes: the tree in the reference layout (download)
    uint32_t* dindices = nullptr;
    uint32_t roots[vrh::MAX_LIST] = {};   // root link of every BVH (one unless a scene list)
    uint32_t num_roots = 1;
    uint32_t num_pairs = 0;          // pair records in `pairs`
    uint32_t quad_depth = 0;
    bool finite_bounds = true;   // every node bound finite (enables the hardware min/max slab path)
    vrh_scene_info info{};
};

struct vrh_shading
{
    vrh_ctx* ctx = nullptr;
    vrh::dev::plastic_t* materials = nullptr;
    vrh::dev::point_light_t* lights = nullptr;
    uint32_t num_materials = 0, num_lights = 0;
};

struct vrh_hit_mask
{
    vrh_ctx* ctx = nullptr;
    float2* tc = nullptr;         // 3 per prim_id
    uint8_t* mask = nullptr;
    uint32_t num_tc = 0, w = 0, h = 0;
};

struct vrh_rt
{
    vrh_ctx* ctx = nullptr;
    uint32_t width = 0, height = 0;
    float4* color = nullptr;
    uint32_t* prim_id = nullptr;
    float* t = nullptr;
    uint8_t* occ = nullptr;
    bool owned = false;
    uint32_t* mh_prim_id = nullptr;   // multi_hit<N> lists [pixel][N] (always owned)
    float* mh_t = nullptr;
    uint32_t mh_n = 0;
    hipEvent_t written = nullptr;     // last vrh_render_sharded unshard into this target (group stream)
    bool written_pending = false;
    // asynchronous frames: the lane that wrote this target last, and when (recorded on that lane after
    // the frame's writes); valid while the context has not joined its lanes since (join_epoch)
    hipEvent_t lane_written = nullptr;
    int lane = -1;
    uint64_t lane_epoch = 0;
};

// a render group's root wrote `rt` on `stream`: record it so the target's own context orders after
inline hipError_t mark_written(vrh_rt* rt, hipStream_t stream)
{
    if (!rt->written)
    {
        const hipError_t e = hipEventCreateWithFlags(&rt->written, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    const hipError_t e = hipEventRecord(rt->written, stream);
    if (e != hipSuccess) return e;
    rt->written_pending = true;
    if (rt->ctx)
    {
        auto& gw = rt->ctx->group_written;
        bool known = false;
        for (hipEvent_t ev : gw) known |= ev == rt->written;
        if (!known) gw.push_back(rt->written);
    }
    return hipSuccess;
}

// asynchronous frames: `stream` waits for every frame issued on the context's frame lanes so far
// (no host synchronisation).  Every entry point that issues work on `stream` or synchronises it calls
// this first, so work issued after a frame sees that frame's results.
// issue the pending scratch copy of lane `l` (vrh_runtime.hip); l < 0: every lane
hipError_t ctx_flush_pending(const vrh_ctx* ctx, int l = -1);

inline hipError_t ctx_join(const vrh_ctx* ctx)
{
    const hipError_t f = ctx_flush_pending(ctx);
    if (f != hipSuccess) return f;
    bool any = false;
    for (const auto& l : ctx->lane)
        if (l.used)
        {
            const hipError_t e = hipStreamWaitEvent(ctx->stream, l.done, 0);
            if (e != hipSuccess) return e;
            any = true;
        }
    if (any) ++ctx->join_epoch;
    return hipSuccess;
}

// status plumbing shared by the C-ABI translation units: every HIP call is checked, nothing throws
#define VRH_HIP(call)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            vrh::set_error(std::string(#call) + ": " + hipGetErrorString(e_));                    \
            return e_ == hipErrorOutOfMemory ? VRH_ERR_OOM : VRH_ERR_HIP;                          \
        }                                                                                          \
    } while (0)

#define VRH_CHECK(cond, msg)                                                                       \
    do {                                                                                           \
        if (!(cond)) { vrh::set_error(msg); return VRH_ERR_INVALID; }                              \
    } while (0)
