// visionaray_amd/csrc/vrh_runtime.cpp -- the C-ABI of libvrh (include/vrh.h).
//
// Host-side runtime: contexts (device + stream + events + counters), scene upload with the
// MI355X layout transform (node pairs, leaf-ordered primitives), render targets, the frame launch
// (cuda_sched<R>::frame replacement, cuda_sched.inl:238-320), multi-GPU shard helpers and the
// host builder entry point.  Every HIP call is checked; nothing throws across the ABI.

#include "vrh_internal.h"
#include "vrh_kernels.h"
#include "vrh_plan.h"
#include "vrh_lbvh.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>

namespace vrh {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

} // namespace vrh

using namespace vrh;

#include "vrh_objects.h"

namespace {

int select_device(vrh_ctx* ctx)
{
    VRH_HIP(hipSetDevice(ctx->device));
    return VRH_OK;
}

// a render group's root writes its target on the group's stream (vrh_render_sharded): work on the
// target's context stream waits for that (an event wait, no host synchronisation)
int rt_wait(vrh_ctx* ctx, vrh_rt* rt)
{
    VRH_HIP(ctx_join(ctx));
    if (rt && rt->written_pending) VRH_HIP(hipStreamWaitEvent(ctx->stream, rt->written, 0));
    return VRH_OK;
}

// the context stream after every asynchronous frame, then the host after the stream
int ctx_drain(vrh_ctx* ctx)
{
    VRH_HIP(ctx_join(ctx));
    VRH_HIP(hipStreamSynchronize(ctx->stream));
    return VRH_OK;
}

} // namespace

extern "C" {

VRH_API const char* vrh_version(void) { return "visionaray-amd 0.1.0 (gfx950)"; }
VRH_API const char* vrh_last_error(void) { return g_last_error.c_str(); }

VRH_API int vrh_device_count(int* count)
{
    VRH_CHECK(count, "vrh_device_count: null");
    *count = 0;
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) { *count = 0; set_error(hipGetErrorString(e)); return VRH_ERR_NO_DEVICE; }
    return VRH_OK;
}

VRH_API int vrh_ctx_create_on_stream(int hip_device, void* hip_stream, vrh_ctx** out)
{
    VRH_CHECK(out, "vrh_ctx_create: null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) { set_error("no HIP device visible"); return VRH_ERR_NO_DEVICE; }
    VRH_CHECK(hip_device >= 0 && hip_device < n, "vrh_ctx_create: device index out of range");
    auto* ctx = new (std::nothrow) vrh_ctx;
    if (!ctx) { set_error("host allocation failed"); return VRH_ERR_OOM; }
    ctx->device = hip_device;
    int rc = VRH_OK;
    do {
        if ((rc = select_device(ctx)) != VRH_OK) break;
        hipDeviceProp_t prop;
        hipError_t e = hipGetDeviceProperties(&prop, hip_device);
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); rc = VRH_ERR_HIP; break; }
        ctx->num_cus = prop.multiProcessorCount;
        if (hip_stream) ctx->stream = static_cast<hipStream_t>(hip_stream);
        else
        {
            // a blocking stream (round 6): like the default stream cuda_sched launches on
            // (cuda_sched.inl:306-320), it is ordered against work on the NULL stream -- a program that
            // reads a target with a plain hipMemcpy after an asynchronous frame() sees the frame
            e = hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault);
            if (e != hipSuccess) { set_error(hipGetErrorString(e)); rc = VRH_ERR_HIP; break; }
            ctx->own_stream = true;
        }
        // one counter block for frames on the context stream, one per frame lane (asynchronous frames)
        e = hipMalloc(&ctx->counters, COUNTER_BLOCKS * COUNTERS_WORDS * sizeof(unsigned long long));
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); rc = VRH_ERR_OOM; break; }
        e = hipMemset(ctx->counters, 0, COUNTER_BLOCKS * COUNTERS_WORDS * sizeof(unsigned long long));
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); rc = VRH_ERR_HIP; break; }
        ctx->last_counters = ctx->counters;
        for (int i = 0; i < VRH_MAX_FRAME_LANES; ++i) ctx->lane[i].counters = ctx->counters + size_t(i + 1) * COUNTERS_WORDS;
    } while (0);
    if (rc != VRH_OK) { vrh_ctx_destroy(ctx); return rc; }
    *out = ctx;
    return VRH_OK;
}

VRH_API int vrh_ctx_create(int hip_device, vrh_ctx** out) { return vrh_ctx_create_on_stream(hip_device, nullptr, out); }

VRH_API int vrh_ctx_get_stream(const vrh_ctx* ctx, int* hip_device, void** hip_stream)
{
    VRH_CHECK(ctx, "vrh_ctx_get_stream: null context");
    // work the caller issues on the stream comes after every frame issued so far (asynchronous frames)
    bool lanes_used = false;
    for (const auto& l : ctx->lane) lanes_used |= l.used;
    if (hip_stream && lanes_used)
    {
        VRH_HIP(hipSetDevice(ctx->device));
        VRH_HIP(ctx_join(ctx));
    }
    if (hip_device) *hip_device = ctx->device;
    if (hip_stream) *hip_stream = ctx->stream;
    return VRH_OK;
}

VRH_API int vrh_ctx_destroy(vrh_ctx* ctx)
{
    if (!ctx) return VRH_OK;
    (void)hipSetDevice(ctx->device);
    for (auto& l : ctx->lane)
        if (l.stream) (void)hipStreamSynchronize(l.stream);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto& l : ctx->lane)
    {
        if (l.spill) (void)hipFree(l.spill);
        for (void* q : { (void*)l.color, (void*)l.prim_id, (void*)l.t, (void*)l.occ })
            if (q) (void)hipFree(q);
        if (l.done) (void)hipEventDestroy(l.done);
        if (l.stream) (void)hipStreamDestroy(l.stream);
    }
    if (ctx->main_mark) (void)hipEventDestroy(ctx->main_mark);
    if (ctx->counters) (void)hipFree(ctx->counters);
    if (ctx->wave_times) (void)hipFree(ctx->wave_times);
    if (ctx->user_queues) (void)hipFree(ctx->user_queues);
    if (ctx->tile_times) (void)hipFree(ctx->tile_times);
    if (ctx->spill) (void)hipFree(ctx->spill);
    for (auto e : ctx->ev_start) (void)hipEventDestroy(e);
    for (auto e : ctx->ev_stop) (void)hipEventDestroy(e);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return VRH_OK;
}

// the accepted range of every option (0 = automatic wherever a range starts at 0); checked on the
// int64 value before it is narrowed, so a negative or huge value is refused, never wrapped
struct option_range { uint32_t option; int64_t lo, hi; const char* what; };
constexpr option_range k_option_ranges[] = {
    { VRH_OPT_BLOCK_THREADS, 0, 256, "block threads is 0 (auto) or a multiple of 64 up to 256" },
    { VRH_OPT_STACK_CAP, 0, 640, "stack cap is 0 (auto) or 1..640 LDS entries per lane" },
    { VRH_OPT_AO_SCHEDULE, 0, 4, "schedule is 0 (auto) or 3 (step loop)" },
    { VRH_OPT_BLOCKS_PER_CU, 0, 32, "blocks per CU is 0 (auto) or 1..32" },
    { VRH_OPT_WAVES_PER_SIMD, 0, 8, "waves per SIMD is 0 (auto), 1, 5, 6 or 8" },
    { VRH_OPT_EXACT_MINMAX, 0, 1, "exact min/max is 0 (auto) or 1 (on)" },
    { VRH_OPT_XCD_QUEUES, 0, 4, "xcd queues is 0 (auto), 1 (strips), 2 (off), 3 (band-interleaved) or 4 (cluster order)" },
    { VRH_OPT_REFILL_MIN, 0, 64, "refill threshold is 0 (auto) or 1..64" },
    { VRH_OPT_WIDE_ANYHIT, 0, 2, "wide any-hit is 0 (auto), 1 (on) or 2 (off)" },
    { VRH_OPT_DESCENT_CAP, 0, 1024, "descent cap is 0 (auto) or 1..1024" },
    { VRH_OPT_POP_ON_MISS, 0, 2, "pop on miss is 0 (auto), 1 (on) or 2 (off)" },
    { VRH_OPT_COOP_FETCH, 0, 2, "cooperative fetch was removed (0 / 2 = off is accepted)" },
    { VRH_OPT_SCALAR_FETCH, 0, 2, "scalar fetch is 0 (auto), 1 (on) or 2 (off)" },
    { VRH_OPT_PAIR_LAYOUT, 0, 2, "pair layout is 0 (auto), 1 (line pairing) or 2 (builder order)" },
    { VRH_OPT_AO_GATE, 0, 2, "AO gate is 0 (auto), 1 (on) or 2 (off)" },
    { VRH_OPT_WAVE_TIMES, 0, 2, "wave times is 0 (off), 1 (on) or 2 (on + tile times of counting one-frame AO launches)" },
    { VRH_OPT_AO_CUT, 0, 3, "AO cut is 0 (auto), 1 (on, entries nearest-first), 2 (off) or 3 (on, entries in cut order)" },
    { VRH_OPT_AO_STEAL, 0, 2, "AO tail stash was removed (0 / 2 = off is accepted)" },
    { VRH_OPT_AO_SHARE, 0, 2, "AO tail sharing is 0 (auto), 1 (on) or 2 (off)" },
    { VRH_OPT_CLUSTER_TILES, 0, 1024, "cluster tiles is 0 (auto) or 1..1024" },
    { VRH_OPT_QUAD_REFILL, 0, 1, "the quad-coherent hand-out was removed (0 is accepted)" },
    { VRH_OPT_GROUP_UNITS, 0, 1, "the block-shared hand-out was removed (0 is accepted)" },
    { VRH_OPT_ASYNC_FRAMES, 0, VRH_MAX_FRAME_LANES, "asynchronous frames is 0 (off), 1 (on, the default number of frame lanes) or 2..4 (on, that many frame lanes)" },
};

VRH_API int vrh_ctx_set_option(vrh_ctx* ctx, uint32_t option, int64_t value)
{
    VRH_CHECK(ctx, "vrh_ctx_set_option: null");
    const option_range* range = nullptr;
    for (const option_range& r : k_option_ranges)
        if (r.option == option) range = &r;
    if (!range) { set_error("vrh_ctx_set_option: unknown option"); return VRH_ERR_INVALID; }
    VRH_CHECK(value >= range->lo && value <= range->hi,
              std::string("vrh_ctx_set_option: value ") + std::to_string(value) + " out of range: " + range->what);
    const int v = int(value);
    switch (option)
    {
    case VRH_OPT_BLOCK_THREADS:
        // the traversal kernels are compiled for at most 256 threads per block (__launch_bounds__(256, ...)):
        // a larger block would break the register allocation's assumptions (a launch failure)
        VRH_CHECK(v % 64 == 0, std::string("vrh_ctx_set_option: ") + range->what);
        ctx->opt_block = v; break;
    case VRH_OPT_STACK_CAP: ctx->opt_stack = v; break;
    case VRH_OPT_AO_SCHEDULE:
        // the item loop (4) was removed in round 2: the step loop measured faster for every kernel
        if (v == 4) { set_error("vrh_ctx_set_option: the item-loop schedule was removed (the step loop is faster, profiles/r02_ab/ab18_sphere_schedule.log)"); return VRH_ERR_UNSUPPORTED; }
        VRH_CHECK(v == 0 || v == 3, std::string("vrh_ctx_set_option: ") + range->what); ctx->opt_sched = v; break;
    case VRH_OPT_WIDE_ANYHIT: ctx->opt_wide = v; break;
    case VRH_OPT_DESCENT_CAP: ctx->opt_dcap = v; break;
    case VRH_OPT_COOP_FETCH:
        // the cooperative quad fetch was removed in round 2 (measured slower, profiles/r01/ab_nocoop.log)
        if (v == 1) { set_error("vrh_ctx_set_option: the cooperative fetch was removed (it measured slower)"); return VRH_ERR_UNSUPPORTED; }
        break;
    case VRH_OPT_WAVE_TIMES: ctx->opt_wave_times = v; break;
    case VRH_OPT_AO_CUT: ctx->opt_cut = v; break;
    case VRH_OPT_AO_STEAL:
        // the AO tail stash was removed in round 3 (measured slower)
        if (v == 1) { set_error("vrh_ctx_set_option: the AO tail stash was removed (it measured slower)"); return VRH_ERR_UNSUPPORTED; }
        break;
    case VRH_OPT_AO_SHARE: ctx->opt_share = v; break;
    case VRH_OPT_AO_GATE: ctx->opt_gate = v; break;
    case VRH_OPT_POP_ON_MISS: ctx->opt_pop = v; break;
    case VRH_OPT_PAIR_LAYOUT: ctx->opt_layout = v; break;
    case VRH_OPT_SCALAR_FETCH: ctx->opt_scalar = v; break;
    case VRH_OPT_REFILL_MIN: ctx->opt_refill = v; break;
    case VRH_OPT_BLOCKS_PER_CU: ctx->opt_bpc = v; break;
    case VRH_OPT_WAVES_PER_SIMD:
        VRH_CHECK(v == 0 || v == 1 || v == 5 || v == 6 || v == 8, std::string("vrh_ctx_set_option: ") + range->what);
        ctx->opt_occ = v; break;
    case VRH_OPT_EXACT_MINMAX: ctx->opt_exact_minmax = v; break;
    case VRH_OPT_XCD_QUEUES: ctx->opt_xcd_queues = v; break;
    case VRH_OPT_GROUP_UNITS:
    case VRH_OPT_QUAD_REFILL:
        // measured in round 4 and removed (slower: profiles/r04/ab/lane_layout/); 0 is accepted
        if (v != 0) { set_error("vrh_ctx_set_option: the quad-coherent and block-shared hand-outs were removed (they measured slower)"); return VRH_ERR_UNSUPPORTED; }
        break;
    case VRH_OPT_ASYNC_FRAMES:
    {
        // a different lane count: every frame issued so far is joined into the context stream first
        const uint32_t lanes = v == 1 ? uint32_t(VRH_DEFAULT_FRAME_LANES) : v > 1 ? uint32_t(v) : ctx->num_lanes;
        if (lanes != ctx->num_lanes)
        {
            VRH_HIP(hipSetDevice(ctx->device));
            VRH_HIP(ctx_join(ctx));
            ctx->num_lanes = lanes;
            ctx->next_lane = 0;
        }
        ctx->opt_async = v ? 1 : 0;
        break;
    }
    case VRH_OPT_CLUSTER_TILES: ctx->opt_cluster = v; break;
    default: set_error("vrh_ctx_set_option: unknown option"); return VRH_ERR_INVALID;
    }
    return VRH_OK;
}

// ---- scene upload -------------------------------------------------------------------------------

VRH_API int vrh_scene_upload(vrh_ctx* ctx, const void* nodes_v, uint32_t num_nodes, const void* prims_v,
                             uint32_t num_prims, uint32_t prim_kind, const uint32_t* indices, uint32_t num_indices,
                             const void* face_normals, vrh_scene** out)
{
    VRH_CHECK(ctx && out && nodes_v && prims_v, "vrh_scene_upload: null argument");
    VRH_CHECK(num_nodes >= 1 && num_prims >= 1, "vrh_scene_upload: empty BVH");
    VRH_CHECK(prim_kind == VRH_PRIM_TRI64 || prim_kind == VRH_PRIM_SPHERE48, "vrh_scene_upload: unknown prim_kind");
    VRH_CHECK(num_nodes % 2 == 1, "vrh_scene_upload: node count must be odd (root + child pairs)");
    *out = nullptr;
    if (!indices) num_indices = num_prims;
    auto nodes = static_cast<const node32*>(nodes_v);

    // -- node pairs + topology validation + depth
    const uint32_t npairs = (num_nodes - 1) / 2;
    std::vector<float4> pairs(4 * std::max<uint32_t>(npairs, 1), make_float4(0, 0, 0, 0));
    std::vector<uint8_t> end_flag(num_indices, 0);
    auto link_of = [&](const node32& c, uint32_t& link) -> bool {
        if (c.num_prims != 0)
        {
            if (uint64_t(c.first) + c.num_prims > num_indices || c.first >= 0x80000000u) return false;
            end_flag[c.first + c.num_prims - 1] = 1;
            link = 0x80000000u | c.first;
            return true;
        }
        if (c.first == 0 || c.first % 2 != 1 || uint64_t(c.first) + 1 >= num_nodes) return false;
        link = (c.first - 1) / 2;
        return true;
    };
    uint32_t root = 0;
    if (!link_of(nodes[0], root)) { set_error("vrh_scene_upload: malformed root node"); return VRH_ERR_INVALID; }
    if (nodes[0].num_prims == 0 && nodes[0].first != 1) { set_error("vrh_scene_upload: root children must be nodes 1,2"); return VRH_ERR_INVALID; }
    for (uint32_t k = 0; k < npairs; ++k)
    {
        const node32& c0 = nodes[2 * k + 1];
        const node32& c1 = nodes[2 * k + 2];
        uint32_t l0, l1;
        if (!link_of(c0, l0) || !link_of(c1, l1)) { set_error("vrh_scene_upload: malformed node pair " + std::to_string(k)); return VRH_ERR_INVALID; }
        float4* q = &pairs[4 * k];
        // slab-major, child-interleaved (vrh_device.h): packed (child 0, child 1) operand pairs
        q[0] = make_float4(c0.bmin[0], c1.bmin[0], c0.bmin[1], c1.bmin[1]);
        q[1] = make_float4(c0.bmin[2], c1.bmin[2], c0.bmax[0], c1.bmax[0]);
        q[2] = make_float4(c0.bmax[1], c1.bmax[1], c0.bmax[2], c1.bmax[2]);
        uint32_t w[4] = { l0, l1, 0u, 0u };
        std::memcpy(&q[3], w, 16);
    }
    // depth (root depth 0) by iterative DFS over links
    uint32_t max_depth = 0;
    {
        // every pair may be reached at most once: a pair reached twice (a DAG or a cycle) is rejected
        std::vector<std::pair<uint32_t, uint32_t>> st;
        std::vector<uint8_t> seen(npairs, 0);
        if (!(root & 0x80000000u)) st.push_back({ root, 1u });
        while (!st.empty())
        {
            auto e = st.back(); st.pop_back();
            if (seen[e.first]) { set_error("vrh_scene_upload: BVH is not a tree (a node pair is reached twice)"); return VRH_ERR_INVALID; }
            seen[e.first] = 1;
            max_depth = std::max(max_depth, e.second);
            uint32_t w[4];
            std::memcpy(w, &pairs[4 * e.first + 3], 16);
            for (int c = 0; c < 2; ++c)
                if (!(w[c] & 0x80000000u))
                {
                    if (w[c] >= npairs) { set_error("vrh_scene_upload: child pair out of range"); return VRH_ERR_INVALID; }
                    st.push_back({ w[c], e.second + 1 });
                }
        }
    }

    // -- cache-line pairing (VRH_OPT_PAIR_LAYOUT = 1; auto off: measured neutral, within 1.3 %,
    // profiles/r01/ab_layout.log): re-lay the pair records in a depth-first
    // preorder that puts each pair's child-0 pair right after it, so a parent and a child share a
    // 128-B line on half of the descent steps (31 % in the builder's order).  Links are renumbered;
    // the tree, the traversal order and every result are unchanged.
    if (ctx->opt_layout == 1 && npairs > 1 && !(root & 0x80000000u))
    {
        std::vector<uint32_t> perm(npairs, 0xFFFFFFFFu);
        uint32_t next = 0;
        std::vector<uint32_t> st{ root };
        while (!st.empty())
        {
            const uint32_t k = st.back(); st.pop_back();
            perm[k] = next++;
            uint32_t w[4];
            std::memcpy(w, &pairs[4 * k + 3], 16);
            if (!(w[1] & 0x80000000u)) st.push_back(w[1]);
            if (!(w[0] & 0x80000000u)) st.push_back(w[0]);
        }
        for (uint32_t k = 0; k < npairs; ++k)
            if (perm[k] == 0xFFFFFFFFu) perm[k] = next++;      // unreachable records keep a slot
        if (next != npairs) { set_error("vrh_scene_upload: pair layout: not a permutation"); return VRH_ERR_INVALID; }
        std::vector<float4> np(pairs.size());
        for (uint32_t k = 0; k < npairs; ++k)
        {
            float4* d = &np[4 * size_t(perm[k])];
            std::memcpy(d, &pairs[4 * size_t(k)], 64);
            uint32_t w[4];
            std::memcpy(w, &d[3], 16);
            for (int c = 0; c < 2; ++c)
                if (!(w[c] & 0x80000000u)) w[c] = perm[w[c]];
            std::memcpy(&d[3], w, 16);
        }
        pairs.swap(np);
        root = perm[root];
    }

    // -- leaf-ordered primitives with END flags
    const uint32_t f4_per = prim_kind == VRH_PRIM_TRI64 ? 3u : 2u;
    std::vector<float4> lp(size_t(f4_per) * num_indices);
    for (uint32_t i = 0; i < num_indices; ++i)
    {
        uint32_t src = indices ? indices[i] : i;
        if (src >= num_prims) { set_error("vrh_scene_upload: index out of range"); return VRH_ERR_INVALID; }
        uint32_t flags = end_flag[i] ? 1u : 0u;
        float4* q = &lp[size_t(f4_per) * i];
        if (prim_kind == VRH_PRIM_TRI64)
        {
            const tri64& t = static_cast<const tri64*>(prims_v)[src];
            q[0] = make_float4(t.v1[0], t.v1[1], t.v1[2], t.e1[0]);
            q[1] = make_float4(t.e1[1], t.e1[2], t.e2[0], t.e2[1]);
            uint32_t w[4];
            std::memcpy(&w[0], &t.e2[2], 4);
            w[1] = t.prim_id; w[2] = t.geom_id; w[3] = flags;
            std::memcpy(&q[2], w, 16);
        }
        else
        {
            const sphere48& s = static_cast<const sphere48*>(prims_v)[src];
            q[0] = make_float4(s.center[0], s.center[1], s.center[2], s.radius);
            uint32_t w[4] = { s.prim_id, s.geom_id, flags, 0u };
            std::memcpy(&q[1], w, 16);
        }
    }

    bool finite_bounds = true;
    for (uint32_t i = 0; i < num_nodes && finite_bounds; ++i)
        for (int a = 0; a < 3; ++a)
            finite_bounds = finite_bounds && std::isfinite(nodes[i].bmin[a]) && std::isfinite(nodes[i].bmax[a]);

    uint32_t max_prim_id = 0, max_geom_id = 0;
    for (uint32_t i = 0; i < num_prims; ++i)
    {
        uint32_t ids[2];
        std::memcpy(ids, static_cast<const uint8_t*>(prims_v) + size_t(i) * (prim_kind == VRH_PRIM_TRI64 ? 64u : 48u), 8);
        max_geom_id = std::max(max_geom_id, ids[0]);
        max_prim_id = std::max(max_prim_id, ids[1]);
    }

    std::vector<float> quads;
    uint32_t quad_root = 0, quad_depth = 0;
    const bool have_quads = finite_bounds && build_quads(nodes, num_nodes, quads, quad_root, quad_depth);

    int rc = select_device(ctx);
    if (rc) return rc;
    auto* sc = new (std::nothrow) vrh_scene;
    if (!sc) { set_error("host allocation failed"); return VRH_ERR_OOM; }
    sc->ctx = ctx;
    sc->roots[0] = root;
    sc->num_pairs = npairs;
    sc->finite_bounds = finite_bounds;
    auto fail = [&](hipError_t e, const char* what) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        vrh_scene_free(sc);
        return e == hipErrorOutOfMemory ? VRH_ERR_OOM : VRH_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipMalloc(&sc->pairs, pairs.size() * sizeof(float4))) != hipSuccess) return fail(e, "hipMalloc(pairs)");
    if ((e = hipMalloc(&sc->prims, lp.size() * sizeof(float4))) != hipSuccess) return fail(e, "hipMalloc(prims)");
    if ((e = hipMemcpy(sc->pairs, pairs.data(), pairs.size() * sizeof(float4), hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "upload pairs");
    if ((e = hipMemcpy(sc->prims, lp.data(), lp.size() * sizeof(float4), hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "upload prims");
    uint64_t bytes = pairs.size() * sizeof(float4) + lp.size() * sizeof(float4);
    if (have_quads)
    {
        const size_t qb = quads.size() * sizeof(float);
        if ((e = hipMalloc(&sc->quads, qb)) != hipSuccess) return fail(e, "hipMalloc(quads)");
        if ((e = hipMemcpy(sc->quads, quads.data(), qb, hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "upload quads");
        sc->quad_depth = quad_depth;
        sc->info.wide_records = uint32_t(quads.size() / 32);
        sc->info.wide_depth = quad_depth;
        bytes += qb;
    }
    if (face_normals)
    {
        if ((e = hipMalloc(&sc->normals, size_t(num_prims) * sizeof(float4))) != hipSuccess) return fail(e, "hipMalloc(normals)");
        if ((e = hipMemcpy(sc->normals, face_normals, size_t(num_prims) * sizeof(float4), hipMemcpyHostToDevice)) != hipSuccess) return fail(e, "upload normals");
        bytes += size_t(num_prims) * sizeof(float4);
    }
    sc->info.num_nodes = num_nodes;
    sc->info.num_bvhs = 1;
    sc->info.num_prims = num_prims;
    sc->info.num_indices = num_indices;
    sc->info.prim_kind = prim_kind;
    sc->info.max_depth = max_depth;
    sc->info.max_prim_id = max_prim_id;
    sc->info.max_geom_id = max_geom_id;
    sc->info.device_bytes = bytes;
    *out = sc;
    return VRH_OK;
}

VRH_API int vrh_scene_get_info(const vrh_scene* scene, vrh_scene_info* info)
{
    VRH_CHECK(scene && info, "vrh_scene_get_info: null");
    *info = scene->info;
    return VRH_OK;
}

VRH_API int vrh_scene_get_view(const vrh_scene* scene, uint32_t bvh, vrh_scene_view* out)
{
    VRH_CHECK(scene && out, "vrh_scene_get_view: null");
    VRH_CHECK(bvh < scene->num_roots, "vrh_scene_get_view: bvh index out of range");
    vrh_scene_view v{};
    v.pairs = scene->pairs;
    v.prims = scene->prims;
    v.normals = scene->normals;
    v.root = scene->roots[bvh];
    v.max_depth = scene->info.max_depth;
    v.prim_kind = scene->info.prim_kind;
    v.finite_bounds = scene->finite_bounds ? 1u : 0u;
    v.num_prims = scene->info.num_indices;
    if (scene->quads && scene->num_roots == 1 && scene->finite_bounds)
    {
        v.quads = scene->quads;
        v.quad_depth = scene->quad_depth;
    }
    *out = v;
    return VRH_OK;
}

VRH_API int vrh_scene_free(vrh_scene* sc)
{
    if (!sc) return VRH_OK;
    if (sc->ctx) (void)hipSetDevice(sc->ctx->device);
    if (sc->pairs) (void)hipFree(sc->pairs);
    if (sc->prims) (void)hipFree(sc->prims);
    if (sc->normals) (void)hipFree(sc->normals);
    if (sc->quads) (void)hipFree(sc->quads);
    if (sc->vnormals) (void)hipFree(sc->vnormals);
    if (sc->dnodes) (void)hipFree(sc->dnodes);
    if (sc->dindices) (void)hipFree(sc->dindices);
    delete sc;
    return VRH_OK;
}

namespace {
// scene lists: the pair records of one member re-based into the combined arrays (inner links by
// the member's first pair, leaf links by its first primitive)
__global__ void rebase_links_kernel(float4* pairs, uint32_t n, uint32_t pair_off, uint32_t prim_off)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* w = reinterpret_cast<uint32_t*>(pairs + 4u * size_t(i) + 3u);
    for (int c = 0; c < 2; ++c)
        w[c] = (w[c] & 0x80000000u) ? (0x80000000u | ((w[c] & 0x7FFFFFFFu) + prim_off)) : w[c] + pair_off;
}
} // namespace

VRH_API int vrh_scene_list_create(vrh_ctx* ctx, const vrh_scene* const* scenes, uint32_t count,
                                  const void* face_normals, uint32_t num_normals, vrh_scene** out)
{
    VRH_CHECK(ctx && scenes && out, "vrh_scene_list_create: null argument");
    VRH_CHECK(count >= 1 && count <= VRH_MAX_SCENE_LIST, "vrh_scene_list_create: 1..VRH_MAX_SCENE_LIST scenes");
    *out = nullptr;
    uint64_t pairs = 0, prims = 0, nodes = 0, bytes = 0;
    uint32_t kind = scenes[0] ? scenes[0]->info.prim_kind : 0u, depth = 0, max_pid = 0, max_gid = 0;
    bool finite = true;
    for (uint32_t i = 0; i < count; ++i)
    {
        const vrh_scene* m = scenes[i];
        VRH_CHECK(m && m->ctx == ctx, "vrh_scene_list_create: scene missing or of another context");
        VRH_CHECK(m->num_roots == 1, "vrh_scene_list_create: members must be single BVHs");
        VRH_CHECK(m->info.prim_kind == kind, "vrh_scene_list_create: members must share one primitive type");
        pairs += m->num_pairs;
        prims += m->info.num_indices;
        nodes += m->info.num_nodes;
        depth = std::max(depth, m->info.max_depth);
        max_pid = std::max(max_pid, m->info.max_prim_id);
        max_gid = std::max(max_gid, m->info.max_geom_id);
        finite = finite && m->finite_bounds;
    }
    VRH_CHECK(pairs < 0x80000000ull && prims < 0x80000000ull && nodes < 0xFFFFFFF0ull, "vrh_scene_list_create: list too large");
    VRH_CHECK(!face_normals || uint64_t(num_normals) > max_pid, "vrh_scene_list_create: face normals must cover every prim_id");
    int rc = select_device(ctx);
    if (rc) return rc;
    auto* sc = new (std::nothrow) vrh_scene;
    if (!sc) { set_error("host allocation failed"); return VRH_ERR_OOM; }
    sc->ctx = ctx;
    auto fail = [&](hipError_t e, const char* what) {
        set_error(std::string("vrh_scene_list_create: ") + what + ": " + hipGetErrorString(e));
        vrh_scene_free(sc);
        return e == hipErrorOutOfMemory ? VRH_ERR_OOM : VRH_ERR_HIP;
    };
    const uint32_t f4_per = kind == VRH_PRIM_TRI64 ? 3u : 2u;
    hipError_t e;
    if ((e = hipMalloc(&sc->pairs, std::max<uint64_t>(pairs, 1) * 64)) != hipSuccess) return fail(e, "pairs");
    if ((e = hipMalloc(&sc->prims, prims * f4_per * 16)) != hipSuccess) return fail(e, "prims");
    uint32_t pair_off = 0, prim_off = 0;
    for (uint32_t i = 0; i < count; ++i)
    {
        const vrh_scene* m = scenes[i];
        if (m->num_pairs)
        {
            if ((e = hipMemcpyAsync(sc->pairs + 4u * size_t(pair_off), m->pairs, size_t(m->num_pairs) * 64,
                                    hipMemcpyDeviceToDevice, ctx->stream)) != hipSuccess) return fail(e, "copy pairs");
            hipLaunchKernelGGL(rebase_links_kernel, dim3((m->num_pairs + 255u) / 256u), dim3(256), 0, ctx->stream,
                               sc->pairs + 4u * size_t(pair_off), m->num_pairs, pair_off, prim_off);
            if ((e = hipGetLastError()) != hipSuccess) return fail(e, "rebase");
        }
        if ((e = hipMemcpyAsync(sc->prims + size_t(f4_per) * prim_off, m->prims, size_t(m->info.num_indices) * f4_per * 16,
                                hipMemcpyDeviceToDevice, ctx->stream)) != hipSuccess) return fail(e, "copy prims");
        const uint32_t r = m->roots[0];
        sc->roots[i] = (r & 0x80000000u) ? (0x80000000u | ((r & 0x7FFFFFFFu) + prim_off)) : r + pair_off;
        pair_off += m->num_pairs;
        prim_off += m->info.num_indices;
    }
    bytes = std::max<uint64_t>(pairs, 1) * 64 + prims * f4_per * 16;
    if (face_normals)
    {
        if ((e = hipMalloc(&sc->normals, size_t(num_normals) * 16)) != hipSuccess) return fail(e, "normals");
        if ((e = hipMemcpyAsync(sc->normals, face_normals, size_t(num_normals) * 16, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
            return fail(e, "upload normals");
        bytes += uint64_t(num_normals) * 16;
    }
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return fail(e, "sync");
    sc->num_roots = count;
    sc->num_pairs = uint32_t(pairs);
    sc->finite_bounds = finite;
    sc->info.num_nodes = uint32_t(nodes);
    sc->info.num_prims = uint32_t(prims);
    sc->info.num_indices = uint32_t(prims);
    sc->info.prim_kind = kind;
    sc->info.max_depth = depth;
    sc->info.max_prim_id = max_pid;
    sc->info.max_geom_id = max_gid;
    sc->info.device_bytes = bytes;
    sc->info.num_bvhs = count;
    *out = sc;
    return VRH_OK;
}

VRH_API int vrh_scene_build(vrh_ctx* ctx, const void* prims, uint32_t num_prims, uint32_t prim_kind,
                            const void* face_normals, const vrh_build_desc* desc, vrh_scene** out)
{
    VRH_CHECK(ctx && prims && out && num_prims >= 1, "vrh_scene_build: bad argument");
    VRH_CHECK(prim_kind == VRH_PRIM_TRI64 || prim_kind == VRH_PRIM_SPHERE48, "vrh_scene_build: unknown prim_kind");
    VRH_CHECK(!desc || desc->method == VRH_BUILD_LBVH, "vrh_scene_build: unknown build method");
    *out = nullptr;
    int rc = select_device(ctx);
    if (rc) return rc;
    lbvh_out b;
    std::string err;
    rc = build_lbvh(prims, num_prims, prim_kind, desc && desc->max_leaf ? desc->max_leaf : 4u, ctx->stream, b, err);
    if (rc) { set_error(err); return rc; }
    auto* sc = new (std::nothrow) vrh_scene;
    if (!sc)
    {
        for (void* p : { (void*)b.nodes, (void*)b.indices, (void*)b.pairs, (void*)b.prims }) (void)hipFree(p);
        set_error("host allocation failed");
        return VRH_ERR_OOM;
    }
    sc->ctx = ctx;
    sc->pairs = b.pairs; sc->prims = b.prims; sc->dnodes = b.nodes; sc->dindices = b.indices;
    sc->roots[0] = b.root;
    sc->num_pairs = b.num_pairs;
    sc->finite_bounds = b.finite;
    uint64_t bytes = uint64_t(std::max(b.num_pairs, 1u)) * 64 + uint64_t(num_prims) * (prim_kind == VRH_PRIM_TRI64 ? 48 : 32);
    if (face_normals)
    {
        hipError_t e = hipMalloc(&sc->normals, size_t(num_prims) * sizeof(float4));
        if (e == hipSuccess) e = hipMemcpy(sc->normals, face_normals, size_t(num_prims) * sizeof(float4), hipMemcpyHostToDevice);
        if (e != hipSuccess)
        {
            set_error(std::string("vrh_scene_build: normals: ") + hipGetErrorString(e));
            vrh_scene_free(sc);
            return VRH_ERR_HIP;
        }
        bytes += uint64_t(num_prims) * sizeof(float4);
    }
    sc->info.num_nodes = b.num_nodes;
    sc->info.num_prims = num_prims;
    sc->info.num_indices = num_prims;
    sc->info.prim_kind = prim_kind;
    sc->info.max_depth = b.max_depth;
    sc->info.device_bytes = bytes;
    sc->info.max_prim_id = b.max_prim_id;
    sc->info.max_geom_id = b.max_geom_id;
    sc->info.gpu_built = 1;
    sc->info.num_bvhs = 1;
    sc->info.build_ms = b.build_ms;
    *out = sc;
    return VRH_OK;
}

VRH_API int vrh_scene_download_bvh(vrh_ctx* ctx, const vrh_scene* sc, void* nodes_out, uint32_t* num_nodes,
                                   uint32_t* indices_out)
{
    VRH_CHECK(ctx && sc && num_nodes, "vrh_scene_download_bvh: null argument");
    if (!sc->dnodes) { set_error("vrh_scene_download_bvh: only GPU-built scenes keep their tree on the device"); return VRH_ERR_UNSUPPORTED; }
    if (!nodes_out) { *num_nodes = sc->info.num_nodes; return VRH_OK; }
    VRH_CHECK(*num_nodes >= sc->info.num_nodes, "vrh_scene_download_bvh: nodes_out too small");
    int rc = select_device(ctx);
    if (rc) return rc;
    if ((rc = ctx_drain(ctx))) return rc;
    VRH_HIP(hipMemcpy(nodes_out, sc->dnodes, size_t(sc->info.num_nodes) * sizeof(node32), hipMemcpyDeviceToHost));
    if (indices_out) VRH_HIP(hipMemcpy(indices_out, sc->dindices, size_t(sc->info.num_indices) * 4, hipMemcpyDeviceToHost));
    *num_nodes = sc->info.num_nodes;
    return VRH_OK;
}

VRH_API int vrh_bvh_sah_cost(const void* nodes_v, uint32_t num_nodes, float ci, float cl, float cp, float* cost)
{
    VRH_CHECK(nodes_v && num_nodes >= 1 && cost, "vrh_bvh_sah_cost: bad argument");
    auto nodes = static_cast<const node32*>(nodes_v);
    // aabb.inl:177-196 surface_area = 2 * (s.x * s.y + s.y * s.z + s.z * s.x), s = max - min
    auto area = [](const node32& n) {
        const float sx = n.bmax[0] - n.bmin[0], sy = n.bmax[1] - n.bmin[1], sz = n.bmax[2] - n.bmin[2];
        return 2.0f * (sx * sy + sy * sz + sz * sx);
    };
    const float A_r = area(nodes[0]);
    float A_l = 0.0f, A_i = 0.0f, A_l_x_N_n = 0.0f;
    for (uint32_t i = 0; i < num_nodes; ++i)
    {
        if (nodes[i].num_prims != 0)
        {
            A_l += area(nodes[i]);
            A_l_x_N_n += area(nodes[i]) * static_cast<float>(nodes[i].num_prims);
        }
        else
            A_i += area(nodes[i]);
    }
    *cost = ci * (A_i / A_r) + cl * (A_l / A_r) + cp * (A_l_x_N_n / A_r);
    return VRH_OK;
}

VRH_API int vrh_scene_set_vertex_normals(vrh_scene* sc, const void* normals, uint32_t num_normals)
{
    VRH_CHECK(sc && normals, "vrh_scene_set_vertex_normals: null argument");
    VRH_CHECK(sc->info.prim_kind == VRH_PRIM_TRI64, "vrh_scene_set_vertex_normals: triangles only");
    VRH_CHECK(uint64_t(num_normals) >= 3ull * (uint64_t(sc->info.max_prim_id) + 1ull),
              "vrh_scene_set_vertex_normals: need 3 normals per prim_id (3 * (max prim_id + 1))");
    int rc = select_device(sc->ctx);
    if (rc) return rc;
    if (sc->vnormals) { (void)hipFree(sc->vnormals); sc->vnormals = nullptr; sc->info.vertex_normals = 0; }
    const size_t bytes = size_t(num_normals) * sizeof(float4);
    VRH_HIP(hipMalloc(&sc->vnormals, bytes));
    VRH_HIP(hipMemcpy(sc->vnormals, normals, bytes, hipMemcpyHostToDevice));
    sc->info.vertex_normals = 1;
    sc->info.device_bytes += bytes;
    return VRH_OK;
}

VRH_API int vrh_shading_create(vrh_ctx* ctx, const vrh_plastic* materials, uint32_t num_materials,
                               const vrh_point_light* lights, uint32_t num_lights, vrh_shading** out)
{
    static_assert(sizeof(vrh_plastic) == sizeof(dev::plastic_t), "plastic layout");
    static_assert(sizeof(vrh_point_light) == sizeof(dev::point_light_t), "light layout");
    VRH_CHECK(ctx && out && materials && num_materials > 0, "vrh_shading_create: need at least one material");
    VRH_CHECK(num_lights == 0 || lights, "vrh_shading_create: null lights");
    *out = nullptr;
    int rc = select_device(ctx);
    if (rc) return rc;
    auto* sh = new (std::nothrow) vrh_shading;
    if (!sh) { set_error("host allocation failed"); return VRH_ERR_OOM; }
    sh->ctx = ctx;
    sh->num_materials = num_materials;
    sh->num_lights = num_lights;
    hipError_t e = hipMalloc(&sh->materials, sizeof(vrh_plastic) * num_materials);
    if (e == hipSuccess) e = hipMemcpy(sh->materials, materials, sizeof(vrh_plastic) * num_materials, hipMemcpyHostToDevice);
    if (e == hipSuccess && num_lights)
    {
        e = hipMalloc(&sh->lights, sizeof(vrh_point_light) * num_lights);
        if (e == hipSuccess) e = hipMemcpy(sh->lights, lights, sizeof(vrh_point_light) * num_lights, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess)
    {
        set_error(std::string("vrh_shading_create: ") + hipGetErrorString(e));
        vrh_shading_free(sh);
        return e == hipErrorOutOfMemory ? VRH_ERR_OOM : VRH_ERR_HIP;
    }
    *out = sh;
    return VRH_OK;
}

VRH_API int vrh_hit_mask_create(vrh_ctx* ctx, const float* tex_coords, uint32_t num_tex_coords,
                                const uint8_t* mask, uint32_t mask_width, uint32_t mask_height, vrh_hit_mask** out)
{
    VRH_CHECK(ctx && out && tex_coords && mask, "vrh_hit_mask_create: null argument");
    VRH_CHECK(num_tex_coords >= 3 && num_tex_coords % 3 == 0, "vrh_hit_mask_create: 3 tex coords per triangle");
    VRH_CHECK(mask_width > 0 && mask_height > 0 && uint64_t(mask_width) * mask_height < (1ull << 32),
              "vrh_hit_mask_create: bad mask size");
    *out = nullptr;
    int rc = select_device(ctx);
    if (rc) return rc;
    auto* m = new (std::nothrow) vrh_hit_mask;
    if (!m) { set_error("host allocation failed"); return VRH_ERR_OOM; }
    m->ctx = ctx;
    m->num_tc = num_tex_coords;
    m->w = mask_width;
    m->h = mask_height;
    const size_t mb = size_t(mask_width) * mask_height;
    hipError_t e = hipMalloc(&m->tc, sizeof(float2) * num_tex_coords);
    if (e == hipSuccess) e = hipMemcpy(m->tc, tex_coords, sizeof(float2) * num_tex_coords, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&m->mask, mb);
    if (e == hipSuccess) e = hipMemcpy(m->mask, mask, mb, hipMemcpyHostToDevice);
    if (e != hipSuccess)
    {
        set_error(std::string("vrh_hit_mask_create: ") + hipGetErrorString(e));
        vrh_hit_mask_free(m);
        return e == hipErrorOutOfMemory ? VRH_ERR_OOM : VRH_ERR_HIP;
    }
    *out = m;
    return VRH_OK;
}

VRH_API int vrh_hit_mask_free(vrh_hit_mask* m)
{
    if (!m) return VRH_OK;
    if (m->ctx) (void)hipSetDevice(m->ctx->device);
    if (m->tc) (void)hipFree(m->tc);
    if (m->mask) (void)hipFree(m->mask);
    delete m;
    return VRH_OK;
}

VRH_API int vrh_shading_free(vrh_shading* sh)
{
    if (!sh) return VRH_OK;
    if (sh->ctx) (void)hipSetDevice(sh->ctx->device);
    if (sh->materials) (void)hipFree(sh->materials);
    if (sh->lights) (void)hipFree(sh->lights);
    delete sh;
    return VRH_OK;
}

// ---- render targets ------------------------------------------------------------------------------

VRH_API int vrh_rt_alloc(vrh_ctx* ctx, uint32_t w, uint32_t h, uint32_t flags, vrh_rt** out)
{
    VRH_CHECK(ctx && out && w > 0 && h > 0, "vrh_rt_alloc: bad argument");
    *out = nullptr;
    int rc = select_device(ctx);
    if (rc) return rc;
    auto* rt = new (std::nothrow) vrh_rt;
    if (!rt) { set_error("host allocation failed"); return VRH_ERR_OOM; }
    rt->ctx = ctx; rt->width = w; rt->height = h; rt->owned = true;
    size_t n = size_t(w) * h;
    hipError_t e = hipSuccess;
    if ((flags & VRH_RT_COLOR) && e == hipSuccess) e = hipMalloc(&rt->color, n * sizeof(float4));
    if ((flags & VRH_RT_PRIM_ID) && e == hipSuccess) e = hipMalloc(&rt->prim_id, n * sizeof(uint32_t));
    if ((flags & VRH_RT_T) && e == hipSuccess) e = hipMalloc(&rt->t, n * sizeof(float));
    if ((flags & VRH_RT_OCC) && e == hipSuccess) e = hipMalloc(&rt->occ, n);
    if (e != hipSuccess)
    {
        set_error(std::string("vrh_rt_alloc: ") + hipGetErrorString(e));
        vrh_rt_free(rt);
        return VRH_ERR_OOM;
    }
    *out = rt;
    return VRH_OK;
}

VRH_API int vrh_rt_wrap(vrh_ctx* ctx, uint32_t w, uint32_t h, void* color, uint32_t* prim_id, float* t, uint8_t* occ,
                        vrh_rt** out)
{
    VRH_CHECK(ctx && out && w > 0 && h > 0, "vrh_rt_wrap: bad argument");
    auto* rt = new (std::nothrow) vrh_rt;
    if (!rt) { set_error("host allocation failed"); return VRH_ERR_OOM; }
    rt->ctx = ctx; rt->width = w; rt->height = h; rt->owned = false;
    rt->color = static_cast<float4*>(color); rt->prim_id = prim_id; rt->t = t; rt->occ = occ;
    *out = rt;
    return VRH_OK;
}

VRH_API int vrh_rt_get_buffers(const vrh_rt* rt, void** color, uint32_t** prim_id, float** t, uint8_t** occ)
{
    VRH_CHECK(rt, "vrh_rt_get_buffers: null");
    if (color) *color = rt->color;
    if (prim_id) *prim_id = rt->prim_id;
    if (t) *t = rt->t;
    if (occ) *occ = rt->occ;
    return VRH_OK;
}

VRH_API int vrh_rt_free(vrh_rt* rt)
{
    if (!rt) return VRH_OK;
    if (rt->owned)
    {
        if (rt->ctx) (void)hipSetDevice(rt->ctx->device);
        if (rt->color) (void)hipFree(rt->color);
        if (rt->prim_id) (void)hipFree(rt->prim_id);
        if (rt->t) (void)hipFree(rt->t);
        if (rt->occ) (void)hipFree(rt->occ);
    }
    if (rt->mh_prim_id || rt->mh_t)
    {
        if (rt->ctx) (void)hipSetDevice(rt->ctx->device);
        if (rt->mh_prim_id) (void)hipFree(rt->mh_prim_id);
        if (rt->mh_t) (void)hipFree(rt->mh_t);
    }
    if (rt->ctx)
        for (auto& l : rt->ctx->lane)
            if (l.pending_rt == rt) l.pending_rt = nullptr;     // a frame nobody can read any more
    if (rt->lane_written)
    {
        if (rt->ctx) (void)hipSetDevice(rt->ctx->device);
        (void)hipEventSynchronize(rt->lane_written);
        (void)hipEventDestroy(rt->lane_written);
    }
    if (rt->written)
    {
        if (rt->ctx) (void)hipSetDevice(rt->ctx->device);
        (void)hipEventSynchronize(rt->written);
        if (rt->ctx)
        {
            auto& gw = rt->ctx->group_written;
            for (size_t i = 0; i < gw.size(); ++i)
                if (gw[i] == rt->written) { gw.erase(gw.begin() + long(i)); break; }
        }
        (void)hipEventDestroy(rt->written);
    }
    delete rt;
    return VRH_OK;
}

namespace {
__global__ void fill_rt_kernel(float4* color, uint32_t* pid, float* t, uint8_t* occ, size_t n, float4 c)
{
    size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (color) color[i] = c;
    if (pid) pid[i] = 0xFFFFFFFFu;
    if (t) t[i] = -1.0f;
    if (occ) occ[i] = 0;
}

// asynchronous frames: a frame rendered into a lane's scratch target lands in its target, scissor box
// only (the pixels a frame writes), once the target's previous writer is done
__global__ void copy_clip_kernel(float4* color, uint32_t* pid, float* t, uint8_t* occ, const float4* s_color,
                                 const uint32_t* s_pid, const float* s_t, const uint8_t* s_occ, uint32_t width,
                                 uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1)
{
    const uint32_t x = x0 + blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t y = y0 + blockIdx.y * blockDim.y + threadIdx.y;
    if (x >= x1 || y >= y1) return;
    const size_t i = size_t(y) * width + x;
    if (color) color[i] = s_color[i];
    if (pid) pid[i] = s_pid[i];
    if (t) t[i] = s_t[i];
    if (occ) occ[i] = s_occ[i];
}
} // namespace

} // extern "C"

// Asynchronous frames into a shared target: the scratch copy of lane l's pending frame, issued on that
// lane after the target's last writer (the other lane, unless joined since); the target's last writer
// is then this lane.  Called before anything else may read or write the target (ctx_join: every entry
// point that works on the context stream; vrh_render_batch for other frames) and before the lane's
// scratch target is reused.
hipError_t ctx_flush_pending(const vrh_ctx* cctx, int only)
{
    vrh_ctx* ctx = const_cast<vrh_ctx*>(cctx);
    for (int l = 0; l < VRH_MAX_FRAME_LANES; ++l)
    {
        if (only >= 0 && l != only) continue;
        vrh_ctx::lane_t& L = ctx->lane[l];
        vrh_rt* rt = L.pending_rt;
        if (!rt) continue;
        L.pending_rt = nullptr;
        hipError_t e;
        if (rt->lane >= 0 && rt->lane != l && rt->lane_epoch == ctx->join_epoch)
            if ((e = hipStreamWaitEvent(L.stream, rt->lane_written, 0)) != hipSuccess) return e;
        const uint32_t* cl = L.pending_clip;
        const dim3 blk(64, 4), grd((cl[2] - cl[0] + 63) / 64, (cl[3] - cl[1] + 3) / 4);
        const bool* fl = L.pending_fields;
        hipLaunchKernelGGL(copy_clip_kernel, grd, blk, 0, L.stream, fl[0] ? rt->color : nullptr, fl[1] ? rt->prim_id : nullptr,
                           fl[2] ? rt->t : nullptr, fl[3] ? rt->occ : nullptr, (const float4*)L.color,
                           (const uint32_t*)L.prim_id, (const float*)L.t, (const uint8_t*)L.occ, rt->width,
                           cl[0], cl[1], cl[2], cl[3]);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = hipEventRecord(rt->lane_written, L.stream)) != hipSuccess) return e;
        rt->lane = l;
        rt->lane_epoch = ctx->join_epoch;
        if ((e = hipEventRecord(L.done, L.stream)) != hipSuccess) return e;
    }
    return hipSuccess;
}

extern "C" {

// gpu_buffer_rt::clear_color_buffer (thrust::fill, gpu_buffer_rt.inl:49-76); side buffers reset to "miss"
VRH_API int vrh_rt_clear(vrh_ctx* ctx, vrh_rt* rt, const float color[4])
{
    VRH_CHECK(ctx && rt, "vrh_rt_clear: null");
    int rc = select_device(ctx);
    if (rc) return rc;
    size_t n = size_t(rt->width) * rt->height;
    float4 c = color ? make_float4(color[0], color[1], color[2], color[3]) : make_float4(0, 0, 0, 0);
    rc = rt_wait(ctx, rt);
    if (rc) return rc;
    hipLaunchKernelGGL(fill_rt_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, ctx->stream,
                       rt->color, rt->prim_id, rt->t, rt->occ, n, c);
    VRH_HIP(hipGetLastError());
    return VRH_OK;
}

// ---- frame ----------------------------------------------------------------------------------------

VRH_API uint32_t vrh_shard_bands(uint32_t height, uint32_t index, uint32_t count)
{
    return plan::shard_bands(height, index, count);
}

VRH_API int vrh_render(vrh_ctx* ctx, const vrh_scene* sc, vrh_rt* rt, const vrh_camera* cam,
                       const vrh_kernel_desc* k, const vrh_shard* shard, uint32_t frame_num)
{
    return vrh_render_batch(ctx, sc, rt, cam, 1, k, shard, frame_num);
}

namespace {
// one pass of a pixel sampler (vrh_render_sampled); null = the uniform sampler, colour stored
struct sampler_pass
{
    float off[2];
    uint32_t jitter, blend;
    float s, d;
    const float* inv_mats;    // vrh_render_view: inverse view, inverse projection (32 floats), else null
};
int render_batch_impl(vrh_ctx* ctx, const vrh_scene* sc, vrh_rt* rt, const vrh_camera* cams, uint32_t num_frames,
                      const vrh_kernel_desc* k, const vrh_shard* shard, uint32_t frame_num, const sampler_pass* sp);
} // namespace

VRH_API int vrh_render_batch(vrh_ctx* ctx, const vrh_scene* sc, vrh_rt* rt, const vrh_camera* cams,
                             uint32_t num_frames, const vrh_kernel_desc* k, const vrh_shard* shard,
                             uint32_t frame_num)
{
    return render_batch_impl(ctx, sc, rt, cams, num_frames, k, shard, frame_num, nullptr);
}

namespace {
// the passes of a pixel sampler (vrh_render_sampled / vrh_render_view); inv_mats: camera matrices
int render_sampled_impl(vrh_ctx* ctx, const vrh_scene* sc, vrh_rt* rt, const vrh_camera* cam,
                        const vrh_kernel_desc* k, const vrh_pixel_sampler* ps, uint32_t frame_num, const float* inv_mats)
{
    VRH_CHECK(ctx && sc && rt && cam && k && ps, "vrh_render_sampled: null argument");
    VRH_CHECK(ps->kind <= VRH_SAMPLER_SSAA, "vrh_render_sampled: unknown pixel sampler");
    if (ps->kind == VRH_SAMPLER_UNIFORM && !inv_mats) return render_batch_impl(ctx, sc, rt, cam, 1, k, nullptr, frame_num, nullptr);
    if (k->kind != VRH_KERNEL_PRIMARY && k->kind != VRH_KERNEL_AO)
    {
        set_error(inv_mats ? "vrh_render_view: camera matrices run the primary and AO kernels"
                           : "vrh_render_sampled: jittered / ssaa samplers run the primary and AO kernels");
        return VRH_ERR_UNSUPPORTED;
    }
    if (ps->kind != VRH_SAMPLER_SSAA)
    {
        // uniform (camera matrices): the pixel's ray, colour stored; jittered: the pixel's jittered
        // ray, colour stored; jittered_blend: blended with a = 1 / frame_num, 1 - a (sched_common.h:480-540)
        sampler_pass p{ { 0.0f, 0.0f }, ps->kind == VRH_SAMPLER_UNIFORM ? 0u : 1u, 0u, 1.0f, 0.0f, inv_mats };
        if (ps->kind == VRH_SAMPLER_JITTERED_BLEND)
        {
            p.blend = 1u;
            p.s = 1.0f / float(frame_num);
            p.d = 1.0f - p.s;
        }
        return render_batch_impl(ctx, sc, rt, cam, 1, k, nullptr, frame_num, &p);
    }
    // ssaa<N> (sched_common.h:219-300, 640-720): colour 0, then every sample blended with 1 / N, 1
    // in order -- one pass per sample on the context's stream
    static const float off2[2][2] = { { -0.25f, -0.25f }, { 0.25f, 0.25f } };
    static const float off4[4][2] = { { -0.125f, -0.375f }, { 0.375f, -0.125f }, { 0.125f, 0.375f }, { -0.375f, 0.125f } };
    static const float off8[8][2] = { { -0.125f, -0.4375f }, { 0.375f, -0.3125f }, { -0.375f, -0.1875f }, { 0.125f, -0.0625f },
                                      { -0.125f, 0.0625f }, { 0.375f, 0.1825f }, { -0.375f, 0.3125f }, { 0.125f, 0.4375f } };
    VRH_CHECK(ps->count == 2 || ps->count == 4 || ps->count == 8, "vrh_render_sampled: ssaa takes 2, 4 or 8 samples");
    const float (*tab)[2] = ps->count == 2 ? off2 : ps->count == 4 ? off4 : off8;
    for (uint32_t i = 0; i < ps->count; ++i)
    {
        sampler_pass p{ { tab[i][0], tab[i][1] }, 0u, i == 0 ? 2u : 1u, 1.0f / float(ps->count), 1.0f, inv_mats };
        const int rc = render_batch_impl(ctx, sc, rt, cam, 1, k, nullptr, frame_num, &p);
        if (rc) return rc;
    }
    return VRH_OK;
}
} // namespace

VRH_API int vrh_render_sampled(vrh_ctx* ctx, const vrh_scene* sc, vrh_rt* rt, const vrh_camera* cam,
                               const vrh_kernel_desc* k, const vrh_pixel_sampler* ps, uint32_t frame_num)
{
    return render_sampled_impl(ctx, sc, rt, cam, k, ps, frame_num, nullptr);
}

// matrix4.inl:209-244 inverse(): the 2x2 sub-determinants of rows 0-1 and 2-3
// (det2(a, b, c, d) = a * d - c * b, math.h:493-496), the cofactor expansion, every entry / det
VRH_API void vrh_matrix_inverse(const float m[16], float out[16])
{
    auto det2 = [](float a, float b, float c, float d) { return a * d - c * b; };
    auto M = [m](int r, int c) { return m[c * 4 + r]; };
    const float s0 = det2(M(0, 0), M(0, 1), M(1, 0), M(1, 1)), s1 = det2(M(0, 0), M(0, 2), M(1, 0), M(1, 2));
    const float s2 = det2(M(0, 0), M(0, 3), M(1, 0), M(1, 3)), s3 = det2(M(0, 1), M(0, 2), M(1, 1), M(1, 2));
    const float s4 = det2(M(0, 1), M(0, 3), M(1, 1), M(1, 3)), s5 = det2(M(0, 2), M(0, 3), M(1, 2), M(1, 3));
    const float c5 = det2(M(2, 2), M(2, 3), M(3, 2), M(3, 3)), c4 = det2(M(2, 1), M(2, 3), M(3, 1), M(3, 3));
    const float c3 = det2(M(2, 1), M(2, 2), M(3, 1), M(3, 2)), c2 = det2(M(2, 0), M(2, 3), M(3, 0), M(3, 3));
    const float c1 = det2(M(2, 0), M(2, 2), M(3, 0), M(3, 2)), c0 = det2(M(2, 0), M(2, 1), M(3, 0), M(3, 1));
    const float det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
    const float r[16] = {
        (M(1, 1) * c5 - M(1, 2) * c4 + M(1, 3) * c3) / det, (-M(1, 0) * c5 + M(1, 2) * c2 + M(1, 3) * c1) / det,
        (M(1, 0) * c4 - M(1, 1) * c2 + M(1, 3) * c0) / det, (-M(1, 0) * c3 + M(1, 1) * c1 + M(1, 2) * c0) / det,
        (-M(0, 1) * c5 + M(0, 2) * c4 - M(0, 3) * c3) / det, (M(0, 0) * c5 - M(0, 2) * c2 + M(0, 3) * c1) / det,
        (-M(0, 0) * c4 + M(0, 1) * c2 - M(0, 3) * c0) / det, (M(0, 0) * c3 - M(0, 1) * c1 + M(0, 2) * c0) / det,
        (M(3, 1) * s5 - M(3, 2) * s4 + M(3, 3) * s3) / det, (-M(3, 0) * s5 + M(3, 2) * s2 - M(3, 3) * s1) / det,
        (M(3, 0) * s4 - M(3, 1) * s2 + M(3, 3) * s0) / det, (-M(3, 0) * s3 + M(3, 1) * s1 - M(3, 2) * s0) / det,
        (-M(2, 1) * s5 + M(2, 2) * s4 - M(2, 3) * s3) / det, (M(2, 0) * s5 - M(2, 2) * s2 + M(2, 3) * s1) / det,
        (-M(2, 0) * s4 + M(2, 1) * s2 - M(2, 3) * s0) / det, (M(2, 0) * s3 - M(2, 1) * s1 + M(2, 2) * s0) / det };
    std::memcpy(out, r, sizeof(r));
}

VRH_API int vrh_render_view(vrh_ctx* ctx, const vrh_scene* sc, vrh_rt* rt, const vrh_view_camera* vc,
                            const vrh_kernel_desc* k, const vrh_pixel_sampler* ps, uint32_t frame_num)
{
    VRH_CHECK(ctx && vc, "vrh_render_view: null argument");
    vrh_camera cam{};
    cam.width = vc->width; cam.height = vc->height;
    std::memcpy(cam.scissor, vc->scissor, sizeof(cam.scissor));
    float inv[32];
    vrh_matrix_inverse(vc->view, inv);
    vrh_matrix_inverse(vc->proj, inv + 16);
    return render_sampled_impl(ctx, sc, rt, &cam, k, ps, frame_num, inv);
}

namespace {
int render_batch_impl(vrh_ctx* ctx, const vrh_scene* sc, vrh_rt* rt, const vrh_camera* cams, uint32_t num_frames,
                      const vrh_kernel_desc* k, const vrh_shard* shard, uint32_t frame_num, const sampler_pass* sp)
{
    VRH_CHECK(ctx && sc && rt && cams && k, "vrh_render: null argument");
    VRH_CHECK(rt->ctx == ctx && sc->ctx == ctx, "vrh_render: scene / render target of another context");
    VRH_CHECK(num_frames >= 1 && num_frames <= VRH_MAX_BATCH, "vrh_render_batch: 1..VRH_MAX_BATCH frames");
    const vrh_camera* cam = cams;
    for (uint32_t f = 1; f < num_frames; ++f)
        VRH_CHECK(cams[f].width == cam->width && cams[f].height == cam->height, "vrh_render_batch: frames differ in size");
    VRH_CHECK(cam->width > 0 && cam->height > 0, "vrh_render: empty image");
    VRH_CHECK(k->kind <= VRH_KERNEL_WHITTED, "vrh_render: unknown kernel kind");
    const bool ao = k->kind == VRH_KERNEL_AO;
    const bool multi = k->kind == VRH_KERNEL_MULTI_HIT;
    const bool whitted = k->kind == VRH_KERNEL_WHITTED;
    const bool shade = k->kind == VRH_KERNEL_SIMPLE || multi || whitted;
    const bool list = sc->num_roots > 1;
    if (multi)
    {
        VRH_CHECK(k->max_hits >= 1 && k->max_hits <= VRH_MAX_HITS, "vrh_render: max_hits must be in [1, 16]");
        VRH_CHECK(rt->mh_n == k->max_hits, "vrh_render: render target needs vrh_rt_alloc_multi_hit(max_hits)");
    }
    if (shade)
    {
        VRH_CHECK(k->shading, "vrh_render: the shading kernels need a vrh_shading (materials, lights)");
        if (sc->info.prim_kind != VRH_PRIM_TRI64) { set_error("vrh_render: the shading kernels support triangles"); return VRH_ERR_UNSUPPORTED; }
        if (list) { set_error("vrh_render: the shading kernels take a single BVH (scene lists: primary and AO kernels)"); return VRH_ERR_UNSUPPORTED; }
        VRH_CHECK(k->shading->num_materials > sc->info.max_geom_id, "vrh_render: a geom_id has no material");
        VRH_CHECK(k->normal_binding <= VRH_NORMALS_PER_VERTEX, "vrh_render: unknown normal binding");
        if (k->normal_binding == VRH_NORMALS_PER_FACE) VRH_CHECK(sc->normals, "vrh_render: per-face shading needs face normals");
        else VRH_CHECK(sc->vnormals, "vrh_render: per-vertex shading needs vrh_scene_set_vertex_normals");
    }
    if (ao)
    {
        VRH_CHECK(k->samples >= 1 && k->samples <= 32, "vrh_render: AO samples must be in [1, 32]");
        // the occlusion target holds one bit per sample in a byte
        VRH_CHECK(!rt->occ || k->samples <= 8 || (k->flags & VRH_KERNEL_NO_OCC),
                  "vrh_render: a VRH_RT_OCC target records at most 8 AO samples (VRH_KERNEL_NO_OCC leaves it out)");
        VRH_CHECK(sc->normals, "vrh_render: AO needs normals");
    }
    const vrh_hit_mask* hmask = k->hit_mask;
    if (hmask)
    {
        VRH_CHECK(hmask->ctx == ctx, "vrh_render: hit mask of another context");
        VRH_CHECK(sc->info.prim_kind != VRH_PRIM_TRI64 || uint64_t(hmask->num_tc) >= 3ull * (uint64_t(sc->info.max_prim_id) + 1),
                  "vrh_render: hit mask has fewer than 3 tex coords per prim_id");
    }
    vrh_shard whole{ 0, 1, 0, 0 };
    const vrh_shard& sh = shard ? *shard : whole;
    VRH_CHECK(sh.count >= 1 && sh.index < sh.count, "vrh_render: bad shard");
    const uint32_t local_bands = vrh_shard_bands(cam->height, sh.index, sh.count);
    VRH_CHECK(rt->width == cam->width, "vrh_render: render target width != camera width");
    // frame f of the batch owns rows [f * frame_rows, (f + 1) * frame_rows) of the target
    uint32_t frame_rows = cam->height;
    if (sh.packed)
    {
        frame_rows = rt->height / num_frames;
        VRH_CHECK(frame_rows >= local_bands * VRH_BAND_ROWS || local_bands == 0, "vrh_render: packed target too small");
    }
    else VRH_CHECK(rt->height == cam->height * num_frames, "vrh_render: render target height != camera height x frames");
    VRH_CHECK(uint64_t(rt->height) * rt->width < (1ull << 32), "vrh_render: render target too large");

    // a depth-first traversal holds at most `max_depth` stack entries (>= 1 for the root push):
    // `total` per lane, of which `cap` in LDS (the rest in a global overflow block, chosen below)
    const uint32_t need = std::max<uint32_t>(sc->info.max_depth, 1u);
    const uint32_t total = std::max((need + 3u) & ~3u, uint32_t(ctx->opt_stack));
    uint32_t cap = ctx->opt_stack ? uint32_t(ctx->opt_stack) : total;
    VRH_CHECK(cap >= 1u, "vrh_render: stack capacity option must be >= 1");
    launch_config lc{};
    lc.kind = sc->info.prim_kind == VRH_PRIM_TRI64 ? 0 : 1;
    lc.ao = ao;
    lc.count = (k->flags & VRH_KERNEL_COUNT_TESTS) != 0;
    // AO tail sharing needs several waves per block (they share LDS): 4 unless the block is set
    const bool ao_share = ctx->opt_share == 1 && ao && !list;
    lc.block = ctx->opt_block ? ctx->opt_block : ao_share ? 256 : 64;
    lc.share = ao_share;
    lc.stack_cap = int(cap);
    lc.epi = whitted ? 3 : multi ? 2 : shade ? 1 : 0;
    lc.max_hits = multi ? int(k->max_hits) : 0;
    // every kernel runs the step loop (the round-1 item loop for sphere primary visibility measured
    // 6-9 % slower than the step loop with its round-2 defaults, profiles/r02_ab/ab18_sphere_schedule.log,
    // and was removed)
    lc.sched = 0;
    if (list) lc.sched = 2;    // BVH lists: the step loop with the list merge
    if (sp)
    {
        // a pixel-sampler pass runs its own instance (the plain ones keep their code and registers)
        if (list || lc.count) { set_error("vrh_render_sampled: pixel samplers take a single BVH and no test counting"); return VRH_ERR_UNSUPPORTED; }
        lc.sched = 6;
    }
    // frames in flight on the step loop (primary / AO, uncounted): the BATCH instantiation
    if (lc.sched == 0 && num_frames > 1 && !lc.count && lc.epi == 0 && !hmask) lc.sched = 3;
    // shading epilogues: no VGPR cap (their lane state spills at 6 waves/SIMD; measured faster at 4,
    // profiles/r01/shade/shade_bench.jsonl), except whitted, whose bounce surface lives in LDS (vrh_shade.h):
    // 96 VGPRs without spills, 5 waves/SIMD, +0.7-2.1 % over 4 (profiles/r03_ab/whitted/).
    // AO on the step loop (round 5, the lean lane state: no VGPR spill or scratch at 80 VGPRs, also in
    // the overflow-stack instances): 6 waves/SIMD, the LDS stack shrunk (below) to 16 entries so that 24
    // waves fit a CU, the rest in the overflow block -- hf1M +4.8 %, hf10M +8.7 % over 5 waves
    // (profiles/r05/occupancy/s6_*); AO tail sharing (opt-in) has 5-wave instances only.  Primary
    // visibility: 8 waves/SIMD (64 VGPRs, no spill: hf1M +6.7-11 %, hf10M +3-9 %); spheres with frames in
    // flight too, with the LDS stack shrunk to 20 entries so that 32 waves fit a CU (sph1M +4.8 % over 7
    // waves, profiles/r05/sweepS/ -- at the whole 28-entry stack in LDS only 22 fit, -1 to -4 %,
    // profiles/r05/occupancy/), but one frame per launch at 7 (the occupancy-6 instance: 8 waves with the
    // overflow stack measured -8 %, profiles/r05/s26/); the counting variants keep 5 / 6 (at 8 they
    // spill hundreds of VGPRs).  BVH lists run at 5 / 6
    const int occ_ao = (ctx->opt_share == 1 || lc.count) ? 5 : 6;
    const int occ_primary = (!lc.count && (lc.kind == 0 || num_frames > 1)) ? 8 : 6;
    lc.occ = ctx->opt_occ ? ctx->opt_occ : whitted ? 5 : lc.epi ? 1 : lc.ao ? occ_ao : occ_primary;
    if (sp) lc.occ = lc.ao ? 5 : 6;                    // the sampler instances exist at the defaults
    if (list) lc.occ = ao ? 5 : 6;
    // tail sharing has instances for uncounted one-frame AO launches at 5 waves / SIMD only: where
    // the kernel selection (vrh_kernels.hip pick_share, asked through render_share_available) has no
    // SHARE instance the option changes nothing, not even the block size
    if (lc.share && !render_share_available(lc))
    {
        lc.share = false;
        if (!ctx->opt_block) lc.block = 64;
    }
    // auto: the LDS part of the stack shrinks (in steps of 4 entries) while LDS, not registers,
    // limits the waves per CU -- a deep BVH (hf10M: depth 26) then keeps the register-bound
    // occupancy and its few deepest entries go to the overflow block
    // (the primary / AO step loops at their default register budgets have overflow-stack instances;
    // every other kernel keeps its whole stack in LDS, as does an explicit VRH_OPT_STACK_CAP >= depth)
    if (render_spill_available(lc) && (!ctx->opt_stack || cap < total))
    {
        lc.spill = true;
        if (!ctx->opt_stack)
        {
            launch_config lo = lc;
            lo.stack_cap = 4;
            const int reg_bound = render_blocks_per_cu(lo);
            while (lc.stack_cap > 4 && render_blocks_per_cu(lc) < reg_bound) lc.stack_cap -= 4;
            // measured: hf10M AO 20 LDS entries +7 % over 24 at the same 20 waves / CU
            // (profiles/r02_ab/ab6_stack.log); no BVH of depth <= 20 spills
            if (total > 20u) lc.stack_cap = std::min(lc.stack_cap, 20);
            cap = uint32_t(lc.stack_cap);
        }
        if (cap >= total) lc.spill = false;     // nothing overflows: the plain instance
    }
    else if (cap < total)
        lc.stack_cap = int(cap = total);         // no overflow instance: the whole stack in LDS
    if (render_lds_bytes(lc) > 160u * 1024u)
    {
        set_error("vrh_render: BVH depth " + std::to_string(sc->info.max_depth) + " needs more LDS stack than a CU has");
        return VRH_ERR_UNSUPPORTED;
    }

    int rc = select_device(ctx);
    if (rc) return rc;
    // asynchronous frames (VRH_OPT_ASYNC_FRAMES): whole-image frames go to a frame lane (below);
    // shard renders (render groups record events on the context stream after their renders) and the
    // timeline diagnostics stay on the context stream
    const bool async = ctx->opt_async && !shard && !ctx->opt_wave_times;
    if (!async)
    {
        rc = rt_wait(ctx, rt);
        if (rc) return rc;
    }

    render_params p{};
    p.pairs = sc->pairs; p.prims = sc->prims; p.normals = sc->normals; p.root = sc->roots[0];
    p.num_roots = sc->num_roots;
    for (uint32_t i = 0; i < sc->num_roots; ++i) p.roots[i] = sc->roots[i];
    p.step_limit = sc->info.num_nodes + sc->info.num_indices + 16u;
    // measured: profiles/r01/ab (AO: refill at 32 free lanes), profiles/r01/ab_primary (primary
    // visibility: pop on a miss and a cap of 8 visits per descent step, +6 % on hf1M and +36 % on
    // hf10M; both hurt AO)
    const bool primary_step = !lc.ao && lc.epi == 0;
    // AO step loop: refill once 24 lanes are free for scenes the 256 MB Infinity Cache holds, 28 above
    // (profiles/r03_ab/refill/, 3 repetitions at 20 frames per launch: hf1M 24 vs 32 +0.6 %, hf10M
    // 28 vs 32 +0.3 % and 24 -0.6 %)
    p.refill_min = ctx->opt_refill ? uint32_t(ctx->opt_refill) : sc->info.device_bytes > (256ull << 20) ? 28u : 24u;
    // primary visibility with frames in flight refills once 16 lanes are free: +3 % sph1M, +2 % hf1M,
    // +1.8 % hf10M at 20 frames per launch (profiles/r02_ab/ab20_refill.log); simple::kernel and
    // whitted once 8 are: +1-2.5 % / +1 % (profiles/r02_ab/shade_refill.jsonl); one-frame primary
    // launches and multi_hit keep 1
    const uint32_t refill_shade = (lc.epi == 1 || lc.epi == 3) ? 8u : 1u;
    p.refill_min_primary = ctx->opt_refill ? uint32_t(ctx->opt_refill)
                         : (primary_step && num_frames > 1) ? 16u : lc.epi ? refill_shade : 1u;
    // primary visibility caps a lane's descent at 8 inner visits per step; at 8 waves / SIMD (round 5,
    // profiles/r05/sweepP2/, 20 frames per launch, min over rounds) triangle scenes the Infinity Cache
    // holds run best at 10 (hf1M +3 %; hf10M, above 256 MB, best at 8: 10 is -3 %), spheres at 6
    // (sph1M +1.5 %)
    const uint32_t dcap_primary = sc->info.prim_kind == VRH_PRIM_SPHERE48 ? 6u : sc->info.device_bytes > (256ull << 20) ? 8u : 10u;
    p.descent_cap = ctx->opt_dcap ? uint32_t(ctx->opt_dcap) : primary_step ? dcap_primary : 0xFFFFFFFFu;
    // shading epilogues (simple / multi_hit / whitted) pop on a miss too: +4-7 % (profiles/r01/shade/)
    // AO (step loop): the tile's AO rays wait for its primaries (ao_gate), any-hit rays descend the
    // 4-wide records and primaries pop on a miss -- together +6 % on hf1M and +10 % on hf10M
    // (profiles/r02_ab/ab4_c4opts.log); each alone is within +-2 %
    const bool ao_step = lc.ao;
    p.ao_gate = (ctx->opt_gate == 1 || (ctx->opt_gate == 0 && ao_step)) ? 1u : 0u;
    const bool pop = ctx->opt_pop == 1 || (ctx->opt_pop == 0 && (primary_step || lc.epi != 0 || ao_step));
    p.step_flags = (pop ? 1u : 0u) | (ctx->opt_scalar == 2 ? 0u : 2u);
    p.stack_cap = cap;
    p.stack_total = lc.spill ? total : cap;
    p.fast_ok = (sc->finite_bounds && !ctx->opt_exact_minmax) ? 1u : 0u;
    p.quads = sc->quads;
    // 4-wide any-hit records: auto on for the AO step loop (with ao_gate), off elsewhere
    const bool wide = ctx->opt_wide == 1 || (ctx->opt_wide == 0 && ao_step);
    // (the AO kernel restarts a 4-wide descent that would overflow its stack at pair 0: the root)
    p.quad_ok = (sc->quads && p.fast_ok && wide && sc->roots[0] == 0u) ? 1u : 0u;
    // per-tile entry cut of the 4-wide tree for AO rays (needs the gate: the tile's hits are known)
    // entries nearest-first (+3.5 % over the cut order, profiles/r02_ab/ab33_ao_cut_order*.log)
    p.ao_cut = (p.quad_ok && p.ao_gate && ctx->opt_cut != 2) ? (ctx->opt_cut == 3 ? 1u : 2u) : 0u;
    p.ao_share = (lc.share && lc.block > 64) ? 1u : 0u;
    for (uint32_t f = 0; f < num_frames; ++f)
    {
        std::memcpy(p.cam[f].eye, cams[f].eye, 12); std::memcpy(p.cam[f].cam_u, cams[f].cam_u, 12);
        std::memcpy(p.cam[f].cam_v, cams[f].cam_v, 12); std::memcpy(p.cam[f].cam_w, cams[f].cam_w, 12);
        // scissor_box (scheduler.h:25-31, default recti(0, 0, w, h) at :175): pixels x0 <= x < x1,
        // y0 <= y < y1 are rendered, the rest of the target is left as it is (cuda_sched.inl:71)
        const uint32_t* sb = cams[f].scissor;
        const bool whole_image = sb[0] == 0 && sb[1] == 0 && sb[2] == 0 && sb[3] == 0;
        p.cam[f].clip[0] = whole_image ? 0u : std::min(sb[0], cam->width);
        p.cam[f].clip[1] = whole_image ? 0u : std::min(sb[1], cam->height);
        p.cam[f].clip[2] = whole_image ? cam->width : std::min(sb[2], cam->width);
        p.cam[f].clip[3] = whole_image ? cam->height : std::min(sb[3], cam->height);
    }
    p.num_frames = num_frames;
    p.frame_num = frame_num;
    p.frame_rows = frame_rows;
    p.width = cam->width; p.height = cam->height;
    p.width_f = float(cam->width); p.height_f = float(cam->height);
    p.samples = ao ? k->samples : 0; p.radius = k->radius; p.eps = k->eps;
    p.samples_recip = ao ? ((1u << 20) + p.samples - 1u) / p.samples : 0u;
    std::memcpy(p.bg, k->bg, 16);
    if (sp)
    {
        p.px_off[0] = sp->off[0]; p.px_off[1] = sp->off[1];
        p.jitter = sp->jitter; p.blend = sp->blend; p.blend_s = sp->s; p.blend_d = sp->d;
        if (sp->inv_mats)
        {
            p.matrix_cam = 1u;
            std::memcpy(p.inv_view, sp->inv_mats, sizeof(p.inv_view));
            std::memcpy(p.inv_proj, sp->inv_mats + 16, sizeof(p.inv_proj));
        }
    }
    p.shard_index = sh.index; p.shard_count = sh.count; p.packed = sh.packed ? 1u : 0u;
    p.tiles_x = (cam->width + 7u) / 8u;
    p.num_tiles = local_bands * p.tiles_x;        // a band is one row of 8x8 tiles
    VRH_CHECK(uint64_t(p.num_tiles) * 64u * num_frames < (1ull << 32) && p.num_tiles < (1u << 26), "vrh_render: image too large");
    p.color = rt->color; p.prim_id = rt->prim_id; p.t = rt->t;
    p.occ = (k->flags & VRH_KERNEL_NO_OCC) ? nullptr : rt->occ;
    p.counters = ctx->counters;
    // tile queues: per-XCD strips; with frames in flight the band-interleaved order (auto) for AO
    // and for scenes larger than the 256 MB Infinity Cache.  Measured with a camera orbiting 0.5 deg
    // per frame (profiles/r02_ab/ab31_tile_order_orbit_*.log): band order hf10M AO +3.5 %, hf10M
    // primary +10 %, hf1M AO +0.3 %, but hf1M primary -2.8 % (its scene fits the MALL, and a
    // strip's primaries then keep their XCD's L2); one-frame launches keep strips (ab30)
    // AO with frames in flight: cluster order (every XCD on its own strip, the F frames of a cluster of
    // 8 tiles handed out back to back): against the band order, round 4, same box, 20 frames per
    // launch (profiles/r04/ab/cluster_hf{1M,10M}_{static,orbit}.log): hf10M +3.3 % (static camera) / +0.3 % (orbiting 0.5 deg per
    // frame), hf1M +0.9 % / +2.3 %; clusters of 4-16 tiles alike, 240 (a whole band) no gain
    const bool band_auto = num_frames > 1 && (lc.ao || sc->info.device_bytes > (256ull << 20));
    const bool cluster_auto = num_frames > 1 && lc.ao;
    p.xcd_queues = ctx->opt_xcd_queues == 2 ? 0u : ctx->opt_xcd_queues == 1 ? 1u
                 : ctx->opt_xcd_queues == 3 ? 2u : ctx->opt_xcd_queues == 4 ? 3u
                 : cluster_auto ? 3u : (band_auto ? 2u : 1u);
    p.cluster = ctx->opt_cluster ? uint32_t(ctx->opt_cluster) : 8u;
    if (shade)
    {
        p.shade.materials = k->shading->materials;
        p.shade.lights = k->shading->lights;
        p.shade.num_lights = k->shading->num_lights;
        p.shade.per_vertex = k->normal_binding == VRH_NORMALS_PER_VERTEX ? 1u : 0u;
        p.shade.vnormals = sc->vnormals;
        std::memcpy(p.shade.ambient, k->ambient, 16);
        for (int i = 0; i < 3; ++i) p.shade.amb[i] = p.shade.ambient[i] * p.shade.ambient[3];   // plastic.inl:13-16
    }
    p.num_bounces = whitted ? k->num_bounces : 0u;
    if (hmask && sc->info.prim_kind == VRH_PRIM_TRI64)
        p.hmask = dev::hit_mask_params{ hmask->tc, hmask->mask, hmask->w, hmask->h };
    if (multi)
    {
        p.max_hits = k->max_hits;
        p.mh_prim_id = rt->mh_prim_id;
        p.mh_t = rt->mh_t;
    }

    int per_cu = render_blocks_per_cu(lc);
    if (ctx->opt_bpc) per_cu = std::min(per_cu, ctx->opt_bpc);
    const int waves_per_block = lc.block / 64;
    const uint64_t units = uint64_t(num_frames) * p.num_tiles;
    int grid = std::max(1, int(std::min<uint64_t>(uint64_t(ctx->num_cus) * per_cu, (units + waves_per_block - 1) / waves_per_block)));

    // where the launch runs: the context stream with its counter / overflow blocks, or a frame lane
    hipStream_t S = ctx->stream;
    unsigned long long* ctr = ctx->counters;
    void** spill = &ctx->spill;
    size_t* spill_bytes = &ctx->spill_bytes;
    vrh_ctx::lane_t* L = nullptr;
    bool via_scratch = false;
    float4* dst_color = p.color; uint32_t* dst_pid = p.prim_id; float* dst_t = p.t; uint8_t* dst_occ = p.occ;
    if (async)
    {
        // cuda_sched issues a frame and returns (cuda_sched.inl:306-320): frames go round robin over the
        // frame lanes, so this frame's waves fill the CUs the earlier frames' launch tails leave idle
        const uint32_t li = ctx->next_lane;
        L = &ctx->lane[li];
        if (!L->stream)
        {
            VRH_HIP(hipStreamCreateWithFlags(&L->stream, hipStreamDefault));    // blocking: see vrh_ctx_create
            VRH_HIP(hipEventCreateWithFlags(&L->done, hipEventDisableTiming));
        }
        if (!ctx->main_mark) VRH_HIP(hipEventCreateWithFlags(&ctx->main_mark, hipEventDisableTiming));
        if (!rt->lane_written) VRH_HIP(hipEventCreateWithFlags(&rt->lane_written, hipEventDisableTiming));
        ctx->next_lane = (ctx->next_lane + 1u) % ctx->num_lanes;
        S = L->stream;
        ctr = L->counters;
        spill = &L->spill;
        spill_bytes = &L->spill_bytes;
        // after everything issued on the context stream before this call (clears, uploads, frames there)
        VRH_HIP(hipEventRecord(ctx->main_mark, ctx->stream));
        VRH_HIP(hipStreamWaitEvent(S, ctx->main_mark, 0));
        if (rt->written_pending) VRH_HIP(hipStreamWaitEvent(S, rt->written, 0));
        // a primary / AO frame of one image through a sampler that does not read the target writes every
        // field of the target at every pixel of its scissor box: it may go through the scratch target,
        // and it supersedes a pending scratch copy into this target of no larger box (that frame's pixels
        // would never be seen: they are dropped, not copied).  Any other pending copy into this target,
        // and one still in this lane's scratch target, is issued first.
        const bool scratch_ok = num_frames == 1 && (k->kind == VRH_KERNEL_PRIMARY || ao) && (!sp || sp->blend == 0);
        const uint32_t* cl = p.cam[0].clip;
        const bool fields[4] = { dst_color != nullptr, dst_pid != nullptr, dst_t != nullptr, dst_occ != nullptr };
        for (uint32_t l = 0; l < uint32_t(VRH_MAX_FRAME_LANES); ++l)
        {
            vrh_ctx::lane_t& Q = ctx->lane[l];
            if (!Q.pending_rt) continue;
            const uint32_t* qc = Q.pending_clip;
            const bool covers = Q.pending_rt == rt && scratch_ok && cl[0] <= qc[0] && cl[1] <= qc[1] && cl[2] >= qc[2]
                                && cl[3] >= qc[3] && fields[0] == Q.pending_fields[0] && fields[1] == Q.pending_fields[1]
                                && fields[2] == Q.pending_fields[2] && fields[3] == Q.pending_fields[3];
            if (covers) Q.pending_rt = nullptr;
            else if (Q.pending_rt == rt || l == li) VRH_HIP(ctx_flush_pending(ctx, int(l)));
        }
        // the target's last writer is the other lane, not yet joined: write order must hold.  A frame that
        // may go through the scratch target renders there now, and its copy becomes the lane's pending
        // copy (issued when something else needs the target, dropped when a later frame supersedes it);
        // anything else waits for that writer
        const bool other_writer = rt->lane >= 0 && rt->lane != int(li) && rt->lane_epoch == ctx->join_epoch;
        if (other_writer)
        {
            if (scratch_ok)
            {
                const size_t n = size_t(rt->width) * rt->height;
                if (n > L->pixels)
                {
                    VRH_HIP(hipStreamSynchronize(S));
                    for (void** q : { (void**)&L->color, (void**)&L->prim_id, (void**)&L->t, (void**)&L->occ })
                        if (*q) { (void)hipFree(*q); *q = nullptr; }
                    L->pixels = 0;
                    VRH_HIP(hipMalloc(&L->color, n * sizeof(float4)));
                    VRH_HIP(hipMalloc(&L->prim_id, n * sizeof(uint32_t)));
                    VRH_HIP(hipMalloc(&L->t, n * sizeof(float)));
                    VRH_HIP(hipMalloc(&L->occ, n));
                    L->pixels = n;
                }
                p.color = dst_color ? L->color : nullptr;
                p.prim_id = dst_pid ? L->prim_id : nullptr;
                p.t = dst_t ? L->t : nullptr;
                p.occ = dst_occ ? L->occ : nullptr;
                via_scratch = true;
            }
            else
                VRH_HIP(hipStreamWaitEvent(S, rt->lane_written, 0));
        }
    }
    p.counters = ctr;

    // the stack overflow blocks of the persistent grid (grown on demand; the stream is drained
    // first, so no launch still uses the old block)
    if (lc.spill)
    {
        const size_t bytes = size_t(grid) * (p.stack_total - p.stack_cap) * size_t(lc.block) * sizeof(uint32_t);
        if (bytes > *spill_bytes)
        {
            VRH_HIP(hipStreamSynchronize(S));
            if (*spill) (void)hipFree(*spill);
            *spill = nullptr;
            *spill_bytes = 0;
            VRH_HIP(hipMalloc(spill, bytes));
            *spill_bytes = bytes;
        }
        p.stack_spill = static_cast<uint32_t*>(*spill);
    }

    // per-wave timeline of this launch (diagnostic, VRH_OPT_WAVE_TIMES)
    ctx->wave_times_used = 0;
    if (ctx->opt_wave_times && (lc.sched == 0 || lc.sched == 3))
    {
        const size_t n = size_t(grid) * waves_per_block;
        if (n > ctx->wave_times_n)
        {
            VRH_HIP(hipStreamSynchronize(ctx->stream));
            if (ctx->wave_times) (void)hipFree(ctx->wave_times);
            ctx->wave_times = nullptr;
            ctx->wave_times_n = 0;
            VRH_HIP(hipMalloc(&ctx->wave_times, n * 2 * sizeof(unsigned long long)));
            ctx->wave_times_n = n;
        }
        p.wave_times = ctx->wave_times;
        ctx->wave_times_used = n;
    }
    ctx->tile_times_used = 0;
    if (ctx->opt_wave_times == 2 && lc.count && lc.ao && num_frames == 1 && p.num_tiles > 0)
    {
        if (p.num_tiles > ctx->tile_times_n)
        {
            VRH_HIP(hipStreamSynchronize(ctx->stream));
            if (ctx->tile_times) (void)hipFree(ctx->tile_times);
            ctx->tile_times = nullptr;
            ctx->tile_times_n = 0;
            VRH_HIP(hipMalloc(&ctx->tile_times, size_t(p.num_tiles) * 3 * sizeof(unsigned long long)));
            ctx->tile_times_n = p.num_tiles;
        }
        VRH_HIP(hipMemsetAsync(ctx->tile_times, 0, size_t(p.num_tiles) * 3 * sizeof(unsigned long long), ctx->stream));
        p.tile_times = ctx->tile_times;
        ctx->tile_times_used = p.num_tiles;
    }

    const uint32_t slot = ctx->frames % VRH_MAX_TIMED_FRAMES;
    while (ctx->ev_start.size() <= slot)
    {
        hipEvent_t a, b;
        VRH_HIP(hipEventCreate(&a));
        VRH_HIP(hipEventCreate(&b));
        ctx->ev_start.push_back(a);
        ctx->ev_stop.push_back(b);
    }
    VRH_HIP(hipMemsetAsync(ctr, 0, COUNTERS_FRAME * sizeof(unsigned long long), S));
    VRH_HIP(hipEventRecord(ctx->ev_start[slot], S));
    if (p.num_tiles > 0) VRH_HIP(launch_render(p, lc, grid, S));
    VRH_HIP(hipEventRecord(ctx->ev_stop[slot], S));
    if (async)
    {
        const uint32_t* cl = p.cam[0].clip;
        if (via_scratch)
        {
            // the scissor box of the scratch target -- every pixel a primary / AO frame writes -- is this
            // lane's pending copy into the target (ctx_flush_pending: after the target's previous writer)
            if (cl[2] > cl[0] && cl[3] > cl[1])
            {
                L->pending_rt = rt;
                for (int i = 0; i < 4; ++i) L->pending_clip[i] = cl[i];
                L->pending_fields[0] = dst_color != nullptr;
                L->pending_fields[1] = dst_pid != nullptr;
                L->pending_fields[2] = dst_t != nullptr;
                L->pending_fields[3] = dst_occ != nullptr;
            }
        }
        else
        {
            VRH_HIP(hipEventRecord(rt->lane_written, S));
            rt->lane = int(L - ctx->lane);
            rt->lane_epoch = ctx->join_epoch;
        }
        VRH_HIP(hipEventRecord(L->done, S));
        L->used = true;
    }
    else
        rt->lane = -1;
    ctx->last_counters = ctr;
    ctx->last_slot = slot;
    ctx->frames++;

    ctx->last = vrh_frame_stats{};
    ctx->last.launches = p.num_tiles > 0 ? 1u : 0u;
    ctx->last.grid_blocks = uint32_t(grid);
    ctx->last.block_threads = uint32_t(lc.block);
    ctx->last.stack_depth = p.stack_total;
    ctx->last.frames = num_frames;
    ctx->have_frame = true;
    return VRH_OK;
}
} // namespace

VRH_API int vrh_sync(vrh_ctx* ctx)
{
    VRH_CHECK(ctx, "vrh_sync: null");
    VRH_HIP(hipSetDevice(ctx->device));
    for (hipEvent_t ev : ctx->group_written) VRH_HIP(hipEventSynchronize(ev));
    return ctx_drain(ctx);
}

VRH_API int vrh_get_tile_times(vrh_ctx* ctx, uint64_t* out, uint64_t capacity, uint64_t* count)
{
    VRH_CHECK(ctx && count, "vrh_get_tile_times: null");
    VRH_HIP(hipSetDevice(ctx->device));
    VRH_HIP(hipStreamSynchronize(ctx->stream));
    *count = ctx->tile_times_used;
    if (out && ctx->tile_times_used)
        VRH_HIP(hipMemcpy(out, ctx->tile_times, std::min<uint64_t>(capacity, 3 * ctx->tile_times_used) * 8, hipMemcpyDeviceToHost));
    return VRH_OK;
}

VRH_API int vrh_ctx_user_queues(vrh_ctx* ctx, uint32_t** queues)
{
    VRH_CHECK(ctx && queues, "vrh_ctx_user_queues: null");
    if (!ctx->user_queues)
    {
        int rc = select_device(ctx);
        if (rc) return rc;
        VRH_HIP(hipMalloc(&ctx->user_queues, 8u * VRH_USER_QUEUE_STRIDE * sizeof(uint32_t)));
    }
    *queues = ctx->user_queues;
    return VRH_OK;
}

VRH_API int vrh_get_wave_times(vrh_ctx* ctx, uint64_t* out, uint64_t capacity, uint64_t* count, double* ticks_per_ms)
{
    VRH_CHECK(ctx && count, "vrh_get_wave_times: null");
    int rc = select_device(ctx);
    if (rc) return rc;
    if ((rc = ctx_drain(ctx))) return rc;
    *count = ctx->wave_times_used;
    if (ticks_per_ms)
    {
        int khz = 0;
        VRH_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
        *ticks_per_ms = double(khz);
    }
    if (out && ctx->wave_times_used)
        VRH_HIP(hipMemcpy(out, ctx->wave_times,
                          std::min<uint64_t>(capacity, 2 * ctx->wave_times_used) * 8,
                          hipMemcpyDeviceToHost));
    return VRH_OK;
}

VRH_API int vrh_last_frame_stats(vrh_ctx* ctx, vrh_frame_stats* stats)
{
    VRH_CHECK(ctx && stats, "vrh_last_frame_stats: null");
    VRH_CHECK(ctx->have_frame, "vrh_last_frame_stats: no frame rendered yet");
    int rc = select_device(ctx);
    if (rc) return rc;
    VRH_HIP(hipEventSynchronize(ctx->ev_stop[ctx->last_slot]));
    float ms = 0.0f;
    VRH_HIP(hipEventElapsedTime(&ms, ctx->ev_start[ctx->last_slot], ctx->ev_stop[ctx->last_slot]));
    unsigned long long c[COUNTERS_LINES + 10];
    VRH_HIP(hipMemcpy(c, ctx->last_counters, sizeof(c), hipMemcpyDeviceToHost));
    ctx->last.kernel_ms = ms;
    ctx->last.rays = c[1];
    ctx->last.hits = c[2];
    ctx->last.box_tests = c[3];
    ctx->last.prim_tests = c[4];
    ctx->last.wave_steps = c[6];
    ctx->last.busy_lane_steps = c[7];
    ctx->last.wave_box_iters = c[9];
    ctx->last.wave_prim_iters = c[10];
    ctx->last.wave_box_uniform_iters = c[11];
    ctx->last.l1_lines = c[COUNTERS_LINES];
    ctx->last.vmem_instrs = c[COUNTERS_LINES + 1];
    ctx->last.l1_requests = c[COUNTERS_LINES + 2];
    ctx->last.l1_group_accesses = c[COUNTERS_LINES + 3];
    ctx->last.l1_ideal_accesses = c[COUNTERS_LINES + 4];
    for (int k = 0; k < 5; ++k) ctx->last.l1_group_by_kind[k] = c[COUNTERS_LINES + 5 + k];
    *stats = ctx->last;
    if (c[5] & 1ull) { set_error("traversal step guard tripped: corrupt BVH (rays were cut short)"); return VRH_ERR_HIP; }
    return VRH_OK;
}

VRH_API int vrh_stats_reset(vrh_ctx* ctx)
{
    VRH_CHECK(ctx, "vrh_stats_reset: null");
    int rc = select_device(ctx);
    if (rc) return rc;
    if ((rc = ctx_drain(ctx))) return rc;
    for (int b = 0; b < COUNTER_BLOCKS; ++b)
        VRH_HIP(hipMemset(ctx->counters + size_t(b) * COUNTERS_WORDS + COUNTERS_TOTAL, 0, 16 * sizeof(unsigned long long)));
    ctx->frames = 0;
    return VRH_OK;
}

VRH_API int vrh_get_accum_stats(vrh_ctx* ctx, vrh_accum_stats* out)
{
    VRH_CHECK(ctx && out, "vrh_get_accum_stats: null");
    int rc = select_device(ctx);
    if (rc) return rc;
    if ((rc = ctx_drain(ctx))) return rc;
    vrh_accum_stats a{};
    a.frames = ctx->frames;
    a.timed_frames = std::min<uint32_t>(ctx->frames, VRH_MAX_TIMED_FRAMES);
    a.kernel_ms_min = 1e300;
    for (uint32_t i = 0; i < a.timed_frames; ++i)
    {
        float ms = 0.0f;
        VRH_HIP(hipEventElapsedTime(&ms, ctx->ev_start[i], ctx->ev_stop[i]));
        a.kernel_ms_total += ms;
        a.kernel_ms_min = std::min<double>(a.kernel_ms_min, ms);
        a.kernel_ms_max = std::max<double>(a.kernel_ms_max, ms);
    }
    if (a.timed_frames == 0) a.kernel_ms_min = 0.0;
    // first launch's start to the last launch's end: overlapping (asynchronous) frames count once
    // (asynchronous frames go round robin over the frame lanes: one of the last frames can end after the
    // last one, and a later frame can start before the first -- the span runs from the earliest start of
    // the first VRH_MAX_FRAME_LANES frames to the latest end of the last ones, measured from the first start)
    if (a.frames >= 1 && a.frames <= VRH_MAX_TIMED_FRAMES)
    {
        float end = -1e30f, begin = 0.0f;
        const uint32_t w = std::min<uint32_t>(a.frames, uint32_t(VRH_MAX_FRAME_LANES));
        for (uint32_t i = 0; i < w; ++i)
        {
            float e = 0.0f, s = 0.0f;
            VRH_HIP(hipEventElapsedTime(&e, ctx->ev_start[0], ctx->ev_stop[a.frames - 1 - i]));
            VRH_HIP(hipEventElapsedTime(&s, ctx->ev_start[0], ctx->ev_start[i]));
            end = std::max(end, e);
            begin = std::min(begin, s);
        }
        a.span_ms = double(end) - double(begin);
    }
    for (int b = 0; b < COUNTER_BLOCKS; ++b)
    {
        unsigned long long c[2];
        VRH_HIP(hipMemcpy(c, ctx->counters + size_t(b) * COUNTERS_WORDS + COUNTERS_TOTAL, sizeof(c), hipMemcpyDeviceToHost));
        a.rays += c[0];
        a.hits += c[1];
    }
    *out = a;
    return VRH_OK;
}

VRH_API int vrh_rt_download(vrh_ctx* ctx, vrh_rt* rt, void* color, uint32_t* prim_id, float* t, uint8_t* occ)
{
    VRH_CHECK(ctx && rt, "vrh_rt_download: null");
    int rc = select_device(ctx);
    if (rc) return rc;
    size_t n = size_t(rt->width) * rt->height;
    rc = rt_wait(ctx, rt);
    if (rc) return rc;
    VRH_HIP(hipStreamSynchronize(ctx->stream));
    if (color) { VRH_CHECK(rt->color, "vrh_rt_download: target has no colour buffer"); VRH_HIP(hipMemcpy(color, rt->color, n * 16, hipMemcpyDeviceToHost)); }
    if (prim_id) { VRH_CHECK(rt->prim_id, "vrh_rt_download: target has no prim_id buffer"); VRH_HIP(hipMemcpy(prim_id, rt->prim_id, n * 4, hipMemcpyDeviceToHost)); }
    if (t) { VRH_CHECK(rt->t, "vrh_rt_download: target has no t buffer"); VRH_HIP(hipMemcpy(t, rt->t, n * 4, hipMemcpyDeviceToHost)); }
    if (occ) { VRH_CHECK(rt->occ, "vrh_rt_download: target has no occlusion buffer"); VRH_HIP(hipMemcpy(occ, rt->occ, n, hipMemcpyDeviceToHost)); }
    return VRH_OK;
}

VRH_API int vrh_rt_alloc_multi_hit(vrh_ctx* ctx, vrh_rt* rt, uint32_t max_hits)
{
    VRH_CHECK(ctx && rt, "vrh_rt_alloc_multi_hit: null");
    VRH_CHECK(max_hits >= 1 && max_hits <= VRH_MAX_HITS, "vrh_rt_alloc_multi_hit: max_hits must be in [1, 16]");
    int rc = select_device(ctx);
    if (rc) return rc;
    if (rt->mh_prim_id) { (void)hipFree(rt->mh_prim_id); rt->mh_prim_id = nullptr; }
    if (rt->mh_t) { (void)hipFree(rt->mh_t); rt->mh_t = nullptr; }
    rt->mh_n = 0;
    const size_t n = size_t(rt->width) * rt->height * max_hits;
    VRH_HIP(hipMalloc(&rt->mh_prim_id, n * 4));
    VRH_HIP(hipMalloc(&rt->mh_t, n * 4));
    rt->mh_n = max_hits;
    return VRH_OK;
}

VRH_API int vrh_rt_download_multi_hit(vrh_ctx* ctx, vrh_rt* rt, uint32_t* prim_ids, float* t)
{
    VRH_CHECK(ctx && rt, "vrh_rt_download_multi_hit: null");
    VRH_CHECK(rt->mh_n, "vrh_rt_download_multi_hit: no multi-hit buffers (vrh_rt_alloc_multi_hit)");
    int rc = select_device(ctx);
    if (rc) return rc;
    const size_t n = size_t(rt->width) * rt->height * rt->mh_n;
    rc = rt_wait(ctx, rt);
    if (rc) return rc;
    VRH_HIP(hipStreamSynchronize(ctx->stream));
    if (prim_ids) VRH_HIP(hipMemcpy(prim_ids, rt->mh_prim_id, n * 4, hipMemcpyDeviceToHost));
    if (t) VRH_HIP(hipMemcpy(t, rt->mh_t, n * 4, hipMemcpyDeviceToHost));
    return VRH_OK;
}

VRH_API int vrh_rt_upload(vrh_ctx* ctx, vrh_rt* rt, const void* color, const uint32_t* prim_id, const float* t,
                          const uint8_t* occ)
{
    VRH_CHECK(ctx && rt, "vrh_rt_upload: null");
    int rc = select_device(ctx);
    if (rc) return rc;
    size_t n = size_t(rt->width) * rt->height;
    rc = rt_wait(ctx, rt);
    if (rc) return rc;
    VRH_HIP(hipStreamSynchronize(ctx->stream));
    if (color) { VRH_CHECK(rt->color, "vrh_rt_upload: target has no colour buffer"); VRH_HIP(hipMemcpy(rt->color, color, n * 16, hipMemcpyHostToDevice)); }
    if (prim_id) { VRH_CHECK(rt->prim_id, "vrh_rt_upload: target has no prim_id buffer"); VRH_HIP(hipMemcpy(rt->prim_id, prim_id, n * 4, hipMemcpyHostToDevice)); }
    if (t) { VRH_CHECK(rt->t, "vrh_rt_upload: target has no t buffer"); VRH_HIP(hipMemcpy(rt->t, t, n * 4, hipMemcpyHostToDevice)); }
    if (occ) { VRH_CHECK(rt->occ, "vrh_rt_upload: target has no occlusion buffer"); VRH_HIP(hipMemcpy(rt->occ, occ, n, hipMemcpyHostToDevice)); }
    return VRH_OK;
}

VRH_API int vrh_unshard(vrh_ctx* ctx, uint32_t width, uint32_t height, uint32_t count, const void* gcolor,
                        const uint32_t* gpid, const uint8_t* gocc, uint64_t stride, const vrh_kernel_desc* k,
                        vrh_rt* dst)
{
    VRH_CHECK(ctx && dst && count >= 1, "vrh_unshard: bad argument");
    VRH_CHECK(dst->width == width && dst->height == height, "vrh_unshard: destination size mismatch");
    VRH_CHECK(gcolor || !dst->color || (gpid && k), "vrh_unshard: colour needs either gathered colour or prim ids + kernel");
    VRH_CHECK(gcolor || !dst->color || k->kind < VRH_KERNEL_SIMPLE,
              "vrh_unshard: shaded colour cannot be re-derived; gather the colour buffer");
    VRH_CHECK(gcolor || !dst->color || k->kind != VRH_KERNEL_AO || (gocc && k->samples <= 8),
              "vrh_unshard: re-deriving AO colour needs the gathered masks and samples <= 8");
    int rc = select_device(ctx);
    if (rc) return rc;
    if ((rc = rt_wait(ctx, dst))) return rc;
    unshard_params u{};
    u.width = width; u.height = height; u.count = count;
    u.rows_per_shard = VRH_BAND_ROWS * vrh_shard_bands(height, 0, count);
    const uint64_t n = uint64_t(u.rows_per_shard) * width;
    u.gcolor = static_cast<const char*>(gcolor);
    u.gpid = reinterpret_cast<const char*>(gpid);
    u.gocc = reinterpret_cast<const char*>(gocc);
    u.stride_color = stride ? stride : 16 * n;
    u.stride_pid = stride ? stride : 4 * n;
    u.stride_occ = stride ? stride : n;
    u.color = dst->color; u.pid = dst->prim_id; u.occ = dst->occ;
    u.clip[0] = 0; u.clip[1] = 0; u.clip[2] = width; u.clip[3] = height;
    if (k)
    {
        u.ao = k->kind == VRH_KERNEL_AO ? 1u : 0u;
        u.samples = k->samples ? k->samples : 1u;
        std::memcpy(u.bg, k->bg, 16);
    }
    VRH_HIP(launch_unshard(u, ctx->stream));
    return VRH_OK;
}

VRH_API int vrh_build_bvh(const void* prims, uint32_t num_prims, uint32_t kind, void* nodes_out,
                          uint32_t* num_nodes_out, uint32_t* indices_out, uint32_t* max_depth_out)
{
    VRH_CHECK(prims && nodes_out && num_nodes_out && indices_out, "vrh_build_bvh: null argument");
    VRH_CHECK(num_prims >= 1, "vrh_build_bvh: no primitives");
    VRH_CHECK(kind == VRH_PRIM_TRI64 || kind == VRH_PRIM_SPHERE48, "vrh_build_bvh: unknown prim kind");
    try
    {
        return build_bvh(prims, num_prims, kind, static_cast<node32*>(nodes_out), num_nodes_out, indices_out, max_depth_out);
    }
    catch (const std::bad_alloc&) { set_error("vrh_build_bvh: out of host memory"); return VRH_ERR_OOM; }
}

} // extern "C"
