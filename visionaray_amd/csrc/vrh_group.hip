// visionaray_amd/csrc/vrh_group.hip -- multi-GPU render groups (include/vrh.h vrh_group_*,
// vrh_render_sharded): image-tile shards rendered on every GPU of a group and gathered to rank 0
// over RCCL (xGMI point-to-point), SURVEY.md §8e.
//
// The reference has no multi-GPU path; what is lifted across devices is tiled_sched's tile
// distribution (tiled_sched.inl:24-25, 175-224: a frame's tiles handed to workers by an atomic
// counter).  Here a frame's 8-row bands are dealt round-robin to shards (band b -> shard b % S,
// interleaved so cheap sky rows and expensive terrain rows spread evenly), shard s is rendered by
// rank s % N (inside a GPU the persistent kernel's own tile queues distribute its bands), every
// shard is rendered packed (its bands back to back, vrh_render_batch with a packed vrh_shard), and
// the packed shards travel to rank 0 -- one ncclSend per shard, one ncclRecv per shard on the root,
// all in one ncclGroupStart/End -- where unshard_kernel lays the bands back into image order and
// re-derives the RGBA32F colour of the built-in kernels from prim id + AO mask (5 B / pixel on the
// wire instead of 20).  A rank may own several shards (S > N), so the whole path -- packed renders,
// the RCCL exchange, the un-interleave -- runs on a one-GPU box with a one-rank group.
//
// Streams: the shards render on the context's stream; the exchange and the un-interleave run on
// the group's own stream, ordered after the renders by an event, so frame batch k + 1 renders while
// batch k's shards are still on the wire (two staging slots; a slot is reused only after its
// previous exchange is done).  vrh_group_sync (or vrh_sync on the context after vrh_group_sync)
// waits for everything.
#include "vrh_objects.h"
#include "vrh_plan.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

using namespace vrh;

struct vrh_group
{
    vrh_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    uint32_t nranks = 1, rank = 0;
    hipStream_t stream = nullptr;          // exchange + un-interleave
    struct slot_t
    {
        hipEvent_t rendered = nullptr;     // on ctx->stream: this slot's shards are rendered
        hipEvent_t done = nullptr;         // on the group stream: this slot's exchange + un-interleave done
        uint8_t* send = nullptr;           // this rank's shards, back to back
        uint8_t* recv = nullptr;           // root: every shard, [S][shard bytes]
        size_t send_bytes = 0, recv_bytes = 0;
        bool used = false;
    } slot[2];
    uint32_t next = 0;
    uint8_t* work = nullptr;               // colour-only gathers: one shard's prim ids + AO masks before packing
    size_t work_bytes = 0;
    // failure containment (vrh.h vrh_group_join_timeout): a joined group's communicator is non-blocking
    // and every wait on a peer has a deadline; a group that missed one or saw an RCCL error is aborted
    bool nonblocking = false;
    bool failed = false;
    uint32_t timeout_ms = VRH_GROUP_TIMEOUT_MS;
};

namespace {

#define VRH_NCCL(call)                                                                             \
    do {                                                                                           \
        ncclResult_t r_ = (call);                                                                  \
        if (r_ != ncclSuccess) {                                                                   \
            set_error(std::string(#call) + ": " + ncclGetErrorString(r_));                        \
            return VRH_ERR_HIP;                                                                    \
        }                                                                                          \
    } while (0)

int group_init_common(vrh_group* g)
{
    VRH_HIP(hipSetDevice(g->ctx->device));
    VRH_HIP(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
    for (auto& s : g->slot)
    {
        VRH_HIP(hipEventCreateWithFlags(&s.rendered, hipEventDisableTiming));
        VRH_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    }
    return VRH_OK;
}

using plan::wire_layout;
using plan::layout_for;

using steady = std::chrono::steady_clock;

// abort the communicator (ncclCommAbort returns without the peers) and mark the group failed
int fail_group(vrh_group* g, int code, const std::string& msg)
{
    if (g->comm) { (void)ncclCommAbort(g->comm); g->comm = nullptr; }
    g->failed = true;
    set_error(msg);
    return code;
}

// poll between checks: yield (no sleep) for the first 2 s, so a finished exchange is seen within
// microseconds whatever the launch length (vrh_group_sync ends bench's timed region; a grouped C4
// launch is ~20-40 ms); past 2 s -- a slow or dead peer, not a timed wait -- sleep 50 us per check,
// an overshoot under 0.01 % of the wait
void poll_pause(steady::time_point t0)
{
    if (steady::now() - t0 < std::chrono::seconds(2)) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(50));
}

// the communicator's state until nothing is in progress (a non-blocking init, or the enqueue of a
// group of send / receive / broadcast calls), against the group's deadline
int wait_comm(vrh_group* g, const char* what)
{
    if (!g->comm) return VRH_OK;
    const auto t0 = steady::now();
    const auto deadline = t0 + std::chrono::milliseconds(g->timeout_ms);
    for (;;)
    {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(g->comm, &st);
        if (r != ncclSuccess) return fail_group(g, VRH_ERR_HIP, std::string(what) + ": ncclCommGetAsyncError: " + ncclGetErrorString(r));
        if (st == ncclSuccess) return VRH_OK;
        if (st != ncclInProgress) return fail_group(g, VRH_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(st));
        if (steady::now() > deadline)
            return fail_group(g, VRH_ERR_TIMEOUT, std::string(what) + ": no answer from a group peer within " +
                                                  std::to_string(g->timeout_ms) + " ms (communicator aborted)");
        poll_pause(t0);
    }
}

// the group's streams (and the context stream, ctx_too) until idle, watching the communicator for
// an asynchronous error, against the deadline -- in place of hipStreamSynchronize, which would wait
// forever for a receive whose sender died
int wait_streams(vrh_group* g, bool ctx_too, const char* what)
{
    VRH_HIP(hipSetDevice(g->ctx->device));
    if (ctx_too) VRH_HIP(ctx_join(g->ctx));
    const auto t0 = steady::now();
    const auto deadline = t0 + std::chrono::milliseconds(g->timeout_ms);
    for (;;)
    {
        bool busy = false;
        for (hipStream_t s : { ctx_too ? g->ctx->stream : nullptr, g->stream })
        {
            if (!s) continue;
            const hipError_t e = hipStreamQuery(s);
            if (e == hipErrorNotReady) busy = true;
            else if (e != hipSuccess)      // a device error: the group's exchanges cannot complete
                return fail_group(g, VRH_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
        }
        if (!busy) return VRH_OK;
        if (g->comm)
        {
            ncclResult_t st = ncclSuccess;
            if (ncclCommGetAsyncError(g->comm, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress)
                return fail_group(g, VRH_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(st));
        }
        if (steady::now() > deadline)
            return fail_group(g, VRH_ERR_TIMEOUT, std::string(what) + ": the exchange did not finish within " +
                                                  std::to_string(g->timeout_ms) + " ms (communicator aborted)");
        poll_pause(t0);
    }
}

#define VRH_GROUP_OK(g, what)                                                                      \
    do {                                                                                           \
        if ((g)->failed) { set_error(std::string(what) + ": the render group failed earlier"); return VRH_ERR_INVALID; } \
    } while (0)

// (re)allocate a staging buffer; an exchange or render still using the old one is waited for first
int grow(vrh_group* g, uint8_t*& p, size_t& have, size_t need)
{
    if (have >= need) return VRH_OK;
    const int rc = wait_streams(g, true, "vrh_render_sharded: staging");
    if (rc) return rc;
    if (p) { VRH_HIP(hipFree(p)); p = nullptr; have = 0; }
    VRH_HIP(hipMalloc(&p, need));
    have = need;
    return VRH_OK;
}


// what a scene replica needs to know before its arrays arrive (vrh_group_broadcast_scene)
struct scene_header
{
    uint64_t bytes[7];                 // pairs, prims, normals, quads, vnormals, dnodes, dindices
    uint32_t roots[vrh::MAX_LIST];
    uint32_t num_roots, num_pairs, quad_depth, finite_bounds;
    vrh_scene_info info;
};

// the device arrays of a scene, in scene_header::bytes order
inline void* const* scene_arrays(vrh_scene* sc, void* (&a)[7])
{
    a[0] = sc->pairs; a[1] = sc->prims; a[2] = sc->normals; a[3] = sc->quads;
    a[4] = sc->vnormals; a[5] = sc->dnodes; a[6] = sc->dindices;
    return a;
}

// allocation size of a device array (0 for null)
int array_bytes(void* p, uint64_t& out)
{
    out = 0;
    if (!p) return VRH_OK;
    size_t n = 0;
    VRH_HIP(hipMemPtrGetInfo(p, &n));
    out = n;
    return VRH_OK;
}

} // namespace

extern "C" {

VRH_API int vrh_group_get_id(vrh_group_id* id)
{
    VRH_CHECK(id, "vrh_group_get_id: null");
    static_assert(sizeof(vrh_group_id) == sizeof(ncclUniqueId), "group id = ncclUniqueId");
    ncclUniqueId u;
    VRH_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return VRH_OK;
}

VRH_API int vrh_group_join_timeout(vrh_ctx* ctx, uint32_t nranks, uint32_t rank, const vrh_group_id* id,
                                   uint32_t timeout_ms, vrh_group** out)
{
    VRH_CHECK(ctx && id && out && nranks >= 1 && rank < nranks, "vrh_group_join: bad argument");
    *out = nullptr;
    auto* g = new (std::nothrow) vrh_group;
    if (!g) { set_error("host allocation failed"); return VRH_ERR_OOM; }
    g->ctx = ctx; g->nranks = nranks; g->rank = rank;
    g->timeout_ms = timeout_ms ? timeout_ms : VRH_GROUP_TIMEOUT_MS;
    int rc = group_init_common(g);
    if (rc == VRH_OK)
    {
        // non-blocking communicator: the init returns at once (ncclInProgress) and is polled against
        // the deadline, so a peer that never joins gives an error instead of a hang
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        const ncclResult_t r = ncclCommInitRankConfig(&g->comm, int(nranks), u, int(rank), &cfg);
        if (r != ncclSuccess && r != ncclInProgress)
        {
            set_error(std::string("vrh_group_join: ncclCommInitRankConfig: ") + ncclGetErrorString(r));
            rc = VRH_ERR_HIP;
        }
        else
        {
            g->nonblocking = true;
            rc = wait_comm(g, "vrh_group_join");
        }
    }
    if (rc != VRH_OK)
    {
        const std::string msg = vrh_last_error();
        vrh_group_free(g);
        set_error(msg);
        return rc;
    }
    *out = g;
    return VRH_OK;
}

VRH_API int vrh_group_join(vrh_ctx* ctx, uint32_t nranks, uint32_t rank, const vrh_group_id* id, vrh_group** out)
{
    return vrh_group_join_timeout(ctx, nranks, rank, id, 0u, out);
}

VRH_API int vrh_group_set_timeout(vrh_group* g, uint32_t timeout_ms)
{
    VRH_CHECK(g && timeout_ms > 0, "vrh_group_set_timeout: bad argument");
    g->timeout_ms = timeout_ms;
    return VRH_OK;
}

VRH_API int vrh_group_failed(const vrh_group* g)
{
    return g && g->failed ? 1 : 0;
}

VRH_API int vrh_group_create_local(uint32_t ndev, vrh_ctx* const* ctxs, vrh_group** out)
{
    VRH_CHECK(ndev >= 1 && ctxs && out, "vrh_group_create_local: bad argument");
    std::vector<int> devs(ndev);
    for (uint32_t i = 0; i < ndev; ++i)
    {
        VRH_CHECK(ctxs[i], "vrh_group_create_local: null context");
        devs[i] = ctxs[i]->device;
        for (uint32_t j = 0; j < i; ++j) VRH_CHECK(devs[j] != devs[i], "vrh_group_create_local: one context per device");
        out[i] = nullptr;
    }
    std::vector<ncclComm_t> comms(ndev, nullptr);
    VRH_NCCL(ncclCommInitAll(comms.data(), int(ndev), devs.data()));
    int rc = VRH_OK;
    for (uint32_t i = 0; i < ndev && rc == VRH_OK; ++i)
    {
        auto* g = new (std::nothrow) vrh_group;
        if (!g) { set_error("host allocation failed"); rc = VRH_ERR_OOM; break; }
        g->ctx = ctxs[i]; g->comm = comms[i]; comms[i] = nullptr;
        g->nranks = ndev; g->rank = i;
        out[i] = g;
        rc = group_init_common(g);
    }
    if (rc != VRH_OK)
    {
        for (uint32_t i = 0; i < ndev; ++i) { vrh_group_free(out[i]); out[i] = nullptr; if (comms[i]) ncclCommDestroy(comms[i]); }
        return rc;
    }
    return VRH_OK;
}

VRH_API int vrh_group_info(const vrh_group* g, uint32_t* nranks, uint32_t* rank)
{
    VRH_CHECK(g, "vrh_group_info: null");
    if (nranks) *nranks = g->nranks;
    if (rank) *rank = g->rank;
    return VRH_OK;
}

VRH_API int vrh_group_sync(vrh_group* g)
{
    VRH_CHECK(g, "vrh_group_sync: null");
    VRH_GROUP_OK(g, "vrh_group_sync");
    return wait_streams(g, true, "vrh_group_sync");
}

VRH_API int vrh_group_free(vrh_group* g)
{
    if (!g) return VRH_OK;
    if (g->ctx) (void)hipSetDevice(g->ctx->device);
    if (!g->failed)
    {
        // the group's work first (with the deadline: a dead peer fails the group instead of hanging)
        if (g->ctx && g->stream) (void)wait_streams(g, true, "vrh_group_free");
        if (g->comm && g->nonblocking)
        {
            // a non-blocking communicator is finalized (polled like every wait) before it is destroyed
            const ncclResult_t r = ncclCommFinalize(g->comm);
            if (r != ncclSuccess && r != ncclInProgress) (void)fail_group(g, VRH_ERR_HIP, "vrh_group_free: ncclCommFinalize");
            else (void)wait_comm(g, "vrh_group_free");
        }
    }
    if (g->comm) (void)(g->failed ? ncclCommAbort(g->comm) : ncclCommDestroy(g->comm));
    for (auto& s : g->slot)
    {
        if (s.rendered) (void)hipEventDestroy(s.rendered);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.send) (void)hipFree(s.send);
        if (s.recv) (void)hipFree(s.recv);
    }
    if (g->work) (void)hipFree(g->work);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
    return VRH_OK;
}

VRH_API int vrh_render_sharded(uint32_t n, vrh_group* const* groups, const vrh_scene* const* scenes,
                               const vrh_kernel_desc* kernels, vrh_rt* dst, uint32_t fields,
                               const vrh_camera* cams, uint32_t num_frames, uint32_t frame_num, uint32_t shards)
{
    VRH_CHECK(n >= 1 && groups && scenes && kernels && cams, "vrh_render_sharded: null argument");
    VRH_CHECK(num_frames >= 1 && num_frames <= VRH_MAX_BATCH, "vrh_render_sharded: 1..VRH_MAX_BATCH frames");
    VRH_CHECK((fields & ~uint32_t(VRH_RT_ALL)) == 0 && fields != 0, "vrh_render_sharded: fields are vrh_rt_flags");
    const uint32_t N = groups[0] ? groups[0]->nranks : 0;
    const uint32_t S = shards ? shards : N;
    const uint32_t W = cams[0].width, H = cams[0].height;
    VRH_CHECK(S >= 1 && S <= 4096, "vrh_render_sharded: shard count");
    int root = -1;
    for (uint32_t i = 0; i < n; ++i)
    {
        VRH_CHECK(groups[i] && scenes[i] && groups[i]->nranks == N, "vrh_render_sharded: groups of one communicator");
        VRH_GROUP_OK(groups[i], "vrh_render_sharded");
        VRH_CHECK(scenes[i]->ctx == groups[i]->ctx, "vrh_render_sharded: scene i must live on group i's context");
        VRH_CHECK(kernels[i].kind == kernels[0].kind && kernels[i].samples == kernels[0].samples,
                  "vrh_render_sharded: one kernel for every rank");
        if (groups[i]->rank == 0) root = int(i);
    }
    const wire_layout wl = layout_for(fields, kernels[0]);
    if (root >= 0)
    {
        VRH_CHECK(dst && dst->ctx == groups[root]->ctx, "vrh_render_sharded: the root needs a target on its context");
        VRH_CHECK(dst->width == W && dst->height == H * num_frames, "vrh_render_sharded: target must be W x (H * frames)");
        VRH_CHECK((!(fields & VRH_RT_COLOR) || dst->color) && (!(fields & VRH_RT_PRIM_ID) || dst->prim_id) &&
                  (!(fields & VRH_RT_T) || dst->t) && (!(fields & VRH_RT_OCC) || dst->occ),
                  "vrh_render_sharded: the target lacks a buffer named in fields");
        VRH_CHECK(!(fields & VRH_RT_OCC) || kernels[0].kind != VRH_KERNEL_AO || kernels[0].samples <= 8,
                  "vrh_render_sharded: an occlusion target records at most 8 AO samples");
    }
    // packed shard geometry: every shard uses shard 0's (largest) band count
    const uint32_t rows = VRH_BAND_ROWS * plan::shard_bands(H, 0, S);
    const size_t px = size_t(rows) * W * num_frames;          // pixels of one shard (all frames)
    const plan::wire_offsets wo = plan::offsets_for(wl, px);
    const size_t shard_bytes = wo.shard_bytes;
    VRH_CHECK(shard_bytes > 0, "vrh_render_sharded: nothing to gather");
    const size_t o_pid = wo.pid, o_occ = wo.occ, o_t = wo.t, o_col = wo.col, o_code = wo.code;
    const bool ao = kernels[0].kind == VRH_KERNEL_AO;

    // 1. every local group renders its shards into this call's staging slot (context stream)
    std::vector<uint32_t> slot_of(n);
    for (uint32_t i = 0; i < n; ++i)
    {
        vrh_group* g = groups[i];
        vrh_ctx* ctx = g->ctx;
        VRH_HIP(hipSetDevice(ctx->device));
        VRH_HIP(ctx_join(ctx));                 // after the context's asynchronous frames
        const uint32_t si = g->next;
        g->next ^= 1u;
        slot_of[i] = si;
        auto& sl = g->slot[si];
        if (sl.used) VRH_HIP(hipStreamWaitEvent(ctx->stream, sl.done, 0));   // the slot's last exchange
        const uint32_t mine = plan::owned_count(S, N, g->rank);              // shards s = rank, rank + N, ...
        int rc = grow(g, sl.send, sl.send_bytes, std::max<size_t>(mine * shard_bytes, 1));
        if (!rc && g->rank == 0) rc = grow(g, sl.recv, sl.recv_bytes, S * shard_bytes);
        if (!rc && wl.code && mine) rc = grow(g, g->work, g->work_bytes, 5 * px);
        if (rc) return rc;
        for (uint32_t j = 0; j < mine; ++j)
        {
            const uint32_t s = plan::owned_shard(g->rank, N, j);
            uint8_t* base = sl.send + size_t(j) * shard_bytes;
            vrh_rt rt{};
            rt.ctx = ctx; rt.width = W; rt.height = rows * num_frames; rt.owned = false;
            rt.prim_id = wl.pid ? reinterpret_cast<uint32_t*>(base + o_pid) : nullptr;
            rt.occ = wl.occ ? base + o_occ : nullptr;
            rt.t = wl.t ? reinterpret_cast<float*>(base + o_t) : nullptr;
            rt.color = wl.color ? reinterpret_cast<float4*>(base + o_col) : nullptr;
            if (wl.code)
            {
                // rendered into the work buffer, packed to one byte per pixel below (same stream,
                // so the next shard's render starts after this pack)
                rt.prim_id = reinterpret_cast<uint32_t*>(g->work);
                rt.occ = ao ? g->work + 4 * px : nullptr;
            }
            vrh_shard sh{ s, S, 1u, 0u };
            // the staging AO masks are the group's own (the root re-derives the colour from them, or the
            // code byte is packed from them): a kernel that leaves the occlusion target out
            // (VRH_KERNEL_NO_OCC) still writes them -- it only may for <= 8 samples, and with more the
            // colour itself crosses the wire (layout_for), so rt.occ is null then
            vrh_kernel_desc kd = kernels[i];
            if (kd.kind == VRH_KERNEL_AO && kd.samples <= 8) kd.flags &= ~uint32_t(VRH_KERNEL_NO_OCC);
            rc = vrh_render_batch(ctx, scenes[i], &rt, cams, num_frames, &kd, &sh, frame_num);
            if (rc) return rc;
            if (wl.code)
                VRH_HIP(launch_pack_code(rt.prim_id, rt.occ, base + o_code, px, ctx->stream));
        }
        VRH_HIP(hipEventRecord(sl.rendered, ctx->stream));
        VRH_HIP(hipStreamWaitEvent(g->stream, sl.rendered, 0));
    }
    // 2. the exchange: every shard to the root, one send / receive pair per shard
    // (an error inside the group still closes it: the thread's next RCCL call must not join a stale group)
    VRH_NCCL(ncclGroupStart());
    ncclResult_t xr = ncclSuccess;
    for (uint32_t i = 0; i < n && xr == ncclSuccess; ++i)
    {
        vrh_group* g = groups[i];
        auto& sl = g->slot[slot_of[i]];
        const uint32_t mine = plan::owned_count(S, N, g->rank);
        for (uint32_t j = 0; j < mine && xr == ncclSuccess; ++j)
            xr = ncclSend(sl.send + size_t(j) * shard_bytes, shard_bytes, ncclUint8, 0, g->comm, g->stream);
        if (g->rank == 0)
            for (uint32_t s = 0; s < S && xr == ncclSuccess; ++s)
                xr = ncclRecv(sl.recv + size_t(s) * shard_bytes, shard_bytes, ncclUint8, int(plan::shard_owner(s, N)),
                              g->comm, g->stream);
    }
    const ncclResult_t xe = ncclGroupEnd();
    if (xr == ncclSuccess) xr = xe;
    if (xr != ncclSuccess && xr != ncclInProgress)
    {
        const std::string msg = std::string("vrh_render_sharded: exchange: ") + ncclGetErrorString(xr);
        for (uint32_t i = 0; i < n; ++i) (void)fail_group(groups[i], VRH_ERR_HIP, msg);
        return VRH_ERR_HIP;
    }
    // non-blocking communicators: the sends / receives are enqueued once nothing is in progress (the
    // first exchange with a peer connects to it -- a dead peer is caught here, at the deadline)
    for (uint32_t i = 0; i < n; ++i)
    {
        VRH_HIP(hipSetDevice(groups[i]->ctx->device));
        const int rc = wait_comm(groups[i], "vrh_render_sharded: exchange");
        if (rc) return rc;
    }
    // 3. the root lays the bands back into image order, frame by frame
    for (uint32_t i = 0; i < n; ++i)
    {
        vrh_group* g = groups[i];
        auto& sl = g->slot[slot_of[i]];
        VRH_HIP(hipSetDevice(g->ctx->device));
        if (g->rank == 0)
        {
            for (uint32_t f = 0; f < num_frames; ++f)
            {
                const unshard_params u = plan::frame_params(wl, wo, sl.recv, W, H, S, rows, f, fields, kernels[i],
                                                            dst->color, dst->prim_id, dst->occ, dst->t, cams[f].scissor);
                VRH_HIP(launch_unshard(u, g->stream));
            }
            // the target is written on the group's stream: its context's downloads, clears, renders
            // and vrh_sync wait for this event (rt_wait) without a host synchronisation
            VRH_HIP(mark_written(dst, g->stream));
        }
        VRH_HIP(hipEventRecord(sl.done, g->stream));
        sl.used = true;
    }
    return VRH_OK;
}

// ---- the plan as host functions (vrh.h; tests/test_multigpu_gloo.py drives them) ----------------

VRH_API uint32_t vrh_group_shards_of(uint32_t nranks, uint32_t rank, uint32_t shards, uint32_t* out, uint32_t cap)
{
    if (nranks == 0 || rank >= nranks) return 0;
    const uint32_t n = plan::owned_count(shards, nranks, rank);
    for (uint32_t j = 0; j < n && j < cap && out; ++j) out[j] = plan::owned_shard(rank, nranks, j);
    return n;
}

VRH_API uint32_t vrh_group_shard_owner(uint32_t nranks, uint32_t shard)
{
    return nranks ? plan::shard_owner(shard, nranks) : 0u;
}

VRH_API int vrh_group_wire_layout(uint32_t fields, const vrh_kernel_desc* k, uint32_t width, uint32_t height,
                                  uint32_t frames, uint32_t shards, vrh_wire_layout* out)
{
    VRH_CHECK(k && out && shards >= 1 && frames >= 1, "vrh_group_wire_layout: bad argument");
    const wire_layout wl = layout_for(fields, *k);
    const uint32_t rows = VRH_BAND_ROWS * plan::shard_bands(height, 0, shards);
    const plan::wire_offsets o = plan::offsets_for(wl, size_t(rows) * width * frames);
    const uint64_t none = ~0ull;
    out->prim_id = wl.pid ? o.pid : none;
    out->occ = wl.occ ? o.occ : none;
    out->t = wl.t ? o.t : none;
    out->color = wl.color ? o.col : none;
    out->code = wl.code ? o.code : none;
    out->shard_bytes = o.shard_bytes;
    out->rows = rows;
    out->derive = wl.derive ? 1u : 0u;
    return VRH_OK;
}

VRH_API int vrh_shard_packed_rows(uint32_t height, uint32_t shard, uint32_t shards, int32_t* rows_out)
{
    VRH_CHECK(rows_out && shards >= 1 && shard < shards, "vrh_shard_packed_rows: bad argument");
    const uint32_t rows = VRH_BAND_ROWS * plan::shard_bands(height, 0, shards);
    for (uint32_t r = 0; r < rows; ++r) rows_out[r] = -1;
    // the inverse of the kernel's packed row (tile_pixel: band lb * S + s, row lb * BAND + in_band),
    // from the root's side: every image row whose home is this shard
    for (uint32_t y = 0; y < height; ++y)
    {
        uint32_t s, lrow;
        plan::row_home(y, shards, s, lrow);
        if (s == shard && lrow < rows) rows_out[lrow] = int32_t(y);
    }
    return VRH_OK;
}

VRH_API int vrh_pack_codes_host(const uint32_t* prim_id, const uint8_t* occ, uint8_t* code, uint64_t n)
{
    VRH_CHECK((prim_id && code) || n == 0, "vrh_pack_codes_host: null argument");
    for (uint64_t i = 0; i < n; ++i) code[i] = plan::pack_code(prim_id[i], occ, size_t(i));
    return VRH_OK;
}

VRH_API int vrh_unshard_host(const void* gathered, const vrh_wire_layout* wire, uint32_t width, uint32_t height,
                             uint32_t shards, uint32_t frame, uint32_t fields, const vrh_kernel_desc* k,
                             void* color, uint32_t* prim_id, uint8_t* occ, float* t)
{
    VRH_CHECK(gathered && wire && k && shards >= 1 && width >= 1, "vrh_unshard_host: bad argument");
    const wire_layout wl = layout_for(fields, *k);
    VRH_CHECK(wl.bytes_per_px() > 0, "vrh_unshard_host: these fields put nothing on the wire");
    const uint32_t rows = VRH_BAND_ROWS * plan::shard_bands(height, 0, shards);
    VRH_CHECK(wire->rows == rows, "vrh_unshard_host: wire layout of another geometry");
    const size_t frames = rows ? size_t(wire->shard_bytes / (wl.bytes_per_px() * size_t(rows) * width)) : 0;
    VRH_CHECK(frame < frames, "vrh_unshard_host: frame out of range");
    const plan::wire_offsets o = plan::offsets_for(wl, size_t(rows) * width * frames);
    // the wire layout passed must be the one these fields and this kernel give (vrh_group_wire_layout)
    const uint64_t none = ~0ull;
    VRH_CHECK(wire->shard_bytes == o.shard_bytes && wire->prim_id == (wl.pid ? o.pid : none) &&
              wire->occ == (wl.occ ? o.occ : none) && wire->t == (wl.t ? o.t : none) &&
              wire->color == (wl.color ? o.col : none) && wire->code == (wl.code ? o.code : none),
              "vrh_unshard_host: wire layout of other fields or another kernel");
    const uint32_t whole[4] = { 0, 0, 0, 0 };
    // the destination buffers hold this one frame: frame_params offsets them by f * W * H, so step back
    const size_t fo = size_t(frame) * width * height;
    float4* c = color ? static_cast<float4*>(color) - fo : nullptr;
    uint32_t* p = prim_id ? prim_id - fo : nullptr;
    uint8_t* q = occ ? occ - fo : nullptr;
    float* tt = t ? t - fo : nullptr;
    const unshard_params u = plan::frame_params(wl, o, static_cast<const uint8_t*>(gathered), width, height, shards, rows,
                                                frame, fields, *k, c, p, q, tt, whole);
    for (uint32_t y = 0; y < height; ++y)
        for (uint32_t x = 0; x < width; ++x) plan::unshard_pixel(u, x, y);
    return VRH_OK;
}

VRH_API int vrh_group_broadcast_scene(uint32_t n, vrh_group* const* groups, const vrh_scene* root_scene, vrh_scene** out)
{
    VRH_CHECK(n >= 1 && groups && out, "vrh_group_broadcast_scene: null argument");
    int root = -1;
    for (uint32_t i = 0; i < n; ++i)
    {
        VRH_CHECK(groups[i] && groups[i]->nranks == groups[0]->nranks, "vrh_group_broadcast_scene: groups of one communicator");
        VRH_GROUP_OK(groups[i], "vrh_group_broadcast_scene");
        out[i] = nullptr;
        if (groups[i]->rank == 0) root = int(i);
    }
    VRH_CHECK(root < 0 || (root_scene && root_scene->ctx == groups[root]->ctx),
              "vrh_group_broadcast_scene: rank 0 passes its scene, on its context");
    // 1. the header, from rank 0's host to every member (a small device buffer per member)
    scene_header h{};
    if (root >= 0)
    {
        vrh_scene* rs = const_cast<vrh_scene*>(root_scene);
        void* a[7];
        scene_arrays(rs, a);
        for (int k = 0; k < 7; ++k)
        {
            const int rc = array_bytes(a[k], h.bytes[k]);
            if (rc) return rc;
        }
        std::memcpy(h.roots, rs->roots, sizeof(h.roots));
        h.num_roots = rs->num_roots; h.num_pairs = rs->num_pairs; h.quad_depth = rs->quad_depth;
        h.finite_bounds = rs->finite_bounds ? 1u : 0u;
        h.info = rs->info;
        // the scene's own uploads / builds on its context stream finish before the broadcast reads it
        VRH_HIP(hipSetDevice(rs->ctx->device));
        VRH_HIP(hipStreamSynchronize(rs->ctx->stream));
    }
    std::vector<scene_header*> dh(n, nullptr);
    auto free_headers = [&]() { for (uint32_t i = 0; i < n; ++i) if (dh[i]) { (void)hipSetDevice(groups[i]->ctx->device); (void)hipFree(dh[i]); } };
    int rc = VRH_OK;
    for (uint32_t i = 0; i < n && rc == VRH_OK; ++i)
    {
        vrh_group* g = groups[i];
        if (hipSetDevice(g->ctx->device) != hipSuccess || hipMalloc(&dh[i], sizeof(scene_header)) != hipSuccess ||
            (int(i) == root && hipMemcpy(dh[i], &h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess))
        { set_error("vrh_group_broadcast_scene: header buffer"); rc = VRH_ERR_HIP; }
    }
    if (rc == VRH_OK)
    {
        ncclResult_t r = ncclGroupStart();
        for (uint32_t i = 0; i < n && r == ncclSuccess; ++i)
            r = ncclBroadcast(dh[i], dh[i], sizeof(scene_header), ncclUint8, 0, groups[i]->comm, groups[i]->stream);
        const ncclResult_t r2 = ncclGroupEnd();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess && r != ncclInProgress) { set_error(std::string("vrh_group_broadcast_scene: header: ") + ncclGetErrorString(r)); rc = VRH_ERR_HIP; }
        for (uint32_t i = 0; i < n && rc == VRH_OK; ++i)
            if (hipSetDevice(groups[i]->ctx->device) == hipSuccess)
                rc = wait_comm(groups[i], "vrh_group_broadcast_scene: header");
    }
    std::vector<scene_header> hh(n);
    for (uint32_t i = 0; i < n && rc == VRH_OK; ++i)
    {
        vrh_group* g = groups[i];
        rc = wait_streams(g, false, "vrh_group_broadcast_scene: header");
        if (rc == VRH_OK && hipMemcpy(&hh[i], dh[i], sizeof(scene_header), hipMemcpyDeviceToHost) != hipSuccess)
        { set_error("vrh_group_broadcast_scene: header download"); rc = VRH_ERR_HIP; }
    }
    free_headers();
    if (rc) return rc;
    // 2. every member allocates its replica (rank 0 too: the replica is a new scene everywhere)
    auto free_out = [&]() { for (uint32_t i = 0; i < n; ++i) { vrh_scene_free(out[i]); out[i] = nullptr; } };
    for (uint32_t i = 0; i < n; ++i)
        VRH_CHECK(hh[i].num_roots >= 1 && hh[i].num_roots <= vrh::MAX_LIST, "vrh_group_broadcast_scene: bad header");
    for (uint32_t i = 0; i < n; ++i)
    {
        const scene_header& x = hh[i];
        auto* sc = new (std::nothrow) vrh_scene;
        if (!sc) { free_out(); set_error("host allocation failed"); return VRH_ERR_OOM; }
        out[i] = sc;
        sc->ctx = groups[i]->ctx;
        std::memcpy(sc->roots, x.roots, sizeof(sc->roots));
        sc->num_roots = x.num_roots; sc->num_pairs = x.num_pairs; sc->quad_depth = x.quad_depth;
        sc->finite_bounds = x.finite_bounds != 0;
        sc->info = x.info;
        void** dst[7] = { reinterpret_cast<void**>(&sc->pairs), reinterpret_cast<void**>(&sc->prims),
                          reinterpret_cast<void**>(&sc->normals), reinterpret_cast<void**>(&sc->quads),
                          reinterpret_cast<void**>(&sc->vnormals), reinterpret_cast<void**>(&sc->dnodes),
                          reinterpret_cast<void**>(&sc->dindices) };
        if (hipSetDevice(sc->ctx->device) != hipSuccess) { free_out(); set_error("hipSetDevice"); return VRH_ERR_HIP; }
        for (int k = 0; k < 7; ++k)
            if (x.bytes[k])
            {
                const hipError_t e = hipMalloc(dst[k], x.bytes[k]);
                if (e != hipSuccess)
                {
                    free_out();
                    set_error(std::string("vrh_group_broadcast_scene: hipMalloc: ") + hipGetErrorString(e));
                    return e == hipErrorOutOfMemory ? VRH_ERR_OOM : VRH_ERR_HIP;
                }
            }
    }
    // 3. the arrays: one broadcast per array from rank 0's scene into every replica
    {
        void* src[7] = {};
        if (root >= 0) scene_arrays(const_cast<vrh_scene*>(root_scene), src);
        ncclResult_t r = ncclGroupStart();
        for (uint32_t i = 0; i < n && r == ncclSuccess; ++i)
        {
            void* d[7];
            scene_arrays(out[i], d);
            for (int k = 0; k < 7 && r == ncclSuccess; ++k)
                if (hh[i].bytes[k])
                    r = ncclBroadcast(int(i) == root ? src[k] : d[k], d[k], hh[i].bytes[k], ncclUint8, 0, groups[i]->comm,
                                      groups[i]->stream);
        }
        const ncclResult_t r2 = ncclGroupEnd();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess && r != ncclInProgress) { free_out(); set_error(std::string("vrh_group_broadcast_scene: ") + ncclGetErrorString(r)); return VRH_ERR_HIP; }
        for (uint32_t i = 0; i < n; ++i)
        {
            int rc2 = hipSetDevice(groups[i]->ctx->device) == hipSuccess ? wait_comm(groups[i], "vrh_group_broadcast_scene")
                                                                         : VRH_ERR_HIP;
            if (rc2) { const std::string m = vrh_last_error(); free_out(); set_error(m); return rc2; }
        }
    }
    for (uint32_t i = 0; i < n; ++i)
    {
        const int rc2 = wait_streams(groups[i], false, "vrh_group_broadcast_scene");
        if (rc2) { const std::string m = vrh_last_error(); free_out(); set_error(m); return rc2; }
    }
    return VRH_OK;
}


} // extern "C"
