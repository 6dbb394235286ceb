// visionaray_amd/csrc/vrh_kernels.hip -- traversal kernels for gfx950 (CDNA4).
//
// Replaces cuda_sched's render<<<grid,block>>> (cuda_sched.inl:53-153, one thread per pixel on a
// 2-D grid) with a persistent-thread design:
//   * the grid is sized to residency (CUs x resident blocks); every wave pulls 8x8 pixel tiles from
//     a device-wide atomic counter until the frame's tiles are exhausted (work stealing: the
//     tiled_sched.inl:194 fetch_add moved onto the GPU); a wave's 64 lanes are one 8x8 tile, so
//     the primary rays of a wave are coherent;
//   * each lane keeps its traversal stack in LDS (dynamic shared memory, column-major
//     [entry][lane] so a wave's pushes/pops are bank-conflict free); the stack capacity is chosen
//     per scene from the BVH depth (a depth-first traversal never holds more than depth entries);
//   * AO (ao/main.cpp:183-246) is fused: the tile's hit records are staged in LDS and its
//     hits x samples any-hit rays are generated on chip -- no ray buffer touches HBM.  Primary and
//     AO rays share one refilling loop: a lane whose ray terminates takes the next ray of the tile
//     at once (ballot + mbcnt compaction of the idle lanes), so the wave stays busy until the
//     tile's ray pool is empty.
#include "vrh_device.h"
#include "vrh_kernels.h"

namespace vrh {
namespace dev {

constexpr int TILE = 8;             // 8x8 pixels per wave
constexpr uint32_t BAND = VRH_BAND_ROWS;   // shard band height = one row of 8x8 tiles
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr int AO_REC_WORDS = 8;     // per hit slot: isect pos xyz, normal xyz, pixel index, lane
// per-wave AO area in LDS: 64 hit records + 64 occlusion masks
constexpr int AO_WAVE_WORDS = 64 * AO_REC_WORDS + 64;

// tile index -> (x, y) of lane, plus the output row (packed shards).  A band is one row of tiles.
__device__ __forceinline__ bool tile_pixel(const render_params& P, uint32_t tile, uint32_t lane,
                                           uint32_t& x, uint32_t& y, uint32_t& out_row)
{
    static_assert(BAND == TILE, "a shard band is one row of 8x8 tiles");
    uint32_t lb = tile / P.tiles_x;               // local band
    uint32_t tx = tile - lb * P.tiles_x;
    uint32_t band = lb * P.shard_count + P.shard_index;
    x = tx * TILE + (lane & 7u);
    uint32_t in_band = lane >> 3;
    y = band * BAND + in_band;
    out_row = P.packed ? lb * BAND + in_band : y;
    return x < P.width && y < P.height;
}

// sched_common.h:130-150 make_primary_ray_impl (pinhole, uniform pixel sampler)
__device__ __forceinline__ ray_t primary_ray(const render_params& P, uint32_t x, uint32_t y)
{
    float fx = (float)x, fy = (float)y;
    float u = 2.0f * (fx + 0.5f) / (float)P.width - 1.0f;
    float v = 2.0f * (fy + 0.5f) / (float)P.height - 1.0f;
    f3 cu = mk3(P.cam_u[0], P.cam_u[1], P.cam_u[2]);
    f3 cv = mk3(P.cam_v[0], P.cam_v[1], P.cam_v[2]);
    f3 cw = mk3(P.cam_w[0], P.cam_w[1], P.cam_w[2]);
    f3 dir = normalize((cu * u + cv * v) + cw);
    return make_ray(mk3(P.eye[0], P.eye[1], P.eye[2]), dir);
}

// Tile work queues.  The frame's tiles are split into 8 contiguous ranges (horizontal image
// strips); a wave first drains the range of the XCD it runs on (hardware register XCC_ID), so the
// BVH nodes of a strip stay in that XCD's L2, then steals from the other ranges in turn.  Which XCD
// a wave lands on only changes speed: every tile is handed out exactly once by one of the 8
// atomic heads.  Called by the whole wave; returns the tile or NONE when all ranges are empty.
struct tile_queue
{
    uint32_t q;       // range currently drained (wave-uniform)
    uint32_t tried;   // ranges found empty so far
};

__device__ __forceinline__ uint32_t xcc_id()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}

__device__ __forceinline__ tile_queue queue_init(const render_params& P)
{
    return tile_queue{ P.xcd_queues ? xcc_id() : 0u, 0u };
}

__device__ __forceinline__ uint32_t next_tile(const render_params& P, tile_queue& tq, uint32_t lane)
{
    const uint32_t nq = P.xcd_queues ? 8u : 1u;
    while (tq.tried < nq)
    {
        const uint32_t lo = (uint32_t)(((uint64_t)P.num_tiles * tq.q) / nq);
        const uint32_t hi = (uint32_t)(((uint64_t)P.num_tiles * (tq.q + 1u)) / nq);
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(reinterpret_cast<uint32_t*>(P.counters + 8u + 8u * tq.q), 1u);
        t = __shfl(t, 0);
        if (lo + t < hi) return lo + t;
        tq.q = (tq.q + 1u) % nq;
        tq.tried += 1u;
    }
    return NONE;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// AO ray j of the tile: hit slot j / S, sample j % S (ao/main.cpp:216-238 with the Appendix-A
// sampler); returns the ray and the slot.
__device__ __forceinline__ ray_t ao_ray(const render_params& P, const float* recs, uint32_t j, uint32_t S,
                                        uint32_t& slot, uint32_t& s)
{
    slot = j / S;
    s = j - slot * S;
    const float* sr = recs + slot * AO_REC_WORDS;
    f3 pos = mk3(sr[0], sr[1], sr[2]);
    f3 n = mk3(sr[3], sr[4], sr[5]);
    uint32_t p = __float_as_uint(sr[6]);
    // vector3.inl:357-367 make_orthonormal_basis(u, v, w = n)
    f3 bv = fabsf(n.x) > fabsf(n.y) ? normalize(mk3(-n.z, 0.0f, n.x)) : normalize(mk3(0.0f, n.z, -n.y));
    f3 bu = cross(bv, n);
    f3 d = ao_direction(p, s, bu, bv, n);
    return make_ray(pos + d * P.eps, d);
}

// One refilling loop per wave.  Primary rays (one per pixel of the wave's tile)
// and AO rays (published as soon as their primary hit is known) are stepped by the same
// instruction stream (ray_step); a lane that finishes a ray immediately takes the next one, so
// neither the primary phase nor the AO phase waits for its slowest lane.  Without AO the wave
// streams pixels tile after tile and writes each pixel when its ray finishes.
template <int KIND, bool AO, bool COUNT, int OCC>
__global__ __launch_bounds__(256, OCC) void render_unified_kernel(render_params P)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = tid >> 6;
    const uint32_t block = blockDim.x;

    lds_stack st;
    st.mem = smem;
    st.base = tid;
    st.stride = block;
    st.top = tid;
    uint32_t* ao_area = smem + P.stack_cap * block + wave * AO_WAVE_WORDS;
    float* recs = reinterpret_cast<float*>(ao_area);
    uint32_t* masks = ao_area + 64 * AO_REC_WORDS;
    test_counts cnt = {};
    uint64_t rays_total = 0, hits_total = 0;

    // lane state: the ray it is stepping
    constexpr uint32_t IDLE = 0, PRIMARY = 1, AORAY = 2;
    uint32_t mode = IDLE;
    ray_t r;
    float best_t = FMAX, max_t = FMAX;
    uint32_t best_prim = 0, steps = 0;
    bool any = false;

    if constexpr (!AO)
    {
        // ---- primary visibility: stream pixels, write each when its ray finishes ------------
        tile_queue tq = queue_init(P);
        uint32_t tile = next_tile(P, tq, lane);
        uint32_t handed = 0;                       // pixels of `tile` handed out (wave-uniform)
        uint32_t out_o = 0;
        for (;;)
        {
            uint64_t idle = __ballot(mode == IDLE);
            if (idle)
            {
                if (handed >= 64u && tile != NONE)
                {
                    tile = next_tile(P, tq, lane);
                    handed = 0;
                }
                if (tile != NONE)
                {
                    uint32_t cand = handed + lane_rank(idle);
                    handed = min(64u, handed + (uint32_t)__popcll(idle));
                    if (mode == IDLE && cand < 64u)
                    {
                        uint32_t x, y, orow;
                        if (tile_pixel(P, tile, cand, x, y, orow))
                        {
                            r = primary_ray(P, x, y);
                            out_o = orow * P.width + x;
                            best_t = FMAX; best_prim = 0; steps = 0;
                            st.reset(); st.push(P.root);
                            mode = PRIMARY;
                            rays_total += 1;
                        }
                    }
                }
            }
            if (__ballot(mode != IDLE) == 0ull)
            {
                if (tile == NONE) break;
                continue;
            }
            const bool busy = mode != IDLE;
            if (mode != IDLE)
            {
                int rc = (P.fast_ok && __ballot(!finite_ray(r)) == 0ull)
                    ? ray_step<KIND, COUNT, true>(P.pairs, P.prims, r, FMAX, false, st, best_t, best_prim, cnt, steps, P.step_limit)
                    : ray_step<KIND, COUNT, false>(P.pairs, P.prims, r, FMAX, false, st, best_t, best_prim, cnt, steps, P.step_limit);
                if (rc != 0)
                {
                    bool hit = best_t != FMAX;
                    hits_total += hit ? 1 : 0;
                    if (P.color) P.color[out_o] = hit ? make_float4(1.0f, 1.0f, 1.0f, 1.0f) : make_float4(P.bg[0], P.bg[1], P.bg[2], P.bg[3]);
                    if (P.prim_id) P.prim_id[out_o] = hit ? best_prim : 0xFFFFFFFFu;
                    if (P.t) P.t[out_o] = hit ? best_t : -1.0f;
                    if (P.occ) P.occ[out_o] = 0;
                    mode = IDLE;
                }
            }
            if (COUNT) count_wave(cnt, busy);
        }
    }
    else
    {
        const uint32_t S = P.samples;
        tile_queue tq = queue_init(P);
        for (;;)
        {
            const uint32_t tile = next_tile(P, tq, lane);
            if (tile == NONE) break;

            uint32_t x, y, orow;
            const bool valid = tile_pixel(P, tile, lane, x, y, orow);
            // own pixel's results
            bool my_hit = false, just_done = false;
            uint32_t my_prim = 0xFFFFFFFFu, my_slot = 0;
            float my_t = -1.0f;
            if (valid)
            {
                r = primary_ray(P, x, y);
                best_t = FMAX; best_prim = 0; steps = 0; max_t = FMAX; any = false;
                st.reset(); st.push(P.root);
                mode = PRIMARY;
            }
            uint32_t pending = (uint32_t)__popcll(__ballot(valid));   // primaries not yet finished
            rays_total += valid ? 1 : 0;
            uint32_t published = 0, issued = 0;                        // hit slots, AO rays handed out
            uint32_t cur_slot = 0, cur_s = 0;
            for (;;)
            {
                // 1. publish primaries that finished last iteration (compacted hit slots)
                const uint64_t fin = __ballot(just_done);
                if (fin)
                {
                    const uint64_t hfin = __ballot(just_done && my_hit);
                    if (just_done && my_hit)
                    {
                        my_slot = published + lane_rank(hfin);
                        f3 pos = r.ori + r.dir * my_t;                  // ao/main.cpp:202
                        float4 nn = P.normals[my_prim];                  // get_normal.h:26-37
                        float* rec = recs + my_slot * AO_REC_WORDS;
                        rec[0] = pos.x; rec[1] = pos.y; rec[2] = pos.z;
                        rec[3] = nn.x; rec[4] = nn.y; rec[5] = nn.z;
                        rec[6] = __uint_as_float(y * P.width + x);       // global pixel index p
                        masks[my_slot] = 0u;
                    }
                    published += (uint32_t)__popcll(hfin);
                    pending -= (uint32_t)__popcll(fin);
                    just_done = false;
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                }
                // 2. hand the published AO rays to idle lanes
                const uint32_t avail = published * S;
                const uint64_t idle = __ballot(mode == IDLE);
                if (idle && issued < avail)
                {
                    uint32_t cand = issued + lane_rank(idle);
                    issued = min(avail, issued + (uint32_t)__popcll(idle));
                    if (mode == IDLE && cand < avail)
                    {
                        r = ao_ray(P, recs, cand, S, cur_slot, cur_s);
                        best_t = FMAX; best_prim = 0; steps = 0; max_t = P.radius; any = true;
                        st.reset(); st.push(P.root);
                        mode = AORAY;
                        rays_total += 1;
                    }
                }
                // 3. done when nothing is in flight and nothing is left to hand out
                if (__ballot(mode != IDLE) == 0ull && pending == 0u && issued >= avail) break;
                // 4. one traversal step for every busy lane (same code for both ray kinds)
                const bool busy = mode != IDLE;
                if (mode != IDLE)
                {
                    int rc = (P.fast_ok && __ballot(!finite_ray(r)) == 0ull)
                        ? ray_step<KIND, COUNT, true>(P.pairs, P.prims, r, max_t, any, st, best_t, best_prim, cnt, steps, P.step_limit)
                        : ray_step<KIND, COUNT, false>(P.pairs, P.prims, r, max_t, any, st, best_t, best_prim, cnt, steps, P.step_limit);
                    if (rc != 0)
                    {
                        if (mode == PRIMARY)
                        {
                            my_hit = best_t != FMAX;
                            my_prim = my_hit ? best_prim : 0xFFFFFFFFu;
                            my_t = my_hit ? best_t : -1.0f;
                            just_done = true;
                        }
                        else if (rc > 0)
                        {
                            atomicOr(&masks[cur_slot], 1u << cur_s);
                        }
                        mode = IDLE;
                    }
                }
                if (COUNT) count_wave(cnt, busy);
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (valid)
            {
                float4 color = make_float4(P.bg[0], P.bg[1], P.bg[2], P.bg[3]);
                uint32_t occ_mask = 0;
                if (my_hit)
                {
                    occ_mask = masks[my_slot];
                    float clr = 1.0f;
                    const float step = 1.0f / (float)S;
                    for (uint32_t s2 = 0; s2 < S; ++s2)
                        if ((occ_mask >> s2) & 1u) clr = clr - step;     // ao/main.cpp:234-238
                    color = make_float4(clr, clr, clr, 1.0f);
                    hits_total += 1;
                }
                size_t o = (size_t)orow * P.width + x;
                if (P.color) P.color[o] = color;
                if (P.prim_id) P.prim_id[o] = my_prim;
                if (P.t) P.t[o] = my_t;
                if (P.occ) P.occ[o] = (uint8_t)occ_mask;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }

    // ---- per-wave totals: one atomic set per wave --------------------------------------------
    unsigned long long rr = rays_total, hh = hits_total, b = cnt.box, q = cnt.prim;
    for (int off = 32; off > 0; off >>= 1)
    {
        rr += __shfl_down(rr, off);
        hh += __shfl_down(hh, off);
        if (COUNT) { b += __shfl_down(b, off); q += __shfl_down(q, off); }
    }
    if (__ballot(cnt.aborted) != 0ull && lane == 0) atomicOr(P.counters + 5, 1ull);
    if (lane == 0)
    {
        atomicAdd(P.counters + 1, rr);
        atomicAdd(P.counters + 2, hh);
        atomicAdd(P.counters + COUNTERS_TOTAL, rr);
        atomicAdd(P.counters + COUNTERS_TOTAL + 1, hh);
        if (COUNT)
        {
            atomicAdd(P.counters + 3, b);
            atomicAdd(P.counters + 4, q);
            atomicAdd(P.counters + 6, (unsigned long long)cnt.w_steps);    // wave-uniform values
            atomicAdd(P.counters + 7, (unsigned long long)cnt.w_busy);
            atomicAdd(P.counters + 9, (unsigned long long)cnt.w_box);
            atomicAdd(P.counters + 10, (unsigned long long)cnt.w_prim);
        }
    }
}

// un-interleave gathered packed shards [count][rows_per_shard][W] into the full image; without a
// gathered colour, re-derive it from prim id + AO mask exactly as the traversal kernel writes it
__global__ void unshard_kernel(unshard_params u)
{
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (x >= u.width || y >= u.height) return;
    uint32_t band = y / BAND;
    uint32_t g = band % u.count;
    uint32_t lrow = (band / u.count) * BAND + (y % BAND);
    size_t src = (size_t)lrow * u.width + x;
    size_t dst = (size_t)y * u.width + x;
    uint32_t pid = u.gpid ? reinterpret_cast<const uint32_t*>(u.gpid + g * u.stride_pid)[src] : 0xFFFFFFFFu;
    uint32_t occ = u.gocc ? (u.gocc + g * u.stride_occ)[src] : 0u;
    if (u.pid && u.gpid) u.pid[dst] = pid;
    if (u.occ && u.gocc) u.occ[dst] = (uint8_t)occ;
    if (!u.color) return;
    if (u.gcolor) { u.color[dst] = reinterpret_cast<const float4*>(u.gcolor + g * u.stride_color)[src]; return; }
    float4 c = make_float4(u.bg[0], u.bg[1], u.bg[2], u.bg[3]);
    if (pid != 0xFFFFFFFFu)
    {
        float clr = 1.0f;
        if (u.ao)
        {
            const float step = 1.0f / (float)u.samples;
            for (uint32_t s = 0; s < u.samples && s < 8u; ++s)
                if ((occ >> s) & 1u) clr = clr - step;           // ao/main.cpp:234-238
        }
        c = make_float4(clr, clr, clr, 1.0f);
    }
    u.color[dst] = c;
}

} // namespace dev

// ------------------------------------------------------------------------------------------------

using kernel_fn = void (*)(render_params);

template <int KIND, int OCC>
static kernel_fn pick_occ(bool ao, bool count)
{
    if (!ao) return count ? dev::render_unified_kernel<KIND, false, true, OCC> : dev::render_unified_kernel<KIND, false, false, OCC>;
    return count ? dev::render_unified_kernel<KIND, true, true, OCC> : dev::render_unified_kernel<KIND, true, false, OCC>;
}

template <int KIND>
static kernel_fn pick(bool ao, bool count, int occ)
{
    if (occ == 8) return pick_occ<KIND, 8>(ao, count);
    if (occ == 6) return pick_occ<KIND, 6>(ao, count);
    return pick_occ<KIND, 1>(ao, count);
}

static kernel_fn select_variant(const launch_config& c)
{
    return c.kind == dev::KIND_TRI ? pick<dev::KIND_TRI>(c.ao, c.count, c.occ)
                                   : pick<dev::KIND_SPHERE>(c.ao, c.count, c.occ);
}

size_t render_lds_bytes(const launch_config& c)
{
    size_t words = size_t(c.stack_cap) * c.block + (c.ao ? size_t(c.block / 64) * dev::AO_WAVE_WORDS : 0);
    return words * 4;
}

hipError_t launch_render(const render_params& p, const launch_config& c, int grid, hipStream_t s)
{
    hipLaunchKernelGGL(select_variant(c), dim3(grid), dim3(c.block), render_lds_bytes(c), s, p);
    return hipGetLastError();
}

int render_blocks_per_cu(const launch_config& c)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, select_variant(c), c.block, render_lds_bytes(c)) != hipSuccess)
        return 1;
    return n > 0 ? n : 1;
}

hipError_t launch_unshard(const unshard_params& u, hipStream_t s)
{
    dim3 block(256), grid((u.width + 255) / 256, u.height);
    hipLaunchKernelGGL(dev::unshard_kernel, grid, block, 0, s, u);
    return hipGetLastError();
}

} // namespace vrh
