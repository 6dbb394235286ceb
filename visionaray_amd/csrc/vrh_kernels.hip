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
// Per-wave AO area in LDS.  A wave keeps up to two tiles in flight: the current tile C (primaries
// and AO rays being handed out) and the draining tile D (all its AO rays handed out, some still
// being traced).  Hit records (isect position, face normal) are read only when an AO ray is handed
// out, so one set serves C; occlusion masks and the slot -> pixel map live until a tile finishes,
// so there are two of each, indexed by the tile's buffer parity.
constexpr int AO_REC_WORDS = 4;                         // pos xyz, prim id (its normal is re-read per AO ray:
                                                        // 512 B less LDS per wave = 24 instead of 22 waves/CU)
constexpr int AO_MASKS = 64 * AO_REC_WORDS;             // u32 masks[2][64]
constexpr int AO_SLOT_PX = AO_MASKS + 2 * 64;           // u8 slot_px[2][64]: pixel (lane) of a hit slot
constexpr int AO_WAVE_WORDS = AO_SLOT_PX + 2 * 64 / 4;

// tile id (next_tile: frame f << TILE_FRAME_SHIFT | tile of that frame) -> (x, y) of lane, plus the
// output row (frame f's rows start at f * frame_rows; packed shards).  A band is one row of tiles.
constexpr uint32_t TILE_FRAME_SHIFT = 26;   // frames < 64, tiles of one frame < 2^26
constexpr uint32_t TILE_MASK = (1u << TILE_FRAME_SHIFT) - 1u;
__device__ __forceinline__ bool tile_pixel(const render_params& P, uint32_t id, uint32_t lane,
                                           uint32_t& x, uint32_t& y, uint32_t& out_row, uint32_t& f)
{
    static_assert(BAND == TILE, "a shard band is one row of 8x8 tiles");
    f = id >> TILE_FRAME_SHIFT;
    const uint32_t tile = id & TILE_MASK;
    uint32_t lb = tile / P.tiles_x;               // local band
    uint32_t tx = tile - lb * P.tiles_x;
    uint32_t band = lb * P.shard_count + P.shard_index;
    x = tx * TILE + (lane & 7u);
    uint32_t in_band = lane >> 3;
    y = band * BAND + in_band;
    out_row = f * P.frame_rows + (P.packed ? lb * BAND + in_band : y);
    return x < P.width && y < P.height;
}

__device__ __forceinline__ bool tile_pixel(const render_params& P, uint32_t unit, uint32_t lane,
                                           uint32_t& x, uint32_t& y, uint32_t& out_row)
{
    uint32_t f;
    return tile_pixel(P, unit, lane, x, y, out_row, f);
}

// sched_common.h:130-150 make_primary_ray_impl (pinhole, uniform pixel sampler), frame f's camera
__device__ __forceinline__ ray_t primary_ray(const render_params& P, uint32_t f, uint32_t x, uint32_t y)
{
    const frame_camera& c = P.cam[f];
    float fx = (float)x, fy = (float)y;
    float u = 2.0f * (fx + 0.5f) / (float)P.width - 1.0f;
    float v = 2.0f * (fy + 0.5f) / (float)P.height - 1.0f;
    f3 cu = mk3(c.cam_u[0], c.cam_u[1], c.cam_u[2]);
    f3 cv = mk3(c.cam_v[0], c.cam_v[1], c.cam_v[2]);
    f3 cw = mk3(c.cam_w[0], c.cam_w[1], c.cam_w[2]);
    f3 dir = normalize((cu * u + cv * v) + cw);
    return make_ray(mk3(c.eye[0], c.eye[1], c.eye[2]), dir);
}

// Tile work queues.  A frame's tiles are split into 8 contiguous ranges (horizontal image strips);
// queue q hands out strip q of frame 0, then strip q of frame 1, ... (frames of one launch,
// vrh_render_batch).  A wave first drains the queue of the XCD it runs on (hardware register
// XCC_ID), so the BVH nodes of a strip stay in that XCD's L2, then steals from the other queues in
// turn -- a wave never idles while another frame of the launch still has tiles.  Which XCD a wave
// lands on only changes speed: every (frame, tile) is handed out exactly once by one of the 8
// atomic heads.  Called by the whole wave; returns the tile id (frame << TILE_FRAME_SHIFT | tile)
// or NONE when all queues are empty.
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

// first tile of strip q of a frame (num_tiles * q / nq)
__device__ __forceinline__ uint32_t strip_lo(const render_params& P, uint32_t q, uint32_t nq)
{
    return (uint32_t)(((uint64_t)P.num_tiles * q) / nq);
}

__device__ __forceinline__ uint32_t next_tile(const render_params& P, tile_queue& tq, uint32_t lane)
{
    const uint32_t nq = P.xcd_queues ? 8u : 1u;
    while (tq.tried < nq)
    {
        const uint32_t lo = strip_lo(P, tq.q, nq);
        const uint32_t len = strip_lo(P, tq.q + 1u, nq) - lo;
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(reinterpret_cast<uint32_t*>(P.counters + 8u + 8u * tq.q), 1u);
        t = __shfl(t, 0);
        if (t < len * P.num_frames)
        {
            const uint32_t f = t / len;
            return (f << TILE_FRAME_SHIFT) | (lo + t - f * len);
        }
        tq.q = (tq.q + 1u) % nq;
        tq.tried += 1u;
    }
    return NONE;
}

// two-pass AO: hit list q holds up to 64 records per (frame, tile) of queue q; its first slot
__device__ __forceinline__ uint32_t list_base(const render_params& P, uint32_t q, uint32_t nq)
{
    return 64u * P.num_frames * strip_lo(P, q, nq);
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// AO ray s of hit slot `slot` whose pixel has global index p (ao/main.cpp:216-238 with the
// Appendix-A sampler)
__device__ __forceinline__ ray_t ao_ray(const render_params& P, const float* recs, uint32_t slot, uint32_t s,
                                        uint32_t p)
{
    const float* sr = recs + slot * AO_REC_WORDS;
    f3 pos = mk3(sr[0], sr[1], sr[2]);
    const float4 nn = P.normals[__float_as_uint(sr[3])];              // get_normal.h:26-37
    f3 n = mk3(nn.x, nn.y, nn.z);
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
// EPI: primary-ray epilogue -- 0 colour = hit ? 1 : bg, 1 simple::kernel shading, 2 multi_hit<N>
// hit lists + the multi_hit example's compositing, 3 whitted::kernel (the lane traces its pixel's
// shadow and reflection rays one after the other before it takes the next pixel)
template <int KIND, bool AO, bool COUNT, int OCC, int EPI = 0>
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
    st.end = tid + P.stack_cap * block;
    uint32_t* ao_area = smem + P.stack_cap * block + wave * AO_WAVE_WORDS;
    test_counts cnt = {};
    uint64_t rays_total = 0, hits_total = 0;
    const hit_mask_params hml = P.hmask;          // a local copy: &P would spill the kernel arguments
    const hit_mask_params* hm = &hml;             // ray_step tests hm->mask

    // lane state: the ray it is stepping
    constexpr uint32_t IDLE = 0, PRIMARY = 1, AORAY = 2;
    uint32_t mode = IDLE;
    ray_t r;
    float best_t = FMAX, max_t = FMAX;
    uint32_t best_prim = 0, steps = 0;
    bool any = false, quad = false, finite = true;
    uint32_t resume = NO_RESUME;

    if constexpr (!AO)
    {
        // ---- primary visibility: stream pixels, write each when its ray finishes ------------
        tile_queue tq = queue_init(P);
        uint32_t tile = next_tile(P, tq, lane);
        uint32_t tile_q = tq.q;                    // the queue range `tile` came from (its hit list)
        uint32_t handed = 0;                       // pixels of `tile` handed out (wave-uniform)
        uint32_t out_o = 0;
        uint32_t lane_q = 0, lane_px = 0;          // EPI 4: hit list and image pixel of the lane's ray
        hit_extra hx = { 0.0f, 0.0f, 0u };
        mh_list mh;
        mh.mem = smem;
        mh.base = P.stack_cap * block + tid;
        mh.stride = block;
        mh.n = EPI == 2 ? P.max_hits : 1u;
        whitted_lane w;
        w.shadow = 0; w.depth = 0;
        for (;;)
        {
            uint64_t idle = __ballot(mode == IDLE);
            if ((uint32_t)__popcll(idle) < P.refill_min_primary && idle != ~0ull) idle = 0ull;
            if (idle)
            {
                if (handed >= 64u && tile != NONE)
                {
                    tile = next_tile(P, tq, lane);
                    tile_q = tq.q;
                    handed = 0;
                }
                if (tile != NONE)
                {
                    uint32_t cand = handed + lane_rank(idle);
                    handed = min(64u, handed + (uint32_t)__popcll(idle));
                    if (mode == IDLE && cand < 64u)
                    {
                        uint32_t x, y, orow, fr;
                        if (tile_pixel(P, tile, cand, x, y, orow, fr))
                        {
                            r = primary_ray(P, fr, x, y);
                            finite = finite_ray(r);
                            out_o = orow * P.width + x;
                            if constexpr (EPI == 4) { lane_q = tile_q; lane_px = y * P.width + x; }
                            best_t = FMAX; best_prim = 0; steps = 0;
                            if constexpr (EPI == 2) mh.reset();
                            if constexpr (EPI == 3)
                            {
                                w.color = mk3(0.0f, 0.0f, 0.0f); w.thr = 1.0f; w.depth = 0; w.shadow = 0;
                                max_t = FMAX; any = false; quad = false;
                            }
                            st.reset(); st.push(P.root); resume = NO_RESUME;
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
            bool publish = false;                  // EPI 4: this lane's primary hit becomes a record
            using ML = typename std::conditional<EPI == 2, mh_list, void>::type;
            constexpr bool UV = EPI == 1 || EPI == 3;
            const float mt = EPI == 3 ? max_t : FMAX;
            const bool an = EPI == 3 ? any : false;
            // cooperative pair fetch: every lane takes part (quad exchanges), idle lanes included
            int rc_coop = 0;
            if (COOP_FETCH && P.coop)
                rc_coop = (P.fast_ok && __ballot(busy && !finite) == 0ull)
                    ? ray_step_coop<KIND, COUNT, true, UV, ML>(busy, P.pairs, P.prims, P.root, r, mt, an, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, &hx, &mh, hm)
                    : ray_step_coop<KIND, COUNT, false, UV, ML>(busy, P.pairs, P.prims, P.root, r, mt, an, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, &hx, &mh, hm);
            if (mode != IDLE)
            {
                int rc = (COOP_FETCH && P.coop) ? rc_coop : (P.fast_ok && __ballot(!finite) == 0ull)
                    ? ray_step<KIND, COUNT, true, UV, ML>(P.pairs, P.prims, P.quads, P.root, quad, r, mt, an, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, &hx, &mh, hm)
                    : ray_step<KIND, COUNT, false, UV, ML>(P.pairs, P.prims, P.quads, P.root, quad, r, mt, an, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, &hx, &mh, hm);
                if constexpr (EPI == 3)
                {
                    if (rc != 0)
                    {
                        // whitted.inl:211-275: 0 = next ray set up, 1 = pixel done (colour in w)
                        int done = 0;
                        if (!w.shadow)
                        {
                            const bool hit = best_t != FMAX;
                            if (w.depth == 0u)
                            {
                                hits_total += hit ? 1 : 0;
                                if (P.prim_id) P.prim_id[out_o] = hit ? best_prim : 0xFFFFFFFFu;
                                if (P.t) P.t[out_o] = hit ? best_t : -1.0f;
                                if (P.occ) P.occ[out_o] = 0;
                                if (!hit)
                                {
                                    if (P.color) P.color[out_o] = make_float4(P.bg[0], P.bg[1], P.bg[2], P.bg[3]);
                                    mode = IDLE;
                                }
                            }
                            if (mode != IDLE)
                            {
                                // loop test: hit && throughput > epsilon && depth++ < num_bounces
                                if (hit && w.thr > P.eps && w.depth < P.num_bounces)
                                {
                                    w.depth += 1u;
                                    whitted_surface(P.shade, P.prims, P.normals, w, r, best_t, best_prim, hx);
                                }
                                else
                                    done = 1;
                            }
                        }
                        else
                            whitted_light_done(P.shade, w, rc > 0);
                        if (mode != IDLE && !done)
                        {
                            if (w.li < P.shade.num_lights)
                            {
                                r = whitted_shadow_ray(P.shade, w, P.eps, max_t);
                                any = true; w.shadow = 1;
                                finite = finite_ray(r);
                                quad = P.quad_ok && finite;
                            }
                            else
                            {
                                // color += shaded * throughput; the reflection ray is traced only
                                // if the next loop test can pass (its result is unused otherwise)
                                w.color = w.color + w.shaded * w.thr;
                                const float thr2 = w.thr * 0.1f;
                                if (thr2 > P.eps && w.depth < P.num_bounces)
                                {
                                    r = make_ray(w.pos + w.rdir * P.eps, w.rdir);
                                    w.thr = thr2; w.shadow = 0;
                                    max_t = FMAX; any = false; quad = false;
                                    finite = finite_ray(r);
                                }
                                else
                                    done = 1;
                            }
                            if (!done)
                            {
                                best_t = FMAX; best_prim = 0; steps = 0;
                                st.reset(); st.push(quad ? 0u : P.root); resume = NO_RESUME;
                                rays_total += 1;
                            }
                        }
                        if (done)
                        {
                            if (P.color) P.color[out_o] = make_float4(w.color.x, w.color.y, w.color.z, 1.0f);
                            mode = IDLE;
                        }
                    }
                }
                else if (rc != 0)
                {
                    if constexpr (EPI == 2)
                    {
                        // multi_hit: the list's first entry is the frame's prim id / t
                        for (uint32_t k = 0; k < mh.n; ++k)
                        {
                            const float tk = mh.t(k);
                            if (P.mh_prim_id) P.mh_prim_id[size_t(out_o) * mh.n + k] = tk < FMAX ? mh.at(1, k) : 0xFFFFFFFFu;
                            if (P.mh_t) P.mh_t[size_t(out_o) * mh.n + k] = tk < FMAX ? tk : -1.0f;
                        }
                        best_t = mh.t(0);
                        best_prim = mh.at(1, 0);
                    }
                    bool hit = best_t != FMAX;
                    hits_total += hit ? 1 : 0;
                    float4 c = hit ? make_float4(1.0f, 1.0f, 1.0f, 1.0f) : make_float4(P.bg[0], P.bg[1], P.bg[2], P.bg[3]);
                    if constexpr (EPI == 1)
                        if (hit) c = shade_simple(P.shade, P.prims, P.normals, r, best_t, best_prim, hx);
                    if constexpr (EPI == 2)
                        c = shade_multi(P.shade, P.prims, P.normals, r, mh);
                    // EPI 4: a hit pixel's colour and AO mask are written by the resolve pass
                    if (P.color && (EPI != 4 || !hit)) P.color[out_o] = c;
                    if (P.prim_id) P.prim_id[out_o] = hit ? best_prim : 0xFFFFFFFFu;
                    if (P.t) P.t[out_o] = hit ? best_t : -1.0f;
                    if (P.occ && (EPI != 4 || !hit)) P.occ[out_o] = 0;
                    if constexpr (EPI == 4) publish = hit;   // the ray state stays valid until the refill
                    mode = IDLE;
                }
            }
            if constexpr (EPI == 4)
            {
                // append the finished hits to their tiles' lists (one atomic per list and step):
                // record = (isect pos, image pixel) (face normal, output offset), ao/main.cpp:202,
                // get_normal.h:26-37
                uint64_t pend = __ballot(publish);
                while (pend)
                {
                    const uint32_t first = (uint32_t)__builtin_ctzll(pend);
                    const uint32_t q0 = __shfl(lane_q, first);
                    const bool mine = publish && lane_q == q0;
                    const uint64_t m = __ballot(mine);
                    uint32_t j0 = 0;
                    if (lane == first)
                        j0 = atomicAdd(reinterpret_cast<uint32_t*>(P.counters + COUNTERS_HITS + 8u * q0), (uint32_t)__popcll(m));
                    j0 = __shfl(j0, first);
                    if (mine)
                    {
                        const uint32_t rec = list_base(P, q0, P.xcd_queues ? 8u : 1u) + j0 + lane_rank(m);
                        const f3 pos = r.ori + r.dir * best_t;
                        const float4 nn = P.normals[best_prim];
                        P.hitrec[2u * rec] = make_float4(pos.x, pos.y, pos.z, __uint_as_float(lane_px));
                        P.hitrec[2u * rec + 1u] = make_float4(nn.x, nn.y, nn.z, __uint_as_float(out_o));
                    }
                    pend &= ~m;
                }
            }
            if (COUNT) count_wave(cnt, busy);
        }
    }
    else
    {
        // ---- primary + AO: one refilling loop over a stream of tiles, two tiles in flight ----
        const uint32_t S = P.samples;
        float* recs = reinterpret_cast<float*>(ao_area);
        uint32_t* masks = ao_area + AO_MASKS;
        uint8_t* slot_px = reinterpret_cast<uint8_t*>(ao_area + AO_SLOT_PX);
        const float4 bg = make_float4(P.bg[0], P.bg[1], P.bg[2], P.bg[3]);
        tile_queue tq = queue_init(P);
        // wave-uniform tile state
        uint32_t tileC = next_tile(P, tq, lane), parC = 0;
        uint32_t handedC = 0, pendC = 0, pubC = 0, issC = 0;  // primaries handed / in flight, slots, AO rays handed
        uint32_t tileD = NONE, parD = 0, slotsD = 0;
        uint32_t inflight0 = 0, inflight1 = 0;                // AO rays in flight per buffer parity
        // lane state: PRIMARY tag = pixel lane k of tile C; AORAY tag = slot | s << 6 | parity << 11
        uint32_t tag = 0;
        for (;;)
        {
            // 1. the draining tile is done when its last AO ray is: write its hit pixels
            if (tileD != NONE && (parD ? inflight1 : inflight0) == 0u)
            {
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (lane < slotsD)
                {
                    const uint32_t k = slot_px[parD * 64u + lane];
                    const uint32_t m = masks[parD * 64u + lane];
                    uint32_t x, y, orow;
                    tile_pixel(P, tileD, k, x, y, orow);
                    float clr = 1.0f;
                    const float step = 1.0f / (float)S;
                    for (uint32_t s2 = 0; s2 < S; ++s2)
                        if ((m >> s2) & 1u) clr = clr - step;                 // ao/main.cpp:234-238
                    const size_t o = (size_t)orow * P.width + x;
                    if (P.color) P.color[o] = make_float4(clr, clr, clr, 1.0f);
                    if (P.occ) P.occ[o] = (uint8_t)m;
                }
                __builtin_amdgcn_wave_barrier();
                tileD = NONE;
            }
            // 2. the current tile has handed out all its rays: it drains, the next tile starts
            if (tileC != NONE && tileD == NONE && handedC >= 64u && pendC == 0u && issC >= pubC * S)
            {
                tileD = tileC; parD = parC; slotsD = pubC;
                tileC = next_tile(P, tq, lane);
                parC ^= 1u;
                handedC = 0; pendC = 0; pubC = 0; issC = 0;
            }
            // 3. hand out rays to idle lanes: the current tile's AO rays, then its primaries --
            //    once P.refill_min lanes are idle (or none is busy), so ray generation runs with
            //    many lanes at once
            uint64_t idle = __ballot(mode == IDLE);
            if ((uint32_t)__popcll(idle) < P.refill_min && idle != ~0ull) idle = 0ull;
            if (idle && issC < pubC * S)
            {
                const uint32_t avail = pubC * S;
                const uint32_t cand = issC + lane_rank(idle);
                const uint32_t n = min(avail - issC, (uint32_t)__popcll(idle));
                if (mode == IDLE && cand < avail)
                {
                    const uint32_t slot = cand / S, smp = cand - slot * S;
                    uint32_t x, y, orow;
                    tile_pixel(P, tileC, slot_px[parC * 64u + slot], x, y, orow);
                    r = ao_ray(P, recs, slot, smp, y * P.width + x);
                    best_t = FMAX; best_prim = 0; steps = 0; max_t = P.radius; any = true;
                    finite = finite_ray(r);
                    quad = P.quad_ok && finite;
                    st.reset(); st.push(quad ? 0u : P.root); resume = NO_RESUME;
                    mode = AORAY;
                    tag = slot | (smp << 6) | (parC << 11);
                    rays_total += 1;
                }
                issC += n;
                if (parC) inflight1 += n; else inflight0 += n;
                idle = __ballot(mode == IDLE);
            }
            if (idle && tileC != NONE && handedC < 64u)
            {
                const uint32_t k = handedC + lane_rank(idle);
                handedC = min(64u, handedC + (uint32_t)__popcll(idle));
                uint32_t x, y, orow, fr;
                bool started = false;
                if (mode == IDLE && k < 64u && tile_pixel(P, tileC, k, x, y, orow, fr))
                {
                    r = primary_ray(P, fr, x, y);
                    finite = finite_ray(r);
                    best_t = FMAX; best_prim = 0; steps = 0; max_t = FMAX; any = false; quad = false;
                    st.reset(); st.push(P.root); resume = NO_RESUME;
                    mode = PRIMARY;
                    tag = k;
                    rays_total += 1;
                    started = true;
                }
                pendC += (uint32_t)__popcll(__ballot(started));
            }
            const bool busy = mode != IDLE;
            if (__ballot(busy) == 0ull)
            {
                if (tileC == NONE && tileD == NONE) break;
                continue;
            }
            // 4. one traversal step for every busy lane (same code for both ray kinds)
            int rc = 0;
            if (COOP_FETCH && P.coop)
            {
                // cooperative pair fetch: every lane takes part (quad exchanges), idle lanes included
                rc = (P.fast_ok && __ballot(busy && !finite) == 0ull)
                    ? ray_step_coop<KIND, COUNT, true>(busy, P.pairs, P.prims, P.root, r, max_t, any, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm)
                    : ray_step_coop<KIND, COUNT, false>(busy, P.pairs, P.prims, P.root, r, max_t, any, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm);
            }
            else if (busy)
            {
                rc = (P.fast_ok && __ballot(!finite) == 0ull)
                    ? ray_step<KIND, COUNT, true>(P.pairs, P.prims, P.quads, P.root, quad, r, max_t, any, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm)
                    : ray_step<KIND, COUNT, false>(P.pairs, P.prims, P.quads, P.root, quad, r, max_t, any, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm);
            }
            if (COUNT) count_wave(cnt, busy);
            // 5. finished AO rays: record occlusion, retire from their tile's in-flight count
            const bool ao_done = mode == AORAY && rc != 0;
            if (ao_done && rc > 0) atomicOr(&masks[(tag >> 11) * 64u + (tag & 63u)], 1u << ((tag >> 6) & 31u));
            inflight0 -= (uint32_t)__popcll(__ballot(ao_done && (tag >> 11) == 0u));
            inflight1 -= (uint32_t)__popcll(__ballot(ao_done && (tag >> 11) != 0u));
            // 6. finished primaries: write prim id / t (and a miss's colour), publish hits as slots
            const bool pr_done = mode == PRIMARY && rc != 0;
            const uint64_t fin = __ballot(pr_done);
            if (fin)
            {
                const bool hit = pr_done && best_t != FMAX;
                const uint64_t hfin = __ballot(hit);
                if (pr_done)
                {
                    uint32_t x, y, orow;
                    tile_pixel(P, tileC, tag, x, y, orow);
                    const size_t o = (size_t)orow * P.width + x;
                    if (P.prim_id) P.prim_id[o] = hit ? best_prim : 0xFFFFFFFFu;
                    if (P.t) P.t[o] = hit ? best_t : -1.0f;
                    if (hit)
                    {
                        const uint32_t slot = pubC + lane_rank(hfin);
                        const f3 pos = r.ori + r.dir * best_t;                   // ao/main.cpp:202
                        float* rec = recs + slot * AO_REC_WORDS;
                        rec[0] = pos.x; rec[1] = pos.y; rec[2] = pos.z;
                        rec[3] = __uint_as_float(best_prim);
                        masks[parC * 64u + slot] = 0u;
                        slot_px[parC * 64u + slot] = (uint8_t)tag;
                    }
                    else
                    {
                        if (P.color) P.color[o] = bg;
                        if (P.occ) P.occ[o] = 0;
                    }
                }
                pubC += (uint32_t)__popcll(hfin);
                pendC -= (uint32_t)__popcll(fin);
                hits_total += hit ? 1 : 0;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            }
            if (rc != 0) mode = IDLE;
        }
    }

    // ---- per-wave totals: one atomic set per wave --------------------------------------------
    unsigned long long rr = rays_total, hh = hits_total, b = cnt.box, q = cnt.prim, uni_sum = cnt.w_uni;
    for (int off = 32; off > 0; off >>= 1)
    {
        rr += __shfl_down(rr, off);
        hh += __shfl_down(hh, off);
        if (COUNT) { b += __shfl_down(b, off); q += __shfl_down(q, off); uni_sum += __shfl_down(uni_sum, off); }
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
            atomicAdd(P.counters + 11, (unsigned long long)uni_sum);
        }
    }
}

// Two-pass AO, pass 2: the AO rays of the hit lists pass 1 published (render_unified_kernel,
// EPI 4).  Ray g of list q = sample g % S of record g / S; lanes take rays straight from the list
// heads (one atomic per refill for all idle lanes of the wave), so the frame's AO work is shared
// out ray by ray instead of tile by tile: a shard of a few thousand tiles still keeps every wave
// of the chip busy to the end.  A wave drains the list of its own XCD first (the strip whose BVH
// nodes pass 1 left in that XCD's L2), then the others.  Same rays, same arithmetic and the same
// any-hit traversal as the fused kernel (ao/main.cpp:216-238), so the occlusion bits are equal.
template <int KIND, bool COUNT, int OCC>
__global__ __launch_bounds__(256, OCC) void ao_pass_kernel(render_params P)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t block = blockDim.x;

    lds_stack st;
    st.mem = smem;
    st.base = tid;
    st.stride = block;
    st.top = tid;
    st.end = tid + P.stack_cap * block;
    test_counts cnt = {};
    uint64_t rays_total = 0;
    const hit_mask_params hml = P.hmask;          // a local copy: &P would spill the kernel arguments
    const hit_mask_params* hm = &hml;             // ray_step tests hm->mask

    const uint32_t S = P.samples;
    const uint32_t nq = P.xcd_queues ? 8u : 1u;
    uint32_t q = P.xcd_queues ? xcc_id() : 0u, tried = 0;
    // hit records of list q: low word of the u64 counter COUNTERS_HITS + 8q (pass 1 is complete)
    auto hits = [&](uint32_t qq) { return *reinterpret_cast<const uint32_t*>(P.counters + COUNTERS_HITS + 8u * qq); };
    uint32_t total = hits(q) * S;                 // AO rays of list q

    bool busy = false, quad = false, finite = true;
    ray_t r;
    float best_t = FMAX;
    uint32_t best_prim = 0, steps = 0, resume = NO_RESUME, tag = 0;
    for (;;)
    {
        uint64_t idle = __ballot(!busy);
        if ((uint32_t)__popcll(idle) < P.refill_min && idle != ~0ull) idle = 0ull;
        while (idle && tried < nq)
        {
            const uint32_t n = (uint32_t)__popcll(idle);
            uint32_t a = 0;
            if (lane == 0) a = atomicAdd(reinterpret_cast<uint32_t*>(P.counters + COUNTERS_AOHEAD + 8u * q), n);
            a = __shfl(a, 0);
            const uint32_t take = a < total ? min(n, total - a) : 0u;
            const uint32_t cand = lane_rank(idle);
            if (!busy && cand < take)
            {
                const uint32_t g = a + cand;
                const uint32_t j = g / S, s = g - j * S;
                const uint32_t rec = list_base(P, q, nq) + j;
                const float4 r0 = P.hitrec[2u * rec], r1 = P.hitrec[2u * rec + 1u];
                const f3 pos = mk3(r0.x, r0.y, r0.z), nrm = mk3(r1.x, r1.y, r1.z);
                // vector3.inl:357-367 make_orthonormal_basis(u, v, w = n)
                const f3 bv = fabsf(nrm.x) > fabsf(nrm.y) ? normalize(mk3(-nrm.z, 0.0f, nrm.x)) : normalize(mk3(0.0f, nrm.z, -nrm.y));
                const f3 bu = cross(bv, nrm);
                const f3 d = ao_direction(__float_as_uint(r0.w), s, bu, bv, nrm);
                r = make_ray(pos + d * P.eps, d);
                best_t = FMAX; best_prim = 0; steps = 0;
                finite = finite_ray(r);
                quad = P.quad_ok && finite;
                st.reset(); st.push(quad ? 0u : P.root); resume = NO_RESUME;
                tag = rec * S + s;
                busy = true;
                rays_total += 1;
            }
            if (take == n) break;
            idle = __ballot(!busy);
            q = (q + 1u) % nq;                    // list q is exhausted: move on to the next
            tried += 1u;
            if (tried < nq) total = hits(q) * S;
        }
        if (__ballot(busy) == 0ull) break;        // every list exhausted, no ray in flight
        int rc = 0;
        if (COOP_FETCH && P.coop)
        {
            rc = (P.fast_ok && __ballot(busy && !finite) == 0ull)
                ? ray_step_coop<KIND, COUNT, true>(busy, P.pairs, P.prims, P.root, r, P.radius, true, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm)
                : ray_step_coop<KIND, COUNT, false>(busy, P.pairs, P.prims, P.root, r, P.radius, true, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm);
        }
        else if (busy)
        {
            rc = (P.fast_ok && __ballot(!finite) == 0ull)
                ? ray_step<KIND, COUNT, true>(P.pairs, P.prims, P.quads, P.root, quad, r, P.radius, true, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm)
                : ray_step<KIND, COUNT, false>(P.pairs, P.prims, P.quads, P.root, quad, r, P.radius, true, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm);
        }
        if (COUNT) count_wave(cnt, busy);
        if (busy && rc != 0)
        {
            P.aobits[tag] = rc > 0 ? 1u : 0u;
            busy = false;
        }
    }

    unsigned long long rr = rays_total, b = cnt.box, pq = cnt.prim, uni_sum = cnt.w_uni;
    for (int off = 32; off > 0; off >>= 1)
    {
        rr += __shfl_down(rr, off);
        if (COUNT) { b += __shfl_down(b, off); pq += __shfl_down(pq, off); uni_sum += __shfl_down(uni_sum, off); }
    }
    if (__ballot(cnt.aborted) != 0ull && lane == 0) atomicOr(P.counters + 5, 1ull);
    if (lane == 0)
    {
        atomicAdd(P.counters + 1, rr);
        atomicAdd(P.counters + COUNTERS_TOTAL, rr);
        if (COUNT)
        {
            atomicAdd(P.counters + 3, b);
            atomicAdd(P.counters + 4, pq);
            atomicAdd(P.counters + 6, (unsigned long long)cnt.w_steps);
            atomicAdd(P.counters + 7, (unsigned long long)cnt.w_busy);
            atomicAdd(P.counters + 9, (unsigned long long)cnt.w_box);
            atomicAdd(P.counters + 10, (unsigned long long)cnt.w_prim);
            atomicAdd(P.counters + 11, (unsigned long long)uni_sum);
        }
    }
}

// Two-pass AO, resolve: record slot -> colour 1 - k/S over the occluded samples in sample order
// (ao/main.cpp:234-238) and the sample mask, at the record's output offset
__global__ void ao_resolve_kernel(render_params P)
{
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= 64u * P.num_frames * P.num_tiles) return;
    const uint32_t nq = P.xcd_queues ? 8u : 1u;
    // list q owns record slots [64 F lo(q), 64 F lo(q + 1)), lo(q) = strip_lo(q), F = frames, so
    // slot / (64 F) is a tile of strip q
    const uint32_t tile = slot / (64u * P.num_frames);
    const uint32_t q = (uint32_t)((((uint64_t)tile + 1u) * nq - 1u) / P.num_tiles);
    const uint32_t j = slot - list_base(P, q, nq);
    if (j >= *reinterpret_cast<const uint32_t*>(P.counters + COUNTERS_HITS + 8u * q)) return;
    const uint32_t o = __float_as_uint(P.hitrec[2u * slot + 1u].w);
    const uint32_t S = P.samples;
    const uint8_t* bits = P.aobits + (size_t)slot * S;
    float clr = 1.0f;
    const float step = 1.0f / (float)S;
    uint32_t m = 0;
    for (uint32_t s = 0; s < S; ++s)
        if (bits[s]) { clr = clr - step; m |= 1u << s; }
    if (P.color) P.color[o] = make_float4(clr, clr, clr, 1.0f);
    if (P.occ) P.occ[o] = (uint8_t)m;
}

// ITEM schedule: the same ray streams as render_unified_kernel (two tiles in flight for AO), but
// a wave iterates on single traversal items (item_step: one node pair or one primitive per lane)
// instead of whole descend-to-leaf steps.  The vector-memory unit charges every wave-level load
// instruction whatever its active lanes, so what counts is how many lanes share each one: a lane
// that has reached a leaf tests its primitives while its neighbours are still descending.
// Finished rays are retired and idle lanes refilled only once at least P.refill_min lanes are
// free (or none is busy), so the ray-generation code runs with many lanes at once.
template <int KIND, bool AO, bool COUNT, int OCC, bool VOTE>
__global__ __launch_bounds__(256, OCC) void render_item_kernel(render_params P)
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
    st.end = tid + P.stack_cap * block;
    uint32_t* ao_area = smem + P.stack_cap * block + wave * AO_WAVE_WORDS;
    float* recs = reinterpret_cast<float*>(ao_area);
    uint32_t* masks = ao_area + AO_MASKS;
    uint8_t* slot_px = reinterpret_cast<uint8_t*>(ao_area + AO_SLOT_PX);
    test_counts cnt = {};
    uint64_t rays_total = 0, hits_total = 0;

    // lane state: mode = ray kind (PRIMARY / AORAY) | DONE once finished and not yet retired
    constexpr uint32_t IDLE = 0, PRIMARY = 1, AORAY = 2, DONE = 4;
    uint32_t mode = IDLE;
    ray_t r;
    float best_t = FMAX, max_t = FMAX;
    uint32_t best_prim = 0, steps = 0, item = 0;
    uint32_t tag = 0;        // PRIMARY: pixel lane k of tile C; AORAY: slot | s << 6 | parity << 11
    bool any = false, occl = false, finite = true;

    const uint32_t S = AO ? P.samples : 1u;
    const float4 bg = make_float4(P.bg[0], P.bg[1], P.bg[2], P.bg[3]);
    tile_queue tq = queue_init(P);
    uint32_t tileC = next_tile(P, tq, lane), parC = 0;
    uint32_t handedC = 0, pendC = 0, pubC = 0, issC = 0;
    uint32_t tileD = NONE, parD = 0, slotsD = 0;
    uint32_t inflight0 = 0, inflight1 = 0;

    for (;;)
    {
        uint64_t busy = __ballot(mode == PRIMARY || mode == AORAY);
        if (busy == 0ull || 64u - (uint32_t)__popcll(busy) >= P.refill_min)
        {
            // ---- A1. retire finished rays ------------------------------------------------------
            if constexpr (AO)
            {
                const bool ao_done = mode == (AORAY | DONE);
                if (ao_done && occl) atomicOr(&masks[(tag >> 11) * 64u + (tag & 63u)], 1u << ((tag >> 6) & 31u));
                inflight0 -= (uint32_t)__popcll(__ballot(ao_done && (tag >> 11) == 0u));
                inflight1 -= (uint32_t)__popcll(__ballot(ao_done && (tag >> 11) != 0u));
            }
            const bool pr_done = mode == (PRIMARY | DONE);
            const uint64_t fin = __ballot(pr_done);
            if (fin)
            {
                const bool hit = pr_done && best_t != FMAX;
                const uint64_t hfin = __ballot(hit);
                if (pr_done)
                {
                    // AO: tile C is still the primary's tile (it cannot drain while primaries are
                    // pending); primary only: tile C may have moved on, the lane kept its pixel
                    size_t o = tag;
                    if constexpr (AO)
                    {
                        uint32_t x, y, orow;
                        tile_pixel(P, tileC, tag, x, y, orow);
                        o = (size_t)orow * P.width + x;
                    }
                    if (P.prim_id) P.prim_id[o] = hit ? best_prim : 0xFFFFFFFFu;
                    if (P.t) P.t[o] = hit ? best_t : -1.0f;
                    if (AO && hit)
                    {
                        const uint32_t slot = pubC + lane_rank(hfin);
                        const f3 pos = r.ori + r.dir * best_t;                   // ao/main.cpp:202
                        float* rec = recs + slot * AO_REC_WORDS;
                        rec[0] = pos.x; rec[1] = pos.y; rec[2] = pos.z;
                        rec[3] = __uint_as_float(best_prim);
                        masks[parC * 64u + slot] = 0u;
                        slot_px[parC * 64u + slot] = (uint8_t)tag;
                    }
                    else
                    {
                        if (P.color) P.color[o] = hit ? make_float4(1.0f, 1.0f, 1.0f, 1.0f) : bg;
                        if (P.occ) P.occ[o] = 0;
                    }
                }
                if (AO) pubC += (uint32_t)__popcll(hfin);
                pendC -= (uint32_t)__popcll(fin);
                hits_total += hit ? 1 : 0;
            }
            if (mode & DONE) mode = IDLE;
            if constexpr (AO)
            {
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                // ---- A2. the draining tile is done when its last AO ray is retired -------------
                if (tileD != NONE && (parD ? inflight1 : inflight0) == 0u)
                {
                    if (lane < slotsD)
                    {
                        const uint32_t k = slot_px[parD * 64u + lane];
                        const uint32_t m = masks[parD * 64u + lane];
                        uint32_t x, y, orow;
                        tile_pixel(P, tileD, k, x, y, orow);
                        float clr = 1.0f;
                        const float step = 1.0f / (float)S;
                        for (uint32_t s2 = 0; s2 < S; ++s2)
                            if ((m >> s2) & 1u) clr = clr - step;             // ao/main.cpp:234-238
                        const size_t o = (size_t)orow * P.width + x;
                        if (P.color) P.color[o] = make_float4(clr, clr, clr, 1.0f);
                        if (P.occ) P.occ[o] = (uint8_t)m;
                    }
                    __builtin_amdgcn_wave_barrier();
                    tileD = NONE;
                }
                // ---- A3. the current tile has handed out every ray: it drains, the next starts -
                if (tileC != NONE && tileD == NONE && handedC >= 64u && pendC == 0u && issC >= pubC * S)
                {
                    tileD = tileC; parD = parC; slotsD = pubC;
                    tileC = next_tile(P, tq, lane);
                    parC ^= 1u;
                    handedC = 0; pendC = 0; pubC = 0; issC = 0;
                }
            }
            else
            {
                if (tileC != NONE && handedC >= 64u)
                {
                    tileC = next_tile(P, tq, lane);
                    handedC = 0;
                }
            }
            // ---- A4. hand out rays to idle lanes: the current tile's AO rays, then primaries ---
            uint64_t idle = __ballot(mode == IDLE);
            if (AO && idle && issC < pubC * S)
            {
                const uint32_t avail = pubC * S;
                const uint32_t cand = issC + lane_rank(idle);
                const uint32_t n = min(avail - issC, (uint32_t)__popcll(idle));
                if (mode == IDLE && cand < avail)
                {
                    const uint32_t slot = cand / S, smp = cand - slot * S;
                    uint32_t x, y, orow;
                    tile_pixel(P, tileC, slot_px[parC * 64u + slot], x, y, orow);
                    r = ao_ray(P, recs, slot, smp, y * P.width + x);
                    best_t = FMAX; best_prim = 0; steps = 0; max_t = P.radius; any = true; occl = false;
                    item = P.root; st.reset();
                    finite = finite_ray(r);
                    mode = AORAY;
                    tag = slot | (smp << 6) | (parC << 11);
                    rays_total += 1;
                }
                issC += n;
                if (parC) inflight1 += n; else inflight0 += n;
                idle = __ballot(mode == IDLE);
            }
            if (idle && tileC != NONE && handedC < 64u)
            {
                const uint32_t k = handedC + lane_rank(idle);
                handedC = min(64u, handedC + (uint32_t)__popcll(idle));
                uint32_t x, y, orow, fr;
                bool started = false;
                if (mode == IDLE && k < 64u && tile_pixel(P, tileC, k, x, y, orow, fr))
                {
                    r = primary_ray(P, fr, x, y);
                    best_t = FMAX; best_prim = 0; steps = 0; max_t = FMAX; any = false; occl = false;
                    item = P.root; st.reset();
                    finite = finite_ray(r);
                    mode = PRIMARY;
                    tag = AO ? k : orow * P.width + x;
                    rays_total += 1;
                    started = true;
                }
                pendC += (uint32_t)__popcll(__ballot(started));
            }
            busy = __ballot(mode == PRIMARY || mode == AORAY);
            if (busy == 0ull)
            {
                if (tileC == NONE && tileD == NONE) break;
                continue;
            }
        }
        // ---- B. one traversal item for every busy lane -------------------------------------------
        const bool my_busy = mode == PRIMARY || mode == AORAY;
        if constexpr (VOTE)
        {
            // the wave runs the node step or the primitive step, whichever more lanes wait for
            // (weighted by P.vote_leaf / 8): lanes of the other kind keep their item meanwhile
            const bool my_leaf = (item & LEAF_BIT) != 0u;
            const uint32_t nl = (uint32_t)__popcll(__ballot(my_busy && my_leaf));
            const uint32_t nn = (uint32_t)__popcll(__ballot(my_busy && !my_leaf));
            const bool leaf_turn = nn == 0u || nl * P.vote_leaf >= nn * 8u;
            bool done = false;
            if (leaf_turn)
            {
                if (my_busy && my_leaf)
                    done = prim_step<KIND, COUNT>(P.prims, r, max_t, any, st, item, best_t, best_prim, occl, cnt, steps, P.step_limit);
            }
            else
            {
                const bool fast = P.fast_ok && __ballot(my_busy && !my_leaf && !finite) == 0ull;
                if (my_busy && !my_leaf)
                    done = fast ? node_step<COUNT, true>(P.pairs, r, max_t, st, item, best_t, cnt, steps, P.step_limit)
                                : node_step<COUNT, false>(P.pairs, r, max_t, st, item, best_t, cnt, steps, P.step_limit);
            }
            if (done) mode |= DONE;
        }
        else
        {
            const bool fast = P.fast_ok && __ballot(my_busy && !finite) == 0ull;
            if (my_busy)
            {
                const bool done = fast
                    ? item_step<KIND, COUNT, true>(P.pairs, P.prims, r, max_t, any, st, item, best_t, best_prim, occl, cnt, steps, P.step_limit)
                    : item_step<KIND, COUNT, false>(P.pairs, P.prims, r, max_t, any, st, item, best_t, best_prim, occl, cnt, steps, P.step_limit);
                if (done) mode |= DONE;
            }
        }
        if (COUNT) count_wave(cnt, my_busy);
    }

    unsigned long long rr = rays_total, hh = hits_total, b = cnt.box, q = cnt.prim, uni_sum = cnt.w_uni;
    for (int off = 32; off > 0; off >>= 1)
    {
        rr += __shfl_down(rr, off);
        hh += __shfl_down(hh, off);
        if (COUNT) { b += __shfl_down(b, off); q += __shfl_down(q, off); uni_sum += __shfl_down(uni_sum, off); }
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
            atomicAdd(P.counters + 6, (unsigned long long)cnt.w_steps);
            atomicAdd(P.counters + 7, (unsigned long long)cnt.w_busy);
            atomicAdd(P.counters + 9, (unsigned long long)cnt.w_box);
            atomicAdd(P.counters + 10, (unsigned long long)cnt.w_prim);
            atomicAdd(P.counters + 11, (unsigned long long)uni_sum);
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
static kernel_fn pick_occ(bool ao, bool count, int sched)
{
    if (sched == 1)
    {
        if (!ao) return count ? dev::render_item_kernel<KIND, false, true, OCC, false> : dev::render_item_kernel<KIND, false, false, OCC, false>;
        return count ? dev::render_item_kernel<KIND, true, true, OCC, false> : dev::render_item_kernel<KIND, true, false, OCC, false>;
    }
    if (sched == 2)
    {
        if (!ao) return count ? dev::render_item_kernel<KIND, false, true, OCC, true> : dev::render_item_kernel<KIND, false, false, OCC, true>;
        return count ? dev::render_item_kernel<KIND, true, true, OCC, true> : dev::render_item_kernel<KIND, true, false, OCC, true>;
    }
    if (!ao) return count ? dev::render_unified_kernel<KIND, false, true, OCC> : dev::render_unified_kernel<KIND, false, false, OCC>;
    return count ? dev::render_unified_kernel<KIND, true, true, OCC> : dev::render_unified_kernel<KIND, true, false, OCC>;
}

// simple::kernel / multi_hit epilogues: triangles, step loop
template <int OCC>
static kernel_fn pick_shade(bool count, int epi)
{
    if (epi == 3)
        return count ? dev::render_unified_kernel<dev::KIND_TRI, false, true, OCC, 3>
                     : dev::render_unified_kernel<dev::KIND_TRI, false, false, OCC, 3>;
    if (epi == 2)
        return count ? dev::render_unified_kernel<dev::KIND_TRI, false, true, OCC, 2>
                     : dev::render_unified_kernel<dev::KIND_TRI, false, false, OCC, 2>;
    return count ? dev::render_unified_kernel<dev::KIND_TRI, false, true, OCC, 1>
                 : dev::render_unified_kernel<dev::KIND_TRI, false, false, OCC, 1>;
}

template <int KIND>
static kernel_fn pick(bool ao, bool count, int occ, int sched)
{
    if (occ == 8) return pick_occ<KIND, 8>(ao, count, sched);
    if (occ == 6) return pick_occ<KIND, 6>(ao, count, sched);
    if (occ == 5) return pick_occ<KIND, 5>(ao, count, sched);
    return pick_occ<KIND, 1>(ao, count, sched);
}

// two-pass AO, pass 1: primary visibility publishing hit records
template <int KIND>
static kernel_fn pick_publish(bool count, int occ)
{
    if (occ == 8) return count ? dev::render_unified_kernel<KIND, false, true, 8, 4> : dev::render_unified_kernel<KIND, false, false, 8, 4>;
    if (occ == 6) return count ? dev::render_unified_kernel<KIND, false, true, 6, 4> : dev::render_unified_kernel<KIND, false, false, 6, 4>;
    return count ? dev::render_unified_kernel<KIND, false, true, 1, 4> : dev::render_unified_kernel<KIND, false, false, 1, 4>;
}

template <int KIND>
static kernel_fn pick_ao_pass(bool count, int occ)
{
    if (occ == 8) return count ? dev::ao_pass_kernel<KIND, true, 8> : dev::ao_pass_kernel<KIND, false, 8>;
    if (occ == 6) return count ? dev::ao_pass_kernel<KIND, true, 6> : dev::ao_pass_kernel<KIND, false, 6>;
    return count ? dev::ao_pass_kernel<KIND, true, 1> : dev::ao_pass_kernel<KIND, false, 1>;
}

static kernel_fn select_variant(const launch_config& c)
{
    if (c.epi == 4) return c.kind == dev::KIND_TRI ? pick_publish<dev::KIND_TRI>(c.count, c.occ)
                                                   : pick_publish<dev::KIND_SPHERE>(c.count, c.occ);
    if (c.epi) return c.occ == 8 ? pick_shade<8>(c.count, c.epi) : c.occ == 6 ? pick_shade<6>(c.count, c.epi) : pick_shade<1>(c.count, c.epi);
    return c.kind == dev::KIND_TRI ? pick<dev::KIND_TRI>(c.ao, c.count, c.occ, c.sched)
                                   : pick<dev::KIND_SPHERE>(c.ao, c.count, c.occ, c.sched);
}

size_t render_lds_bytes(const launch_config& c)
{
    size_t words = size_t(c.stack_cap) * c.block + (c.ao ? size_t(c.block / 64) * dev::AO_WAVE_WORDS : 0)
                 + (c.epi == 2 ? size_t(5) * c.max_hits * c.block : 0);
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

size_t ao_pass_lds_bytes(const launch_config& c) { return size_t(c.stack_cap) * c.block * 4; }

static kernel_fn ao_pass_variant(const launch_config& c)
{
    return c.kind == dev::KIND_TRI ? pick_ao_pass<dev::KIND_TRI>(c.count, c.occ) : pick_ao_pass<dev::KIND_SPHERE>(c.count, c.occ);
}

hipError_t launch_ao_pass(const render_params& p, const launch_config& c, int grid, hipStream_t s)
{
    hipLaunchKernelGGL(ao_pass_variant(c), dim3(grid), dim3(c.block), ao_pass_lds_bytes(c), s, p);
    return hipGetLastError();
}

int ao_pass_blocks_per_cu(const launch_config& c)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ao_pass_variant(c), c.block, ao_pass_lds_bytes(c)) != hipSuccess)
        return 1;
    return n > 0 ? n : 1;
}

hipError_t launch_ao_resolve(const render_params& p, hipStream_t s)
{
    const uint32_t n = 64u * p.num_frames * p.num_tiles;
    hipLaunchKernelGGL(dev::ao_resolve_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_unshard(const unshard_params& u, hipStream_t s)
{
    dim3 block(256), grid((u.width + 255) / 256, u.height);
    hipLaunchKernelGGL(dev::unshard_kernel, grid, block, 0, s, u);
    return hipGetLastError();
}

} // namespace vrh
