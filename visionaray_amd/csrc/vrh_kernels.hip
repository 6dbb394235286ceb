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
#include "visionaray_hip/detail/vrh_device.h"

#include <map>
#include <mutex>
#include <tuple>
#include "vrh_kernels.h"
#include "vrh_plan.h"

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
#ifndef VRH_AO_CUT
#define VRH_AO_CUT 1    // compile the AO entry cut in (render_params::ao_cut switches it per launch)
#endif
constexpr int AO_CUT = AO_SLOT_PX + 2 * 64 / 4;         // the current tile's entry cut (ao_cut_build)
#ifndef VRH_AO_CUT_SPILL
#define VRH_AO_CUT_SPILL 1   // 0: the cut only in the instances whose stack fits LDS (A/B)
#endif
#ifndef VRH_AO_CUT_MAX
#define VRH_AO_CUT_MAX 8
#endif
// the AO kernel's lane state: 1 = max_t derived from `any` (AO rays: the radius, primaries: max())
#ifndef VRH_AO_LEAN
#define VRH_AO_LEAN 1
#endif
// 1 = the AO instances honour a descent cap (VRH_OPT_DESCENT_CAP; measured no gain on AO, round 4
// profiles/r04/ab/cut16_dcap.log); 0 = compiled out (no `resume` / visit counter per lane)
#ifndef VRH_AO_DCAP
#define VRH_AO_DCAP 0
#endif
constexpr bool AO_CAPPED = VRH_AO_DCAP != 0;
constexpr uint32_t CUT_MAX = VRH_AO_CUT_MAX;            // records of a cut
constexpr int AO_SH = AO_CUT + 2 * 8 * CUT_MAX;        // two levels x entries of box lo xyz, hi xyz, link, pad
// Tail sharing (render_params::ao_share, blocks of several waves): once the tile queues are dry, a
// wave publishes its last tile's AO rays in a header of its LDS area and hands them out through an
// LDS counter, so idle sibling waves of the block trace some of them.  Header words: the published
// tile (NONE: none), its buffer parity, the next AO ray to hand out (LDS atomic), the tile's AO rays,
// rays in flight on sibling waves (LDS atomic), the tile's cut size; word SH_DRY of wave 0: the block
// has seen the queues run dry.
constexpr int AO_WAVE_WORDS = AO_SH + 8;
constexpr uint32_t SH_TILE = 0, SH_PAR = 1, SH_NEXT = 2, SH_AVAIL = 3, SH_HELP = 4, SH_CUTN = 5, SH_DRY = 6;
constexpr uint32_t TAG_NONFINITE = 0x80000000u;   // AO kernel lane tag: the ray is not finite
// the root link, read from the kernel's argument segment where it is used (a scalar load) instead of
// being held in a register across the refill loop, where the register allocator of the 6-wave AO
// instances copied it to a VGPR and spilled that to scratch
__device__ __forceinline__ uint32_t kernarg_root();

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

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
    // the frame's scissor box, clamped to the image on the host (cuda_sched.inl:71: x < sb.x,
    // y < sb.y, x >= sb.w, y >= sb.h are skipped -- w / h are the exclusive right / bottom edges)
    const frame_camera& c = P.cam[f];
    return x >= c.clip[0] && y >= c.clip[1] && x < c.clip[2] && y < c.clip[3];
}

__device__ __forceinline__ bool tile_pixel(const render_params& P, uint32_t unit, uint32_t lane,
                                           uint32_t& x, uint32_t& y, uint32_t& out_row)
{
    uint32_t f;
    return tile_pixel(P, unit, lane, x, y, out_row, f);
}

// per-wave totals (rays, hits, test counts): one atomic set per wave, at the end of the kernel
template <bool COUNT>
__device__ __forceinline__ void flush_totals(const render_params& P, uint32_t lane, uint64_t rays_total,
                                             uint64_t hits_total, const test_counts& cnt)
{
    unsigned long long rr = rays_total, hh = hits_total, b = cnt.box, q = cnt.prim, uni_sum = cnt.w_uni;
    unsigned long long li = cnt.lines, rq = cnt.reqs, vm = cnt.vmem, a4 = cnt.acc4, ai = cnt.acc_ideal;
    unsigned long long ak[5];
    for (int k = 0; k < 5; ++k) ak[k] = cnt.acc_kind[k];
    for (int off = 32; off > 0; off >>= 1)
    {
        rr += __shfl_down(rr, off);
        hh += __shfl_down(hh, off);
        if (COUNT)
        {
            b += __shfl_down(b, off); q += __shfl_down(q, off); uni_sum += __shfl_down(uni_sum, off);
            li += __shfl_down(li, off); rq += __shfl_down(rq, off); vm += __shfl_down(vm, off);
            a4 += __shfl_down(a4, off); ai += __shfl_down(ai, off);
            for (int k = 0; k < 5; ++k) ak[k] += __shfl_down(ak[k], off);
        }
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
            atomicAdd(P.counters + 11, uni_sum);
            atomicAdd(P.counters + COUNTERS_LINES, li);
            atomicAdd(P.counters + COUNTERS_LINES + 1, vm);
            atomicAdd(P.counters + COUNTERS_LINES + 2, rq);
            atomicAdd(P.counters + COUNTERS_LINES + 3, a4);
            atomicAdd(P.counters + COUNTERS_LINES + 4, ai);
            for (int k = 0; k < 5; ++k) atomicAdd(P.counters + COUNTERS_LINES + 5 + k, ak[k]);
        }
    }
}

// sched_common.h:130-150 make_primary_ray_impl (pinhole, uniform pixel sampler), frame f's camera
template <bool SAMPLED = false>
__device__ __forceinline__ ray_t primary_ray(const render_params& P, uint32_t f, uint32_t x, uint32_t y)
{
    const frame_camera& c = P.cam[f];
    float fx = (float)x, fy = (float)y;
    if constexpr (!SAMPLED) {}
    else if (P.jitter)
    {
        // jittered samplers (sched_common.h:196-216): x + (U - 0.5), y + (U - 0.5) with the
        // deterministic draws of vrh.h vrh_pixel_sampler -- y takes the first, as the reference's
        // jitter vector evaluates its constructor arguments under g++ (oracle vo_sampler_offsets)
        const uint32_t n = P.frame_num + f;
        const uint32_t k = (y * P.width + x) * 2u + 0x632BE5ABu + n * 0x68E31DA4u;
        fy = fy + (uniform01(k) - 0.5f);
        fx = fx + (uniform01(k + 1u) - 0.5f);
    }
    else
    {
        fx = fx + P.px_off[0];                    // ssaa<N>: the sample's offset
        fy = fy + P.px_off[1];
    }
    // (float)width / (float)height converted on the host (the same value: the conversion is exact
    // below 2^24): a device conversion of the uniform value was hoisted into a spilled VGPR
    float u = 2.0f * (fx + 0.5f) / P.width_f - 1.0f;
    float v = 2.0f * (fy + 0.5f) / P.height_f - 1.0f;
    if (SAMPLED && P.matrix_cam)
    {
        // sched_common.h:152-176 (camera matrices): o = inv_view (inv_proj (u, v, -1, 1)), d at
        // z = +1; matrix * vector row by row, left to right (matrix4.inl:171-181)
        const float* iv = P.inv_view;
        const float* ip = P.inv_proj;
        float a[4], b[4], o[4], d[4];
        for (int r = 0; r < 4; ++r)
        {
            a[r] = ip[r] * u + ip[4 + r] * v + ip[8 + r] * -1.0f + ip[12 + r] * 1.0f;
            b[r] = ip[r] * u + ip[4 + r] * v + ip[8 + r] * 1.0f + ip[12 + r] * 1.0f;
        }
        for (int r = 0; r < 4; ++r)
        {
            o[r] = iv[r] * a[0] + iv[4 + r] * a[1] + iv[8 + r] * a[2] + iv[12 + r] * a[3];
            d[r] = iv[r] * b[0] + iv[4 + r] * b[1] + iv[8 + r] * b[2] + iv[12 + r] * b[3];
        }
        const f3 ori = mk3(o[0] / o[3], o[1] / o[3], o[2] / o[3]);
        const f3 far = mk3(d[0] / d[3], d[1] / d[3], d[2] / d[3]);
        return make_ray(ori, normalize(far - ori));
    }
    f3 cu = mk3(c.cam_u[0], c.cam_u[1], c.cam_u[2]);
    f3 cv = mk3(c.cam_v[0], c.cam_v[1], c.cam_v[2]);
    f3 cw = mk3(c.cam_w[0], c.cam_w[1], c.cam_w[2]);
    f3 dir = normalize((cu * u + cv * v) + cw);
    return make_ray(mk3(c.eye[0], c.eye[1], c.eye[2]), dir);
}

// colour of output pixel o: stored, or blended onto the target (pixel_access.h:1155-1176:
// dst = c * s + dst * d) for the jittered_blend / ssaa samplers
template <bool SAMPLED>
__device__ __forceinline__ void put_color(const render_params& P, size_t o, float4 c)
{
    if (SAMPLED && P.blend)
    {
        const float4 d = P.blend == 2u ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : P.color[o];
        c = make_float4(c.x * P.blend_s + d.x * P.blend_d, c.y * P.blend_s + d.y * P.blend_d,
                        c.z * P.blend_s + d.z * P.blend_d, c.w * P.blend_s + d.w * P.blend_d);
    }
    P.color[o] = c;
}

// Tile work queues.  One frame per launch: a frame's tiles are split into 8 contiguous ranges
// (horizontal image strips), queue q hands out strip q.  Frames in flight (vrh_render_batch): the
// launch's (band, frame) units go round robin to the queues in band-major order, so the 8 XCDs
// sweep the image together, each on other frames of the same bands (+4 % hf10M AO, +10 % hf10M
// primary against strip q of every frame per queue, profiles/r02_ab/ab28_tile_order_*.log: the
// MALL then holds the bands' working set once for all XCDs).  A wave first drains the queue of the
// XCD it runs on (hardware register
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

#ifndef VRH_PRIMARY_CLUSTER
#define VRH_PRIMARY_CLUSTER 1
#endif
// CLUSTER = false: an instance without the cluster order's code (its launches hand out the band order
// for xcd_queues 3)
template <bool CLUSTER = true>
__device__ __forceinline__ uint32_t next_tile(const render_params& P, tile_queue& tq, uint32_t lane)
{
    const uint32_t nq = P.xcd_queues ? 8u : 1u;
    if (CLUSTER && P.xcd_queues == 3u)
    {
        // cluster order (frames in flight): queue q owns strip q of the launch's bands; a band is cut
        // into clusters of P.cluster tiles, and the units of a strip are (cluster, frame, tile) with
        // the tile fastest, then the frame -- the F frames of one cluster are handed out back to back,
        // so the waves in flight on one XCD trace the same few clusters of the image in every frame
        // in flight and their nodes and triangles stay in that XCD's L2
        const uint32_t tx = P.tiles_x, F = P.num_frames, C = P.cluster;
        const uint32_t nb = P.num_tiles / tx;
        while (tq.tried < 8u)
        {
            const uint32_t b0 = (uint32_t)(((uint64_t)nb * tq.q) >> 3);
            const uint32_t b1 = (uint32_t)(((uint64_t)nb * (tq.q + 1u)) >> 3);
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(reinterpret_cast<uint32_t*>(P.counters + 8u + 8u * tq.q), 1u);
            t = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(t, 0));
            const uint32_t per_band = tx * F;
            if (t < (b1 - b0) * per_band)
            {
                const uint32_t lb = t / per_band;
                const uint32_t r = t - lb * per_band;
                const uint32_t c = r / (C * F);                 // cluster of the band (the last may be narrower)
                const uint32_t r2 = r - c * C * F;
                const uint32_t cw = min(C, tx - c * C);
                const uint32_t f = r2 / cw;
                const uint32_t j = r2 - f * cw;
                return (f << TILE_FRAME_SHIFT) | ((b0 + lb) * tx + c * C + j);
            }
            tq.q = (tq.q + 1u) & 7u;
            tq.tried += 1u;
        }
        return NONE;
    }
    if (P.xcd_queues == 2u || (!CLUSTER && P.xcd_queues == 3u))
    {
        // band-interleaved (frames in flight): the launch's (band, frame) units in band-major order,
        // unit u = band * num_frames + frame dealt to queue u % 8 -- all 8 XCDs sweep the image's
        // bands together, each on other frames of the same band, so the nodes and triangles under
        // a band are fetched from HBM once for every XCD and frame in flight (the MALL and each
        // L2 hold the band's working set) instead of once per XCD strip
        const uint32_t tx = P.tiles_x;
        const uint32_t units = (P.num_tiles / tx) * P.num_frames;
        while (tq.tried < 8u)
        {
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(reinterpret_cast<uint32_t*>(P.counters + 8u + 8u * tq.q), 1u);
            t = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(t, 0));   // wave-uniform (SGPR)
            const uint32_t k = t / tx;
            const uint32_t u = k * 8u + tq.q;
            if (u < units)
            {
                const uint32_t band = u / P.num_frames;
                const uint32_t f = u - band * P.num_frames;
                return (f << TILE_FRAME_SHIFT) | (band * tx + (t - k * tx));
            }
            tq.q = (tq.q + 1u) & 7u;
            tq.tried += 1u;
        }
        return NONE;
    }
    while (tq.tried < nq)
    {
        const uint32_t lo = strip_lo(P, tq.q, nq);
        const uint32_t len = strip_lo(P, tq.q + 1u, nq) - lo;
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(reinterpret_cast<uint32_t*>(P.counters + 8u + 8u * tq.q), 1u);
        t = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(t, 0));
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

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// AO ray s of hit slot `slot` whose pixel has global index p in frame f of the launch
// (ao/main.cpp:216-238 with the Appendix-A sampler, offset by the frame number)
template <bool COUNT>
__device__ __forceinline__ ray_t ao_ray(const render_params& P, const float* recs, uint32_t slot, uint32_t s,
                                        uint32_t p, uint32_t f, test_counts& cnt)
{
    const float* sr = recs + slot * AO_REC_WORDS;
    f3 pos = mk3(sr[0], sr[1], sr[2]);
    const float4* np = P.normals + __float_as_uint(sr[3]);
    const float4 nn = *np;                                             // get_normal.h:26-37
    if (COUNT) count_vmem(cnt, np, 1u, VMEM_NORMAL);
    f3 n = mk3(nn.x, nn.y, nn.z);
    // vector3.inl:357-367 make_orthonormal_basis(u, v, w = n)
    f3 bv = fabsf(n.x) > fabsf(n.y) ? normalize(mk3(-n.z, 0.0f, n.x)) : normalize(mk3(0.0f, n.z, -n.y));
    f3 bu = cross(bv, n);
    f3 d = ao_direction(p, s, bu, bv, n, frame_salt(P.frame_num + f));
    return make_ray(pos + d * P.eps, d);
}

// Entry cut of the 4-wide any-hit tree for the AO rays of one tile (render_params::ao_cut).
// R = the box of the tile's hit positions grown by the AO reach (eps + radius, plus a margin of
// 1e-4 (1 + |coordinate|), orders of magnitude above the float error of a slab test).  Starting at
// the root, every record of the frontier is replaced by its children whose boxes meet R, level by
// level, while the frontier holds at most CUT_MAX entries.  An AO ray then starts with the cut
// entries whose boxes it passes (quad_entry, the test its parent record would apply) on its stack.
// Exact: (1) a leaf the any-hit traversal reaches passes its own box test, so its box comes within
// float error of the ray segment, which lies in R -- the leaf box, and every ancestor box (they
// contain it), meets R, so the leaf lies under a cut entry; (2) the slab test is monotone in the box
// bounds under round-to-nearest, so a ray that passes a cut entry's box passes every ancestor's, and
// the traversal from the root would reach that entry too.  Both traversals therefore reach the same
// leaves, and an any-hit result does not depend on the order.  Returns the
// number of entries written to `cut` (0: no AO ray of the tile can reach a leaf), or NONE when the
// root's children do not fit (the rays then start at the root).
__device__ __forceinline__ float wave_min(float v)
{
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v)
{
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
// The cut is built with wave-uniform values only: records through the scalar cache (s_load on a
// wave-uniform address, as ray_step's uniform pair fetch), frontier entries in LDS (two halves,
// one level each), so it needs no vector registers beyond the rays the other lanes are tracing.
typedef const __attribute__((address_space(4))) float cut_cfloat;
__device__ __forceinline__ float ufl(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }
__device__ __forceinline__ uint32_t uu(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
// the children of 4-wide record `k` whose boxes meet [lo, hi] (bit c = entry c)
__device__ __forceinline__ uint32_t cut_children(const float4* quads, uint32_t k, const float* lo, const float* hi)
{
    cut_cfloat* q = (cut_cfloat*)(const float*)(quads) + 32u * k;
    uint32_t m = 0u;
#pragma unroll
    for (uint32_t c = 0; c < 4u; ++c)
    {
        const bool meet = (__float_as_uint(q[24u + c]) != QUAD_NONE) & (q[c] <= hi[0]) & (q[12u + c] >= lo[0])
                        & (q[4u + c] <= hi[1]) & (q[16u + c] >= lo[1]) & (q[8u + c] <= hi[2]) & (q[20u + c] >= lo[2]);
        m |= meet ? (1u << c) : 0u;
    }
    return uu(m);
}
template <bool COUNT>
__device__ __forceinline__ uint32_t ao_cut_build(const render_params& P, const float* recs, uint32_t nslots, float* cut,
                                                 uint32_t lane, test_counts& cnt)
{
    const bool v = lane < nslots;
    float lo[3], hi[3];
    float mag = 0.0f;
    for (int a = 0; a < 3; ++a)
    {
        const float x = recs[(v ? lane : 0u) * AO_REC_WORDS + a];
        lo[a] = ufl(wave_min(v ? x : INFINITY));
        hi[a] = ufl(wave_max(v ? x : -INFINITY));
        mag = fmaxf(mag, fmaxf(fabsf(lo[a]), fabsf(hi[a])));
    }
    const float ext = ufl((P.eps + P.radius) * 1.001f + 1e-4f * (1.0f + mag));
    if (!(ext < INFINITY)) return NONE;
    for (int a = 0; a < 3; ++a) { lo[a] -= ext; hi[a] += ext; }
    auto put = [&](float* e, cut_cfloat* q, uint32_t c) {           // entry c of record q -> e
        // seven wave-uniform (scalar) loads, lane k keeps word k: no per-lane record address stays
        // live across the kernel (it was spilled to scratch)
        float w = q[c];
        w = lane == 1u ? q[4u + c] : w;
        w = lane == 2u ? q[8u + c] : w;
        w = lane == 3u ? q[12u + c] : w;
        w = lane == 4u ? q[16u + c] : w;
        w = lane == 5u ? q[20u + c] : w;
        w = lane == 6u ? q[24u + c] : w;
        if (lane < 7u) e[lane] = w;
    };
    // level 0: the root record's children
    float* cur = cut;
    float* nxt = cut + 8u * CUT_MAX;
    {
        const uint32_t ok = cut_children(P.quads, 0u, lo, hi);
        cut_cfloat* q = (cut_cfloat*)(const float*)(P.quads);
        uint32_t n = 0;
        for (uint32_t c = 0; c < 4u; ++c)
            if (ok & (1u << c)) { put(cur + 8u * n, q, c); n += 1u; }
        if (COUNT && lane == 0u) cnt.box += 4u;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        // deeper levels while the frontier fits
#pragma unroll 1
        for (uint32_t level = 0; level < 32u; ++level)
        {
            uint32_t total = 0, inner = 0;
#pragma unroll 1
            for (uint32_t j = 0; j < n; ++j)
            {
                const uint32_t k = uu(__float_as_uint(cur[8u * j + 6u]));
                if (k & LEAF_BIT) { total += 1u; continue; }
                inner += 1u;
                total += (uint32_t)__popc(cut_children(P.quads, k, lo, hi));
            }
            if (inner == 0u || total > CUT_MAX) break;
            uint32_t o = 0;
#pragma unroll 1
            for (uint32_t j = 0; j < n; ++j)
            {
                const uint32_t k = uu(__float_as_uint(cur[8u * j + 6u]));
                if (k & LEAF_BIT)
                {
                    if (lane < 7u) nxt[8u * o + lane] = cur[8u * j + lane];
                    o += 1u;
                    continue;
                }
                const uint32_t ok = cut_children(P.quads, k, lo, hi);
                if (COUNT && lane == 0u) cnt.box += 4u;
                cut_cfloat* q = (cut_cfloat*)(const float*)(P.quads) + 32u * k;
                for (uint32_t c = 0; c < 4u; ++c)
                    if (ok & (1u << c)) { put(nxt + 8u * o, q, c); o += 1u; }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            float* t = cur; cur = nxt; nxt = t;
            n = total;
        }
        if (P.ao_cut == 2u && n > 1u)
        {
            // order the entries by the distance of their box centre to R's centre, farthest first:
            // the nearest is pushed last and popped first (an AO occluder is usually near the hit)
            float key = -1.0f;
            if (lane < n)
            {
                const float* e = cur + 8u * lane;
                const float dx = (e[0] + e[3]) - (lo[0] + hi[0]), dy = (e[1] + e[4]) - (lo[1] + hi[1]);
                const float dz = (e[2] + e[5]) - (lo[2] + hi[2]);
                key = dx * dx + dy * dy + dz * dz;
            }
            uint32_t rank = 0;
            for (uint32_t j = 0; j < n; ++j)
            {
                const float kj = __shfl(key, (int)j);
                rank += ((kj > key) | ((kj == key) & (j < lane))) ? 1u : 0u;
            }
            for (uint32_t w = 0; w < 7u; ++w)
                if (lane < n) nxt[8u * rank + w] = cur[8u * lane + w];
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            float* t = cur; cur = nxt; nxt = t;
        }
        if (cur != cut)
        {
            if constexpr (CUT_MAX <= 8u)
            {
                if (lane < 8u * n) cut[lane] = cur[lane];
            }
            else
                for (uint32_t k = lane; k < 8u * n; k += 64u) cut[k] = cur[k];   // more words than lanes
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
        return n;
    }
}

// coalescer model of the output stores of one pixel (counting variant), by buffer: 1 colour,
// 2 occlusion mask, 4 prim id, 8 t
constexpr uint32_t ST_COLOR = 1u, ST_OCC = 2u, ST_PID = 4u, ST_T = 8u;
__device__ __forceinline__ void count_stores(test_counts& cnt, const render_params& P, size_t o, uint32_t which)
{
    if ((which & ST_COLOR) && P.color) count_vmem(cnt, P.color + o, 1u, VMEM_STORE);
    if ((which & ST_OCC) && P.occ) count_vmem(cnt, P.occ + o, 1u, VMEM_STORE);
    if ((which & ST_PID) && P.prim_id) count_vmem(cnt, P.prim_id + o, 1u, VMEM_STORE);
    if ((which & ST_T) && P.t) count_vmem(cnt, P.t + o, 1u, VMEM_STORE);
}

// BVH-ref lists (traverse_linear.inl:76-141): the ray's BVH `bk` is exhausted (rc < 0).  Every BVH
// of the list is traversed on its own (fresh result, the same max_t), and its hit is merged into
// the running result by update_if(result, hr, is_closer(hr, result, max_t)) (update_if.h:27-79,
// hit_record.h:54-64: strictly closer only).  Any hit stops at the first BVH with a hit (rc > 0,
// exit_traversal.h:49-56), so only exhausted BVHs come here.  Returns the new rc: 0 = the next BVH
// was started, -1 = the list is done (best_t / best_prim hold the merged result).
template <class Stack>
__device__ __forceinline__ int list_next(const render_params& P, bool any, uint32_t& bk, float& res_t, uint32_t& res_prim,
                                         float& best_t, uint32_t& best_prim, Stack& st, uint32_t& resume)
{
    if (!any && best_t < res_t) { res_t = best_t; res_prim = best_prim; }
    if (bk + 1u < P.num_roots)
    {
        bk += 1u;
        best_t = FMAX; best_prim = 0;
        st.reset(); st.push(P.roots[bk]); resume = NO_RESUME;
        return 0;
    }
    best_t = res_t; best_prim = res_prim;
    return -1;
}

__device__ __forceinline__ uint32_t kernarg_root()
{
    typedef const volatile __attribute__((address_space(4))) uint32_t karg_u32;
    karg_u32* ka = (karg_u32*)__builtin_amdgcn_kernarg_segment_ptr();
    return ka[offsetof(render_params, root) / 4u];
}

// One refilling loop per wave.  Primary rays (one per pixel of the wave's tile)
// and AO rays (published as soon as their primary hit is known) are stepped by the same
// instruction stream (ray_step); a lane that finishes a ray immediately takes the next one, so
// neither the primary phase nor the AO phase waits for its slowest lane.  Without AO the wave
// streams pixels tile after tile and writes each pixel when its ray finishes.
// EPI: primary-ray epilogue -- 0 colour = hit ? 1 : bg, 1 simple::kernel shading, 2 multi_hit<N>
// hit lists + the multi_hit example's compositing, 3 whitted::kernel (the lane traces its pixel's
// shadow and reflection rays one after the other before it takes the next pixel).
// LIST: the scene is a list of BVHs (vrh_scene_list_create), traversed one after the other per ray
// and merged as traverse_linear.inl:76-141 does (list_next); EPI 0 only.
// BATCH: the same code, instantiated separately for launches of several frames (vrh_render_batch,
// frames in flight) so that profiles tell them apart from one-frame launches (hip_sched::frame).
// SPILL: the traversal stack may continue in the global overflow block (stack_t<true>).
template <int KIND, bool AO, bool COUNT, int OCC, int EPI = 0, bool LIST = false, bool BATCH = false, bool SPILL = false,
          bool SAMPLED = false, bool SHARE = false>
__global__ __launch_bounds__(256, OCC) void render_unified_kernel(render_params P)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = tid >> 6;
    const uint32_t block = blockDim.x;

    stack_t<SPILL> st;
    // the overflow entries of this block: (stack_total - stack_cap) entries per lane, same column layout
    st.init(smem, tid, block, P.stack_cap, SPILL ? P.stack_total : P.stack_cap,
            SPILL ? P.stack_spill + size_t(blockIdx.x) * (P.stack_total - P.stack_cap) * block : nullptr);
    uint32_t* ao_area = smem + P.stack_cap * block + wave * AO_WAVE_WORDS;
    test_counts cnt = {};
    // per-lane ray / hit counts of this launch (below 2^32 per lane: a launch traces < 2^32 rays)
    uint32_t rays_total = 0, hits_total = 0;
    const hit_mask_params hml = P.hmask;          // a local copy: &P would spill the kernel arguments
    const hit_mask_params* hm = &hml;             // ray_step tests hm->mask
    // the wave's (start, end) slot: the start is stored at once, the end slot kept as a wave-uniform
    // pointer (nothing of the prologue's per-lane values stays live across the loop)
    unsigned long long* const wt_slot = P.wave_times ? P.wave_times + 2 * (size_t(blockIdx.x) * (blockDim.x >> 6) + uu(wave)) : nullptr;
    if (wt_slot && lane == 0) wt_slot[0] = wall_clock64();

    // lane state: the ray it is stepping
    constexpr uint32_t IDLE = 0, PRIMARY = 1, AORAY = 2;
    uint32_t mode = IDLE;
    ray_t r;
    float best_t = FMAX, max_t = FMAX;
    uint32_t best_prim = 0, steps = 0;
    bool any = false, quad = false, finite = true;
    uint32_t resume = NO_RESUME;
    uint32_t bk = 0, res_prim = 0;                 // LIST: the ray's current BVH, merged result
    float res_t = FMAX;
    static_assert(!LIST || EPI == 0, "BVH lists: primary and AO kernels");

    if constexpr (!AO)
    {
        // ---- primary visibility: stream pixels, write each when its ray finishes ------------
        tile_queue tq = queue_init(P);
        uint32_t tile = next_tile<VRH_PRIMARY_CLUSTER != 0>(P, tq, lane);
        uint32_t handed = 0;                       // pixels of `tile` handed out (wave-uniform)
        uint32_t out_o = 0;
        hit_extra hx = { 0.0f, 0.0f, 0u };
        mh_list mh;
        mh.mem = smem;
        mh.base = P.stack_cap * block + tid;
        mh.stride = block;
        mh.n = EPI == 2 ? P.max_hits : 1u;
        whitted_lane w;
        w.shadow = 0; w.depth = 0;
        w.sm = reinterpret_cast<float*>(smem); w.base = P.stack_cap * block + tid; w.stride = block;   // EPI 3 LDS words
        for (;;)
        {
            uint64_t idle = __ballot(mode == IDLE);
            if ((uint32_t)__popcll(idle) < P.refill_min_primary && idle != ~0ull) idle = 0ull;
            if (idle)
            {
                if (handed >= 64u && tile != NONE)
                {
                    tile = next_tile<VRH_PRIMARY_CLUSTER != 0>(P, tq, lane);
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
                            r = primary_ray<SAMPLED>(P, fr, x, y);
                            finite = finite_ray(r);
                            out_o = orow * P.width + x;
                            best_t = FMAX; best_prim = 0; steps = 0;
                            if constexpr (EPI == 2) mh.reset();
                            if constexpr (EPI == 3)
                            {
                                w.color = mk3(0.0f, 0.0f, 0.0f); w.thr = 1.0f; w.depth = 0; w.shadow = 0;
                                max_t = FMAX; any = false; quad = false;
                            }
                            st.reset(); st.push(P.root); resume = NO_RESUME;
                            bk = 0; res_t = FMAX; res_prim = 0;
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
            using ML = typename std::conditional<EPI == 2, mh_list, void>::type;
            constexpr bool UV = EPI == 1 || EPI == 3;
            const float mt = EPI == 3 ? max_t : FMAX;
            const bool an = EPI == 3 ? any : false;
            if (mode != IDLE)
            {
                int rc = (P.fast_ok && __ballot(!finite) == 0ull)
                    ? ray_step<KIND, COUNT, true, UV, ML>(P.pairs, P.prims, P.quads, P.root, quad, r, mt, an, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, &hx, &mh, hm)
                    : ray_step<KIND, COUNT, false, UV, ML>(P.pairs, P.prims, P.quads, P.root, quad, r, mt, an, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, &hx, &mh, hm);
                if constexpr (LIST)
                    if (rc != 0) rc = list_next(P, false, bk, res_t, res_prim, best_t, best_prim, st, resume);
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
                                w.color = w.color + w.ld3(WL_SHADED) * w.thr;
                                const float thr2 = w.thr * 0.1f;
                                if (thr2 > P.eps && w.depth < P.num_bounces)
                                {
                                    const f3 rdir = whitted_reflect(w);
                                    r = make_ray(w.ld3(WL_POS) + rdir * P.eps, rdir);
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
                    if (P.color) put_color<SAMPLED>(P, out_o, c);
                    if (P.prim_id) P.prim_id[out_o] = hit ? best_prim : 0xFFFFFFFFu;
                    if (P.t) P.t[out_o] = hit ? best_t : -1.0f;
                    if (P.occ) P.occ[out_o] = 0;
                    if (COUNT) count_stores(cnt, P, out_o, ST_COLOR | ST_OCC | ST_PID | ST_T);
                    mode = IDLE;
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
        float* cut = reinterpret_cast<float*>(ao_area + AO_CUT);
        uint32_t cutN = NONE;                                 // entries of tile C's cut (NONE: root)
        uint32_t* const ao_base = smem + P.stack_cap * block; // wave w's AO area: ao_base + w * AO_WAVE_WORDS
        uint32_t* const sh = ao_area + AO_SH;
        const uint32_t nwaves = block >> 6;
        const bool share = SHARE && !LIST && P.ao_share && nwaves > 1u;
        bool shC = false, shD = false;                        // tile C / D published to the sibling waves
        uint32_t* const dry = ao_base + AO_SH + SH_DRY;       // wave 0's word: the block saw the queues dry
        if (share)
        {
            if (lane == 0u) { sh[SH_TILE] = NONE; sh[SH_HELP] = 0u; sh[SH_NEXT] = 0u; sh[SH_AVAIL] = 0u; sh[SH_DRY] = 0u; }
            __syncthreads();
        }
        auto mark_dry = [&](uint32_t tile) {
            if (share && tile == NONE && lane == 0u) __hip_atomic_store(dry, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        const float4 bg = make_float4(P.bg[0], P.bg[1], P.bg[2], P.bg[3]);
        tile_queue tq = queue_init(P);
        // wave-uniform tile state
        uint32_t tileC = next_tile(P, tq, lane), parC = 0;
        mark_dry(tileC);
        // tile timeline (counting instance only): [3 t] hand-out, [3 t + 1] primaries done, [3 t + 2] written
        auto tile_mark = [&](uint32_t id, uint32_t k) {
            if constexpr (COUNT)
                if (P.tile_times && id != NONE && lane == 0u) P.tile_times[3u * (id & TILE_MASK) + k] = wall_clock64();
        };
        tile_mark(tileC, 0u);
        uint32_t handedC = 0, pendC = 0, pubC = 0, issC = 0;  // primaries handed / in flight, slots, AO rays handed
        uint32_t tileD = NONE, parD = 0, slotsD = 0;
        uint32_t inflight0 = 0, inflight1 = 0;                // AO rays in flight per buffer parity
        // lane state: PRIMARY tag = pixel lane k of tile C; AORAY tag = slot | s << 6 | parity << 11 |
        // owner wave << 12; bit 31 (TAG_NONFINITE) = the ray has a non-finite origin or inverse
        // direction (it takes the literal slab test) -- kept in the tag rather than in a register of its
        // own, which the 6-wave instances spilled
        // owner wave << 12 (the wave whose tile the ray belongs to: this one unless it helps a sibling)
        uint32_t tag = 0;
        // AO ray `cand` (slot-major: slot cand / S, sample cand % S) of the tile `tile` whose hit records,
        // slot pixels and cut are recs_ / spx / cut_, cutn (this wave's, or a sibling's it helps)
        auto start_ao = [&](const float* recs_, const uint8_t* spx, const float* cut_, uint32_t cutn, uint32_t tile,
                            uint32_t par, uint32_t cand, uint32_t owner) {
            // cand / S by the host's reciprocal (exact for cand < 64 S, render_params::samples_recip)
            const uint32_t slot = (cand * P.samples_recip) >> 20, smp = cand - slot * S;
            uint32_t x, y, orow, fr;
            tile_pixel(P, tile, spx[par * 64u + slot], x, y, orow, fr);
            r = ao_ray<COUNT>(P, recs_, slot, smp, y * P.width + x, fr, cnt);
            best_t = FMAX; best_prim = 0; steps = 0; max_t = P.radius; any = true;
            bk = 0; res_t = FMAX; res_prim = 0;
            const bool fin = finite_ray(r);
            quad = P.quad_ok && fin;
            st.reset(); resume = NO_RESUME;
            if (!LIST && (!SPILL || VRH_AO_CUT_SPILL) && VRH_AO_CUT && quad && cutn != NONE)
            {
                // start at the tile's cut: the entries whose boxes this ray passes
#pragma unroll 1
                for (uint32_t j = 0; j < cutn; ++j)
                {
                    // quad_entry's test, one axis at a time (max / min of non-NaN values
                    // are exact in any order: the same tn / tf, fewer live registers)
                    const float* e = cut_ + 8u * j;
                    float t1 = (e[0] - r.ori.x) * r.inv.x, t2 = (e[3] - r.ori.x) * r.inv.x;
                    float tn = __builtin_fminf(t1, t2), tf = __builtin_fmaxf(t1, t2);
                    t1 = (e[1] - r.ori.y) * r.inv.y; t2 = (e[4] - r.ori.y) * r.inv.y;
                    tn = __builtin_fmaxf(tn, __builtin_fminf(t1, t2)); tf = __builtin_fminf(tf, __builtin_fmaxf(t1, t2));
                    t1 = (e[2] - r.ori.z) * r.inv.z; t2 = (e[5] - r.ori.z) * r.inv.z;
                    tn = __builtin_fmaxf(tn, __builtin_fminf(t1, t2)); tf = __builtin_fminf(tf, __builtin_fmaxf(t1, t2));
                    if ((tf >= tn) & (tn < FMAX) & (tf >= 0.0f) & (tn < max_t)) st.push(__float_as_uint(e[6]));
                }
                if (COUNT) cnt.box += cutn;
            }
            else
                st.push(quad ? 0u : P.root);
            mode = AORAY;
            tag = slot | (smp << 6) | (par << 11) | (SHARE ? owner << 12 : 0u) | (fin ? 0u : TAG_NONFINITE);
            rays_total += 1;
        };
        for (;;)
        {
            // 1. the draining tile is done when its last AO ray is: write its hit pixels
            if (tileD != NONE && (parD ? inflight1 : inflight0) == 0u && (!shD || lds_ld(&sh[SH_HELP]) == 0u))
            {
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // the siblings' mask bits
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
                    if (P.color) put_color<SAMPLED>(P, o, make_float4(clr, clr, clr, 1.0f));
                    if (P.occ) P.occ[o] = (uint8_t)m;
                    if (COUNT) count_stores(cnt, P, o, ST_COLOR | ST_OCC);
                }
                __builtin_amdgcn_wave_barrier();
                tile_mark(tileD, 2u);
                tileD = NONE;
                if (shD && lane == 0u) __hip_atomic_store(&sh[SH_TILE], NONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                shD = false;
            }
            // 2. the current tile has handed out all its rays: it drains, the next tile starts
            if (tileC != NONE && tileD == NONE && handedC >= 64u && pendC == 0u && issC >= pubC * S)
            {
                tileD = tileC; parD = parC; slotsD = pubC;
                shD = shC; shC = false;
                tileC = next_tile(P, tq, lane);
                mark_dry(tileC);
                tile_mark(tileC, 0u);
                parC ^= 1u;
                handedC = 0; pendC = 0; pubC = 0; issC = 0;
            }
            // 3. hand out rays to idle lanes: the current tile's AO rays, then its primaries --
            //    once P.refill_min lanes are idle (or none is busy), so ray generation runs with
            //    many lanes at once
            uint64_t idle = __ballot(mode == IDLE);
            if ((uint32_t)__popcll(idle) < P.refill_min && idle != ~0ull) idle = 0ull;
            // ao_gate: a tile's AO rays wait until all its primaries have finished, so the waves'
            // steps are mostly all-primary or all-AO (binary closest-hit and 4-wide any-hit descents
            // then rarely share a step); +1 % alone, +6 % (hf1M) / +10 % (hf10M) with the 4-wide
            // any-hit records (profiles/r02_ab/ab4_c4opts.log)
            if (idle && issC < pubC * S && (!P.ao_gate || (pendC == 0u && handedC >= 64u)))
            {
                const uint32_t avail = pubC * S;
                // measured with entries nearest-first: hf1M +9 %, hf10M +4.8 %
                // (profiles/r02_ab/ab32_*, ab33_*, ab34_ao_cut_spill.log)
                constexpr bool CUT = !LIST && (!SPILL || VRH_AO_CUT_SPILL) && VRH_AO_CUT;
                if constexpr (CUT)
                    if (P.ao_cut && issC == 0u)
                    {
                        // the tile's first AO hand-out: all its hits are published (ao_gate)
                        cutN = uu(ao_cut_build<COUNT>(P, recs, pubC, cut, lane, cnt));   // wave-uniform (SGPR)
                        if (cutN != NONE && cutN + 4u > P.stack_cap) cutN = NONE;
                    }
                // once the block's queues are dry, the tile's AO rays are handed out through the LDS
                // counter of its header, which idle sibling waves claim from too (step 3b)
                if (share && !shC && lds_ld(dry) != 0u)
                {
                    if (lane == 0u)
                    {
                        sh[SH_PAR] = parC; sh[SH_NEXT] = issC; sh[SH_AVAIL] = avail; sh[SH_CUTN] = cutN; sh[SH_HELP] = 0u;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __hip_atomic_store(&sh[SH_TILE], tileC, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    shC = true;
                }
                uint32_t base = issC;
                const uint32_t want = (uint32_t)__popcll(idle);
                if (shC)
                {
                    uint32_t b = 0u;
                    if (lane == 0u) b = atomicAdd(&sh[SH_NEXT], want);
                    base = uu((uint32_t)__shfl((int)b, 0));
                }
                const uint32_t cand = base + lane_rank(idle);
                const uint32_t n = base < avail ? min(avail - base, want) : 0u;
                if (mode == IDLE && cand < avail)
                    start_ao(recs, slot_px, cut, cutN, tileC, parC, cand, wave);
                issC = shC ? min(avail, base + want) : issC + n;
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
                    r = primary_ray<SAMPLED>(P, fr, x, y);
                    best_t = FMAX; best_prim = 0; steps = 0; max_t = FMAX; any = false; quad = false;
                    st.reset(); st.push(LIST ? P.root : kernarg_root()); resume = NO_RESUME;
                    bk = 0; res_t = FMAX; res_prim = 0;
                    mode = PRIMARY;
                    tag = k | (finite_ray(r) ? 0u : TAG_NONFINITE);
                    rays_total += 1;
                    started = true;
                }
                pendC += (uint32_t)__popcll(__ballot(started));
            }
            // 3b. nothing of its own left to hand out once the queues are dry: idle lanes claim AO
            //     rays of a sibling wave's published tile (their occlusion bits go to the sibling's
            //     masks, the sibling writes the pixels once its helpers' rays are done)
            if (share && tileC == NONE)
            {
                uint64_t hidle = __ballot(mode == IDLE);
                if (hidle != 0ull && ((uint32_t)__popcll(hidle) >= P.refill_min || hidle == ~0ull))
                {
#pragma unroll 1
                    for (uint32_t k = 1; k < nwaves && hidle != 0ull; ++k)
                    {
                        const uint32_t o = (wave + k) % nwaves;
                        uint32_t* const ao_o = ao_base + o * AO_WAVE_WORDS;
                        uint32_t* const so = ao_o + AO_SH;
                        const uint32_t t = uu(lds_ld(&so[SH_TILE]));
                        if (t == NONE) continue;
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // the header words
                        const uint32_t avail = uu(lds_ld(&so[SH_AVAIL]));
                        if (uu(lds_ld(&so[SH_NEXT])) >= avail) continue;
                        const uint32_t want = (uint32_t)__popcll(hidle);
                        uint32_t b = 0u;
                        if (lane == 0u)
                        {
                            atomicAdd(&so[SH_HELP], want);            // before the claim: the owner waits
                            b = atomicAdd(&so[SH_NEXT], want);
                        }
                        b = uu((uint32_t)__shfl((int)b, 0));
                        const uint32_t got = b < avail ? min(avail - b, want) : 0u;
                        if (lane == 0u && got < want) atomicSub(&so[SH_HELP], want - got);
                        if (got == 0u) continue;
                        const uint32_t rk = lane_rank(hidle);
                        if (mode == IDLE && rk < got)
                            start_ao(reinterpret_cast<const float*>(ao_o), reinterpret_cast<const uint8_t*>(ao_o + AO_SLOT_PX),
                                     reinterpret_cast<const float*>(ao_o + AO_CUT), uu(lds_ld(&so[SH_CUTN])), t,
                                     uu(lds_ld(&so[SH_PAR])), b + rk, o);
                        hidle = __ballot(mode == IDLE);
                    }
                }
            }
            const bool busy = mode != IDLE;
            if (__ballot(busy) == 0ull)
            {
                if (tileC == NONE && tileD == NONE) break;
                continue;
            }
            // 4. one traversal step for every busy lane (same code for both ray kinds)
            int rc = 0;
            if (busy)
            {
                // the AO kernel's rays: any-hit AO rays up to the radius, closest-hit primaries unbounded
                // (derived from `any` instead of a per-lane max_t).  The root link ray_step restarts a
                // 4-wide descent at is pair 0: 4-wide records exist only for trees whose root is a pair,
                // stored first (render_params::quad_ok checks it), so no register holds it
                const float mt = VRH_AO_LEAN ? (any ? P.radius : FMAX) : max_t;
                rc = (P.fast_ok && __ballot((tag & TAG_NONFINITE) != 0u) == 0ull)
                    ? ray_step<KIND, COUNT, true, false, void, AO_CAPPED>(P.pairs, P.prims, P.quads, 0u, quad, r, mt, any, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm)
                    : ray_step<KIND, COUNT, false, false, void, AO_CAPPED>(P.pairs, P.prims, P.quads, 0u, quad, r, mt, any, st, best_t, best_prim, cnt, steps, P.step_limit, resume, P.descent_cap, P.step_flags, nullptr, static_cast<const void*>(nullptr), hm);
            }
            if constexpr (LIST)
                if (busy && rc < 0) rc = list_next(P, any, bk, res_t, res_prim, best_t, best_prim, st, resume);
            if (COUNT) count_wave(cnt, busy);
            // 5. finished AO rays: record occlusion, retire from their tile's in-flight count
            const bool ao_done = mode == AORAY && rc != 0;
            const uint32_t own = SHARE ? (tag >> 12) & 7u : wave;    // the wave whose tile the ray belongs to
            const bool mine = own == wave;
            uint32_t* const mk = mine ? masks : ao_base + own * AO_WAVE_WORDS + AO_MASKS;
            if (ao_done && rc > 0) atomicOr(&mk[((tag >> 11) & 1u) * 64u + (tag & 63u)], 1u << ((tag >> 6) & 31u));
            inflight0 -= (uint32_t)__popcll(__ballot(ao_done && mine && ((tag >> 11) & 1u) == 0u));
            inflight1 -= (uint32_t)__popcll(__ballot(ao_done && mine && ((tag >> 11) & 1u) != 0u));
            if (share && __ballot(ao_done && !mine) != 0ull)
            {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");     // mask bits before the count
#pragma unroll 1
                for (uint32_t o = 0; o < nwaves; ++o)
                {
                    const uint32_t c = (uint32_t)__popcll(__ballot(ao_done && !mine && own == o));
                    if (c != 0u && lane == 0u) atomicSub(&ao_base[o * AO_WAVE_WORDS + AO_SH + SH_HELP], c);
                }
            }
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
                    tile_pixel(P, tileC, tag & 63u, x, y, orow);
                    const size_t o = (size_t)orow * P.width + x;
                    if (P.prim_id) P.prim_id[o] = hit ? best_prim : 0xFFFFFFFFu;
                    if (P.t) P.t[o] = hit ? best_t : -1.0f;
                    if (COUNT) count_stores(cnt, P, o, ST_PID | ST_T);
                    if (hit)
                    {
                        const uint32_t slot = pubC + lane_rank(hfin);
                        const f3 pos = r.ori + r.dir * best_t;                   // ao/main.cpp:202
                        float* rec = recs + slot * AO_REC_WORDS;
                        rec[0] = pos.x; rec[1] = pos.y; rec[2] = pos.z;
                        rec[3] = __uint_as_float(best_prim);
                        masks[parC * 64u + slot] = 0u;
                        slot_px[parC * 64u + slot] = (uint8_t)(tag & 63u);
                    }
                    else
                    {
                        if (P.color) put_color<SAMPLED>(P, o, bg);
                        if (P.occ) P.occ[o] = 0;
                        if (COUNT) count_stores(cnt, P, o, ST_COLOR | ST_OCC);
                    }
                }
                pubC += (uint32_t)__popcll(hfin);
                pendC -= (uint32_t)__popcll(fin);
                if (pendC == 0u && handedC >= 64u) tile_mark(tileC, 1u);
                hits_total += hit ? 1 : 0;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            }
            if (rc != 0) mode = IDLE;
        }
    }

    if (wt_slot && __lane_id() == 0u) wt_slot[1] = wall_clock64();
    flush_totals<COUNT>(P, __lane_id(), rays_total, hits_total, cnt);
}

// un-interleave gathered packed shards [count][rows_per_shard][W] into the full image (vrh_plan.h
// unshard_pixel: the same function the host export vrh_unshard_host runs)
__global__ void unshard_kernel(unshard_params u)
{
    plan::unshard_pixel(u, blockIdx.x * blockDim.x + threadIdx.x, blockIdx.y);
}

__global__ void pack_code_kernel(const uint32_t* __restrict__ pid, const uint8_t* __restrict__ occ,
                                 uint8_t* __restrict__ code, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    code[i] = plan::pack_code(pid[i], occ, i);
}

} // namespace dev

// ------------------------------------------------------------------------------------------------

using kernel_fn = void (*)(render_params);

template <int KIND, int OCC>
static kernel_fn pick_occ(bool ao, bool count, int sched)
{
    if (sched == 2)   // BVH list (step loop), at the default register budgets
    {
        if (!ao) return count ? dev::render_unified_kernel<KIND, false, true, 6, 0, true> : dev::render_unified_kernel<KIND, false, false, 6, 0, true>;
        return count ? dev::render_unified_kernel<KIND, true, true, 5, 0, true> : dev::render_unified_kernel<KIND, true, false, 5, 0, true>;
    }
    if (sched == 6)   // a pixel-sampler pass (vrh_render_sampled): jittered / offset rays, blended colour
    {
        if constexpr (OCC == 5 || OCC == 6)
            return ao ? dev::render_unified_kernel<KIND, true, false, OCC, 0, false, false, false, true>
                      : dev::render_unified_kernel<KIND, false, false, OCC, 0, false, false, false, true>;
        return nullptr;
    }
    if (sched == 3)   // frames in flight (a distinct symbol for profiles), step loop
        return ao ? dev::render_unified_kernel<KIND, true, false, OCC, 0, false, true>
                  : dev::render_unified_kernel<KIND, false, false, OCC, 0, false, true>;
    if (sched == 4)   // sched 0 / 3 with the stack overflow block (launch_config::spill)
        return ao ? dev::render_unified_kernel<KIND, true, false, OCC, 0, false, false, true>
                  : dev::render_unified_kernel<KIND, false, false, OCC, 0, false, false, true>;
    if (sched == 5)
        return ao ? dev::render_unified_kernel<KIND, true, false, OCC, 0, false, true, true>
                  : dev::render_unified_kernel<KIND, false, false, OCC, 0, false, true, true>;
    if (!ao) return count ? dev::render_unified_kernel<KIND, false, true, OCC> : dev::render_unified_kernel<KIND, false, false, OCC>;
    return count ? dev::render_unified_kernel<KIND, true, true, OCC> : dev::render_unified_kernel<KIND, true, false, OCC>;
}

// simple::kernel / multi_hit / whitted epilogues: triangles, step loop
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

// the overflow-stack instances exist at the register budgets the defaults choose from: AO 5 or 6
// waves / SIMD (triangles), primary visibility 6 or 8
template <int KIND>
static kernel_fn pick_spill(bool ao, int occ, int sched)
{
    const int s = sched == 3 ? 5 : 4;
    if (ao && KIND == dev::KIND_TRI && occ == 5) return pick_occ<KIND, 5>(true, false, s);
    if (ao && KIND == dev::KIND_TRI && occ == 6) return pick_occ<KIND, 6>(true, false, s);
    if (!ao && occ == 6) return pick_occ<KIND, 6>(false, false, s);
    if (!ao && occ == 8) return pick_occ<KIND, 8>(false, false, s);
    return nullptr;
}

// AO tail sharing instances: one-frame AO launches (sched 0) at the default 5 waves / SIMD, with and
// without the stack overflow block
template <int KIND>
static kernel_fn pick_share(const launch_config& c)
{
    if (!c.ao || c.count || c.epi || c.occ != 5 || c.sched != 0) return nullptr;
    return c.spill ? dev::render_unified_kernel<KIND, true, false, 5, 0, false, false, true, false, true>
                   : dev::render_unified_kernel<KIND, true, false, 5, 0, false, false, false, false, true>;
}

static kernel_fn select_variant(const launch_config& c)
{
    if (c.share)
        if (kernel_fn f = c.kind == dev::KIND_TRI ? pick_share<dev::KIND_TRI>(c) : pick_share<dev::KIND_SPHERE>(c)) return f;
    if (c.epi) return c.occ == 8 ? pick_shade<8>(c.count, c.epi) : c.occ == 6 ? pick_shade<6>(c.count, c.epi)
                    : c.occ == 5 ? pick_shade<5>(c.count, c.epi) : pick_shade<1>(c.count, c.epi);
    if (c.spill)
        return c.kind == dev::KIND_TRI ? pick_spill<dev::KIND_TRI>(c.ao, c.occ, c.sched)
                                       : pick_spill<dev::KIND_SPHERE>(c.ao, c.occ, c.sched);
    return c.kind == dev::KIND_TRI ? pick<dev::KIND_TRI>(c.ao, c.count, c.occ, c.sched)
                                   : pick<dev::KIND_SPHERE>(c.ao, c.count, c.occ, c.sched);
}

bool render_spill_available(const launch_config& c)
{
    if (c.epi || c.count || (c.sched != 0 && c.sched != 3)) return false;
    launch_config s = c;
    s.spill = true;
    return select_variant(s) != nullptr;
}

bool render_share_available(const launch_config& c)
{
    return c.kind == dev::KIND_TRI ? pick_share<dev::KIND_TRI>(c) != nullptr : pick_share<dev::KIND_SPHERE>(c) != nullptr;
}

size_t render_lds_bytes(const launch_config& c)
{
    size_t words = size_t(c.stack_cap) * c.block + (c.ao ? size_t(c.block / 64) * dev::AO_WAVE_WORDS : 0)
                 + (c.epi == 2 ? size_t(5) * c.max_hits * c.block : 0)
                 + (c.epi == 3 ? size_t(dev::WL_WORDS) * c.block : 0);
    return words * 4;
}

hipError_t launch_render(const render_params& p, const launch_config& c, int grid, hipStream_t s)
{
    hipLaunchKernelGGL(select_variant(c), dim3(grid), dim3(c.block), render_lds_bytes(c), s, p);
    return hipGetLastError();
}

int render_blocks_per_cu(const launch_config& c)
{
    // cached per (variant, block, LDS bytes): vrh_render asks several times per frame
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, size_t>, int> cache;
    const auto key = std::make_tuple(reinterpret_cast<const void*>(select_variant(c)), c.block, render_lds_bytes(c));
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, select_variant(c), c.block, render_lds_bytes(c)) != hipSuccess)
        return 1;
    n = n > 0 ? n : 1;
    std::lock_guard<std::mutex> g(mu);
    cache[key] = n;
    return n;
}

hipError_t launch_pack_code(const uint32_t* prim_id, const uint8_t* occ, uint8_t* code, size_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::pack_code_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, prim_id, occ, code, n);
    return hipGetLastError();
}

hipError_t launch_unshard(const unshard_params& u, hipStream_t s)
{
    dim3 block(256), grid((u.width + 255) / 256, u.height);
    hipLaunchKernelGGL(dev::unshard_kernel, grid, block, 0, s, u);
    return hipGetLastError();
}

} // namespace vrh
