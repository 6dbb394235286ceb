// visionaray_amd/csrc/vrh_kernels.hip -- traversal kernels for gfx950 (CDNA4).
//
// Replaces cuda_sched's render<<<grid,block>>> (cuda_sched.inl:53-153, one thread per pixel on a
// 2-D grid) with a persistent-thread design:
//   * the grid is sized to residency (CUs x blocks/CU); every wave pulls 8x8 pixel tiles from a
//     device-wide atomic counter until the frame's tiles are exhausted (work stealing, the
//     tiled_sched.inl:194 fetch_add moved onto the GPU); a wave's 64 lanes are one 8x8 tile, so
//     primary rays of a wave are coherent;
//   * each lane keeps its traversal stack in LDS (column-major, conflict-free);
//   * AO (ao/main.cpp:183-246) is fused: the hit pixels' 8 any-hit rays are generated on chip and
//     redistributed over the wave's lanes (ballot + mbcnt compaction through LDS), so no ray buffer
//     touches HBM and lanes whose pixel missed still trace AO rays.
#include "vrh_device.h"
#include "vrh_kernels.h"

namespace vrh {
namespace dev {

constexpr int BLOCK = 256;          // 4 waves
constexpr int TILE = 8;             // 8x8 pixels per wave
constexpr uint32_t BAND = 16;       // shard band height (tiled_sched tile_height)

// tile index -> (x, y) of lane, plus the output row (packed shards)
__device__ __forceinline__ bool tile_pixel(const render_params& P, uint32_t tile, uint32_t lane,
                                           uint32_t& x, uint32_t& y, uint32_t& out_row)
{
    uint32_t per_band = 2u * P.tiles_x;           // two 8-row tile rows per 16-row band
    uint32_t lb = tile / per_band;
    uint32_t r = tile - lb * per_band;
    uint32_t sub = r / P.tiles_x;
    uint32_t tx = r - sub * P.tiles_x;
    uint32_t band = lb * P.shard_count + P.shard_index;
    x = tx * TILE + (lane & 7u);
    uint32_t in_band = sub * TILE + (lane >> 3);
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

template <int KIND, int CAP, bool AO, bool COUNT>
__global__ __launch_bounds__(BLOCK) void render_kernel(render_params P)
{
    // LDS: traversal stacks [CAP][BLOCK] + per-wave AO work list (pixel slot per ray)
    __shared__ uint32_t stack_mem[CAP * BLOCK];
    __shared__ uint32_t ao_pix[AO ? BLOCK : 1];         // lane -> hit record slot, per wave 64
    __shared__ float ao_hit[AO ? BLOCK * 8 : 1];        // per lane: isect pos xyz, basis n xyz, t, pad

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = tid >> 6;
    lds_stack<CAP, BLOCK> st;
    st.col = stack_mem + tid;
    st.sp = 0;
    test_counts cnt = { 0u, 0u, false };

    for (;;)
    {
        uint32_t tile = 0;
        if (lane == 0) tile = atomicAdd(reinterpret_cast<uint32_t*>(P.counters), 1u);
        tile = __shfl(tile, 0);
        if (tile >= P.num_tiles) break;

        uint32_t x, y, orow;
        bool valid = tile_pixel(P, tile, lane, x, y, orow);

        hit_t h = miss_record();
        ray_t r;
        if (valid)
        {
            r = primary_ray(P, x, y);
            h = trace<KIND, false, COUNT>(P.pairs, P.prims, P.root, r, 3.402823466e+38f, st, cnt, P.step_limit);
        }
        float4 color = make_float4(P.bg[0], P.bg[1], P.bg[2], P.bg[3]);
        uint32_t occ_mask = 0;
        uint64_t hitmask = __ballot(valid && h.hit);
        uint32_t nrays = (uint32_t)__popcll(__ballot(valid));

        if constexpr (AO)
        {
            // ---- stage hit records of this wave in LDS -------------------------------------
            float* rec = ao_hit + (wave * 64u + lane) * 8u;
            if (valid && h.hit)
            {
                f3 pos = r.ori + r.dir * h.t;                       // ao/main.cpp:202
                float4 nn = P.normals[h.prim_id];                   // get_normal.h:26-37
                rec[0] = pos.x; rec[1] = pos.y; rec[2] = pos.z;
                rec[3] = nn.x; rec[4] = nn.y; rec[5] = nn.z;
                rec[6] = __uint_as_float(y * P.width + x);          // global pixel index p
            }
            // compact the hit lanes: slot k of the wave's list = k-th hit lane
            uint32_t hits = (uint32_t)__popcll(hitmask);
            uint32_t slot = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(hitmask >> 32),
                                 __builtin_amdgcn_mbcnt_lo((uint32_t)hitmask, 0u));
            uint32_t* list = ao_pix + wave * 64u;
            if (valid && h.hit) list[slot] = lane;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

            // ---- AO rays: ray j = (hit slot j / S, sample j % S), spread over all 64 lanes ----
            const uint32_t S = P.samples;
            const uint32_t total = hits * S;
            uint32_t my_occ_bits = 0;   // bits gathered for the lane's OWN pixel (set below)
            const float step = 1.0f / (float)S;
            for (uint32_t base = 0; base < total; base += 64u)
            {
                uint32_t j = base + lane;
                bool occl = false;
                uint32_t src_lane = 0, s = 0;
                if (j < total)
                {
                    uint32_t hs = j / S;
                    s = j - hs * S;
                    src_lane = list[hs];
                    const float* sr = ao_hit + (wave * 64u + src_lane) * 8u;
                    f3 pos = mk3(sr[0], sr[1], sr[2]);
                    f3 n = mk3(sr[3], sr[4], sr[5]);
                    uint32_t p = __float_as_uint(sr[6]);
                    // vector3.inl:357-367 make_orthonormal_basis(u, v, w = n)
                    f3 bv = fabsf(n.x) > fabsf(n.y) ? normalize(mk3(-n.z, 0.0f, n.x)) : normalize(mk3(0.0f, n.z, -n.y));
                    f3 bu = cross(bv, n);
                    f3 d = ao_direction(p, s, bu, bv, n);
                    ray_t ar = make_ray(pos + d * P.eps, d);
                    hit_t a = trace<KIND, true, COUNT>(P.pairs, P.prims, P.root, ar, P.radius, st, cnt, P.step_limit);
                    occl = a.hit;
                }
                // route occlusion bits back to the owning lanes: owner lane collects its bits
                uint64_t occ_ball = __ballot(occl);
                // each owner lane checks which of rays [base, base+64) are its own
                if (valid && h.hit)
                {
                    uint32_t my_first = slot * S;                    // my rays: [my_first, my_first+S)
                    for (uint32_t s2 = 0; s2 < S; ++s2)
                    {
                        uint32_t jj = my_first + s2;
                        if (jj >= base && jj < base + 64u && ((occ_ball >> (jj - base)) & 1ull))
                            my_occ_bits |= 1u << s2;
                    }
                }
                (void)src_lane;
            }
            nrays += total;
            if (valid && h.hit)
            {
                occ_mask = my_occ_bits;
                float clr = 1.0f;
                for (uint32_t s2 = 0; s2 < S; ++s2)
                    if ((occ_mask >> s2) & 1u) clr = clr - step;     // ao/main.cpp:234-238
                color = make_float4(clr, clr, clr, 1.0f);
            }
            __builtin_amdgcn_wave_barrier();
        }
        else
        {
            if (valid && h.hit) color = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
        }

        if (valid)
        {
            size_t o = (size_t)orow * P.width + x;
            if (P.color) P.color[o] = color;
            if (P.prim_id) P.prim_id[o] = h.hit ? h.prim_id : 0xFFFFFFFFu;
            if (P.t) P.t[o] = h.hit ? h.t : -1.0f;
            if (P.occ) P.occ[o] = (uint8_t)occ_mask;
        }
        if (__ballot(cnt.aborted) != 0ull && lane == 0) atomicOr(P.counters + 5, 1ull);
        if (lane == 0)
        {
            unsigned long long nh = (unsigned long long)__popcll(hitmask);
            atomicAdd(P.counters + 1, (unsigned long long)nrays);
            atomicAdd(P.counters + 2, nh);
            atomicAdd(P.counters + 8, (unsigned long long)nrays);
            atomicAdd(P.counters + 9, nh);
        }
    }
    if (COUNT)
    {
        // wave-reduce the per-lane test counts, one atomic per wave
        unsigned long long b = cnt.box, q = cnt.prim;
        for (int off = 32; off > 0; off >>= 1)
        {
            b += __shfl_down(b, off);
            q += __shfl_down(q, off);
        }
        if (lane == 0)
        {
            atomicAdd(P.counters + 3, b);
            atomicAdd(P.counters + 4, q);
        }
    }
}

// un-interleave gathered packed shards [count][bands_max*16][W] into the full image
__global__ void unshard_kernel(uint32_t W, uint32_t H, uint32_t count, uint32_t rows_per_shard,
                               const float4* __restrict__ gcolor, const uint32_t* __restrict__ gpid,
                               float4* __restrict__ color, uint32_t* __restrict__ pid)
{
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (x >= W || y >= H) return;
    uint32_t band = y / BAND;
    uint32_t g = band % count;
    uint32_t lrow = (band / count) * BAND + (y % BAND);
    size_t src = ((size_t)g * rows_per_shard + lrow) * W + x;
    size_t dst = (size_t)y * W + x;
    if (color && gcolor) color[dst] = gcolor[src];
    if (pid && gpid) pid[dst] = gpid[src];
}

} // namespace dev

// ------------------------------------------------------------------------------------------------

// one table entry per compiled variant: kind x AO x COUNT x stack capacity
struct variant
{
    void (*kernel)(render_params);
};

template <int KIND, int CAP, bool AO, bool COUNT>
static constexpr variant make_variant() { return { dev::render_kernel<KIND, CAP, AO, COUNT> }; }

template <int KIND, bool AO, bool COUNT>
static variant pick_cap(int cap)
{
    return cap <= 32 ? make_variant<KIND, 32, AO, COUNT>() : make_variant<KIND, 64, AO, COUNT>();
}

template <int KIND>
static variant pick(bool ao, bool count, int cap)
{
    if (ao) return count ? pick_cap<KIND, true, true>(cap) : pick_cap<KIND, true, false>(cap);
    return count ? pick_cap<KIND, false, true>(cap) : pick_cap<KIND, false, false>(cap);
}

static variant select_variant(int kind, bool ao, bool count, int cap)
{
    return kind == dev::KIND_TRI ? pick<dev::KIND_TRI>(ao, count, cap) : pick<dev::KIND_SPHERE>(ao, count, cap);
}

hipError_t launch_render(const render_params& p, int kind, bool ao, bool count, int cap, int grid, hipStream_t s)
{
    variant v = select_variant(kind, ao, count, cap);
    hipLaunchKernelGGL(v.kernel, dim3(grid), dim3(dev::BLOCK), 0, s, p);
    return hipGetLastError();
}

int render_blocks_per_cu(int kind, bool ao, bool count, int cap)
{
    variant v = select_variant(kind, ao, count, cap);
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, v.kernel, dev::BLOCK, 0) != hipSuccess) return 1;
    return n > 0 ? n : 1;
}

int render_block_threads() { return dev::BLOCK; }

hipError_t launch_unshard(uint32_t W, uint32_t H, uint32_t count, uint32_t rows_per_shard, const void* gcolor,
                          const uint32_t* gpid, void* color, uint32_t* pid, hipStream_t s)
{
    dim3 block(256), grid((W + 255) / 256, H);
    hipLaunchKernelGGL(dev::unshard_kernel, grid, block, 0, s, W, H, count, rows_per_shard,
                       (const float4*)gcolor, gpid, (float4*)color, pid);
    return hipGetLastError();
}

} // namespace vrh
