// visionaray_amd/csrc/vrh_kernels.h -- kernel launch interface (host side of vrh_kernels.hip).
#pragma once

#include "../../include/vrh.h"
#include "vrh_shade.h"

#include <hip/hip_runtime.h>
#include <cstdint>

namespace vrh {

struct frame_camera
{
    float eye[3], cam_u[3], cam_v[3], cam_w[3];
    uint32_t clip[4];         // scissor box clamped to the image: x0, y0, x1, y1 (exclusive)
};

constexpr uint32_t MAX_LIST = 8;   // BVHs of a scene list (VRH_MAX_SCENE_LIST)

struct render_params
{
    const float4* pairs;      // 4 float4 per inner node pair record
    const float4* prims;      // leaf-ordered primitives (3 float4 tri, 2 float4 sphere)
    const float4* normals;    // per prim_id
    uint32_t root;            // root link (pair 0, or LEAF_BIT|0 for a single-leaf tree) = roots[0]
    uint32_t roots[MAX_LIST]; // scene list (launch_config::sched 2): root link of each BVH
    uint32_t num_roots;
    uint32_t step_limit;      // per-ray traversal step bound (nodes + primitives)
    uint32_t stack_cap;       // LDS stack entries per lane
    uint32_t stack_total;     // stack entries per lane in all (>= BVH depth): LDS + global overflow
    uint32_t* stack_spill;    // overflow entries, (stack_total - stack_cap) x threads per block, per block
    uint32_t fast_ok;         // node bounds all finite: hardware min/max slab path allowed
    const float4* quads;      // 8 float4 per 4-wide any-hit record (vrh_quad.cpp)
    uint32_t quad_ok;         // any-hit rays with finite origin / inverse direction use `quads`

    frame_camera cam[VRH_MAX_BATCH];   // pinhole basis of every frame of the launch
    uint32_t num_frames;      // frames rendered by this launch (vrh_render_batch)
    uint32_t frame_num;       // frame number of frame 0 of the launch (frame f: frame_num + f), AO sampler offset
    uint32_t frame_rows;      // output rows per frame: frame f owns rows [f * frame_rows, (f + 1) * frame_rows)
    uint32_t width, height;
    float width_f, height_f;  // (float)width, (float)height (sched_common.h:137-138 divides by them)

    uint32_t samples;
    // ceil(2^20 / samples): (c * samples_recip) >> 20 == c / samples for every c < 64 * samples
    // (checked for samples 1..32: the error c * (recip - 2^20 / samples) / 2^20 stays below
    // 1 / samples), a multiply instead of a division whose reciprocal the compiler kept in a VGPR
    uint32_t samples_recip;
    float radius, eps;
    float bg[4];
    // pixel sampler pass (vrh_render_sampled): primary rays through (x + px_off, y + px_off) or, with
    // `jitter`, through the pixel's jittered position; colour stored (blend 0) or blended as
    // c * blend_s + dst * blend_d with dst read (1) or taken as 0 (2: ssaa's first sample)
    float px_off[2];
    uint32_t jitter, blend;
    float blend_s, blend_d;
    // camera matrices (vrh_render_view; pixel-sampler instances only): the ray of pixel (x, y) runs
    // through inv_view * (inv_proj * (u, v, -+1, 1)) instead of the pinhole basis of cam[f]
    uint32_t matrix_cam;
    float inv_view[16], inv_proj[16];   // column-major

    uint32_t shard_index, shard_count, packed;
    uint32_t tiles_x, num_tiles;   // tiles of ONE frame (the launch has num_frames x num_tiles units)

    float4* color;
    uint32_t* prim_id;
    float* t;
    uint8_t* occ;

    // counters (u64): [1] frame rays, [2] frame hits, [3] frame box tests, [4] frame primitive
    // tests, [5] frame error flags (1 = traversal step guard tripped), [6] [7] [9] [10] [11] SIMD
    // utilisation (wave steps, busy lane-steps, wave descent / leaf iterations, wave-uniform
    // descents; counting variant only), [8 + 8q] tile queue head q (q = 0..7, one 64-B line each),
    // [COUNTERS_LINES] vector-L1 line accesses and [COUNTERS_LINES + 1] wave-level vector-memory
    // instructions of the traversal loads (counting variant: the coalescer model, vrh_device.h
    // count_lines) -- [0, COUNTERS_FRAME) reset per frame -- [COUNTERS_TOTAL + 0/1] total rays / hits
    // since vrh_stats_reset
    unsigned long long* counters;
    uint32_t xcd_queues;      // 1: per-XCD tile queues (strips) with stealing; 2: per-XCD queues over
                              // band-interleaved (band, frame) units; 3: per-XCD strips in cluster
                              // order (cluster, frame, tile); 0: one global queue
    uint32_t cluster;         // xcd_queues 3: tiles per cluster (>= 1)
    uint32_t refill_min;      // retire / refill once this many lanes are free (AO step loop)
    uint32_t refill_min_primary;   // the same for the step loop's primary-only stream
    uint32_t ao_cut;          // AO step loop: any-hit rays start at the tile's cut of the 4-wide tree
                              // (1: entries in cut order, 2: nearest-first)
    uint32_t ao_gate;         // AO step loop: a tile's AO rays are handed out once its primaries are done
    uint32_t ao_share;        // AO step loop, blocks of several waves: tail sharing of the last tiles' AO rays
    unsigned long long* wave_times;   // VRH_OPT_WAVE_TIMES: per wave (start, end) of wall_clock64(), else null
    // VRH_OPT_WAVE_TIMES = 2, counting kernels of one-frame AO launches: per tile (hand-out, primaries
    // done, pixels written) of wall_clock64() -- where a launch's tail comes from
    unsigned long long* tile_times;
    uint32_t descent_cap;     // step loop: inner visits per step before a descent is resumed later
    uint32_t step_flags;      // step loop: bit 0 a descent that misses both children pops and continues;
                              // bit 1 wave-uniform pair records fetched through the scalar cache
    dev::shade_params shade;  // VRH_KERNEL_SIMPLE / MULTI_HIT: materials, lights, normal binding, ambient
    uint32_t max_hits;        // VRH_KERNEL_MULTI_HIT: N
    uint32_t num_bounces;     // VRH_KERNEL_WHITTED: loop iterations (eps = scene epsilon)
    uint32_t* mh_prim_id;     // [pixel][N] hit lists (render target side buffers)
    float* mh_t;
    dev::hit_mask_params hmask;   // mask intersector (vrh_hit_mask), hmask.mask == null: none
};

constexpr int COUNTERS_FRAME = 208;     // u64 words reset before every frame
constexpr int COUNTERS_LINES = 80;      // [80] L1 128-B lines, [81] wave-level vector-memory instructions, [82] 16-B requests,
                                        // [83] 4-lane-group accesses, [84] ideal-grouping accesses (counting variant)
constexpr int COUNTERS_TOTAL = 208;     // u64 words [208], [209]: totals
constexpr int COUNTERS_WORDS = 256;
constexpr int VRH_MAX_FRAME_LANES = 4;  // asynchronous frames: frame lanes of a context, at most
#ifndef VRH_DEFAULT_FRAME_LANES
// VRH_OPT_ASYNC_FRAMES = 1.  Measured (round 6, tools/async_lanes_ab.py, ten frames into one target,
// profiles/r06/async_lanes/): 3 lanes 8-10 % slower than 2 on C2 / C3 / C4 / C5, 4 lanes within -1..+1 %
// of 2.  Why 3 loses is not established (the process has 4 hardware queues, GPU_MAX_HW_QUEUES, for the
// context stream and the lanes); 2 stays the default, 3 and 4 are selectable and tested
#define VRH_DEFAULT_FRAME_LANES 2
#endif
constexpr int COUNTER_BLOCKS = 1 + VRH_MAX_FRAME_LANES;   // per context: frames on its stream + one per frame lane

struct launch_config
{
    int kind;          // 0 triangles, 1 spheres
    bool ao;
    bool count;        // VRH_KERNEL_COUNT_TESTS variant
    int block;         // threads per block (multiple of 64)
    int stack_cap;     // LDS stack entries per lane
    int occ;           // register budget: min waves per SIMD (1, 6 or 8)
    int sched;         // 0: step loop (render_unified_kernel),
                       // 2: step loop over a BVH list (render_unified_kernel<..., LIST>),
                       // 3: step loop, frames in flight (render_unified_kernel<..., BATCH>: same code),
                       // 6: a pixel-sampler pass (render_unified_kernel<..., SAMPLED>)
    int epi;           // primary epilogue: 0 plain, 1 VRH_KERNEL_SIMPLE, 2 VRH_KERNEL_MULTI_HIT, 3 VRH_KERNEL_WHITTED (triangles)
    int max_hits;      // MULTI_HIT: N (LDS hit lists)
    bool spill;        // the traversal stack continues in a global overflow block (render_unified_kernel<..., SPILL>)
    bool share;        // AO tail sharing (render_unified_kernel<..., SHARE>): one-frame AO launches at 5 waves / SIMD
};

size_t render_lds_bytes(const launch_config& c);
hipError_t launch_render(const render_params& p, const launch_config& c, int grid, hipStream_t s);
int render_blocks_per_cu(const launch_config& c);
bool render_spill_available(const launch_config& c);   // an overflow-stack instance exists for c
bool render_share_available(const launch_config& c);   // an AO tail-sharing instance exists for c
struct unshard_params
{
    uint32_t width, height, count, rows_per_shard;
    const char* gcolor;          // gathered colour (float4), or null: re-derive from prim id + occ
    const char* gpid;            // gathered prim ids (u32)
    const char* gocc;            // gathered AO masks (u8)
    const char* gt;              // gathered closest-hit t (f32), or null
    const char* gcode;           // gathered colour codes (u8: 0xFF miss, else occluded samples), or null
    uint64_t stride_color, stride_pid, stride_occ, stride_t, stride_code;   // bytes between consecutive shards
    float4* color;
    uint32_t* pid;
    uint8_t* occ;
    float* t;
    uint32_t ao, samples;        // colour re-derivation (kernel kind, AO samples)
    float bg[4];
    uint32_t clip[4];            // scissor box x0, y0, x1, y1: pixels outside are left untouched
};
hipError_t launch_unshard(const unshard_params& u, hipStream_t s);
// colour codes of n rendered pixels: 0xFF where prim_id is a miss, else the popcount of the AO mask
// (occ null: 0)
hipError_t launch_pack_code(const uint32_t* prim_id, const uint8_t* occ, uint8_t* code, size_t n, hipStream_t s);

} // namespace vrh
