// visionaray_amd/csrc/vrh_plan.h -- the render-group plan, host and device code in
// one place: which shards a rank renders and in which order it sends them, which rank the root
// receives shard s from, the byte layout of a packed shard on the wire, where an image row lives in a
// packed shard, the one-byte colour code and the root's un-interleave of a pixel.  vrh_group.hip
// (vrh_render_sharded), the unshard / pack kernels of vrh_kernels.hip and the host exports of vrh.h
// (vrh_group_shards_of, vrh_group_wire_layout, vrh_shard_packed_rows, vrh_pack_codes_host,
// vrh_unshard_host -- what the multi-process CPU tests drive) all call these functions, so the
// protocol the tests check is the one the GPUs run.
#pragma once

#include "vrh_kernels.h"

#include <cstdint>
#include <cstring>

namespace vrh {
namespace plan {

constexpr uint32_t BAND = VRH_BAND_ROWS;

__host__ __device__ inline uint32_t bands_of(uint32_t height) { return (height + BAND - 1u) / BAND; }

// bands shard `index` of `count` owns: band b -> shard b % count
__host__ __device__ inline uint32_t shard_bands(uint32_t height, uint32_t index, uint32_t count)
{
    const uint32_t bands = bands_of(height);
    if (count == 0u || index >= count || index >= bands) return 0u;
    return (bands - index + count - 1u) / count;
}

// shards rank `rank` of `nranks` renders (0 when shards <= rank): s = rank, rank + N, ...
__host__ __device__ inline uint32_t owned_count(uint32_t shards, uint32_t nranks, uint32_t rank)
{
    return shards > rank ? (shards - rank + nranks - 1u) / nranks : 0u;
}
// the j-th shard rank renders -- also the order in which it sends them to the root
__host__ __device__ inline uint32_t owned_shard(uint32_t rank, uint32_t nranks, uint32_t j) { return rank + j * nranks; }
// the rank that renders shard s: the root receives shard s (s = 0, 1, ...) from it, so sends and
// receives pair up in order per peer
__host__ __device__ inline uint32_t shard_owner(uint32_t shard, uint32_t nranks) { return shard % nranks; }

// image row y -> (shard, row inside the packed shard)
__host__ __device__ inline void row_home(uint32_t y, uint32_t shards, uint32_t& shard, uint32_t& lrow)
{
    const uint32_t band = y / BAND;
    shard = band % shards;
    lrow = (band / shards) * BAND + (y % BAND);
}

// what one pixel of a shard carries over the wire for a root target with buffers `fields`
struct wire_layout
{
    bool pid = false, occ = false, t = false, color = false;
    bool derive = false;                   // colour re-derived on the root from prim id (+ AO mask)
    bool code = false;                     // ... from one byte: 0xFF miss, else the occluded-sample count
    size_t bytes_per_px() const { return (pid ? 4 : 0) + (occ ? 1 : 0) + (t ? 4 : 0) + (color ? 16 : 0) + (code ? 1 : 0); }
};

inline wire_layout layout_for(uint32_t fields, const vrh_kernel_desc& k)
{
    wire_layout w;
    const bool builtin_colour = k.kind <= VRH_KERNEL_AO && (k.kind != VRH_KERNEL_AO || k.samples <= 8);
    w.derive = (fields & VRH_RT_COLOR) && builtin_colour;
    w.color = (fields & VRH_RT_COLOR) && !builtin_colour;
    w.pid = (fields & VRH_RT_PRIM_ID) || w.derive;
    w.occ = k.kind == VRH_KERNEL_AO && (((fields & VRH_RT_OCC) && k.samples <= 8) || w.derive);
    w.t = (fields & VRH_RT_T) != 0;
    // a colour target without prim id / mask targets: the built-in colour depends only on hit and
    // the number of occluded samples (ao/main.cpp:234-238), so 1 B per pixel crosses the wire, not 5
    w.code = w.derive && !(fields & VRH_RT_PRIM_ID) && !(fields & VRH_RT_OCC);
    if (w.code) w.pid = w.occ = false;
    return w;
}

// byte offsets of the fields in one packed shard of `px` pixels (all frames): [prim ids | masks | t |
// colour | codes], every field for every frame of the shard
struct wire_offsets
{
    size_t pid, occ, t, col, code, shard_bytes;
};
inline wire_offsets offsets_for(const wire_layout& w, size_t px)
{
    wire_offsets o;
    o.pid = 0;
    o.occ = o.pid + (w.pid ? 4 * px : 0);
    o.t = o.occ + (w.occ ? px : 0);
    o.col = o.t + (w.t ? 4 * px : 0);
    o.code = o.col + (w.color ? 16 * px : 0);
    o.shard_bytes = w.bytes_per_px() * px;
    return o;
}

// one code byte per rendered pixel: 0xFF on a miss, else the number of occluded AO samples
__host__ __device__ inline uint8_t pack_code(uint32_t pid, const uint8_t* occ, size_t i)
{
    if (pid == 0xFFFFFFFFu) return 0xFFu;
    if (!occ) return 0u;
    uint32_t m = occ[i], c = 0;
    for (; m; m &= m - 1u) ++c;
    return (uint8_t)c;
}

// the root's un-interleave of pixel (x, y) of one frame from the gathered packed shards, re-deriving the
// RGBA32F colour of the built-in kernels exactly as the traversal kernel writes it
__host__ __device__ inline void unshard_pixel(const unshard_params& u, uint32_t x, uint32_t y)
{
    if (x >= u.width || y >= u.height) return;
    if (x < u.clip[0] || y < u.clip[1] || x >= u.clip[2] || y >= u.clip[3]) return;
    uint32_t g, lrow;
    row_home(y, u.count, g, lrow);
    const size_t src = (size_t)lrow * u.width + x;
    const size_t dst = (size_t)y * u.width + x;
    uint32_t pid = u.gpid ? reinterpret_cast<const uint32_t*>(u.gpid + g * u.stride_pid)[src] : 0xFFFFFFFFu;
    const uint32_t occ = u.gocc ? (u.gocc + g * u.stride_occ)[src] : 0u;
    uint32_t count = 0xFFFFFFFFu;                           // occluded samples, from a colour code
    if (u.gcode)
    {
        const uint32_t c = (uint8_t)(u.gcode + g * u.stride_code)[src];
        pid = c == 0xFFu ? 0xFFFFFFFFu : 0u;
        count = c;
    }
    if (u.pid && u.gpid) u.pid[dst] = pid;
    if (u.occ && u.gocc) u.occ[dst] = (uint8_t)occ;
    if (u.t && u.gt) u.t[dst] = reinterpret_cast<const float*>(u.gt + g * u.stride_t)[src];
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
                if (count != 0xFFFFFFFFu ? s < count : ((occ >> s) & 1u) != 0u) clr = clr - step;   // ao/main.cpp:234-238
        }
        c = make_float4(clr, clr, clr, 1.0f);
    }
    u.color[dst] = c;
}

// the un-interleave parameters of frame f of a vrh_render_sharded call: the gathered shards at `recv`
// (S shards of `o.shard_bytes`), `rows` packed rows per shard and frame, into the frame's rows of the
// destination buffers (any may be null); scissor box `sb` (all zero: the whole image)
inline unshard_params frame_params(const wire_layout& wl, const wire_offsets& o, const uint8_t* recv, uint32_t W,
                                   uint32_t H, uint32_t S, uint32_t rows, uint32_t f, uint32_t fields,
                                   const vrh_kernel_desc& k, float4* color, uint32_t* prim_id, uint8_t* occ, float* t,
                                   const uint32_t* sb)
{
    unshard_params u{};
    const size_t fpx = size_t(rows) * W;               // pixels of one frame of one shard
    u.width = W; u.height = H; u.count = S; u.rows_per_shard = rows;
    u.gpid = wl.pid ? reinterpret_cast<const char*>(recv + o.pid + 4 * f * fpx) : nullptr;
    u.gocc = wl.occ ? reinterpret_cast<const char*>(recv + o.occ + f * fpx) : nullptr;
    u.gt = wl.t ? reinterpret_cast<const char*>(recv + o.t + 4 * f * fpx) : nullptr;
    u.gcolor = wl.color ? reinterpret_cast<const char*>(recv + o.col + 16 * f * fpx) : nullptr;
    u.gcode = wl.code ? reinterpret_cast<const char*>(recv + o.code + f * fpx) : nullptr;
    u.stride_pid = u.stride_occ = u.stride_t = u.stride_color = u.stride_code = o.shard_bytes;
    const size_t fo = size_t(f) * W * H;
    u.color = (fields & VRH_RT_COLOR) && color ? color + fo : nullptr;
    u.pid = (fields & VRH_RT_PRIM_ID) && prim_id ? prim_id + fo : nullptr;
    u.occ = (fields & VRH_RT_OCC) && wl.occ && occ ? occ + fo : nullptr;
    u.t = (fields & VRH_RT_T) && t ? t + fo : nullptr;
    u.ao = k.kind == VRH_KERNEL_AO ? 1u : 0u;
    u.samples = k.samples ? k.samples : 1u;
    std::memcpy(u.bg, k.bg, 16);
    const bool whole = sb[0] == 0 && sb[1] == 0 && sb[2] == 0 && sb[3] == 0;
    u.clip[0] = whole ? 0u : (sb[0] < W ? sb[0] : W); u.clip[1] = whole ? 0u : (sb[1] < H ? sb[1] : H);
    u.clip[2] = whole ? W : (sb[2] < W ? sb[2] : W); u.clip[3] = whole ? H : (sb[3] < H ? sb[3] : H);
    return u;
}

} // namespace plan
} // namespace vrh
