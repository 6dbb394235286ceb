// visionaray_amd/csrc/vrh_lbvh.hip -- GPU BVH construction.
//
// A linear BVH (Karras 2012: Morton-ordered primitives, one hierarchy node per pair of adjacent
// codes found by a prefix-length binary search, bottom-up bounds by atomically counted arrivals),
// collapsed to leaves of up to `max_leaf` primitives and emitted directly in the two layouts the
// traversal needs:
//   * the reference's bvh_node array (bvh.h:52-119; root at 0, children as pairs at odd indices,
//     build.inl:45-50) + index array, kept for download, oracle parity and sah_cost;
//   * the device pair records and leaf-ordered primitives of vrh_scene_upload (vrh_device.h).
// The tree differs from build<index_bvh<P>> (binned SAH, host), so closest-hit ties on shared edges
// may resolve to a different primitive; its quality is gated by sah_cost (statistics.h) in tests.
//
// Kernels are HBM-bound integer/float streaming passes over n primitives plus a radix sort
// (rocPRIM) of 30-bit Morton codes; everything stays on the device.
#include "vrh_internal.h"
#include "vrh_lbvh.h"

#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstring>
#include <string>

namespace vrh {
namespace lbvh {

constexpr uint32_t LEAF_FLAG = 0x80000000u;

struct aabb_t { float4 lo, hi; };

__device__ __forceinline__ uint32_t f2ord(float f)             // order-preserving float -> uint
{
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u)
{
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// primitive bounds the way the reference's get_bounds computes them (v1, v1 + e1, v1 + e2;
// center -/+ radius), centroids, scene-wide centroid bounds, finiteness and id maxima
__global__ void k_prim_bounds(const float4* __restrict__ raw, uint32_t n, uint32_t kind, aabb_t* __restrict__ box,
                              uint32_t* __restrict__ gstat)
{
    // gstat: [0..2] centroid min (ordered), [3..5] centroid max, [6] non-finite flag, [7] max prim_id,
    // [8] max geom_id
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    float3 cmin = make_float3(INFINITY, INFINITY, INFINITY), cmax = make_float3(-INFINITY, -INFINITY, -INFINITY);
    uint32_t bad = 0, mpid = 0, mgid = 0;
    if (i < n)
    {
        float3 lo, hi;
        uint32_t gid, pid;
        if (kind == VRH_PRIM_TRI64)
        {
            const float4* t = raw + 4u * i;                 // geom_id prim_id pad pad | v1 | e1 | e2
            const float4 h = t[0], v1 = t[1], e1 = t[2], e2 = t[3];
            gid = __float_as_uint(h.x); pid = __float_as_uint(h.y);
            const float3 a = make_float3(v1.x, v1.y, v1.z);
            const float3 b = make_float3(v1.x + e1.x, v1.y + e1.y, v1.z + e1.z);
            const float3 c = make_float3(v1.x + e2.x, v1.y + e2.y, v1.z + e2.z);
            lo = make_float3(fminf(fminf(a.x, b.x), c.x), fminf(fminf(a.y, b.y), c.y), fminf(fminf(a.z, b.z), c.z));
            hi = make_float3(fmaxf(fmaxf(a.x, b.x), c.x), fmaxf(fmaxf(a.y, b.y), c.y), fmaxf(fmaxf(a.z, b.z), c.z));
        }
        else
        {
            const float4* s = raw + 3u * i;                 // geom_id prim_id pad pad | center | radius
            const float4 h = s[0], c = s[1], r = s[2];
            gid = __float_as_uint(h.x); pid = __float_as_uint(h.y);
            lo = make_float3(c.x - r.x, c.y - r.x, c.z - r.x);
            hi = make_float3(c.x + r.x, c.y + r.x, c.z + r.x);
        }
        box[i].lo = make_float4(lo.x, lo.y, lo.z, 0.0f);
        box[i].hi = make_float4(hi.x, hi.y, hi.z, 0.0f);
        const float3 cen = make_float3((lo.x + hi.x) * 0.5f, (lo.y + hi.y) * 0.5f, (lo.z + hi.z) * 0.5f);
        bad = !(isfinite(lo.x) && isfinite(lo.y) && isfinite(lo.z) && isfinite(hi.x) && isfinite(hi.y) && isfinite(hi.z));
        if (!bad) { cmin = cen; cmax = cen; }
        mpid = pid; mgid = gid;
    }
    // wave reduction, one atomic per wave and quantity
    for (int off = 32; off > 0; off >>= 1)
    {
        cmin.x = fminf(cmin.x, __shfl_xor(cmin.x, off)); cmin.y = fminf(cmin.y, __shfl_xor(cmin.y, off));
        cmin.z = fminf(cmin.z, __shfl_xor(cmin.z, off));
        cmax.x = fmaxf(cmax.x, __shfl_xor(cmax.x, off)); cmax.y = fmaxf(cmax.y, __shfl_xor(cmax.y, off));
        cmax.z = fmaxf(cmax.z, __shfl_xor(cmax.z, off));
        bad |= __shfl_xor(bad, off);
        mpid = max(mpid, (uint32_t)__shfl_xor((int)mpid, off));
        mgid = max(mgid, (uint32_t)__shfl_xor((int)mgid, off));
    }
    if ((threadIdx.x & 63u) == 0)
    {
        atomicMin(gstat + 0, f2ord(cmin.x)); atomicMin(gstat + 1, f2ord(cmin.y)); atomicMin(gstat + 2, f2ord(cmin.z));
        atomicMax(gstat + 3, f2ord(cmax.x)); atomicMax(gstat + 4, f2ord(cmax.y)); atomicMax(gstat + 5, f2ord(cmax.z));
        if (bad) atomicOr(gstat + 6, 1u);
        atomicMax(gstat + 7, mpid);
        atomicMax(gstat + 8, mgid);
    }
}

__device__ __forceinline__ uint32_t expand10(uint32_t v)          // 10 bits -> every third bit
{
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void k_morton(const aabb_t* __restrict__ box, uint32_t n, const uint32_t* __restrict__ gstat,
                         uint32_t* __restrict__ codes, uint32_t* __restrict__ ids)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float lo[3] = { ord2f(gstat[0]), ord2f(gstat[1]), ord2f(gstat[2]) };
    const float hi[3] = { ord2f(gstat[3]), ord2f(gstat[4]), ord2f(gstat[5]) };
    const float c[3] = { (box[i].lo.x + box[i].hi.x) * 0.5f, (box[i].lo.y + box[i].hi.y) * 0.5f,
                         (box[i].lo.z + box[i].hi.z) * 0.5f };
    // one scale for all axes (the centroid bounds' largest extent): a cube keeps the Morton
    // splits spatially balanced for flat or elongated scenes
    const float ext = fmaxf(fmaxf(hi[0] - lo[0], hi[1] - lo[1]), hi[2] - lo[2]);
    uint32_t q[3];
    for (int a = 0; a < 3; ++a)
    {
        float u = ext > 0.0f ? (c[a] - lo[a]) / ext : 0.5f;
        u = isfinite(u) ? fminf(fmaxf(u, 0.0f), 1.0f) : 0.5f;
        q[a] = min((uint32_t)(u * 1024.0f), 1023u);
    }
    codes[i] = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
    ids[i] = i;
}

// longest common prefix of sorted keys i and j, ties broken by index (Karras 2012 §4)
__device__ __forceinline__ int delta(const uint32_t* __restrict__ codes, int n, int i, int j)
{
    if (j < 0 || j >= n) return -1;
    const uint32_t a = codes[i], b = codes[j];
    if (a == b) return 32 + __clz((uint32_t)(i ^ j));
    return __clz(a ^ b);
}

// one thread per hierarchy node i in [0, n-1): its key range, split, children and parents.
// child encoding: LEAF_FLAG | sorted position, or internal node index
__global__ void k_karras(const uint32_t* __restrict__ codes, int n, uint32_t* __restrict__ child,
                         uint2* __restrict__ range, uint32_t* __restrict__ parent_int, uint32_t* __restrict__ parent_leaf)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(codes, n, i, i + 1) - delta(codes, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(codes, n, i, i - d);
    int lmax = 2;
    while (delta(codes, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (delta(codes, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(codes, n, i, j);
    int s = 0;
    int t = l;
    for (;;)
    {
        t = (t + 1) >> 1;
        if (delta(codes, n, i, i + (s + t) * d) > dnode) s += t;
        if (t <= 1) break;
    }
    const int gamma = i + s * d + min(d, 0);
    const int first = min(i, j), last = max(i, j);
    const uint32_t left = (first == gamma) ? (LEAF_FLAG | (uint32_t)gamma) : (uint32_t)gamma;
    const uint32_t right = (last == gamma + 1) ? (LEAF_FLAG | (uint32_t)(gamma + 1)) : (uint32_t)(gamma + 1);
    child[2 * i] = left;
    child[2 * i + 1] = right;
    range[i] = make_uint2((uint32_t)first, (uint32_t)last);
    if (left & LEAF_FLAG) parent_leaf[gamma] = (uint32_t)i; else parent_int[gamma] = (uint32_t)i;
    if (right & LEAF_FLAG) parent_leaf[gamma + 1] = (uint32_t)i; else parent_int[gamma + 1] = (uint32_t)i;
}

__device__ __forceinline__ aabb_t merge(aabb_t a, aabb_t b)
{
    aabb_t r;
    r.lo = make_float4(fminf(a.lo.x, b.lo.x), fminf(a.lo.y, b.lo.y), fminf(a.lo.z, b.lo.z), 0.0f);
    r.hi = make_float4(fmaxf(a.hi.x, b.hi.x), fmaxf(a.hi.y, b.hi.y), fmaxf(a.hi.z, b.hi.z), 0.0f);
    return r;
}

__device__ __forceinline__ aabb_t load_aabb_coherent(const aabb_t* p)
{
    // bounds written by another workgroup: bypass the (non-coherent) L1
    aabb_t r;
    const float* f = reinterpret_cast<const float*>(p);
    r.lo = make_float4(__hip_atomic_load(f + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load(f + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load(f + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0.0f);
    r.hi = make_float4(__hip_atomic_load(f + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load(f + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load(f + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0.0f);
    return r;
}

__device__ __forceinline__ void store_aabb_coherent(aabb_t* p, aabb_t v)
{
    float* f = reinterpret_cast<float*>(p);
    __hip_atomic_store(f + 0, v.lo.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(f + 1, v.lo.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(f + 2, v.lo.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(f + 4, v.hi.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(f + 5, v.hi.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(f + 6, v.hi.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bottom-up bounds: every leaf climbs; at each node the second arrival (atomic counter) merges the
// two children and continues, the first stops.  Every thread ends (the root is reached once).
__global__ void k_refit(const aabb_t* __restrict__ leaf_box, const uint32_t* __restrict__ order, int n,
                        const uint32_t* __restrict__ child, const uint32_t* __restrict__ parent_int,
                        const uint32_t* __restrict__ parent_leaf, aabb_t* __restrict__ node_box,
                        uint32_t* __restrict__ arrivals)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint32_t node = parent_leaf[k];
    for (int guard = 0; guard < 64 * 1024; ++guard)
    {
        __threadfence();
        if (atomicAdd(arrivals + node, 1u) == 0u) return;          // sibling not done yet
        __threadfence();
        const uint32_t a = child[2 * node], b = child[2 * node + 1];
        const aabb_t ba = (a & LEAF_FLAG) ? leaf_box[order[a & ~LEAF_FLAG]] : load_aabb_coherent(node_box + a);
        const aabb_t bb = (b & LEAF_FLAG) ? leaf_box[order[b & ~LEAF_FLAG]] : load_aabb_coherent(node_box + b);
        store_aabb_coherent(node_box + node, merge(ba, bb));
        if (node == 0u) return;
        node = parent_int[node];
    }
}

__global__ void k_visible(const uint2* __restrict__ range, int m, uint32_t max_leaf, uint32_t* __restrict__ vis)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    vis[j] = (range[j].y - range[j].x + 1u > max_leaf) ? 1u : 0u;
}

// emit, for every visible node j (slot s = slot[j]): its two children as reference bvh_nodes at
// 2s+1, 2s+2 and as device pair record s; the root node at 0.  Leaves (single primitives or
// collapsed subtrees) cover contiguous Morton ranges; their last primitive gets the END flag.
__global__ void k_emit(const uint32_t* __restrict__ child, const uint2* __restrict__ range,
                       const uint32_t* __restrict__ vis, const uint32_t* __restrict__ slot,
                       const aabb_t* __restrict__ node_box, const aabb_t* __restrict__ leaf_box,
                       const uint32_t* __restrict__ order, int m, node32* __restrict__ nodes,
                       float4* __restrict__ pairs, uint8_t* __restrict__ end_flag, uint32_t* __restrict__ owner)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m || !vis[j]) return;
    const uint32_t s = slot[j];
    owner[s] = (uint32_t)j;
    if (j == 0)
    {
        const aabb_t r = node_box[0];
        node32 root{};
        root.bmin[0] = r.lo.x; root.bmin[1] = r.lo.y; root.bmin[2] = r.lo.z;
        root.bmax[0] = r.hi.x; root.bmax[1] = r.hi.y; root.bmax[2] = r.hi.z;
        root.first = 2u * s + 1u;
        root.num_prims = 0;
        nodes[0] = root;
    }
    aabb_t cb[2];
    uint32_t link[2];
    for (int side = 0; side < 2; ++side)
    {
        const uint32_t c = child[2 * j + side];
        node32 out{};
        aabb_t b;
        if (c & LEAF_FLAG)
        {
            const uint32_t p = c & ~LEAF_FLAG;
            b = leaf_box[order[p]];
            out.first = p; out.num_prims = 1;
            link[side] = LEAF_FLAG | p;
            end_flag[p] = 1;
        }
        else if (vis[c])
        {
            b = node_box[c];
            out.first = 2u * slot[c] + 1u; out.num_prims = 0;
            link[side] = slot[c];
        }
        else
        {
            b = node_box[c];
            out.first = range[c].x; out.num_prims = range[c].y - range[c].x + 1u;
            link[side] = LEAF_FLAG | range[c].x;
            end_flag[range[c].y] = 1;
        }
        out.bmin[0] = b.lo.x; out.bmin[1] = b.lo.y; out.bmin[2] = b.lo.z;
        out.bmax[0] = b.hi.x; out.bmax[1] = b.hi.y; out.bmax[2] = b.hi.z;
        nodes[2u * s + 1u + side] = out;
        cb[side] = b;
    }
    // device pair record (vrh_device.h layout)
    float4* q = pairs + 4u * s;
    q[0] = make_float4(cb[0].lo.x, cb[1].lo.x, cb[0].lo.y, cb[1].lo.y);
    q[1] = make_float4(cb[0].lo.z, cb[1].lo.z, cb[0].hi.x, cb[1].hi.x);
    q[2] = make_float4(cb[0].hi.y, cb[1].hi.y, cb[0].hi.z, cb[1].hi.z);
    q[3] = make_float4(__uint_as_float(link[0]), __uint_as_float(link[1]), 0.0f, 0.0f);
}

// depth of every visible node's children (root depth 0) by climbing the hierarchy
__global__ void k_depth(const uint32_t* __restrict__ vis, const uint32_t* __restrict__ parent_int, int m,
                        uint32_t* __restrict__ max_depth)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m || !vis[j]) return;
    uint32_t d = 1, node = (uint32_t)j;
    while (node != 0u && d < 1u << 20) { node = parent_int[node]; ++d; }
    atomicMax(max_depth, d);
}

// leaf-ordered primitives with END flags (the vrh_scene_upload layout, vrh_device.h)
__global__ void k_prims(const float4* __restrict__ raw, const uint32_t* __restrict__ order, const uint8_t* end_flag,
                        uint32_t n, uint32_t kind, float4* __restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t src = order[i], flags = end_flag[i] ? 1u : 0u;
    if (kind == VRH_PRIM_TRI64)
    {
        const float4* t = raw + 4u * src;
        const float4 h = t[0], v1 = t[1], e1 = t[2], e2 = t[3];
        float4* q = out + 3u * i;
        q[0] = make_float4(v1.x, v1.y, v1.z, e1.x);
        q[1] = make_float4(e1.y, e1.z, e2.x, e2.y);
        q[2] = make_float4(e2.z, h.y, h.x, __uint_as_float(flags));
    }
    else
    {
        const float4* s = raw + 3u * src;
        const float4 h = s[0], c = s[1], r = s[2];
        float4* q = out + 2u * i;
        q[0] = make_float4(c.x, c.y, c.z, r.x);
        q[1] = make_float4(h.y, h.x, __uint_as_float(flags), 0.0f);
    }
}

} // namespace lbvh

namespace {
inline unsigned blocks(size_t n, unsigned b) { return unsigned((n + b - 1) / b); }
}

int build_lbvh(const void* prims_host, uint32_t n, uint32_t kind, uint32_t max_leaf, hipStream_t stream,
               lbvh_out& out, std::string& err)
{
    using namespace lbvh;
    out = lbvh_out{};
    const size_t psz = kind == VRH_PRIM_TRI64 ? 64u : 48u;
    max_leaf = std::max(1u, std::min(max_leaf, 64u));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<void*> tmp;
    auto dalloc = [&](void** p, size_t bytes) -> bool {
        if (hipMalloc(p, std::max<size_t>(bytes, 16)) != hipSuccess) return false;
        return true;
    };
    auto fail = [&](const char* what) {
        err = std::string("GPU BVH build: ") + what + ": " + hipGetErrorString(hipGetLastError());
        for (void* p : tmp) (void)hipFree(p);
        for (void* p : { (void*)out.nodes, (void*)out.pairs, (void*)out.prims, (void*)out.indices })
            if (p) (void)hipFree(p);
        out = lbvh_out{};
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        return VRH_ERR_HIP;
    };
    const uint32_t m = n > 0 ? n - 1 : 0;                     // hierarchy nodes
    float4* raw = nullptr; aabb_t* box = nullptr; uint32_t* gstat = nullptr;
    uint32_t *codes = nullptr, *codes2 = nullptr, *ids = nullptr, *order = nullptr;
    uint32_t *child = nullptr, *pint = nullptr, *pleaf = nullptr, *arrivals = nullptr, *vis = nullptr, *slot = nullptr;
    uint2* range = nullptr; aabb_t* nbox = nullptr; uint8_t* endf = nullptr; uint32_t* owner = nullptr;
    uint32_t* dmax = nullptr;
    if (!dalloc((void**)&raw, n * psz)) return fail("alloc");
    tmp.push_back(raw);
    if (hipMemcpyAsync(raw, prims_host, n * psz, hipMemcpyHostToDevice, stream) != hipSuccess) return fail("upload");
    (void)hipEventRecord(e0, stream);
    const size_t need[] = { n * sizeof(aabb_t), 16 * 4, n * 4, n * 4, n * 4, n * 4, 2 * size_t(m) * 4, size_t(m) * 8,
                            size_t(m) * 4, size_t(n) * 4, size_t(m) * 4, size_t(m) * 4, size_t(m) * 4,
                            size_t(m) * sizeof(aabb_t), n, size_t(m) * 4, 4 };
    void** ptrs[] = { (void**)&box, (void**)&gstat, (void**)&codes, (void**)&codes2, (void**)&ids, (void**)&order,
                      (void**)&child, (void**)&range, (void**)&pint, (void**)&pleaf, (void**)&arrivals, (void**)&vis,
                      (void**)&slot, (void**)&nbox, (void**)&endf, (void**)&owner, (void**)&dmax };
    for (size_t k = 0; k < sizeof(ptrs) / sizeof(ptrs[0]); ++k)
    {
        if (!dalloc(ptrs[k], need[k])) return fail("alloc");
        tmp.push_back(*ptrs[k]);
    }
    uint32_t init[16] = { 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0, 0, 0, 0, 0 };
    if (hipMemcpyAsync(gstat, init, sizeof(init), hipMemcpyHostToDevice, stream) != hipSuccess) return fail("init");
    hipLaunchKernelGGL(k_prim_bounds, dim3(blocks(n, 256)), dim3(256), 0, stream, raw, n, kind, box, gstat);
    hipLaunchKernelGGL(k_morton, dim3(blocks(n, 256)), dim3(256), 0, stream, box, n, gstat, codes, ids);
    size_t tsz = 0;
    if (rocprim::radix_sort_pairs(nullptr, tsz, codes, codes2, ids, order, n, 0, 30, stream) != hipSuccess) return fail("sort size");
    void* tstore = nullptr;
    if (!dalloc(&tstore, tsz)) return fail("alloc");
    tmp.push_back(tstore);
    if (rocprim::radix_sort_pairs(tstore, tsz, codes, codes2, ids, order, n, 0, 30, stream) != hipSuccess) return fail("sort");

    uint32_t V = 0;                                          // visible hierarchy nodes = pair records
    if (n > max_leaf && m > 0)
    {
        hipLaunchKernelGGL(k_karras, dim3(blocks(m, 256)), dim3(256), 0, stream, codes2, int(n), child, range, pint, pleaf);
        if (hipMemsetAsync(arrivals, 0, size_t(m) * 4, stream) != hipSuccess) return fail("memset");
        hipLaunchKernelGGL(k_refit, dim3(blocks(n, 256)), dim3(256), 0, stream, box, order, int(n), child, pint, pleaf,
                           nbox, arrivals);
        hipLaunchKernelGGL(k_visible, dim3(blocks(m, 256)), dim3(256), 0, stream, range, int(m), max_leaf, vis);
        size_t ssz = 0;
        if (rocprim::exclusive_scan(nullptr, ssz, vis, slot, 0u, m, rocprim::plus<uint32_t>(), stream) != hipSuccess) return fail("scan size");
        void* sstore = nullptr;
        if (!dalloc(&sstore, ssz)) return fail("alloc");
        tmp.push_back(sstore);
        if (rocprim::exclusive_scan(sstore, ssz, vis, slot, 0u, m, rocprim::plus<uint32_t>(), stream) != hipSuccess) return fail("scan");
        uint32_t last_slot = 0, last_vis = 0;
        if (hipMemcpyAsync(&last_slot, slot + (m - 1), 4, hipMemcpyDeviceToHost, stream) != hipSuccess) return fail("d2h");
        if (hipMemcpyAsync(&last_vis, vis + (m - 1), 4, hipMemcpyDeviceToHost, stream) != hipSuccess) return fail("d2h");
        if (hipStreamSynchronize(stream) != hipSuccess) return fail("sync");
        V = last_slot + last_vis;
    }
    const uint32_t num_nodes = 1u + 2u * V;
    if (!dalloc((void**)&out.nodes, size_t(num_nodes) * sizeof(node32))) return fail("alloc");
    if (!dalloc((void**)&out.pairs, size_t(std::max(V, 1u)) * 64)) return fail("alloc");
    if (!dalloc((void**)&out.prims, size_t(n) * (kind == VRH_PRIM_TRI64 ? 48u : 32u))) return fail("alloc");
    out.indices = order;                                     // sorted original indices = index array
    tmp.erase(std::find(tmp.begin(), tmp.end(), (void*)order));
    if (hipMemsetAsync(endf, 0, n, stream) != hipSuccess) return fail("memset");
    if (hipMemsetAsync(dmax, 0, 4, stream) != hipSuccess) return fail("memset");
    if (V > 0)
    {
        hipLaunchKernelGGL(k_emit, dim3(blocks(m, 256)), dim3(256), 0, stream, child, range, vis, slot, nbox, box, order,
                           int(m), out.nodes, out.pairs, endf, owner);
        hipLaunchKernelGGL(k_depth, dim3(blocks(m, 256)), dim3(256), 0, stream, vis, pint, int(m), dmax);
    }
    else
    {
        // a single leaf over all primitives: root = leaf (bounds computed on the host below)
        if (hipMemsetAsync(endf + (n - 1), 1, 1, stream) != hipSuccess) return fail("memset");
    }
    hipLaunchKernelGGL(k_prims, dim3(blocks(n, 256)), dim3(256), 0, stream, raw, order, endf, n, kind, out.prims);
    (void)hipEventRecord(e1, stream);
    uint32_t gs[16] = {};
    if (hipMemcpyAsync(gs, gstat, sizeof(gs), hipMemcpyDeviceToHost, stream) != hipSuccess) return fail("d2h");
    uint32_t depth = 0;
    if (hipMemcpyAsync(&depth, dmax, 4, hipMemcpyDeviceToHost, stream) != hipSuccess) return fail("d2h");
    if (hipStreamSynchronize(stream) != hipSuccess) return fail("sync");
    if (hipGetLastError() != hipSuccess) return fail("kernel");
    if (V == 0)
    {
        // root leaf: bounds of all primitives (host-side union of the device boxes)
        std::vector<aabb_t> hb(n);
        if (hipMemcpy(hb.data(), box, n * sizeof(aabb_t), hipMemcpyDeviceToHost) != hipSuccess) return fail("d2h");
        node32 root{};
        for (int a = 0; a < 3; ++a) { root.bmin[a] = INFINITY; root.bmax[a] = -INFINITY; }
        for (auto const& b : hb)
        {
            root.bmin[0] = std::min(root.bmin[0], b.lo.x); root.bmin[1] = std::min(root.bmin[1], b.lo.y);
            root.bmin[2] = std::min(root.bmin[2], b.lo.z); root.bmax[0] = std::max(root.bmax[0], b.hi.x);
            root.bmax[1] = std::max(root.bmax[1], b.hi.y); root.bmax[2] = std::max(root.bmax[2], b.hi.z);
        }
        root.first = 0;
        root.num_prims = n;
        if (hipMemcpy(out.nodes, &root, sizeof(root), hipMemcpyHostToDevice) != hipSuccess) return fail("h2d");
        depth = 0;
    }
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    out.build_ms = ms;
    out.num_nodes = num_nodes;
    out.num_pairs = V;
    out.root = V > 0 ? 0u : (0x80000000u | 0u);
    out.max_depth = depth;
    out.finite = gs[6] == 0;
    out.max_prim_id = gs[7];
    out.max_geom_id = gs[8];
    for (void* p : tmp) (void)hipFree(p);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return VRH_OK;
}

} // namespace vrh
