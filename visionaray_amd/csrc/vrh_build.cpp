// visionaray_amd/csrc/vrh_build.cpp -- host binned-SAH BVH builder (product side).
//
// Produces the identical tree to the reference builder build<index_bvh<P>>(prims, n)
// (detail/bvh/build.inl:165-178 -> binned_sah_builder, detail/bvh/sah.h:150-763): same node
// numbering (children allocated as an adjacent pair, right subtree built first, build.inl:45-72),
// same leaf index order (sah.h:657-672), same float arithmetic (compiled with -ffp-contract=off).
// Tree identity matters because closest-hit ties are resolved by traversal order.
//
// Structure differs from the reference: an explicit work stack instead of recursion, primitive
// references kept as flat arrays, object splits only (no config uses spatial splits), and large
// subtrees built on parallel threads and spliced back in the sequential numbering (build_fork).

#include "vrh_internal.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

namespace vrh {
namespace {

// math/detail/math.h:48-60 ternary min/max (NaN behaviour follows the comparison)
inline float tmin(float x, float y) { return x < y ? x : y; }
inline float tmax(float x, float y) { return x < y ? y : x; }

struct bounds3
{
    float lo[3], hi[3];

    void reset() { for (int a = 0; a < 3; ++a) { lo[a] = FLT_MAX; hi[a] = -FLT_MAX; } }
    void grow(const float p[3]) { for (int a = 0; a < 3; ++a) { lo[a] = tmin(lo[a], p[a]); hi[a] = tmax(hi[a], p[a]); } }
    void grow(const bounds3& b) { for (int a = 0; a < 3; ++a) { lo[a] = tmin(lo[a], b.lo[a]); hi[a] = tmax(hi[a], b.hi[a]); } }
    void centre(float c[3]) const { for (int a = 0; a < 3; ++a) c[a] = (hi[a] + lo[a]) * 0.5f; }
    // aabb.inl safe_half_surface_area: extents clamped at 0, (x*y + y*z) + z*x
    float half_area() const
    {
        float s[3];
        for (int a = 0; a < 3; ++a) s[a] = tmax(0.0f, hi[a] - lo[a]);
        return s[0] * s[1] + s[1] * s[2] + s[2] * s[0];
    }
};

struct ref_t { bounds3 box; int prim; };

struct range_t   // a subtree under construction: its node slot + the refs [first, end-of-list)
{
    uint32_t node;
    int      first;
    unsigned depth;
    bounds3  box;    // primitive bounds (stored in the node)
    bounds3  cbox;   // centroid bounds (used to pick the axis and bins)
};

constexpr int kBins = 16;
constexpr int kMaxLeaf = 4;

struct bin_t { bounds3 box, cbox; int n; };

inline void make_node(node32& n, const bounds3& b, uint32_t first, uint32_t count)
{
    for (int a = 0; a < 3; ++a) { n.bmin[a] = b.lo[a]; n.bmax[a] = b.hi[a]; }
    n.first = first;
    n.num_prims = count;
}

// Object split of refs[r.first, nrefs) -- sah.h:678-762 without spatial splits.
// Returns false when the range should become a leaf.
bool try_split(std::vector<ref_t>& refs, size_t nrefs, const range_t& r, range_t& left, range_t& right)
{
    const int count = static_cast<int>(nrefs - static_cast<size_t>(r.first));
    if (count <= kMaxLeaf) return false;

    float ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = r.cbox.hi[a] - r.cbox.lo[a];
    int axis = ext[1] < ext[0] ? 0 : 1;                       // vector.inl max_index
    axis = ext[2] < ext[axis] ? axis : 2;
    if (ext[axis] <= 0.0f) return false;

    const float k0 = r.cbox.lo[axis];
    const float k1 = static_cast<float>(kBins) / (r.cbox.hi[axis] - k0);
    auto bin_of = [&](const bounds3& b) {                    // projection::project_unsafe
        float c = (b.hi[axis] + b.lo[axis]) * 0.5f;
        return static_cast<int>(k1 * (c - k0));
    };

    bin_t bins[kBins];
    for (auto& b : bins) { b.box.reset(); b.cbox.reset(); b.n = 0; }
    for (size_t i = static_cast<size_t>(r.first); i < nrefs; ++i)
    {
        const bounds3& b = refs[i].box;
        int k = std::min(std::max(bin_of(b), 0), kBins - 1);
        float c[3];
        b.centre(c);
        bins[k].box.grow(b);
        bins[k].cbox.grow(c);
        bins[k].n++;
    }

    // prefix from the left, suffix from the right; first minimum of the right-to-left sweep wins
    bin_t pre[kBins], suf[kBins];
    pre[0] = bins[0];
    for (int i = 1; i < kBins; ++i) { pre[i] = pre[i - 1]; pre[i].box.grow(bins[i].box); pre[i].cbox.grow(bins[i].cbox); pre[i].n += bins[i].n; }
    suf[kBins - 1] = bins[kBins - 1];
    const float parent = r.box.half_area();
    float best = FLT_MAX;
    int split = -1;
    for (int i = kBins - 1; i > 0; --i)
    {
        suf[i - 1] = suf[i]; suf[i - 1].box.grow(bins[i - 1].box); suf[i - 1].cbox.grow(bins[i - 1].cbox); suf[i - 1].n += bins[i - 1].n;
        const bin_t& L = pre[i - 1];
        const bin_t& R = suf[i];
        float cost = 1.0f + (L.box.half_area() / parent) * (3.0f * static_cast<float>(L.n))
                          + (R.box.half_area() / parent) * (3.0f * static_cast<float>(R.n));
        if (cost < best) { best = cost; split = i; }
    }
    if (split <= 0) return false;
    if (best > 3.0f * static_cast<float>(count)) return false;   // leaf is cheaper

    // libstdc++ std::partition on random-access iterators (bidirectional algorithm)
    auto mid = std::partition(refs.begin() + r.first, refs.begin() + static_cast<long>(nrefs),
                              [&](const ref_t& x) { return bin_of(x.box) < split; });

    left.first = r.first;
    left.box = pre[split - 1].box; left.cbox = pre[split - 1].cbox;
    right.first = static_cast<int>(mid - refs.begin());
    right.box = suf[split].box; right.cbox = suf[split].cbox;
    return true;
}

// A subtree built on its own: nodes numbered as the sequential loop numbers them relative to the
// subtree's root (local 0; its children pairs from 1, right subtree first), leaf primitive indices in
// the order the sequential loop appends them, leaf `first` relative to the subtree's first index.
struct subtree
{
    std::vector<node32> nodes;
    std::vector<uint32_t> idx;
    unsigned max_depth = 0;
};

// the sequential loop (build.inl:28-81 with an explicit stack) over refs[r.first, end)
void build_local(std::vector<ref_t>& refs, range_t r, size_t end, subtree& out)
{
    size_t nrefs = end;      // refs beyond nrefs have been consumed by finished leaves
    r.node = 0;
    out.nodes.assign(1, node32{});
    out.idx.clear();
    out.max_depth = 0;
    std::vector<range_t> work{ r };
    while (!work.empty())
    {
        range_t w = work.back();
        work.pop_back();
        out.max_depth = std::max(out.max_depth, w.depth);
        range_t left, right;
        if (try_split(refs, nrefs, w, left, right))
        {
            const uint32_t c0 = static_cast<uint32_t>(out.nodes.size());
            out.nodes.resize(c0 + 2u);
            make_node(out.nodes[w.node], w.box, c0, 0);
            left.node = c0; right.node = c0 + 1;
            left.depth = right.depth = w.depth + 1;
            work.push_back(left);    // popped after the whole right subtree
            work.push_back(right);
        }
        else
        {
            const uint32_t cnt = static_cast<uint32_t>(nrefs - static_cast<size_t>(w.first));
            make_node(out.nodes[w.node], w.box, static_cast<uint32_t>(out.idx.size()), cnt);
            for (size_t i = static_cast<size_t>(w.first); i < nrefs; ++i) out.idx.push_back(static_cast<uint32_t>(refs[i].prim));
            nrefs = static_cast<size_t>(w.first);
        }
    }
}

// Parallel build, same tree.  A range of at least kForkMin refs is split here (the same try_split
// on the same refs: subtrees own disjoint ref ranges, [first, mid) and [mid, end), so the in-place
// partitions do not interact); its right subtree is built on another thread while this one builds
// the left.  Smaller ranges run the sequential loop into their own arrays.  assemble() then replays
// the sequential order -- pair allocated, right subtree, then left -- and copies every node once.
constexpr size_t kForkMin = size_t(1) << 15;

struct fork_node
{
    bool split = false;
    bounds3 box;
    std::unique_ptr<fork_node> left, right;
    subtree sub;                 // !split: the subtree built by build_local
};

struct fork_pool
{
    std::atomic<int> spare;      // threads that may still be started
};

void build_fork(std::vector<ref_t>& refs, const range_t& r, size_t end, fork_node& out, fork_pool& pool)
{
    range_t left, right;
    if (end - static_cast<size_t>(r.first) >= kForkMin && try_split(refs, end, r, left, right))
    {
        out.split = true;
        out.box = r.box;
        out.sub.max_depth = r.depth;
        out.left.reset(new fork_node);
        out.right.reset(new fork_node);
        left.depth = right.depth = r.depth + 1;
        std::thread t;
        if (pool.spare.fetch_sub(1) > 0)
            t = std::thread([&] { build_fork(refs, right, end, *out.right, pool); });
        else
        {
            pool.spare.fetch_add(1);
            build_fork(refs, right, end, *out.right, pool);
        }
        build_fork(refs, left, static_cast<size_t>(right.first), *out.left, pool);
        if (t.joinable())
        {
            t.join();
            pool.spare.fetch_add(1);
        }
        return;
    }
    build_local(refs, r, end, out.sub);
}

struct assembly
{
    node32* nodes;
    uint32_t* indices;
    uint32_t num_nodes, num_idx;
    unsigned max_depth;
};

void assemble(const fork_node& f, uint32_t slot, assembly& a)
{
    if (f.split)
    {
        const uint32_t c0 = a.num_nodes;
        a.num_nodes += 2;
        make_node(a.nodes[slot], f.box, c0, 0);
        a.max_depth = std::max(a.max_depth, f.sub.max_depth);
        assemble(*f.right, c0 + 1, a);
        assemble(*f.left, c0, a);
        return;
    }
    // local node c >= 1 -> a.num_nodes + c - 1; leaf first -> a.num_idx + first
    const uint32_t node_shift = a.num_nodes - 1u, idx_shift = a.num_idx;
    for (size_t i = 0; i < f.sub.nodes.size(); ++i)
    {
        node32 n = f.sub.nodes[i];
        n.first += n.num_prims ? idx_shift : node_shift;
        a.nodes[i == 0 ? slot : node_shift + static_cast<uint32_t>(i)] = n;
    }
    a.num_nodes += static_cast<uint32_t>(f.sub.nodes.size()) - 1u;
    std::memcpy(a.indices + a.num_idx, f.sub.idx.data(), f.sub.idx.size() * sizeof(uint32_t));
    a.num_idx += static_cast<uint32_t>(f.sub.idx.size());
    a.max_depth = std::max(a.max_depth, f.sub.max_depth);
}

template <typename GetBox>
int build_impl(size_t n, GetBox get_box, node32* nodes_out, uint32_t* num_nodes_out, uint32_t* indices_out,
               uint32_t* max_depth_out)
{
    std::vector<ref_t> refs(n);
    range_t root;
    root.node = 0; root.first = 0; root.depth = 0;
    root.box.reset(); root.cbox.reset();
    for (size_t i = 0; i < n; ++i)
    {
        refs[i].box = get_box(i);
        refs[i].prim = static_cast<int>(i);
        float c[3];
        refs[i].box.centre(c);
        root.box.grow(refs[i].box);
        root.cbox.grow(c);
    }
    fork_pool pool;
    const unsigned hw = std::thread::hardware_concurrency();
    pool.spare = static_cast<int>(std::min(16u, hw ? hw : 1u)) - 1;   // the box's CPU share is 16 threads
    fork_node top;
    build_fork(refs, root, n, top, pool);
    assembly a{ nodes_out, indices_out, 1u, 0u, 0u };
    assemble(top, 0, a);
    *num_nodes_out = a.num_nodes;
    if (max_depth_out) *max_depth_out = a.max_depth;
    return VRH_OK;
}

} // namespace

int build_bvh(const void* prims, uint32_t n, uint32_t kind, node32* nodes_out, uint32_t* num_nodes_out,
              uint32_t* indices_out, uint32_t* max_depth_out)
{
    if (kind == VRH_PRIM_TRI64)
    {
        auto tris = static_cast<const tri64*>(prims);
        return build_impl(n, [&](size_t i) {
            const tri64& t = tris[i];
            bounds3 b; b.reset();
            float p[3];
            b.grow(t.v1);
            for (int a = 0; a < 3; ++a) p[a] = t.v1[a] + t.e1[a];
            b.grow(p);
            for (int a = 0; a < 3; ++a) p[a] = t.v1[a] + t.e2[a];
            b.grow(p);
            return b;
        }, nodes_out, num_nodes_out, indices_out, max_depth_out);
    }
    auto sph = static_cast<const sphere48*>(prims);
    return build_impl(n, [&](size_t i) {
        const sphere48& s = sph[i];
        bounds3 b; b.reset();
        float p[3];
        for (int a = 0; a < 3; ++a) p[a] = s.center[a] - s.radius;
        b.grow(p);
        for (int a = 0; a < 3; ++a) p[a] = s.center[a] + s.radius;
        b.grow(p);
        return b;
    }, nodes_out, num_nodes_out, indices_out, max_depth_out);
}

} // namespace vrh
