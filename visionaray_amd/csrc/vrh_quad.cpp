// visionaray_amd/csrc/vrh_quad.cpp -- 4-wide node records for any-hit rays, derived from the
// reference's binary BVH at upload.
//
// An any-hit ray's result (exit_traversal.h:49-56: the first accepted hit ends the ray) depends
// only on WHICH leaves it reaches, not on the order: before its first hit the running best_t is
// max(), so every box test (update_if.h:60-66) compares against constants.  A leaf is reached iff
// the box test passes for every node on its root path.  If a grandchild's box lies inside its
// parent's box (and every box has min <= max), the slab distances are monotone in the bounds --
// (b - o) * inv rounds monotonically for a fixed finite o and inv -- so the grandchild's tnear is
// >= and its tfar <= the parent's, and passing the grandchild's test implies passing the parent's.
// The parent's test can then be skipped: a record holding the (up to) four grandchildren of a
// node reaches exactly the leaves the binary traversal reaches, in half the dependent steps.
// build_quads checks containment and box validity for every skipped node; if any check fails the
// scene keeps the binary path for all rays.  Only rays with finite origin and inverse direction
// over finite bounds use the records (the slab distances are then never NaN).
//
// Record (32 floats, 128 B): xmin[4] ymin[4] zmin[4] xmax[4] ymax[4] zmax[4] link[4] pad[4];
// link = quad index of an inner grandchild, LEAF_BIT | first primitive (leaf order) of a leaf,
// QUAD_NONE for an unused entry.
#include "vrh_internal.h"

#include <algorithm>
#include <cstring>
#include <deque>
#include <unordered_map>

#ifndef VRH_QUAD_ORDER
#define VRH_QUAD_ORDER 0      // record order: 0 = breadth-first, 1 = depth-first (sibling groups)
#endif

namespace vrh {

namespace {

bool valid_box(const node32& n)
{
    for (int a = 0; a < 3; ++a)
        if (!(n.bmin[a] <= n.bmax[a])) return false;
    return true;
}

bool inside(const node32& g, const node32& p)
{
    for (int a = 0; a < 3; ++a)
        if (!(g.bmin[a] >= p.bmin[a] && g.bmax[a] <= p.bmax[a])) return false;
    return true;
}

} // namespace

bool build_quads(const node32* nodes, uint32_t num_nodes, std::vector<float>& out, uint32_t& root_link,
                 uint32_t& quad_depth)
{
    out.clear();
    quad_depth = 0;
    if (num_nodes < 3 || nodes[0].num_prims != 0) return false;     // single leaf: nothing to widen
    std::unordered_map<uint32_t, uint32_t> index;                    // binary inner node -> quad
    std::deque<std::pair<uint32_t, uint32_t>> queue;                 // (binary node, quad depth)
    index[0] = 0;
    queue.push_back({ 0u, 1u });
    out.resize(32, 0.0f);
    while (!queue.empty())
    {
#if VRH_QUAD_ORDER == 1
        // depth-first: a record's inner entries get consecutive indices (as in breadth-first), and
        // the first of them is expanded next, so a descent's records lie close together
        const uint32_t n = queue.back().first, depth = queue.back().second;
        queue.pop_back();
#else
        const uint32_t n = queue.front().first, depth = queue.front().second;
        queue.pop_front();
#endif
        quad_depth = std::max(quad_depth, depth);
        const uint32_t q = index[n];
        uint32_t entries[4];
        uint32_t links[4];
        uint32_t ne = 0;
        const uint32_t fc = nodes[n].first;
        if (uint64_t(fc) + 1 >= num_nodes) return false;
        for (uint32_t c = fc; c < fc + 2; ++c)
        {
            const node32& cn = nodes[c];
            if (!valid_box(cn)) return false;
            if (cn.num_prims != 0)
            {
                entries[ne] = c;
                links[ne++] = 0x80000000u | cn.first;
                continue;
            }
            if (uint64_t(cn.first) + 1 >= num_nodes) return false;
            for (uint32_t g = cn.first; g < cn.first + 2; ++g)
            {
                const node32& gn = nodes[g];
                if (!valid_box(gn) || !inside(gn, cn)) return false;
                entries[ne] = g;
                if (gn.num_prims != 0)
                    links[ne++] = 0x80000000u | gn.first;
                else
                {
                    auto it = index.find(g);
                    uint32_t gq;
                    if (it == index.end())
                    {
                        gq = uint32_t(out.size() / 32);
                        if (gq >= 0x7FFFFFFFu) return false;
                        index[g] = gq;
                        out.resize(out.size() + 32, 0.0f);
                        queue.push_back({ g, depth + 1 });
                    }
                    else
                        return false;                                // not a tree
                    links[ne++] = gq;
                }
            }
        }
#if VRH_QUAD_ORDER == 1
        // the entries were queued in order; depth-first expands the first one next
        std::reverse(queue.end() - std::count_if(links, links + ne, [](uint32_t l) { return !(l & 0x80000000u); }), queue.end());
#endif
        float* rec = &out[size_t(q) * 32];
        for (uint32_t e = 0; e < 4; ++e)
        {
            const bool used = e < ne;
            const node32& b = nodes[used ? entries[e] : entries[0]];
            for (int a = 0; a < 3; ++a)
            {
                rec[a * 4 + e] = b.bmin[a];
                rec[12 + a * 4 + e] = b.bmax[a];
            }
            const uint32_t l = used ? links[e] : QUAD_NONE;
            std::memcpy(&rec[24 + e], &l, 4);
        }
    }
    root_link = 0;
    return true;
}

} // namespace vrh
