// rt_bvh.h -- host-side BVH build over the Triangle colliders of a scene (TriangleMesh,
// the reference's own TODO, `sightpy/geometry/triangle_mesh.py:7-9`).
//
// Used by srt_upload_scene (rt_kernels.hip) and by the CPU check harness (rt_hostcheck.cpp), so the
// traversal in rt_device.h (bvh_nearest / bvh_shadow) is tested on both sides.  The BVH is only an
// accelerator: nearest_hit merges its triangles with the reference's order-independent rule
// (smallest distance, then lowest collider index, ties recorded), so results equal the linear loop
// over `scene.collider_list` (ray.py:124-132).
//
// Build: a binary BVH by binned SAH (16 bins on the longest centroid axis), leaves of at most 2
// triangles, depth capped at BVH_MAX_DEPTH; then collapsed into 4-wide nodes (rt_device.h BvhNode):
// a node's slots are its grandchildren (a leaf child stands for itself), so every 4-wide level spans
// two binary levels and the traversal stack stays within BVH_STACK.  Leaves keep < 64 triangles and
// their slots < 2^25 (the traversal's child codes); a mesh beyond that (a depth-capped leaf of 64 or
// more triangles) stays in the linear collider loop.  Boxes are the
// triangles' vertex boxes inflated by 1e-9 * (1 + max |coordinate|) -- the reference intersects the
// plane through the centroid and tests edge half-spaces with >= 0, so a hit point may sit a few ulps
// outside the vertex box -- then rounded outward to float.
#pragma once

#include <algorithm>
#include <cmath>
#include <vector>

#include "rt_device.h"

namespace rt {

constexpr int BVH_MIN_TRIANGLES = 8;  // fewer triangles stay in the linear collider loop
#ifndef RT_BVH_LEAF
#define RT_BVH_LEAF 2
#endif
constexpr int BVH_LEAF = RT_BVH_LEAF;  // triangles per leaf before the split stops (2: profiles/r05_bvh_f32_box_ab.txt; -DRT_BVH_LEAF for experiments)
constexpr int BVH_MAX_DEPTH = 20;  // binary levels (so at most 10 4-wide levels: 31 stack entries <= BVH_STACK)
static_assert(3 * ((BVH_MAX_DEPTH + 1) / 2) + 1 <= BVH_STACK, "traversal stack holds the deepest path");
constexpr int BVH_LEAF_MAX = 63;            // triangles per leaf (6-bit count in the child code)
constexpr int32_t BVH_SLOTS_MAX = 1 << 25;  // leaf slots (first << 6 fits the child code)

struct BvhBuild {
    std::vector<BvhNode> nodes;
    std::vector<int32_t> tri;  // collider index per leaf slot
    std::vector<int32_t> lin;  // colliders outside the BVH, ascending
    float bound = 0.0f;        // max |coordinate| over the nodes' (non-empty) boxes: rt_device.h box_ray
};

namespace bvh_detail {
struct BinNode {  // binary build node: count > 0 leaf of tri[first, first + count), else children first, first + 1
    double lo[3], hi[3];
    int32_t first, count;
};
struct Item {
    double lo[3], hi[3], c[3];
    int32_t col;
};
inline void grow(double* lo, double* hi, const double* plo, const double* phi) {
    for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(lo[k], plo[k]);
        hi[k] = std::max(hi[k], phi[k]);
    }
}
inline double area(const double* lo, const double* hi) {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0.0)) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
}
}  // namespace bvh_detail

inline void bvh_build(const srt_collider* col, int n, BvhBuild& out) {
    using namespace bvh_detail;
    out.nodes.clear();
    out.tri.clear();
    out.lin.clear();
    out.bound = 0.0f;
    std::vector<Item> items;
    for (int i = 0; i < n; ++i)
        if (col[i].type == SRT_TRIANGLE) {
            Item it;
            const double* p = col[i].p;  // p1 = p[6..8], p2 = p[9..11], p3 = p[12..14]
            double m = 0.0;
            for (int k = 0; k < 3; ++k) {
                it.lo[k] = std::min(std::min(p[6 + k], p[9 + k]), p[12 + k]);
                it.hi[k] = std::max(std::max(p[6 + k], p[9 + k]), p[12 + k]);
                m = std::max(m, std::max(std::fabs(it.lo[k]), std::fabs(it.hi[k])));
            }
            const double eps = 1e-9 * (1.0 + m);
            for (int k = 0; k < 3; ++k) {
                it.lo[k] -= eps;
                it.hi[k] += eps;
                it.c[k] = 0.5 * (it.lo[k] + it.hi[k]);
            }
            it.col = i;
            items.push_back(it);
        }
    if ((int)items.size() < BVH_MIN_TRIANGLES) {
        for (int i = 0; i < n; ++i) out.lin.push_back(i);
        return;
    }
    for (int i = 0; i < n; ++i)
        if (col[i].type != SRT_TRIANGLE) out.lin.push_back(i);

    struct Task {
        int node, begin, end, depth;
    };
    std::vector<BinNode> bin;
    bin.push_back(BinNode{});
    std::vector<Task> tasks{{0, 0, (int)items.size(), 0}};
    while (!tasks.empty()) {
        const Task t = tasks.back();
        tasks.pop_back();
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = t.begin; i < t.end; ++i) {
            grow(lo, hi, items[i].lo, items[i].hi);
            grow(clo, chi, items[i].c, items[i].c);
        }
        BinNode& nd = bin[t.node];
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = lo[k];
            nd.hi[k] = hi[k];
        }
        const int cnt = t.end - t.begin;
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
        const double ext = chi[axis] - clo[axis];
        int mid = -1;
        if (cnt > BVH_LEAF && t.depth < BVH_MAX_DEPTH && ext > 0.0) {
            // binned SAH on the longest centroid axis
            constexpr int NB = 16;
            double blo[NB][3], bhi[NB][3];
            int bc[NB] = {};
            for (int b = 0; b < NB; ++b)
                for (int k = 0; k < 3; ++k) {
                    blo[b][k] = INFINITY;
                    bhi[b][k] = -INFINITY;
                }
            auto bin_of = [&](const Item& it) {
                int b = (int)((it.c[axis] - clo[axis]) / ext * NB);
                return std::min(NB - 1, std::max(0, b));
            };
            for (int i = t.begin; i < t.end; ++i) {
                const int b = bin_of(items[i]);
                bc[b]++;
                grow(blo[b], bhi[b], items[i].lo, items[i].hi);
            }
            double best = INFINITY;
            int best_split = -1;
            for (int s = 1; s < NB; ++s) {
                double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
                double rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
                int nl = 0, nr = 0;
                for (int b = 0; b < s; ++b) {
                    nl += bc[b];
                    if (bc[b]) grow(llo, lhi, blo[b], bhi[b]);
                }
                for (int b = s; b < NB; ++b) {
                    nr += bc[b];
                    if (bc[b]) grow(rlo, rhi, blo[b], bhi[b]);
                }
                if (!nl || !nr) continue;
                const double cost = nl * area(llo, lhi) + nr * area(rlo, rhi);
                if (cost < best) {
                    best = cost;
                    best_split = s;
                }
            }
            if (best_split > 0) {
                auto it = std::partition(items.begin() + t.begin, items.begin() + t.end,
                                         [&](const Item& x) { return bin_of(x) < best_split; });
                mid = (int)(it - items.begin());
            } else {
                // every centroid in one bin: median split
                mid = t.begin + cnt / 2;
                std::nth_element(items.begin() + t.begin, items.begin() + mid, items.begin() + t.end,
                                 [&](const Item& a, const Item& b) { return a.c[axis] < b.c[axis]; });
            }
            if (mid <= t.begin || mid >= t.end) mid = -1;
        }
        if (mid < 0) {
            // leaf (also when too deep: larger leaves keep the traversal stack bounded)
            nd.first = (int32_t)out.tri.size();
            nd.count = cnt;
            for (int i = t.begin; i < t.end; ++i) out.tri.push_back(items[i].col);
            continue;
        }
        const int left = (int)bin.size();
        nd.first = left;
        nd.count = 0;
        bin.push_back(BinNode{});
        bin.push_back(BinNode{});
        tasks.push_back({left, t.begin, mid, t.depth + 1});
        tasks.push_back({left + 1, mid, t.end, t.depth + 1});
    }
    // collapse into 4-wide nodes (node 0 = the root's children)
    auto fdown = [](double x) {
        float f = (float)x;
        if ((double)f > x) f = std::nextafter(f, -INFINITY);
        return f;
    };
    auto fup = [](double x) {
        float f = (float)x;
        if ((double)f < x) f = std::nextafter(f, INFINITY);
        return f;
    };
    if (bin[0].count > 0) {  // a single leaf (not reached: BVH_MIN_TRIANGLES > BVH_LEAF)
        bin.push_back(bin[0]);
        bin[0].first = (int32_t)bin.size() - 1;
        bin[0].count = 0;
        bin.push_back(BinNode{});  // an empty box: never hit
        for (int k = 0; k < 3; ++k) {
            bin.back().lo[k] = INFINITY;
            bin.back().hi[k] = -INFINITY;
        }
        bin.back().count = 0;
        bin.back().first = -1;
    }
    std::vector<std::pair<int, int>> work{{0, 0}};  // (binary inner node, 4-wide node)
    out.nodes.push_back(BvhNode{});
    while (!work.empty()) {
        const auto [bn, wn] = work.back();
        work.pop_back();
        std::vector<int> slots;
        for (int h = 0; h < 2; ++h) {
            const BinNode& c = bin[bin[bn].first + h];
            if (c.count > 0 || c.first < 0) {
                slots.push_back(bin[bn].first + h);
            } else {
                slots.push_back(c.first);
                slots.push_back(c.first + 1);
            }
        }
        BvhNode nd4{};
        for (int k = 0; k < 4; ++k) {
            if (k >= (int)slots.size() || bin[slots[k]].first < 0) {
                nd4.child[k] = BVH_EMPTY;
                nd4.count[k] = 0;
                for (int a = 0; a < 3; ++a) {
                    nd4.lo[a][k] = INFINITY;
                    nd4.hi[a][k] = -INFINITY;
                }
                continue;
            }
            const BinNode& c = bin[slots[k]];
            for (int a = 0; a < 3; ++a) {
                nd4.lo[a][k] = fdown(c.lo[a]);
                nd4.hi[a][k] = fup(c.hi[a]);
            }
            if (c.count > 0) {
                nd4.child[k] = -(c.first + 1);
                nd4.count[k] = c.count;
            } else {
                nd4.child[k] = (int32_t)out.nodes.size();
                nd4.count[k] = 0;
                work.push_back({slots[k], (int)out.nodes.size()});
                out.nodes.push_back(BvhNode{});
            }
        }
        out.nodes[wn] = nd4;
    }
    for (const BinNode& b : bin)
        if (b.count > BVH_LEAF_MAX || (b.count > 0 && b.first + b.count > BVH_SLOTS_MAX)) {
            out.nodes.clear();
            out.tri.clear();
            out.lin.clear();
            for (int i = 0; i < n; ++i) out.lin.push_back(i);
            return;
        }
    for (const BvhNode& nd : out.nodes)
        for (int k = 0; k < 4; ++k)
            if (nd.child[k] != BVH_EMPTY)
                for (int a = 0; a < 3; ++a)
                    out.bound = std::max(out.bound, std::max(std::fabs(nd.lo[a][k]), std::fabs(nd.hi[a][k])));
}

}  // namespace rt
