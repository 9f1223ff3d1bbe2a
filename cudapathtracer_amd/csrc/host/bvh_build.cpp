// bvh_build.cpp -- the reference's BVH (BVH.h:133-474), re-authored with an index-based node
// pool.  The output node array must be byte-identical to BVH_array.root, so every
// floating-point expression keeps the reference's types and operation order:
//   * boxes merge with std::min/std::max semantics, (b < a ? b : a) / (a < b ? b : a), in the
//     reference's argument order (AABBUnion(ret, b1, b2) = min(b1, b2)), which fixes signed-zero
//     and NaN outcomes;
//   * each level bins centroids into a 3x3x3 grid over the union box, cell = clamp((int)(c/d))
//     with x86 truncation (NaN -> INT_MIN -> cell 0);
//   * QUIRK kept (BVH.h:190): a cell's box grows by nodes[i] -- the i-th triangle of the whole
//     scene -- not by nodes[list[i]], the triangle whose centroid chose the cell;
//   * 9 candidate planes scored count*SA(side)/SA(parent) in double, strict '<' (first wins);
//   * a candidate with an empty side falls back to halving the list in input order (:263-288);
//   * two items always pair into one node (:136-150); depth of such a pair node is 2;
//   * breadth-first flattening: child index = current index + queue length after the push
//     (:331-382); leaves are (triangle | 0x80000000).
#include <cfloat>
#include <cmath>
#include <cstring>
#include <deque>

#include "host_internal.h"

namespace pt {

namespace {

struct Box {
    float lo[3], hi[3];
};

inline float fmin_ref(float a, float b) { return (b < a) ? b : a; }   // std::min(a, b)
inline float fmax_ref(float a, float b) { return (a < b) ? b : a; }   // std::max(a, b)

inline Box empty_box()   // AABB::makeNegative (BVH.h:21-25)
{
    Box b;
    for (int k = 0; k < 3; ++k) { b.lo[k] = 10000.0f; b.hi[k] = -10000.0f; }
    return b;
}

inline void grow(Box& acc, const Box& b)   // AABBUnion(&acc, &acc, &b) (BVH.h:33-37)
{
    for (int k = 0; k < 3; ++k) {
        acc.lo[k] = fmin_ref(acc.lo[k], b.lo[k]);
        acc.hi[k] = fmax_ref(acc.hi[k], b.hi[k]);
    }
}

inline float area2(const Box& b)   // AABB::weight (BVH.h:27-31): 2*(dx*dy + dx*dz + dy*dz)
{
    float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return 2 * (dx * dy + dx * dz + dy * dz);
}

inline int cell_of(float c, float d)   // min(2, max(0, (int)(c / d))) with x86 (int)
{
    float q = c / d;
    int i = (q > -2147483649.0f && q < 2147483648.0f) ? static_cast<int>(q) : INT32_MIN;
    i = (0 < i) ? i : 0;
    return (i < 2) ? i : 2;
}

struct Node {
    Box box;
    int left = -1, right = -1;   // pool indices
    int tri = -1;                // >= 0 for leaves
    int descendants = 0;         // BVH_node::numChildNodes
    int depth = 0;
};

class Builder {
public:
    explicit Builder(std::vector<Node>& pool) : pool_(pool) {}

    int build(std::vector<int>& list, int level)
    {
        if (level > 100000) { overflow_ = true; return 0; }
        const int n = static_cast<int>(list.size());
        if (n == 2) {
            Box tb = empty_box();
            grow(tb, pool_[list[0]].box);
            grow(tb, pool_[list[1]].box);
            return make_inner(tb, list[0], list[1], 2, 2);
        }
        if (n == 1) return list[0];

        Box total = empty_box();
        for (int i = 0; i < n; ++i) grow(total, pool_[list[i]].box);
        const float total_area = area2(total);

        Box cells[3][3][3];
        int counts[3][3][3];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b)
                for (int c = 0; c < 3; ++c) { cells[a][b][c] = empty_box(); counts[a][b][c] = 0; }
        float unit[3];
        for (int k = 0; k < 3; ++k) unit[k] = (total.hi[k] - total.lo[k]) / static_cast<float>(3);

        std::vector<int> cell(3 * static_cast<size_t>(n));
        for (int i = 0; i < n; ++i) {
            const Box& b = pool_[list[i]].box;
            int ci[3];
            for (int k = 0; k < 3; ++k) {
                float ctr = (b.hi[k] + b.lo[k]) / static_cast<float>(2) - total.lo[k];
                ci[k] = cell_of(ctr, unit[k]);
                cell[3 * static_cast<size_t>(i) + k] = ci[k];
            }
            grow(cells[ci[0]][ci[1]][ci[2]], pool_[i].box);   // BVH.h:190 quirk: nodes[i]
            counts[ci[0]][ci[1]][ci[2]] += 1;
        }

        int best_axis = 0, best_plane = 0, best_l = 0, best_r = 0;
        double best = DBL_MAX;
        for (int axis = 0; axis < 3; ++axis) {
            for (int plane = 0; plane < 3; ++plane) {
                int lo_end[3] = {3, 3, 3}, hi_begin[3] = {0, 0, 0};
                lo_end[axis] = plane;
                hi_begin[axis] = plane;
                Box lb = empty_box(), rb = empty_box();
                int lc = 0, rc = 0;
                for (int a = 0; a < lo_end[0]; ++a)
                    for (int b = 0; b < lo_end[1]; ++b)
                        for (int c = 0; c < lo_end[2]; ++c)
                            if (counts[a][b][c] > 0) { lc += counts[a][b][c]; grow(lb, cells[a][b][c]); }
                for (int a = hi_begin[0]; a < 3; ++a)
                    for (int b = hi_begin[1]; b < 3; ++b)
                        for (int c = hi_begin[2]; c < 3; ++c)
                            if (counts[a][b][c] > 0) { rc += counts[a][b][c]; grow(rb, cells[a][b][c]); }
                const double pl = area2(lb) / total_area;
                const double pr = area2(rb) / total_area;
                const double score = lc * pl + rc * pr;
                if (score < best) { best = score; best_axis = axis; best_plane = plane; best_l = lc; best_r = rc; }
            }
        }

        std::vector<int> lhs, rhs;
        if (best_l == 0 || best_r == 0) {            // BVH.h:263-288: halve in input order
            const int lcount = best_r / 2;
            const int rcount = best_r - lcount;
            lhs.assign(list.begin(), list.begin() + lcount);
            rhs.assign(list.begin() + lcount, list.begin() + lcount + rcount);
        } else {
            lhs.reserve(best_l);
            rhs.reserve(best_r);
            for (int i = 0; i < n; ++i) {
                if (static_cast<float>(cell[3 * static_cast<size_t>(i) + best_axis]) < static_cast<float>(best_plane))
                    lhs.push_back(list[i]);
                else
                    rhs.push_back(list[i]);
            }
        }
        std::vector<int>().swap(cell);
        const int l = build(lhs, level + 1);
        const int r = build(rhs, level + 1);
        const int d = std::max(pool_[l].depth, pool_[r].depth) + 1;
        return make_inner(total, l, r, pool_[l].descendants + pool_[r].descendants + 2, d);
    }

    bool overflow() const { return overflow_; }

private:
    int make_inner(const Box& b, int l, int r, int desc, int depth)
    {
        Node nd;
        nd.box = b;
        nd.left = l;
        nd.right = r;
        nd.descendants = desc;
        nd.depth = depth;
        pool_.push_back(nd);
        return static_cast<int>(pool_.size()) - 1;
    }

    std::vector<Node>& pool_;
    bool overflow_ = false;
};

}  // namespace

int build_bvh(const std::vector<pt_vec3>& verts, const std::vector<pt_triangle>& tris, std::vector<pt_bvh_node>* out,
              int32_t* depth)
{
    const size_t nt = tris.size();
    if (nt < 2) return fail(PT_E_SCENE, "buildBVH needs at least 2 triangles (got %zu)", nt);   // decision d5
    if (nt > 0x7fffffffu) return fail(PT_E_SCENE, "too many triangles for 31-bit BVH indices");
    std::vector<Node> pool;
    pool.reserve(2 * nt);
    for (size_t i = 0; i < nt; ++i) {                                        // BVH.h:451-462
        const pt_triangle& t = tris[i];
        if (t.v0 < 0 || t.v1 < 0 || t.v2 < 0 || static_cast<size_t>(t.v0) >= verts.size() ||
            static_cast<size_t>(t.v1) >= verts.size() || static_cast<size_t>(t.v2) >= verts.size())
            return fail(PT_E_SCENE, "triangle %zu has a vertex index out of range", i);
        const float* a = &verts[t.v0].x;
        const float* b = &verts[t.v1].x;
        const float* c = &verts[t.v2].x;
        Node leaf;
        for (int k = 0; k < 3; ++k) {
            leaf.box.lo[k] = fmin_ref(fmin_ref(a[k], b[k]), c[k]);
            leaf.box.hi[k] = fmax_ref(fmax_ref(a[k], b[k]), c[k]);
        }
        leaf.tri = static_cast<int>(i);
        pool.push_back(leaf);
    }
    std::vector<int> all(nt);
    for (size_t i = 0; i < nt; ++i) all[i] = static_cast<int>(i);
    Builder bld(pool);
    const int root = bld.build(all, 0);
    if (bld.overflow()) return fail(PT_E_BVH_DEPTH, "BVH recursion too deep");

    const size_t count = static_cast<size_t>(pool[root].descendants) + 1 - nt;
    out->assign(count, pt_bvh_node());
    std::deque<int> queue;
    queue.push_back(root);
    uint32_t at = 0;
    while (!queue.empty()) {                                                // BVH.h:349-377
        const Node& nd = pool[queue.front()];
        queue.pop_front();
        pt_bvh_node& dst = (*out)[at];
        const int kids[2] = {nd.left, nd.right};
        uint32_t* slots[2] = {&dst.left, &dst.right};
        for (int s = 0; s < 2; ++s) {
            const Node& kid = pool[kids[s]];
            if (kid.tri < 0) {
                queue.push_back(kids[s]);
                *slots[s] = at + static_cast<uint32_t>(queue.size());
            } else {
                *slots[s] = static_cast<uint32_t>(kid.tri) | PT_BVH_LEAF_FLAG;
            }
        }
        memcpy(&dst.lo, nd.box.lo, sizeof(float) * 3);
        memcpy(&dst.hi, nd.box.hi, sizeof(float) * 3);
        ++at;
    }
    *depth = pool[root].depth;
    return PT_OK;
}

}  // namespace pt
