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
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <deque>
#include <thread>

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

// Parallel build.  The top levels are split serially into ~4 subtrees per host thread; the
// subtrees are built concurrently (std::thread, jobs taken from an atomic counter); the top
// is then joined bottom-up.  Safe because a call only reads leaf boxes (pool_[0..nt), including
// the BVH.h:190 `nodes[i]` quirk: i < n <= nt) and its own range of the index array, and inner
// nodes take pool slots from an atomic counter; the array the reference emits depends only on
// the tree's shape (BFS flattening below), not on slot order.  No allocation per call: the list
// of a call is idx_[b, e), partitioned stably in place through tmp_ (the reference's lhs/rhs
// vectors keep input order), cells live in cell_.
class Builder {
public:
    Builder(std::vector<Node>& pool, int first_free, size_t nt)
        : pool_(pool), idx_(nt), tmp_(nt), cell_(3 * nt), next_(first_free)
    {
        for (size_t i = 0; i < nt; ++i) idx_[i] = static_cast<int>(i);
    }

    int build(size_t b, size_t e, int level)
    {
        if (level > 100000) { overflow_ = true; return 0; }
        if (e - b <= 2) return small(b, e);
        Box total;
        size_t nl, nr;
        split(b, e, &total, &nl, &nr);
        const int lft = build(b, b + nl, level + 1);
        const int rgt = build(b + nl, b + nl + nr, level + 1);
        return join(total, lft, rgt);
    }

    // the whole tree on `threads` host threads; returns the root's pool index
    int build_parallel(size_t nt, unsigned threads)
    {
        const size_t cutoff = std::max<size_t>(4096, nt / (4 * std::max(1u, threads)));
        const auto c0 = std::chrono::steady_clock::now();
        const int top = plan(0, nt, 0, cutoff);
        const auto c1 = std::chrono::steady_clock::now();
        std::atomic<size_t> next_job{0};
        auto worker = [&]() {
            for (size_t j; (j = next_job.fetch_add(1)) < jobs_.size();) {
                Skel& k = skel_[jobs_[j]];
                k.result = build(k.b, k.e, k.level);
            }
        };
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < threads && t < jobs_.size(); ++t) pool.emplace_back(worker);
        worker();
        for (std::thread& t : pool) t.join();
        const auto c2 = std::chrono::steady_clock::now();
        if (getenv("PT_TIMING"))
            fprintf(stderr, "build_bvh: %u threads, %zu jobs: plan %.1f ms, jobs %.1f ms\n", threads, jobs_.size(),
                    std::chrono::duration<double, std::milli>(c1 - c0).count(),
                    std::chrono::duration<double, std::milli>(c2 - c1).count());
        return finish(top);
    }

    bool overflow() const { return overflow_.load(); }

private:
    struct Skel {
        size_t b = 0, e = 0;
        int level = 0;
        int left = -1, right = -1;   // skeleton children; -1 = a job (built by build())
        Box total;
        int result = -1;
    };

    int plan(size_t b, size_t e, int level, size_t cutoff)
    {
        const int me = static_cast<int>(skel_.size());
        skel_.emplace_back();
        skel_[me].b = b; skel_[me].e = e; skel_[me].level = level;
        if (e - b <= cutoff || e - b <= 2 || level > 100000) { jobs_.push_back(me); return me; }
        Box total;
        size_t nl, nr;
        split(b, e, &total, &nl, &nr);
        const int l = plan(b, b + nl, level + 1, cutoff);
        const int r = plan(b + nl, b + nl + nr, level + 1, cutoff);
        skel_[me].left = l; skel_[me].right = r; skel_[me].total = total;
        return me;
    }

    int finish(int k)
    {
        if (skel_[k].left < 0) return skel_[k].result;
        const int l = finish(skel_[k].left);
        const int r = finish(skel_[k].right);
        return join(skel_[k].total, l, r);
    }

    int small(size_t b, size_t e)
    {
        const int* list = idx_.data() + b;
        if (e - b == 1) return list[0];
        Box tb = empty_box();
        grow(tb, pool_[list[0]].box);
        grow(tb, pool_[list[1]].box);
        return make_inner(tb, list[0], list[1], 2, 2);
    }

    int join(const Box& total, int lft, int rgt)
    {
        const int d = std::max(pool_[lft].depth, pool_[rgt].depth) + 1;
        return make_inner(total, lft, rgt, pool_[lft].descendants + pool_[rgt].descendants + 2, d);
    }

    // BVH.h:133-328 for one node with > 2 primitives: 3x3x3 centroid grid, 9 candidate planes
    // scored countL*SA(L)/SA + countR*SA(R)/SA (strict < keeps the first), then the partition.
    void split(size_t b, size_t e, Box* total_out, size_t* nl_out, size_t* nr_out)
    {
        const size_t n = e - b;
        const int* list = idx_.data() + b;
        Box total = empty_box();
        for (size_t i = 0; i < n; ++i) grow(total, pool_[list[i]].box);
        const float total_area = area2(total);

        Box cells[3][3][3];
        int counts[3][3][3];
        for (int a = 0; a < 3; ++a)
            for (int bb = 0; bb < 3; ++bb)
                for (int c = 0; c < 3; ++c) { cells[a][bb][c] = empty_box(); counts[a][bb][c] = 0; }
        float unit[3];
        for (int k = 0; k < 3; ++k) unit[k] = (total.hi[k] - total.lo[k]) / static_cast<float>(3);

        uint8_t* cell = cell_.data() + 3 * b;
        for (size_t i = 0; i < n; ++i) {
            const Box& bx = pool_[list[i]].box;
            int ci[3];
            for (int k = 0; k < 3; ++k) {
                float ctr = (bx.hi[k] + bx.lo[k]) / static_cast<float>(2) - total.lo[k];
                ci[k] = cell_of(ctr, unit[k]);
                cell[3 * i + k] = static_cast<uint8_t>(ci[k]);
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
                    for (int bb = 0; bb < lo_end[1]; ++bb)
                        for (int c = 0; c < lo_end[2]; ++c)
                            if (counts[a][bb][c] > 0) { lc += counts[a][bb][c]; grow(lb, cells[a][bb][c]); }
                for (int a = hi_begin[0]; a < 3; ++a)
                    for (int bb = hi_begin[1]; bb < 3; ++bb)
                        for (int c = hi_begin[2]; c < 3; ++c)
                            if (counts[a][bb][c] > 0) { rc += counts[a][bb][c]; grow(rb, cells[a][bb][c]); }
                const double pl = area2(lb) / total_area;
                const double pr = area2(rb) / total_area;
                const double score = lc * pl + rc * pr;
                if (score < best) { best = score; best_axis = axis; best_plane = plane; best_l = lc; best_r = rc; }
            }
        }

        size_t nl, nr;
        if (best_l == 0 || best_r == 0) {            // BVH.h:263-288: halve in input order
            nl = static_cast<size_t>(best_r / 2);
            nr = static_cast<size_t>(best_r) - nl;   // lhs = list[0, nl), rhs = list[nl, nl + nr)
        } else {
            nl = static_cast<size_t>(best_l);
            nr = static_cast<size_t>(best_r);
            int* t = tmp_.data() + b;
            size_t l = 0, r = nl;
            for (size_t i = 0; i < n; ++i) {
                if (static_cast<float>(cell[3 * i + best_axis]) < static_cast<float>(best_plane)) t[l++] = list[i];
                else t[r++] = list[i];
            }
            memcpy(idx_.data() + b, t, n * sizeof(int));
        }
        *total_out = total;
        *nl_out = nl;
        *nr_out = nr;
    }

    int make_inner(const Box& bx, int l, int r, int desc, int depth)
    {
        Node nd;
        nd.box = bx;
        nd.left = l;
        nd.right = r;
        nd.descendants = desc;
        nd.depth = depth;
        const int at = next_.fetch_add(1);
        pool_[at] = nd;
        return at;
    }

    std::vector<Node>& pool_;
    std::vector<int> idx_, tmp_;
    std::vector<uint8_t> cell_;
    std::vector<Skel> skel_;
    std::vector<int> jobs_;
    std::atomic<int> next_;
    std::atomic<bool> overflow_{false};
};

}  // namespace

int build_bvh(const std::vector<pt_vec3>& verts, const std::vector<pt_triangle>& tris, std::vector<pt_bvh_node>* out,
              int32_t* depth)
{
    const size_t nt = tris.size();
    if (nt < 2) return fail(PT_E_SCENE, "buildBVH needs at least 2 triangles (got %zu)", nt);   // decision d5
    if (nt > 0x7fffffffu) return fail(PT_E_SCENE, "too many triangles for 31-bit BVH indices");
    std::vector<Node> pool(2 * nt);                                          // nt leaves + nt-1 inner
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
        pool[i] = leaf;
    }
    Builder bld(pool, static_cast<int>(nt), nt);
    const int root = bld.build_parallel(nt, host_threads());
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
