// accel_build.cpp -- the render path's private acceleration structure: a binned-SAH binary BVH
// over the scene's triangles, built at pt_create (outside the timed region, as the reference
// builds its BVH before its render loop, kernel.cu:601-704).
//
// It is ONLY a culling structure.  Which triangles the reference considers, and the tie-break
// order among equal distances, stay those of the reference's own BVH (BVH.h): every leaf record
// carries the triangle's rank in the reference's left-first DFS leaf order and the index of its
// reference parent node, and the kernel accepts a winner only after the reference slab test
// (BVH.h:51-83) passes on that parent (DESIGN.md "Traversal": with correctly rounded slab values
// and nested boxes, the parent test implies every ancestor test).  Boxes are inflated by a
// margin far above the slab arithmetic's rounding so the culling stays conservative.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "host_internal.h"

namespace pt {

namespace {

struct TriBox {
    float lo[3], hi[3];
    float c[3];
};

inline float surface(const float* lo, const float* hi)
{
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0.0f) || !(dy >= 0.0f) || !(dz >= 0.0f)) return 0.0f;
    return dx * dy + dy * dz + dz * dx;
}

struct Builder {
    const std::vector<TriBox>& tb;
    std::vector<uint32_t>& items;
    AccelBvh& out;
    float margin;
    int max_depth = 0;
    // Leaves of up to 2 triangles where the SAH favours them (measured on C3: 7% fewer BVH4 node
    // visits for 16% more triangle tests, +3% Msamples/s; 3 or 4 gain nothing more)
    size_t leaf_max = kAccelLeafMax;   // largest leaf (triangles; PT_LEAF_MAX)
    float node_cost = 1.0f;            // SAH cost of a binary node visit, in triangle tests (PT_LEAF_NODE_COST)

    Builder(const std::vector<TriBox>& t, std::vector<uint32_t>& it, AccelBvh& o, float m)
        : tb(t), items(it), out(o), margin(m)
    {
        if (const char* v = getenv("PT_LEAF_MAX")) leaf_max = std::min<size_t>(kAccelLeafMax, std::max(1, atoi(v)));
        if (const char* v = getenv("PT_LEAF_NODE_COST")) node_cost = (float)atof(v);
    }

    void bounds(size_t b, size_t e, float* lo, float* hi) const
    {
        for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
        for (size_t i = b; i < e; ++i) {
            const TriBox& t = tb[items[i]];
            for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], t.lo[k]); hi[k] = std::max(hi[k], t.hi[k]); }
        }
    }

    // 128-bin SAH split of items[b, e) (n > 1): partitions in place, returns the split point
    size_t split(size_t b, size_t e) const
    {
        const size_t n = e - b;
        size_t mid = b + n / 2;
        if (n <= 2) return mid;
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t i = b; i < e; ++i)
            for (int k = 0; k < 3; ++k) {
                clo[k] = std::min(clo[k], tb[items[i]].c[k]);
                chi[k] = std::max(chi[k], tb[items[i]].c[k]);
            }
        constexpr int kBins = 128;
        float best_cost = INFINITY;
        int best_axis = -1, best_split = 0;
        for (int k = 0; k < 3; ++k) {
            const float ext = chi[k] - clo[k];
            if (!(ext > 0.0f)) continue;
            int cnt[kBins] = {0};
            float blo[kBins][3], bhi[kBins][3];
            for (int q = 0; q < kBins; ++q)
                for (int j = 0; j < 3; ++j) { blo[q][j] = INFINITY; bhi[q][j] = -INFINITY; }
            const float scale = kBins / ext;
            for (size_t i = b; i < e; ++i) {
                const TriBox& t = tb[items[i]];
                int q = static_cast<int>((t.c[k] - clo[k]) * scale);
                q = std::min(kBins - 1, std::max(0, q));
                ++cnt[q];
                for (int j = 0; j < 3; ++j) { blo[q][j] = std::min(blo[q][j], t.lo[j]); bhi[q][j] = std::max(bhi[q][j], t.hi[j]); }
            }
            float rlo[kBins][3], rhi[kBins][3];
            int rc[kBins];
            float alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int ac = 0;
            for (int q = kBins - 1; q >= 0; --q) {
                for (int j = 0; j < 3; ++j) { alo[j] = std::min(alo[j], blo[q][j]); ahi[j] = std::max(ahi[j], bhi[q][j]); }
                ac += cnt[q];
                memcpy(rlo[q], alo, sizeof(alo));
                memcpy(rhi[q], ahi, sizeof(ahi));
                rc[q] = ac;
            }
            float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int lc = 0;
            for (int q = 0; q < kBins - 1; ++q) {
                for (int j = 0; j < 3; ++j) { llo[j] = std::min(llo[j], blo[q][j]); lhi[j] = std::max(lhi[j], bhi[q][j]); }
                lc += cnt[q];
                if (lc == 0 || rc[q + 1] == 0) continue;
                const float cost = lc * surface(llo, lhi) + rc[q + 1] * surface(rlo[q + 1], rhi[q + 1]);
                if (cost < best_cost) { best_cost = cost; best_axis = k; best_split = q + 1; }
            }
        }
        if (best_axis >= 0) {
            const int k = best_axis;
            const float scale = kBins / (chi[k] - clo[k]);
            auto it = std::partition(items.begin() + b, items.begin() + e, [&](uint32_t id) {
                int q = static_cast<int>((tb[id].c[k] - clo[k]) * scale);
                q = std::min(kBins - 1, std::max(0, q));
                return q < best_split;
            });
            mid = static_cast<size_t>(it - items.begin());
            if (mid == b || mid == e) mid = b + n / 2;
        }
        return mid;
    }

    void child_box(size_t b, size_t e, float* box) const
    {
        float lo[3], hi[3];
        bounds(b, e, lo, hi);
        for (int k = 0; k < 3; ++k) { box[k] = lo[k] - margin; box[3 + k] = hi[k] + margin; }
    }

    // Returns the child reference of the subtree over items[b, e); nodes in preorder, leaf
    // slots in left-first DFS order.
    uint32_t leaf(size_t b, size_t e)
    {
        const uint32_t slot = static_cast<uint32_t>(out.leaf_order.size());
        for (size_t i = b; i < e; ++i) out.leaf_order.push_back(items[i]);
        return PT_BVH_LEAF_FLAG | (static_cast<uint32_t>(e - b - 1) << 29) | slot;
    }

    uint32_t build(size_t b, size_t e, int depth)
    {
        max_depth = std::max(max_depth, depth);
        if (e - b == 1) return leaf(b, e);
        const size_t mid = split(b, e);
        // a leaf of up to leaf_max triangles when its SAH cost (one test per triangle) is no more
        // than the split's: node_cost + (n_L A_L + n_R A_R) / A -- never at the root, which must be a
        // node (a two-triangle scene, e.g. one quad, would otherwise have no node at all)
        if (e - b <= leaf_max && depth > 0) {
            float lo[3], hi[3], llo[3], lhi[3], rlo[3], rhi[3];
            bounds(b, e, lo, hi);
            bounds(b, mid, llo, lhi);
            bounds(mid, e, rlo, rhi);
            const float a = surface(lo, hi);
            const float split_cost = node_cost + (a > 0.0f ? ((mid - b) * surface(llo, lhi) + (e - mid) * surface(rlo, rhi)) / a
                                                            : (float)(e - b));
            if ((float)(e - b) <= split_cost) return leaf(b, e);
        }
        const uint32_t me = static_cast<uint32_t>(out.nodes.size());
        out.nodes.emplace_back();
        float box[2][6];
        const size_t ranges[2][2] = {{b, mid}, {mid, e}};
        uint32_t refs[2];
        for (int c = 0; c < 2; ++c) {
            child_box(ranges[c][0], ranges[c][1], box[c]);
            refs[c] = build(ranges[c][0], ranges[c][1], depth + 1);
        }
        AccelNode& nd = out.nodes[me];
        memcpy(nd.box, box, sizeof(box));
        nd.child[0] = refs[0];
        nd.child[1] = refs[1];
        return me;
    }
};

// Parallel form of Builder::build with the identical result: the top levels are split serially
// into ~4 subtrees per host thread, the subtrees are built concurrently into private arrays
// (they only touch their own items range), then spliced in preorder with their node and leaf
// indices offset -- exactly where the serial recursion would have emitted them.
struct ParallelBuild {
    struct Skel {
        size_t b, e;
        int depth;
        int left = -1, right = -1;   // -1: a job
        float box[2][6];
        AccelBvh local;
        uint32_t local_root = 0;
        int local_depth = 0;
    };
    const std::vector<TriBox>& tb;
    std::vector<uint32_t>& items;
    float margin;
    std::vector<Skel> skel;
    std::vector<int> jobs;

    int plan(Builder& planner, size_t b, size_t e, int depth, size_t cutoff)
    {
        const int me = static_cast<int>(skel.size());
        skel.emplace_back();
        skel[me].b = b; skel[me].e = e; skel[me].depth = depth;
        if (e - b <= cutoff) { jobs.push_back(me); return me; }
        const size_t mid = planner.split(b, e);
        planner.child_box(b, mid, skel[me].box[0]);
        planner.child_box(mid, e, skel[me].box[1]);
        const int l = plan(planner, b, mid, depth + 1, cutoff);
        const int r = plan(planner, mid, e, depth + 1, cutoff);
        skel[me].left = l;
        skel[me].right = r;
        return me;
    }

    uint32_t emit(int k, AccelBvh& out, int* max_depth)
    {
        Skel& s = skel[k];
        if (s.left < 0) {
            const uint32_t no = static_cast<uint32_t>(out.nodes.size());
            const uint32_t lo = static_cast<uint32_t>(out.leaf_order.size());
            auto remap = [&](uint32_t ref) { return (ref & PT_BVH_LEAF_FLAG) ? ref + lo : ref + no; };
            for (AccelNode nd : s.local.nodes) {
                nd.child[0] = remap(nd.child[0]);
                nd.child[1] = remap(nd.child[1]);
                out.nodes.push_back(nd);
            }
            out.leaf_order.insert(out.leaf_order.end(), s.local.leaf_order.begin(), s.local.leaf_order.end());
            *max_depth = std::max(*max_depth, s.local_depth);
            return remap(s.local_root);
        }
        *max_depth = std::max(*max_depth, s.depth);
        const uint32_t me = static_cast<uint32_t>(out.nodes.size());
        out.nodes.emplace_back();
        const uint32_t l = emit(s.left, out, max_depth);
        const uint32_t r = emit(s.right, out, max_depth);
        AccelNode& nd = out.nodes[me];
        memcpy(nd.box, s.box, sizeof(s.box));
        nd.child[0] = l;
        nd.child[1] = r;
        return me;
    }
};


}  // namespace

double accel_sah_cost(const AccelBvh& acc)
{
    double c = 0.0;
    for (const AccelNode& nd : acc.nodes)
        for (int k = 0; k < 2; ++k)
            if (!(nd.child[k] & PT_BVH_LEAF_FLAG)) c += surface(nd.box[k], nd.box[k] + 3);
    return c + surface(acc.root_box, acc.root_box + 3);
}

int build_accel(const pt_scene& sc, AccelBvh* out)
{
    const uint32_t nt = sc.num_tris;
    if (nt < 2) return fail(PT_E_SCENE, "build_accel: need >= 2 triangles");
    std::vector<TriBox> tb(nt);
    float ext = 0.0f;
    for (uint32_t i = 0; i < nt; ++i) {
        const pt_triangle& t = sc.tris[i];
        const float* v[3] = {&sc.verts[t.v0].x, &sc.verts[t.v1].x, &sc.verts[t.v2].x};
        for (int k = 0; k < 3; ++k) {
            tb[i].lo[k] = std::min(std::min(v[0][k], v[1][k]), v[2][k]);
            tb[i].hi[k] = std::max(std::max(v[0][k], v[1][k]), v[2][k]);
            tb[i].c[k] = 0.5f * (tb[i].lo[k] + tb[i].hi[k]);
            ext = std::max(ext, std::max(std::fabs(tb[i].lo[k]), std::fabs(tb[i].hi[k])));
        }
    }
    if (!std::isfinite(ext)) return fail(PT_E_SCENE, "build_accel: non-finite vertex coordinates");
    // 2^-16 of the scene's coordinate magnitude: ~100x the rounding of any slab value.
    const float margin = std::max(ext, 1.0f) * 0x1p-16f;
    std::vector<uint32_t> items(nt);
    for (uint32_t i = 0; i < nt; ++i) items[i] = i;
    out->nodes.clear();
    out->leaf_order.clear();
    out->nodes.reserve(nt);
    out->leaf_order.reserve(nt);
    AccelBvh scratch;
    Builder planner(tb, items, scratch, margin);
    const unsigned threads = host_threads();
    ParallelBuild pb{tb, items, margin, {}, {}};
    pb.skel.reserve(64 * threads + 16);
    const int top = pb.plan(planner, 0, nt, 0, std::max<size_t>(2048, nt / (4 * std::max(1u, threads))));
    std::atomic<size_t> next_job{0};
    auto worker = [&]() {
        for (size_t j; (j = next_job.fetch_add(1)) < pb.jobs.size();) {
            ParallelBuild::Skel& k = pb.skel[pb.jobs[j]];
            Builder sub(tb, items, k.local, margin);
            k.local.nodes.reserve(k.e - k.b);
            k.local.leaf_order.reserve(k.e - k.b);
            k.local_root = sub.build(k.b, k.e, k.depth);
            k.local_depth = sub.max_depth;
        }
    };
    std::vector<std::thread> ths;
    for (unsigned t = 1; t < threads && t < pb.jobs.size(); ++t) ths.emplace_back(worker);
    worker();
    for (std::thread& t : ths) t.join();
    int max_depth = 0;
    const uint32_t root = pb.emit(top, *out, &max_depth);
    if (root != 0) return fail(PT_E_SCENE, "build_accel: internal error (root %u)", root);
    float lo[3], hi[3];
    planner.bounds(0, nt, lo, hi);
    for (int k = 0; k < 3; ++k) { out->root_box[k] = lo[k] - margin; out->root_box[3 + k] = hi[k] + margin; }
    out->depth = max_depth;
    out->margin = margin;
    return PT_OK;
}

namespace {

float area_of(const float* b)
{
    return surface(b, b + 3);
}

// W-wide collapse (W = 4: Accel4), at most kTris triangles in a node's leaf children
template <int W, uint32_t kTris, class Node, class Out>
struct Collapser {
    const AccelBvh& bin;
    Out& out;
    int max_depth = 0;

    // Collapse the subtree whose binary root is inner node `b`; returns its W-wide index.
    uint32_t run(uint32_t b, int depth)
    {
        max_depth = std::max(max_depth, depth);
        struct Cand { uint32_t ref; float box[6]; };
        Cand c[W];
        int n = 2;
        for (int k = 0; k < 2; ++k) {
            c[k].ref = bin.nodes[b].child[k];
            memcpy(c[k].box, bin.nodes[b].box[k], sizeof(c[k].box));
        }
        // triangles in the leaf children (the walk queues a node's entered leaf triangles as one
        // entry with a kTris-bit slot mask)
        auto leaf_tris = [](uint32_t ref) { return (ref & PT_BVH_LEAF_FLAG) ? accel_leaf_count(ref) : 0u; };
        uint32_t tris = leaf_tris(c[0].ref) + leaf_tris(c[1].ref);
        while (n < W) {   // expand the inner candidate with the largest surface area
            int pick = -1;
            float best = -1.0f;
            for (int k = 0; k < n; ++k) {
                if (c[k].ref & PT_BVH_LEAF_FLAG) continue;
                const AccelNode& y = bin.nodes[c[k].ref];
                if (tris + leaf_tris(y.child[0]) + leaf_tris(y.child[1]) > kTris) continue;
                const float a = area_of(c[k].box);
                if (a > best) { best = a; pick = k; }
            }
            if (pick < 0) break;
            const AccelNode& x = bin.nodes[c[pick].ref];
            Cand second;
            second.ref = x.child[1];
            memcpy(second.box, x.box[1], sizeof(second.box));
            c[pick].ref = x.child[0];
            memcpy(c[pick].box, x.box[0], sizeof(c[pick].box));
            c[n++] = second;
            tris += leaf_tris(x.child[0]) + leaf_tris(x.child[1]);
        }
        const uint32_t me = static_cast<uint32_t>(out.nodes.size());
        out.nodes.emplace_back();
        uint32_t refs[W];
        for (int k = 0; k < W; ++k) {
            if (k >= n) { refs[k] = kAccel4Empty; continue; }
            refs[k] = (c[k].ref & PT_BVH_LEAF_FLAG) ? c[k].ref : run(c[k].ref, depth + 1);
        }
        Node& nd = out.nodes[me];
        for (int k = 0; k < W; ++k) {
            for (int ax = 0; ax < 3; ++ax) {
                // empty slot: a point at 2^100 -- every ray rejects it (entry >= 2^99 beyond any
                // best distance, or exit behind the origin; o*inv stays finite, so no NaN), which
                // keeps the kernel's four box tests branch-free
                nd.lo[ax][k] = (k < n) ? c[k].box[ax] : 0x1p100f;
                nd.hi[ax][k] = (k < n) ? c[k].box[3 + ax] : 0x1p100f;
            }
            nd.child[k] = refs[k];
        }
        return me;
    }
};

// SAH-optimal 4-wide collapse by dynamic programming over the binary tree (the wide-BVH
// conversion of Ylitie et al. 2017 for W = 4): every binary inner node x gets the least cost of
// standing for its subtree in at most m = 1..4 slots of a wide node, where a slot is
//   a leaf (a binary leaf, or an inner node of <= kAccelLeafMax triangles merged into one):
//     c_tri * area * triangles, or
//   a wide node of its own: c_node * area + the best spread of x's two children over 4 slots,
// and m >= 2 may instead pass x's two children on (one slot each or more, split m between them).
// Leaves of <= 2 triangles in <= 4 slots keep a node's leaf triangles within kAccel4LeafTris.
struct DpCollapser {
    const AccelBvh& bin;
    Accel4& out;
    float cn, ct;
    int max_depth = 0;
    struct Rec {
        float area = 0.0f;
        const float* box = nullptr;   // the node's box as its parent holds it (root: root_box)
        uint32_t tris = 0;
        bool as_leaf = false;         // a single slot for it is a merged leaf (else its own wide node)
        float E[5];                   // E[m]: the subtree in <= m slots
        bool self[5];                 // E[m] takes one slot for the node itself
        int8_t split[5];              // passing on: slots for the left child (the right gets the rest)
    };
    std::vector<Rec> rec;

    float leaf_cost(uint32_t ref, const float* box) const { return ct * area_of(box) * (float)accel_leaf_count(ref); }
    float E(uint32_t ref, const float* box, int m) const
    {
        return (ref & PT_BVH_LEAF_FLAG) ? leaf_cost(ref, box) : rec[ref].E[m];
    }
    uint32_t tris_of(uint32_t ref) const { return (ref & PT_BVH_LEAF_FLAG) ? accel_leaf_count(ref) : rec[ref].tris; }

    void solve()
    {
        const size_t n = bin.nodes.size();
        rec.assign(n, Rec());
        rec[0].box = bin.root_box;
        for (size_t i = 0; i < n; ++i)   // preorder: a parent comes before its children
            for (int k = 0; k < 2; ++k)
                if (!(bin.nodes[i].child[k] & PT_BVH_LEAF_FLAG)) rec[bin.nodes[i].child[k]].box = bin.nodes[i].box[k];
        for (size_t i = n; i-- > 0;) {   // reverse preorder: children first
            const AccelNode& x = bin.nodes[i];
            Rec& r = rec[i];
            r.area = area_of(r.box);
            r.tris = tris_of(x.child[0]) + tris_of(x.child[1]);
            float D[5] = {INFINITY, INFINITY, INFINITY, INFINITY, INFINITY};
            int8_t Dk[5] = {0, 0, 0, 0, 0};
            for (int j = 2; j <= 4; ++j)
                for (int k = 1; k < j; ++k) {
                    const float c = E(x.child[0], x.box[0], k) + E(x.child[1], x.box[1], j - k);
                    if (c < D[j]) { D[j] = c; Dk[j] = (int8_t)k; }
                }
            const float wide = cn * r.area + D[4];
            const float leaf = (r.tris <= kAccelLeafMax) ? ct * r.area * (float)r.tris : INFINITY;
            r.as_leaf = leaf <= wide;
            const float one = r.as_leaf ? leaf : wide;
            r.E[0] = INFINITY;
            r.E[1] = one; r.self[1] = true; r.split[1] = 0;
            for (int m = 2; m <= 4; ++m) {
                r.self[m] = one <= D[m];
                r.E[m] = r.self[m] ? one : D[m];
                r.split[m] = Dk[m];
            }
        }
    }

    uint32_t first_slot(uint32_t ref) const
    {
        while (!(ref & PT_BVH_LEAF_FLAG)) ref = bin.nodes[ref].child[0];
        return accel_leaf_slot(ref);
    }

    struct Slot { uint32_t ref; const float* box; bool wide; };
    mutable bool overflow = false;   // place() was asked for a fifth slot (a malformed DP table)
    void place(uint32_t ref, const float* box, int m, Slot* s, int* n) const
    {
        // a slot budget m < 1 or a fifth slot cannot come from a well-formed table (split[] in 1..m-1);
        // refuse it instead of writing past the node's 4 slots
        if (m < 1 || *n >= 4) { overflow = true; return; }
        if (ref & PT_BVH_LEAF_FLAG) { s[(*n)++] = {ref, box, false}; return; }
        const Rec& r = rec[ref];
        if (r.self[m]) {
            if (r.as_leaf) s[(*n)++] = {PT_BVH_LEAF_FLAG | ((r.tris - 1u) << 29) | first_slot(ref), box, false};
            else s[(*n)++] = {ref, box, true};
            return;
        }
        spread(ref, m, s, n);
    }
    void spread(uint32_t ref, int m, Slot* s, int* n) const
    {
        const AccelNode& x = bin.nodes[ref];
        const int k = rec[ref].split[m];
        place(x.child[0], x.box[0], k, s, n);
        place(x.child[1], x.box[1], m - k, s, n);
    }

    uint32_t emit(uint32_t b, int depth)
    {
        max_depth = std::max(max_depth, depth);
        Slot s[4];
        int n = 0;
        spread(b, 4, s, &n);
        const uint32_t me = static_cast<uint32_t>(out.nodes.size());
        out.nodes.emplace_back();
        uint32_t refs[4];
        for (int k = 0; k < 4; ++k) refs[k] = (k >= n) ? kAccel4Empty : s[k].wide ? emit(s[k].ref, depth + 1) : s[k].ref;
        Accel4Node& nd = out.nodes[me];
        for (int k = 0; k < 4; ++k) {
            for (int ax = 0; ax < 3; ++ax) {
                nd.lo[ax][k] = (k < n) ? s[k].box[ax] : 0x1p100f;   // (empty slot: as in Collapser)
                nd.hi[ax][k] = (k < n) ? s[k].box[3 + ax] : 0x1p100f;
            }
            nd.child[k] = refs[k];
        }
        return me;
    }
};

}  // namespace

int collapse_accel4(const AccelBvh& bin, Accel4* out)
{
    out->nodes.clear();
    out->nodes.reserve(bin.nodes.size() / 2 + 1);
    // (PT_COLLAPSE=greedy: the round-1..4 largest-area expansion; the DP measured C3 -0.7% node
    // visits, +0.5% Msamples/s, profiles/r04_dp)
    const char* mode = getenv("PT_COLLAPSE");
    if (!(mode && strcmp(mode, "greedy") == 0)) {
        // cost knobs: finite and positive, else every comparison of the DP fails and no slot split is
        // ever chosen (PT_E_INVALID names the knob instead of building a malformed tree)
        float knob[2] = {1.0f, 0.3f};
        const char* names[2] = {"PT_COLLAPSE_CN", "PT_COLLAPSE_CT"};
        for (int i = 0; i < 2; ++i)
            if (const char* v = getenv(names[i])) {
                char* end = nullptr;
                const double x = strtod(v, &end);
                if (end == v || *end != '\0' || !std::isfinite(x) || !(x > 0.0) || x > 1e30)
                    return fail(PT_E_INVALID, "collapse_accel4: %s=\"%s\" is not a finite positive number", names[i], v);
                knob[i] = (float)x;
            }
        DpCollapser dp{bin, *out, knob[0], knob[1]};
        dp.solve();
        const uint32_t root = dp.emit(0, 0);
        if (dp.overflow) return fail(PT_E_SCENE, "collapse_accel4: a node was given more than 4 slots");
        if (root != 0) return fail(PT_E_SCENE, "collapse_accel4: internal error");
        out->depth = dp.max_depth;
        return PT_OK;
    }
    Collapser<4, kAccel4LeafTris, Accel4Node, Accel4> col{bin, *out};
    const uint32_t root = col.run(0, 0);
    if (root != 0) return fail(PT_E_SCENE, "collapse_accel4: internal error");
    out->depth = col.max_depth;
    return PT_OK;
}

// Structural check of a collapsed tree (host diagnostic, pt_accel_digest): every inner node is
// reached exactly once from the root, every leaf slot of the binary tree exactly once, a node's
// leaf children hold at most kAccel4LeafTris triangles, and every child box of an inner child
// contains that child's own child boxes (the nesting the culling relies on).
int validate_accel4(const AccelBvh& bin, const Accel4& t)
{
    const size_t n4 = t.nodes.size(), nslots = bin.leaf_order.size();
    std::vector<uint8_t> seen_node(n4, 0), seen_slot(nslots, 0);
    std::vector<uint32_t> todo{0};
    seen_node[0] = 1;
    while (!todo.empty()) {
        const uint32_t i = todo.back();
        todo.pop_back();
        const Accel4Node& x = t.nodes[i];
        uint32_t leaf_tris = 0;
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = x.child[k];
            if (c == kAccel4Empty) continue;
            if (c & PT_BVH_LEAF_FLAG) {
                const uint32_t s0 = accel_leaf_slot(c), cnt = accel_leaf_count(c);
                leaf_tris += cnt;
                for (uint32_t j = 0; j < cnt; ++j) {
                    if (s0 + j >= nslots || seen_slot[s0 + j]) return fail(PT_E_SCENE, "validate_accel4: leaf slot %u", s0 + j);
                    seen_slot[s0 + j] = 1;
                }
                continue;
            }
            if (c >= n4 || seen_node[c]) return fail(PT_E_SCENE, "validate_accel4: node %u reached twice or out of range", c);
            seen_node[c] = 1;
            const Accel4Node& y = t.nodes[c];
            for (int q = 0; q < 4; ++q) {
                if (y.child[q] == kAccel4Empty) continue;
                for (int ax = 0; ax < 3; ++ax)
                    if (!(y.lo[ax][q] >= x.lo[ax][k] && y.hi[ax][q] <= x.hi[ax][k]))
                        return fail(PT_E_SCENE, "validate_accel4: node %u child %d leaves its parent's box", c, q);
            }
            todo.push_back(c);
        }
        if (leaf_tris > kAccel4LeafTris) return fail(PT_E_SCENE, "validate_accel4: node %u has %u leaf triangles", i, leaf_tris);
    }
    for (size_t i = 0; i < n4; ++i) if (!seen_node[i]) return fail(PT_E_SCENE, "validate_accel4: node %zu unreachable", i);
    for (size_t s = 0; s < nslots; ++s) if (!seen_slot[s]) return fail(PT_E_SCENE, "validate_accel4: leaf slot %zu unreachable", s);
    return PT_OK;
}

// SAH-style cost of a 4-wide tree (diagnostic): c_node x the surface of every inner node's box
// as its parent holds it + c_tri x surface x triangles of every leaf child, over the root's.
double accel4_cost(const Accel4& t, const float* root_box, double cn, double ct)
{
    double c = cn * area_of(root_box);
    for (const Accel4Node& x : t.nodes)
        for (int k = 0; k < 4; ++k) {
            if (x.child[k] == kAccel4Empty) continue;
            const float b[6] = {x.lo[0][k], x.lo[1][k], x.lo[2][k], x.hi[0][k], x.hi[1][k], x.hi[2][k]};
            c += (x.child[k] & PT_BVH_LEAF_FLAG) ? ct * area_of(b) * accel_leaf_count(x.child[k]) : cn * area_of(b);
        }
    return c / area_of(root_box);
}

}  // namespace pt

// Host-side diagnostic (tests/test_host_surface.py): FNV-1a digest of the render-path BVH that
// pt_create builds (binary SAH nodes + leaf order + BVH4 nodes), its BVH4 node count and depth.
extern "C" int pt_accel_digest(const pt_scene* sc, uint64_t* digest, uint32_t* num_nodes4, int32_t* depth4)
{
    pt::clear_error();
    if (!sc || !digest) return pt::fail(PT_E_INVALID, "pt_accel_digest: null argument");
    pt::AccelBvh acc;
    pt::Accel4 acc4;
    int rc = pt::build_accel(*sc, &acc);
    if (rc == PT_OK) rc = pt::collapse_accel4(acc, &acc4);
    if (rc == PT_OK) rc = pt::validate_accel4(acc, acc4);
    if (rc != PT_OK) return rc;
    if (getenv("PT_TIMING"))
        fprintf(stderr, "pt_accel_digest: SAH cost %.6g, binary depth %d, BVH4 depth %d, BVH4 nodes %zu, BVH4 cost (1, 0.3) %.6g\n",
                pt::accel_sah_cost(acc), acc.depth, acc4.depth, acc4.nodes.size(), pt::accel4_cost(acc4, acc.root_box, 1.0, 0.3));
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        const unsigned char* c = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) { h ^= c[i]; h *= 1099511628211ull; }
    };
    mix(acc.nodes.data(), acc.nodes.size() * sizeof(pt::AccelNode));
    mix(acc.leaf_order.data(), acc.leaf_order.size() * sizeof(uint32_t));
    mix(acc4.nodes.data(), acc4.nodes.size() * sizeof(acc4.nodes[0]));
    *digest = h;
    if (num_nodes4) *num_nodes4 = static_cast<uint32_t>(acc4.nodes.size());
    if (depth4) *depth4 = acc4.depth;
    return PT_OK;
}
