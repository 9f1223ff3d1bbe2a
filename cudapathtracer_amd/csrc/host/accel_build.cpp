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
#include <cmath>
#include <cstring>

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

    Builder(const std::vector<TriBox>& t, std::vector<uint32_t>& it, AccelBvh& o, float m)
        : tb(t), items(it), out(o), margin(m) {}

    void bounds(size_t b, size_t e, float* lo, float* hi) const
    {
        for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
        for (size_t i = b; i < e; ++i) {
            const TriBox& t = tb[items[i]];
            for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], t.lo[k]); hi[k] = std::max(hi[k], t.hi[k]); }
        }
    }

    // Returns the child reference of the subtree over items[b, e).
    uint32_t build(size_t b, size_t e, int depth)
    {
        max_depth = std::max(max_depth, depth);
        const size_t n = e - b;
        if (n == 1) {
            const uint32_t slot = static_cast<uint32_t>(out.leaf_order.size());
            out.leaf_order.push_back(items[b]);
            return PT_BVH_LEAF_FLAG | slot;
        }
        size_t mid = b + n / 2;
        if (n > 2) {
            float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (size_t i = b; i < e; ++i)
                for (int k = 0; k < 3; ++k) {
                    clo[k] = std::min(clo[k], tb[items[i]].c[k]);
                    chi[k] = std::max(chi[k], tb[items[i]].c[k]);
                }
            constexpr int kBins = 32;
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
        }
        const uint32_t me = static_cast<uint32_t>(out.nodes.size());
        out.nodes.emplace_back();
        float box[2][6];
        const size_t ranges[2][2] = {{b, mid}, {mid, e}};
        uint32_t refs[2];
        for (int c = 0; c < 2; ++c) {
            float lo[3], hi[3];
            bounds(ranges[c][0], ranges[c][1], lo, hi);
            for (int k = 0; k < 3; ++k) { box[c][k] = lo[k] - margin; box[c][3 + k] = hi[k] + margin; }
            refs[c] = build(ranges[c][0], ranges[c][1], depth + 1);
        }
        AccelNode& nd = out.nodes[me];
        memcpy(nd.box, box, sizeof(box));
        nd.child[0] = refs[0];
        nd.child[1] = refs[1];
        return me;
    }
};

}  // namespace

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
    Builder bld(tb, items, *out, margin);
    const uint32_t root = bld.build(0, nt, 0);
    if (root != 0) return fail(PT_E_SCENE, "build_accel: internal error (root %u)", root);
    float lo[3], hi[3];
    bld.bounds(0, nt, lo, hi);
    for (int k = 0; k < 3; ++k) { out->root_box[k] = lo[k] - margin; out->root_box[3 + k] = hi[k] + margin; }
    out->depth = bld.max_depth;
    out->margin = margin;
    return PT_OK;
}

namespace {

float area_of(const float* b)
{
    return surface(b, b + 3);
}

struct Collapser {
    const AccelBvh& bin;
    Accel4& out;
    int max_depth = 0;

    // Collapse the subtree whose binary root is inner node `b`; returns its 4-wide index.
    uint32_t run(uint32_t b, int depth)
    {
        max_depth = std::max(max_depth, depth);
        struct Cand { uint32_t ref; float box[6]; };
        Cand c[4];
        int n = 2;
        for (int k = 0; k < 2; ++k) {
            c[k].ref = bin.nodes[b].child[k];
            memcpy(c[k].box, bin.nodes[b].box[k], sizeof(c[k].box));
        }
        while (n < 4) {   // expand the inner candidate with the largest surface area
            int pick = -1;
            float best = -1.0f;
            for (int k = 0; k < n; ++k) {
                if (c[k].ref & PT_BVH_LEAF_FLAG) continue;
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
        }
        const uint32_t me = static_cast<uint32_t>(out.nodes.size());
        out.nodes.emplace_back();
        uint32_t refs[4];
        for (int k = 0; k < 4; ++k) {
            if (k >= n) { refs[k] = kAccel4Empty; continue; }
            refs[k] = (c[k].ref & PT_BVH_LEAF_FLAG) ? c[k].ref : run(c[k].ref, depth + 1);
        }
        Accel4Node& nd = out.nodes[me];
        for (int k = 0; k < 4; ++k) {
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

}  // namespace

int collapse_accel4(const AccelBvh& bin, Accel4* out)
{
    out->nodes.clear();
    out->nodes.reserve(bin.nodes.size() / 2 + 1);
    Collapser col{bin, *out};
    const uint32_t root = col.run(0, 0);
    if (root != 0) return fail(PT_E_SCENE, "collapse_accel4: internal error");
    out->depth = col.max_depth;
    return PT_OK;
}

}  // namespace pt
