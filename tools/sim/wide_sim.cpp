// wide_sim.cpp -- host-side model of the wavefront walk's cost on W-wide collapses of the render-path
// SAH BVH (W = 4, the kernel's, and wider), on the bench's stand-in scene and camera: per ray, node
// visits, triangle tests and WALK STEPS under the kernel's step rule (walk4_step, pt_device.h: a step
// visits at most one node and tests at most one queued leaf triangle; a node's entered leaf children
// are one leaf-queue entry; inner children nearest first; boxes entered iff max(entry,0) <= min(exit,
// best_t * (1 + 2^-10))).  Rays: the C3 camera's primary rays (sampled pixels) and one cosine bounce
// from each primary hit.  A decision aid for wider nodes, not part of the product.
//
// build: g++ -O2 -std=c++17 -I include tools/sim/wide_sim.cpp -o /tmp/wide_sim -L cudapathtracer_amd
//        -lptamd -Wl,-rpath,$PWD/cudapathtracer_amd
// run:   /tmp/wide_sim <obj> <mtl_dir/> [rays] [top_nodes]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "pt/pt.h"

namespace pt {
struct AccelNode { float box[2][6]; uint32_t child[2]; };
struct AccelBvh {
    std::vector<AccelNode> nodes;
    std::vector<uint32_t> leaf_order;
    float root_box[6];
    int depth = 0;
    float margin = 0.0f;
};
int build_accel(const pt_scene& sc, AccelBvh* out);
}  // namespace pt

namespace {

constexpr uint32_t kLeafFlag = PT_BVH_LEAF_FLAG;
uint32_t leaf_count(uint32_t ref) { return ((ref >> 29) & 3u) + 1u; }
uint32_t leaf_slot(uint32_t ref) { return ref & 0x1fffffffu; }

float area(const float* b)
{
    const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0f;
    return dx * dy + dy * dz + dz * dx;
}

struct WNode {
    int n = 0;
    float box[8][6];
    uint32_t child[8];   // inner index or leaf ref
    int depth = 0;
};

// largest-area expansion up to W children and at most max_tris triangles in leaf children
// (collapse_accel4's rule, accel_build.cpp)
struct Collapse {
    const pt::AccelBvh& bin;
    int W;
    uint32_t max_tris;
    std::vector<WNode> out;
    uint32_t run(uint32_t b, int depth)
    {
        struct Cand { uint32_t ref; float box[6]; };
        Cand c[8];
        int n = 2;
        for (int k = 0; k < 2; ++k) { c[k].ref = bin.nodes[b].child[k]; memcpy(c[k].box, bin.nodes[b].box[k], 24); }
        auto lt = [](uint32_t r) { return (r & kLeafFlag) ? leaf_count(r) : 0u; };
        uint32_t tris = lt(c[0].ref) + lt(c[1].ref);
        while (n < W) {
            int pick = -1;
            float best = -1;
            for (int k = 0; k < n; ++k) {
                if (c[k].ref & kLeafFlag) continue;
                const pt::AccelNode& y = bin.nodes[c[k].ref];
                if (tris + lt(y.child[0]) + lt(y.child[1]) > max_tris) continue;
                const float a = area(c[k].box);
                if (a > best) { best = a; pick = k; }
            }
            if (pick < 0) break;
            const pt::AccelNode& x = bin.nodes[c[pick].ref];
            Cand s;
            s.ref = x.child[1];
            memcpy(s.box, x.box[1], 24);
            c[pick].ref = x.child[0];
            memcpy(c[pick].box, x.box[0], 24);
            c[n++] = s;
            tris += lt(x.child[0]) + lt(x.child[1]);
        }
        const uint32_t me = (uint32_t)out.size();
        out.emplace_back();
        out[me].n = n;
        out[me].depth = depth;
        for (int k = 0; k < n; ++k) {
            memcpy(out[me].box[k], c[k].box, 24);
            const uint32_t r = (c[k].ref & kLeafFlag) ? c[k].ref : run(c[k].ref, depth + 1);
            out[me].child[k] = r;
        }
        return me;
    }
};

struct Tri { float v0[3], e1[3], e2[3]; };

// Moller-Trumbore in float (any consistent t suffices for the cost model)
float tri_hit(const Tri& T, const float* o, const float* d)
{
    const float* e1 = T.e1;
    const float* e2 = T.e2;
    const float p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
    const float a = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    if (std::fabs(a) < 1e-5f) return INFINITY;
    const float f = 1.0f / a;
    const float s[3] = {o[0] - T.v0[0], o[1] - T.v0[1], o[2] - T.v0[2]};
    const float u = f * (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]);
    if (u < 0.0f || u > 1.0f) return INFINITY;
    const float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const float v = f * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
    if (v < 0.0f || u + v > 1.0f) return INFINITY;
    const float t = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
    return t > 0.0f ? t : INFINITY;
}

struct Stats {
    double rays = 0, steps = 0, visits = 0, top_visits = 0, tris = 0, leaf_only_steps = 0, entered = 0;
};

struct Walker {
    const std::vector<WNode>& nodes;
    const std::vector<Tri>& tris;   // by leaf slot
    uint32_t ntop;                  // nodes < ntop: LDS-staged (best-first top)
    // returns best t; counts per the step model
    float walk(const float* o, const float* d, Stats& st) const
    {
        float inv[3], oi[3];
        for (int k = 0; k < 3; ++k) {
            inv[k] = d[k] != 0.0f ? 1.0f / d[k] : std::copysign(0x1p100f, d[k]);
            oi[k] = o[k] * inv[k];
        }
        const float cull = 1.0f + 1.0f / 1024.0f;
        float best = 3.402823466e+38f;
        std::vector<std::pair<float, uint32_t>> stack;
        std::vector<std::vector<uint32_t>> lq;   // leaf-queue entries (LIFO), each a list of slots
        std::vector<uint32_t> pending;           // the entry being tested
        uint32_t node = 0;
        bool have_node = true;
        st.rays += 1;
        while (have_node || !pending.empty()) {
            st.steps += 1;
            const bool visit = have_node && lq.size() <= 3;
            if (!pending.empty()) {
                st.tris += 1;
                const float t = tri_hit(tris[pending.back()], o, d);
                pending.pop_back();
                if (t < best) best = t;
                if (!visit) st.leaf_only_steps += 1;
            }
            if (visit) {
                st.visits += 1;
                if (node < ntop) st.top_visits += 1;
                const WNode& nd = nodes[node];
                const float lim = best * cull;
                std::vector<std::pair<float, uint32_t>> inner;
                std::vector<uint32_t> leaves;
                for (int k = 0; k < nd.n; ++k) {
                    float tn = 0.0f, tf = lim;
                    for (int ax = 0; ax < 3; ++ax) {
                        const float a = nd.box[k][ax] * inv[ax] - oi[ax], b = nd.box[k][3 + ax] * inv[ax] - oi[ax];
                        tn = std::max(tn, std::min(a, b));
                        tf = std::min(tf, std::max(a, b));
                    }
                    if (!(tn <= tf)) continue;
                    st.entered += 1;
                    const uint32_t r = nd.child[k];
                    if (r & kLeafFlag) {
                        for (uint32_t s = 0; s < leaf_count(r); ++s) leaves.push_back(leaf_slot(r) + s);
                    } else {
                        inner.push_back({tn, r});
                    }
                }
                if (!leaves.empty()) {
                    std::reverse(leaves.begin(), leaves.end());   // test lowest slot first
                    if (pending.empty()) pending = leaves;
                    else lq.push_back(leaves);
                }
                std::sort(inner.begin(), inner.end());
                have_node = !inner.empty();
                if (have_node) node = inner[0].second;
                for (size_t k = inner.size(); k-- > 1;) stack.push_back(inner[k]);
            }
            // advance
            if (pending.empty() && !lq.empty()) { pending = lq.back(); lq.pop_back(); }
            if (!have_node) {
                while (!stack.empty()) {
                    const auto e = stack.back();
                    stack.pop_back();
                    if (e.first > best * cull) continue;
                    node = e.second;
                    have_node = true;
                    break;
                }
            }
        }
        return best;
    }
};

// best-first top (by a breadth-first order, which approximates the kernel's area-ordered top)
std::vector<WNode> reorder_bfs(const std::vector<WNode>& in)
{
    std::vector<uint32_t> order, map(in.size());
    order.push_back(0);
    for (size_t i = 0; i < order.size(); ++i)
        for (int k = 0; k < in[order[i]].n; ++k)
            if (!(in[order[i]].child[k] & kLeafFlag)) order.push_back(in[order[i]].child[k]);
    for (size_t i = 0; i < order.size(); ++i) map[order[i]] = (uint32_t)i;
    std::vector<WNode> out(in.size());
    for (size_t i = 0; i < order.size(); ++i) {
        out[i] = in[order[i]];
        for (int k = 0; k < out[i].n; ++k)
            if (!(out[i].child[k] & kLeafFlag)) out[i].child[k] = map[out[i].child[k]];
    }
    return out;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 3) { fprintf(stderr, "usage: wide_sim obj mtl_dir [rays] [top_bytes]\n"); return 2; }
    const int nrays = argc > 3 ? atoi(argv[3]) : 200000;
    const double top_bytes = argc > 4 ? atof(argv[4]) : 97 * 112.0;   // the kernel's LDS top budget
    pt_host_scene* hs = pt_scene_new();
    if (pt_scene_load_obj(hs, argv[1], argv[2], pt_vec3{0.0f, 0.0f, 0.0f}, 1.0f, 0) != 0) { fprintf(stderr, "load failed\n"); return 1; }
    pt_scene sc;
    pt_scene_view(hs, &sc);
    pt::AccelBvh bin;
    if (pt::build_accel(sc, &bin) != 0) { fprintf(stderr, "accel failed\n"); return 1; }
    std::vector<Tri> tris(bin.leaf_order.size());
    for (size_t s = 0; s < tris.size(); ++s) {
        const pt_triangle& t = sc.tris[bin.leaf_order[s]];
        const pt_vec3 a = sc.verts[t.v0], b = sc.verts[t.v1], c = sc.verts[t.v2];
        tris[s] = Tri{{a.x, a.y, a.z}, {b.x - a.x, b.y - a.y, b.z - a.z}, {c.x - a.x, c.y - a.y, c.z - a.z}};
    }
    pt_camera cam{{0.0f, 2.6f, 13.2f}, 1.0f, 3.0f, 0.0f, 1920, 1080};
    // rays: primary (sampled pixels) and a cosine bounce from each primary hit
    std::mt19937 rng(1234);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    struct Ray { float o[3], d[3]; };
    std::vector<Ray> prim, bounce;
    std::vector<WNode> n4;
    {
        Collapse c4{bin, 4, 8, {}};
        c4.run(0, 0);
        n4 = reorder_bfs(c4.out);
    }
    Walker w4{n4, tris, 0};
    Stats dummy;
    for (int i = 0; i < nrays; ++i) {
        const uint32_t x = rng() % 1920, y = rng() % 1080;
        Ray r;
        pt_vec3 o, d;
        pt_camera_ray(&cam, pt_morton_pxl_to_i(x, y), 0, 0.0f, 0.0f, &o, &d);
        r.o[0] = o.x; r.o[1] = o.y; r.o[2] = o.z; r.d[0] = d.x; r.d[1] = d.y; r.d[2] = d.z;
        // pixel (x, y) of the camera's film: pt_camera_ray takes the Morton index
        prim.push_back(r);
        const float t = w4.walk(r.o, r.d, dummy);
        if (!(t < 1e30f)) continue;
        // hit: normal of the triangle hit (recomputed: a second walk would be needed for the id;
        // approximate with the geometric normal of a small probe) -- use a random hemisphere about
        // the reversed ray instead, which has the bounce rays' statistics in a closed scene
        Ray b;
        for (int k = 0; k < 3; ++k) b.o[k] = r.o[k] + r.d[k] * (t - 0.001f);
        float nd[3] = {-r.d[0], -r.d[1], -r.d[2]};
        // cosine-weighted about nd
        const float u1 = U(rng), u2 = U(rng);
        const float rr = std::sqrt(u1), th = 6.2831853f * u2;
        float tx[3] = {std::fabs(nd[0]) > 0.1f ? 0.0f : 1.0f, std::fabs(nd[0]) > 0.1f ? 1.0f : 0.0f, 0.0f};
        float t1[3] = {nd[1] * tx[2] - nd[2] * tx[1], nd[2] * tx[0] - nd[0] * tx[2], nd[0] * tx[1] - nd[1] * tx[0]};
        const float l1 = std::sqrt(t1[0] * t1[0] + t1[1] * t1[1] + t1[2] * t1[2]);
        for (float& v : t1) v /= l1;
        const float t2[3] = {nd[1] * t1[2] - nd[2] * t1[1], nd[2] * t1[0] - nd[0] * t1[2], nd[0] * t1[1] - nd[1] * t1[0]};
        const float z = std::sqrt(std::max(0.0f, 1.0f - u1));
        for (int k = 0; k < 3; ++k) b.d[k] = t1[k] * rr * std::cos(th) + t2[k] * rr * std::sin(th) + nd[k] * z;
        bounce.push_back(b);
    }
    printf("scene tris %u, primary rays %zu, bounce rays %zu, LDS top budget %.0f B\n", sc.num_tris, prim.size(),
           bounce.size(), top_bytes);
    // quant: child planes as 8-bit steps of a power-of-two grid from the node's lower corner,
    // rounded outward (a compressed node of one 128-B line: origin, exponents, 48 plane bytes,
    // 8 child words)
    const struct { int W; uint32_t max_tris; double node_bytes; bool quant; } cfgs[] = {
        {4, 8, 112, false}, {4, 8, 64, true}, {6, 12, 176, false}, {8, 16, 224, false}, {8, 8, 224, false},
        {8, 16, 112, true}};
    for (const auto& cf : cfgs) {
        Collapse col{bin, cf.W, cf.max_tris, {}};
        col.run(0, 0);
        std::vector<WNode> nodes = reorder_bfs(col.out);
        if (cf.quant)
            for (WNode& nd : nodes)
                for (int ax = 0; ax < 3; ++ax) {
                    float lo = INFINITY, hi = -INFINITY;
                    for (int k = 0; k < nd.n; ++k) { lo = std::min(lo, nd.box[k][ax]); hi = std::max(hi, nd.box[k][3 + ax]); }
                    const float step = std::ldexp(1.0f, (int)std::ceil(std::log2(std::max((hi - lo) / 255.0f, 1e-30f))));
                    for (int k = 0; k < nd.n; ++k) {
                        const float ql = std::floor((nd.box[k][ax] - lo) / step), qh = std::ceil((nd.box[k][3 + ax] - lo) / step);
                        nd.box[k][ax] = lo + ql * step;
                        nd.box[k][3 + ax] = lo + std::min(qh, 255.0f) * step;
                    }
                }
        const uint32_t ntop = (uint32_t)std::min<double>(nodes.size(), top_bytes / cf.node_bytes);
        Walker w{nodes, tris, ntop};
        int maxd = 0;
        double fill = 0;
        for (const WNode& n : nodes) { maxd = std::max(maxd, n.depth); fill += n.n; }
        for (int set = 0; set < 2; ++set) {
            Stats st;
            for (const Ray& r : set ? bounce : prim) w.walk(r.o, r.d, st);
            printf("W=%d%s maxtris=%2u nodes %7zu fill %.2f depth %2d top %3u | %s: steps %.2f visits %.2f (global %.2f) "
                   "tris %.2f leaf-only steps %.2f entered/visit %.2f\n",
                   cf.W, cf.quant ? "q" : " ", cf.max_tris, nodes.size(), fill / nodes.size(), maxd, ntop, set ? "bounce " : "primary",
                   st.steps / st.rays, st.visits / st.rays, (st.visits - st.top_visits) / st.rays, st.tris / st.rays,
                   st.leaf_only_steps / st.rays, st.entered / std::max(1.0, st.visits));
        }
    }
    pt_scene_free(hs);
    return 0;
}
