// pt_render.hip -- gfx950 render kernels and the render half of the C-ABI (include/pt/pt.h).
//
// One wave renders one 8x8 image tile: lane l owns pixel (8*tx + mx(l), 8*ty + my(l)) with
// (mx, my) the Morton decode of l, and runs ALL of that pixel's samples in order with its
// XORWOW state and f64 running mean in registers (the reference keeps both in HBM and
// re-launches drawPixel per sample, kernel.cu:535-553, 709-736).  Waves are persistent and pull
// tiles from an atomic counter; tile t belongs to shard t % shard_count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../host/host_internal.h"
#include "pt_device.h"

using namespace ptd;

namespace {

constexpr uint32_t kTile = 8;   // 8x8 = 64 pixels = one wave

// A box is skipped when its entry lies beyond best_t * kCullRel (DESIGN.md "Traversal" 4)
constexpr float kCullRel = 1.0f + 1.0f / 1024.0f;
struct Args {
    const DNode* nodes;
    const RNode* rnodes;
    const DTri* tris_leaf;     // DFS leaf order (culled walk)
    const DTri* tris_orig;     // original order (reference walk)
    const DShade* shade;
    const DMat* mats;
    const DLight* lights;
    const uint32_t* jump;
    const uint32_t* jump_bytes;     // byte-position jump matrices J(b << 8) and J(b << 16), b < 256,
                                    // byte-sliced (build_jump_byte_tables); null: per-bit jumps only
    const uint32_t* seed_states;    // curand_init(seed, s0, 0) for s0 < 256: v0..v4 (kJumpEntryWords
                                    // words each; seed_table), with jump_bytes
    float* out;
    unsigned long long* counters;   // [0] traced [1] reference [2] nodes [3] tris [4] samples
    uint32_t* tile_counter;
    uint32_t num_lights;
    float total_light_area;
    float root[6];
    Cam cam;
    int32_t w, h, spp, bounces;
    uint32_t flags;
    uint64_t seed;
    int32_t shard_index, shard_count;
    uint32_t tiles_x, ntiles_shard;
    uint32_t tile_w, tile_h;        // shard tile (multiples of 8): 8x8 blocks of 64 work slots, row-major
    uint32_t tile_bx, tile_blocks;  // 8x8 blocks per tile row / per tile
    uint32_t morton_out;            // PT_ORDER_MORTON: pixel (x,y) written at out[mortonPxltoI(x,y)*3]
    uint32_t stack_words;           // LDS words per wave
    float cull_rel, cull_abs;
    uint32_t* pixel_counter;        // wavefront kernel: next pixel unit
    uint32_t nunits;                // work units: npix * chunks
    uint32_t scene_fast;            // all scene coordinates admit the Markstein quotient
    uint32_t wf_threshold;          // leave the walk when this many lanes wait for shading
    uint32_t wf_iters;              // shading iterations a lane may run per pass before yielding
    uint32_t node_mask;             // low bits of a packed stack entry holding the node index
    uint32_t top_nodes;             // wavefront kernel: BVH4 nodes 0..top_nodes-1 staged in LDS
    uint32_t root_first;            // wavefront kernel: a new ray's root visit in the shading pass (begin_trace)
    uint32_t unit_queues;           // wavefront kernel: units dealt from kQueues counters (> 1) or one
    uint32_t tile_fast4;            // tile kernel: trace with the render-path BVH4 walk (winner check, exact
                                    // slow walk as fallback) instead of the reference-BVH culled walk
    const DNode4* nodes4;           // render-path BVH4 (collapsed SAH BVH)
    const DTri* acc_tris;           // its leaf-order triangle records (id, reference rank, parent)
    const uint32_t* rparent;        // reference BVH: parent of each node (winner chain check)
    const float4* hrec;             // per render-path slot, 48 B: {reference parent's lo, hi.x}, {hi.y, hi.z,
                                    // parent index, triangle id}, {normal, material} -- the winner check's
                                    // words (both integrators) and, for integrator 0, the checked hit's
                                    // shading normal and material on the same line
    uint32_t* spill;                // LDS-stack overflow, entry k of lane g at spill[(k-kRing)*stride + g]
    uint32_t spill_stride;
    uint32_t cold_stride;           // records of the cold array (one per resident lane)
    float acc_root[6];
    uint32_t* cold;                 // per-lane shading state of the wavefront kernel (ColdRec)
    const uint32_t* pix_states;     // per work unit u, word k at [k*nunits + u] (kUnitWords, init_pixel_states)
    uint32_t npix;                  // pixel slots of this shard (ntiles_shard * 64)
    uint32_t nwhole;                // slots 0..nwhole-1 are whole-pixel units (unit u = slot u); the
    uint32_t ntail;                 // ntail = npix - nwhole last slots are split: the first nmid of them
    uint32_t nmid;                  // into chunks_mid sample chunks, the rest into `chunks`; units are
    uint32_t chunks_mid;            // numbered whole, then mid (chunk-major), then the rest (chunk-major)
    uint32_t chunks;                // (init_pixel_states writes each unit's pixel and sample range)
    uint32_t nfin;                  // ... of which the last nfin slots form a third grade of chunks_fin
    uint32_t chunks_fin;            // chunks (the queue's final, shortest units)
    uint32_t* pmemo;                // split slots: primary hit of tail slot t as one 64-bit word: lo = tri + 2
                                    // (0 = not yet), hi = t
    double* lbuf;                   // split slots: per-sample radiance, channel k of sample n of tail slot t
                                    // at lbuf[((n-1) * ntail + t) * 3 + k] (sample-major: a wave of
                                    // finalize_pixels reads 64 slots' sample n as 1.5 KB in a row)
    const float4* spheres;          // sphere primitives: center xyz, radius (hit ids num_tris + i)
    uint32_t num_spheres;
    uint32_t num_tris;
    uint32_t sphere_mat_base;       // material of sphere i = mats[sphere_mat_base + i]
    uint32_t* tri_counts;           // PT_FLAG_COUNT: per-triangle test counts by original id (kernel.cu:133)
    const float4* shade_m;          // per triangle 48 B: {normal, Le.r}, {albedo, Le.g}, {Le.b, material, -, -} --
                                    // the material's f64 colours as floats, set only when every material's colours
                                    // are float-exact (MTL values are floats): one fetch per bounce, not two
                                    // dependent ones (shade, then mats); null: shade + mats
    const DTri* emis;               // last-bounce light probe: the emissive triangles' records (see begin_trace)
    uint32_t num_emis;              // 0 = probe off
    uint32_t rec_shading;           // integrator 0's checked hits take their normal and material from hrec (a
                                    // scene larger than the LDS top); 0: from shade_m by triangle id (a tree
                                    // held whole in LDS -- C2 -- where that one fetch is an L2 hit anyway)
    unsigned long long* lane_times; // diagnostic (PT_LANE_TIMING): wall clock of each lane's end, then each
                                    // wave's start and exit (render_unidir_wf), or null
    uint32_t head;                  // integrator 1 on the wavefront kernel (init_pixel_states' replay)
};

__device__ __forceinline__ V3 ld_norm(const DShade* s, int32_t tri)
{
    const float4 q = *reinterpret_cast<const float4*>(s + tri);
    return v3(q.x, q.y, q.z);
}
__device__ __forceinline__ int32_t ld_mat(const DShade* s, int32_t tri) { return s[tri].mat; }

// ------------------------------------------------------------------ spheres
// The reference has sphere.h but no sphere code; the semantics are this build's, shared with
// the oracle (or_sphere_t): unit d, oc = o - c, b = oc.d, disc = b*b - (oc.oc - r*r), nearer
// root -b - sqrt(disc) if > 0, else -b + sqrt(disc) if > 0.  Spheres are tested after every
// triangle with strict <, so a tie keeps the triangle.
__device__ __forceinline__ float sphere_t(V3 o, V3 d, float4 sp)
{
    const V3 oc = o - v3(sp.x, sp.y, sp.z);
    const float b = dot(oc, d);
    const float c = dot(oc, oc) - sp.w * sp.w;
    const float disc = b * b - c;
    if (!(disc >= 0.0f)) return kMaxFloat;
    const float q = sqrtf(disc);
    float t = -b - q;
    if (t > 0.0f) return t;
    t = -b + q;
    if (t > 0.0f) return t;
    return kMaxFloat;
}
// closest of (htri, ht) and the spheres
__device__ __forceinline__ void apply_spheres(const Args& a, V3 o, V3 d, int32_t* htri, float* ht)
{
    for (uint32_t k = 0; k < a.num_spheres; ++k) {
        const float t = sphere_t(o, d, a.spheres[k]);
        if (0.0f < t && t < *ht) { *ht = t; *htri = (int32_t)(a.num_tris + k); }
    }
}
// primitive id -> material index / normal at p (spheres: (p - c) / r)
__device__ __forceinline__ int32_t prim_mat(const Args& a, int32_t id)
{
    return ((uint32_t)id < a.num_tris) ? ld_mat(a.shade, id) : (int32_t)(a.sphere_mat_base + ((uint32_t)id - a.num_tris));
}
__device__ __forceinline__ V3 prim_normal(const Args& a, int32_t id, V3 p)
{
    if ((uint32_t)id < a.num_tris) return ld_norm(a.shade, id);
    const float4 sp = a.spheres[(uint32_t)id - a.num_tris];
    return (p - v3(sp.x, sp.y, sp.z)) / sp.w;
}

// ------------------------------------------------------------------ per-lane tracer
template <bool kRefWalk, bool kCount>
struct Tracer {
    const Args* a;
    uint32_t* stack;
    int lane;
    Counters cnt;
    uint32_t traced;
    uint32_t reference;
    // primary-ray memo (exact: keyed on the ray's bits)
    bool have;
    uint32_t ko[3], kd[3];
    Hit kh;


    __device__ __forceinline__ Hit trace(V3 o, V3 d)
    {
        ++traced;
        Hit h;
        h.tri = -1;
        h.t = kMaxFloat;
        if (a->num_tris > 0) {
            if (kRefWalk) {
                h = trace_reference<kCount>(o, d, a->rnodes, a->tris_orig, stack, lane, cnt);
            } else if (a->tile_fast4) {
                // the wavefront kernel's walk, run to its end by this lane (DESIGN.md "Traversal"); its
                // LDS rings (this block's one wave) and HBM spill column
                const uint32_t lane_off = (blockIdx.x * 64u + (uint32_t)lane) * 4u;
                Stack4 S;
                S.ring = stack + lane;
                S.stride = a->spill_stride;
                S.spill_base = a->spill;
                S.lane_off = &lane_off;
                S.off_mask = ~0u;
                if ((a->scene_fast != 0u) && ray_fast(o, d)) {
                W4 w;
                if (walk4_begin(w, o, d, a->acc_root, a->cull_abs)) {
                    while (walk4_step<kCount>(w, o, d, a->nodes4, a->acc_tris, S, a->cull_rel, a->cull_abs, a->node_mask,
                                              cnt)) {
                    }
                    h.t = w.best_t;
                    bool ok = true;
                    if (w.best_slot != kNone) {
                        const float4 C = a->acc_tris[w.best_slot].c;
                        h.tri = (int32_t)__float_as_uint(C.y);
                        ok = ref_tested(__float_as_uint(C.w), o, d, a->rnodes, a->rparent);
                    }
                    if (!ok) {
                        atomicAdd(a->counters + 8, 1ull);   // (accel_fallbacks, as trace_rays counts them)
                        trace_slow(o, d, a->root, a->nodes, a->tris_leaf, S.spill(), S.stride, a->cull_rel, a->cull_abs,
                                   &h.tri, &h.t, cnt.tri_counts);
                    }
                }
                } else {   // outside the Markstein preconditions: the exact slow walk
                    atomicAdd(a->counters + 8, 1ull);
                    trace_slow(o, d, a->root, a->nodes, a->tris_leaf, S.spill(), S.stride, a->cull_rel, a->cull_abs,
                               &h.tri, &h.t, cnt.tri_counts);
                }
            } else {
                h = trace_culled<kCount>(o, d, a->root, a->nodes, a->tris_leaf, stack, lane, a->cull_rel, a->cull_abs, cnt);
            }
        }
        if (a->num_spheres) apply_spheres(*a, o, d, &h.tri, &h.t);
        return h;
    }

    __device__ Hit trace_primary(V3 o, V3 d, bool memo)
    {
        ++reference;
        if (memo && have && ko[0] == __float_as_uint(o.x) && ko[1] == __float_as_uint(o.y) &&
            ko[2] == __float_as_uint(o.z) && kd[0] == __float_as_uint(d.x) && kd[1] == __float_as_uint(d.y) &&
            kd[2] == __float_as_uint(d.z))
            return kh;
        Hit h = trace(o, d);
        if (memo) {
            have = true;
            ko[0] = __float_as_uint(o.x); ko[1] = __float_as_uint(o.y); ko[2] = __float_as_uint(o.z);
            kd[0] = __float_as_uint(d.x); kd[1] = __float_as_uint(d.y); kd[2] = __float_as_uint(d.z);
            kh = h;
        }
        return h;
    }

    __device__ Hit trace_secondary(V3 o, V3 d)
    {
        ++reference;
        return trace(o, d);
    }
};


// kernel.cu:44-54
__device__ __forceinline__ V3 get_tangent(V3 n)
{
    const V3 c1 = cross(n, v3(0, 0, 1));
    const V3 c2 = cross(n, v3(0, 1, 0));
    return (dot(c1, c1) > dot(c2, c2)) ? c1 : c2;
}
__device__ __forceinline__ V3 to_frame(V3 n, float lx, float ly, float lz)   // kernel.cu:70-75, 91-96
{
    const V3 tg = get_tangent(n);
    const V3 bt = cross(n, tg);
    return normalized(n * ly + tg * lx + bt * lz);
}
__device__ __forceinline__ V3 cosine_ray(V3 n, Rng& rng)                     // kernel.cu:78-99
{
    const float u1 = rng_uniform(rng);
    const float u2 = rng_uniform(rng);
    const float r = sqrtf(u1);
    const float theta = (float)(2 * 3.14159 * (double)u2);
    float s, c;
    det_sincos(theta, &s, &c);
    const float x = r * c;
    const float z = r * s;
    const float y = sqrtf(__builtin_fmaxf(0.0f, 1.0f - u1));
    return to_frame(n, x, y, z);
}
__device__ __forceinline__ V3 rand_ray(V3 n, Rng& rng)                       // kernel.cu:60-77
{
    const float u1 = rng_uniform(rng);
    const float u2 = rng_uniform(rng);
    const float r = sqrtf(1.0f - u1 * u1);
    const float phi = (float)(2 * 3.14159 * (double)u2);
    float s, c;
    det_sincos(phi, &s, &c);
    return to_frame(n, r * c, u1, r * s);
}
__device__ __forceinline__ C3 mat_albedo(const DMat* m) { return c3(m->albedo[0], m->albedo[1], m->albedo[2]); }
__device__ __forceinline__ C3 mat_emission(const DMat* m) { return c3(m->emission[0], m->emission[1], m->emission[2]); }
__device__ __forceinline__ C3 brdf(const DMat* m) { return cmulf(mat_albedo(m), (float)(1 / 3.14159)); }  // kernel.cu:101-104

// Area-CDF pick over the emissive triangles + uniform point (kernel.cu:466-495 / 231-262).
// The scan stops once randArea <= 0: no later light can then satisfy randArea > 0 (areas are
// >= 0), so the selection is unchanged.
__device__ __forceinline__ int32_t pick_light(const Args& a, Rng& rng, V3* p)
{
    float ra = a.total_light_area * rng_uniform(rng);
    uint32_t sel = a.num_lights;   // slot of triangle 0 (nothing picked)
    for (uint32_t j = 0; j < a.num_lights && ra > 0; ++j) {
        const float area = a.lights[j].area;
        if (ra < area && ra > 0) sel = j;
        ra -= area;
    }
    float u = rng_uniform(rng);
    float v = rng_uniform(rng);
    const DLight& L = a.lights[sel];
    if (L.pad != 0.0f) {   // sphere light (d8): uniform point, z = 1 - 2u, phi = 2*3.14159*v
        const float z = 1.0f - 2.0f * u;
        const float rxy = sqrtf(__builtin_fmaxf(0.0f, 1.0f - z * z));
        const float phi = (float)(2 * 3.14159 * (double)v);
        float si, co;
        det_sincos(phi, &si, &co);
        *p = v3(L.v0[0], L.v0[1], L.v0[2]) + v3(rxy * co, rxy * si, z) * L.a1[0];
        return L.tri;
    }
    const V3 v0 = v3(L.v0[0], L.v0[1], L.v0[2]);
    const V3 a1 = v3(L.a1[0], L.a1[1], L.a1[2]);
    const V3 a2 = v3(L.a2[0], L.a2[1], L.a2[2]);
    if ((double)(u + v) > 1.0) {
        u = (float)((double)u + 2 * (0.5 - (double)u));
        v = (float)((double)v + 2 * (0.5 - (double)v));
    }
    *p = v0 + a1 * u + a2 * v;
    return L.tri;
}

// ------------------------------------------------------------------ integrator 0
// radianceAlongSingleStep2, kernel.cu:417-515.  Dead-path skip: once weight == 0 every later
// bounce adds weight*Le = 0, so (unless PT_FLAG_NO_DEAD_PATH_SKIP) the lane stops tracing and
// only replays the RNG draws each remaining bounce would make (1 + 2, or 1 + 3 and the
// i = max(i, D-2) jump), keeping its stream aligned with the reference.
template <bool kRefWalk, bool kCount>
__device__ C3 radiance_unidir(const Args& a, Tracer<kRefWalk, kCount>& tr, V3 o, V3 dir, Rng& rng, bool skip_dead,
                              bool memo)
{
    C3 accum = c3(0, 0, 0);
    C3 weight = c3(1, 1, 1);
    const int D = a.bounces;
    for (int i = 0; i < D; ++i) {
        if (skip_dead && i > 0 && czero(weight)) {
            ++tr.reference;
            const float u = rng_uniform(rng);
            if (u < 0.5) { rng_next(rng); rng_next(rng); }
            else { rng_next(rng); rng_next(rng); rng_next(rng); i = (i > D - 2) ? i : D - 2; }
            continue;
        }
        Hit h = (i == 0) ? tr.trace_primary(o, dir, memo) : tr.trace_secondary(o, dir);
        int32_t tri = h.tri;
        float t = (float)((double)h.t - 0.001);                                 // :431
        if ((double)t < 0.001) weight = c3(0, 0, 0);                             // :432
        if (t > kMaxFloat - 1) { weight = c3(0, 0, 0); tri = 0; t = 0; }         // :436
        const V3 pos = o + dir * t;                                               // :449
        const DMat* cm = a.mats + prim_mat(a, tri);
        const V3 normal = prim_normal(a, tri, pos);
        if (cm->emission[0] != 0) {                                               // :453
            accum = cadd(accum, cmul(weight, mat_emission(cm)));
            weight = c3(0, 0, 0);
        }
        V3 ldir;
        const float u = rng_uniform(rng);
        if (u < 0.5) {                                                            // :460
            ldir = cosine_ray(normal, rng);
            weight = cmul(weight, cmulf(brdf(cm), (float)3.14159));
        } else {                                                                  // :466
            V3 p1;
            pick_light(a, rng, &p1);
            const V3 d = p1 - pos;
            ldir = normalized(d);
            const float inv_prob = a.total_light_area;
            const float cos_l = __builtin_fmaxf(0.0f, dot(ldir, normal));
            const float cos_o = __builtin_fmaxf(0.0f, dot(v3(0, -1, 0), ldir * -1));
            const float G = cos_l * cos_o / dot(d, d);
            weight = cmul(weight, cmulf(cmulf(brdf(cm), G), inv_prob));
            i = (i > D - 2) ? i : D - 2;
        }
        o = pos;
        dir = ldir;
    }
    return accum;
}

// ------------------------------------------------------------------ integrator 1
__device__ __forceinline__ float geo_term(V3 xa, V3 xb, V3 na, V3 nb)      // kernel.cu:370-373
{
    const V3 seg = xa - xb;
    const V3 ray = normalized(seg);
    float G = __builtin_fabsf(dot(ray, na) * dot(ray, nb)) / dot(seg, seg);
    if (G != G) G = 0;
    return G;
}

// radianceAlongSingleStep, kernel.cu:217-415 (decision d2: a miss on the camera's second
// bounce uses triangle 0 and t = 0 instead of reading tris[-1]).
template <bool kRefWalk, bool kCount>
__device__ C3 radiance_head(const Args& a, Tracer<kRefWalk, kCount>& tr, V3 cam_o, V3 cam_d, Rng& rng, bool memo)
{
    V3 x[5], nrm[5];
    int32_t mat[5] = {0, 0, 0, 0, 0};
    float ip[5];
    {
        V3 p;
        const int32_t sel = pick_light(a, rng, &p);
        const V3 n = prim_normal(a, sel, p);
        x[0] = p + n * 0.001f;
        nrm[0] = n;
        mat[0] = prim_mat(a, sel);
        ip[0] = a.total_light_area;
    }
    {
        const V3 od = rand_ray(nrm[0], rng);
        Hit h = tr.trace_secondary(x[0], od);
        int32_t tri = h.tri;
        float t = (float)((double)h.t - 0.001);
        if (t > kMaxFloat - 1) { tri = 0; t = 0; }
        const V3 pos = x[0] + od * t;
        const V3 n2 = prim_normal(a, tri, pos);
        const float G = __builtin_fabsf(dot(n2, od)) / __builtin_fmaxf(0.001f, t * t);
        x[1] = pos; nrm[1] = n2; mat[1] = prim_mat(a, tri);
        ip[1] = (float)(2 * 3.14159 / (double)G);
    }
    x[4] = cam_o; nrm[4] = cam_d; ip[4] = 1;
    {
        Hit h = tr.trace_primary(cam_o, cam_d, memo);
        int32_t tri = h.tri;
        float t = (float)((double)h.t - 0.001);
        if (t > kMaxFloat - 1) { tri = 0; t = 0; }
        x[3] = cam_o + cam_d * t;
        nrm[3] = prim_normal(a, tri, x[3]);
        mat[3] = prim_mat(a, tri);
        ip[3] = 1;
    }
    {
        const V3 d = cosine_ray(nrm[3], rng);
        Hit h = tr.trace_secondary(x[3], d);
        int32_t tri = h.tri;
        float t = (float)((double)h.t - 0.001);
        if (t > kMaxFloat - 1 || tri < 0) { tri = 0; t = 0; }
        x[2] = x[3] + d * t;
        const V3 n = prim_normal(a, tri, x[2]);
        float G = __builtin_fabsf(dot(nrm[3], d) * dot(n, d)) / (t * t);
        if (G == 0) G = 1;
        if (G != G) G = 1;
        nrm[2] = n;
        mat[2] = prim_mat(a, tri);
        ip[2] = (float)(3.14159 / (double)G);
    }
    C3 accum = c3(0, 0, 0);
    const C3 le = mat_emission(a.mats + mat[0]);
    const C3 e3 = mat_emission(a.mats + mat[3]);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 2; j < 4; ++j) {
            C3 w = cmulf(le, ip[0]);
#pragma unroll
            for (int k = 1; k <= i; ++k) {
                const float G = geo_term(x[k], x[k - 1], nrm[k], nrm[k - 1]);
                w = cmulf(cmulf(cmul(w, cdivf(mat_albedo(a.mats + mat[k]), 3.14159f)), G), ip[k]);
            }
#pragma unroll
            for (int k = j + 1; k < 4; ++k) {
                const float G = geo_term(x[k], x[k - 1], nrm[k], nrm[k - 1]);
                w = cmulf(cmulf(cmul(w, cdivf(mat_albedo(a.mats + mat[k]), 3.14159f)), G), ip[k]);
            }
            const V3 seg = x[j] - x[i];
            const float len = length(seg);
            const V3 ray = normalized(seg);
            float G = __builtin_fmaxf(0.0f, dot(ray, nrm[j]) * dot(ray * -1, nrm[i])) / dot(seg, seg);
            if (G != G) G = 0;
            w = cmulf(cmulf(cmul(w, cdivf(mat_albedo(a.mats + mat[j]), 3.14159f)), G), ip[j]);
            const float m = (float)fmax(w.r, fmax(w.g, w.b));
            float V = 0;
            if ((double)m > 0.01) {
                Hit h = tr.trace_secondary(x[i], ray);
                if ((double)__builtin_fabsf(h.t - len) <= 0.01) V = 1;
            }
            w = cmulf(w, V);
            accum = cadd(accum, w);
            accum = cadd(accum, e3);
        }
    }
    return accum;
}

// ------------------------------------------------------------------ camera (camera.h:77-97)
// A kernel-argument value made opaque at its use, so that the compiler derives what it needs from
// it there (e.g. a conversion) instead of hoisting the result out of the persistent loop into
// registers that stay live across the walk (where they cost spills).
template <typename T>
__device__ __forceinline__ T fresh(T x)
{
    asm volatile("" : "+s"(x));
    return x;
}

// (kFresh: the image size made opaque at its use -- the wavefront kernel's register discipline; the
// tile kernel, whose arguments may live in memory, takes them as they are)
template <bool kFresh = true>
__device__ __forceinline__ void camera_ray(const Cam& cam, uint32_t px, uint32_t py, bool lens, float u1, float u2,
                                           V3* o, V3* d)
{
    const int cw = kFresh ? fresh(cam.w) : cam.w, ch = kFresh ? fresh(cam.h) : cam.h;
    V3 film = v3((float)px / (float)cw - 0.5f, (float)py / (float)ch - 0.5f, 0.0f);
    V3 lo = v3(0.0f, 0.0f, 0.0f);
    if (lens) {
        const float r = cam.radius * sqrtf(u1);
        const float theta = (float)(2 * 3.14159 * (double)u2);
        float s, c;
        det_sincos(theta, &s, &c);
        lo = v3(r * c, r * s, 0.0f);
    }
    film.z = cam.dist;
    film = (film * -cam.focal) / cam.dist;
    *o = lo + v3(cam.pos[0], cam.pos[1], cam.pos[2]);
    *d = normalized(film - lo);
}

__device__ __forceinline__ uint32_t morton2(uint32_t x, uint32_t y)   // camera.h:66-75
{
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        r |= ((x >> b) & 1u) << (2 * b);
        r |= ((y >> b) & 1u) << (2 * b + 1);
    }
    return r;
}

// Work slot q of this shard -> pixel: tile q / (tile_w*tile_h) of the shard (tile t = shard_index +
// that * shard_count, row-major over the tile grid), 8x8 block ((q >> 6) mod tile_blocks) of the tile
// (row-major), Morton order within the block -- 64 consecutive slots (a wave's lanes) are one 8x8
// block.  False for a slot outside the image (partial tiles at the right / bottom edge).
// (host and device: pt_shard_pixels exports the same mapping; T = Args or TileMap)
template <typename T>
__host__ __device__ __forceinline__ bool unit_pixel(const T& a, uint32_t q, uint32_t* px, uint32_t* py)
{
    const uint32_t k = q >> 6, l = q & 63u;
    const uint32_t tl = (a.tile_blocks == 1u) ? k : k / a.tile_blocks;
    const uint32_t b = k - tl * a.tile_blocks;
    const uint32_t t = (uint32_t)a.shard_index + tl * (uint32_t)a.shard_count;
    const uint32_t qx = (l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4);
    const uint32_t qy = ((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4);
    const uint32_t by = (a.tile_bx == 1u) ? b : b / a.tile_bx;
    *px = (t % a.tiles_x) * a.tile_w + (b - by * a.tile_bx) * kTile + qx;
    *py = (t / a.tiles_x) * a.tile_h + by * kTile + qy;
    return *px < (uint32_t)a.w && *py < (uint32_t)a.h;
}
// the tile-map fields of Args, for the host
struct TileMap {
    int32_t w, h, shard_index, shard_count;
    uint32_t tiles_x, tile_w, tile_h, tile_bx, tile_blocks;
};
// index of pixel (px, py) in the output buffer (pt_params.pixel_order)
__device__ __forceinline__ size_t out_pixel(const Args& a, uint32_t px, uint32_t py)
{
    return a.morton_out ? (size_t)morton2(px, py) : (size_t)py * (size_t)a.w + px;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ------------------------------------------------------------------ the render kernel
template <int kIntegrator, bool kRefWalk, bool kCount>
__global__ __launch_bounds__(64) void render_tiles(Args a)
{
    extern __shared__ uint32_t lds_stack[];
    const int lane = threadIdx.x;
    Tracer<kRefWalk, kCount> tr;
    tr.a = &a;
    tr.stack = lds_stack;
    tr.lane = lane;
    if (kCount) tr.cnt.tri_counts = a.tri_counts;
    tr.traced = 0;
    tr.reference = 0;
    unsigned long long samples = 0;
    const bool skip_dead = !(a.flags & PT_FLAG_NO_DEAD_PATH_SKIP);
    const bool memo = !(a.flags & PT_FLAG_NO_PRIMARY_CACHE);
    for (;;) {
        uint32_t k = 0;   // the next 8x8 block of this shard's tiles (64 work slots)
        if (lane == 0) k = atomicAdd(a.tile_counter, 1u);
        k = __shfl(k, 0, 64);
        if (k >= a.ntiles_shard * a.tile_blocks) break;
        uint32_t px, py;
        if (!unit_pixel(a, k * 64u + (uint32_t)lane, &px, &py)) continue;
        const uint32_t idx = morton2(px, py);
        Rng rng;
        rng_init(rng, a.seed, idx, a.jump);
        const bool lens = (idx == 0) || (a.cam.radius != 0.0f);
        tr.have = false;
        double m0 = 0.0, m1 = 0.0, m2 = 0.0;
        for (int n = 1; n <= a.spp; ++n) {
            float u1 = 0.0f, u2 = 0.0f;
            if (lens) { u1 = rng_uniform(rng); u2 = rng_uniform(rng); }
            V3 o, d;
            camera_ray<false>(a.cam, px, py, lens, u1, u2, &o, &d);
            C3 L;
            if (kIntegrator == PT_INTEGRATOR_HEAD) L = radiance_head(a, tr, o, d, rng, memo);
            else L = radiance_unidir(a, tr, o, d, rng, skip_dead, memo);
            const double fn1 = (double)(float)(n - 1), fn = (double)(float)n;   // kernel.cu:551-552
            m0 = (m0 * fn1) / fn + L.r / fn;
            m1 = (m1 * fn1) / fn + L.g / fn;
            m2 = (m2 * fn1) / fn + L.b / fn;
        }
        samples += (unsigned long long)a.spp;
        float* o3 = a.out + out_pixel(a, px, py) * 3;
        o3[0] = (float)m0;
        o3[1] = (float)m1;
        o3[2] = (float)m2;
    }
    const unsigned long long c0 = wave_sum(tr.traced), c1 = wave_sum(tr.reference), c4 = wave_sum(samples);
    unsigned long long c2 = 0, c3v = 0;
    if (kCount) { c2 = wave_sum(tr.cnt.nodes); c3v = wave_sum(tr.cnt.tris); }
    if (lane == 0) {
        atomicAdd(a.counters + 0, c0);
        atomicAdd(a.counters + 1, c1);
        atomicAdd(a.counters + 4, c4);
        if (kCount) { atomicAdd(a.counters + 2, c2); atomicAdd(a.counters + 3, c3v); }
    }
}

// ------------------------------------------------------------------ wavefront kernel
// Integrator 0 as a per-lane state machine (the persistent "while-while" scheme): each lane owns
// one pixel at a time and walks through its samples and bounces; the wave alternates between
// (a) BVH walk steps for the lanes that are tracing, kept running until wf_threshold lanes are
// waiting, and (b) a shading pass in which every waiting lane consumes its hit, draws its next
// direction, finishes samples / pixels and fetches new pixels.  Lanes therefore do not idle
// until the slowest ray of the wave is done, which is where the tile kernel loses most time.
// Arithmetic and RNG consumption per lane are exactly those of radianceAlongSingleStep2.
enum : uint32_t { ST_IDLE = 0, ST_TRACE = 1, ST_SHADE = 2, ST_DONE = 3, ST_SLOW = 4, ST_CHECK = 5,
                  ST_WALKED = 6 };   // (walk finished in this walk phase: CHECK / SHADE / SLOW decided after it)

// Per-lane shading state ("cold": not needed while the lane walks) lives in HBM and is loaded /
// stored only around the shading phase, so the walk phase's register footprint is the ray, the
// walk state and the stack -- which is what sets the kernel's occupancy.
// Layout: 16-B cells, lane-major within a cell row -- word w of record g at byte
// ((w / 4) * records + g) * 16 + (w % 4) * 4 -- so the words a pass always needs come as four
// coalesced 16-B-per-lane loads (and stores) instead of fifteen 4-B ones: a vector-memory
// instruction costs about the same address-pipeline time at 4 and at 16 B per lane.
enum : int {
    CW_N = 0, CW_I, CW_FLAGS, CW_RNG_D,       // cell 0
    CW_RNG_V0 = 4,                            // cell 1: v0..v3
    CW_WGT = 8,                               // cells 2, 3.lo: wgt (f64 x 3, lo/hi words)
    CW_RNG_V4 = 14, CW_NEND = 15,             // cell 3.hi: v4, last sample number of the unit
    CW_ACC = 16,                              // cells 4, 5.lo: acc (f64 x 3)
    CW_M = 22,                                // cells 5.hi, 6: running mean m0..m2 (f64)
    CW_PX = 28, CW_PY, CW_MTRI, CW_MT,        // cell 7: pixel, primary memo (tri, t)
    CW_CD = 32,                               // cell 8: camera ray direction of a pinhole unit (CF_CAMC) ...
    CW_Q = 35,                                //         ... and a split unit's tail slot (per-sample buffer row)
    kColdWords = 36
};
// CF_ACC0: the sample's accumulator is 0 (not yet written: the record's acc words are stale)
enum : uint32_t { CF_LENS = 1, CF_HAVE = 2, CF_PRIMARY = 4, CF_OWNER = 8, CF_SHARE = 16, CF_MEMO = 32, CF_CAMC = 64,
                  CF_ACC0 = 128, CF_SPLIT = 256, CF_CHUNK0 = 512 };
// CF_CHUNK0 (integrator 0): a split pixel's first chunk (samples 1..chunk_first(1)) keeps the running mean
// itself, as a whole pixel does, and leaves it in its slot's sample-1 row of lbuf for finalize_pixels to
// continue from.

// Accessed as raw buffer loads/stores: one VGPR lane offset for the whole record and the cell
// offset (w / 4) * stride in an SGPR, so no per-word 64-bit addresses are held across the phase.
// ld/st: one word; ld2/st2: words k, k+1 (k even); ld4/st4: a whole cell (k % 4 == 0).
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
struct ColdRec {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t voff;      // lane byte offset (16 * record)
    uint32_t sbytes;    // bytes between consecutive cells of one record (16 * records)
    __device__ __forceinline__ int vo(int k) const { return (int)(voff + 4u * (uint32_t)(k & 3)); }
    __device__ __forceinline__ int so(int k) const { return (int)((uint32_t)(k >> 2) * sbytes); }
    __device__ __forceinline__ uint32_t ld(int k) const
    {
        return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, vo(k), so(k), 0);
    }
    __device__ __forceinline__ void st(int k, uint32_t v) const
    {
        __builtin_amdgcn_raw_buffer_store_b32(v, rs, vo(k), so(k), 0);
    }
    __device__ __forceinline__ uint2 ld2(int k) const
    {
        const u2v v = __builtin_amdgcn_raw_buffer_load_b64(rs, vo(k), so(k), 0);
        return make_uint2(v.x, v.y);
    }
    __device__ __forceinline__ void st2(int k, uint32_t x, uint32_t y) const
    {
        __builtin_amdgcn_raw_buffer_store_b64(u2v{x, y}, rs, vo(k), so(k), 0);
    }
    __device__ __forceinline__ uint4 ld4(int k) const
    {
        const u4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, vo(k), so(k), 0);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    __device__ __forceinline__ void st4(int k, uint32_t x, uint32_t y, uint32_t z, uint32_t w) const
    {
        __builtin_amdgcn_raw_buffer_store_b128(u4v{x, y, z, w}, rs, vo(k), so(k), 0);
    }
    __device__ __forceinline__ double ldd(int k) const
    {
        const uint2 v = ld2(k);
        return __hiloint2double((int)v.y, (int)v.x);
    }
    __device__ __forceinline__ void std_(int k, double v) const
    {
        st2(k, (uint32_t)__double2loint(v), (uint32_t)__double2hiint(v));
    }
};
__device__ __forceinline__ double dbl(uint32_t lo, uint32_t hi) { return __hiloint2double((int)hi, (int)lo); }
__device__ __forceinline__ uint32_t dlo(double v) { return (uint32_t)__double2loint(v); }
__device__ __forceinline__ uint32_t dhi(double v) { return (uint32_t)__double2hiint(v); }

// kMinWaves: waves per SIMD the register allocation must allow (launch bound); 4 = 128 VGPRs,
// 5 = 96, 6 = 80 -- more resident waves hide more memory latency, at the price of spilling
// shading-phase values (the walk loop itself stays spill-free down to 96).
// Work unit u = sample chunk c = u / npix of pixel slot q = u % npix: samples
// [c*spp/chunks, (c+1)*spp/chunks).  With one chunk a unit is a whole pixel.
// Per-unit words of init_pixel_states' output beyond the XORWOW state (words 0..5: v0..v4, d)
enum : uint32_t { UW_PXY = 6, UW_N0, UW_NEND, UW_TQ, UW_CD, kUnitWords = UW_CD + 3 };
constexpr uint32_t kNoPixel = 0xffffffffu;   // UW_PXY of a slot outside the image
constexpr uint32_t kNoUnit = 0xffffffffu;
constexpr int kCounterWords = 96;   // counters[]: 0..63 as listed, 64..95 the tail bins
constexpr uint32_t kQueues = 8;              // unit counters (Args::unit_queues > 1)
constexpr uint32_t kQueueBlock = 64;         // units per block of a counter's class
constexpr uint32_t kQueueStride = 32;        // words between the counters (one 128-B line each)
constexpr uint32_t kMaxProbeEmitters = 4;    // last-bounce light probe: at most this many emissive triangles
// LDS of a wavefront block after the counters: the probe's emitter count (16 B) and records, then the
// staged BVH4 top nodes
// then the NEE light records (lights[0..num_lights], the last being "nothing picked") when at most
// kLdsLights of them: the area-CDF pick and the picked record read LDS, not two dependent fetches
constexpr uint32_t kLdsLights = 5;
constexpr uint32_t kProbeLdsBytes = 16 + kMaxProbeEmitters * (uint32_t)sizeof(DTri) + kLdsLights * (uint32_t)sizeof(DLight);
__device__ __forceinline__ uint32_t chunk_first(const Args& a, uint32_t c, uint32_t chunks)
{
    return (uint32_t)(((uint64_t)c * (uint32_t)a.spp) / chunks);
}
// The chunk count of split slot t (its grade: the first nmid slots mid, the last nfin final, the rest fine) -- the one
// definition init_pixel_states (which deals the chunks), the render kernel (CF_CHUNK0's end) and finalize_pixels
// (which continues chunk 0's running mean from sample chunk_first(1) on) share.
__device__ __forceinline__ uint32_t slot_chunks(const Args& a, uint32_t t)
{
    return t < a.nmid ? a.chunks_mid : t >= a.ntail - a.nfin ? a.chunks_fin : a.chunks;
}

// The XORWOW draws one sample of radianceAlongSingleStep2 consumes, without tracing: the count
// depends only on the draws themselves (lens pair; per bounce u, then 2 for a cosine direction or
// 3 for a light sample, which also jumps i to D-2) -- the same replay as the dead-path skip.
__device__ __forceinline__ void replay_sample(Rng& rng, bool lens, int D)
{
    if (lens) { rng_next(rng); rng_next(rng); }
    int i = 0;
    while (i < D) {
        const float u = rng_uniform(rng);
        if (u < 0.5) { rng_next(rng); rng_next(rng); }
        else { rng_next(rng); rng_next(rng); rng_next(rng); i = (i > D - 2) ? i : D - 2; }
        ++i;
    }
}

// setupCurand (kernel.cu:527-533) for the wavefront kernel: the XORWOW state of every work unit
// of this shard -- curand_init of its pixel, fast-forwarded over the unit's earlier samples --
// computed in parallel before the render, so that a lane starting a unit inside the state
// machine loads 20 B instead of running the jump-ahead with its wave waiting.
__global__ __launch_bounds__(256) void init_pixel_states(Args a, uint32_t* __restrict__ st)
{
    // one lane per pixel slot: curand_init, then one pass over the samples that writes the state
    // at the start of every chunk, with everything else a lane needs to start the unit (pixel,
    // sample range, pinhole camera ray): the refill in the render kernel is then a few loads
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (blockIdx.x == 0) {   // this render's counters, unit counters and wall-clock minima (no memset launches)
        for (uint32_t k = threadIdx.x; k < (uint32_t)kCounterWords; k += 256u)
            a.counters[k] = (k == 20u || k == 21u) ? ~0ull : 0ull;
        for (uint32_t k = threadIdx.x; k < kQueueStride * (kQueues + 1); k += 256u) a.pixel_counter[k] = 0u;
        if (threadIdx.x < 4) a.tile_counter[threadIdx.x] = 0u;
    }
    if (q >= a.npix) return;
    const bool split = q >= a.nwhole;
    const uint32_t t = q - a.nwhole;   // split slot (row of the per-sample buffer)
    if (split) {   // its primary-hit word (pmemo): none yet
        a.pmemo[2 * t] = 0u;
        a.pmemo[2 * t + 1] = 0u;
    }
    const bool mid = split && t < a.nmid;
    const uint32_t f0 = a.ntail - a.nfin;   // first slot of the final grade
    const bool fin = split && t >= f0;
    const uint32_t nc = split ? slot_chunks(a, t) : 1u;
    auto unit = [&](uint32_t c) -> size_t {
        if (!split) return (size_t)q;
        if (mid) return (size_t)a.nwhole + (size_t)c * a.nmid + t;
        const size_t fine0 = (size_t)a.nwhole + (size_t)a.chunks_mid * a.nmid;
        if (!fin) return fine0 + (size_t)c * (f0 - a.nmid) + (t - a.nmid);
        return fine0 + (size_t)a.chunks * (f0 - a.nmid) + (size_t)c * a.nfin + (t - f0);
    };
    const size_t N = a.nunits;
    uint32_t px, py;
    if (!unit_pixel(a, q, &px, &py)) {   // a slot outside the image (partial tile): no unit
        for (uint32_t c = 0; c < nc; ++c) st[UW_PXY * N + unit(c)] = kNoPixel;
        return;
    }
    const uint32_t idx = morton2(px, py);
    Rng r;
    if (a.jump_bytes) {
        // curand_init(seed, idx, 0) = J(idx) v(seed): the jump matrices are powers of one matrix,
        // so they commute and J(idx) = J(idx & 0xff0000) J(idx & 0xff00) J(idx & 0xff) -- the low
        // byte's product is tabulated per render (seed_states), the next two bytes' per context
        // (jump_bytes): 40 lookups instead of 20 per set bit of idx
        uint32_t v[5];
        const uint32_t* p0 = a.seed_states + (size_t)(idx & 255u) * kJumpEntryWords;
        for (int k = 0; k < 5; ++k) v[k] = p0[k];
        const uint32_t b1 = (idx >> 8) & 255u, b2 = (idx >> 16) & 255u;
        constexpr size_t kMat = (size_t)20 * 256 * kJumpEntryWords;
        if (b1) jump_apply(v, a.jump_bytes + (size_t)b1 * kMat);
        if (b2) jump_apply(v, a.jump_bytes + (size_t)(256u + b2) * kMat);
        for (int k = 24; k < 32; ++k)   // (images beyond 4096 x 4096: the remaining bits one by one)
            if ((idx >> k) & 1u) jump_apply(v, a.jump + (size_t)k * kMat);
        r.d = rng_seed_d(a.seed);
        r.v0 = v[0]; r.v1 = v[1]; r.v2 = v[2]; r.v3 = v[3]; r.v4 = v[4];
    } else {
        rng_init(r, a.seed, idx, a.jump);
    }
    const bool lens = (idx == 0) || (a.cam.radius != 0.0f);
    V3 o, d = v3(0.0f, 0.0f, 0.0f);
    if (!lens) camera_ray(a.cam, px, py, false, 0.0f, 0.0f, &o, &d);   // the pixel's pinhole ray
    uint32_t done = 0;
    for (uint32_t c = 0; c < nc; ++c) {
        const uint32_t s0 = split ? chunk_first(a, c, nc) : 0u;
        if (a.head) {   // integrator 1: a fixed 7 draws per sample (+2 lens): light pick 3, rand_ray 2, cosine 2
            for (; done < s0; ++done)
                for (int k = (lens ? 9 : 7); k > 0; --k) rng_next(r);
        }
        for (; done < s0; ++done) replay_sample(r, lens, a.bounces);
        const size_t u = unit(c);
        st[u] = r.v0;
        st[N + u] = r.v1;
        st[2 * N + u] = r.v2;
        st[3 * N + u] = r.v3;
        st[4 * N + u] = r.v4;
        st[5 * N + u] = r.d;       // the Weyl counter advances with every draw
        st[UW_PXY * N + u] = px | (py << 16);
        st[UW_N0 * N + u] = (s0 + 1u) | (lens ? 0x80000000u : 0u);
        st[UW_NEND * N + u] = split ? chunk_first(a, c + 1, nc) : (uint32_t)a.spp;
        st[UW_TQ * N + u] = split ? t : 0u;
        st[UW_CD * N + u] = __float_as_uint(d.x);
        st[(UW_CD + 1) * N + u] = __float_as_uint(d.y);
        st[(UW_CD + 2) * N + u] = __float_as_uint(d.z);
    }
}

// The per-render table of init_pixel_states: curand_init(seed, s0, 0) for the 256 low bytes s0.
__global__ __launch_bounds__(256) void seed_table(Args a, uint32_t* __restrict__ out)
{
    Rng r;
    rng_init(r, a.seed, threadIdx.x, a.jump);
    uint32_t* e = out + (size_t)threadIdx.x * kJumpEntryWords;
    e[0] = r.v0; e[1] = r.v1; e[2] = r.v2; e[3] = r.v3; e[4] = r.v4;
}

// Per context: the byte-sliced matrices J(b << 8) (m = b) and J(b << 16) (m = 256 + b), b < 256,
// entry (j, x) = J * (x << 8j), each the product of the per-bit matrices J_k of b's set bits
// (applied to the entry's basis combination through the per-bit byte-sliced tables).
__global__ __launch_bounds__(256) void build_jump_byte_tables(const uint32_t* __restrict__ jb, uint32_t* __restrict__ out)
{
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;   // (m, j, x), x fastest
    if (g >= 512u * 20u * 256u) return;
    const uint32_t x = g & 255u, j = (g >> 8) % 20u, m = (g >> 8) / 20u;
    const uint32_t b = m & 255u, shift = (m < 256u) ? 8u : 16u;
    uint32_t v[5] = {0u, 0u, 0u, 0u, 0u};
    v[j >> 2] = x << (8 * (j & 3));
    constexpr size_t kMat = (size_t)20 * 256 * kJumpEntryWords;
    for (uint32_t i = 0; i < 8; ++i)
        if ((b >> i) & 1u) jump_apply(v, jb + (size_t)(shift + i) * kMat);
    uint32_t* e = out + (size_t)g * kJumpEntryWords;
    e[0] = v[0]; e[1] = v[1]; e[2] = v[2]; e[3] = v[3]; e[4] = v[4];
    e[5] = 0u; e[6] = 0u; e[7] = 0u;
}

// Split slots: the running mean of kernel.cu:551-552, in sample order, over the stored
// per-sample radiance of each split pixel of this shard.
__global__ __launch_bounds__(256) void finalize_pixels(Args a)
{
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= a.ntail) return;
    uint32_t px, py;
    if (!unit_pixel(a, a.nwhole + t, &px, &py)) return;
    const size_t pix = out_pixel(a, px, py);
    const double* L = a.lbuf + (size_t)t * 3;
    const size_t stride = (size_t)a.ntail * 3;   // one sample of every slot
    // integrator 0: chunk 0 left its running mean after samples 1..e0 in the sample-1 row (CF_CHUNK0);
    // integrator 1 stores every sample (its chunk 0 keeping the mean measured -1% on the 1/8 shard)
    const uint32_t e0 = a.head ? 0u : chunk_first(a, 1u, slot_chunks(a, t));
    double m0 = 0.0, m1 = 0.0, m2 = 0.0;
    if (e0 != 0u) { m0 = L[0]; m1 = L[1]; m2 = L[2]; }
    L += (size_t)e0 * stride;
    // one sample: the six quotients by fn as one IEEE reciprocal + Markstein corrections (RN(x/fn)
    // for finite x clear of under/overflow, as in the render kernel's sample end) -- else the wave
    // divides
    auto step = [&](int n, double l0, double l1, double l2) {
        const double fn1 = (double)(float)(n - 1), fn = (double)(float)n;
        const double x0 = m0 * fn1, x1 = m1 * fn1, x2 = m2 * fn1;
        if (__ballot(!(quot_ok(x0) && quot_ok(x1) && quot_ok(x2) && quot_ok(l0) && quot_ok(l1) && quot_ok(l2))) == 0ull) {
            const double rf = 1.0 / fn;
            m0 = div_mk_d(x0, fn, rf) + div_mk_d(l0, fn, rf);
            m1 = div_mk_d(x1, fn, rf) + div_mk_d(l1, fn, rf);
            m2 = div_mk_d(x2, fn, rf) + div_mk_d(l2, fn, rf);
        } else {
            m0 = x0 / fn + l0 / fn;
            m1 = x1 / fn + l1 / fn;
            m2 = x2 / fn + l2 / fn;
        }
    };
    // eight samples' loads issued together, the next eight issued before these are consumed (a wave's
    // loads of one sample are 64 consecutive slots: whole lines)
    int n = (int)e0 + 1;
    double v[24];
    if (n + 7 <= a.spp) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { v[3 * k] = L[k * stride]; v[3 * k + 1] = L[k * stride + 1]; v[3 * k + 2] = L[k * stride + 2]; }
    }
    for (; n + 7 <= a.spp; n += 8) {
        L += 8 * stride;
        double q[24];
        const bool more = n + 15 <= a.spp;
        if (more) {
#pragma unroll
            for (int k = 0; k < 8; ++k) { q[3 * k] = L[k * stride]; q[3 * k + 1] = L[k * stride + 1]; q[3 * k + 2] = L[k * stride + 2]; }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) step(n + k, v[3 * k], v[3 * k + 1], v[3 * k + 2]);
        if (more) {
#pragma unroll
            for (int k = 0; k < 24; ++k) v[k] = q[k];
        }
    }
    for (; n <= a.spp; ++n, L += stride) step(n, L[0], L[1], L[2]);
    float* o3 = a.out + pix * 3;
    o3[0] = (float)m0;
    o3[1] = (float)m1;
    o3[2] = (float)m2;
}

// One event per active lane added to an LDS counter with a single atomic per wave.
__device__ __forceinline__ void wave_count(unsigned long long* c, int lane)
{
    const uint64_t m = __ballot(1);
    if (lane == __ffsll((long long)m) - 1) atomicAdd(c, (unsigned long long)__popcll(m));
}

// The shading half of the wavefront state machine, for the lanes that are not tracing: consume
// the pending hit (winner check; exact slow walk when needed), run bounces, finish and start
// samples until the lane needs a trace or its unit is done, then give finished lanes new units.
// On return the lane's state is ST_TRACE (w set up for its ray), ST_SHADE / ST_SLOW (shading
// pending: a memo hit, a root miss or a slow ray right after a refill) or ST_DONE.
// Counting variant only: SEC(k) counts the waves that execute section k of the shading code
// (counters[32 + k]; a profile of where shading issue slots go -- DESIGN.md "Measurement").
enum : int { SEC_PASS = 0, SEC_CHECK, SEC_SLOW, SEC_BOUNCE, SEC_EMIT, SEC_COSINE, SEC_LIGHT, SEC_SAMPLE_END,
             SEC_START, SEC_CAMERA, SEC_DEAD, SEC_BEGIN, SEC_REFILL, SEC_MEMO, SEC_RECORD, SEC_PROBE, kSections = 16 };
constexpr int kHist = 16;   // counting variant: walk steps per ray, log2 buckets (counters[48 + b])
constexpr int kTailBins = 16;   // counting variant: lane end / wave exit times after the queue drained,
                                // bin k = [10 us x 2^(k-1), 10 us x 2^k) of the 100-MHz wall clock (bin 0: < 10 us)
__device__ __forceinline__ uint32_t tail_bin(unsigned long long ticks)
{
    const unsigned long long q = ticks / 1000ull;
    return q == 0ull ? 0u : min((uint32_t)kTailBins - 1, 64u - (uint32_t)__clzll((long long)q));
}
#ifdef PT_SEC_MARKERS   // analysis builds: mark the sections in the ISA listing
#define SEC_MARK(k) asm volatile("; SEC " #k)
#else
#define SEC_MARK(k)
#endif
#define SEC(k)                                                                                   \
    do {                                                                                         \
        SEC_MARK(k);                                                                             \
        if (kCount) {                                                                            \
            const uint64_t m_ = __ballot(1);                                                     \
            if (lane == __ffsll((long long)m_) - 1)                                              \
                atomicAdd(reinterpret_cast<uint32_t*>(lcnt + 4) + (k), 1u);                      \
        }                                                                                        \
    } while (0)

// The kernel arguments as the shading pass reads them: from the kernarg segment (render_unidir_wf's
// only explicit argument, at offset 0) through a pointer made opaque at the pass's start, so that the
// scalar loads of the shading-only fields cannot be hoisted to the kernel's entry -- which would keep
// dozens of SGPRs live across the walk loop and push the walk's own values into SGPR spills.
typedef const __attribute__((address_space(4))) Args KArgs;
__device__ __forceinline__ const Args& kernel_args_opaque()
{
    KArgs* p = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const Args*)p;
}

template <bool kCount>
__device__ __forceinline__ void shade_lane(const Args& a_in, const ColdRec& R, int lane, uint32_t& state, V3& ro, V3& rd,
                                           int32_t& htri, float& ht, W4& w, const Stack4& S,
                                           unsigned long long* lcnt, const uint32_t* lprobe, uint32_t* done_rel,
                                           Counters& cnt)
{
    (void)a_in;
    const Args& a = kernel_args_opaque();
    const int D = a.bounces;
    SEC(SEC_PASS);
    // the words every pass needs: four 16-B cells (issued first: their round trip overlaps the
    // winner check's two dependent ones)
    const uint4 k0 = R.ld4(CW_N), k1 = R.ld4(CW_RNG_V0), k2 = R.ld4(CW_WGT), k3 = R.ld4(CW_WGT + 4);
    // the checked winner's slot: the bounce that follows reads its normal and material from the slot's
    // record (the line the check just fetched) instead of the triangle's shading record
    uint32_t hslot = kNone;
    if (state == ST_CHECK) {
        SEC(SEC_CHECK);
        // the winner must be a triangle the reference tests (DESIGN.md "Traversal"); if not
        // (rare), the exact reference-BVH walk redoes the ray
        const uint32_t slot = (uint32_t)htri;
        const float4* hr = a.hrec + 3 * (size_t)slot;
        const float4 b0 = hr[0], b1 = hr[1];
        htri = (int32_t)__float_as_uint(b1.w);
        state = ref_tested_box(b0, b1, __float_as_uint(b1.z), ro, rd, a.rnodes, a.rparent) ? ST_SHADE : ST_SLOW;
        if (state == ST_SHADE && a.num_spheres == 0 && a.rec_shading) hslot = slot;
    }
    int n = (int)k0.x, i = (int)k0.y;
    uint32_t fl = k0.z;
    Rng rng;
    rng.d = k0.w; rng.v0 = k1.x; rng.v1 = k1.y; rng.v2 = k1.z; rng.v3 = k1.w; rng.v4 = k3.z;
    uint32_t nend = k3.w;
    C3 wgt = c3(dbl(k2.x, k2.y), dbl(k2.z, k2.w), dbl(k3.x, k3.y));

    // begin a trace of (o, d); true = the lane continues shading at once (root miss, or
    // a ray outside the Markstein preconditions, which takes the exact slow walk).  bound: the walk
    // accepts hits with t < bound (kMaxFloat: a plain trace; see the light probe below)
    auto begin_trace = [&](V3 o, V3 d, float bound) -> bool {
        wave_count(lcnt + 0, lane);
        SEC(SEC_BEGIN);
        if (a.num_tris == 0) { htri = -1; ht = kMaxFloat; state = ST_SHADE; return true; }   // spheres only
        if (!((a.scene_fast != 0u) && ray_fast(o, d))) { state = ST_SLOW; return true; }
        if (!walk4_begin(w, o, d, a.acc_root, a.cull_abs)) {
            htri = -1; ht = kMaxFloat;
            state = (bound == kMaxFloat) ? ST_SHADE : ST_SLOW;
            return true;
        }
        w.best_t = bound;
        state = ST_TRACE;
        return false;
    };
    // start sample n of pixel (px, py): camera ray, then memo or trace
    // (c7 / c8: the record's cells 7 (pixel, memo) and 8 (pinhole direction) when the caller already
    // holds them -- fetched with the previous sample's end, or just written by the refill -- so the
    // start costs no dependent fetch)
    auto start_sample = [&](uint32_t px, uint32_t py, bool have_cells, uint4 c7, uint4 c8) -> bool {
        i = 0;
        fl |= CF_ACC0;   // acc = 0 (stored on the sample's first emission)
        wgt = c3(1, 1, 1);
        float u1 = 0.0f, u2 = 0.0f;
        const bool lens = (fl & CF_LENS) != 0u;
        if (lens) { u1 = rng_uniform(rng); u2 = rng_uniform(rng); }
        SEC(SEC_START);
        if (lens || !(fl & CF_CAMC)) {
            SEC(SEC_CAMERA);
            camera_ray(a.cam, px, py, lens, u1, u2, &ro, &rd);
            if (!lens) {   // a pinhole ray is the same for every sample of the pixel
                R.st(CW_CD, __float_as_uint(rd.x)); R.st(CW_CD + 1, __float_as_uint(rd.y)); R.st(CW_CD + 2, __float_as_uint(rd.z));
                fl |= CF_CAMC;
            }
        } else {
            ro = v3(0.0f, 0.0f, 0.0f) + v3(fresh(a.cam.pos[0]), fresh(a.cam.pos[1]), fresh(a.cam.pos[2]));   // as camera_ray forms it
            const uint4 cd = have_cells ? c8 : R.ld4(CW_CD);
            rd = v3(__uint_as_float(cd.x), __uint_as_float(cd.y), __uint_as_float(cd.z));
        }
        wave_count(lcnt + 1, lane);
        if (fl & CF_HAVE) {
            SEC(SEC_MEMO);
            const uint2 mm = have_cells ? make_uint2(c7.z, c7.w) : R.ld2(CW_MTRI);
            htri = (int32_t)mm.x; ht = __uint_as_float(mm.y);
            fl = (fl & ~CF_PRIMARY) | CF_MEMO; state = ST_SHADE;
            return true;
        }
        if (fl & CF_SHARE) {
            // the pixel's chunk 0 may have published the (sample-invariant) primary hit
            const uint32_t q = have_cells ? c8.w : R.ld(CW_Q);
            // hit and flag in one word: a relaxed agent-scope load (coherent across the XCDs' L2s
            // for this word) needs no acquire, i.e. no invalidation of this XCD's L2
            const uint64_t mv = __hip_atomic_load(reinterpret_cast<uint64_t*>(a.pmemo) + q, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)mv != 0u) {
                htri = (int32_t)((uint32_t)mv - 2u);
                ht = __uint_as_float((uint32_t)(mv >> 32));
                fl = (fl | CF_PRIMARY | CF_MEMO) & ~CF_SHARE;   // stores the unit memo on shading
                state = ST_SHADE;
                return true;
            }
        }
        fl = (!(a.flags & PT_FLAG_NO_PRIMARY_CACHE) && !lens) ? (fl | CF_PRIMARY) : (fl & ~CF_PRIMARY);
        return begin_trace(ro, rd, kMaxFloat);
    };

    // A lane whose samples need no trace (primary memo hit on an emitter or a miss: the path is
    // dead after bounce 0) would otherwise run sample after sample here while the rest of the
    // wave waits; after wf_iters shading iterations it yields with its pending hit (ST_SHADE /
    // ST_SLOW) and resumes in the next pass, alongside the other lanes' work.
    // The refill (lanes whose unit is finished take the next units of this shard) runs after the
    // first shading iteration, so a unit that starts from a known first hit (a split pixel's memo)
    // is shaded in the second iteration of the same pass instead of waiting out a walk phase.
    bool again = (state == ST_SHADE || state == ST_SLOW);
    for (uint32_t iters = 0; iters < a.wf_iters; ++iters) {
      if (again) {
        again = false;
        if (state == ST_SLOW) {
            wave_count(lcnt + 3, lane);
            SEC(SEC_SLOW);
            trace_slow(ro, rd, a.root, a.nodes, a.tris_leaf, S.spill(), S.stride, a.cull_rel, a.cull_abs,
                       &htri, &ht, kCount ? a.tri_counts : nullptr);
        }
        state = ST_SHADE;
        if (a.num_spheres && !(fl & CF_MEMO)) apply_spheres(a, ro, rd, &htri, &ht);
        fl &= ~CF_MEMO;
        if (fl & CF_PRIMARY) {
            fl = (fl | CF_HAVE) & ~CF_PRIMARY;
            R.st2(CW_MTRI, (uint32_t)htri, __float_as_uint(ht));
            if (fl & CF_OWNER) {
                const uint32_t q = R.ld(CW_Q);
                // (one relaxed 64-bit store: no release, i.e. no write-back of this XCD's L2)
                __hip_atomic_store(reinterpret_cast<uint64_t*>(a.pmemo) + q,
                                   ((uint64_t)__float_as_uint(ht) << 32) | (uint32_t)(htri + 2), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                fl &= ~CF_OWNER;
            }
        }
        // bounce i of radianceAlongSingleStep2 (kernel.cu:427-512) on hit (htri, ht)
        {
            SEC(SEC_BOUNCE);
            int32_t tri = htri;
            float t = (float)((double)ht - 0.001);
            if ((double)t < 0.001) wgt = c3(0, 0, 0);
            if (t > kMaxFloat - 1) { wgt = c3(0, 0, 0); tri = 0; t = 0; }
            const V3 pos = ro + rd * t;
            V3 normal;
            C3 m_em, m_alb;   // the material's emission and albedo (materialDesc, f64)
            if (hslot != kNone) {   // (a checked hit: finite t, so tri is the winner)
                const float4 q2 = a.hrec[3 * (size_t)hslot + 2];
                const DMat* cm = a.mats + (int32_t)__float_as_uint(q2.w);
                normal = v3(q2.x, q2.y, q2.z);
                m_em = mat_emission(cm);
                m_alb = mat_albedo(cm);
                hslot = kNone;
            } else if (a.shade_m && (uint32_t)tri < a.num_tris) {
                const float4* rec = a.shade_m + 3 * (size_t)(uint32_t)tri;
                const float4 q0 = rec[0], q1 = rec[1], q2 = rec[2];
                normal = v3(q0.x, q0.y, q0.z);
                m_em = c3(q0.w, q1.w, q2.x);
                m_alb = c3(q1.x, q1.y, q1.z);
            } else {
                const DMat* cm = a.mats + prim_mat(a, tri);
                normal = prim_normal(a, tri, pos);
                m_em = mat_emission(cm);
                m_alb = mat_albedo(cm);
            }
            if (m_em.r != 0) {
                SEC(SEC_EMIT);
                C3 acc = c3(0.0, 0.0, 0.0);
                if (!(fl & CF_ACC0)) {
                    const uint4 a01 = R.ld4(CW_ACC);
                    const uint2 a2 = R.ld2(CW_ACC + 4);
                    acc = c3(dbl(a01.x, a01.y), dbl(a01.z, a01.w), dbl(a2.x, a2.y));
                }
                fl &= ~CF_ACC0;
                acc = cadd(acc, cmul(wgt, m_em));
                R.st4(CW_ACC, dlo(acc.r), dhi(acc.r), dlo(acc.g), dhi(acc.g)); R.st2(CW_ACC + 4, dlo(acc.b), dhi(acc.b));
                wgt = c3(0, 0, 0);
            }
            // The two sampling branches (kernel.cu:470-497 light sample, 498-509 cosine) with their
            // common steps done once for the wave instead of once per branch: the draws (cosine:
            // u1, u2; light: area pick, u, v -- the same first two positions), the one sin/cos
            // (cosine theta, or a sphere light's phi), the normalisation and the f64 weight
            // update.  Per lane the operations and their order are those of cosine_ray() /
            // pick_light() + the reference's weight expressions.
            V3 ldir;
            const float u = rng_uniform(rng);
            const bool cosb = u < 0.5;
            const float r1 = rng_uniform(rng), r2 = rng_uniform(rng);
            float r3 = 0.0f;
            const DLight* L = nullptr;
            bool need_sc = cosb;
            float ang = r2;
            if (!cosb) {
                SEC(SEC_LIGHT);
                r3 = rng_uniform(rng);
                // area-CDF pick (pick_light); the scan stops once randArea <= 0
                float ra = a.total_light_area * r1;
                uint32_t sel = a.num_lights;
                // (the records staged in the block's LDS when few; the pick reads them there)
                const DLight* const lt = (a.num_lights < kLdsLights)
                                             ? reinterpret_cast<const DLight*>(lprobe + 4 + kMaxProbeEmitters * 12)
                                             : a.lights;
                for (uint32_t j = 0; j < a.num_lights && ra > 0; ++j) {
                    const float area = lt[j].area;
                    if (ra < area && ra > 0) sel = j;
                    ra -= area;
                }
                L = lt + sel;
                if (L->pad != 0.0f) { need_sc = true; ang = r3; }   // sphere light: phi = 2*3.14159*v
            } else {
                SEC(SEC_COSINE);
            }
            float sn = 0.0f, cs = 0.0f;
            if (need_sc) det_sincos((float)(2 * 3.14159 * (double)ang), &sn, &cs);
            V3 vec;   // the direction before normalisation (light: dd = p1 - pos)
            if (cosb) {
                const float r = sqrtf(r1);
                const float x = r * cs, z = r * sn;
                const float y = sqrtf(__builtin_fmaxf(0.0f, 1.0f - r1));
                const V3 tg = get_tangent(normal);
                const V3 bt = cross(normal, tg);
                vec = normal * y + tg * x + bt * z;
            } else {
                V3 p1;
                if (L->pad != 0.0f) {
                    const float zz = 1.0f - 2.0f * r2;
                    const float rxy = sqrtf(__builtin_fmaxf(0.0f, 1.0f - zz * zz));
                    p1 = v3(L->v0[0], L->v0[1], L->v0[2]) + v3(rxy * cs, rxy * sn, zz) * L->a1[0];
                } else {
                    float lu = r2, lv = r3;
                    if ((double)(lu + lv) > 1.0) {
                        lu = (float)((double)lu + 2 * (0.5 - (double)lu));
                        lv = (float)((double)lv + 2 * (0.5 - (double)lv));
                    }
                    p1 = v3(L->v0[0], L->v0[1], L->v0[2]) + v3(L->a1[0], L->a1[1], L->a1[2]) * lu +
                         v3(L->a2[0], L->a2[1], L->a2[2]) * lv;
                }
                vec = p1 - pos;
            }
            ldir = normalized(vec);
            float f = (float)3.14159;
            if (!cosb) {
                const float cos_l = __builtin_fmaxf(0.0f, dot(ldir, normal));
                const float cos_o = __builtin_fmaxf(0.0f, dot(v3(0, -1, 0), ldir * -1));
                f = cos_l * cos_o / dot(vec, vec);   // G
                i = (i > D - 2) ? i : D - 2;
            }
            C3 bw = cmulf(cmulf(m_alb, (float)(1 / 3.14159)), f);   // brdf (kernel.cu:101-104) * f
            if (!cosb) bw = cmulf(bw, fresh(a.total_light_area));
            wgt = cmul(wgt, bw);
            ro = pos;
            rd = ldir;
            ++i;
        }
        // advance to the next trace this lane needs
        for (;;) {
            if (i >= D) {
                wave_count(lcnt + 2, lane);
                SEC(SEC_SAMPLE_END);
                // cells 7 (pixel, memo) and 8 (pinhole direction) with the accumulator and mean: the
                // next sample's start needs no fetch of its own
                const uint4 c7 = R.ld4(CW_PX), c8 = R.ld4(CW_CD);
                const uint32_t px = c7.x, py = c7.y;
                // acc and the running mean: cells 4..6 = acc.r, acc.g | acc.b, m0 | m1, m2
                uint4 a01 = make_uint4(0u, 0u, 0u, 0u);
                if (!(fl & CF_ACC0)) a01 = R.ld4(CW_ACC);
                const uint4 a2m0 = R.ld4(CW_ACC + 4);   // (acc.b, only when !CF_ACC0) and m0
                const C3 acc = (fl & CF_ACC0) ? c3(0.0, 0.0, 0.0)
                                              : c3(dbl(a01.x, a01.y), dbl(a01.z, a01.w), dbl(a2m0.x, a2m0.y));
                if (!(fl & CF_SPLIT) || (fl & CF_CHUNK0)) {
                    const uint4 m12 = R.ld4(CW_M + 2);
                    const double fn1 = (double)(float)(n - 1), fn = (double)(float)n;   // kernel.cu:551-552
                    const double x0 = dbl(a2m0.z, a2m0.w) * fn1, x1 = dbl(m12.x, m12.y) * fn1,
                                 x2 = dbl(m12.z, m12.w) * fn1;
                    double m0, m1, m2;
                    // the six quotients by fn: one IEEE reciprocal + Markstein corrections (RN(x/fn)
                    // for finite x clear of under/overflow -- else the whole wave divides)
                    if (__ballot(!(quot_ok(x0) && quot_ok(x1) && quot_ok(x2) && quot_ok(acc.r) && quot_ok(acc.g) &&
                                   quot_ok(acc.b))) == 0ull) {
                        const double rf = 1.0 / fn;
                        m0 = div_mk_d(x0, fn, rf) + div_mk_d(acc.r, fn, rf);
                        m1 = div_mk_d(x1, fn, rf) + div_mk_d(acc.g, fn, rf);
                        m2 = div_mk_d(x2, fn, rf) + div_mk_d(acc.b, fn, rf);
                    } else {
                        m0 = x0 / fn + acc.r / fn;
                        m1 = x1 / fn + acc.g / fn;
                        m2 = x2 / fn + acc.b / fn;
                    }
                    if ((uint32_t)n >= nend) {   // (a whole pixel's unit ends at spp)
                        if (fl & CF_CHUNK0) {
                            double* P = a.lbuf + (size_t)c8.w * 3;
                            P[0] = m0; P[1] = m1; P[2] = m2;
                        } else {
                            float* o3 = a.out + out_pixel(a, px, py) * 3;
                            o3[0] = (float)m0;
                            o3[1] = (float)m1;
                            o3[2] = (float)m2;
                        }
                        state = ST_IDLE;
                        break;
                    }
                    R.std_(CW_M, m0); R.st4(CW_M + 2, dlo(m1), dhi(m1), dlo(m2), dhi(m2));
                } else {
                    // split pixel: keep L_n, finalize_pixels forms the ordered mean
                    // (the slot is cell 8's last word, fetched with this sample's end: no dependent fetch
                    // before the stores)
                    double* L = a.lbuf + ((size_t)(uint32_t)(n - 1) * a.ntail + c8.w) * 3;
                    L[0] = acc.r;
                    L[1] = acc.g;
                    L[2] = acc.b;
                    if ((uint32_t)n >= nend) {
                        state = ST_IDLE;
                        break;
                    }
                }
                ++n;
                again = start_sample(px, py, true, c7, c8);
                break;
            }
            // Last-bounce light probe.  The hit of bounce D-1 only decides the emission it adds
            // (weight * Le if its material has emission.r != 0, kernel.cu:453); its position, normal
            // and next direction are never used, and the draws that follow do not depend on it (u,
            // then 2 or 3).  a.emis holds every triangle whose material has emission.r != 0 (the
            // integrator's own test, not the caller's light list); each is tested exactly (the
            // walk's triIntersect bits):
            //  * no hit with 0 < t < MAX_FLOAT: the reference's winner is not emissive (or there is
            //    none), so the bounce adds 0 -- the path is dead: replay its draws, no trace at all;
            //  * otherwise the winner has t <= t_min (the emitter at t_min is a triangle the reference
            //    may test; if it does not, the final winner check sends the ray to the exact slow
            //    walk), so the walk starts with its bound at t_min instead of MAX_FLOAT.
            float bound = kMaxFloat;
            const uint32_t nem = lprobe[0];   // (the emitters are staged in the block's LDS)
            if (i == D - 1 && nem != 0u && !(a.flags & PT_FLAG_NO_DEAD_PATH_SKIP) && !czero(wgt) &&
                a.scene_fast != 0u && ray_fast(ro, rd)) {
                SEC(SEC_PROBE);
                float bt = kMaxFloat;
                const float4* er = reinterpret_cast<const float4*>(lprobe + 4);
                for (uint32_t k = 0; k < nem; ++k, er += 3) {
                    const float t = tri_hit_pk(f2{ro.x, ro.y}, ro.z, f2{rd.x, rd.y}, rd.z, er[0], er[1], er[2].x);
                    if (0.0f < t && t < bt) bt = t;
                }
                if (bt == kMaxFloat) wgt = c3(0.0, 0.0, 0.0);   // adds nothing: dead from here
                else bound = __uint_as_float(__float_as_uint(bt) + 1u);   // the next float above t_min
            }
            if (!(a.flags & PT_FLAG_NO_DEAD_PATH_SKIP) && czero(wgt)) {   // dead path: replay the draws
                wave_count(lcnt + 1, lane);
                SEC(SEC_DEAD);
                const float u = rng_uniform(rng);
                if (u < 0.5) { rng_next(rng); rng_next(rng); }
                else { rng_next(rng); rng_next(rng); rng_next(rng); i = (i > D - 2) ? i : D - 2; }
                ++i;
                continue;
            }
            wave_count(lcnt + 1, lane);
            again = begin_trace(ro, rd, bound);
            break;
        }
      }
      if (iters != 0u) {
          if (__ballot(again) == 0ull) break;
          continue;
      }
    // refill: lanes whose unit is finished take the next units of this shard
    uint64_t idle = __ballot(state == ST_IDLE);
    if (idle) {
        SEC(SEC_REFILL);
        uint32_t u = kNoUnit;
        if (a.unit_queues > 1u) {
            // The units dealt from kQueues counters (one 128-B line each), counter x owning the blocks
            // j = x (mod kQueues) of kQueueBlock units in order -- so the unit sequence is still taken
            // roughly front to back -- each wave starting at its block's counter and moving on when
            // that one is exhausted (the block's LDS mask, so every wave of the block and every lane
            // sees the same): the refill's atomics spread over kQueues addresses.  Which units a lane
            // gets never changes what it computes.
            uint32_t qdone = *reinterpret_cast<volatile const uint32_t*>(lprobe + 1);
            const uint32_t x0 = blockIdx.x & (kQueues - 1u);
            for (uint32_t r = 0; r < kQueues && idle && qdone != (1u << kQueues) - 1u; ++r) {
                const uint32_t x = (x0 + r) & (kQueues - 1u);
                if (qdone & (1u << x)) continue;
                const int leader = __ffsll((long long)idle) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(a.pixel_counter + kQueueStride * (x + 1u), (uint32_t)__popcll(idle));
                base = __shfl(base, leader, 64);
                if (state == ST_IDLE && u == kNoUnit) {
                    const uint32_t k = base + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                    const uint64_t uq = ((uint64_t)(k / kQueueBlock) * kQueues + x) * kQueueBlock + (k % kQueueBlock);
                    if (uq < a.nunits) u = (uint32_t)uq;
                }
                const uint64_t left = __ballot(state == ST_IDLE && u == kNoUnit);
                if (left) {   // (a counter only grows: past its class's end for good)
                    qdone |= 1u << x;
                    if (lane == leader) atomicOr(const_cast<uint32_t*>(lprobe + 1), 1u << x);
                }
                idle = left;
            }
            if (state == ST_IDLE && u == kNoUnit) u = a.nunits;   // every counter exhausted
        } else {
            const uint32_t need = (uint32_t)__popcll(idle);
            const int leader = __ffsll((long long)idle) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(a.pixel_counter, need);
            base = __shfl(base, leader, 64);
            if (state == ST_IDLE) u = base + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
        }
        if (state == ST_IDLE) {
            if (u >= a.nunits) {
                if (kCount) {   // queue drained; this lane's end after it and since the start (binned at the end)
                    const unsigned long long now = wall_clock64();
                    atomicMin(a.counters + 21, now);
                    const unsigned long long d0 = __hip_atomic_load(a.counters + 21, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long s0 = __hip_atomic_load(a.counters + 20, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    done_rel[0] = (uint32_t)min(now - min(now, d0), 0xffffffffull);
                    done_rel[1] = (uint32_t)min(now - min(now, s0), 0xffffffffull);
                }
                if (a.lane_times) a.lane_times[R.voff >> 4] = wall_clock64();
                state = ST_DONE;
            } else {
                // the unit as init_pixel_states prepared it (pixel, sample range, curand_init's
                // state fast-forwarded to the range, the pinhole camera ray)
                const size_t N = a.nunits;
                const uint32_t pxy = a.pix_states[UW_PXY * N + u];
                if (pxy != kNoPixel) {
                    const uint32_t px = pxy & 0xffffu, py = pxy >> 16;
                    const uint32_t n0 = a.pix_states[UW_N0 * N + u];
                    rng.v0 = a.pix_states[u];
                    rng.v1 = a.pix_states[N + u];
                    rng.v2 = a.pix_states[2 * N + u];
                    rng.v3 = a.pix_states[3 * N + u];
                    rng.v4 = a.pix_states[4 * N + u];
                    rng.d = a.pix_states[5 * N + u];
                    nend = a.pix_states[UW_NEND * N + u];
                    n = (int)(n0 & 0x7fffffffu);
                    const bool split = u >= a.nwhole;
                    fl = (n0 >> 31) ? CF_LENS : CF_CAMC;
                    uint4 c8 = make_uint4(0u, 0u, 0u, 0u);
                    if (!(fl & CF_LENS)) {
                        c8 = make_uint4(a.pix_states[UW_CD * N + u], a.pix_states[(UW_CD + 1) * N + u],
                                        a.pix_states[(UW_CD + 2) * N + u], a.pix_states[UW_TQ * N + u]);
                        R.st4(CW_CD, c8.x, c8.y, c8.z, c8.w);
                    }
                    if (split) fl |= (n == 1) ? CF_SPLIT | CF_CHUNK0 : CF_SPLIT;
#ifdef PT_DEBUG_CHECKS
                    // finalize_pixels continues a CF_CHUNK0 slot's mean from sample chunk_first(1): the unit must end there
                    if (split && n == 1 && nend != chunk_first(a, 1u, slot_chunks(a, a.pix_states[UW_TQ * N + u])))
                        __builtin_trap();
#endif
                    if (split && !(fl & CF_LENS) && !(a.flags & PT_FLAG_NO_PRIMARY_CACHE))
                        fl |= (n == 1) ? CF_OWNER : CF_SHARE;   // (chunk 0 starts at sample 1)
                    R.st2(CW_PX, px, py);
                    if (split && (fl & CF_LENS)) R.st(CW_Q, a.pix_states[UW_TQ * N + u]);
                    R.st2(CW_M, 0u, 0u); R.st4(CW_M + 2, 0u, 0u, 0u, 0u);
                    // (a new unit: no memo yet; its pinhole direction and slot are in c8 -- a lens
                    // unit reads neither, and its slot from the record)
                    again = start_sample(px, py, !(fl & CF_LENS), make_uint4(0u, 0u, 0u, 0u), c8);
                }
            }
        }
    }
      if (__ballot(again) == 0ull) break;
    }

    // the first visits of every ray begun in this pass (the root and, while the next node is staged
    // in LDS and no leaf is queued, up to root_first - 1 more), here -- all such lanes together, one
    // copy of the code -- instead of as walk steps: the walk is that many steps shorter per ray.  (A
    // fresh walk is the only one at node 0.)  Nothing entered: the walk is over without a candidate,
    // as a finished walk would be; the lane shades in the next pass.
    if (a.root_first && state == ST_TRACE && w.node == 0u) {
        bool more = walk4_root<kCount>(w, S, kCullRel, a.node_mask, cnt);
        // (up to root_first visits: the next node too while it is staged in LDS and no leaf is queued)
        for (uint32_t k = 1; more && k < a.root_first && w.node < S.ntop && !leaf4_pending(w); ++k)
            more = walk4_root<kCount>(w, S, kCullRel, a.node_mask, cnt);
        if (!more) state = (w.best_t == kMaxFloat) ? ST_SHADE : ST_SLOW;
    }
    SEC(SEC_RECORD);
    R.st4(CW_N, (uint32_t)n, (uint32_t)i, fl, rng.d);
    R.st4(CW_RNG_V0, rng.v0, rng.v1, rng.v2, rng.v3);
    R.st4(CW_WGT, dlo(wgt.r), dhi(wgt.r), dlo(wgt.g), dhi(wgt.g));
    R.st4(CW_WGT + 4, dlo(wgt.b), dhi(wgt.b), rng.v4, nend);
}


// The refill's unit dealing (as in shade_lane): lanes `idle` of the wave take the next units of this
// shard from the unit counters; returns this lane's unit (`me`: this lane is idle), a.nunits once
// every counter is exhausted.
template <bool kCount>
__device__ __forceinline__ uint32_t take_unit(const Args& a, int lane, uint64_t idle, bool me, const uint32_t* lprobe,
                                              uint32_t* done_rel)
{
    uint32_t u = kNoUnit;
    if (a.unit_queues > 1u) {
        uint32_t qdone = *reinterpret_cast<volatile const uint32_t*>(lprobe + 1);
        const uint32_t x0 = blockIdx.x & (kQueues - 1u);
        for (uint32_t r = 0; r < kQueues && idle && qdone != (1u << kQueues) - 1u; ++r) {
            const uint32_t x = (x0 + r) & (kQueues - 1u);
            if (qdone & (1u << x)) continue;
            const int leader = __ffsll((long long)idle) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(a.pixel_counter + kQueueStride * (x + 1u), (uint32_t)__popcll(idle));
            base = __shfl(base, leader, 64);
            if (me && u == kNoUnit) {
                const uint32_t k = base + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                const uint64_t uq = ((uint64_t)(k / kQueueBlock) * kQueues + x) * kQueueBlock + (k % kQueueBlock);
                if (uq < a.nunits) u = (uint32_t)uq;
            }
            const uint64_t left = __ballot(me && u == kNoUnit);
            if (left) {
                qdone |= 1u << x;
                if (lane == leader) atomicOr(const_cast<uint32_t*>(lprobe + 1), 1u << x);
            }
            idle = left;
        }
        if (me && u == kNoUnit) u = a.nunits;
    } else {
        const uint32_t need = (uint32_t)__popcll(idle);
        const int leader = __ffsll((long long)idle) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(a.pixel_counter, need);
        base = __shfl(base, leader, 64);
        if (me) u = base + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
    }
    if (kCount && me && u >= a.nunits) {   // queue drained; this lane's end after it and since the start
        const unsigned long long now = wall_clock64();
        atomicMin(a.counters + 21, now);
        const unsigned long long d0 = __hip_atomic_load(a.counters + 21, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long s0 = __hip_atomic_load(a.counters + 20, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done_rel[0] = (uint32_t)min(now - min(now, d0), 0xffffffffull);
        done_rel[1] = (uint32_t)min(now - min(now, s0), 0xffffffffull);
    }
    return u;
}
// ------------------------------------------------------------------ wavefront kernel, integrator 1
// radianceAlongSingleStep (kernel.cu:217-415) on the same state machine.  A sample is a fixed data
// flow of traces: T1 the light subpath's bounce from the area-sampled light vertex x0 (kernel.cu:263-
// 287), T2 the camera ray (the pixel's memo when the camera has no lens, :289-305), T3 the camera's
// cosine bounce (:306-350), then one visibility ray x_i -> x_j for each connection (i in {0,1}, j in
// {2,3}, :353-412) whose weight exceeds 0.01.  None of its XORWOW draws depends on a trace (lens 2,
// light pick 3, rand_ray 2, cosine 2), so all of them are drawn when the sample starts.  The record
// keeps the path vertices; the connection weights are recomputed from them in the sample's last pass,
// in the reference's order, with the visibility bits the shadow walks left (the weights' arithmetic
// is identical both times, so the set of connections that trace cannot differ).
// Cells are grouped by the pass that reads them, so that a pass touches few cells (a wave's access to
// one word of a cell spans the same 1 KiB as the whole cell): every pass reads cell 0 only, the
// sample's last pass cells 10-12.
enum : int {
    HW_N = 0, HW_SF, HW_RNG_D, HW_CU1,        // cell 0: sample, stage | flags << 16, XORWOW d, the pending
                                              //         visibility ray's length
    HW_RNG_V0 = 4,                            // cell 1: v0..v3
    HW_RNG_V4 = 8, HW_NEND, HW_DU1, HW_DU2,   // cell 2: v4, unit end, the cosine draws of T3
    HW_X0 = 12, HW_MAT0 = 15,                 // cell 3: light vertex x0 (offset along its normal), material
    HW_N0 = 16, HW_IP1 = 19,                  // cell 4: its normal, ip[1]
    HW_X1 = 20, HW_MAT1 = 23,                 // cell 5: light bounce hit x1, material
    HW_N1 = 24,                               // cell 6: its normal
    HW_X3 = 28, HW_MAT3 = 31,                 // cell 7: camera hit x3, material
    HW_N3 = 32,                               // cell 8: its normal
    HW_X2 = 36,                               // cell 9: camera bounce hit x2
    HW_GC = 40,                               // cell 10: G of the four connections (written with T3's end)
    HW_FA = 44,                               // cell 11: G1, G3, ip[1], ip[2] (T3's end)
    HW_FB = 48,                               // cell 12: the four materials (T3's end)
    HW_M = 52,                                // cells 13, 14.lo: running mean m0..m2 (f64)
    HW_PXY = 60, HW_Q, HW_MTRI, HW_MT,        // cell 15: pixel (x | y << 16), split slot, primary memo (tri, t)
    HW_CD = 64,                               // cell 16: camera direction (pinhole: the unit's; lens: the sample's)
    HW_CO = 68,                               // cell 17: camera origin of a lens sample
    kHeadWords = 72
};
// stage word: bits 0-1 the pending trace, 2-3 the connection whose visibility ray it is (k = 2i + j-2),
// 4-7 visibility bits, 8-11 the connections that need a ray
enum : uint32_t { HS_T1 = 0, HS_T2 = 1, HS_T3 = 2, HS_SH = 3 };
constexpr int kHeadLdsLightBytes = (int)kLdsLights * 16;   // per staged light: its normal and material

// The geometric factors of one HEAD sample's connections (kernel.cu:353-412): G1 = geo_term of the
// light subpath edge x1-x0, G3 = of the camera edge x3-x2, Gc[k] = the connection term of (i, j),
// k = 2i + j-2 -- the float parts of the weights, computed once from the vertices (x[4], nrm[4] as
// radianceAlongSingleStep holds them); the f64 chain (head_weights) needs only these.
struct HeadGeo {
    float G1, G3, Gc[4];
};
__device__ __forceinline__ void head_geometry(const V3 (&x)[4], const V3 (&nrm)[4], HeadGeo& g)
{
    g.G1 = geo_term(x[1], x[0], nrm[1], nrm[0]);
    g.G3 = geo_term(x[3], x[2], nrm[3], nrm[2]);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 2; j < 4; ++j) {
            const V3 seg = x[j] - x[i];
            const V3 ray = normalized(seg);
            float G = __builtin_fmaxf(0.0f, dot(ray, nrm[j]) * dot(ray * -1, nrm[i])) / dot(seg, seg);
            if (G != G) G = 0;
            g.Gc[2 * i + (j - 2)] = G;
        }
    }
}
// The four connections' weights in the reference's order and arithmetic: w = le*ip0, times
// (albedo_k/pi, G, ip_k) for k = 1..i and k = j+1..3, times (albedo_j/pi, Gc, ip_j); a connection whose
// weight max exceeds 0.01 traces (its bit in *need) and counts only if visible (bit in vis); the
// radiance adds w*V and the camera hit's emission per connection.  mat[4] and ip[0..2] as the
// reference's arrays (ip[3] = 1).
__device__ __forceinline__ C3 head_weights(const Args& a, const int32_t (&mat)[4], const float (&ip)[3], const HeadGeo& g,
                                           uint32_t vis, uint32_t* need)
{
    const C3 le = mat_emission(a.mats + mat[0]);
    const C3 e3 = mat_emission(a.mats + mat[3]);
    const C3 A1 = cdivf(mat_albedo(a.mats + mat[1]), 3.14159f);
    const C3 A2 = cdivf(mat_albedo(a.mats + mat[2]), 3.14159f);
    const C3 A3 = cdivf(mat_albedo(a.mats + mat[3]), 3.14159f);
    C3 accum = c3(0, 0, 0);
    uint32_t nd = 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 2; j < 4; ++j) {
            C3 w = cmulf(le, ip[0]);
            if (i == 1) w = cmulf(cmulf(cmul(w, A1), g.G1), ip[1]);      // k = 1
            if (j == 2) w = cmulf(cmulf(cmul(w, A3), g.G3), 1.0f);       // k = 3 (ip[3] = 1)
            const int k = 2 * i + (j - 2);
            w = cmulf(cmulf(cmul(w, (j == 2) ? A2 : A3), g.Gc[k]), (j == 2) ? ip[2] : 1.0f);
            const float m = (float)fmax(w.r, fmax(w.g, w.b));
            float V = 0;
            if ((double)m > 0.01) {
                nd |= 1u << k;
                if (vis & (1u << k)) V = 1;
            }
            w = cmulf(w, V);
            accum = cadd(accum, w);
            accum = cadd(accum, e3);
        }
    }
    if (need) *need = nd;
    return accum;
}

__device__ __forceinline__ V3 u3f(uint4 q) { return v3(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z)); }

// The visibility ray of connection k (kernel.cu:397-405: from x_i along normalized(x_j - x_i); visible
// iff the hit's |t - len| <= 0.01) -- the expressions of head_connections, so the same bits.
__device__ __forceinline__ void head_vis_ray(V3 xi, V3 xj, V3* ro, V3* rd, float* len)
{
    const V3 seg = xj - xi;
    *len = length(seg);
    *ro = xi;
    *rd = normalized(seg);
}
// A visibility walk only needs hits up to len + 0.01: every t >= RN(len + 0.02) has |t - len| > 0.016
// (len < MAX_FLOAT, so ulp(len) <= 2^-7), so the walk is bounded there and finding no hit below the
// bound means "not visible" -- exactly as the reference's closest hit, wherever it lies beyond, does.
__device__ __forceinline__ float head_vis_bound(float len)
{
    const float b = len + 0.02f;
    return (b < kMaxFloat) ? b : kMaxFloat;
}
// ... and any hit with t <= RN(len - 0.03) decides "not visible" at once: then len - t >= 0.026 (exact, or
// far larger), so |t - len| > 0.01 for it and for the closest hit, which is no farther (the walk stops
// there; the winner check still confirms it is a triangle the reference tests).
__device__ __forceinline__ float head_vis_occluded(float len)
{
    return (len > 0.04f) ? len - 0.03f : -1.0f;
}

template <bool kCount>
__device__ __forceinline__ void shade_lane_head(const ColdRec& R, int lane, uint32_t& state, V3& ro, V3& rd,
                                                int32_t& htri, float& ht, W4& w, const Stack4& S,
                                                unsigned long long* lcnt, const uint32_t* lprobe, uint32_t* done_rel,
                                                Counters& cnt)
{
    const Args& a = kernel_args_opaque();
    SEC(SEC_PASS);
    // (the XORWOW words v0..v3 are read and written only where a sample starts -- the only place a
    // sample draws -- so they are not live across the pass: the shading code then fits 96 VGPRs)
    const uint4 k0 = R.ld4(HW_N);
    if (state == ST_CHECK) {
        SEC(SEC_CHECK);
        const float4* hr = a.hrec + 3 * (size_t)(uint32_t)htri;
        const float4 b0 = hr[0], b1 = hr[1];
        htri = (int32_t)__float_as_uint(b1.w);
        state = ref_tested_box(b0, b1, __float_as_uint(b1.z), ro, rd, a.rnodes, a.rparent) ? ST_SHADE : ST_SLOW;
    }
    int n = (int)k0.x;
    uint32_t stage = k0.y & 0xffffu, fl = k0.y >> 16;
    Rng rng;
    rng.d = k0.z;
    // (likewise v4, the unit end and the cosine draws: each read where it is used, written where it
    // changes; only cell 0 -- n, stage, flags, XORWOW d -- is live across the pass)
    float cu1 = __uint_as_float(k0.w);   // the pending visibility ray's length (its check below)
    // (the staged light records and, behind them, each one's normal and material)
    const DLight* const llt = reinterpret_cast<const DLight*>(lprobe + 4 + kMaxProbeEmitters * 12);
    const float4* const lnm = reinterpret_cast<const float4*>(lprobe + 4 + kMaxProbeEmitters * 12 + kLdsLights * 12);

    // begin a trace of (ro, rd) below `bound`; true = the lane continues shading at once (no triangles, a
    // root miss -- the hit is a miss --, or a ray outside the Markstein preconditions: the exact slow walk)
    auto begin_trace = [&](float bound, float occ) -> bool {
        wave_count(lcnt + 0, lane);
        SEC(SEC_BEGIN);
        if (a.num_tris == 0) { htri = -1; ht = kMaxFloat; state = ST_SHADE; return true; }
        if (!((a.scene_fast != 0u) && ray_fast(ro, rd))) { state = ST_SLOW; return true; }
        if (!walk4_begin(w, ro, rd, a.acc_root, a.cull_abs)) { htri = -1; ht = kMaxFloat; state = ST_SHADE; return true; }
        w.best_t = bound;
        w.occ = occ;
        state = ST_TRACE;
        return false;
    };
    // a hit is at hand (after a walk, the slow walk or the memo): spheres, primary memo bookkeeping
    auto take_hit = [&]() {
        if (a.num_spheres && !(fl & CF_MEMO)) apply_spheres(a, ro, rd, &htri, &ht);
        fl &= ~CF_MEMO;
        if (fl & CF_PRIMARY) {
            fl = (fl | CF_HAVE) & ~CF_PRIMARY;
            R.st2(HW_MTRI, (uint32_t)htri, __float_as_uint(ht));
            if (fl & CF_OWNER) {
                const uint32_t q = R.ld(HW_Q);
                __hip_atomic_store(reinterpret_cast<uint64_t*>(a.pmemo) + q,
                                   ((uint64_t)__float_as_uint(ht) << 32) | (uint32_t)(htri + 2), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                fl &= ~CF_OWNER;
            }
        }
    };
    // start sample n: all of its draws, the light vertex, the camera ray of a lens sample; trace T1
    auto start_sample = [&](uint32_t px, uint32_t py, bool have_rng) -> bool {
        SEC(SEC_START);
        if (!have_rng) {
            const uint4 k1 = R.ld4(HW_RNG_V0);
            rng.v0 = k1.x; rng.v1 = k1.y; rng.v2 = k1.z; rng.v3 = k1.w;
            rng.v4 = R.ld(HW_RNG_V4);
        }
        const bool lens = (fl & CF_LENS) != 0u;
        float lu1 = 0.0f, lu2 = 0.0f;
        if (lens) { lu1 = rng_uniform(rng); lu2 = rng_uniform(rng); }   // drawPixel's cameraRay (kernel.cu:547)
        // light vertex: the area-CDF pick + uniform point (pick_light, kernel.cu:231-262)
        float ra = a.total_light_area * rng_uniform(rng);
        uint32_t sel = a.num_lights;
        const bool staged = a.num_lights < kLdsLights;
        const DLight* const lt = staged ? llt : a.lights;
        for (uint32_t j = 0; j < a.num_lights && ra > 0; ++j) {
            const float area = lt[j].area;
            if (ra < area && ra > 0) sel = j;
            ra -= area;
        }
        float u = rng_uniform(rng);
        float v = rng_uniform(rng);
        const DLight* L = lt + sel;
        V3 p, n0;
        int32_t m0;
        if (L->pad != 0.0f) {   // sphere light (d8)
            const float z = 1.0f - 2.0f * u;
            const float rxy = sqrtf(__builtin_fmaxf(0.0f, 1.0f - z * z));
            const float phi = (float)(2 * 3.14159 * (double)v);
            float si, co;
            det_sincos(phi, &si, &co);
            p = v3(L->v0[0], L->v0[1], L->v0[2]) + v3(rxy * co, rxy * si, z) * L->a1[0];
            n0 = prim_normal(a, L->tri, p);
            m0 = prim_mat(a, L->tri);
        } else {
            if ((double)(u + v) > 1.0) {
                u = (float)((double)u + 2 * (0.5 - (double)u));
                v = (float)((double)v + 2 * (0.5 - (double)v));
            }
            p = v3(L->v0[0], L->v0[1], L->v0[2]) + v3(L->a1[0], L->a1[1], L->a1[2]) * u + v3(L->a2[0], L->a2[1], L->a2[2]) * v;
            if (staged) {
                const float4 q = lnm[sel];
                n0 = v3(q.x, q.y, q.z);
                m0 = (int32_t)__float_as_uint(q.w);
            } else {
                n0 = ld_norm(a.shade, L->tri);
                m0 = ld_mat(a.shade, L->tri);
            }
        }
        ro = p + n0 * 0.001f;                 // x[0] (kernel.cu:259)
        rd = rand_ray(n0, rng);               // the light bounce (kernel.cu:264)
        const float du1 = rng_uniform(rng);   // cosine_ray's draws for T3 (kernel.cu:307)
        const float du2 = rng_uniform(rng);
        R.st(HW_RNG_V4, rng.v4);
        R.st2(HW_DU1, __float_as_uint(du1), __float_as_uint(du2));
        R.st4(HW_RNG_V0, rng.v0, rng.v1, rng.v2, rng.v3);
        R.st4(HW_X0, __float_as_uint(ro.x), __float_as_uint(ro.y), __float_as_uint(ro.z), (uint32_t)m0);
        R.st4(HW_N0, __float_as_uint(n0.x), __float_as_uint(n0.y), __float_as_uint(n0.z), 0u);
        if (lens) {   // this sample's camera ray (its draws came first)
            V3 co, cd;
            camera_ray(a.cam, px, py, true, lu1, lu2, &co, &cd);
            R.st4(HW_CD, __float_as_uint(cd.x), __float_as_uint(cd.y), __float_as_uint(cd.z), 0u);
            R.st4(HW_CO, __float_as_uint(co.x), __float_as_uint(co.y), __float_as_uint(co.z), 0u);
        }
        stage = HS_T1;
        wave_count(lcnt + 1, lane);
        return begin_trace(kMaxFloat, -1.0f);
    };
    // T2: the camera ray -- the memo of a pinhole pixel, or a trace
    auto camera_stage = [&]() -> bool {
        stage = HS_T2;
        wave_count(lcnt + 1, lane);
        const uint4 cd = R.ld4(HW_CD);
        rd = v3(__uint_as_float(cd.x), __uint_as_float(cd.y), __uint_as_float(cd.z));
        const bool lens = (fl & CF_LENS) != 0u;
        if (lens) {
            const uint4 co = R.ld4(HW_CO);
            ro = v3(__uint_as_float(co.x), __uint_as_float(co.y), __uint_as_float(co.z));
        } else {
            ro = v3(0.0f, 0.0f, 0.0f) + v3(fresh(a.cam.pos[0]), fresh(a.cam.pos[1]), fresh(a.cam.pos[2]));
        }
        if (fl & CF_HAVE) {
            SEC(SEC_MEMO);
            const uint2 mm = R.ld2(HW_MTRI);
            htri = (int32_t)mm.x; ht = __uint_as_float(mm.y);
            fl = (fl & ~CF_PRIMARY) | CF_MEMO; state = ST_SHADE;
            return true;
        }
        if (fl & CF_SHARE) {
            const uint32_t q = R.ld(HW_Q);
            const uint64_t mv = __hip_atomic_load(reinterpret_cast<uint64_t*>(a.pmemo) + q, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)mv != 0u) {
                htri = (int32_t)((uint32_t)mv - 2u);
                ht = __uint_as_float((uint32_t)(mv >> 32));
                fl = (fl | CF_PRIMARY | CF_MEMO) & ~CF_SHARE;
                state = ST_SHADE;
                return true;
            }
        }
        fl = (!(a.flags & PT_FLAG_NO_PRIMARY_CACHE) && !lens) ? (fl | CF_PRIMARY) : (fl & ~CF_PRIMARY);
        return begin_trace(kMaxFloat, -1.0f);
    };
    // begin the visibility ray of connection k
    auto vis_stage = [&](uint32_t k, V3 xi, V3 xj) -> bool {
        float len;
        head_vis_ray(xi, xj, &ro, &rd, &len);
        cu1 = len;   // (stored with cell 0 at the pass's end; its walk may end in this pass: a root miss)
        stage = (stage & ~0xfu) | HS_SH | (k << 2);
        wave_count(lcnt + 1, lane);
        return begin_trace(head_vis_bound(len), head_vis_occluded(len));
    };
    auto ldv = [&](int k) -> V3 { return u3f(R.ld4(k)); };
    bool again = (state == ST_SHADE || state == ST_SLOW);
    for (uint32_t iters = 0; iters < a.wf_iters; ++iters) {
      if (again) {
        again = false;
        if (state == ST_SLOW) {
            wave_count(lcnt + 3, lane);
            SEC(SEC_SLOW);
            trace_slow(ro, rd, a.root, a.nodes, a.tris_leaf, S.spill(), S.stride, a.cull_rel, a.cull_abs,
                       &htri, &ht, kCount ? a.tri_counts : nullptr);
        }
        state = ST_SHADE;
        take_hit();
        for (;;) {   // consume the hit; advance until the lane needs a trace or its unit is done
            SEC(SEC_BOUNCE);
            bool sample_done = false;
            C3 acc = c3(0, 0, 0);
            if ((stage & 3u) == HS_T1) {
                // light bounce hit x[1] (kernel.cu:266-287)
                int32_t tri = htri;
                float t = (float)((double)ht - 0.001);
                if (t > kMaxFloat - 1) { tri = 0; t = 0; }
                const V3 pos = ro + rd * t;
                const V3 n2 = prim_normal(a, tri, pos);
                const float G = __builtin_fabsf(dot(n2, rd)) / __builtin_fmaxf(0.001f, t * t);
                const float ip1 = (float)(2 * 3.14159 / (double)G);
                R.st4(HW_X1, __float_as_uint(pos.x), __float_as_uint(pos.y), __float_as_uint(pos.z), (uint32_t)prim_mat(a, tri));
                R.st(HW_IP1, __float_as_uint(ip1));
                R.st4(HW_N1, __float_as_uint(n2.x), __float_as_uint(n2.y), __float_as_uint(n2.z), 0u);
                if (camera_stage()) {
                    if (state == ST_SLOW) { again = true; break; }
                    take_hit();
                    continue;   // the camera hit is at hand (memo or a root miss)
                }
                break;
            } else if ((stage & 3u) == HS_T2) {
                // camera hit x[3] (kernel.cu:289-305)
                int32_t tri = htri;
                float t = (float)((double)ht - 0.001);
                if (t > kMaxFloat - 1) { tri = 0; t = 0; }
                const V3 x3 = ro + rd * t;
                const V3 n3 = prim_normal(a, tri, x3);
                R.st4(HW_X3, __float_as_uint(x3.x), __float_as_uint(x3.y), __float_as_uint(x3.z), (uint32_t)prim_mat(a, tri));
                R.st4(HW_N3, __float_as_uint(n3.x), __float_as_uint(n3.y), __float_as_uint(n3.z), 0u);
                // the camera bounce: cosine_ray (kernel.cu:78-99) with the draws taken at the start
                SEC(SEC_COSINE);
                const uint2 cc = R.ld2(HW_DU1);
                const float du1 = __uint_as_float(cc.x), du2 = __uint_as_float(cc.y);
                const float r = sqrtf(du1);
                const float theta = (float)(2 * 3.14159 * (double)du2);
                float sn, cs;
                det_sincos(theta, &sn, &cs);
                const float y = sqrtf(__builtin_fmaxf(0.0f, 1.0f - du1));
                ro = x3;
                rd = to_frame(n3, r * cs, y, r * sn);
                stage = HS_T3;
                wave_count(lcnt + 1, lane);
                if (begin_trace(kMaxFloat, -1.0f)) {
                    if (state == ST_SLOW) { again = true; break; }
                    take_hit();
                    continue;
                }
                break;
            } else if ((stage & 3u) == HS_T3) {
                // camera bounce hit x[2] (kernel.cu:324-350; decision d2: a miss is triangle 0, t 0)
                int32_t tri = htri;
                float t = (float)((double)ht - 0.001);
                if (t > kMaxFloat - 1 || tri < 0) { tri = 0; t = 0; }
                const uint4 c3v = R.ld4(HW_X0), c4 = R.ld4(HW_N0), c5 = R.ld4(HW_X1), c6 = R.ld4(HW_N1),
                            c7 = R.ld4(HW_X3), c8 = R.ld4(HW_N3);
                V3 x[4], nrm[4];
                x[0] = u3f(c3v); nrm[0] = u3f(c4); x[1] = u3f(c5); nrm[1] = u3f(c6); x[3] = u3f(c7); nrm[3] = u3f(c8);
                x[2] = ro + rd * t;
                nrm[2] = prim_normal(a, tri, x[2]);
                float G = __builtin_fabsf(dot(nrm[3], rd) * dot(nrm[2], rd)) / (t * t);
                if (G == 0) G = 1;
                if (G != G) G = 1;
                const int32_t mat[4] = {(int32_t)c3v.w, (int32_t)c5.w, prim_mat(a, tri), (int32_t)c7.w};
                const float ip[3] = {fresh(a.total_light_area), __uint_as_float(c4.w), (float)(3.14159 / (double)G)};
                HeadGeo g;
                head_geometry(x, nrm, g);
                R.st4(HW_X2, __float_as_uint(x[2].x), __float_as_uint(x[2].y), __float_as_uint(x[2].z), 0u);
                R.st4(HW_GC, __float_as_uint(g.Gc[0]), __float_as_uint(g.Gc[1]), __float_as_uint(g.Gc[2]), __float_as_uint(g.Gc[3]));
                R.st4(HW_FA, __float_as_uint(g.G1), __float_as_uint(g.G3), __float_as_uint(ip[1]), __float_as_uint(ip[2]));
                R.st4(HW_FB, (uint32_t)mat[0], (uint32_t)mat[1], (uint32_t)mat[2], (uint32_t)mat[3]);
                uint32_t need = 0;
                acc = head_weights(a, mat, ip, g, 0u, &need);
                if (need == 0u) {
                    sample_done = true;   // no connection needs a visibility ray: acc is the sample's radiance
                } else {
                    stage = (need << 8);
                    const uint32_t k = (uint32_t)__builtin_ctz(need);
                    // (the endpoints re-read from the record: the vertices need not stay live across the weights)
                    asm volatile("" ::: "memory");
                    if (vis_stage(k, ldv((k >> 1) ? HW_X1 : HW_X0), ldv((k & 1u) ? HW_X3 : HW_X2))) {
                        if (state == ST_SLOW) { again = true; break; }
                        take_hit();
                        continue;
                    }
                    break;
                }
            } else {
                // visibility ray of connection k (kernel.cu:397-405)
                const uint32_t k = (stage >> 2) & 3u, need = (stage >> 8) & 15u;
                if ((double)__builtin_fabsf(ht - cu1) <= 0.01) stage |= 1u << (4 + k);
                const uint32_t rest = need & ~((2u << k) - 1u);
                if (rest != 0u) {
                    const uint32_t k2 = (uint32_t)__builtin_ctz(rest);
                    const V3 xi = ldv((k2 >> 1) ? HW_X1 : HW_X0), xj = ldv((k2 & 1u) ? HW_X3 : HW_X2);
                    if (vis_stage(k2, xi, xj)) {
                        if (state == ST_SLOW) { again = true; break; }
                        take_hit();
                        continue;
                    }
                    break;
                }
                // the sample's last pass: the weights again, now with the visibility bits
                HeadGeo g;
                const uint4 gc = R.ld4(HW_GC), fa = R.ld4(HW_FA), fb = R.ld4(HW_FB);

                g.Gc[0] = __uint_as_float(gc.x); g.Gc[1] = __uint_as_float(gc.y); g.Gc[2] = __uint_as_float(gc.z);
                g.Gc[3] = __uint_as_float(gc.w);
                g.G1 = __uint_as_float(fa.x);
                g.G3 = __uint_as_float(fa.y);
                const int32_t mat[4] = {(int32_t)fb.x, (int32_t)fb.y, (int32_t)fb.z, (int32_t)fb.w};
                const float ip[3] = {fresh(a.total_light_area), __uint_as_float(fa.z), __uint_as_float(fa.w)};
                acc = head_weights(a, mat, ip, g, (stage >> 4) & 15u, nullptr);
                sample_done = true;
            }
            if (!sample_done) break;
            // sample n's end: the running mean (kernel.cu:551-552), or the split pixel's per-sample slot
            wave_count(lcnt + 2, lane);
            SEC(SEC_SAMPLE_END);
            const uint4 c13 = R.ld4(HW_PXY);
            // the next sample's XORWOW words and the unit end, fetched with the sample's end
            const uint4 r1 = R.ld4(HW_RNG_V0), r2 = R.ld4(HW_RNG_V4);
            const uint32_t px = c13.x & 0xffffu, py = c13.x >> 16;
            if (!(fl & CF_SPLIT)) {
                const uint4 m01 = R.ld4(HW_M);
                const uint2 m2 = R.ld2(HW_M + 4);
                const double fn1 = (double)(float)(n - 1), fn = (double)(float)n;
                const double x0 = dbl(m01.x, m01.y) * fn1, x1 = dbl(m01.z, m01.w) * fn1, x2 = dbl(m2.x, m2.y) * fn1;
                double m0, mm1, mm2;
                if (__ballot(!(quot_ok(x0) && quot_ok(x1) && quot_ok(x2) && quot_ok(acc.r) && quot_ok(acc.g) &&
                               quot_ok(acc.b))) == 0ull) {
                    const double rf = 1.0 / fn;
                    m0 = div_mk_d(x0, fn, rf) + div_mk_d(acc.r, fn, rf);
                    mm1 = div_mk_d(x1, fn, rf) + div_mk_d(acc.g, fn, rf);
                    mm2 = div_mk_d(x2, fn, rf) + div_mk_d(acc.b, fn, rf);
                } else {
                    m0 = x0 / fn + acc.r / fn;
                    mm1 = x1 / fn + acc.g / fn;
                    mm2 = x2 / fn + acc.b / fn;
                }
                if (n >= a.spp) {
                    float* o3 = a.out + out_pixel(a, px, py) * 3;
                    o3[0] = (float)m0;
                    o3[1] = (float)mm1;
                    o3[2] = (float)mm2;
                    state = ST_IDLE;
                    break;
                }
                R.st4(HW_M, dlo(m0), dhi(m0), dlo(mm1), dhi(mm1));
                R.st2(HW_M + 4, dlo(mm2), dhi(mm2));
            } else {
                double* Lb = a.lbuf + ((size_t)(uint32_t)(n - 1) * a.ntail + c13.y) * 3;
                Lb[0] = acc.r;
                Lb[1] = acc.g;
                Lb[2] = acc.b;
                if ((uint32_t)n >= r2.y) {
                    state = ST_IDLE;
                    break;
                }
            }
            ++n;
            rng.v0 = r1.x; rng.v1 = r1.y; rng.v2 = r1.z; rng.v3 = r1.w; rng.v4 = r2.x;
            again = start_sample(px, py, true);
            break;
        }
      }
      if (iters != 0u) {
          if (__ballot(again) == 0ull) break;
          continue;
      }
      // refill: lanes whose unit is finished take the next units of this shard
      uint64_t idle = __ballot(state == ST_IDLE);
      if (idle) {
          SEC(SEC_REFILL);
          const uint32_t u = take_unit<kCount>(a, lane, idle, state == ST_IDLE, lprobe, done_rel);
          if (state == ST_IDLE) {
              if (u >= a.nunits) {
                  if (a.lane_times) a.lane_times[R.voff >> 4] = wall_clock64();
                  state = ST_DONE;
              } else {
                  const size_t N = a.nunits;
                  const uint32_t pxy = a.pix_states[UW_PXY * N + u];
                  if (pxy != kNoPixel) {
                      const uint32_t n0 = a.pix_states[UW_N0 * N + u];
                      rng.v0 = a.pix_states[u];
                      rng.v1 = a.pix_states[N + u];
                      rng.v2 = a.pix_states[2 * N + u];
                      rng.v3 = a.pix_states[3 * N + u];
                      rng.v4 = a.pix_states[4 * N + u];
                      rng.d = a.pix_states[5 * N + u];
                      R.st(HW_NEND, a.pix_states[UW_NEND * N + u]);
                      n = (int)(n0 & 0x7fffffffu);
                      const bool split = u >= a.nwhole;
                      fl = (n0 >> 31) ? CF_LENS : CF_CAMC;
                      if (!(fl & CF_LENS))
                          R.st4(HW_CD, a.pix_states[UW_CD * N + u], a.pix_states[(UW_CD + 1) * N + u],
                                a.pix_states[(UW_CD + 2) * N + u], 0u);
                      if (split) fl |= CF_SPLIT;
                      if (split && !(fl & CF_LENS) && !(a.flags & PT_FLAG_NO_PRIMARY_CACHE))
                          fl |= (n == 1) ? CF_OWNER : CF_SHARE;
                      R.st4(HW_PXY, pxy, split ? a.pix_states[UW_TQ * N + u] : 0u, 0u, 0u);
                      R.st4(HW_M, 0u, 0u, 0u, 0u); R.st2(HW_M + 4, 0u, 0u);
                      again = start_sample(pxy & 0xffffu, pxy >> 16, true);
                  }
              }
          }
      }
      if (__ballot(again) == 0ull) break;
    }
    if (a.root_first && state == ST_TRACE && w.node == 0u) {
        bool more = walk4_root<kCount>(w, S, kCullRel, a.node_mask, cnt);
        for (uint32_t k = 1; more && k < a.root_first && w.node < S.ntop && !leaf4_pending(w); ++k)
            more = walk4_root<kCount>(w, S, kCullRel, a.node_mask, cnt);
        if (!more) {   // nothing below the bound: a miss
            w.best_t = kMaxFloat;
            state = ST_SHADE;
        }
    }
    SEC(SEC_RECORD);
    R.st4(HW_N, (uint32_t)n, stage | (fl << 16), rng.d, __float_as_uint(cu1));
}

// The wavefront kernel's body, shared by both integrators (kHead: integrator 1, shade_lane_head).
// kLdsWalk: walk steps read the staged top from LDS (integrator 1 always; integrator 0 when the LDS
// top holds the whole tree) instead of issuing every node's loads to memory.
template <bool kCount, bool kHead, bool kLdsWalk = kHead>
__device__ __forceinline__ void wf_main(const Args& a)
{
    extern __shared__ uint32_t lds_wf[];
    // after the four waves' rings (kWaveLdsWords each): the block counters (traced, reference,
    // samples, slow walks)
    unsigned long long* lcnt = reinterpret_cast<unsigned long long*>(lds_wf + 4 * kWaveLdsWords);
    // 4 counters + the section counts + the walk-length histogram (counting variant)
    if (threadIdx.x < 4 + kSections / 2 + kHist / 2) lcnt[threadIdx.x] = 0ull;
    uint32_t* const lhist = reinterpret_cast<uint32_t*>(lcnt + 4) + kSections;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    Counters cnt;
    if (kCount) cnt.tri_counts = a.tri_counts;
    if (kCount && threadIdx.x == 0) atomicMin(a.counters + 20, (unsigned long long)wall_clock64());   // first start
    uint32_t walk_slots = 0, shade_slots = 0;   // counting variant: SIMD lane-slot usage
    uint32_t trace_slots = 0, steps = 0;        // counting variant: lanes tracing per iteration; steps of this walk
    uint32_t start_wait = 0;                    // counting variant: lanes without a ray when a walk phase starts
    uint32_t itc[6] = {0, 0, 0, 0, 0, 0};       // counting variant: walk-iteration classes (counters[14..19])
    unsigned long long walk_clk = 0, shade_clk = 0;   // counting variant: wave-clock per phase
    uint32_t done_rel[2] = {0, 0};                    // counting variant: ticks from the queue's drain / the
                                                      // kernel's start to this lane's end

    // hot state: what the walk phase needs
    uint32_t state = ST_IDLE;
    V3 ro = v3(0, 0, 0), rd = v3(0, 0, 1);
    W4 w;
    int32_t& htri = reinterpret_cast<int32_t&>(w.best_slot);   // the pending hit lives in the walk state
    float& ht = w.best_t;                                        // (a finished walk leaves it there)
    htri = -1;
    ht = kMaxFloat;
    Stack4 S;
    S.ring = lds_wf + (threadIdx.x >> 6) * kWaveLdsWords + lane;
    S.stride = a.spill_stride;
    constexpr uint32_t kRecWords = kHead ? (uint32_t)kHeadWords : (uint32_t)kColdWords;
    const ColdRec R{__builtin_amdgcn_make_buffer_rsrc(a.cold, 0, (int)(kRecWords * a.cold_stride * 4u), 0x00020000),
                    (uint32_t)(blockIdx.x * blockDim.x + threadIdx.x) * 16u, a.cold_stride * 16u};
    S.spill_base = a.spill;   // spill column of lane g at byte offset 4g = R.voff / 4
    S.lane_off = &R.voff;
    S.off_mask = ~0u;
    S.off_shift = 2;
    // the light probe's emitters (count, then records), then the top of the BVH4 (kTopNodeBytes per node)
    uint32_t* const lprobe = reinterpret_cast<uint32_t*>(lcnt + 4 + (kSections + kHist) / 2);
    if (threadIdx.x == 0) { lprobe[0] = a.num_emis; lprobe[1] = 0u; }   // ([1]: the refill's exhausted unit counters)
    if (a.num_lights < kLdsLights)
        for (uint32_t k = threadIdx.x; k < (a.num_lights + 1) * 3; k += blockDim.x)
            reinterpret_cast<float4*>(lprobe + 4 + kMaxProbeEmitters * 12)[k] = reinterpret_cast<const float4*>(a.lights)[k];
    for (uint32_t k = threadIdx.x; k < a.num_emis * 3; k += blockDim.x)
        reinterpret_cast<float4*>(lprobe + 4)[k] = reinterpret_cast<const float4*>(a.emis)[k];
    if (kHead && a.num_lights < kLdsLights) {   // integrator 1: each staged light's normal and material
        float4* const lnm = reinterpret_cast<float4*>(lprobe + 4 + kMaxProbeEmitters * 12 + kLdsLights * 12);
        for (uint32_t k = threadIdx.x; k <= a.num_lights; k += blockDim.x) {
            const DLight& L = a.lights[k];
            float4 q = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (L.pad == 0.0f) {
                const DShade& sh = a.shade[L.tri];
                q = make_float4(sh.nx, sh.ny, sh.nz, __uint_as_float((uint32_t)sh.mat));
            }
            lnm[k] = q;
        }
    }
    float4* const ltop = reinterpret_cast<float4*>(reinterpret_cast<char*>(lprobe) + kProbeLdsBytes +
                                                   (kHead ? kHeadLdsLightBytes : 0));
    for (uint32_t k = threadIdx.x; k < a.top_nodes * (kTopNodeBytes / 16); k += blockDim.x) {
        const uint32_t nd = k / (kTopNodeBytes / 16), q = k - nd * (kTopNodeBytes / 16);
        ltop[k] = reinterpret_cast<const float4*>(a.nodes4 + nd)[q];
    }
    S.top = reinterpret_cast<const char*>(ltop);
    S.ntop = a.top_nodes;
    __syncthreads();
    const uint32_t nlanes = gridDim.x * blockDim.x, wave_id = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (a.lane_times && lane == 0) a.lane_times[nlanes + wave_id] = wall_clock64();

    for (;;) {
        // ---------------------------------------------------------------- walk
        // walk phases issue ahead of other waves' shading passes (wave priority 1 vs 0): a walk
        // step's node fetch goes out sooner, so more of its round trip overlaps the shading VALU
        // (C3 +2.7%, 1/8 shard +1.0%, same box; priorities 2 and 3 the same, shading first -0.7%)
        __builtin_amdgcn_s_setprio(1);
        unsigned long long clk0 = 0;
        if (kCount) clk0 = clock64();
        const uint64_t live = __ballot(state != ST_DONE);   // (no lane becomes DONE while walking)
        if (kCount) start_wait += (uint32_t)__popcll(live & ~__ballot(state == ST_TRACE));
        // (the threshold as an opaque scalar: left a kernel argument, it was reloaded and waited for at
        // the head of every step)
        uint32_t thr;
        asm volatile("s_mov_b32 %0, %1" : "=s"(thr) : "s"(a.wf_threshold));
        for (;;) {
            const uint64_t tracing = __ballot(state == ST_TRACE);
            if (tracing == 0ull) break;
            if ((uint32_t)__popcll(live & ~tracing) >= thr) break;   // lanes waiting to shade
            if (kCount) {
                ++walk_slots;
                if (state == ST_TRACE) ++trace_slots;
                // wave iterations by the number of lanes needing a global node fetch (0, 1-4, 5-8,
                // more), with no pending leaf in the wave, and with neither
                const bool vis = state == ST_TRACE && w.node != kNone && w.lsp <= kLeafRing - 1;
                const uint32_t deep = (uint32_t)__popcll(__ballot(vis && w.node >= S.ntop));
                const bool noleaf = __ballot(state == ST_TRACE && leaf4_pending(w)) == 0ull;
                ++itc[deep == 0u ? 0 : deep <= 4u ? 1 : deep <= 8u ? 2 : 3];
                if (noleaf) ++itc[4];
                if (noleaf && deep == 0u) ++itc[5];
            }
            if (state == ST_TRACE) {
                // (the culling factor as the literal it always is: a kernel argument here was a scalar
                // load and wait on every step's chain, the compiler rematerialising it for want of SGPRs)
                const bool more = walk4_step<kCount, true, NoSetup, kHead, !kLdsWalk>(
                    w, ro, rd, a.nodes4, a.acc_tris, S, kCullRel, a.cull_abs, a.node_mask, cnt);
                if (kCount) ++steps;
                if (kCount && !more) {   // walk length histogram, log2 buckets
                    atomicAdd(lhist + min(31 - __clz((int)steps), kHist - 1), 1u);
                    steps = 0;
                }
                if (!more) state = ST_WALKED;
            }
        }
        __builtin_amdgcn_s_setprio(0);
        // the winner's check against the reference BVH runs in the shading phase
        // (htri, ht) == (w.best_slot, w.best_t): the hit is already in place
        // (no winner: a miss -- or, for a bounded last-bounce walk, never expected: exact slow walk)
        if (state == ST_WALKED) {
            if (kHead) {   // integrator 1: no hit below the bound is a miss (a visibility walk's "not visible")
                if (w.best_slot != kNone) state = ST_CHECK;
                else { w.best_t = kMaxFloat; state = ST_SHADE; }
            } else {
                state = (w.best_slot != kNone) ? ST_CHECK : (w.best_t == kMaxFloat) ? ST_SHADE : ST_SLOW;
            }
        }

        if (kCount) {
            const unsigned long long c = clock64();
            walk_clk += c - clk0;
            clk0 = c;
        }
        // ---------------------------------------------------------------- shade + refill
        // Only the per-bounce part of the shading state is held in registers here (sample
        // index, bounce, flags, RNG, path weight); accumulator, running mean, pixel and memo
        // words are read and written in the record where they are used.
        if (kCount) ++shade_slots;
        // (the lane id is recomputed for the shading pass: one VGPR less live across the walk loop)
        if (state != ST_TRACE && state != ST_DONE) {
            if (kHead) shade_lane_head<kCount>(R, (int)__lane_id(), state, ro, rd, htri, ht, w, S, lcnt, lprobe, done_rel, cnt);
            else shade_lane<kCount>(a, R, (int)__lane_id(), state, ro, rd, htri, ht, w, S, lcnt, lprobe, done_rel, cnt);
        }
        if (kCount) shade_clk += clock64() - clk0;
        if (__ballot(state != ST_DONE) == 0ull) break;
    }
    if (a.lane_times && lane == 0) a.lane_times[nlanes + nlanes / 64 + wave_id] = wall_clock64();
    if (kCount) {
        if (lane == 0) { atomicAdd(a.counters + 9, walk_clk); atomicAdd(a.counters + 10, shade_clk); }
        if (lane == 0) {   // wave exit times (wall clock): last, the sum for the mean, and after the drain
            const unsigned long long t = wall_clock64();
            atomicMax(a.counters + 22, t);
            atomicAdd(a.counters + 23, t);
            atomicAdd(a.counters + 24, 1ull);
            const unsigned long long d0 = __hip_atomic_load(a.counters + 21, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicAdd(a.counters + 80 + tail_bin(t - min(t, d0)), 1ull);
        }
        // lane ends after the drain (log2 bins: one atomic per occupied bin and wave), and their sum
        // since the kernel's start (the tail's idle lane-time = lanes x last exit - that sum)
        const uint32_t bin = tail_bin(done_rel[0]);
        for (uint32_t k = 0; k < (uint32_t)kTailBins; ++k) {
            const uint64_t m = __ballot(bin == k);
            if (m && lane == 0) atomicAdd(a.counters + 64 + k, (unsigned long long)__popcll(m));
        }
        const unsigned long long dsum = wave_sum(done_rel[1]);
        if (lane == 0) atomicAdd(a.counters + 26, dsum);
        const unsigned long long c2 = wave_sum(cnt.nodes), c3v = wave_sum(cnt.tris), c5 = wave_sum(walk_slots);
        const unsigned long long c13 = wave_sum(cnt.top), c25 = wave_sum(cnt.spills);
        const unsigned long long c6 = wave_sum(cnt.leaf_steps), c7 = wave_sum(shade_slots);
        const unsigned long long c11 = wave_sum(trace_slots);
        if (lane == 0) {
            atomicAdd(a.counters + 2, c2); atomicAdd(a.counters + 3, c3v); atomicAdd(a.counters + 5, c5);
            atomicAdd(a.counters + 6, c6); atomicAdd(a.counters + 7, c7); atomicAdd(a.counters + 11, c11);
            atomicAdd(a.counters + 12, (unsigned long long)start_wait);
            atomicAdd(a.counters + 13, c13);
            atomicAdd(a.counters + 25, c25);
            for (int k = 0; k < 6; ++k) atomicAdd(a.counters + 14 + k, (unsigned long long)itc[k]);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(a.counters + 0, lcnt[0]);
        atomicAdd(a.counters + 1, lcnt[1]);
        atomicAdd(a.counters + 4, lcnt[2]);
        if (lcnt[3]) atomicAdd(a.counters + 8, lcnt[3]);
    }
    if (kCount && threadIdx.x < kSections + kHist) {   // section counts, then the histogram
        const uint32_t v = reinterpret_cast<const uint32_t*>(lcnt + 4)[threadIdx.x];
        if (v) atomicAdd(a.counters + 32 + threadIdx.x, (unsigned long long)v);
    }
}

template <bool kCount, int kMinWaves, bool kLdsWalk = false>
__global__ __launch_bounds__(256, kMinWaves) void render_unidir_wf(Args a)
{
    wf_main<kCount, false, kLdsWalk>(a);
}

// integrator 1 (radianceAlongSingleStep, kernel.cu:217-415) on the wavefront state machine
template <bool kCount, int kMinWaves>
__global__ __launch_bounds__(256, kMinWaves) void render_head_wf(Args a)
{
    wf_main<kCount, true>(a);
}

// ------------------------------------------------------------------ output step
// kernel.cu:763-778 / color.h:59-71 on the GPU: code = (int)(pow(c/(c+1), (float)(1/2.2))*255)
// per channel, read off a table of the 255 boundaries the HOST's libm puts between codes
// (pt::tonemap_thresholds), so the codes equal pt_tonemap_u8 exactly.
__global__ __launch_bounds__(256) void tonemap_codes(const float* __restrict__ rgb, size_t n,
                                                     const float* __restrict__ thr, int32_t* __restrict__ out)
{
    __shared__ float t[256];
    t[threadIdx.x] = thr[threadIdx.x];
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float c = rgb[i];
        int32_t code;
        if (!(c == c) || c == INFINITY) {
            code = INT32_MIN;                // c/(c+1) is NaN: (int)NaN on x86
        } else if (c < 0.0f) {
            code = INT32_MAX;                // never produced by the integrator; redone on the host
        } else {
            int lo = 0, hi = 255;            // largest k with t[k] <= c (t[0] = 0)
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (t[mid] <= c) lo = mid; else hi = mid - 1;
            }
            code = lo;
        }
        out[i] = code;
    }
}

// ------------------------------------------------------------------ batched trace()
// pt_trace: the reference's trace() (kernel.cu:112-161) for a batch of rays, one lane per ray,
// on the same walk the wavefront kernel uses (BVH4 + winner check + exact slow path), or on the
// reference BVH with the reference's own stack walk (kRef).
template <bool kRef, bool kCount>
__global__ __launch_bounds__(256) void trace_rays(Args a, const float* __restrict__ rays, uint32_t n,
                                                  int32_t* __restrict__ tri_out, float* __restrict__ t_out)
{
    extern __shared__ uint32_t lds_tr[];
    const int lane = threadIdx.x & 63;
    Counters cnt;
    if (kCount) cnt.tri_counts = a.tri_counts;
    Stack4 S;
    // per wave: the reference walk's stack (stack_words) or the BVH4 rings (kWaveLdsWords)
    uint32_t* const wave_lds = lds_tr + (threadIdx.x >> 6) * a.stack_words;
    S.ring = wave_lds + lane;
    S.stride = a.spill_stride;
    const uint32_t lane_off = (blockIdx.x * blockDim.x + threadIdx.x) * 4u;
    S.spill_base = a.spill;
    S.lane_off = &lane_off;
    S.off_mask = ~0u;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        const V3 o = v3(rays[6 * r], rays[6 * r + 1], rays[6 * r + 2]);
        const V3 d = v3(rays[6 * r + 3], rays[6 * r + 4], rays[6 * r + 5]);
        int32_t htri = -1;
        float ht = kMaxFloat;
        if (a.num_tris == 0) {
            // spheres only
        } else if (kRef) {
            const Hit h = trace_reference<kCount>(o, d, a.rnodes, a.tris_orig, wave_lds, lane, cnt);
            htri = h.tri; ht = h.t;
        } else if (!((a.scene_fast != 0u) && ray_fast(o, d))) {
            atomicAdd(a.counters + 8, 1ull);
            trace_slow(o, d, a.root, a.nodes, a.tris_leaf, S.spill(), S.stride, a.cull_rel, a.cull_abs, &htri, &ht,
                       cnt.tri_counts);
        } else {
            W4 w;
            if (walk4_begin(w, o, d, a.acc_root, a.cull_abs)) {
                while (walk4_step<kCount>(w, o, d, a.nodes4, a.acc_tris, S, a.cull_rel, a.cull_abs, a.node_mask, cnt)) {
                }
                ht = w.best_t;
                bool ok = true;
                if (w.best_slot != kNone) {
                    const float4 C = a.acc_tris[w.best_slot].c;
                    htri = (int32_t)__float_as_uint(C.y);
                    ok = ref_tested(__float_as_uint(C.w), o, d, a.rnodes, a.rparent);
                }
                if (!ok) {
                    atomicAdd(a.counters + 8, 1ull);
                    trace_slow(o, d, a.root, a.nodes, a.tris_leaf, S.spill(), S.stride, a.cull_rel, a.cull_abs,
                               &htri, &ht, cnt.tri_counts);
                }
            }
        }
        if (a.num_spheres) apply_spheres(a, o, d, &htri, &ht);
        tri_out[r] = htri;
        t_out[r] = ht;
    }
    if (kCount) {
        const unsigned long long sp = wave_sum(cnt.spills);
        if (lane == 0 && sp) atomicAdd(a.counters + 25, sp);
    }
}

// ------------------------------------------------------------------ host side
#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return pt::fail(PT_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

template <typename T>
int upload(T** dst, const std::vector<T>& src)
{
    size_t bytes = src.size() * sizeof(T);
    if (bytes == 0) bytes = sizeof(T);
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(dst), bytes));
    if (!src.empty()) HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return PT_OK;
}

}  // namespace

// GF(2) jump tables J_k = A^(2^(67+k)), k = 0..31, rocRAND's bit-image layout.
static void build_jump_tables(std::vector<uint32_t>& out)
{
    auto apply = [](const uint32_t* img, uint32_t v[5]) {
        uint32_t r[5] = {0, 0, 0, 0, 0};
        for (int b = 0; b < 160; ++b)
            if ((v[b >> 5] >> (b & 31)) & 1u)
                for (int w = 0; w < 5; ++w) r[w] ^= img[b * 5 + w];
        memcpy(v, r, sizeof(r));
    };
    std::vector<uint32_t> m(800), tmp(800);
    for (int b = 0; b < 160; ++b) {   // one XORWOW step on the 160-bit xorshift state
        uint32_t v[5] = {0, 0, 0, 0, 0};
        v[b >> 5] = 1u << (b & 31);
        const uint32_t t = v[0] ^ (v[0] >> 2);
        uint32_t nv[5] = {v[1], v[2], v[3], v[4], (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1))};
        memcpy(&m[b * 5], nv, sizeof(nv));
    }
    auto square = [&]() {
        for (int b = 0; b < 160; ++b) {
            uint32_t v[5];
            memcpy(v, &m[b * 5], sizeof(v));
            apply(m.data(), v);
            memcpy(&tmp[b * 5], v, sizeof(v));
        }
        m.swap(tmp);
    };
    for (int i = 0; i < 67; ++i) square();
    out.resize(32 * 800);
    for (int k = 0; k < 32; ++k) {
        memcpy(&out[k * 800], m.data(), 800 * sizeof(uint32_t));
        square();
    }
}

// Byte-sliced form of the jump tables for rng_init: entry (k, j, x) = J_k * (x << 8j).
static void build_jump_bytes(const std::vector<uint32_t>& img, std::vector<uint32_t>& out)
{
    out.assign((size_t)32 * 20 * 256 * kJumpEntryWords, 0u);
    for (int k = 0; k < 32; ++k)
        for (int j = 0; j < 20; ++j)
            for (int x = 0; x < 256; ++x) {
                uint32_t* e = &out[(((size_t)k * 20 + j) * 256 + x) * kJumpEntryWords];
                for (int i = 0; i < 8; ++i)
                    if ((x >> i) & 1)
                        for (int w = 0; w < 5; ++w) e[w] ^= img[(size_t)k * 800 + (8 * j + i) * 5 + w];
            }
}

void pt::sincos_det(float theta, float* s, float* c) { det_sincos(theta, s, c); }

struct pt_ctx {
    int device = 0;
    DNode* nodes = nullptr;
    RNode* rnodes = nullptr;
    DTri* tris_leaf = nullptr;
    DTri* tris_orig = nullptr;
    DShade* shade = nullptr;
    DMat* mats = nullptr;
    DLight* lights = nullptr;
    uint32_t* jump = nullptr;
    float4* shade_m = nullptr;        // merged shading records (Args::shade_m), or none
    uint32_t* jump_bytes = nullptr;   // byte-position jump matrices (built on the first wavefront render)
    hipEvent_t jump_ready = nullptr;  // recorded behind their build
    bool use_jump_bytes = true;       // PT_JUMP_BYTES=0: per-bit jumps only
    bool tile_fast4 = true;           // PT_TILE_FAST4=0: the tile kernel walks the reference BVH (culled)
    float* scratch_out = nullptr;
    size_t scratch_bytes = 0;
    uint32_t num_lights = 0;
    float total_light_area = 0;
    float root[6];
    int32_t depth = 0;
    uint32_t num_tris = 0;
    float scene_extent = 1.0f;
    void* pinned = nullptr;                    // pt_render: pinned staging buffer of the image copy-out
    size_t pinned_bytes = 0;
    // renders in flight (pt_render_device_async / pt_render_wait): a FIFO of kFlights slots, each with
    // its events and a pinned host copy of the render's counters
    struct Flight {
        hipEvent_t ev0 = nullptr, ev1 = nullptr;   // the whole render
        hipEvent_t ek0 = nullptr, ek1 = nullptr;   // the integration kernel alone
        hipEvent_t done = nullptr;                 // after the counters' copy
        unsigned long long* hcnt = nullptr;        // pinned: the counters, copied behind the render
        bool kernel_events = false, count = false;
        uint64_t units = 0, split = 0;
        int32_t spp = 0, bounces = 0;
    };
    static constexpr int kFlights = 2;
    Flight fl[kFlights];
    // A render's device scratch, one set per in-flight slot, so that two queued renders (e.g. frames on
    // two streams) never share a buffer; set 0 also serves the batched trace entry points.
    struct Bufs {
        uint32_t* spill = nullptr;            // per-lane stack spill columns, then the shading records
        size_t spill_words = 0;
        uint32_t* pix_states = nullptr;       // init_pixel_states output (kUnitWords per work unit)
        size_t pix_states_words = 0;
        double* lbuf = nullptr;               // per-sample radiance of split pixels
        size_t lbuf_words = 0;
        uint32_t* pmemo = nullptr;            // per-pixel-slot primary hit shared by a split pixel's chunks
        size_t pmemo_words = 0;
        unsigned long long* counters = nullptr;
        uint32_t* pixel_counter = nullptr;    // the unit queues
        uint32_t* tile_counter = nullptr;
        uint32_t* seed_states = nullptr;      // per-render seed_table output
        uint64_t seed_cached = 0;             // the seed seed_states was built for
        bool seed_valid = false;
    };
    Bufs rb[kFlights];
    int fl_head = 0, fl_n = 0;                 // oldest in-flight slot, number in flight
    int num_cus = 256;
    bool scene_fast = false;
    uint32_t node_mask = 0;
    uint32_t wf_threshold = 56;     // measured best at 5 waves/SIMD (C3: 24..64 swept)
    uint32_t wf_queues = kQueues;   // unit counters (PT_WF_QUEUES=1: one; 8: the 1/8 shard +5.8%, C3 +1.2%)
    uint32_t wf_root_first = 4;     // a new ray's first visits (root + up to 3 staged nodes) in the shading pass
                                    // (PT_WF_ROOT_FIRST; C3 1/2/3/4/6: 5331/5417/5461/5509/5406)
    uint32_t wf_waves_per_cu = 16;
    int wf_min_waves = 5;           // register budget of the wavefront kernel (PT_WF_MIN_WAVES: 4/5/6)
    int wf_chunks = 0;              // sample chunks per pixel, 0 = automatic (PT_WF_CHUNKS)
    int wf_tail_chunks = 6;         // chunks of each tail pixel (PT_WF_TAIL_CHUNKS; 1 = no tail split)
    double wf_tail_px = 1.5;        // tail pixels per resident lane (PT_WF_TAIL_PX; round 2 re-sweep after the
                                    // shading-pass fetch merges: C3 0.75 -> 1.5 +4.7%, the 1/2 shard +8%)
    int64_t wf_tail_npix = -1;      // explicit number of tail pixel slots (PT_WF_TAIL_NPIX), -1 = by wf_tail_px
    int wf_mid_chunks = -1;         // split shards: chunks of all but the last pixels (PT_WF_MID_CHUNKS;
                                    // -1 = automatic, 0 or 1 = one split for all)
    double wf_fine_px = 0.5;        // ... the last pixels per resident lane (PT_WF_FINE_PX)
    double wf_whole_px = 0.5;       // split shards with >= wf_whole_min pixels per lane: whole pixels per lane
    double wf_whole_min = 1.25;     // first (PT_WF_WHOLE_PX, PT_WF_WHOLE_MIN)
    int wf_fine_chunks = 0;         // ... and their chunks (PT_WF_FINE_CHUNKS; 0 = the automatic count)
    double wf_fin_px = 0.2;         // final grade: the last pixels per resident lane (PT_WF_FIN_PX) ...
    int wf_fin_chunks = 64;         // ... in this many chunks (PT_WF_FIN_CHUNKS; <= the fine count = off)
                                    // (measured: 1/8 and 1/4 shards +3%, full frame and 1/2 neutral)
    uint32_t wf_iters = 2;          // (PT_WF_ITERS)
    uint32_t wf_top = kTopNodesMax; // BVH4 nodes staged in each block's LDS (PT_WF_TOP; 0 = none)
    bool head_wf = true;            // integrator 1 on the wavefront kernel (PT_HEAD_WF=0: the tile kernel)
    int head_min_waves = 5;         // its register budget (PT_HEAD_MIN_WAVES: 4 = 128 VGPRs, 5 = 96)
    uint32_t top_nodes = 0;         // nodes of this scene's BVH4 that are LDS-staged (<= wf_top)
    uint32_t n4 = 0;                // nodes of this scene's BVH4
    bool wf_lds_tree = true;        // (PT_WF_LDS_TREE)
    DNode4* nodes4 = nullptr;
    DTri* acc_tris = nullptr;
    uint32_t* rparent = nullptr;
    float4* hrec = nullptr;
    float* tone_thr = nullptr;        // output step: the host libm's 255 code boundaries (+ t[0] = 0)
    bool tone_ok = false;
    float4* spheres = nullptr;        // sphere primitives (center, radius)
    uint32_t num_spheres = 0;
    uint32_t sphere_mat_base = 0;
    float acc_root[6];
    int32_t acc4_depth = 0;
    uint32_t node4_mask = 0;
    uint32_t* tri_counts = nullptr;   // PT_FLAG_COUNT: per-triangle test counts (num_tris entries, >= 1)
    DTri* emis = nullptr;             // last-bounce light probe: records of the emissive triangles
    uint32_t num_emis = 0;            // (0 = probe off: spheres present, too many emitters, PT_NO_LIGHT_PROBE)
};

int pt::ctx_device(const pt_ctx* c) { return c->device; }

// Per-lane HBM words the walks may need: the BVH4 ring's overflow (at most 3 pushes per level)
// and trace_slow's full stack on the reference BVH.
static size_t stack_words_per_lane(const pt_ctx* c);
static int ensure_spill(pt_ctx::Bufs& B, size_t words);
static bool alloc_bufs(pt_ctx::Bufs& B);

extern "C" {

static bool create_flights(pt_ctx* c)
{
    for (pt_ctx::Flight& f : c->fl) {
        if (hipEventCreate(&f.ev0) != hipSuccess || hipEventCreate(&f.ev1) != hipSuccess ||
            hipEventCreate(&f.ek0) != hipSuccess || hipEventCreate(&f.ek1) != hipSuccess ||
            hipEventCreateWithFlags(&f.done, hipEventDisableTiming) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&f.hcnt), kCounterWords * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess)
            return false;
    }
    return true;
}

pt_ctx* pt_create(const pt_scene* sc, int device, int* err)
{
    // PT_TIMING=1: host-side phase times on stderr (ingest-speed measurements)
    const bool timing = getenv("PT_TIMING") != nullptr;
    auto tstart = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!timing) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "pt_create: %-28s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tstart).count());
        tstart = now;
    };
    auto bail = [&](int code) -> pt_ctx* { if (err) *err = code; return nullptr; };
    if (!sc || (sc->num_tris == 0 && sc->num_spheres == 0) || (sc->num_tris > 0 && (!sc->verts || !sc->tris || !sc->bvh)) ||
        (sc->num_mats > 0 && !sc->mats) ||
        (sc->num_spheres > 0 && !sc->spheres) || (sc->num_lights > 0 && !sc->lights))
        return bail(pt::fail(PT_E_INVALID, "pt_create: incomplete scene"));
    const bool spheres_only = sc->num_tris == 0 && sc->num_spheres > 0 && sc->bvh_size == 0;
    if (!spheres_only && (sc->num_tris < 2 || sc->bvh_size != sc->num_tris - 1))
        return bail(pt::fail(PT_E_SCENE, "pt_create: need >= 2 triangles and a BVH of num_tris-1 nodes, or spheres only "
                             "(got %u tris, %u nodes, %u spheres)", sc->num_tris, sc->bvh_size, sc->num_spheres));
    if (sc->bvh_depth >= PT_MAX_BVH_DEPTH)
        return bail(pt::fail(PT_E_BVH_DEPTH, "Critical Error: BVH depth is too big (%d)", sc->bvh_depth));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return bail(pt::fail(PT_E_NODEV, "pt_create: no HIP device"));
    if (device < 0 || device >= ndev) return bail(pt::fail(PT_E_NODEV, "pt_create: device %d out of range (%d)", device, ndev));
    if (hipSetDevice(device) != hipSuccess) return bail(pt::fail(PT_E_HIP, "hipSetDevice(%d) failed", device));
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return bail(pt::fail(PT_E_HIP, "hipGetDeviceProperties failed"));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return bail(pt::fail(PT_E_NODEV, "pt_create: device %d is %s, this build targets gfx950", device, prop.gcnArchName));

    const uint32_t nt = sc->num_tris, nn = sc->bvh_size;
    for (uint32_t i = 0; i < nt; ++i) {
        const pt_triangle& t = sc->tris[i];
        if ((uint32_t)t.v0 >= sc->num_verts || (uint32_t)t.v1 >= sc->num_verts || (uint32_t)t.v2 >= sc->num_verts ||
            (uint32_t)t.mat >= sc->num_mats)
            return bail(pt::fail(PT_E_SCENE, "pt_create: triangle %u has an out-of-range vertex or material index", i));
    }
    for (uint32_t j = 0; j < sc->num_lights; ++j) {
        const uint32_t e = sc->lights[j];
        if ((e & PT_LIGHT_SPHERE) ? (e ^ PT_LIGHT_SPHERE) >= sc->num_spheres : e >= nt)
            return bail(pt::fail(PT_E_SCENE, "pt_create: light %u has an out-of-range primitive (0x%x)", j, e));
    }
    for (uint32_t k = 0; k < sc->num_spheres; ++k)
        if (!(sc->spheres[k].rad > 0.0f) || !std::isfinite(sc->spheres[k].rad))
            return bail(pt::fail(PT_E_SCENE, "pt_create: sphere %u has radius %g", k, (double)sc->spheres[k].rad));
    // validate the BVH: every reference must be in range, every triangle reachable once
    lap("device query");
    std::vector<uint32_t> leaf_rank(nt, 0xffffffffu);
    std::vector<uint32_t> leaf_order;
    leaf_order.reserve(nt);
    if (nt > 0) {
        std::vector<uint32_t> st;
        st.push_back(0);
        size_t visits = 0;
        while (!st.empty()) {   // left-first DFS = the order trace() meets leaves
            const uint32_t e = st.back();
            st.pop_back();
            if (++visits > 4ull * nt + 8) return bail(pt::fail(PT_E_SCENE, "pt_create: BVH is not a tree"));
            if (e & PT_BVH_LEAF_FLAG) {
                const uint32_t k = e ^ PT_BVH_LEAF_FLAG;
                if (k >= nt || leaf_rank[k] != 0xffffffffu) return bail(pt::fail(PT_E_SCENE, "pt_create: bad BVH leaf %u", k));
                leaf_rank[k] = (uint32_t)leaf_order.size();
                leaf_order.push_back(k);
            } else {
                if (e >= nn) return bail(pt::fail(PT_E_SCENE, "pt_create: BVH child %u out of range", e));
                st.push_back(sc->bvh[e].right);
                st.push_back(sc->bvh[e].left);
            }
        }
        if (leaf_order.size() != nt) return bail(pt::fail(PT_E_SCENE, "pt_create: BVH reaches %zu of %u triangles", leaf_order.size(), nt));
    }

    pt_ctx* c = new (std::nothrow) pt_ctx();
    if (!c) return bail(pt::fail(PT_E_OOM, "pt_create: out of host memory"));
    c->device = device;
    c->num_cus = prop.multiProcessorCount;
    c->num_tris = nt;
    c->depth = sc->bvh_depth;

    std::vector<uint32_t> ref_parent(nt, 0u);
    for (uint32_t i = 0; i < nn; ++i) {
        if (sc->bvh[i].left & PT_BVH_LEAF_FLAG) ref_parent[sc->bvh[i].left ^ PT_BVH_LEAF_FLAG] = i;
        if (sc->bvh[i].right & PT_BVH_LEAF_FLAG) ref_parent[sc->bvh[i].right ^ PT_BVH_LEAF_FLAG] = i;
    }
    auto tri_rec = [&](uint32_t k) {
        const pt_triangle& t = sc->tris[k];
        const pt_vec3 a = sc->verts[t.v0], b = sc->verts[t.v1], cc = sc->verts[t.v2];
        DTri r;
        const float e1x = b.x - a.x, e1y = b.y - a.y, e1z = b.z - a.z;   // modelLoader.h:58
        const float e2x = cc.x - a.x, e2y = cc.y - a.y, e2z = cc.z - a.z; // modelLoader.h:59
        r.a = make_float4(a.x, a.y, a.z, e1x);
        r.b = make_float4(e1y, e1z, e2x, e2y);
        const uint32_t words[3] = {k, leaf_rank[k], ref_parent[k]};
        float f[3];
        memcpy(f, words, sizeof(f));
        r.c = make_float4(e2z, f[0], f[1], f[2]);
        return r;
    };
    std::vector<DTri> tl(nt), to(nt);
    for (uint32_t i = 0; i < nt; ++i) { to[i] = tri_rec(i); tl[i] = tri_rec(leaf_order[i]); }
    std::vector<RNode> rn(nn);
    std::vector<DNode> dn(nn);
    auto box_of = [&](uint32_t ref, float* b) {   // box of a child; leaves carry no box
        if (ref & PT_BVH_LEAF_FLAG) { for (int q = 0; q < 6; ++q) b[q] = 0.0f; return; }
        const pt_bvh_node& x = sc->bvh[ref];
        b[0] = x.lo.x; b[1] = x.lo.y; b[2] = x.lo.z; b[3] = x.hi.x; b[4] = x.hi.y; b[5] = x.hi.z;
    };
    auto remap = [&](uint32_t ref) {
        return (ref & PT_BVH_LEAF_FLAG) ? (PT_BVH_LEAF_FLAG | leaf_rank[ref ^ PT_BVH_LEAF_FLAG]) : ref;
    };
    float lo_all[3] = {1e30f, 1e30f, 1e30f}, hi_all[3] = {-1e30f, -1e30f, -1e30f};
    for (uint32_t i = 0; i < nn; ++i) {
        const pt_bvh_node& x = sc->bvh[i];
        memcpy(rn[i].lo, &x.lo, 12);
        memcpy(rn[i].hi, &x.hi, 12);
        rn[i].left = x.left;
        rn[i].right = x.right;
        float b0[6], b1[6];
        box_of(x.left, b0);
        box_of(x.right, b1);
        dn[i].a = make_float4(b0[0], b0[1], b0[2], b0[3]);
        dn[i].b = make_float4(b0[4], b0[5], b1[0], b1[1]);
        dn[i].c = make_float4(b1[2], b1[3], b1[4], b1[5]);
        dn[i].d = make_uint4(remap(x.left), remap(x.right), 0u, 0u);
    }
    if (nt > 0) {
        const pt_bvh_node& r = sc->bvh[0];
        c->root[0] = r.lo.x; c->root[1] = r.lo.y; c->root[2] = r.lo.z;
        c->root[3] = r.hi.x; c->root[4] = r.hi.y; c->root[5] = r.hi.z;
        for (int q = 0; q < 3; ++q) { lo_all[q] = c->root[q]; hi_all[q] = c->root[3 + q]; }
    }
    for (uint32_t k = 0; k < sc->num_spheres; ++k) {   // the scene extent covers the spheres too
        const pt_sphere& sp = sc->spheres[k];
        const float cc[3] = {sp.pos.x, sp.pos.y, sp.pos.z};
        for (int q = 0; q < 3; ++q) {
            lo_all[q] = std::fmin(lo_all[q], cc[q] - sp.rad);
            hi_all[q] = std::fmax(hi_all[q], cc[q] + sp.rad);
        }
    }
    {
        float ext = 0.0f;
        for (int q = 0; q < 3; ++q) {
            const float e = std::fabs(hi_all[q]) > std::fabs(lo_all[q]) ? std::fabs(hi_all[q]) : std::fabs(lo_all[q]);
            ext = ext > e ? ext : e;
        }
        c->scene_extent = (ext > 0.0f && std::isfinite(ext)) ? ext : 1.0f;
    }
    {
        // Markstein-quotient precondition on the scene (pt_device.h div_mk): every vertex
        // coordinate is 0 or has magnitude in [2^-50, 2^20].  Boxes are min/max of vertices.
        bool ok = true;
        for (uint32_t v = 0; v < sc->num_verts && ok; ++v) {
            const float q[3] = {sc->verts[v].x, sc->verts[v].y, sc->verts[v].z};
            for (int k = 0; k < 3; ++k) {
                const float m = std::fabs(q[k]);
                if (!(m == 0.0f || (m >= 0x1p-50f && m <= 0x1p20f))) ok = false;
            }
        }
        c->scene_fast = ok;
        uint32_t bits = 1;
        while ((1u << bits) < nn) ++bits;
        c->node_mask = (bits >= 31) ? 0x7fffffffu : ((1u << bits) - 1u);
        if (const char* e = getenv("PT_WF_THRESHOLD")) c->wf_threshold = (uint32_t)atoi(e);
        if (const char* e = getenv("PT_WF_ROOT_FIRST")) c->wf_root_first = (uint32_t)atoi(e);
        if (const char* e = getenv("PT_WF_QUEUES")) c->wf_queues = (atoi(e) > 1) ? kQueues : 1u;
        if (const char* e = getenv("PT_JUMP_BYTES")) c->use_jump_bytes = atoi(e) != 0;
        if (const char* e = getenv("PT_TILE_FAST4")) c->tile_fast4 = atoi(e) != 0;
        if (const char* e = getenv("PT_HEAD_WF")) c->head_wf = atoi(e) != 0;
        if (const char* e = getenv("PT_HEAD_MIN_WAVES")) c->head_min_waves = (atoi(e) == 5) ? 5 : 4;
        if (const char* e = getenv("PT_WF_MIN_WAVES")) {
            const int v = atoi(e);
            c->wf_min_waves = (v == 4 || v == 6) ? v : 5;
        }
        c->wf_waves_per_cu = 4u * (uint32_t)c->wf_min_waves;
        if (const char* e = getenv("PT_WF_WAVES_PER_CU")) c->wf_waves_per_cu = (uint32_t)atoi(e);
        if (const char* e = getenv("PT_WF_CHUNKS")) c->wf_chunks = atoi(e);
        if (const char* e = getenv("PT_WF_TAIL_CHUNKS")) c->wf_tail_chunks = atoi(e);
        if (const char* e = getenv("PT_WF_TAIL_PX")) c->wf_tail_px = std::max(0.0, atof(e));
        if (const char* e = getenv("PT_WF_TAIL_NPIX")) c->wf_tail_npix = atoll(e);
        if (const char* e = getenv("PT_WF_MID_CHUNKS")) c->wf_mid_chunks = atoi(e);
        if (const char* e = getenv("PT_WF_FINE_PX")) c->wf_fine_px = std::max(0.0, atof(e));
        if (const char* e = getenv("PT_WF_FINE_CHUNKS")) c->wf_fine_chunks = atoi(e);
        if (const char* e = getenv("PT_WF_WHOLE_PX")) c->wf_whole_px = std::max(0.0, atof(e));
        if (const char* e = getenv("PT_WF_WHOLE_MIN")) c->wf_whole_min = std::max(0.0, atof(e));
        if (const char* e = getenv("PT_WF_FIN_PX")) c->wf_fin_px = std::max(0.0, atof(e));
        if (const char* e = getenv("PT_WF_FIN_CHUNKS")) c->wf_fin_chunks = atoi(e);
        if (const char* e = getenv("PT_WF_ITERS")) c->wf_iters = (uint32_t)std::max(1, atoi(e));
        if (const char* e = getenv("PT_WF_TOP")) c->wf_top = std::min<uint32_t>((uint32_t)std::max(0, atoi(e)), kTopNodesMax);
    }
    // render-path BVH4 (accel_build.cpp): binned SAH binary BVH collapsed to 4 wide
    std::vector<DNode4> an;
    std::vector<DTri> at;
    if (nt == 0) {   // spheres only: no triangle structures (kernels skip the walk)
        for (int q = 0; q < 3; ++q) { c->acc_root[q] = INFINITY; c->acc_root[3 + q] = -INFINITY; }
        c->acc4_depth = 0;
        c->node4_mask = 1u;
    } else {
        pt::AccelBvh acc;
        constexpr int kW = 4;
        pt::Accel4 acc4;
        lap("reference-BVH records");
        int rc4 = pt::build_accel(*sc, &acc);
        lap("SAH BVH build");
        if (timing && rc4 == PT_OK) fprintf(stderr, "pt_create: render BVH SAH cost %.6g\n", pt::accel_sah_cost(acc));
        if (rc4 == PT_OK) rc4 = pt::collapse_accel4(acc, &acc4);
        lap("BVH4 collapse");
        // the structural check (every node and slot reached once, <= 8 leaf triangles per node, nested
        // boxes) is O(nodes): the walk's exactness argument and its 8-bit leaf masks rely on it
        if (rc4 == PT_OK) rc4 = pt::validate_accel4(acc, acc4);
        lap("BVH4 validate");
        if (rc4 != PT_OK) { delete c; return bail(rc4); }
        // Node order: the kTopNodesMax nodes most likely to be visited first (best-first by box
        // surface area from the root: a connected top subtree, staged in LDS by the wavefront
        // kernel), then the others in their DFS order.
        const uint32_t n4 = (uint32_t)acc4.nodes.size();
        std::vector<uint32_t> new_of(n4, ~0u), old_of;
        old_of.reserve(n4);
        {
            std::vector<std::pair<float, uint32_t>> heap{{INFINITY, 0u}};
            while (!heap.empty() && old_of.size() < kTopNodesMax) {
                std::pop_heap(heap.begin(), heap.end());
                const uint32_t o = heap.back().second;
                heap.pop_back();
                new_of[o] = (uint32_t)old_of.size();
                old_of.push_back(o);
                const auto& x = acc4.nodes[o];
                for (int k = 0; k < kW; ++k) {
                    if (x.child[k] == pt::kAccel4Empty || (x.child[k] & PT_BVH_LEAF_FLAG)) continue;
                    const float b[6] = {x.lo[0][k], x.lo[1][k], x.lo[2][k], x.hi[0][k], x.hi[1][k], x.hi[2][k]};
                    const float ex = b[3] - b[0], ey = b[4] - b[1], ez = b[5] - b[2];
                    heap.push_back({ex * ey + ey * ez + ez * ex, x.child[k]});
                    std::push_heap(heap.begin(), heap.end());
                }
            }
            for (uint32_t o = 0; o < n4; ++o)
                if (new_of[o] == ~0u) { new_of[o] = (uint32_t)old_of.size(); old_of.push_back(o); }
        }
        c->top_nodes = std::min(std::max(c->wf_top, 1u), n4);   // (>= 1: the wavefront walk reads the LDS top unconditionally)
        c->n4 = n4;
        if (const char* e = getenv("PT_WF_LDS_TREE")) c->wf_lds_tree = atoi(e) != 0;
        // A tree the LDS top holds whole (small scenes: C2's Cornell box) is walked with no node fetch
        // from memory, so a walk step is cheap: waves stay in the walk phase until 62 lanes wait to
        // shade, and a new ray's first two visits (not four) run in the shading pass (C2: 6879 -> 7081
        // Msamples/s, same box, profiles/r03_c2_knobs; the stand-in's defaults are unchanged).
        if (n4 <= c->top_nodes) {
            if (!getenv("PT_WF_THRESHOLD")) c->wf_threshold = 62;
            if (!getenv("PT_WF_ROOT_FIRST")) c->wf_root_first = 2;
        }
        an.resize(n4);
        // Triangle slots: the triangles of each node's leaf children (in node order) get consecutive
        // slots, and each node lists its leaf children first -- the walk queues a node's entered
        // leaves as one entry (first slot, 8-bit mask of slots).  A leaf child's word is
        // kLeaf | the node's first leaf slot << kLeafBits | its slot bits relative to it.
        // slot_leaf[s] = the binary BVH's leaf slot (one triangle) of render slot s.
        std::vector<uint32_t> slot_leaf;
        slot_leaf.reserve(nt);
        for (size_t i = 0; i < n4; ++i) {
            auto x0 = acc4.nodes[old_of[i]], x = x0;
            auto is_leaf = [](uint32_t r) { return r != pt::kAccel4Empty && (r & PT_BVH_LEAF_FLAG); };
            int order[kW], m = 0;
            for (int k = 0; k < kW; ++k) if (is_leaf(x0.child[k])) order[m++] = k;
            for (int k = 0; k < kW; ++k) if (!is_leaf(x0.child[k])) order[m++] = k;
            const uint32_t base = (uint32_t)slot_leaf.size();
            for (int k = 0; k < kW; ++k) {
                const int q = order[k];
                for (int ax = 0; ax < 3; ++ax) { x.lo[ax][k] = x0.lo[ax][q]; x.hi[ax][k] = x0.hi[ax][q]; }
                x.child[k] = x0.child[q];
                if (is_leaf(x.child[k])) {
                    const uint32_t first = (uint32_t)slot_leaf.size() - base, cnt = pt::accel_leaf_count(x.child[k]);
                    for (uint32_t j = 0; j < cnt; ++j) slot_leaf.push_back(pt::accel_leaf_slot(x.child[k]) + j);
                    static_assert(pt::kAccel4LeafTris <= kLeafBits, "leaf slot mask width");
                    if (first + cnt > kLeafBits || base >= (1u << (31 - kLeafBits))) {
                        delete c;
                        return bail(pt::fail(PT_E_SCENE, "pt_create: %u triangles exceed the render path's leaf slot range", nt));
                    }
                    x.child[k] = PT_BVH_LEAF_FLAG | (base << kLeafBits) | (((1u << cnt) - 1u) << first);
                }
            }
            for (int k = 0; k < kW; ++k)
                if (x.child[k] != pt::kAccel4Empty && !(x.child[k] & PT_BVH_LEAF_FLAG)) x.child[k] = new_of[x.child[k]];
            an[i].lox = make_float4(x.lo[0][0], x.lo[0][1], x.lo[0][2], x.lo[0][3]);
            an[i].loy = make_float4(x.lo[1][0], x.lo[1][1], x.lo[1][2], x.lo[1][3]);
            an[i].loz = make_float4(x.lo[2][0], x.lo[2][1], x.lo[2][2], x.lo[2][3]);
            an[i].hix = make_float4(x.hi[0][0], x.hi[0][1], x.hi[0][2], x.hi[0][3]);
            an[i].hiy = make_float4(x.hi[1][0], x.hi[1][1], x.hi[1][2], x.hi[1][3]);
            an[i].hiz = make_float4(x.hi[2][0], x.hi[2][1], x.hi[2][2], x.hi[2][3]);
            an[i].child = make_uint4(x.child[0], x.child[1], x.child[2], x.child[3]);
            an[i].pad = make_uint4(0u, 0u, 0u, 0u);
        }
        if (slot_leaf.size() != nt) { delete c; return bail(pt::fail(PT_E_SCENE, "pt_create: BVH4 reaches %zu of %u triangles", slot_leaf.size(), nt)); }
        at.resize(nt);
        for (uint32_t i = 0; i < nt; ++i) {   // permuted for tri_hit_pk: {v0.xy, e1.xy}, {e2.xy, v0.z, e1.z}
            const DTri r = tri_rec(acc.leaf_order[slot_leaf[i]]);
            at[i].a = make_float4(r.a.x, r.a.y, r.a.w, r.b.x);
            at[i].b = make_float4(r.b.z, r.b.w, r.a.z, r.b.y);
            at[i].c = r.c;
        }
        memcpy(c->acc_root, acc.root_box, sizeof(c->acc_root));
        c->acc4_depth = acc4.depth;
        uint32_t bits = 1;
        while ((1u << bits) < (uint32_t)an.size()) ++bits;
        c->node4_mask = (1u << bits) - 1u;
    }
    std::vector<uint32_t> rpar(nn, 0u);
    for (uint32_t i = 0; i < nn; ++i) {
        if (!(sc->bvh[i].left & PT_BVH_LEAF_FLAG)) rpar[sc->bvh[i].left] = i;
        if (!(sc->bvh[i].right & PT_BVH_LEAF_FLAG)) rpar[sc->bvh[i].right] = i;
    }
    // per render-path slot: the reference parent's node of its triangle (into Args::hrec below)
    std::vector<RNode> wb(std::max<size_t>(at.size(), 1));
    for (size_t sl = 0; sl < at.size(); ++sl) {
        uint32_t parent;
        memcpy(&parent, &at[sl].c.w, 4);
        wb[sl] = rn[parent];
        wb[sl].left = parent;
        wb[sl].right = 0u;
    }
    // per render-path slot: the winner check's box, parent and triangle id, and the shading normal and
    // material (Args::hrec)
    std::vector<float4> hr((size_t)3 * std::max<size_t>(at.size(), 1));
    for (size_t sl = 0; sl < at.size(); ++sl) {
        uint32_t tid;
        memcpy(&tid, &at[sl].c.y, 4);
        const RNode& b = wb[sl];
        float fpar, ftid, fmat;
        memcpy(&fpar, &b.left, 4);
        memcpy(&ftid, &tid, 4);
        memcpy(&fmat, &sc->tris[tid].mat, 4);
        hr[3 * sl] = make_float4(b.lo[0], b.lo[1], b.lo[2], b.hi[0]);
        hr[3 * sl + 1] = make_float4(b.hi[1], b.hi[2], fpar, ftid);
        hr[3 * sl + 2] = make_float4(sc->tris[tid].norm.x, sc->tris[tid].norm.y, sc->tris[tid].norm.z, fmat);
    }
    // last-bounce light probe (shade_lane begin_trace): every triangle whose material has
    // emission.r != 0 (the integrator's emission test, kernel.cu:453 -- not the caller's light list)
    std::vector<DTri> em;
    for (uint32_t i = 0; i < nt; ++i)
        if (sc->mats[sc->tris[i].mat].emission[0] != 0) {
            const DTri r = tri_rec(i);   // permuted for tri_hit_pk, as the render path's records
            DTri q;
            q.a = make_float4(r.a.x, r.a.y, r.a.w, r.b.x);
            q.b = make_float4(r.b.z, r.b.w, r.a.z, r.b.y);
            q.c = r.c;
            em.push_back(q);
        }
    if (em.size() > kMaxProbeEmitters || sc->num_spheres > 0 || getenv("PT_NO_LIGHT_PROBE")) em.clear();
    c->num_emis = (uint32_t)em.size();
    std::vector<DShade> sh(nt);
    for (uint32_t i = 0; i < nt; ++i) {
        sh[i].nx = sc->tris[i].norm.x; sh[i].ny = sc->tris[i].norm.y; sh[i].nz = sc->tris[i].norm.z;
        sh[i].mat = sc->tris[i].mat;
    }
    // the merged per-triangle shading record (Args::shade_m) when every material colour is a float
    std::vector<float4> shm;
    {
        bool exact = nt > 0 && !getenv("PT_NO_SHADE_M");
        for (uint32_t i = 0; i < sc->num_mats && exact; ++i)
            for (int q = 0; q < 3; ++q)
                exact = exact && (double)(float)sc->mats[i].albedo[q] == sc->mats[i].albedo[q] &&
                        (double)(float)sc->mats[i].emission[q] == sc->mats[i].emission[q];
        if (exact) {
            shm.resize((size_t)3 * nt);
            for (uint32_t i = 0; i < nt; ++i) {
                const pt_material& m = sc->mats[sc->tris[i].mat];
                shm[3 * (size_t)i] = make_float4(sc->tris[i].norm.x, sc->tris[i].norm.y, sc->tris[i].norm.z, (float)m.emission[0]);
                shm[3 * (size_t)i + 1] = make_float4((float)m.albedo[0], (float)m.albedo[1], (float)m.albedo[2], (float)m.emission[1]);
                float mbits;
                memcpy(&mbits, &sc->tris[i].mat, 4);
                shm[3 * (size_t)i + 2] = make_float4((float)m.emission[2], mbits, 0.0f, 0.0f);
            }
        }
    }
    // scene materials, then one per sphere (sphere.h diffuse / emm)
    std::vector<DMat> mt(sc->num_mats + sc->num_spheres);
    for (uint32_t i = 0; i < sc->num_mats; ++i) {
        for (int q = 0; q < 3; ++q) { mt[i].albedo[q] = sc->mats[i].albedo[q]; mt[i].emission[q] = sc->mats[i].emission[q]; }
    }
    for (uint32_t k = 0; k < sc->num_spheres; ++k) {
        DMat& m = mt[sc->num_mats + k];
        for (int q = 0; q < 3; ++q) { m.albedo[q] = sc->spheres[k].diffuse[q]; m.emission[q] = sc->spheres[k].emission[q]; }
    }
    std::vector<float4> sp(sc->num_spheres);
    for (uint32_t k = 0; k < sc->num_spheres; ++k)
        sp[k] = make_float4(sc->spheres[k].pos.x, sc->spheres[k].pos.y, sc->spheres[k].pos.z, sc->spheres[k].rad);
    c->num_spheres = sc->num_spheres;
    c->sphere_mat_base = sc->num_mats;
    std::vector<DLight> lt(sc->num_lights + 1);
    auto light_rec = [&](uint32_t tri) {
        const pt_triangle& t = sc->tris[tri];
        const pt_vec3 a = sc->verts[t.v0], b = sc->verts[t.v1], cc = sc->verts[t.v2];
        DLight L;
        const float a1x = b.x - a.x, a1y = b.y - a.y, a1z = b.z - a.z;
        const float a2x = cc.x - a.x, a2y = cc.y - a.y, a2z = cc.z - a.z;
        // length(cross(a1, a2)) / 2, kernel.cu:477-478
        const float cx = a1y * a2z - a1z * a2y, cy = a1z * a2x - a1x * a2z, cz = a1x * a2y - a1y * a2x;
        L.area = sqrtf(cx * cx + cy * cy + cz * cz) / 2;
        L.tri = (int32_t)tri;
        L.v0[0] = a.x; L.v0[1] = a.y; L.v0[2] = a.z;
        L.a1[0] = a1x; L.a1[1] = a1y; L.a1[2] = a1z;
        L.a2[0] = a2x; L.a2[1] = a2y; L.a2[2] = a2z;
        L.pad = 0.0f;
        return L;
    };
    // sphere light (d8 policy): area 4*3.14159*r^2, center in v0, radius in a1[0], pad = 1
    auto sphere_light = [&](uint32_t k) {
        DLight L;
        memset(&L, 0, sizeof(L));
        const pt_sphere& q = sc->spheres[k];
        L.area = pt::sphere_area(q.rad);
        L.tri = (int32_t)(nt + k);
        L.v0[0] = q.pos.x; L.v0[1] = q.pos.y; L.v0[2] = q.pos.z;
        L.a1[0] = q.rad;
        L.pad = 1.0f;
        return L;
    };
    for (uint32_t j = 0; j < sc->num_lights; ++j) {
        const uint32_t e = sc->lights[j];
        lt[j] = (e & PT_LIGHT_SPHERE) ? sphere_light(e ^ PT_LIGHT_SPHERE) : light_rec(e);
    }
    lt[sc->num_lights] = (nt > 0) ? light_rec(0) : sphere_light(0);   // "nothing picked": primitive 0
    c->num_lights = sc->num_lights;
    c->total_light_area = sc->total_light_area;
    std::vector<uint32_t> jump_img, jump;
    build_jump_tables(jump_img);
    build_jump_bytes(jump_img, jump);
    std::vector<float> tone(256);
    c->tone_ok = pt::tonemap_thresholds(tone.data());

    // the BVH4 walk addresses nodes and triangle records by 32-bit byte offsets (pt_device.h
    // walk4_step): larger structures take the exact reference-BVH walk for every ray
    if ((uint64_t)an.size() * sizeof(an[0]) >= (1ull << 32) || (uint64_t)at.size() * sizeof(at[0]) >= (1ull << 32))
        c->scene_fast = false;
    int rc = PT_OK;
    lap("records + jump/tone tables");
    if ((rc = upload(&c->nodes, dn)) || (rc = upload(&c->rnodes, rn)) || (rc = upload(&c->tris_leaf, tl)) ||
        (rc = upload(&c->tris_orig, to)) || (rc = upload(&c->shade, sh)) || (!shm.empty() && (rc = upload(&c->shade_m, shm))) || (rc = upload(&c->mats, mt)) ||
        (rc = upload(&c->lights, lt)) || (rc = upload(&c->jump, jump)) || (rc = upload(&c->tone_thr, tone)) || (rc = upload(&c->spheres, sp)) ||
        (rc = upload(&c->nodes4, an)) || (rc = upload(&c->acc_tris, at)) || (rc = upload(&c->rparent, rpar)) || (rc = upload(&c->hrec, hr)) ||
        (rc = upload(&c->tri_counts, std::vector<uint32_t>(std::max<uint32_t>(nt, 1u), 0u))) ||
        (rc = upload(&c->emis, em))) {
        pt_destroy(c);
        return bail(rc);
    }
    if (!alloc_bufs(c->rb[0]) || !create_flights(c)) {
        pt_destroy(c);
        return bail(pt::fail(PT_E_HIP, "pt_create: device allocation failed"));
    }
    if (err) *err = PT_OK;
    lap("uploads");
    return c;
}

void pt_destroy(pt_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    void* bufs[] = {c->nodes, c->rnodes, c->tris_leaf, c->tris_orig, c->shade, c->mats,
                    c->lights, c->jump, c->jump_bytes, c->shade_m, c->scratch_out,
                    c->nodes4, c->acc_tris, c->rparent, c->hrec,
                    c->tone_thr, c->spheres, c->tri_counts, c->emis};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (pt_ctx::Bufs& B : c->rb)
        for (void* b : {(void*)B.spill, (void*)B.pix_states, (void*)B.lbuf, (void*)B.pmemo, (void*)B.counters,
                        (void*)B.pixel_counter, (void*)B.tile_counter, (void*)B.seed_states})
            if (b) (void)hipFree(b);
    pt::free_pinned(c->pinned);
    if (c->jump_ready) (void)hipEventDestroy(c->jump_ready);
    for (pt_ctx::Flight& f : c->fl) {
        for (hipEvent_t e : {f.ev0, f.ev1, f.ek0, f.ek1, f.done})
            if (e) (void)hipEventDestroy(e);
        if (f.hcnt) (void)hipHostFree(f.hcnt);
    }
    delete c;
}

// PT_LANE_TIMING summary of one wavefront render: wall-clock ticks (100 MHz) from the first wave's start
// to the queue's drain (the first lane without a unit), to the mean and the last lane end, and to the
// last wave exit; idle = the lane-time after each lane's end, as a fraction of lanes x kernel span.
static void write_lane_timing(const char* path, const std::vector<unsigned long long>& t, size_t lanes, int shards)
{
    const size_t waves = lanes / 64;
    unsigned long long t0 = ~0ull, drain = ~0ull, lend = 0, wexit = 0;
    for (size_t w = 0; w < waves; ++w) {
        if (t[lanes + w]) t0 = std::min(t0, t[lanes + w]);
        wexit = std::max(wexit, t[lanes + waves + w]);
    }
    double sum = 0.0;
    size_t n = 0;
    for (size_t l = 0; l < lanes; ++l) {
        if (!t[l]) continue;
        drain = std::min(drain, t[l]);
        lend = std::max(lend, t[l]);
        sum += (double)(t[l] - t0);
        ++n;
    }
    if (!n || t0 == ~0ull) return;
    const double span = (double)(wexit - t0);
    if (FILE* f = fopen(path, "a")) {
        fprintf(f, "lane_timing shards %d lanes %zu span %.0f drain %.0f mean_end %.0f last_end %.0f idle_frac %.4f\n", shards,
                n, span, (double)(drain - t0), sum / (double)n, (double)(lend - t0), 1.0 - (sum / (double)n) / span);
        fclose(f);
    }
}

int pt_render_device_async(pt_ctx* c, const pt_params* p, const pt_camera* cam, float* d_out, void* stream_v)
{
    if (!c || !p || !cam || !d_out) return pt::fail(PT_E_INVALID, "pt_render: null argument");
    if (c->fl_n >= pt_ctx::kFlights)
        return pt::fail(PT_E_INVALID, "pt_render_device_async: %d renders in flight (pt_render_wait first)", c->fl_n);
    if (p->width <= 0 || p->height <= 0 || p->width > 65535 || p->height > 65535)
        return pt::fail(PT_E_INVALID, "pt_render: image size %dx%d out of range (1..65535)", p->width, p->height);
    if (p->spp < 0) return pt::fail(PT_E_INVALID, "pt_render: spp < 0");
    if (p->integrator != PT_INTEGRATOR_UNIDIR && p->integrator != PT_INTEGRATOR_HEAD)
        return pt::fail(PT_E_INVALID, "pt_render: unknown integrator %d", p->integrator);
    if (p->integrator == PT_INTEGRATOR_UNIDIR && (p->bounces < 1 || p->bounces > 64))
        return pt::fail(PT_E_INVALID, "pt_render: bounces %d out of range (1..64)", p->bounces);
    if (p->shard_count < 1 || p->shard_index < 0 || p->shard_index >= p->shard_count)
        return pt::fail(PT_E_INVALID, "pt_render: shard %d of %d", p->shard_index, p->shard_count);
    if (cam->pxl_width <= 0 || cam->pxl_height <= 0) return pt::fail(PT_E_INVALID, "pt_render: camera pixel size must be > 0");
    if (p->pixel_order != PT_ORDER_SCANLINE && p->pixel_order != PT_ORDER_MORTON)
        return pt::fail(PT_E_INVALID, "pt_render: unknown pixel order %d", p->pixel_order);
    if (p->pixel_order == PT_ORDER_MORTON && !pt::morton_size_ok(p->width, p->height))
        return pt::fail(PT_E_INVALID, "pt_render: Morton pixel order needs a square power-of-two image, not %dx%d "
                        "(the reference's imgBuff indexing, kernel.cu:543,771)", p->width, p->height);
    for (const int32_t v : {p->tile_w, p->tile_h})
        if (v != 0 && (v < 8 || v > 256 || v % 8 != 0))
            return pt::fail(PT_E_INVALID, "pt_render: tile size %dx%d (0 = 8, else multiples of 8 up to 256)", p->tile_w, p->tile_h);
    // the per-triangle counts live in one context-wide buffer (pt_tri_counts reads it back): only one render
    // in flight may fill them
    if ((p->flags & PT_FLAG_COUNT) && (p->flags & PT_FLAG_TRI_COUNTS) && c->fl_n > 0)
        return pt::fail(PT_E_INVALID, "pt_render_device_async: PT_FLAG_TRI_COUNTS while a render is in flight");
    {   // the padded tile grid (tiles x tile_w x tile_h slots) must fit the kernels' 32-bit unit indices
        const uint64_t tw64 = p->tile_w ? (uint64_t)p->tile_w : 8u, th64 = p->tile_h ? (uint64_t)p->tile_h : 8u;
        const uint64_t slots = (((uint64_t)p->width + tw64 - 1) / tw64) * (((uint64_t)p->height + th64 - 1) / th64) * tw64 * th64;
        if (slots > 0xffffffffull)
            return pt::fail(PT_E_INVALID, "pt_render: %dx%d in %llux%llu tiles pads to %llu pixel slots (limit 2^32-1)",
                            p->width, p->height, (unsigned long long)tw64, (unsigned long long)th64, (unsigned long long)slots);
    }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_v);
    // this render's slot: its events and its buffer set.  The slot's previous render was collected by
    // pt_render_wait (its events synchronised), so two queued renders -- on one stream or on two, where
    // they may run concurrently -- never share a buffer.
    const int slot = (c->fl_head + c->fl_n) % pt_ctx::kFlights;
    pt_ctx::Flight& F = c->fl[slot];
    pt_ctx::Bufs& B = c->rb[slot];
    if (!alloc_bufs(B)) return pt::fail(PT_E_HIP, "pt_render: device allocation failed");

    Args a;
    memset(&a, 0, sizeof(a));
    a.nodes = c->nodes; a.rnodes = c->rnodes; a.tris_leaf = c->tris_leaf; a.tris_orig = c->tris_orig;
    a.shade = c->shade; a.mats = c->mats; a.lights = c->lights; a.jump = c->jump; a.shade_m = c->shade_m;
    a.out = d_out; a.counters = B.counters; a.tile_counter = B.tile_counter;
    a.num_lights = c->num_lights; a.total_light_area = c->total_light_area;
    a.spheres = c->spheres; a.num_spheres = c->num_spheres; a.num_tris = c->num_tris;
    a.sphere_mat_base = c->sphere_mat_base;
    a.emis = c->emis; a.num_emis = c->num_emis;
    memcpy(a.root, c->root, sizeof(a.root));
    a.cam.pos[0] = cam->pos.x; a.cam.pos[1] = cam->pos.y; a.cam.pos[2] = cam->pos.z;
    a.cam.dist = cam->dist_from_film; a.cam.focal = cam->focal_length; a.cam.radius = cam->radius;
    a.cam.w = cam->pxl_width; a.cam.h = cam->pxl_height;
    a.w = p->width; a.h = p->height; a.spp = p->spp; a.bounces = p->bounces; a.flags = p->flags; a.seed = p->seed;
    a.shard_index = p->shard_index; a.shard_count = p->shard_count;
    const uint32_t tw = p->tile_w ? (uint32_t)p->tile_w : kTile, th = p->tile_h ? (uint32_t)p->tile_h : kTile;
    const uint32_t tx = (p->width + tw - 1) / tw, ty = (p->height + th - 1) / th;
    const uint32_t ntiles = tx * ty;
    a.tiles_x = tx;
    a.tile_w = tw; a.tile_h = th;
    a.tile_bx = tw / kTile; a.tile_blocks = (tw / kTile) * (th / kTile);
    a.morton_out = (p->pixel_order == PT_ORDER_MORTON) ? 1u : 0u;
    a.ntiles_shard = (ntiles > (uint32_t)p->shard_index) ? (ntiles - (uint32_t)p->shard_index + (uint32_t)p->shard_count - 1) / (uint32_t)p->shard_count : 0;
    a.cull_rel = kCullRel;
    a.cull_abs = c->scene_extent * 1e-4f;
    const bool refwalk = (p->flags & PT_FLAG_REFERENCE_TRAVERSAL) != 0;
    const bool count = (p->flags & PT_FLAG_COUNT) != 0;
    const uint32_t levels = (uint32_t)c->depth + 2;
    a.stack_words = std::max<uint32_t>(levels * 128, (uint32_t)kWaveLdsWords);   // (culled walk's stack, or the BVH4 rings)
    const size_t lds = (size_t)a.stack_words * 4;
    if (lds > 160 * 1024) return pt::fail(PT_E_BVH_DEPTH, "pt_render: BVH depth %d needs %zu B of LDS stack", c->depth, lds);

    a.pixel_counter = B.pixel_counter;
    a.nunits = a.ntiles_shard * tw * th;
    a.scene_fast = c->scene_fast ? 1u : 0u;
    a.wf_threshold = c->wf_threshold;
    a.root_first = c->wf_root_first;
    a.unit_queues = c->wf_queues;
    a.wf_iters = c->wf_iters;
    a.node_mask = c->node_mask;
    a.nodes4 = c->nodes4;
    a.acc_tris = c->acc_tris;
    a.rparent = c->rparent;
    a.hrec = c->hrec;
    memcpy(a.acc_root, c->acc_root, sizeof(a.acc_root));
    // the render-path BVH's box margin assumes ray origins within ~2^6 of the scene extent
    const float cam_ext = std::fmax(std::fabs(cam->pos.x), std::fmax(std::fabs(cam->pos.y), std::fabs(cam->pos.z)));
    const bool near_cam = cam_ext <= 64.0f * c->scene_extent;
    // integrator 1 takes the wavefront kernel too (PT_HEAD_WF=0: the tile kernel, for comparisons)
    const bool head = p->integrator == PT_INTEGRATOR_HEAD;
    const bool wavefront = (p->integrator == PT_INTEGRATOR_UNIDIR || (head && c->head_wf)) && !refwalk &&
                           !(p->flags & PT_FLAG_REFERENCE_BVH) && near_cam &&
                           p->width < 65536 && p->height < 65536;   // (16-bit pixel coordinates per unit)

    // (the wavefront path's init_pixel_states resets the counters itself: one launch less per frame)
    if (!(p->spp > 0 && a.ntiles_shard > 0 && wavefront)) {
        HIP_TRY(hipMemsetAsync(B.counters, 0, kCounterWords * sizeof(unsigned long long), stream));
        HIP_TRY(hipMemsetAsync(B.counters + 20, 0xff, 2 * sizeof(unsigned long long), stream));   // (atomicMin slots)
        HIP_TRY(hipMemsetAsync(B.tile_counter, 0, 16, stream));
        HIP_TRY(hipMemsetAsync(B.pixel_counter, 0, kQueueStride * (kQueues + 1) * 4, stream));
    }
    if (count && (p->flags & PT_FLAG_TRI_COUNTS)) {   // per-triangle test counts of this render (pt_tri_counts)
        HIP_TRY(hipMemsetAsync(c->tri_counts, 0, (size_t)std::max<uint32_t>(c->num_tris, 1u) * 4, stream));
        a.tri_counts = c->tri_counts;
    }
    const uint32_t waves_per_cu = 16;
    uint32_t grid = (uint32_t)c->num_cus * waves_per_cu;
    if (grid > a.ntiles_shard * a.tile_blocks) grid = a.ntiles_shard > 0 ? a.ntiles_shard * a.tile_blocks : 1;
    // the tile kernel traces with the render-path BVH4 walk under the wavefront kernel's conditions
    // (PT_TILE_FAST4=0: the reference-BVH culled walk, as before)
    a.tile_fast4 = (!refwalk && !(p->flags & PT_FLAG_REFERENCE_BVH) && near_cam && c->tile_fast4 && c->num_tris > 0) ? 1u : 0u;
    HIP_TRY(hipEventRecord(F.ev0, stream));
    bool kernel_events = false;   // ek0/ek1 recorded around the integration kernel (wavefront path)
    bool seeded_now = false;      // seed_table enqueued for p->seed by this render
    uint64_t units = 0, split = 0;
    if (p->spp > 0 && a.ntiles_shard > 0 && wavefront) {
        // 4 waves per block; per wave an LDS ring of kRing packed entries x 64 lanes, deeper
        // entries spill to HBM (a BVH4 walk pushes at most 3 entries per level)
        Args b = a;
        b.stack_words = kRing * 64;
        b.node_mask = c->node4_mask;
        b.top_nodes = c->top_nodes;
        b.head = head ? 1u : 0u;
        const uint32_t wpc = (head && !count) ? 4u * (uint32_t)c->head_min_waves : c->wf_waves_per_cu;
        const size_t lds_fixed = (size_t)kWaveLdsWords * 4 * 4 + 4 * sizeof(unsigned long long) + (kSections + kHist) * 4 +
                                 kProbeLdsBytes + (head ? (size_t)kHeadLdsLightBytes : 0);
        {   // as many top nodes as leave every block of a CU its LDS (granted in 1280-B granules): integrator 1's
            // staged light normals cost it one node at 5 blocks per CU (97 -> 96), which kept it at 4 blocks
            const uint32_t bpc = std::max(1u, wpc / 4u);
            const size_t per_block = (size_t)(163840u / bpc) / 1280u * 1280u;
            const uint32_t cap = per_block > lds_fixed ? (uint32_t)((per_block - lds_fixed) / kTopNodeBytes) : 1u;
            if (b.top_nodes > 0) b.top_nodes = std::max(1u, std::min(b.top_nodes, cap));   // (0: no triangles, no BVH4)
        }
        const size_t lds_wf = lds_fixed + (size_t)b.top_nodes * kTopNodeBytes;
        // the whole tree staged in LDS (small scenes: C2): integrator 0's walk steps read it there too
        // (PT_WF_LDS_TREE=0: memory loads, as for a tree larger than the top)
        const bool lds_tree = c->wf_lds_tree && c->n4 > 0 && b.top_nodes >= c->n4;
        // (C2: 7181 with the record's second fetch against 7267 by triangle id; C3 the other way)
        b.rec_shading = lds_tree ? 0u : 1u;
        uint32_t blocks = (uint32_t)c->num_cus * (wpc / 4 ? wpc / 4 : 1);
        // Work units: a pixel's samples run in sequence, so a unit lasts one pixel's time and the
        // kernel's end waits for the last units started.  Whole pixels first; the last `ntail`
        // pixel slots are split into sample chunks, so the final units are short.
        // A shard with too few pixels to keep every resident lane busy is split entirely.
        b.npix = a.ntiles_shard * tw * th;
        const uint32_t paths_per_block = 256u;
        const uint64_t lanes = (uint64_t)blocks * paths_per_block;   // concurrently running paths
        uint32_t chunks = 1, ntail = 0, nmid = 0, chunks_mid = 1;
        if (c->wf_tail_npix >= 0) {   // (tests: an explicit tail)
            chunks = (uint32_t)(c->wf_chunks > 0 ? c->wf_chunks : c->wf_tail_chunks);
            ntail = (uint32_t)std::min<int64_t>(b.npix, c->wf_tail_npix);
        } else if (c->wf_chunks > 0) {
            chunks = (uint32_t)c->wf_chunks;
            ntail = b.npix;
        } else if (2 * (uint64_t)b.npix < 5 * lanes) {
            // ~16 fine units per lane, at most 8 chunks per pixel (round 2, after the shading pass got
            // cheaper: the 1/8 C3 shard +5..6% with 8 chunks instead of 21 and 4 mid chunks instead of
            // 6, profiles/r02_s4_units; the 1/4 shard alike with 8 or 11)
            chunks = (uint32_t)std::min<uint64_t>((16 * lanes + b.npix - 1) / b.npix, 8);
            // longer units first, the finer split for the last wf_fine_px pixels per lane
            // (measured on C3 shards: 1/4 shard 3 mid chunks, 1/8 shard 6: +3..4% over one split)
            const uint32_t nfine = (uint32_t)std::min<uint64_t>(b.npix, (uint64_t)(c->wf_fine_px * (double)lanes));
            // whole pixels first for wf_whole_px of the lanes when the shard has at least wf_whole_min pixels
            // per lane (a lane's whole pixel is then well within its share of the samples); the rest split
            // (round 5, profiles/r05_whole: the 1/4 shard with 0.3 / 0.5 / 0.7 / 0.9 whole pixels per lane
            // against none: C3 +3.4 / +5.0 / -0.6 / -12%, C4 +3.5 / +5.8 / +1.4%)
            uint32_t nwhole = 0;
            if ((double)b.npix >= c->wf_whole_min * (double)lanes)
                nwhole = (uint32_t)std::min<uint64_t>(b.npix - nfine, (uint64_t)(c->wf_whole_px * (double)lanes));
            ntail = b.npix - nwhole;
            int mc = c->wf_mid_chunks;
            if (mc < 0 && nfine < ntail)   // automatic: ~2.5 mid units per lane, at most 3 chunks
                // (round 5, sample-major split radiance: 3 against 4 at the 1/8 shard, C3 +0.9%, C4 +0.8%,
                // profiles/r05_mid)
                mc = std::min(3, (int)std::ceil(2.5 * (double)lanes / (double)(ntail - nfine)));
            if (mc > 1 && nfine < ntail) {
                nmid = ntail - nfine;
                chunks_mid = (uint32_t)std::min(mc, p->spp);
                if (c->wf_fine_chunks > 0) chunks = (uint32_t)c->wf_fine_chunks;
            }
        } else if (c->wf_tail_chunks > 1) {
            // (measured on C3: +6% with 0.5..1 tail pixel per lane in 4..8 chunks, 0.75 x 6 in round 1;
            // 1.5 x 6 since the shading pass's fetches were merged)
            chunks = (uint32_t)c->wf_tail_chunks;
            ntail = (uint32_t)std::min<uint64_t>(b.npix, (uint64_t)(c->wf_tail_px * (double)lanes));
        }
        // (measured on C3 shards: whole pixels down to ~3 per lane; below that ~16 units per lane:
        // 1/8 shard 20 chunks, 1/4 shard 10)
        if (chunks > (uint32_t)p->spp) chunks = (uint32_t)p->spp;
        // Split pixels keep their per-sample radiance (lbuf: 24 B per sample), so the split is
        // capped at a memory budget (PT_LBUF_BUDGET_MB; default a quarter of the device memory
        // free now, plus what lbuf already holds): beyond it the first tail slots become whole-pixel
        // units instead (the split only shortens the kernel's tail; results are identical).
        if (ntail > 0 && chunks > 1) {
            uint64_t budget;
            if (const char* e = getenv("PT_LBUF_BUDGET_MB")) {
                budget = (uint64_t)(std::max(0.0, atof(e)) * (double)(1ull << 20));   // (fractional MB kept)
            } else {
                size_t fr = 0, tot = 0;
                HIP_TRY(hipMemGetInfo(&fr, &tot));
                budget = ((uint64_t)fr + (uint64_t)B.lbuf_words * sizeof(double)) / 4;
            }
            const uint64_t cap = budget / ((uint64_t)p->spp * 3 * sizeof(double));
            if (ntail > cap) {
                const uint32_t drop = ntail - (uint32_t)cap;   // taken from the front: mid grade first
                nmid = nmid > drop ? nmid - drop : 0;
                ntail = (uint32_t)cap;
            }
        }
        // final grade: the queue's last units shorter still (the kernel ends when the units started
        // last are done), carved from the end of the fine grade
        uint32_t nfin = 0, chunks_fin = 1;
        if (ntail > nmid && c->wf_fin_px > 0.0 && c->wf_fin_chunks > (int)chunks) {
            nfin = (uint32_t)std::min<uint64_t>(ntail - nmid, (uint64_t)(c->wf_fin_px * (double)lanes));
            chunks_fin = (uint32_t)std::min(c->wf_fin_chunks, p->spp);
        }
        if ((uint64_t)b.npix + (uint64_t)ntail * (std::max(std::max(chunks, chunks_mid), chunks_fin) - 1) > 0xffffffffull)
            chunks = 1;
        if (chunks <= 1 || ntail == 0) { chunks = 1; ntail = 0; nmid = 0; }
        if (nmid == 0) chunks_mid = 1;
        if (ntail == 0 || chunks_fin <= chunks) { nfin = 0; chunks_fin = 1; }
        b.chunks = chunks;
        b.ntail = ntail;
        b.nmid = nmid;
        b.chunks_mid = chunks_mid;
        b.nfin = nfin;
        b.chunks_fin = chunks_fin;
        b.nwhole = b.npix - ntail;
        b.nunits = b.nwhole + nmid * chunks_mid + (ntail - nmid - nfin) * chunks + nfin * chunks_fin;
        const uint32_t need = (b.nunits + paths_per_block - 1) / paths_per_block;
        if (blocks > need) blocks = need;
        if (ntail > 0) {
            const size_t lw = (size_t)ntail * (size_t)p->spp * 3;
            if (B.lbuf_words < lw) {
                if (B.lbuf) (void)hipFree(B.lbuf);
                B.lbuf = nullptr;
                B.lbuf_words = 0;
                HIP_TRY(hipMalloc(reinterpret_cast<void**>(&B.lbuf), lw * sizeof(double)));
                B.lbuf_words = lw;
            }
            b.lbuf = B.lbuf;
            const size_t mw = (size_t)ntail * 2;
            if (B.pmemo_words < mw) {
                if (B.pmemo) (void)hipFree(B.pmemo);
                B.pmemo = nullptr;
                B.pmemo_words = 0;
                HIP_TRY(hipMalloc(reinterpret_cast<void**>(&B.pmemo), mw * 4));
                B.pmemo_words = mw;
            }
            b.pmemo = B.pmemo;
        }
        const size_t per_lane = stack_words_per_lane(c);
        const size_t rec_words = head ? (size_t)kHeadWords : (size_t)kColdWords;   // shading record per lane
        if (int rc = ensure_spill(B, per_lane * (size_t)blocks * 256 + rec_words * (size_t)blocks * paths_per_block))
            return rc;
        b.spill = B.spill;
        b.spill_stride = blocks * 256;
        b.cold_stride = blocks * paths_per_block;
        b.cold = B.spill + per_lane * (size_t)b.spill_stride;
        const size_t sw = (size_t)kUnitWords * b.nunits;
        if (B.pix_states_words < sw) {
            if (B.pix_states) (void)hipFree(B.pix_states);
            B.pix_states = nullptr;
            B.pix_states_words = 0;
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&B.pix_states), sw * 4));
            B.pix_states_words = sw;
        }
        b.pix_states = B.pix_states;
        // diagnostic: per-lane end / per-wave start and exit times (PT_LANE_TIMING=file appends a summary)
        const char* timing_path = getenv("PT_LANE_TIMING");
        std::vector<unsigned long long> times;
        unsigned long long* d_times = nullptr;
        if (timing_path) {
            times.assign((size_t)blocks * 256 + 2 * (size_t)blocks * 4, 0ull);
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_times), times.size() * 8));
            HIP_TRY(hipMemsetAsync(d_times, 0, times.size() * 8, stream));
            b.lane_times = d_times;
        }
        if (c->use_jump_bytes) {
            if (!c->jump_bytes) {   // once per context: 512 byte-sliced 160x160 GF(2) matrices (84 MB)
                // (built into locals and published only once the build launched: a failure leaves the
                // context without tables, so the next render tries again instead of seeding from garbage)
                // (a render queued on another stream meanwhile waits for the build: jump_ready)
                uint32_t* jb = nullptr;
                const bool ok = hipMalloc(reinterpret_cast<void**>(&jb), (size_t)512 * 20 * 256 * kJumpEntryWords * 4) == hipSuccess &&
                                (c->jump_ready || hipEventCreateWithFlags(&c->jump_ready, hipEventDisableTiming) == hipSuccess);
                if (ok) hipLaunchKernelGGL(build_jump_byte_tables, dim3(512 * 20), dim3(256), 0, stream, c->jump, jb);
                if (!ok || hipGetLastError() != hipSuccess || hipEventRecord(c->jump_ready, stream) != hipSuccess) {
                    if (jb) (void)hipFree(jb);
                    return pt::fail(ok ? PT_E_HIP : PT_E_OOM, "pt_render: jump-table setup failed");
                }
                c->jump_bytes = jb;
            } else {
                HIP_TRY(hipStreamWaitEvent(stream, c->jump_ready, 0));
            }
            if (!B.seed_states) {
                HIP_TRY(hipMalloc(reinterpret_cast<void**>(&B.seed_states), (size_t)256 * kJumpEntryWords * 4));
                B.seed_valid = false;
            }
            if (!B.seed_valid || B.seed_cached != p->seed) {   // (depends on the seed only: kept across renders)
                // (marked valid only once the whole render is enqueued: any error return below leaves the
                // slot unseeded, so the next render seeds again instead of trusting a table never written)
                B.seed_valid = false;
                hipLaunchKernelGGL(seed_table, dim3(1), dim3(256), 0, stream, b, B.seed_states);
                HIP_TRY(hipGetLastError());
                seeded_now = true;
            }
            b.jump_bytes = c->jump_bytes;
            b.seed_states = B.seed_states;
        }
        hipLaunchKernelGGL(init_pixel_states, dim3((b.npix + 255) / 256), dim3(256), 0, stream, b, B.pix_states);
        // A render queued on another stream while one is in flight: its seeding pre-pass runs beside the
        // earlier render's last waves (its own buffers), but the integration kernel waits until the earlier
        // render is complete (finalisation included), so a persistent grid never takes the CU slots an
        // earlier frame's finalisation needs (that one would otherwise wait out the whole next frame)
        if (c->fl_n > 0) HIP_TRY(hipStreamWaitEvent(stream, c->fl[(c->fl_head + c->fl_n - 1) % pt_ctx::kFlights].ev1, 0));
        HIP_TRY(hipEventRecord(F.ek0, stream));
        kernel_events = true;
        units = b.nunits;
        split = b.ntail;
        if (head) {
            if (count) hipLaunchKernelGGL((render_head_wf<true, 5>), dim3(blocks), dim3(256), lds_wf, stream, b);
            else if (c->head_min_waves == 4) hipLaunchKernelGGL((render_head_wf<false, 4>), dim3(blocks), dim3(256), lds_wf, stream, b);
            else hipLaunchKernelGGL((render_head_wf<false, 5>), dim3(blocks), dim3(256), lds_wf, stream, b);
        }
        else if (count && c->wf_min_waves == 4) hipLaunchKernelGGL((render_unidir_wf<true, 4>), dim3(blocks), dim3(256), lds_wf, stream, b);
        else if (count && lds_tree) hipLaunchKernelGGL((render_unidir_wf<true, 5, true>), dim3(blocks), dim3(256), lds_wf, stream, b);
        else if (count) hipLaunchKernelGGL((render_unidir_wf<true, 5>), dim3(blocks), dim3(256), lds_wf, stream, b);
        else if (c->wf_min_waves == 6) hipLaunchKernelGGL((render_unidir_wf<false, 6>), dim3(blocks), dim3(256), lds_wf, stream, b);
        else if (c->wf_min_waves == 5 && lds_tree) hipLaunchKernelGGL((render_unidir_wf<false, 5, true>), dim3(blocks), dim3(256), lds_wf, stream, b);
        else if (c->wf_min_waves == 5) hipLaunchKernelGGL((render_unidir_wf<false, 5>), dim3(blocks), dim3(256), lds_wf, stream, b);
        else hipLaunchKernelGGL((render_unidir_wf<false, 4>), dim3(blocks), dim3(256), lds_wf, stream, b);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(F.ek1, stream));
        if (b.ntail > 0) hipLaunchKernelGGL(finalize_pixels, dim3((b.ntail + 255) / 256), dim3(256), 0, stream, b);
        HIP_TRY(hipGetLastError());
        if (d_times) {
            HIP_TRY(hipMemcpyAsync(times.data(), d_times, times.size() * 8, hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            (void)hipFree(d_times);
            write_lane_timing(timing_path, times, (size_t)blocks * 256, p->shard_count);
        }
    } else if (p->spp > 0 && a.ntiles_shard > 0) {
        if (a.tile_fast4) {   // the BVH4 walk's ring overflow and the slow walk's stack: one HBM column per lane
            if (int rc = ensure_spill(B, stack_words_per_lane(c) * (size_t)grid * 64)) return rc;
            a.spill = B.spill;
            a.spill_stride = grid * 64;
        }
#define PT_LAUNCH(I, R, C) hipLaunchKernelGGL((render_tiles<I, R, C>), dim3(grid), dim3(64), lds, stream, a)
        if (p->integrator == PT_INTEGRATOR_HEAD) {
            if (refwalk) { if (count) PT_LAUNCH(1, true, true); else PT_LAUNCH(1, true, false); }
            else { if (count) PT_LAUNCH(1, false, true); else PT_LAUNCH(1, false, false); }
        } else {
            if (refwalk) { if (count) PT_LAUNCH(0, true, true); else PT_LAUNCH(0, true, false); }
            else { if (count) PT_LAUNCH(0, false, true); else PT_LAUNCH(0, false, false); }
        }
#undef PT_LAUNCH
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(F.ev1, stream));
    HIP_TRY(hipMemcpyAsync(F.hcnt, B.counters, kCounterWords * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipEventRecord(F.done, stream));
    F.kernel_events = kernel_events;
    F.count = count;
    F.units = units;
    F.split = split;
    F.spp = p->spp;
    F.bounces = p->bounces;
    if (seeded_now) {
        B.seed_cached = p->seed;
        B.seed_valid = true;
    }
    ++c->fl_n;
    return PT_OK;
}

int pt_render_wait(pt_ctx* c, pt_stats* st)
{
    if (!c) return pt::fail(PT_E_INVALID, "pt_render_wait: null context");
    if (c->fl_n == 0) return pt::fail(PT_E_INVALID, "pt_render_wait: no render in flight");
    HIP_TRY(hipSetDevice(c->device));
    pt_ctx::Flight& F = c->fl[c->fl_head];
    c->fl_head = (c->fl_head + 1) % pt_ctx::kFlights;
    --c->fl_n;
    // (the counters' copy is the render's last operation on its stream)
    HIP_TRY(hipEventSynchronize(F.done));
    const unsigned long long* cnt = F.hcnt;
    if (F.count) {
        if (const char* path = getenv("PT_SECTION_DUMP")) {   // counting runs: shading section profile
            if (FILE* f = fopen(path, "a")) {
                fprintf(f, "sections");
                for (int k = 0; k < kSections; ++k) fprintf(f, " %llu", cnt[32 + k]);
                fprintf(f, "\nwalk_hist");
                for (int k = 0; k < kHist; ++k) fprintf(f, " %llu", cnt[32 + kSections + k]);
                fprintf(f, "\ntrace_slots %llu walk_slots %llu nodes %llu leaf_steps %llu start_wait %llu top_visits %llu\n", cnt[11], cnt[5],
                        cnt[2], cnt[6], cnt[12], cnt[13]);
                fprintf(f, "wall_clock start %llu drained %llu last_exit %llu mean_exit %.1f waves %llu (ticks)\n", cnt[20], cnt[21],
                        cnt[22], cnt[24] ? (double)cnt[23] / (double)cnt[24] : 0.0, cnt[24]);
                fprintf(f, "lane_end_mean %.1f (ticks since start)\ntail_lane_end_log2_10us",
                        cnt[24] ? (double)cnt[26] / (64.0 * (double)cnt[24]) : 0.0);
                for (int k = 0; k < kTailBins; ++k) fprintf(f, " %llu", cnt[64 + k]);
                fprintf(f, "\ntail_wave_exit_log2_10us");
                for (int k = 0; k < kTailBins; ++k) fprintf(f, " %llu", cnt[80 + k]);
                fprintf(f, "\niters_by_deep_lanes 0:%llu 1-4:%llu 5-8:%llu more:%llu no_leaf %llu neither %llu\n", cnt[14],
                        cnt[15], cnt[16], cnt[17], cnt[18], cnt[19]);
                fclose(f);
            }
        }
    }
    float ms = 0.0f, kms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, F.ev0, F.ev1));
    if (F.kernel_events) HIP_TRY(hipEventElapsedTime(&kms, F.ek0, F.ek1));
    else kms = ms;   // (the tile kernel is the render's only launch)
    if (st) {
        st->seconds = ms * 1e-3;
        st->kernel_ms = kms;
        st->work_units = F.units;
        st->split_pixels = F.split;
        st->rays_traced = cnt[0];
        st->rays_reference = cnt[1];
        st->node_tests = cnt[2];
        st->tri_tests = cnt[3];
        st->samples = cnt[4];
        st->walk_lane_slots = cnt[5];
        st->leaf_steps = cnt[6];
        st->shade_lane_slots = cnt[7];
        st->accel_fallbacks = cnt[8];
        st->walk_cycles = cnt[9];
        st->shade_cycles = cnt[10];
        st->spill_entries = cnt[25];
        st->lds_node_tests = cnt[13];
        const uint64_t shard_px = cnt[4] / (uint64_t)(F.spp > 0 ? F.spp : 1);
        st->rays_nominal = shard_px * (uint64_t)F.spp * (uint64_t)(F.bounces + 1);
    }
    return PT_OK;
}

int pt_render_device(pt_ctx* c, const pt_params* p, const pt_camera* cam, float* d_out, void* stream, pt_stats* st)
{
    if (c && c->fl_n > 0)
        return pt::fail(PT_E_INVALID, "pt_render_device: %d asynchronous renders in flight (pt_render_wait first)", c->fl_n);
    if (int rc = pt_render_device_async(c, p, cam, d_out, stream)) return rc;
    return pt_render_wait(c, st);
}

}  // extern "C"

int pt::copy_to_host(void* dst, const void* src, size_t bytes, void* stream_v, void** pinned, size_t* pinned_bytes)
{
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_v);
    if (*pinned_bytes < bytes) {
        free_pinned(*pinned);
        *pinned = nullptr;
        *pinned_bytes = 0;
        if (hipHostMalloc(pinned, bytes, hipHostMallocDefault) != hipSuccess) {
            *pinned = nullptr;   // (no pinned memory: the runtime's own pageable path)
            HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            return PT_OK;
        }
        *pinned_bytes = bytes;
    }
    HIP_TRY(hipMemcpyAsync(*pinned, src, bytes, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    const unsigned nt = (unsigned)std::min<size_t>(pt::host_threads(), std::max<size_t>(1, bytes >> 21));   // >= 2 MB each
    const char* s = static_cast<const char*>(*pinned);
    char* d = static_cast<char*>(dst);
    auto part = [&](unsigned k) {
        const size_t b0 = (bytes * k / nt) & ~(size_t)4095, b1 = (k + 1 == nt) ? bytes : ((bytes * (k + 1) / nt) & ~(size_t)4095);
        memcpy(d + b0, s + b0, b1 - b0);
    };
    if (nt <= 1) {
        memcpy(d, s, bytes);
    } else {
        std::vector<std::thread> th;
        th.reserve(nt - 1);
        for (unsigned k = 1; k < nt; ++k) th.emplace_back(part, k);
        part(0);
        for (std::thread& t : th) t.join();
    }
    return PT_OK;
}

void pt::free_pinned(void* p)
{
    if (p) (void)hipHostFree(p);
}

extern "C" {

int pt_render(pt_ctx* c, const pt_params* p, const pt_camera* cam, float* out_rgb, pt_stats* st)
{
    if (!c || !p || !out_rgb) return pt::fail(PT_E_INVALID, "pt_render: null argument");
    if (p->width <= 0 || p->height <= 0) return pt::fail(PT_E_INVALID, "pt_render: bad image size");
    HIP_TRY(hipSetDevice(c->device));
    const size_t bytes = (size_t)p->width * (size_t)p->height * 3 * sizeof(float);
    if (c->scratch_bytes < bytes) {
        if (c->scratch_out) (void)hipFree(c->scratch_out);
        c->scratch_out = nullptr;
        c->scratch_bytes = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&c->scratch_out), bytes));
        c->scratch_bytes = bytes;
    }
    HIP_TRY(hipMemsetAsync(c->scratch_out, 0, bytes, nullptr));
    int rc = pt_render_device(c, p, cam, c->scratch_out, nullptr, st);
    if (rc != PT_OK) return rc;
    return pt::copy_to_host(out_rgb, c->scratch_out, bytes, nullptr, &c->pinned, &c->pinned_bytes);
}

}  // extern "C"

static size_t stack_words_per_lane(const pt_ctx* c)
{
    size_t per_lane = (size_t)(3 * c->acc4_depth + 4);
    if (per_lane < (size_t)(2 * (c->depth + 2))) per_lane = (size_t)(2 * (c->depth + 2));
    return per_lane;
}

static int ensure_spill(pt_ctx::Bufs& B, size_t words)
{
    if (B.spill_words >= words) return PT_OK;
    if (B.spill) (void)hipFree(B.spill);
    B.spill = nullptr;
    B.spill_words = 0;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&B.spill), words * 4));
    B.spill_words = words;
    return PT_OK;
}

static bool alloc_bufs(pt_ctx::Bufs& B)
{
    if (B.counters && B.tile_counter && B.pixel_counter) return true;
    // (all three or none: a partial failure is released, so the next call allocates again)
    for (void** q : {reinterpret_cast<void**>(&B.counters), reinterpret_cast<void**>(&B.tile_counter),
                     reinterpret_cast<void**>(&B.pixel_counter)})
        if (*q) { (void)hipFree(*q); *q = nullptr; }
    if (hipMalloc(reinterpret_cast<void**>(&B.counters), kCounterWords * sizeof(unsigned long long)) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&B.tile_counter), 16) == hipSuccess &&
        hipMalloc(reinterpret_cast<void**>(&B.pixel_counter), kQueueStride * (kQueues + 1) * 4) == hipSuccess)
        return true;
    for (void** q : {reinterpret_cast<void**>(&B.counters), reinterpret_cast<void**>(&B.tile_counter),
                     reinterpret_cast<void**>(&B.pixel_counter)})
        if (*q) { (void)hipFree(*q); *q = nullptr; }
    return false;
}

extern "C" int pt_trace(pt_ctx* c, uint32_t n, const float* rays, int32_t* tri_out, float* t_out, uint32_t flags)
{
    return pt_trace_counts(c, n, rays, tri_out, t_out, flags, nullptr, nullptr);
}

extern "C" int pt_tri_counts(pt_ctx* c, uint32_t* counts, uint32_t n)
{
    pt::clear_error();
    if (!c || !counts) return pt::fail(PT_E_INVALID, "pt_tri_counts: null argument");
    if (c->fl_n > 0) return pt::fail(PT_E_INVALID, "pt_tri_counts: renders in flight (pt_render_wait first)");
    if (n != c->num_tris) return pt::fail(PT_E_INVALID, "pt_tri_counts: n = %u, the scene has %u triangles", n, c->num_tris);
    if (n == 0) return PT_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpy(counts, c->tri_counts, (size_t)n * 4, hipMemcpyDeviceToHost));
    return PT_OK;
}

extern "C" int pt_trace_counts(pt_ctx* c, uint32_t n, const float* rays, int32_t* tri_out, float* t_out, uint32_t flags,
                               uint32_t* tri_counts, uint64_t* spill_entries)
{
    pt::clear_error();
    if (!c) return pt::fail(PT_E_INVALID, "pt_trace: null context");
    if (c->fl_n > 0) return pt::fail(PT_E_INVALID, "pt_trace: renders in flight (pt_render_wait first)");
    if (n == 0) return PT_OK;
    if (!rays || !tri_out || !t_out) return pt::fail(PT_E_INVALID, "pt_trace: null buffer");
    HIP_TRY(hipSetDevice(c->device));
    Args a;
    memset(&a, 0, sizeof(a));
    a.nodes = c->nodes; a.rnodes = c->rnodes; a.tris_leaf = c->tris_leaf; a.tris_orig = c->tris_orig;
    a.counters = c->rb[0].counters;
    a.spheres = c->spheres; a.num_spheres = c->num_spheres; a.num_tris = c->num_tris;
    a.sphere_mat_base = c->sphere_mat_base;
    memcpy(a.root, c->root, sizeof(a.root));
    memcpy(a.acc_root, c->acc_root, sizeof(a.acc_root));
    a.cull_rel = kCullRel;
    a.cull_abs = c->scene_extent * 1e-4f;
    a.scene_fast = c->scene_fast ? 1u : 0u;
    a.node_mask = c->node4_mask;
    a.nodes4 = c->nodes4;
    a.acc_tris = c->acc_tris;
    a.rparent = c->rparent;
    a.stack_words = (uint32_t)(c->depth + 2) * 64;
    if (a.stack_words < (uint32_t)kWaveLdsWords) a.stack_words = kWaveLdsWords;
    const size_t lds = (size_t)a.stack_words * 4 * 4;
    if (lds > 160 * 1024) return pt::fail(PT_E_BVH_DEPTH, "pt_trace: BVH depth %d too deep for the LDS stack", c->depth);
    uint32_t blocks = (n + 255) / 256;
    const uint32_t cap = (uint32_t)c->num_cus * 8u;
    if (blocks > cap) blocks = cap;
    if (int rc = ensure_spill(c->rb[0], stack_words_per_lane(c) * (size_t)blocks * 256)) return rc;
    a.spill = c->rb[0].spill;
    a.spill_stride = blocks * 256;
    float* d_rays = nullptr;
    int32_t* d_tri = nullptr;
    float* d_t = nullptr;
    uint32_t* d_cnt = nullptr;
    int rc = PT_OK;
    auto run = [&]() -> int {
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_rays), (size_t)n * 24));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_tri), (size_t)n * 4));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_t), (size_t)n * 4));
        HIP_TRY(hipMemcpy(d_rays, rays, (size_t)n * 24, hipMemcpyHostToDevice));
        HIP_TRY(hipMemset(c->rb[0].counters, 0, kCounterWords * sizeof(unsigned long long)));
        const bool count = tri_counts != nullptr || spill_entries != nullptr;
        if (tri_counts && c->num_tris > 0) {   // (own scratch: the last render's counts stay for pt_tri_counts)
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_cnt), (size_t)c->num_tris * 4));
            HIP_TRY(hipMemset(d_cnt, 0, (size_t)c->num_tris * 4));
            a.tri_counts = d_cnt;
        }
        const bool ref = (flags & PT_FLAG_REFERENCE_BVH) != 0;
        if (ref && count) hipLaunchKernelGGL((trace_rays<true, true>), dim3(blocks), dim3(256), lds, 0, a, d_rays, n, d_tri, d_t);
        else if (ref) hipLaunchKernelGGL((trace_rays<true, false>), dim3(blocks), dim3(256), lds, 0, a, d_rays, n, d_tri, d_t);
        else if (count) hipLaunchKernelGGL((trace_rays<false, true>), dim3(blocks), dim3(256), lds, 0, a, d_rays, n, d_tri, d_t);
        else hipLaunchKernelGGL((trace_rays<false, false>), dim3(blocks), dim3(256), lds, 0, a, d_rays, n, d_tri, d_t);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpy(tri_out, d_tri, (size_t)n * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(t_out, d_t, (size_t)n * 4, hipMemcpyDeviceToHost));
        if (tri_counts && c->num_tris > 0) {   // added to the caller's counts (kernel.cu:133 accumulates)
            std::vector<uint32_t> h(c->num_tris);
            HIP_TRY(hipMemcpy(h.data(), d_cnt, (size_t)c->num_tris * 4, hipMemcpyDeviceToHost));
            for (uint32_t k = 0; k < c->num_tris; ++k) tri_counts[k] += h[k];
        }
        if (spill_entries) {
            unsigned long long v = 0;
            HIP_TRY(hipMemcpy(&v, c->rb[0].counters + 25, sizeof(v), hipMemcpyDeviceToHost));
            *spill_entries = v;
        }
        return PT_OK;
    };
    rc = run();
    if (d_rays) (void)hipFree(d_rays);
    if (d_tri) (void)hipFree(d_tri);
    if (d_t) (void)hipFree(d_t);
    if (d_cnt) (void)hipFree(d_cnt);
    return rc;
}

extern "C" int pt_shard_pixels(int w, int h, int shard_index, int shard_count, int tile_w, int tile_h, uint32_t* out,
                               uint32_t cap, uint32_t* n_out)
{
    pt::clear_error();
    if (w <= 0 || h <= 0 || w > 65535 || h > 65535 || shard_count < 1 || shard_index < 0 || shard_index >= shard_count || !n_out)
        return pt::fail(PT_E_INVALID, "pt_shard_pixels: bad arguments");
    for (const int v : {tile_w, tile_h})
        if (v != 0 && (v < 8 || v > 256 || v % 8 != 0)) return pt::fail(PT_E_INVALID, "pt_shard_pixels: tile size %dx%d", tile_w, tile_h);
    TileMap m;
    m.w = w; m.h = h; m.shard_index = shard_index; m.shard_count = shard_count;
    m.tile_w = tile_w ? (uint32_t)tile_w : kTile;
    m.tile_h = tile_h ? (uint32_t)tile_h : kTile;
    m.tiles_x = ((uint32_t)w + m.tile_w - 1) / m.tile_w;
    const uint32_t ntiles = m.tiles_x * (((uint32_t)h + m.tile_h - 1) / m.tile_h);
    m.tile_bx = m.tile_w / kTile;
    m.tile_blocks = m.tile_bx * (m.tile_h / kTile);
    const uint32_t nts = (ntiles > (uint32_t)shard_index) ? (ntiles - (uint32_t)shard_index + (uint32_t)shard_count - 1) / (uint32_t)shard_count : 0u;
    const uint64_t slots = (uint64_t)nts * m.tile_w * m.tile_h;
    if ((uint64_t)(((uint32_t)h + m.tile_h - 1) / m.tile_h) * m.tiles_x * m.tile_w * m.tile_h > 0xffffffffull)
        return pt::fail(PT_E_INVALID, "pt_shard_pixels: %dx%d pads to more than 2^32-1 pixel slots", w, h);
    uint32_t n = 0;
    for (uint64_t q = 0; q < slots; ++q) {
        uint32_t px, py;
        if (!unit_pixel(m, (uint32_t)q, &px, &py)) continue;
        if (out) {
            if (n >= cap) return pt::fail(PT_E_INVALID, "pt_shard_pixels: buffer of %u entries too small", cap);
            out[n] = py * (uint32_t)w + px;
        }
        ++n;
    }
    *n_out = n;
    return PT_OK;
}

extern "C" int pt_tonemap_device(pt_ctx* c, const float* d_rgb, int w, int h, int32_t* d_codes, void* stream_v)
{
    pt::clear_error();
    if (!c || !d_rgb || !d_codes || w <= 0 || h <= 0) return pt::fail(PT_E_INVALID, "pt_tonemap_device: bad arguments");
    if (!c->tone_ok) return pt::fail(PT_E_INVALID, "pt_tonemap_device: host tone map not monotone; use pt_tonemap_u8");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_v);
    const size_t n = (size_t)w * (size_t)h * 3;
    size_t blocks = (n + 255) / 256;
    if (blocks > (size_t)c->num_cus * 32) blocks = (size_t)c->num_cus * 32;
    hipLaunchKernelGGL(tonemap_codes, dim3((unsigned)blocks), dim3(256), 0, stream, d_rgb, n, c->tone_thr, d_codes);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(stream));
    return PT_OK;
}

extern "C" int pt_tonemap(pt_ctx* c, const float* rgb, int w, int h, int32_t* codes)
{
    pt::clear_error();
    if (!c || !rgb || !codes || w <= 0 || h <= 0) return pt::fail(PT_E_INVALID, "pt_tonemap: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = (size_t)w * (size_t)h * 3;
    float* d_rgb = nullptr;
    int32_t* d_codes = nullptr;
    auto run = [&]() -> int {
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_rgb), n * sizeof(float)));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d_codes), n * sizeof(int32_t)));
        HIP_TRY(hipMemcpy(d_rgb, rgb, n * sizeof(float), hipMemcpyHostToDevice));
        if (int rc = pt_tonemap_device(c, d_rgb, w, h, d_codes, nullptr)) return rc;
        HIP_TRY(hipMemcpy(codes, d_codes, n * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; ++i)
            if (codes[i] == INT32_MAX) codes[i] = pt_tonemap_u8((double)rgb[i]);
        return PT_OK;
    };
    const int rc = run();
    if (d_rgb) (void)hipFree(d_rgb);
    if (d_codes) (void)hipFree(d_codes);
    return rc;
}
