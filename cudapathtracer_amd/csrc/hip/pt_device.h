// pt_device.h -- gfx950 device code of the path tracer: data layout in HBM, arithmetic
// helpers, XORWOW, slab/triangle tests and the two BVH walks.
//
// Arithmetic contract (DESIGN.md "Arithmetic spec"): the whole library is compiled with
// -ffp-contract=off, so every float/double expression below is evaluated as the reference's
// C++ spells it -- IEEE single/double ops in source order, correctly rounded '/' and sqrt --
// and matches the CPU oracle bit for bit.  Places that intentionally use FMA say so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptd {

constexpr float kMaxFloat = 100000.0f;        // limits.h:3 MAX_FLOAT
constexpr uint32_t kLeaf = 0x80000000u;       // limits.h:6 BVH_LEAF_FLAG
constexpr int kStack = 64;                    // kernel.cu:35 MAX_BVH_DEPTH

// ------------------------------------------------------------------ HBM layout
// Both children of one reference BVH node in one 64-B record (4 x 16-B loads).  Child ref:
// inner -> node index (same index as the reference's BFS array), leaf -> kLeaf | slot, where
// slot is the triangle's position in left-first DFS leaf order (its tie-break rank).
struct alignas(16) DNode {
    float4 a;   // c0.lo.xyz, c0.hi.x
    float4 b;   // c0.hi.yz, c1.lo.xy
    float4 c;   // c1.lo.z, c1.hi.xyz
    uint4 d;    // c0 ref, c1 ref, -, -
};
static_assert(sizeof(DNode) == 64, "node record is 64 B");

// The reference's own node (BVH.h:111-115), used by the reference-order walk.
struct alignas(16) RNode {
    float lo[3], hi[3];
    uint32_t left, right;
};
static_assert(sizeof(RNode) == 32, "reference node is 32 B");

// Intersection record: v0, e1 = v1-v0, e2 = v2-v0 (the exact subtractions triIntersect does,
// modelLoader.h:58-59, so precomputing them is bit-exact), original triangle id.
struct alignas(16) DTri {
    float4 a;   // v0.xyz, e1.x
    float4 b;   // e1.yz, e2.xy
    float4 c;   // e2.z, id, rank, parent (bits): rank = position in the reference's left-first DFS
                //   leaf order (tie-break), parent = the reference BVH node whose child it is
};
static_assert(sizeof(DTri) == 48, "triangle record is 48 B");

// Shading record by original triangle id: normal + material (modelLoader.h:14-19).
struct alignas(16) DShade {
    float nx, ny, nz;
    int32_t mat;
};

struct DMat {   // materialDesc (modelLoader.h:21-25)
    double albedo[3];
    double emission[3];
};

// Emissive triangle for the area-CDF pick (kernel.cu:468-495): area precomputed with the
// reference's float expression length(cross(a1,a2))/2; slot num_lights holds triangle 0,
// the reference's fallback when nothing is picked.
struct alignas(16) DLight {
    float area;
    int32_t tri;
    float v0[3], a1[3], a2[3];
    float pad;
};
static_assert(sizeof(DLight) == 48, "light record is 48 B");

struct Cam {    // camera.h:26-34
    float pos[3];
    float dist, focal, radius;
    int32_t w, h;
};

// ------------------------------------------------------------------ vec3 (vec3.h)
struct V3 { float x, y, z; };
__host__ __device__ __forceinline__ V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
__host__ __device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__host__ __device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__host__ __device__ __forceinline__ V3 operator*(V3 a, float f) { return v3(a.x * f, a.y * f, a.z * f); }
__host__ __device__ __forceinline__ V3 operator/(V3 a, float f) { return v3(a.x / f, a.y / f, a.z / f); }
__host__ __device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ __forceinline__ V3 cross(V3 a, V3 b)
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__host__ __device__ __forceinline__ float length(V3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
__host__ __device__ __forceinline__ V3 normalized(V3 v)
{
    float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return v3(v.x / len, v.y / len, v.z / len);
}

// ------------------------------------------------------------------ colour (color.h, f64)
struct C3 { double r, g, b; };
__device__ __forceinline__ C3 c3(double r, double g, double b) { C3 c; c.r = r; c.g = g; c.b = b; return c; }
__device__ __forceinline__ C3 cadd(C3 a, C3 b) { return c3(a.r + b.r, a.g + b.g, a.b + b.b); }
__device__ __forceinline__ C3 cmulf(C3 a, float f) { return c3(a.r * (double)f, a.g * (double)f, a.b * (double)f); }
__device__ __forceinline__ C3 cdivf(C3 a, float f) { return c3(a.r / (double)f, a.g / (double)f, a.b / (double)f); }
__device__ __forceinline__ C3 cmul(C3 a, C3 b) { return c3(a.r * b.r, a.g * b.g, a.b * b.b); }
__device__ __forceinline__ bool czero(C3 a) { return a.r == 0.0 && a.g == 0.0 && a.b == 0.0; }

// ------------------------------------------------------------------ deterministic sin/cos
// Double-precision Cody-Waite reduction + Taylor polynomials, rounded once to float; plain
// IEEE double ops in a fixed order, shared with the host (camera) and mirrored by the oracle.
__host__ __device__ __forceinline__ void det_sincos(float theta, float* s_out, float* c_out)
{
    const double x = (double)theta;
    const double kd = rint(x * 0.6366197723675814);
    const int k = (int)kd;
    const double r = (x - kd * 1.5707963267948966) - kd * 6.123233995736766e-17;
    const double r2 = r * r;
    double sp = 2.8114572543455206e-15;
    sp = sp * r2 + -7.647163731819816e-13;
    sp = sp * r2 + 1.6059043836821613e-10;
    sp = sp * r2 + -2.505210838544172e-08;
    sp = sp * r2 + 2.7557319223985893e-06;
    sp = sp * r2 + -0.0001984126984126984;
    sp = sp * r2 + 0.008333333333333333;
    sp = sp * r2 + -0.16666666666666666;
    const double sn = r + r * (r2 * sp);
    double cp = -1.5619206968586225e-16;
    cp = cp * r2 + 4.779477332387385e-14;
    cp = cp * r2 + -1.1470745597729725e-11;
    cp = cp * r2 + 2.08767569878681e-09;
    cp = cp * r2 + -2.755731922398589e-07;
    cp = cp * r2 + 2.48015873015873e-05;
    cp = cp * r2 + -0.001388888888888889;
    cp = cp * r2 + 0.041666666666666664;
    cp = cp * r2 + -0.5;
    const double cs = 1.0 + r2 * cp;
    double sv, cv;
    switch (k & 3) {
    case 0: sv = sn; cv = cs; break;
    case 1: sv = cs; cv = -sn; break;
    case 2: sv = -sn; cv = -cs; break;
    default: sv = -cs; cv = sn; break;
    }
    *s_out = (float)sv;
    *c_out = (float)cv;
}

// ------------------------------------------------------------------ XORWOW (cuRAND)
struct Rng {
    uint32_t d, v0, v1, v2, v3, v4;
};

__device__ __forceinline__ uint32_t rng_next(Rng& s)
{
    const uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1; s.v1 = s.v2; s.v2 = s.v3; s.v3 = s.v4;
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v4 + s.d;
}

// curand_uniform (kernel.cu:58): x * 2^-32 + 2^-33 in float, contracted as nvcc emits it.
__device__ __forceinline__ float rng_uniform(Rng& s)
{
    return __builtin_fmaf((float)rng_next(s), 2.3283064e-10f, 2.3283064e-10f / 2.0f);
}

// curand_init(seed, subsequence, 0) (kernel.cu:532): cuRAND seeding salts, then
// v <- A^(subsequence * 2^67) v through the tables J_k = A^(2^(67+k)) (160 rows x 5 words).
// curand_init(seed, subseq, 0) (kernel.cu:532): seed scrambling, then v <- J_k v for every set
// bit k of subseq, J_k = A^(2^(67+k)).  J_k is applied byte-sliced: jb holds, for each k and
// each of the 20 state bytes j, the 256 products J_k * (x << 8j) (5 words padded to 8), so a
// jump is 20 independent 32-B lookups XORed together -- no data-dependent bit loop.
constexpr int kJumpEntryWords = 8;
__device__ __forceinline__ uint32_t rng_seed_d(uint64_t seed)
{
    const uint32_t t0 = 1099087573u * ((uint32_t)seed ^ 0xaad26b49u);
    const uint32_t t1 = 2591861531u * ((uint32_t)(seed >> 32) ^ 0xf7dcefddu);
    return 6615241u + t1 + t0;
}
__device__ __forceinline__ void rng_init(Rng& s, uint64_t seed, uint32_t subseq, const uint32_t* __restrict__ jb)
{
    const uint32_t t0 = 1099087573u * ((uint32_t)seed ^ 0xaad26b49u);
    const uint32_t t1 = 2591861531u * ((uint32_t)(seed >> 32) ^ 0xf7dcefddu);
    s.d = 6615241u + t1 + t0;
    uint32_t v0 = 123456789u + t0, v1 = 362436069u ^ t0, v2 = 521288629u + t1, v3 = 88675123u ^ t1, v4 = 5783321u + t0;
    for (int k = 0; k < 32; ++k) {
        if (!((subseq >> k) & 1u)) continue;
        const uint32_t* m = jb + (size_t)k * (20 * 256 * kJumpEntryWords);
        uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
#pragma unroll
        for (int j = 0; j < 20; ++j) {
            const uint32_t w = (j < 4) ? v0 : (j < 8) ? v1 : (j < 12) ? v2 : (j < 16) ? v3 : v4;
            const uint32_t x = (w >> (8 * (j & 3))) & 255u;
            const uint32_t* e = m + ((size_t)j * 256 + x) * kJumpEntryWords;
            const uint4 q = *reinterpret_cast<const uint4*>(e);
            r0 ^= q.x; r1 ^= q.y; r2 ^= q.z; r3 ^= q.w; r4 ^= e[4];
        }
        v0 = r0; v1 = r1; v2 = r2; v3 = r3; v4 = r4;
    }
    s.v0 = v0; s.v1 = v1; s.v2 = v2; s.v3 = v3; s.v4 = v4;
}

// v <- M v for a GF(2) matrix M in byte-sliced form (m: 20 x 256 entries of kJumpEntryWords words,
// entry (j, x) = M * (x << 8j)): 20 independent lookups XORed together.
__device__ __forceinline__ void jump_apply(uint32_t v[5], const uint32_t* __restrict__ m)
{
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
#pragma unroll
    for (int j = 0; j < 20; ++j) {
        const uint32_t w = v[j >> 2];
        const uint32_t x = (w >> (8 * (j & 3))) & 255u;
        const uint32_t* e = m + ((size_t)j * 256 + x) * kJumpEntryWords;
        const uint4 q = *reinterpret_cast<const uint4*>(e);
        r0 ^= q.x; r1 ^= q.y; r2 ^= q.z; r3 ^= q.w; r4 ^= e[4];
    }
    v[0] = r0; v[1] = r1; v[2] = r2; v[3] = r3; v[4] = r4;
}

// ------------------------------------------------------------------ geometry tests
// triIntersect (modelLoader.h:49-83) on a precomputed {v0, e1, e2} record.
__device__ __forceinline__ float tri_t(V3 o, V3 d, V3 v0, V3 e1, V3 e2)
{
    const V3 q = cross(d, e2);
    const float a = dot(e1, q);
    if ((double)__builtin_fabsf(a) < 0.00001) return kMaxFloat;
    const V3 s = (o - v0) / a;
    const V3 r = cross(s, e1);
    const float b0 = dot(s, q);
    const float b1 = dot(r, d);
    const float b2 = 1.0f - b0 - b1;
    if (b0 < 0.0f) return kMaxFloat;
    if (b1 < 0.0f) return kMaxFloat;
    if (b2 < 0.0f) return kMaxFloat;
    return dot(e2, r);
}

__device__ __forceinline__ float tri_t_rec(V3 o, V3 d, const DTri* __restrict__ tr, uint32_t* id)
{
    const float4 a = tr->a, b = tr->b, c = tr->c;
    *id = __float_as_uint(c.y);
    return tri_t(o, d, v3(a.x, a.y, a.z), v3(a.w, b.x, b.y), v3(b.z, b.w, c.x));
}

// rayAABBIntersect (BVH.h:51-83): IEEE divisions, compare/swap with the reference's NaN
// behaviour.  Also returns a conservative entry/exit (NaN-ignoring max/min of the slab
// values) that the culled walk uses for ordering and distance culling only.
__device__ __forceinline__ bool slab_ref(V3 o, V3 d, float lx, float ly, float lz, float hx, float hy, float hz,
                                         float* t_in, float* t_out)
{
    float tmin = (lx - o.x) / d.x, tmax = (hx - o.x) / d.x, tt;
    if (tmin > tmax) { tt = tmin; tmin = tmax; tmax = tt; }
    float tymin = (ly - o.y) / d.y, tymax = (hy - o.y) / d.y;
    if (tymin > tymax) { tt = tymin; tymin = tymax; tymax = tt; }
    float tzmin = (lz - o.z) / d.z, tzmax = (hz - o.z) / d.z;
    if (tzmin > tzmax) { tt = tzmin; tzmin = tzmax; tzmax = tt; }
    *t_in = __builtin_fmaxf(__builtin_fmaxf(tmin, tymin), tzmin);
    *t_out = __builtin_fminf(__builtin_fminf(tmax, tymax), tzmax);
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    return true;
}

struct Counters {
    uint32_t nodes = 0;        // node records fetched (64 B culled walk, 32 B reference walk)
    uint32_t tris = 0;         // triangle records tested (48 B)
    uint32_t leaf_steps = 0;   // walk steps that tested at least one triangle
    uint32_t top = 0;          // BVH4 node visits served by the LDS copy of the tree's top
    uint32_t spills = 0;       // BVH4 stack entries written beyond the LDS ring (to the HBM spill column)
    uint32_t* tri_counts = nullptr;   // per-triangle tests by ORIGINAL id (kernel.cu:133 test[k] += 1), or none
    __device__ __forceinline__ void tri_tested(uint32_t id) const
    {
        if (tri_counts) atomicAdd(tri_counts + id, 1u);
    }
};

// ------------------------------------------------------------------ exact division, cheaply
// Markstein's correction: with y = RN(1/d), q0 = RN(x*y), r = x - d*q0 (exact by FMA),
// RN(q0 + r*y) == RN(x/d) -- the correctly rounded quotient the reference's '/' produces --
// whenever nothing under/overflows.  The walks use it only when every numerator is 0 or has
// magnitude >= 2^-80 and every divisor magnitude lies in [2^-100, 2^45]: guaranteed when all
// scene coordinates and the ray origin are 0 or in [2^-50, 2^20] and |d_k| >= 2^-100 (checked
// per scene at pt_create and per ray in ray_fast()); otherwise the wave takes the IEEE '/'
// path.  Verified bit-exact on 2e9 random pairs over those ranges.
__device__ __forceinline__ float div_mk(float x, float d, float y)
{
    const float q0 = x * y;
    const float r = __builtin_fmaf(-q0, d, x);
    // d = +-0: y = +-inf and x*y is exactly x/d (+-inf, or NaN for x = 0)
    return (d == 0.0f) ? q0 : __builtin_fmaf(r, y, q0);
}

__device__ __forceinline__ bool coord_ok(float v)
{
    const float a = __builtin_fabsf(v);
    return a == 0.0f || (a >= 0x1p-50f && a <= 0x1p20f);
}

__device__ __forceinline__ bool dir_ok(float v)
{
    const float a = __builtin_fabsf(v);
    return a == 0.0f || (a >= 0x1p-100f && a <= 0x1p45f);
}

__device__ __forceinline__ bool ray_fast(V3 o, V3 d)
{
    return coord_ok(o.x) && coord_ok(o.y) && coord_ok(o.z) && dir_ok(d.x) && dir_ok(d.y) && dir_ok(d.z);
}

// slab test of BVH.h:51-83; kMk selects the Markstein quotient (same bits as '/').
template <bool kMk>
__device__ __forceinline__ bool slab(V3 o, V3 d, V3 y, float lx, float ly, float lz, float hx, float hy, float hz,
                                     float* t_in, float* t_out)
{
    float tmin, tmax, tymin, tymax, tzmin, tzmax, tt;
    if (kMk) {
        tmin = div_mk(lx - o.x, d.x, y.x); tmax = div_mk(hx - o.x, d.x, y.x);
        tymin = div_mk(ly - o.y, d.y, y.y); tymax = div_mk(hy - o.y, d.y, y.y);
        tzmin = div_mk(lz - o.z, d.z, y.z); tzmax = div_mk(hz - o.z, d.z, y.z);
    } else {
        tmin = (lx - o.x) / d.x; tmax = (hx - o.x) / d.x;
        tymin = (ly - o.y) / d.y; tymax = (hy - o.y) / d.y;
        tzmin = (lz - o.z) / d.z; tzmax = (hz - o.z) / d.z;
    }
    if (tmin > tmax) { tt = tmin; tmin = tmax; tmax = tt; }
    if (tymin > tymax) { tt = tymin; tymin = tymax; tymax = tt; }
    if (tzmin > tzmax) { tt = tzmin; tzmin = tzmax; tzmax = tt; }
    *t_in = __builtin_fmaxf(__builtin_fmaxf(tmin, tymin), tzmin);
    *t_out = __builtin_fminf(__builtin_fminf(tmax, tymax), tzmax);
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    return true;
}

// Materialise a loaded value here: keeps the compiler from sinking the load into the branch
// that first uses it (which would turn one memory round trip into several dependent ones).
__device__ __forceinline__ void pin(float4& v)
{
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}
__device__ __forceinline__ void pin(uint4& v)
{
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}
// The same for a value that is only read afterwards: an input-only use (no register copies).
__device__ __forceinline__ void pin_use(const float4& v)
{
    asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
}
__device__ __forceinline__ void pin_use1(float v)
{
    asm volatile("" ::"v"(v));
}

// The smallest float whose double is >= 0.00001: for float a, (double)a < 0.00001 <=> a < kTriEps.
constexpr float kTriEps = 0x1.4f8b5ap-17f;

// RN(1/a) for 2^-100 <= |a| <= 2^100 from the hardware reciprocal and one Newton step:
// verified equal to IEEE 1.0f / a for every float of that range, both signs, on gfx950
// (tools/gpu/rcp_check.hip; DESIGN.md "Exact division").  Under the Markstein preconditions
// (coordinates <= 2^20, 2^-100 <= |d_k| <= 2^45) every divisor lies in it: direction
// components, and triangle determinants kTriEps <= |a| <= ~2^88.
__device__ __forceinline__ float rcp_rn(float a)
{
    const float y0 = __builtin_amdgcn_rcpf(a);
    const float e = __builtin_fmaf(-a, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}
// IEEE 1/d for d = 0 (+-inf) or 2^-100 <= |d| <= 2^100
__device__ __forceinline__ float rcp_or_inf(float d)
{
    return (d == 0.0f) ? __builtin_copysignf(INFINITY, d) : rcp_rn(d);
}
// Double-precision Markstein quotient: with y = RN(1/d) (an IEEE division), q0 = RN(x*y),
// r = x - d*q0 (exact by FMA), RN(q0 + r*y) == RN(x/d) for finite x, d without under/overflow.
// quot_ok(x): x is 0 or 2^-969 <= |x| <= 2^1000, so that for the divisors used here (integers
// 1..2^24) every quotient and intermediate is a normal double.
__device__ __forceinline__ bool quot_ok(double x)
{
    const double ax = __builtin_fabs(x);
    return x == 0.0 || (ax >= 0x1p-969 && ax <= 0x1p1000);
}
__device__ __forceinline__ double div_mk_d(double x, double d, double y)
{
    const double q0 = x * y;
    return __builtin_fma(__builtin_fma(-q0, d, x), y, q0);
}
// div_mk for a divisor known to be nonzero
__device__ __forceinline__ float div_mk_nz(float x, float d, float y)
{
    const float q0 = x * y;
    return __builtin_fmaf(__builtin_fmaf(-q0, d, x), y, q0);
}

// Packed f32 pairs (VOP3P): one v_pk_* instruction performs two independent IEEE f32 operations,
// each bit-identical to the scalar instruction (same rounding, same denormal mode; no
// contraction).  op_sel / op_sel_hi pick, per result half, the lo or hi word of each source
// (so swizzles and broadcasts are free); neg_lo / neg_hi negate a source for that half
// (a + (-b) is IEEE a - b, and (-a) + b is b - a).
typedef float f2 __attribute__((ext_vector_type(2)));
#define PK2(op, mods, a, b)                                                                   \
    ({                                                                                        \
        f2 r_;                                                                                \
        asm("v_pk_" op "_f32 %0, %1, %2 " mods : "=v"(r_) : "v"(a), "v"(b));                  \
        r_;                                                                                   \
    })
#define PK3(op, mods, a, b, c)                                                                \
    ({                                                                                        \
        f2 r_;                                                                                \
        asm("v_pk_" op "_f32 %0, %1, %2, %3 " mods : "=v"(r_) : "v"(a), "v"(b), "v"(c));      \
        r_;                                                                                   \
    })
__device__ __forceinline__ f2 bcast(float x)   // x in the lo word (the hi word is never read)
{
    f2 r;
    r.x = x;
    return r;
}

// Render-path triangle record (acc_tris) in registers: the words are permuted so that the
// operand pairs of the packed test sit in aligned register pairs:
//   A = {v0.x, v0.y, e1.x, e1.y}, B = {e2.x, e2.y, v0.z, e1.z}, C = {e2.z, id, rank, parent};
// the test reads A, B and e2.z only (36 B: vector-memory data return is paid per byte of the whole
// wave-instruction, so the third load is a single dword).
// triIntersect (modelLoader.h:49-83) with RN(1/a) and Markstein quotients, the x/y halves of every
// vector expression as one packed op: per component the same IEEE operations in the same order
// as tri_hit<true> (dot = (x*x' + y*y') + z*z'; cross component = product - product), i.e. the
// same bits.  O, DD = {o.x, o.y}, {d.x, d.y}.
__device__ __forceinline__ float tri_hit_pk(f2 O, float oz, f2 DD, float dz, float4 A, float4 B, float e2z)
{
    const f2 V0 = {A.x, A.y}, E1 = {A.z, A.w}, E2 = {B.x, B.y}, VZ = {B.z, B.w}, CZ = bcast(e2z);
    const float v0z = B.z, e1z = B.w;
    // q = cross(d, e2)
    const f2 P1 = PK2("mul", "op_sel:[1,0] op_sel_hi:[0,0]", DD, CZ);          // {dy*e2z, dx*e2z}
    const f2 P2 = PK2("mul", "op_sel:[0,1] op_sel_hi:[0,0]", bcast(dz), E2);   // {dz*e2y, dz*e2x}
    const f2 Q = PK2("add", "neg_lo:[0,1] neg_hi:[1,0]", P1, P2);              // {qx, qy}
    const f2 P3 = PK2("mul", "op_sel:[0,1] op_sel_hi:[1,0]", DD, E2);          // {dx*e2y, dy*e2x}
    const float qz = P3.x - P3.y;
    const f2 EQ = PK2("mul", "", E1, Q);
    const float a = (EQ.x + EQ.y) + e1z * qz;                                   // dot(e1, q)
    if (__builtin_fabsf(a) < kTriEps) return kMaxFloat;   // == (double)|a| < 0.00001, NaN included
    // s = (o - v0) / a
    const f2 W = PK2("add", "neg_lo:[0,1] neg_hi:[0,1]", O, V0);
    const float wz = oz - v0z;
    const float ya = rcp_rn(a);
    const f2 Q0 = PK2("mul", "op_sel_hi:[1,0]", W, bcast(ya));
    const f2 RR = PK3("fma", "op_sel_hi:[1,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]", Q0, bcast(a), W);
    const f2 S = PK3("fma", "op_sel_hi:[1,0,1]", RR, bcast(ya), Q0);           // div_mk_nz(w.xy, a, ya)
    const float sz = div_mk_nz(wz, a, ya);
    // r = cross(s, e1)
    const f2 R1 = PK2("mul", "op_sel:[1,1] op_sel_hi:[0,1]", S, VZ);           // {sy*e1z, sx*e1z}
    const f2 R2 = PK2("mul", "op_sel:[0,1] op_sel_hi:[0,0]", bcast(sz), E1);   // {sz*e1y, sz*e1x}
    const f2 R = PK2("add", "neg_lo:[0,1] neg_hi:[1,0]", R1, R2);              // {rx, ry}
    const f2 R3 = PK2("mul", "op_sel:[0,1] op_sel_hi:[1,0]", S, E1);           // {sx*e1y, sy*e1x}
    const float rz = R3.x - R3.y;
    const f2 SQ = PK2("mul", "", S, Q);
    const float b0 = (SQ.x + SQ.y) + sz * qz;                                   // dot(s, q)
    const f2 RD = PK2("mul", "", R, DD);
    const float b1 = (RD.x + RD.y) + rz * dz;                                   // dot(r, d)
    const float b2 = 1.0f - b0 - b1;
    if (b0 < 0.0f) return kMaxFloat;
    if (b1 < 0.0f) return kMaxFloat;
    if (b2 < 0.0f) return kMaxFloat;
    const f2 ER = PK2("mul", "", E2, R);
    return (ER.x + ER.y) + e2z * rz;                                            // dot(e2, r)
}

// triIntersect (modelLoader.h:49-83); kMk: one IEEE reciprocal of `a`, Markstein quotients.
template <bool kMk>
__device__ __forceinline__ float tri_hit(V3 o, V3 d, const DTri* __restrict__ tr, uint32_t* id)
{
    const float4 A = tr->a, B = tr->b, C = tr->c;
    *id = __float_as_uint(C.y);
    const V3 v0 = v3(A.x, A.y, A.z), e1 = v3(A.w, B.x, B.y), e2 = v3(B.z, B.w, C.x);
    const V3 q = cross(d, e2);
    const float a = dot(e1, q);
    if ((double)__builtin_fabsf(a) < 0.00001) return kMaxFloat;
    const V3 w = o - v0;
    V3 s;
    if (kMk) {
        const float ya = 1.0f / a;
        s = v3(div_mk(w.x, a, ya), div_mk(w.y, a, ya), div_mk(w.z, a, ya));
    } else {
        s = w / a;
    }
    const V3 r = cross(s, e1);
    const float b0 = dot(s, q);
    const float b1 = dot(r, d);
    const float b2 = 1.0f - b0 - b1;
    if (b0 < 0.0f) return kMaxFloat;
    if (b1 < 0.0f) return kMaxFloat;
    if (b2 < 0.0f) return kMaxFloat;
    return dot(e2, r);
}

// ------------------------------------------------------------------ 4-wide render-path walk
// Node of the render-path BVH4 (collapsed SAH BVH): 4 child boxes SoA + 4 child refs, 128 B.
struct alignas(16) DNode4 {
    float4 lox, loy, loz, hix, hiy, hiz;
    uint4 child;     // inner index, kLeaf | slot, or 0xffffffff (empty); leaf children first, with
                     // consecutive triangle slots (child k of a node's leaves at slot base + k)
    uint4 pad;
};
static_assert(sizeof(DNode4) == 128, "BVH4 node is 128 B");
constexpr uint32_t kEmpty = 0xffffffffu;
constexpr uint32_t kNone = 0xffffffffu;    // no node / no leaf pending
constexpr int kLeafRing = 4;               // LDS leaf-queue entries per lane (one per node with entered leaves)
constexpr int kRing = 16;                 // LDS stack entries per lane; deeper entries spill to HBM

struct W4 {
    V3 inv;              // RN(1/d): also the Markstein reciprocal for the exact checks
    V3 oi;               // o * inv, for the conservative box test t = fma(b, inv, -oi)
    uint32_t node;       // next node to visit, kNone = pop one
    uint32_t leaf;       // leaves to test: (first slot << 8) | mask of the entered leaves' slots; none
                         // pending when the mask is 0 (leaf4_pending)
    int32_t sp;          // node stack depth
    int32_t lsp;         // leaf entries queued in the LDS leaf ring (besides `leaf`)
    float best_t;
    uint32_t best_slot;  // render-path triangle slot of the best hit, kNone = none
    uint32_t nx, ny, nz; // byte offsets in DNode4 of the near plane per axis (lo, or hi for inv < 0)
    float occ;           // walk4_step<kAnyHit>: a hit with t <= occ ends the walk (any-hit); unused otherwise
};

// The exact reference test a winner must pass (DESIGN.md "Traversal" 2): the reference slab test
// on its reference parent -- or, when a direction component is 0 (NaN slab values possible),
// on every ancestor up the reference tree.
__device__ __forceinline__ bool ref_tested(uint32_t parent, V3 o, V3 d,
                                           const RNode* __restrict__ rnodes, const uint32_t* __restrict__ rparent)
{
    const bool zero_dir = d.x == 0.0f || d.y == 0.0f || d.z == 0.0f;
    const V3 y = v3(rcp_or_inf(d.x), rcp_or_inf(d.y), rcp_or_inf(d.z));   // == IEEE 1/d: div_mk's y
    uint32_t n = parent;
    for (;;) {
        const RNode* p = rnodes + n;
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(&p->hi[1]);
        float ti, to;
        if (!slab<true>(o, d, y, a.x, a.y, a.z, a.w, b.x, b.y, &ti, &to)) return false;
        if (!zero_dir || n == 0u) return true;
        n = rparent[n];
    }
}

// The same with the reference parent's record already fetched (a, b: its first two 16-B words; a
// per-slot copy, so it arrives with the winner's ids instead of behind them).
__device__ __forceinline__ bool ref_tested_box(float4 a, float4 b, uint32_t parent, V3 o, V3 d,
                                               const RNode* __restrict__ rnodes, const uint32_t* __restrict__ rparent)
{
    const bool zero_dir = d.x == 0.0f || d.y == 0.0f || d.z == 0.0f;
    const V3 y = v3(rcp_or_inf(d.x), rcp_or_inf(d.y), rcp_or_inf(d.z));
    float ti, to;
    if (!slab<true>(o, d, y, a.x, a.y, a.z, a.w, b.x, b.y, &ti, &to)) return false;
    if (!zero_dir || parent == 0u) return true;
    return ref_tested(rparent[parent], o, d, rnodes, rparent);
}

// leaf queue entry: (the node's first leaf slot << kLeafBits) | mask of the entered leaves' slots
// (a node's leaf children hold at most kLeafBits triangles; slots < 2^(31 - kLeafBits))
constexpr uint32_t kLeafBits = 8;
__device__ __forceinline__ bool leaf4_pending(const W4& w) { return (w.leaf & ((1u << kLeafBits) - 1u)) != 0u; }
// the pending entry's lowest entered leaf slot (the mask is the low 4 bits: the word's lowest set
// bit); an opaque v_ffbl so that the compiler recomputes it instead of keeping it live
__device__ __forceinline__ uint32_t leaf4_slot(const W4& w)
{
    uint32_t b;
    asm volatile("v_ffbl_b32 %0, %1" : "=v"(b) : "v"(w.leaf));
    return (w.leaf >> kLeafBits) + b;
}

// walk4_begin in two halves: the ray-independent reset, and the per-ray reciprocals / plane
// offsets (the path-pool kernel runs the latter after the first node fetch is in flight).
__device__ __forceinline__ void walk4_reset(W4& w)
{
    w.node = 0; w.leaf = 0; w.sp = 0; w.lsp = 0;
    w.best_t = kMaxFloat; w.best_slot = kNone;
}
__device__ __forceinline__ void walk4_setup(W4& w, V3 o, V3 d)
{
    // Conservative slab values are lo*inv - o*inv (one FMA).  A zero component would make that
    // inf - inf = NaN on one plane and -inf on the other, which min/max cannot repair, so the
    // reciprocal is clamped to +-2^100: o*inv stays finite (|o| <= 2^20), and the inflated boxes
    // keep every plane >= margin from an origin inside the true slab, so the signs -- hence
    // "inside: unbounded, outside: rejected" -- come out right.  Exact tests use 1/d itself.
    w.inv = v3(rcp_rn(d.x), rcp_rn(d.y), rcp_rn(d.z));   // ray_fast: d_k is 0 or in rcp_rn's range
    if (d.x == 0.0f) w.inv.x = __builtin_copysignf(0x1p100f, d.x);   // (1/+-0 = +-inf: same sign as d)
    if (d.y == 0.0f) w.inv.y = __builtin_copysignf(0x1p100f, d.y);
    if (d.z == 0.0f) w.inv.z = __builtin_copysignf(0x1p100f, d.z);
    w.oi = v3(o.x * w.inv.x, o.y * w.inv.y, o.z * w.inv.z);
    w.nx = (w.inv.x < 0.0f) ? 48u : 0u;    // hix : lox  (the far plane is at nx ^ 48)
    w.ny = (w.inv.y < 0.0f) ? 64u : 16u;   // hiy : loy  (ny ^ 80)
    w.nz = (w.inv.z < 0.0f) ? 80u : 32u;   // hiz : loz  (nz ^ 112)
}
// Only rays satisfying ray_fast() walk the BVH4 (all exact tests use Markstein quotients);
// the others take trace_slow() below.  Returns the conservative root test.
__device__ __forceinline__ bool walk4_begin(W4& w, V3 o, V3 d, const float* root, float cull_abs)
{
    walk4_setup(w, o, d);
    walk4_reset(w);
    // conservative root test (boxes inflated; NaN planes are ignored by min/max)
    const float x0 = __builtin_fmaf(root[0], w.inv.x, -w.oi.x), x1 = __builtin_fmaf(root[3], w.inv.x, -w.oi.x);
    const float y0 = __builtin_fmaf(root[1], w.inv.y, -w.oi.y), y1 = __builtin_fmaf(root[4], w.inv.y, -w.oi.y);
    const float z0 = __builtin_fmaf(root[2], w.inv.z, -w.oi.z), z1 = __builtin_fmaf(root[5], w.inv.z, -w.oi.z);
    const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(x0, x1), __builtin_fminf(y0, y1)), __builtin_fminf(z0, z1));
    const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(x0, x1), __builtin_fmaxf(y0, y1)), __builtin_fmaxf(z0, z1));
    return !(tn > tf) && !(tf < -cull_abs);
}

// Conservative test of two child boxes (packed: one v_pk_fma_f32 per plane pair).  The near /
// far planes were picked per ray by the load offsets, so t_near <= t_far per axis already (FMA
// rounding is monotonic and lo <= hi): the entry is max3 of the near values, the exit min3 of the
// far ones, and no NaN can arise (finite bounds, |inv| <= 2^100).  A box is entered iff
// max(entry, 0) <= min(exit, limit), i.e. entry <= exit, exit >= 0 and entry <= limit.
// Clamping at 0 (not at -cull_abs) is conservative: a triangle the reference accepts (t > 0) lies
// inside its box, which is inflated by the margin m (accel_build.cpp), so the exit is >= t + m > 0
// exactly and the computed exit's rounding error (~2^-23 of the plane magnitudes) is far below m.
// The clamped entry (>= 0) is also the stack key's distance.
__device__ __forceinline__ f2 pk_fma(f2 a, float b, float c)
{
    return __builtin_elementwise_fma(a, f2{b, b}, f2{c, c});
}
// max/min of values known not to be NaN, as bare v_max3/v_min3 (IEEE mode would otherwise
// canonicalize each operand the compiler cannot prove canonical, e.g. packed-FMA halves).
__device__ __forceinline__ float entry4(float a, float b, float c)
{
    float m, r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(a), "v"(b), "v"(c));
    asm("v_max_f32_e32 %0, 0, %1" : "=v"(r) : "v"(m));
    return r;
}
__device__ __forceinline__ float exit4(float a, float b, float c, float limit)
{
    float m, r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(a), "v"(b), "v"(c));
    asm("v_min_f32_e32 %0, %1, %2" : "=v"(r) : "v"(limit), "v"(m));
    return r;
}
// entry distances (>= 0) and entered flags of two children
__device__ __forceinline__ void box_enter2(const W4& w, f2 nx, f2 ny, f2 nz, f2 fx, f2 fy, f2 fz, float limit,
                                           float& t0, float& t1, bool& e0, bool& e1)
{
    const f2 ax = pk_fma(nx, w.inv.x, -w.oi.x), ay = pk_fma(ny, w.inv.y, -w.oi.y), az = pk_fma(nz, w.inv.z, -w.oi.z);
    const f2 bx = pk_fma(fx, w.inv.x, -w.oi.x), by = pk_fma(fy, w.inv.y, -w.oi.y), bz = pk_fma(fz, w.inv.z, -w.oi.z);
    t0 = entry4(ax.x, ay.x, az.x);
    t1 = entry4(ax.y, ay.y, az.y);
    e0 = t0 <= exit4(bx.x, by.x, bz.x, limit);
    e1 = t1 <= exit4(bx.y, by.y, bz.y, limit);
}
// x * 48 as (x << 5) + (x << 4): two full-rate ops instead of a quarter-rate v_mul_lo_u32
__device__ __forceinline__ uint32_t mul48(uint32_t x)
{
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 5, %2" : "=v"(r) : "v"(x), "v"(x << 4));
    return r;
}
__device__ __forceinline__ float4 ld_f4(const void* base, uint32_t off)
{
    return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(base) + off);
}
__device__ __forceinline__ uint4 ld_u4(const void* base, uint32_t off)
{
    return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(base) + off);
}
// The same with the address space explicit (LDS: ds_read_b128; global: global_load_dwordx4), so
// that the two sides of a branch can never be merged into one flat load.
typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 lds_f4(const char* base, uint32_t off)
{
    const f4v v = *(__attribute__((address_space(3))) const f4v*)(base + off);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 lds_u4(const char* base, uint32_t off)
{
    const u4v v = *(__attribute__((address_space(3))) const u4v*)(base + off);
    return make_uint4(v.x, v.y, v.z, v.w);
}
// the same at a 32-bit LDS byte address (constant offsets added to it fold into the instruction)
__device__ __forceinline__ uint32_t lds_addr(const char* p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ float4 lds_f4a(uint32_t a)
{
    const f4v v = *(__attribute__((address_space(3))) const f4v*)(uintptr_t)a;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 lds_u4a(uint32_t a)
{
    const u4v v = *(__attribute__((address_space(3))) const u4v*)(uintptr_t)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}
// a - b as one opaque v_sub (the compiler would otherwise form -b and add it)
__device__ __forceinline__ uint32_t vsub_u32(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_sub_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float4 glb_f4(const void* base, uint32_t off)
{
    const f4v v = *(__attribute__((address_space(1))) const f4v*)(reinterpret_cast<const char*>(base) + off);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 glb_u4(const void* base, uint32_t off)
{
    const u4v v = *(__attribute__((address_space(1))) const u4v*)(reinterpret_cast<const char*>(base) + off);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Per wave, LDS holds a node ring of kRing x 64 words followed by a leaf ring of kLeafRing x 64;
// `ring` points at this lane's word 0 (wave base + lane).
// The lane's HBM spill column (entry k >= kRing at spill()[(k - kRing) * stride]) is addressed from
// a byte offset the kernel keeps in a register anyway (its shading record's lane offset), masked,
// so the walk holds no 64-bit spill pointer.
struct Stack4 {
    uint32_t* ring;            // LDS: node entry k at ring[(k % kRing) * 64], queued leaf k at ring[(kRing + k) * 64]
    uint32_t* spill_base;      // HBM (uniform)
    const uint32_t* lane_off;  // -> lane byte offset (a caller variable), & off_mask
    uint32_t off_mask;
    uint32_t off_shift = 0;      // lane byte offset = (*lane_off & off_mask) >> off_shift
    uint32_t stride;
    const char* top = nullptr;   // LDS copy of BVH4 nodes 0..ntop-1 (kTopNodeBytes each), or none
    uint32_t ntop = 0;
    __device__ __forceinline__ uint32_t* spill() const
    {
        return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(spill_base) + ((*lane_off & off_mask) >> off_shift));
    }
};
constexpr int kWaveLdsWords = (kRing + kLeafRing) * 64;
// BVH4 nodes 0..top-1 (the best-first top of the tree, pt_create) are staged in the block's LDS
// by the wavefront kernel, 112 B each (the node without its pad; stride 28 dwords, so 16
// consecutive nodes occupy disjoint banks): lanes visiting them read LDS instead of issuing
// vector-memory loads -- the kernel's limiting pipe (TA/TD, DESIGN.md "Measurement").
constexpr uint32_t kTopNodeBytes = 112;
// what fits next to the rings with 5 blocks of 256 threads per CU: LDS is granted in 1280-B granules,
// 32000 B per block = 4 x 5120 B of rings + 160 B of counters + 208 B of light-probe emitters
// (pt_render.hip) + 240 B of NEE light records + 97 x 112 B
constexpr uint32_t kTopNodesMax = 97;

template <bool kCount>
__device__ __forceinline__ void push4(W4& w, const Stack4& S, uint32_t e, Counters& cnt)
{
    const int slot = (w.sp & (kRing - 1)) * 64;   // sp >= 0, kRing a power of two
    if (w.sp >= kRing) {
        S.spill()[(size_t)(w.sp - kRing) * S.stride] = S.ring[slot];
        if (kCount) ++cnt.spills;
    }
    S.ring[slot] = e;
    ++w.sp;
}

__device__ __forceinline__ uint32_t pop4(W4& w, const Stack4& S)
{
    --w.sp;
    const int slot = (w.sp & (kRing - 1)) * 64;
    const uint32_t e = S.ring[slot];
    if (w.sp >= kRing) S.ring[slot] = S.spill()[(size_t)(w.sp - kRing) * S.stride];
    return e;
}

// One BVH4 node visit on the loaded node (planes, child words): the four box tests, the entered
// leaves queued as one entry, the entered inner children pushed far-to-near, the nearest one next.
template <bool kCount>
__device__ __forceinline__ void visit4(W4& w, const float4& NX, const float4& FX, const float4& NY, const float4& FY,
                                       const float4& NZ, const float4& FZ, const uint4& ch, const Stack4& S,
                                       float cull_rel, uint32_t node_mask, Counters& cnt)
{
    const float lim = w.best_t * cull_rel;
    // empty slots hold a box no ray enters (accel_build.cpp), so all four tests run unguarded
    float t0, t1, t2, t3;
    bool e0, e1, e2, e3;
    box_enter2(w, f2{NX.x, NX.y}, f2{NY.x, NY.y}, f2{NZ.x, NZ.y}, f2{FX.x, FX.y}, f2{FY.x, FY.y}, f2{FZ.x, FZ.y},
               lim, t0, t1, e0, e1);
    box_enter2(w, f2{NX.z, NX.w}, f2{NY.z, NY.w}, f2{NZ.z, NZ.w}, f2{FX.z, FX.w}, f2{FY.z, FY.w}, f2{FZ.z, FZ.w},
               lim, t2, t3, e2, e3);
    uint32_t r0 = ch.x, r1 = ch.y, r2 = ch.z, r3 = ch.w;
    // entered leaf children as one queue entry: the node's leaf triangles have consecutive
    // slots from its first (leaf children come first; each leaf child's word carries its slot
    // bits), so the entry is that slot and an 8-bit mask
    // (ek: child k entered, lk: child k is a leaf; both also select the stack keys below)
    const bool l0 = (int32_t)r0 < 0, l1 = (int32_t)r1 < 0, l2 = (int32_t)r2 < 0, l3 = (int32_t)r3 < 0;
    // a leaf child's word is kLeaf | first slot << kLeafBits | its slot bits, the first slot
    // being the node's for all its leaf children: the OR of the entered leaf children's words
    // is the queue entry (with kLeaf set)
    const uint32_t lw = (e0 && l0 ? r0 : 0u) | (e1 && l1 ? r1 : 0u) | (e2 && l2 ? r2 : 0u) | (e3 && l3 ? r3 : 0u);
    if ((lw & ((1u << kLeafBits) - 1u)) != 0u) {
        const uint32_t e = lw & ~kLeaf;
        if (!leaf4_pending(w)) w.leaf = e;
        else { S.ring[(kRing + w.lsp) * 64] = e; ++w.lsp; }
    }
    // inner children, nearest first.  Each entered child becomes a key (entry distance, >= 0,
    // truncated to the bits above node_mask | its child word): non-negative floats order like their
    // bit patterns, so four u32 min/max pairs sort the keys by distance.  An inner child's word is its
    // node index, so its key is >= 0 as an int; a leaf child's word carries kLeaf (bit 31), so its key
    // sorts after every inner key, and a box not entered is ~0 and sorts last: a key is a stack entry
    // iff it is >= 0 as an int -- no per-child leaf test (round 6: 3 VALU fewer per step, +0.3-0.4% at
    // C3, profiles/r06_leafkey).
    auto key = [&](float t, uint32_t r, bool e) -> uint32_t {
        return e ? ((__float_as_uint(t) & ~node_mask) | r) : kNone;
    };
    auto valid = [](uint32_t k) { return (int32_t)k >= 0; };
    uint32_t k0 = key(t0, r0, e0), k1 = key(t1, r1, e1), k2 = key(t2, r2, e2), k3 = key(t3, r3, e3);
    auto ksort = [](uint32_t& a, uint32_t& b) { const uint32_t lo = min(a, b); b = max(a, b); a = lo; };
    ksort(k0, k1); ksort(k2, k3); ksort(k0, k2); ksort(k1, k3); ksort(k1, k2);
    if (__ballot(w.sp > kRing - 3) == 0ull) {
        // no ring wrap-around possible in this wave: the stack entries (a sorted prefix) go to
        // slots sp.. far-to-near with three unconditional writes (the slots above the new top
        // are free)
        const bool v1 = valid(k1), v2 = valid(k2), v3 = valid(k3);
        uint32_t* const top = S.ring + w.sp * 64;
        top[0] = v3 ? k3 : (v2 ? k2 : k1);
        top[64] = v3 ? k2 : k1;
        top[128] = k1;
        w.sp += (int)v1 + (int)v2 + (int)v3;
    } else {
        if (valid(k3)) push4<kCount>(w, S, k3, cnt);
        if (valid(k2)) push4<kCount>(w, S, k2, cnt);
        if (valid(k1)) push4<kCount>(w, S, k1, cnt);
    }
    w.node = valid(k0) ? (k0 & node_mask) : kNone;
}
// After a step: take the next queued leaf entry when the pending one is done, and pop the next stack
// entry not culled by the best hit when there is no node to visit.
__device__ __forceinline__ void advance4(W4& w, const Stack4& S, float cull_rel, uint32_t node_mask)
{
    if (!leaf4_pending(w) && w.lsp > 0) {
        --w.lsp;
        w.leaf = S.ring[(kRing + w.lsp) * 64];
    }
    if (w.node == kNone) {
        while (w.sp > 0) {
            const uint32_t e = pop4(w, S);
            if (__uint_as_float(e & ~node_mask) > w.best_t * cull_rel) continue;
            w.node = e & node_mask;
            break;
        }
    }
}

// One walk step.  Returns true while the walk continues.
// A step fetches the next node AND the next pending leaf triangle in one memory round trip, tests
// the triangle, then the node's four child boxes; entered leaf children are queued (tested in
// later steps, overlapped with later node fetches), inner children are visited near-first.
// Deferring a leaf test only delays best_t improvements, i.e. culls less: the result is the
// same exact minimum.  A node is visited only while the leaf queue has room for its children.
// `setup(w)` runs once the step's fetches are issued (the pool kernel fetches a new ray there and
// runs walk4_setup, so the ray's round trip overlaps the root node's).
struct NoSetup {
    __device__ void operator()(W4&) const {}
};
// kTop: the caller guarantees S.ntop >= 1 (no per-step test of an empty LDS top).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wsometimes-uninitialized"   // (a lane's triangle words, read only if it has a leaf)
// kAnyHit: the walk ends at the first hit with t <= w.occ (integrator 1's visibility rays: any such hit
// decides "occluded"; the winner check still runs on it).
// kUniform (integrator 0's walks, the batched traces): every lane issues the triangle's loads and then the
// node's, as buffer loads -- a lane without a triangle (or node) at an out-of-range offset, which reads
// nothing and returns zeros -- so no exec-masked branch hides how many loads follow the triangle's: the
// test waits for the triangle alone (vmcnt(7)) and runs under the node's round trip instead of after it
// (the compiler had to wait for everything at the join behind the masked node loads).  The node is then
// always read from memory, not from the LDS top (the top's hot lines hit L2): C3 +1.5% (5630 -> 5713,
// same box, alternated, profiles/r03_uni).  Integrator 1 (kAnyHit) keeps the LDS top: bound by bytes, it
// lost 2.7% this way.
template <bool kCount, bool kTop = false, class Setup = NoSetup, bool kAnyHit = false, bool kUniform = !kAnyHit>
__device__ __forceinline__ bool walk4_step(W4& w, V3 o, V3 d, const DNode4* __restrict__ nodes,
                                           const DTri* __restrict__ tris, const Stack4& S, float cull_rel,
                                           float cull_abs, uint32_t node_mask, Counters& cnt,
                                           const Setup& setup = Setup())
{
    const bool visit = (w.node != kNone) && (w.lsp <= kLeafRing - 1);
    const bool leaf = leaf4_pending(w);
    // 32-bit byte offsets from the (uniform) array bases: pt_create keeps both arrays < 4 GiB
    // (slots < 2^23, see kLeafBits: a full-rate 24-bit multiply; the slot is formed unconditionally
    // and selected, no branch)
    // Only the lanes with a pending leaf load it (TA -3%, TD -1%, +0.8%; tools/gpu/pmc_ab.sh).  The
    // other lanes' A, B, e2z are never read (pin_use below only orders the loads before the node's).
    float4 A, B;
    float e2z;
    // (buffers of 2 GiB - 256 B: pt_create keeps the arrays far below; offset 2^31 is out of range)
    const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(const_cast<DTri*>(tris), 0, 0x7fffff00, 0x00020000);
    const __amdgpu_buffer_rsrc_t nrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<DNode4*>(nodes), 0, 0x7fffff00, 0x00020000);
    if constexpr (kUniform) {
        const uint32_t tb = leaf ? __umul24(leaf4_slot(w), (uint32_t)sizeof(DTri)) : 0x80000000u;
        const f4v a4 = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(trs, tb, 0, 0));
        const f4v b4 = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(trs, tb + 16u, 0, 0));
        A = make_float4(a4.x, a4.y, a4.z, a4.w);
        B = make_float4(b4.x, b4.y, b4.z, b4.w);
        e2z = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(trs, tb + 32u, 0, 0));
    } else if (leaf) {
        const uint32_t tb = __umul24(leaf4_slot(w), (uint32_t)sizeof(DTri));
        A = glb_f4(tris, tb);
        B = glb_f4(reinterpret_cast<const char*>(tris) + 16, tb);
        e2z = *(__attribute__((address_space(1))) const float*)(reinterpret_cast<const char*>(tris) + 32 + tb);
    }
    // a lane with no node to visit reads node 0 (the LDS copy when there is one)
    const uint32_t nidx = visit ? w.node : 0u;
    float4 NX, FX, NY, FY, NZ, FZ;
    uint4 ch;
    if constexpr (kUniform) {
        const uint32_t nb = visit ? nidx * 128u : 0x80000000u;
        auto bl = [&](uint32_t off) {
            const f4v v = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(nrs, off, 0, 0));
            return make_float4(v.x, v.y, v.z, v.w);
        };
        const uint32_t ox = nb | w.nx, oy = nb | w.ny, oz = nb | w.nz;
        NX = bl(ox); FX = bl(ox ^ 48u); NY = bl(oy); FY = bl(oy ^ 80u); NZ = bl(oz); FZ = bl(oz ^ 112u);
        const float4 c4 = bl(nb + 96u);
        ch = make_uint4(__float_as_uint(c4.x), __float_as_uint(c4.y), __float_as_uint(c4.z), __float_as_uint(c4.w));
    } else {
    // Every lane reads the LDS copy first (a deep node's lane reads node 0: a broadcast), then the
    // deep nodes' lanes overwrite it with their global loads -- in this order, because the loads
    // write the same registers and an LDS read issued behind outstanding global loads to them
    // would have to wait out their whole latency.
    if (kTop || S.ntop != 0u) {
        const uint32_t m = __umul24(nidx < S.ntop ? nidx : 0u, kTopNodeBytes);   // (full-rate multiply)
        // far plane offsets: nx ^ 48 == 48 - nx for nx in {0, 48} (likewise 80 - ny, 112 - nz), so a
        // far address is (m - near offset) with the constants (and the top's base) in the offset field
        const uint32_t mb = lds_addr(S.top) + m;
        NX = lds_f4a(mb + w.nx); FX = lds_f4a(vsub_u32(mb, w.nx) + 48u);
        NY = lds_f4a(mb + w.ny); FY = lds_f4a(vsub_u32(mb, w.ny) + 80u);
        NZ = lds_f4a(mb + w.nz); FZ = lds_f4a(vsub_u32(mb, w.nz) + 112u);
        ch = lds_u4a(mb + 96u);
    }
    if (nidx >= S.ntop) {
        const uint32_t nb = nidx * 128u;
        const uint32_t ox = nb | w.nx, oy = nb | w.ny, oz = nb | w.nz;
        NX = glb_f4(nodes, ox); FX = glb_f4(nodes, ox ^ 48u);
        NY = glb_f4(nodes, oy); FY = glb_f4(nodes, oy ^ 80u);
        NZ = glb_f4(nodes, oz); FZ = glb_f4(nodes, oz ^ 112u);
        ch = glb_u4(nodes, nb + 96u);
    }
    }
    setup(w);
    pin_use(A); pin_use(B); pin_use1(e2z);   // (the node's fields feed unconditional tests: no pin needed)
    if (kCount) { if (visit) ++cnt.nodes; if (visit && nidx < S.ntop && !kUniform) ++cnt.top; if (leaf) { ++cnt.tris; ++cnt.leaf_steps; } }
    if (leaf) {
        const float t = tri_hit_pk(f2{o.x, o.y}, o.z, f2{d.x, d.y}, d.z, A, B, e2z);
        const uint32_t lslot = leaf4_slot(w);   // (recomputed here: one register less across the loads)
        if (kCount) cnt.tri_tested(__float_as_uint(tris[lslot].c.y));
        // ties go to the lower reference DFS rank (the reference's first-visited); exact ties are
        // rare, so both ranks are read only then
        if (0.0f < t && (t < w.best_t ||
                         (t == w.best_t && w.best_slot != kNone &&
                          __float_as_uint(tris[lslot].c.z) < __float_as_uint(tris[w.best_slot].c.z)))) {
            w.best_t = t; w.best_slot = lslot;
        }
        w.leaf &= w.leaf - 1u;   // that leaf is done
    }
    if (visit) visit4<kCount>(w, NX, FX, NY, FY, NZ, FZ, ch, S, cull_rel, node_mask, cnt);
    advance4(w, S, cull_rel, node_mask);
    if (kAnyHit && w.best_t <= w.occ) return false;
    return w.node != kNone || leaf4_pending(w);
}
#pragma clang diagnostic pop

// The walk's first step for a ray just begun (walk4_begin passed): the root's visit from the LDS top
// (no leaf can be pending yet), run where the ray is set up -- in the shading pass, where the lanes
// beginning traces do it together -- instead of as a walk-phase step.  Returns true while the walk
// continues (false: nothing entered, the ray misses).
template <bool kCount>
__device__ __forceinline__ bool walk4_root(W4& w, const Stack4& S, float cull_rel, uint32_t node_mask, Counters& cnt)
{
    const uint32_t mb = lds_addr(S.top) + __umul24(w.node, kTopNodeBytes);   // node 0 (or a staged node: walk4_top)
    const float4 NX = lds_f4a(mb + w.nx), FX = lds_f4a(vsub_u32(mb, w.nx) + 48u);
    const float4 NY = lds_f4a(mb + w.ny), FY = lds_f4a(vsub_u32(mb, w.ny) + 80u);
    const float4 NZ = lds_f4a(mb + w.nz), FZ = lds_f4a(vsub_u32(mb, w.nz) + 112u);
    const uint4 ch = lds_u4a(mb + 96u);
    if (kCount) { ++cnt.nodes; ++cnt.top; }
    visit4<kCount>(w, NX, FX, NY, FY, NZ, FZ, ch, S, cull_rel, node_mask, cnt);
    advance4(w, S, cull_rel, node_mask);
    return w.node != kNone || leaf4_pending(w);
}

// Exact walk for the rare rays the fast path does not take (outside the Markstein
// preconditions, or a BVH4 winner the reference would not have tested): the culled near-first
// walk on the reference BVH's child-pair records with IEEE '/' everywhere -- the reference's own
// slab bits, so every entered box is one the reference enters -- and its stack in HBM
// (entry k of this lane: node at gs[2k*stride], entry distance at gs[(2k+1)*stride]).
__device__ __forceinline__ void trace_slow(V3 o, V3 d, const float* root, const DNode* __restrict__ nodes,
                                        const DTri* __restrict__ tris, uint32_t* gs, uint32_t stride,
                                        float cull_rel, float cull_abs, int32_t* tri_out, float* t_out,
                                        uint32_t* tri_counts = nullptr)
{
    const V3 y = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    float best_t = kMaxFloat;
    uint32_t best_rank = 0u, best_id = 0xffffffffu;
    float ti, to;
    *tri_out = -1;
    *t_out = kMaxFloat;
    if (!slab<false>(o, d, y, root[0], root[1], root[2], root[3], root[4], root[5], &ti, &to) || to < -cull_abs)
        return;
    int sp = 0;
    uint32_t node = 0;
    for (;;) {
        const DNode* nd = nodes + node;
        const float4 A = nd->a, B = nd->b, C = nd->c;
        const uint4 D = nd->d;
        bool h0 = false, h1 = false;
        float t0 = 0.0f, t1 = 0.0f;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t r = c ? D.y : D.x;
            if (r & kLeaf) {
                const DTri* tr = tris + (r ^ kLeaf);
                uint32_t id;
                const float t = tri_hit<false>(o, d, tr, &id);
                if (tri_counts) atomicAdd(tri_counts + id, 1u);
                const uint32_t rank = __float_as_uint(tr->c.z);
                if (0.0f < t && (t < best_t || (t == best_t && rank < best_rank))) { best_t = t; best_rank = rank; best_id = id; }
            } else {
                const bool hit = c ? slab<false>(o, d, y, B.z, B.w, C.x, C.y, C.z, C.w, &ti, &to)
                                   : slab<false>(o, d, y, A.x, A.y, A.z, A.w, B.x, B.y, &ti, &to);
                const bool in = hit && !(to < -cull_abs) && !(ti > best_t * cull_rel);
                if (c) { h1 = in; t1 = ti; } else { h0 = in; t0 = ti; }
            }
        }
        h0 = h0 && !(t0 > best_t * cull_rel);
        if (h0 && h1) {
            const bool sw = t1 < t0;
            gs[(size_t)(2 * sp) * stride] = sw ? D.x : D.y;
            gs[(size_t)(2 * sp + 1) * stride] = __float_as_uint(sw ? t0 : t1);
            ++sp;
            node = sw ? D.y : D.x;
            continue;
        }
        if (h0 | h1) { node = h0 ? D.x : D.y; continue; }
        bool found = false;
        while (sp > 0) {
            --sp;
            if (__uint_as_float(gs[(size_t)(2 * sp + 1) * stride]) > best_t * cull_rel) continue;
            node = gs[(size_t)(2 * sp) * stride];
            found = true;
            break;
        }
        if (!found) break;
    }
    *tri_out = (best_id == 0xffffffffu) ? -1 : (int32_t)best_id;
    *t_out = best_t;
}

// ------------------------------------------------------------------ traversal results
struct Hit {
    int32_t tri;     // original triangle id, -1 = miss
    float t;         // closestT (MAX_FLOAT on miss)
};


// kernel.cu:112-161 trace(): the reference's exact walk -- left child first, every box the
// line overlaps, strict 0 < t < closestT.  The stack lives in LDS (kStack entries per lane,
// lane-interleaved: entry k of lane l at stack[k*64 + l]).
template <bool kCount>
__device__ __forceinline__ Hit trace_reference(V3 o, V3 d, const RNode* __restrict__ nodes, const DTri* __restrict__ tris,
                                               uint32_t* stack, int lane, Counters& cnt)
{
    float closest = kMaxFloat;
    int32_t best = -1;
    int i = 0;
    stack[lane] = 0;
    while (i >= 0) {
        const uint32_t e = stack[i * 64 + lane];
        if (e & kLeaf) {
            const uint32_t k = e ^ kLeaf;
            uint32_t id;
            const float t = tri_t_rec(o, d, tris + k, &id);
            if (0.0f < t && t < closest) { closest = t; best = (int32_t)k; }
            if (kCount) { ++cnt.tris; cnt.tri_tested(k); }   // kernel.cu:133 (tris is in original order)
            --i;
        } else {
            const RNode* nd = nodes + e;
            const float4 p = *reinterpret_cast<const float4*>(nd);
            const float4 q = *reinterpret_cast<const float4*>(&nd->hi[1]);
            if (kCount) ++cnt.nodes;
            float ti, to;
            // p = lo.xyz, hi.x ; q = hi.yz, left, right
            if (slab_ref(o, d, p.x, p.y, p.z, p.w, q.x, q.y, &ti, &to)) {
                stack[i * 64 + lane] = __float_as_uint(q.w);
                stack[(i + 1) * 64 + lane] = __float_as_uint(q.z);
                ++i;
            } else {
                --i;
            }
        }
    }
    Hit h;
    h.tri = best;
    h.t = closest;
    return h;
}

// Distance-culled, near-first walk over the 64-B child-pair records.  It returns the SAME
// hit as trace_reference: the winner is the minimum of (t, DFS rank) over 0 < t < MAX_FLOAT,
// which is what the reference's left-first strict '<' scan selects; boxes are entered only if
// the reference's own slab test accepts them; and a box is skipped only when its entry
// distance exceeds the current best by the relative margin cull_rel, or its exit lies behind
// the origin by more than cull_abs (DESIGN.md "Traversal").  Stack entries are (node, entry t).
template <bool kCount>
__device__ __forceinline__ Hit trace_culled(V3 o, V3 d, const float* root, const DNode* __restrict__ nodes,
                                            const DTri* __restrict__ tris, uint32_t* stack, int lane,
                                            float cull_rel, float cull_abs, Counters& cnt)
{
    // best_slot starts at 0 so a tie with the MAX_FLOAT sentinel is never accepted (the
    // reference needs t < closestT = MAX_FLOAT); best_id = ~0 marks "no hit yet".
    float best_t = kMaxFloat;
    uint32_t best_slot = 0u;   // on the reference tree the leaf slot IS the DFS rank
    uint32_t best_id = 0xffffffffu;
    float ti, to;
    if (!slab_ref(o, d, root[0], root[1], root[2], root[3], root[4], root[5], &ti, &to) || to < -cull_abs) {
        Hit h; h.tri = -1; h.t = kMaxFloat; return h;
    }
    int sp = 0;
    uint32_t node = 0;
    for (;;) {
        const DNode* nd = nodes + node;
        const float4 A = nd->a, B = nd->b, C = nd->c;
        const uint4 D = nd->d;
        if (kCount) ++cnt.nodes;   // one 64-B record fetched
        bool h0 = false, h1 = false;
        float t0 = 0.0f, t1 = 0.0f;
        if (D.x & kLeaf) {
            const uint32_t slot = D.x ^ kLeaf;
            uint32_t id;
            const float t = tri_t_rec(o, d, tris + slot, &id);
            if (kCount) { ++cnt.tris; cnt.tri_tested(id); }
            if (0.0f < t && (t < best_t || (t == best_t && slot < best_slot))) { best_t = t; best_slot = slot; best_id = id; }
        } else {
            const bool hit = slab_ref(o, d, A.x, A.y, A.z, A.w, B.x, B.y, &ti, &to);
            h0 = hit && !(to < -cull_abs) && !(ti > best_t * cull_rel);
            t0 = ti;
        }
        if (D.y & kLeaf) {
            const uint32_t slot = D.y ^ kLeaf;
            uint32_t id;
            const float t = tri_t_rec(o, d, tris + slot, &id);
            if (kCount) { ++cnt.tris; cnt.tri_tested(id); }
            if (0.0f < t && (t < best_t || (t == best_t && slot < best_slot))) { best_t = t; best_slot = slot; best_id = id; }
            // a leaf found now may already beat the left box: re-check it
            h0 = h0 && !(t0 > best_t * cull_rel);
        } else {
            const bool hit = slab_ref(o, d, B.z, B.w, C.x, C.y, C.z, C.w, &ti, &to);
            h1 = hit && !(to < -cull_abs) && !(ti > best_t * cull_rel);
            t1 = ti;
        }
        if (h0 && h1) {
            const bool swap = t1 < t0;
            const uint32_t nearn = swap ? D.y : D.x;
            const uint32_t farn = swap ? D.x : D.y;
            const float fart = swap ? t0 : t1;
            stack[sp * 128 + lane] = farn;
            stack[sp * 128 + 64 + lane] = __float_as_uint(fart);
            ++sp;
            node = nearn;
            continue;
        }
        if (h0) { node = D.x; continue; }
        if (h1) { node = D.y; continue; }
        // pop, skipping entries the current best already beats
        bool found = false;
        while (sp > 0) {
            --sp;
            const float et = __uint_as_float(stack[sp * 128 + 64 + lane]);
            if (et > best_t * cull_rel) continue;
            node = stack[sp * 128 + lane];
            found = true;
            break;
        }
        if (!found) break;
    }
    Hit h;
    h.tri = (best_id == 0xffffffffu) ? -1 : (int32_t)best_id;
    h.t = best_t;
    return h;
}

}  // namespace ptd
