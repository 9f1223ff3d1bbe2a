/*
 * pt_oracle.c -- CPU restatement of CulDeVu/CUDAPathTracer's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see pt_oracle.h).  Build: oracle/Makefile
 * (gcc -O2 -ffp-contract=off -fno-fast-math, OpenMP over pixels).
 *
 * Citations are file:line into the reference.  Types follow the reference's
 * C++ exactly: `vec3` is 3 x float, `color` is 3 x double, double literals
 * (0.001, 3.14159, 1.0, 0.5, 0.00001) promote the float operand and the
 * result is rounded back to float on assignment to a float.
 */
#include "pt_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_MAX_FLOAT 100000.0f       /* limits.h:3 */
#define OR_LEAF_FLAG 0x80000000u     /* limits.h:6 */
#define OR_STACK 64                  /* kernel.cu:35 MAX_BVH_DEPTH */

/* ------------------------------------------------------------------ vec3.h */
static inline or_vec3 v3(float x, float y, float z) { or_vec3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline or_vec3 vadd(or_vec3 a, or_vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }  /* vec3.h:15 */
static inline or_vec3 vsub(or_vec3 a, or_vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }  /* vec3.h:19 */
static inline or_vec3 vmul(or_vec3 a, float f) { return v3(a.x * f, a.y * f, a.z * f); }          /* vec3.h:23 */
static inline or_vec3 vdiv(or_vec3 a, float f) { return v3(a.x / f, a.y / f, a.z / f); }          /* vec3.h:27 */
static inline float vdot(or_vec3 a, or_vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }      /* vec3.h:63 */
static inline or_vec3 vcross(or_vec3 a, or_vec3 b)                                                /* vec3.h:67 */
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float vlength(or_vec3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }      /* vec3.h:72 */
static inline or_vec3 vnormalized(or_vec3 v)                                                      /* vec3.h:58 */
{
    float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return v3(v.x / len, v.y / len, v.z / len);
}
/* CUDA device max/min on float/double are fmaxf/fmax: a NaN operand is ignored. */
static inline float fmax_f(float a, float b) { return fmaxf(a, b); }

/* ----------------------------------------------------------------- color.h */
typedef struct { double r, g, b; } col;
static inline col c3(double r, double g, double b) { col c; c.r = r; c.g = g; c.b = b; return c; }
static inline col cadd(col a, col b) { return c3(a.r + b.r, a.g + b.g, a.b + b.b); }               /* color.h:46 */
static inline col cmulf(col a, float f) { return c3(a.r * (double)f, a.g * (double)f, a.b * (double)f); } /* color.h:27,50 */
static inline col cdivf(col a, float f) { return c3(a.r / (double)f, a.g / (double)f, a.b / (double)f); } /* color.h:31,35 */
static inline col cmul(col a, col b) { return c3(a.r * b.r, a.g * b.g, a.b * b.b); }               /* color.h:55 */
static inline col mat_albedo(const or_mat* m) { return c3(m->albedo[0], m->albedo[1], m->albedo[2]); }
static inline col mat_emission(const or_mat* m) { return c3(m->emission[0], m->emission[1], m->emission[2]); }

/* ------------------------------------------------------------------ XORWOW */
/* One XORWOW step on the 160-bit xorshift part (cuRAND curand(), recurrence identical to
 * rocRAND xorwow_engine::next): t = v0^(v0>>2); shift; v4 = (v4^(v4<<4))^(t^(t<<1)). */
static void xs_step(uint32_t v[5])
{
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}

/* Bit images: img[b*5 + k] = word k of M * e_b (b = 32*word + bit), the layout of
 * rocRAND's precomputed jump matrices (rocrand_xorwow.h mul_mat_vec_inplace). */
static void img_apply(const uint32_t* img, uint32_t v[5])
{
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < 160; ++b) {
        if ((v[b >> 5] >> (b & 31)) & 1u) {
            const uint32_t* row = img + b * 5;
            r[0] ^= row[0]; r[1] ^= row[1]; r[2] ^= row[2]; r[3] ^= row[3]; r[4] ^= row[4];
        }
    }
    memcpy(v, r, sizeof(r));
}

void or_xorwow_step_images(uint32_t img[160 * 5])
{
    for (int b = 0; b < 160; ++b) {
        uint32_t v[5] = {0, 0, 0, 0, 0};
        v[b >> 5] = 1u << (b & 31);
        xs_step(v);
        memcpy(img + b * 5, v, sizeof(v));
    }
}

static void img_square(uint32_t* img)
{
    static uint32_t tmp[160 * 5];
    uint32_t* out = (uint32_t*)malloc(sizeof(uint32_t) * 800);
    for (int b = 0; b < 160; ++b) {
        uint32_t v[5];
        memcpy(v, img + b * 5, sizeof(v));
        img_apply(img, v);
        memcpy(out + b * 5, v, sizeof(v));
    }
    memcpy(img, out, sizeof(uint32_t) * 800);
    free(out);
    (void)tmp;
}

void or_xorwow_jump_images(int log2_steps, uint32_t img[160 * 5])
{
    or_xorwow_step_images(img);
    for (int i = 0; i < log2_steps; ++i) img_square(img);
}

/* Subsequence jump tables J_k = A^(2^(67+k)), k = 0..31, built once. */
static uint32_t g_seq_jump[32][800];
static int g_seq_ready = 0;
static void seq_tables(void)
{
    if (g_seq_ready) return;
#ifdef _OPENMP
#pragma omp critical(or_seq_tables)
#endif
    {
        if (!g_seq_ready) {
            static uint32_t m[800];
            or_xorwow_jump_images(67, m);
            for (int k = 0; k < 32; ++k) {
                memcpy(g_seq_jump[k], m, sizeof(m));
                img_square(m);
            }
            __atomic_store_n(&g_seq_ready, 1, __ATOMIC_RELEASE);
        }
    }
}

/* curand_init(seed, subsequence, 0, &state): kernel.cu:532.  Salts/multipliers are the
 * published cuRAND (curand_kernel.h _curand_init_scratch) constants; the subsequence skip
 * multiplies v by A^(subsequence * 2^67) and leaves d unchanged (2^67 = 0 mod 2^32). */
void or_xorwow_init(uint64_t seed, uint64_t subsequence, or_xorwow* st)
{
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    st->d = 6615241u + t1 + t0;
    st->v[0] = 123456789u + t0;
    st->v[1] = 362436069u ^ t0;
    st->v[2] = 521288629u + t1;
    st->v[3] = 88675123u ^ t1;
    st->v[4] = 5783321u + t0;
    seq_tables();
    for (int k = 0; k < 32 && subsequence; ++k, subsequence >>= 1)
        if (subsequence & 1u) img_apply(g_seq_jump[k], st->v);
}

uint32_t or_xorwow_next(or_xorwow* st)
{
    xs_step(st->v);
    st->d += 362437u;
    return st->v[4] + st->d;
}

/* curand_uniform (kernel.cu:58): x * CURAND_2POW32_INV + CURAND_2POW32_INV/2, contracted.
 * OR_UNIFORM_UNFUSED (sensitivity variant, tools/parity/ref_gap.py): the same expression rounded
 * twice, as a build without FMA contraction would evaluate it. */
float or_uniform(or_xorwow* st)
{
    uint32_t x = or_xorwow_next(st);
#ifdef OR_UNIFORM_UNFUSED
    volatile float p = (float)x * 2.3283064e-10f;   /* (volatile: no contraction in any build) */
    return p + 2.3283064e-10f / 2.0f;
#else
    return fmaf((float)x, 2.3283064e-10f, 2.3283064e-10f / 2.0f);
#endif
}

/* ---------------------------------------------------------------- sin/cos */
/* Sensitivity variants (tools/parity/ref_gap.py; the default build defines neither):
 *   OR_SINCOS_LIBM       glibc sinf/cosf instead of det_sincos;
 *   OR_SINCOS_PERTURB=k  det_sincos's results moved by a pseudo-random j ulp, |j| <= k, chosen by a
 *                        hash of the argument's bits -- CUDA documents sinf/cosf to within 2 ulp, so
 *                        k = 2 is the worst case the reference's device library allows. */
#ifdef OR_SINCOS_PERTURB
static float ulp_move(float v, uint32_t h)
{
    int j = (int)(h % (2u * OR_SINCOS_PERTURB + 1u)) - OR_SINCOS_PERTURB;
    for (; j > 0; --j) v = nextafterf(v, INFINITY);
    for (; j < 0; ++j) v = nextafterf(v, -INFINITY);
    return v;
}
#endif

/* Deterministic float sin/cos for the sampling angles (kernel.cu:65-68, 84-88; camera.h:85-87):
 * double-precision Cody-Waite reduction by pi/2 and Taylor polynomials to degree 17/18, rounded
 * once to float.  Plain IEEE double ops in a fixed order, so gfx950 reproduces it exactly.
 * (Never contracted, whatever the build's -ffp-contract: the FMA-contraction variant of
 * ref_gap.py contracts the reference's own expressions, not this function's stand-in for cosf.) */
__attribute__((optimize("fp-contract=off")))
void or_sincos(float theta, float* s_out, float* c_out)
{
#ifdef OR_SINCOS_LIBM
    *s_out = sinf(theta);
    *c_out = cosf(theta);
    return;
#endif
    const double x = (double)theta;
    const double two_over_pi = 0.63661977236758138;
    const double pio2_hi = 1.5707963267948966;
    const double pio2_lo = 6.123233995736766e-17;
    double kd = nearbyint(x * two_over_pi);
    int k = (int)kd;
    double r = (x - kd * pio2_hi) - kd * pio2_lo;
    double r2 = r * r;
    double sp = 2.8114572543455206e-15;            /*  1/17! */
    sp = sp * r2 + -7.647163731819816e-13;         /* -1/15! */
    sp = sp * r2 + 1.6059043836821613e-10;         /*  1/13! */
    sp = sp * r2 + -2.505210838544172e-08;         /* -1/11! */
    sp = sp * r2 + 2.7557319223985893e-06;         /*  1/9!  */
    sp = sp * r2 + -0.0001984126984126984;         /* -1/7!  */
    sp = sp * r2 + 0.008333333333333333;           /*  1/5!  */
    sp = sp * r2 + -0.16666666666666666;           /* -1/3!  */
    double sn = r + r * (r2 * sp);
    double cp = -1.5619206968586225e-16;           /* -1/18! */
    cp = cp * r2 + 4.779477332387385e-14;          /*  1/16! */
    cp = cp * r2 + -1.1470745597729725e-11;        /* -1/14! */
    cp = cp * r2 + 2.08767569878681e-09;           /*  1/12! */
    cp = cp * r2 + -2.755731922398589e-07;         /* -1/10! */
    cp = cp * r2 + 2.48015873015873e-05;           /*  1/8!  */
    cp = cp * r2 + -0.001388888888888889;          /* -1/6!  */
    cp = cp * r2 + 0.041666666666666664;           /*  1/4!  */
    cp = cp * r2 + -0.5;                           /* -1/2!  */
    double cs = 1.0 + r2 * cp;
    double sv, cv;
    switch (k & 3) {
    case 0: sv = sn; cv = cs; break;
    case 1: sv = cs; cv = -sn; break;
    case 2: sv = -sn; cv = -cs; break;
    default: sv = -cs; cv = sn; break;
    }
    *s_out = (float)sv;
    *c_out = (float)cv;
#ifdef OR_SINCOS_PERTURB
    {
        uint32_t b;
        memcpy(&b, &theta, 4);
        const uint32_t h = b * 0x9e3779b1u;
        *s_out = ulp_move(*s_out, h >> 7);
        *c_out = ulp_move(*c_out, (h ^ 0x5bd1e995u) * 0x85ebca6bu >> 9);
    }
#endif
}

/* -------------------------------------------------------------- geometry */
/* modelLoader.h:49-83 triIntersect.  (OR_TRI_NO_CONTRACT: the fma_notri sensitivity variant keeps this one
 * function uncontracted while the rest of the build contracts; OR_TRI_CONTRACT: the fma_tri variant
 * contracts this one function only, as the compiler chooses; OR_TRI_FMA = 1 / 2: the fmal_tri / fmar_tri
 * variants spell the contraction out -- vec3.h's a*b + c*d and a*b - c*d with the LEFT product fused
 * (fma(a, b, c*d), fma(a, b, -(c*d)): LLVM's DAG combiner folds (fadd (fmul a b) z) first, GCC's
 * widening_mul converts the first product in statement order) or the RIGHT one (fma(c, d, a*b),
 * fma(-c, d, a*b)); the dot product's last term fuses either way.  tools/parity/ref_gap.py) */
#if defined(OR_TRI_FMA)
static inline float tdot(or_vec3 a, or_vec3 b)
{
#if OR_TRI_FMA == 1
    return fmaf(a.z, b.z, fmaf(a.x, b.x, a.y * b.y));
#else
    return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x));
#endif
}
static inline float tdiff(float a, float b, float c, float d)   /* a*b - c*d */
{
#if OR_TRI_FMA == 1
    return fmaf(a, b, -(c * d));
#else
    return fmaf(-c, d, a * b);
#endif
}
static inline or_vec3 tcross(or_vec3 a, or_vec3 b)
{
    return v3(tdiff(a.y, b.z, a.z, b.y), tdiff(a.z, b.x, a.x, b.z), tdiff(a.x, b.y, a.y, b.x));
}
#else
#define tdot vdot
#define tcross vcross
#endif
#ifdef OR_TRI_NO_CONTRACT
__attribute__((optimize("fp-contract=off")))
#endif
#ifdef OR_TRI_CONTRACT
__attribute__((optimize("fp-contract=fast")))
#endif
float or_tri_intersect(or_vec3 o, or_vec3 ray, const or_vec3* verts, const or_tri* t)
{
    or_vec3 v0 = verts[t->v0], v1 = verts[t->v1], v2 = verts[t->v2];
    or_vec3 e1 = vsub(v1, v0);
    or_vec3 e2 = vsub(v2, v0);
    or_vec3 q = tcross(ray, e2);
    float a = tdot(e1, q);
    if ((double)fabsf(a) < 0.00001) return OR_MAX_FLOAT;
    or_vec3 s = vdiv(vsub(o, v0), a);
    or_vec3 r = tcross(s, e1);
    float b0 = tdot(s, q);
    float b1 = tdot(r, ray);
    float b2 = 1.0f - b0 - b1;
    if (b0 < 0.0f) return OR_MAX_FLOAT;
    if (b1 < 0.0f) return OR_MAX_FLOAT;
    if (b2 < 0.0f) return OR_MAX_FLOAT;
    return tdot(e2, r);
}

/* BVH.h:51-83 rayAABBIntersect (IEEE division, NaN-propagating compare/swap) */
int or_ray_aabb(or_vec3 o, or_vec3 ray, or_vec3 lo, or_vec3 hi)
{
    float tmin = (lo.x - o.x) / ray.x, tmax = (hi.x - o.x) / ray.x, tt;
    if (tmin > tmax) { tt = tmin; tmin = tmax; tmax = tt; }
    float tymin = (lo.y - o.y) / ray.y, tymax = (hi.y - o.y) / ray.y;
    if (tymin > tymax) { tt = tymin; tymin = tymax; tymax = tt; }
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (lo.z - o.z) / ray.z, tzmax = (hi.z - o.z) / ray.z;
    if (tzmin > tzmax) { tt = tzmin; tzmin = tzmax; tzmax = tt; }
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    return 1;
}

/* camera.h:66-75 mortonPxltoI / :57-65 mortonItoPxl (16 bits per axis) */
uint32_t or_morton_pxl_to_i(uint32_t x, uint32_t y)
{
    uint32_t idx = 0;
    for (int i = 0; i < 16; ++i) {
        idx |= ((x >> i) & 1u) << (2 * i);
        idx |= ((y >> i) & 1u) << (2 * i + 1);
    }
    return idx;
}
void or_morton_i_to_pxl(uint32_t idx, uint32_t* x, uint32_t* y)
{
    uint32_t xx = 0, yy = 0;
    for (int i = 0; i < 16; ++i) {
        xx |= ((idx >> (2 * i)) & 1u) << i;
        yy |= ((idx >> (2 * i + 1)) & 1u) << i;
    }
    *x = xx & 0xffffu;
    *y = yy & 0xffffu;
}

/* camera.h:77-97 cameraRay.  (u1,u2) are the lens draws; when the caller passes NAN the
 * lens term is exactly zero (no draws consumed: see DESIGN.md decision d1). */
void or_camera_ray(const or_camera* cam, uint32_t idx, float u1, float u2, or_vec3* o_out, or_vec3* d_out)
{
    uint32_t px, py;
    or_morton_i_to_pxl(idx, &px, &py);
    or_vec3 film;
    film.x = (float)(uint16_t)px / (float)cam->pxl_width - 0.5f;     /* camera.h:39 */
    film.y = (float)(uint16_t)py / (float)cam->pxl_height - 0.5f;    /* camera.h:40 */
    film.z = 0.0f;
    or_vec3 o = v3(0.0f, 0.0f, 0.0f);
    if (!(u1 != u1)) {
        float r = cam->radius * sqrtf(u1);
        float theta = (float)(2 * 3.14159 * (double)u2);
        float s, c;
        or_sincos(theta, &s, &c);
        o = v3(r * c, r * s, 0.0f);
    }
    film.z = cam->dist_from_film;
    film = vdiv(vmul(film, -cam->focal_length), cam->dist_from_film);  /* camera.h:91 */
    *o_out = vadd(o, cam->pos);
    *d_out = vnormalized(vsub(film, o));
}

/* ------------------------------------------------------------- spheres (d8) */
/* Ray/sphere for unit d, in float and in this order: oc = o - c, b = oc.d,
 * disc = b*b - (oc.oc - r*r); the nearer root -b - sqrt(disc) if > 0, else -b + sqrt(disc)
 * if > 0, else a miss (MAX_FLOAT).  The caller keeps it only if t < closestT (strict). */
float or_sphere_t(or_vec3 o, or_vec3 d, const or_sphere* s)
{
    or_vec3 oc = vsub(o, s->pos);
    float b = vdot(oc, d);
    float c = vdot(oc, oc) - s->rad * s->rad;
    float disc = b * b - c;
    if (!(disc >= 0.0f)) return OR_MAX_FLOAT;
    float q = sqrtf(disc);
    float t = -b - q;
    if (t > 0.0f) return t;
    t = -b + q;
    if (t > 0.0f) return t;
    return OR_MAX_FLOAT;
}

static inline float sphere_area(float r) { return 4.0f * 3.14159f * r * r; }

/* primitive id -> material handle / normal at p (triangles: modelLoader.h:14-19; spheres:
 * material num_mats + i, normal (p - c) / r) */
static inline int32_t prim_mat(const or_scene* sc, int32_t id)
{
    return (uint32_t)id < sc->num_tris ? sc->tris[id].mat : (int32_t)(sc->num_mats + ((uint32_t)id - sc->num_tris));
}
static inline const or_mat* mat_ptr(const or_scene* sc, int32_t m)
{
    return (uint32_t)m < sc->num_mats ? sc->mats + m : (const or_mat*)(const void*)sc->spheres[(uint32_t)m - sc->num_mats].diffuse;
}
static inline or_vec3 prim_normal(const or_scene* sc, int32_t id, or_vec3 p)
{
    if ((uint32_t)id < sc->num_tris) return sc->tris[id].norm;
    const or_sphere* s = sc->spheres + ((uint32_t)id - sc->num_tris);
    return vdiv(vsub(p, s->pos), s->rad);
}

/* ------------------------------------------------------------- traversal */
/* kernel.cu:112-161 trace(): explicit stack, left child on top, strict 0<t<closestT. */
int or_trace(const or_scene* sc, or_vec3 o, or_vec3 dir, int32_t* tri_out, float* t_out, or_counters* cnt)
{
    uint32_t stack[OR_STACK + 1];
    stack[0] = 0;
    float closest = OR_MAX_FLOAT;
    int32_t tri = -1;
    int i = 0;
    uint64_t nt = 0, tt = 0;
    if (sc->bvh_size == 0) i = -1;             /* no triangles */
    while (i >= 0) {
        uint32_t e = stack[i];
        if (e & OR_LEAF_FLAG) {
            uint32_t k = e ^ OR_LEAF_FLAG;
            float t = or_tri_intersect(o, dir, sc->verts, sc->tris + k);
            if (0.0f < t && t < closest) { closest = t; tri = (int32_t)k; }
            ++tt;
            if (cnt && cnt->tri_counts) __atomic_fetch_add(cnt->tri_counts + k, 1u, __ATOMIC_RELAXED);  /* :133 */
            --i;
        } else {
            const or_node* nd = sc->bvh + e;
            ++nt;
            if (or_ray_aabb(o, dir, nd->lo, nd->hi)) {
                if (i + 1 >= OR_STACK) return -1;
                stack[i] = nd->right;
                stack[i + 1] = nd->left;
                ++i;
            } else {
                --i;
            }
        }
    }
    for (uint32_t k = 0; k < sc->num_spheres; ++k) {       /* after every triangle: ties keep the triangle */
        float t = or_sphere_t(o, dir, sc->spheres + k);
        if (0.0f < t && t < closest) { closest = t; tri = (int32_t)(sc->num_tris + k); }
    }
    *tri_out = tri;
    *t_out = closest;
    if (cnt) { cnt->traces += 1; cnt->node_tests += nt; cnt->tri_tests += tt; }
    return 0;
}

int or_trace_batch(const or_scene* sc, uint32_t n, const float* rays, int32_t* tri, float* t)
{
    return or_trace_batch_counts(sc, n, rays, tri, t, NULL);
}

int or_trace_batch_counts(const or_scene* sc, uint32_t n, const float* rays, int32_t* tri, float* t,
                          uint32_t* tri_counts)
{
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : bad)
    for (long r = 0; r < (long)n; ++r) {
        or_counters cnt;
        memset(&cnt, 0, sizeof(cnt));
        cnt.tri_counts = tri_counts;
        const float* q = rays + 6 * r;
        or_vec3 o = {q[0], q[1], q[2]}, d = {q[3], q[4], q[5]};
        bad += or_trace(sc, o, d, tri + r, t + r, &cnt) != 0;
    }
    return bad;
}

/* ------------------------------------------------------- sampling helpers */
static or_vec3 get_tangent(or_vec3 n)                                  /* kernel.cu:44-54 */
{
    or_vec3 c1 = vcross(n, v3(0, 0, 1));
    or_vec3 c2 = vcross(n, v3(0, 1, 0));
    return (vdot(c1, c1) > vdot(c2, c2)) ? c1 : c2;
}
static or_vec3 to_frame(or_vec3 n, or_vec3 local)                      /* kernel.cu:70-75 / 91-96 */
{
    or_vec3 tg = get_tangent(n);
    or_vec3 bt = vcross(n, tg);
    or_vec3 w = vadd(vadd(vmul(n, local.y), vmul(tg, local.x)), vmul(bt, local.z));
    return vnormalized(w);
}
static or_vec3 rand_ray(or_vec3 n, or_xorwow* rng)                     /* kernel.cu:60-77 */
{
    float u1 = or_uniform(rng);
    float u2 = or_uniform(rng);
    float r = sqrtf(1.0f - u1 * u1);
    float phi = (float)(2 * 3.14159 * (double)u2);
    float s, c;
    or_sincos(phi, &s, &c);
    return to_frame(n, v3(r * c, u1, r * s));
}
static or_vec3 cosine_ray(or_vec3 n, or_xorwow* rng)                   /* kernel.cu:78-99 */
{
    float u1 = or_uniform(rng);
    float u2 = or_uniform(rng);
    float r = sqrtf(u1);
    float theta = (float)(2 * 3.14159 * (double)u2);
    float s, c;
    or_sincos(theta, &s, &c);
    float x = r * c;
    float z = r * s;
    float y = sqrtf(fmax_f(0.0f, 1.0f - u1));
    return to_frame(n, v3(x, y, z));
}
static col brdf(const or_mat* m) { return cmulf(mat_albedo(m), (float)(1 / 3.14159)); }  /* kernel.cu:101-104 */

/* exported for the golden checks of getTangent / BRDF against the reference's own code (refgen helpers) */
void or_get_tangent(or_vec3 n, or_vec3* out) { *out = get_tangent(n); }
void or_brdf(const double albedo[3], double out[3])
{
    or_mat m;
    memset(&m, 0, sizeof(m));
    m.albedo[0] = albedo[0]; m.albedo[1] = albedo[1]; m.albedo[2] = albedo[2];
    const col c = brdf(&m);
    out[0] = c.r; out[1] = c.g; out[2] = c.b;
}

/* Area-CDF light pick + uniform point (kernel.cu:466-495, 231-262).  Returns the chosen
 * primitive id; a triangle gives p = v0 + a1*u + a2*v.  Sphere lights (d8 policy) enter the
 * CDF with area 4*3.14159*r^2 and give the uniform point c + r*(sqrt(1-z^2)cos(phi),
 * sqrt(1-z^2)sin(phi), z), z = 1 - 2u, phi = 2*3.14159*v -- the same three draws. */
static int32_t pick_light(const or_scene* sc, or_xorwow* rng, or_vec3* p_out)
{
    float rand_area = sc->total_light_area * or_uniform(rng);
    int32_t sel = 0;
    for (uint32_t j = 0; j < sc->num_lights; ++j) {
        const uint32_t e = sc->lights[j];
        float area;
        int32_t id;
        if (e & OR_LIGHT_SPHERE) {
            area = sphere_area(sc->spheres[e ^ OR_LIGHT_SPHERE].rad);
            id = (int32_t)(sc->num_tris + (e ^ OR_LIGHT_SPHERE));
        } else {
            const or_tri* lt = sc->tris + e;
            or_vec3 a1 = vsub(sc->verts[lt->v1], sc->verts[lt->v0]);
            or_vec3 a2 = vsub(sc->verts[lt->v2], sc->verts[lt->v0]);
            area = vlength(vcross(a1, a2)) / 2;
            id = (int32_t)e;
        }
        if (rand_area < area && rand_area > 0) sel = id;
        rand_area -= area;
    }
    float u = or_uniform(rng);
    float v = or_uniform(rng);
    if ((uint32_t)sel >= sc->num_tris) {
        const or_sphere* s = sc->spheres + ((uint32_t)sel - sc->num_tris);
        float z = 1.0f - 2.0f * u;
        float rxy = sqrtf(fmax_f(0.0f, 1.0f - z * z));
        float phi = (float)(2 * 3.14159 * (double)v);
        float si, co;
        or_sincos(phi, &si, &co);
        *p_out = vadd(s->pos, vmul(v3(rxy * co, rxy * si, z), s->rad));
        return sel;
    }
    const or_tri* st = sc->tris + sel;
    or_vec3 v0 = sc->verts[st->v0];
    or_vec3 a1 = vsub(sc->verts[st->v1], v0);
    or_vec3 a2 = vsub(sc->verts[st->v2], v0);
    if ((double)(u + v) > 1.0) {
        u = (float)((double)u + 2 * (0.5 - (double)u));
        v = (float)((double)v + 2 * (0.5 - (double)v));
    }
    *p_out = vadd(vadd(v0, vmul(a1, u)), vmul(a2, v));
    return sel;
}

/* --------------------------------------------------------- integrator 0 */
/* kernel.cu:417-515 radianceAlongSingleStep2 */
void or_radiance_unidir(const or_scene* sc, or_vec3 o, or_vec3 dir, int bounces,
                        or_xorwow* rng, double out[3], or_counters* cnt)
{
    col accum = c3(0, 0, 0);
    col weight = c3(1, 1, 1);
    for (int i = 0; i < bounces; ++i) {
        int32_t tri;
        float t;
        or_trace(sc, o, dir, &tri, &t, cnt);
        t = (float)((double)t - 0.001);                           /* :431 */
        if ((double)t < 0.001) weight = c3(0, 0, 0);               /* :432-435 */
        if (t > OR_MAX_FLOAT - 1) { weight = c3(0, 0, 0); tri = 0; t = 0; }   /* :436-441 */
        or_vec3 pos = vadd(o, vmul(dir, t));                      /* :449 */
        const or_mat* cm = mat_ptr(sc, prim_mat(sc, tri));
        or_vec3 normal = prim_normal(sc, tri, pos);
        or_vec3 odir = vmul(dir, -1);
        or_vec3 ldir;
        if (cm->emission[0] != 0) {                               /* :453-457 */
            accum = cadd(accum, cmul(weight, mat_emission(cm)));
            weight = c3(0, 0, 0);
        }
        float a = or_uniform(rng);
        if (a < 0.5) {                                            /* :460-465 */
            ldir = cosine_ray(normal, rng);
            col cw = cmulf(brdf(cm), (float)3.14159);
            weight = cmul(weight, cw);
        } else {                                                  /* :466-509 */
            or_vec3 p1;
            pick_light(sc, rng, &p1);
            or_vec3 d = vsub(p1, pos);
            ldir = vnormalized(d);
            float inv_prob = sc->total_light_area;
            float cos_l = fmax_f(0.0f, vdot(ldir, normal));
            float cos_o = fmax_f(0.0f, vdot(v3(0, -1, 0), vmul(ldir, -1)));
            float G = cos_l * cos_o / vdot(d, d);
            weight = cmul(weight, cmulf(cmulf(brdf(cm), G), inv_prob));
            i = (i > bounces - 2) ? i : bounces - 2;
        }
        (void)odir;
        o = pos;
        dir = ldir;
    }
    out[0] = accum.r; out[1] = accum.g; out[2] = accum.b;
}

/* --------------------------------------------------------- integrator 1 */
static float geo_term(or_vec3 xa, or_vec3 xb, or_vec3 na, or_vec3 nb)  /* kernel.cu:370-373 */
{
    or_vec3 seg = vsub(xa, xb);
    or_vec3 ray = vnormalized(seg);
    float G = fabsf(vdot(ray, na) * vdot(ray, nb)) / vdot(seg, seg);
    if (G != G) G = 0;
    return G;
}

/* kernel.cu:217-415 radianceAlongSingleStep (5-vertex estimator).  Decision d2: a miss on
 * the camera's second bounce (reference reads tris[-1], :333-346) uses triangle 0 and t = 0,
 * the miss convention of :279-283. */
void or_radiance_head(const or_scene* sc, or_vec3 cam_o, or_vec3 cam_d,
                      or_xorwow* rng, double out[3], or_counters* cnt)
{
    or_vec3 x[5], norm[5];
    int32_t mat[5] = {0, 0, 0, 0, 0};
    float inv_prob[5];
    /* light vertex (:231-270) */
    {
        or_vec3 p;
        int32_t sel = pick_light(sc, rng, &p);
        or_vec3 normal = prim_normal(sc, sel, p);
        x[0] = vadd(p, vmul(normal, 0.001f));
        norm[0] = normal;
        mat[0] = prim_mat(sc, sel);
        inv_prob[0] = sc->total_light_area;
    }
    /* light bounce (:271-301) */
    {
        or_vec3 odir = rand_ray(norm[0], rng);
        int32_t tri; float t;
        or_trace(sc, x[0], odir, &tri, &t, cnt);
        t = (float)((double)t - 0.001);
        if (t > OR_MAX_FLOAT - 1) { tri = 0; t = 0; }
        or_vec3 pos = vadd(x[0], vmul(odir, t));
        or_vec3 n2 = prim_normal(sc, tri, pos);
        float G = fabsf(vdot(n2, odir)) / fmax_f(0.001f, t * t);
        x[1] = pos; norm[1] = n2; mat[1] = prim_mat(sc, tri);
        inv_prob[1] = (float)(2 * 3.14159 / (double)G);
    }
    /* camera vertex (:304-308) */
    x[4] = cam_o; norm[4] = cam_d; inv_prob[4] = 1;
    /* camera first hit (:309-331) */
    {
        int32_t tri; float t;
        or_trace(sc, cam_o, cam_d, &tri, &t, cnt);
        t = (float)((double)t - 0.001);
        if (t > OR_MAX_FLOAT - 1) { tri = 0; t = 0; }
        x[3] = vadd(cam_o, vmul(cam_d, t));
        norm[3] = prim_normal(sc, tri, x[3]);
        mat[3] = prim_mat(sc, tri);
        inv_prob[3] = 1;
    }
    /* camera second hit (:332-350) */
    {
        or_vec3 d = cosine_ray(norm[3], rng);
        int32_t tri; float t;
        or_trace(sc, x[3], d, &tri, &t, cnt);
        t = (float)((double)t - 0.001);
        if (t > OR_MAX_FLOAT - 1 || tri < 0) { tri = 0; t = 0; }    /* d2 */
        x[2] = vadd(x[3], vmul(d, t));
        or_vec3 n = prim_normal(sc, tri, x[2]);
        float G = fabsf(vdot(norm[3], d) * vdot(n, d)) / (t * t);
        if (G == 0) G = 1;
        if (G != G) G = 1;
        norm[2] = n;
        mat[2] = prim_mat(sc, tri);
        inv_prob[2] = (float)(3.14159 / (double)G);
    }
    /* connections (:352-412) */
    col accum = c3(0, 0, 0);
    col le = mat_emission(mat_ptr(sc, mat[0]));
    for (int i = 0; i < 2; ++i) {
        for (int j = 2; j < 4; ++j) {
            col w = cmulf(le, inv_prob[0]);
            for (int k = 1; k <= i; ++k) {
                float G = geo_term(x[k], x[k - 1], norm[k], norm[k - 1]);
                col fs = cdivf(mat_albedo(mat_ptr(sc, mat[k])), 3.14159f);
                w = cmulf(cmulf(cmul(w, fs), G), inv_prob[k]);
            }
            for (int k = j + 1; k < 4; ++k) {
                float G = geo_term(x[k], x[k - 1], norm[k], norm[k - 1]);
                col fs = cdivf(mat_albedo(mat_ptr(sc, mat[k])), 3.14159f);
                w = cmulf(cmulf(cmul(w, fs), G), inv_prob[k]);
            }
            {
                or_vec3 seg = vsub(x[j], x[i]);
                float len = vlength(seg);
                or_vec3 ray = vnormalized(seg);
                float G = fmax_f(0.0f, vdot(ray, norm[j]) * vdot(vmul(ray, -1), norm[i])) / vdot(seg, seg);
                if (G != G) G = 0;
                col fs = cdivf(mat_albedo(mat_ptr(sc, mat[j])), 3.14159f);
                w = cmulf(cmulf(cmul(w, fs), G), inv_prob[j]);
                float m = (float)fmax(w.r, fmax(w.g, w.b));
                float V = 0;
                if ((double)m > 0.01) {
                    int32_t tri; float t;
                    or_trace(sc, x[i], ray, &tri, &t, cnt);
                    if ((double)fabsf(t - len) <= 0.01) V = 1;
                }
                w = cmulf(w, V);
            }
            accum = cadd(accum, w);
            accum = cadd(accum, mat_emission(mat_ptr(sc, mat[3])));
        }
    }
    out[0] = accum.r; out[1] = accum.g; out[2] = accum.b;
}

/* ------------------------------------------------------------------ render */
/* Camera draws (kernel.cu:547 reads &randState[0] from every thread: a race).  Decision d1:
 * a pixel consumes the two lens draws from its own stream iff it is Morton index 0 (the
 * race-free reading of the reference) or the lens radius is non-zero; otherwise the lens
 * term is exactly zero, which is what radius 0 yields for every draw. */
int or_render(const or_scene* sc, const or_camera* cam, int width, int height,
              int spp, int bounces, int integrator, uint64_t seed,
              const uint32_t* pixels, uint32_t num_pixels, int threads,
              double* out, or_counters* cnt)
{
    (void)height;
    seq_tables();
    uint64_t tr = 0, nt = 0, tt = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : tr, nt, tt)
#endif
    for (long pi = 0; pi < (long)num_pixels; ++pi) {
        uint32_t pix = pixels[pi];
        uint32_t px = pix % (uint32_t)width, py = pix / (uint32_t)width;
        uint32_t idx = or_morton_pxl_to_i(px, py);
        or_xorwow rng;
        or_xorwow_init(seed, idx, &rng);
        or_counters c = {0, 0, 0, cnt ? cnt->tri_counts : NULL};
        double mean[3] = {0, 0, 0};
        int lens_draws = (idx == 0) || (cam->radius != 0.0f);
        for (int n = 1; n <= spp; ++n) {
            float u1 = NAN, u2 = NAN;
            if (lens_draws) { u1 = or_uniform(&rng); u2 = or_uniform(&rng); }
            or_vec3 o, d;
            or_camera_ray(cam, idx, u1, u2, &o, &d);
            double L[3];
            if (integrator == 1) or_radiance_head(sc, o, d, &rng, L, &c);
            else or_radiance_unidir(sc, o, d, bounces, &rng, L, &c);
            /* kernel.cu:551-552: prev * (float)(n-1) / n + result / n, all in double */
            double fn1 = (double)(float)(n - 1), fn = (double)(float)n;
            for (int ch = 0; ch < 3; ++ch) mean[ch] = (mean[ch] * fn1) / fn + L[ch] / fn;
        }
        double* o3 = out + (size_t)pix * 3;
        o3[0] = mean[0]; o3[1] = mean[1]; o3[2] = mean[2];
        tr += c.traces; nt += c.node_tests; tt += c.tri_tests;
    }
    if (cnt) { cnt->traces += tr; cnt->node_tests += nt; cnt->tri_tests += tt; }
    return 0;
}

/* kernel.cu:763-778 (the reference's "save the file" loop) over its Morton-indexed imgBuffer_host;
 * color.h:59-62 normalized = c/(c+1) per channel, color.h:68-71 gammaCorrect = pow(c, (float)(1/2.2))
 * (the exponent is a float parameter), then (int)(c*255) */
static int tone_ref(double c)
{
    const double n = c / (c + 1);
    const double g = pow(n, (double)(float)(1 / 2.2));
    return (int)(g * 255);
}

int or_write_ppm_imgbuf(const char* path, const double* imgbuf, int width, int height)
{
    FILE* fp = fopen(path, "w");
    if (!fp) return -1;
    fprintf(fp, "P3 %d %d 255\n", width, height);
    for (int y = 0; y < height; ++y) {
        for (int x = width - 1; x >= 0; --x) {
            const double* c = imgbuf + (size_t)or_morton_pxl_to_i((uint32_t)x, (uint32_t)y) * 3;   /* :771 */
            fprintf(fp, "%d %d %d ", tone_ref(c[0]), tone_ref(c[1]), tone_ref(c[2]));
        }
    }
    return fclose(fp) == 0 ? 0 : -1;
}
