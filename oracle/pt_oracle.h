/*
 * pt_oracle.h -- CPU restatement of the reference's per-pixel path-integration loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker.  The product
 * (cudapathtracer_amd / libptamd.so) never links, loads or calls it.
 *
 * Every function cites the reference file:line it restates (reference =
 * CulDeVu/CUDAPathTracer, mounted read-only at /root/reference in the build
 * container).  Arithmetic follows the reference's C++ typing exactly (float
 * geometry, double colour, double literals promoting float expressions) with
 * IEEE single/double ops, no FMA contraction (built with -ffp-contract=off),
 * correctly rounded division and sqrt.  The only spec choices not dictated by
 * the reference are listed in DESIGN.md section "Arithmetic spec":
 *   - cosf/sinf of the sampling angles use pt's deterministic double-precision
 *     kernel (or_sincos) so CPU and gfx950 agree bit-for-bit;
 *   - curand_uniform is fmaf((float)x, 2^-32_f, 2^-33_f) (nvcc contracts it);
 *   - the cuRAND XORWOW seeding salts are the published curand_kernel.h
 *     constants, which cannot be verified in this container (parity to the
 *     original CUDA binary's RNG is unpinned; the recurrence and the 2^67
 *     subsequence jump ARE pinned against rocRAND's precomputed matrices).
 *
 * Pinning: kernel.cu cannot be built here (CUDA/cuRAND/NVML/windows.h
 * absent, triple.h broken), so the integrator itself is a restatement.  Its
 * building blocks (triIntersect, rayAABBIntersect, cameraRay, Morton maps, OBJ
 * ingest, BVH build) are pinned against golden vectors emitted by the
 * reference's own sources compiled with g++ (oracle/refgen, outputs in
 * tests/golden).
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y, z; } or_vec3;                         /* vec3.h:4-7            */
typedef struct { int32_t v0, v1, v2; or_vec3 norm; int32_t mat; } or_tri;   /* modelLoader.h:14-19 */
typedef struct { double albedo[3]; double emission[3]; } or_mat;  /* modelLoader.h:21-25, color.h:4-6 */
typedef struct { or_vec3 lo, hi; uint32_t left, right; } or_node; /* BVH.h:13-15, 111-115  */
typedef struct {                                                   /* camera.h:26-34        */
    or_vec3 pos;
    float dist_from_film, focal_length, radius;
    int32_t pxl_width, pxl_height;
} or_camera;
typedef struct { uint32_t d; uint32_t v[5]; } or_xorwow;          /* curandStateXORWOW d, v[5] */
/* sphere.h:7-12; the tail {diffuse, emission} has or_mat's layout.  Semantics are the build's
 * (reference has none): see or_sphere_t, prim_normal, pick_light. */
typedef struct { or_vec3 pos; float rad; double diffuse[3]; double emission[3]; } or_sphere;
#define OR_LIGHT_SPHERE 0x80000000u   /* lights[] entry of an emissive sphere */

typedef struct {                                                   /* modelLoader.h:29-41 + BVH.h:116-121 */
    uint32_t num_verts, num_tris, num_mats, num_lights;
    const or_vec3* verts;
    const or_tri* tris;
    const or_mat* mats;
    const uint32_t* lights;
    float total_light_area;
    const or_node* bvh;
    uint32_t bvh_size;             /* 0: no triangles (a scene of spheres)                     */
    const or_sphere* spheres;      /* hit ids num_tris + i; material handles num_mats + i        */
    uint32_t num_spheres;
} or_scene;

typedef struct {
    uint64_t traces, node_tests, tri_tests;
    uint32_t* tri_counts;   /* optional (NULL = off): per-triangle test counts, kernel.cu:133 test[k] += 1 */
} or_counters;

/* ---- RNG (kernel.cu:527-533 curand_init(1234, idx, 0); kernel.cu:56-59 curand_uniform) */
void     or_xorwow_step_images(uint32_t img[160 * 5]);            /* one-step matrix A      */
void     or_xorwow_jump_images(int log2_steps, uint32_t img[160 * 5]); /* A^(2^log2_steps) */
void     or_xorwow_init(uint64_t seed, uint64_t subsequence, or_xorwow* st);
uint32_t or_xorwow_next(or_xorwow* st);
float    or_uniform(or_xorwow* st);

/* ---- math kernels */
void     or_sincos(float theta, float* s, float* c);

/* ---- geometry (modelLoader.h:49-83, BVH.h:51-83, camera.h:36-97) */
float    or_tri_intersect(or_vec3 o, or_vec3 dir, const or_vec3* verts, const or_tri* t);
int      or_ray_aabb(or_vec3 o, or_vec3 dir, or_vec3 lo, or_vec3 hi);
uint32_t or_morton_pxl_to_i(uint32_t x, uint32_t y);
void     or_morton_i_to_pxl(uint32_t idx, uint32_t* x, uint32_t* y);
void     or_camera_ray(const or_camera* cam, uint32_t idx, float u1, float u2, or_vec3* o, or_vec3* dir);

/* ---- traversal (kernel.cu:112-161); returns 0, or -1 on stack overflow */
int      or_trace(const or_scene* sc, or_vec3 o, or_vec3 dir, int32_t* tri, float* t, or_counters* cnt);
float    or_sphere_t(or_vec3 o, or_vec3 d, const or_sphere* s);   /* MAX_FLOAT on a miss */
/* or_trace over rays[6n] = {o.xyz, d.xyz} (OpenMP); returns the number of stack overflows. */
int      or_trace_batch(const or_scene* sc, uint32_t n, const float* rays, int32_t* tri, float* t);
/* The same, also adding every triangle test to tri_counts[num_tris] (kernel.cu:133). */
int      or_trace_batch_counts(const or_scene* sc, uint32_t n, const float* rays, int32_t* tri, float* t,
                               uint32_t* tri_counts);

/* ---- integrators */
/* kernel.cu:417-515 radianceAlongSingleStep2 (integrator 0) */
void     or_radiance_unidir(const or_scene* sc, or_vec3 o, or_vec3 dir, int bounces,
                            or_xorwow* rng, double out[3], or_counters* cnt);
/* kernel.cu:217-415 radianceAlongSingleStep (integrator 1, HEAD default) */
void     or_radiance_head(const or_scene* sc, or_vec3 o, or_vec3 dir,
                          or_xorwow* rng, double out[3], or_counters* cnt);

/* Render the pixels listed in `pixels` (scanline ids y*W+x) with `spp` samples each,
 * writing the f64 running mean (kernel.cu:551-552) into out[(y*W+x)*3 + c].
 * Mirrors kernel.cu:527-553 + 702-737 for one pixel: fresh curand_init(seed, morton(x,y), 0),
 * then samples n = 1..spp (NUM_SAMPLES-1 in the reference).  threads <= 0 -> all cores. */
int      or_render(const or_scene* sc, const or_camera* cam, int width, int height,
                   int spp, int bounces, int integrator, uint64_t seed,
                   const uint32_t* pixels, uint32_t num_pixels, int threads,
                   double* out, or_counters* cnt);

/* ---- output (kernel.cu:763-778, color.h:59-71): the reference's PPM loop over its Morton-indexed
 * framebuffer imgBuffer_host (W*H x 3 f64, pixel (x,y) at mortonPxltoI(x,y)): "P3 W H 255\n", rows
 * y ascending, x descending, "%d %d %d " of (int)(gammaCorrect(normalized(c), 1/2.2)*255).
 * Returns 0, or -1 when the file cannot be written. */
int      or_write_ppm_imgbuf(const char* path, const double* imgbuf, int width, int height);

/* kernel.cu:44-54 getTangent, :101-104 BRDF (the restatement's, exported for golden checks) */
void or_get_tangent(or_vec3 n, or_vec3* out);
void or_brdf(const double albedo[3], double out[3]);

#ifdef __cplusplus
}
#endif
#endif
