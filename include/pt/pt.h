/*
 * pt.h -- C-ABI of the MI355X-native path tracer (libptamd.so).
 *
 * Drop-in boundary for CulDeVu/CUDAPathTracer's render call.  Plain C types,
 * plain pointers and sizes; no torch, no HIP types in any signature.
 *
 * Two halves:
 *   1. Host surface (plain C++ behind C entry points), the reference's callers of the path:
 *        pt_scene_*      <- modelLoader.h:43-47 globals + loadOBJ (modelLoader.h:125-210)
 *                           via tinyobj::LoadObj (tiny_obj_loader.cc:638-884)
 *        pt_scene_build_bvh <- buildBVH (BVH.h:443-474) + depth guard (kernel.cu:627-631)
 *        pt_camera_ray / pt_morton_* <- camera.h:36-97
 *        pt_write_ppm    <- kernel.cu:763-778 + color.h:59-71
 *   2. Render (hand-written gfx950 HIP kernels):
 *        pt_create       <- the uploads of kernel.cu:637-700 (scene, camera, BVH to device)
 *        pt_render       <- setupCurand (kernel.cu:527-533, :639) + setupImgBuffer (:520-526, :662)
 *                           + the NUM_SAMPLES-1 launches of drawPixel (kernel.cu:535-553, :709-736)
 *        pt_destroy      <- cudaFree (kernel.cu:782-783)
 *        pt_last_error   <- checkError (kernel.cu:37-42), but returned instead of printed
 *
 * Errors: every int-returning entry point returns PT_OK (0) or a negative PT_E* code and
 * records a message for pt_last_error() (thread-local).  Nothing calls exit().
 * Ownership: the caller owns every array it passes; pt_create copies what it needs and keeps
 * no pointer into caller memory.  A pt_ctx is used by one host thread at a time.
 */
#ifndef PT_PT_H
#define PT_PT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 6

/* ---- status codes */
#define PT_OK 0
#define PT_E_INVALID (-1)    /* bad argument                                              */
#define PT_E_IO (-2)         /* cannot open / read / write a file                          */
#define PT_E_SCENE (-3)      /* scene unusable (fewer than 2 triangles, bad indices, ...)  */
#define PT_E_BVH_DEPTH (-4)  /* BVH depth >= 64 (kernel.cu:627-631 "BVH depth is too big") */
#define PT_E_HIP (-5)        /* HIP runtime error (message names the call)                 */
#define PT_E_NODEV (-6)      /* no gfx950 device / device index out of range               */
#define PT_E_OOM (-7)

/* ---- POD mirrors of the reference layouts (static_assert'ed in the implementation) */
typedef struct { float x, y, z; } pt_vec3;                                      /* vec3.h:4-7, 12 B       */
typedef struct { int32_t v0, v1, v2; pt_vec3 norm; int32_t mat; } pt_triangle; /* modelLoader.h:14-19, 28 B */
typedef struct { double albedo[3]; double emission[3]; } pt_material;          /* modelLoader.h:21-25, 48 B */
typedef struct { pt_vec3 lo, hi; uint32_t left, right; } pt_bvh_node;          /* BVH.h:111-115, 32 B    */
typedef struct {                                                                /* camera.h:26-34, 32 B   */
    pt_vec3 pos;
    float dist_from_film;
    float focal_length;
    float radius;
    int32_t pxl_width, pxl_height;
} pt_camera;

#define PT_BVH_LEAF_FLAG 0x80000000u   /* limits.h:6 */
#define PT_MAX_BVH_DEPTH 64            /* kernel.cu:35 */
#define PT_LIGHT_SPHERE 0x80000000u    /* lights[] entry: PT_LIGHT_SPHERE | sphere index    */

/* sphere.h:7-12 (64 B).  The reference has the struct but no intersection code (its include is
 * commented out, kernel.cu:21); the semantics here are this build's:
 * hit ids num_tris + i, closest root with 0 < t < MAX_FLOAT, normal (p - pos) / rad, material
 * {diffuse, emission}; emissive spheres are area lights of area 4*3.14159*rad^2. */
typedef struct { pt_vec3 pos; float rad; double diffuse[3]; double emission[3]; } pt_sphere;

/* Read-only view of a scene: sceneDesc (modelLoader.h:29-41) + BVH_array (BVH.h:116-121). */
typedef struct {
    uint32_t num_verts, num_tris, num_mats, num_lights;
    const pt_vec3* verts;
    const pt_triangle* tris;
    const pt_material* mats;
    const uint32_t* lights;
    float total_light_area;
    const pt_bvh_node* bvh;    /* breadth-first array, node 0 = root            */
    uint32_t bvh_size;         /* = num_tris - 1 (0 for a scene of spheres only) */
    int32_t bvh_depth;         /* BVH_node::depth of the root (BVH.h:322, :346)  */
    const pt_sphere* spheres;  /* sphere primitives (hit ids num_tris + i)      */
    uint32_t num_spheres;
} pt_scene;

/* ======================================================================= host surface */
typedef struct pt_host_scene pt_host_scene;

/* Empty scene (the reference's global vectors, modelLoader.h:43-47, as an object). */
pt_host_scene* pt_scene_new(void);
void pt_scene_free(pt_host_scene* s);

/* loadOBJ(filename, origin, scale, flipNormals) -- modelLoader.h:125-210.  Appends to the
 * scene exactly as the reference appends to its globals.  mtl_basepath: the directory
 * prefix tinyobj prepends to `mtllib` names (the reference hard-codes "models/",
 * modelLoader.h:132); NULL means "models/".  A tinyobj warning/error (e.g. a missing .mtl,
 * which makes tinyobj stop reading the OBJ at the mtllib line) does not fail the call, as in
 * the reference: it is returned through pt_scene_last_warning(). */
int pt_scene_load_obj(pt_host_scene* s, const char* obj_path, const char* mtl_basepath,
                      pt_vec3 origin, float scale, int flip_normals);
const char* pt_scene_last_warning(const pt_host_scene* s);

/* buildBVH() -- BVH.h:443-474, byte-identical node array.  Fails with PT_E_SCENE for
 * fewer than 2 triangles (decision d5) and PT_E_BVH_DEPTH when depth >= 64. */
int pt_scene_build_bvh(pt_host_scene* s);

/* Append a sphere primitive (sphere.h); an emissive one (emission[0] != 0, the triangle rule of
 * modelLoader.h:188) joins the light list and totalLightArea.  rad must be finite and > 0. */
int pt_scene_add_sphere(pt_host_scene* scene, const pt_sphere* sphere);

/* Borrow a view of the scene arrays (valid until the next mutation or pt_scene_free). */
int pt_scene_view(const pt_host_scene* s, pt_scene* out);

/* camera.h:57-75 Morton maps and camera.h:77-97 cameraRay.  `lens` = 0: no lens draws
 * (exactly zero lens offset); otherwise (u1,u2) are the lens draws. */
uint32_t pt_morton_pxl_to_i(uint32_t x, uint32_t y);
void pt_morton_i_to_pxl(uint32_t idx, uint32_t* x, uint32_t* y);
void pt_camera_ray(const pt_camera* cam, uint32_t idx, int lens, float u1, float u2,
                   pt_vec3* origin, pt_vec3* dir);

/* kernel.cu:763-778: "P3 W H 255\n" then "%d %d %d " for rows y = 0..H-1 and x = W-1..0,
 * c = (int)(pow(c/(c+1), (float)(1/2.2)) * 255).  rgb is the scanline mean buffer written by
 * pt_render (pixel (x,y) at rgb[(y*W + x)*3]); the f64 variant takes the reference's own
 * double accumulator type. */
int pt_write_ppm(const char* path, const float* rgb, int width, int height);
/* Same for a buffer in either pixel order (PT_ORDER_MORTON: the reference's imgBuffer_host
 * indexing, kernel.cu:771; square power-of-two sizes only). */
int pt_write_ppm_order(const char* path, const float* rgb, int width, int height, int pixel_order);
int pt_write_ppm_f64(const char* path, const double* rgb, int width, int height);
/* PPM tone map of one value: (int)(pow(c/(c+1), (double)(float)(1/2.2)) * 255). */
int pt_tonemap_u8(double c);

/* The PPM text of kernel.cu:763-778 from already tone-mapped codes codes[(y*W+x)*3+k] (the
 * values pt_tonemap_u8 / pt_tonemap produce), and a PFM float dump of the fp32 mean image
 * (lossless; rows bottom-up, little-endian, per the PFM format). */
int pt_write_ppm_codes(const char* path, const int32_t* codes, int width, int height);
int pt_write_pfm(const char* path, const float* rgb, int width, int height);

/* ============================================================================ render */
typedef struct pt_ctx pt_ctx;

#define PT_INTEGRATOR_UNIDIR 0   /* radianceAlongSingleStep2, kernel.cu:417-515 (north star) */
#define PT_INTEGRATOR_HEAD 1     /* radianceAlongSingleStep,  kernel.cu:217-415 (HEAD :549)  */

/* pt_params.flags */
#define PT_FLAG_REFERENCE_TRAVERSAL 0x1u  /* left-first stack walk with no distance culling,
                                             the exact node/triangle sequence of kernel.cu:112-161 */
#define PT_FLAG_NO_DEAD_PATH_SKIP 0x2u    /* trace every bounce even after the path weight is 0   */
#define PT_FLAG_NO_PRIMARY_CACHE 0x4u     /* re-trace the (sample-invariant) camera ray per sample  */
#define PT_FLAG_COUNT 0x8u                /* fill node/triangle test counters (slower variant)     */
#define PT_FLAG_REFERENCE_BVH 0x10u       /* culled walk on the reference BVH only (no SAH BVH)     */
#define PT_FLAG_TRI_COUNTS 0x20u          /* with PT_FLAG_COUNT: also the per-triangle test counts of
                                             kernel.cu:133 (read back with pt_tri_counts; one atomic
                                             per triangle test)                                      */

typedef struct {
    int32_t width, height;   /* image size (IMAGE_WIDTH/HEIGHT, kernel.cu:28-29)                    */
    int32_t spp;             /* samples per pixel = the reference's NUM_SAMPLES - 1 (kernel.cu:709) */
    int32_t bounces;         /* NUM_BOUNCES (kernel.cu:33), integrator 0 only, 1..64                 */
    int32_t integrator;      /* PT_INTEGRATOR_*                                                     */
    uint32_t flags;          /* PT_FLAG_*                                                           */
    uint64_t seed;           /* curand_init seed (kernel.cu:532 uses 1234)                          */
    int32_t shard_index;     /* this renderer's shard in [0, shard_count)                           */
    int32_t shard_count;     /* image tiles (tile_w x tile_h) are dealt round-robin: tile t -> shard
                                t % count, tiles numbered row-major                                 */
    int32_t pixel_order;     /* PT_ORDER_*: how the output buffer is indexed                        */
    int32_t tile_w, tile_h;  /* shard tile size in pixels: 0 = 8; multiples of 8 up to 256           */
} pt_params;

/* pt_params.pixel_order.  SCANLINE: pixel (x,y) at out[(y*W + x)*3 + k].  MORTON: at
 * out[mortonPxltoI(x,y)*3 + k] -- the reference's own imgBuff indexing (drawPixel writes
 * imgBuff[idx] with idx the Morton index, kernel.cu:543,552; the PPM loop reads
 * imgBuffer_host[cam.mortonPxltoI(x,y)], kernel.cu:771), defined only where the reference's is:
 * square power-of-two images (others: PT_E_INVALID). */
#define PT_ORDER_SCANLINE 0
#define PT_ORDER_MORTON 1

typedef struct {
    double seconds;            /* device time of the whole render (hipEvent pair around every
                                  launch: RNG seeding, integration, split-pixel finalisation)     */
    double kernel_ms;          /* device time of the integration kernel alone, in ms (its own
                                  hipEvent pair)                                                  */
    uint64_t samples;          /* pixel samples computed                                         */
    uint64_t rays_traced;      /* trace() calls actually executed on the device                   */
    uint64_t rays_reference;   /* trace() calls the reference integrator performs for the same
                                  samples (differs from rays_traced by the primary-ray cache and
                                  the dead-path skip)                                             */
    uint64_t rays_nominal;     /* pixels*spp*(bounces+1) over THIS render's pixels (its shard; the
                                  whole image for pt_render_group): the kernel.cu:757 formula, in
                                  64-bit                                                          */
    uint64_t node_tests;       /* node records fetched (PT_FLAG_COUNT only)                       */
    uint64_t tri_tests;        /* triangle records tested (PT_FLAG_COUNT only)                    */
    uint64_t walk_lane_slots;  /* PT_FLAG_COUNT, wavefront kernel: 64 x BVH-walk iterations; with
                                  node_tests gives the SIMD lane utilisation of the walk          */
    uint64_t leaf_steps;       /* PT_FLAG_COUNT: walk steps that tested a triangle                */
    uint64_t shade_lane_slots; /* PT_FLAG_COUNT, wavefront kernel: 64 x shading passes            */
    uint64_t accel_fallbacks;  /* rays taking the exact reference-BVH walk: outside the fast-path
                                  preconditions, or the BVH4 winner failed the reference-parent
                                  check                                                          */
    uint64_t walk_cycles;      /* PT_FLAG_COUNT, wavefront kernel: wave-clock cycles spent in walk
                                  phases, summed over waves                                     */
    uint64_t shade_cycles;     /* same for shading (+ refill) phases                              */
    uint64_t spill_entries;    /* PT_FLAG_COUNT, BVH4 walk: stack entries pushed beyond the 16-entry
                                  per-lane LDS ring into the lane's HBM spill column (the reference's
                                  fixed stack[64] of kernel.cu:114 has no such tier)              */
    uint64_t lds_node_tests;   /* PT_FLAG_COUNT, wavefront kernel: the node_tests served by the copy
                                  of the BVH4's top nodes in LDS (no vector-memory fetch)         */
    uint64_t work_units;       /* wavefront kernel: work units of this render (whole pixels + sample
                                  chunks of split pixels); 0 for the tile kernel                  */
    uint64_t split_pixels;     /* wavefront kernel: pixel slots split into sample chunks          */
} pt_stats;

/* Host-only diagnostic: builds the render path's private acceleration structure for `scene`
 * exactly as pt_create does (SAH BVH collapsed to BVH4) and returns an FNV-1a digest
 * of it, its BVH4 node count and depth.  Used to check that the parallel host build is
 * deterministic. */
int pt_accel_digest(const pt_scene* scene, uint64_t* digest, uint32_t* num_nodes4, int32_t* depth4);

/* Upload a scene to HIP device `device` (ordinal among visible devices). */
pt_ctx* pt_create(const pt_scene* scene, int device, int* err);

/* Render into a HOST buffer out_rgb[W*H*3] (fp32 mean radiance, in params->pixel_order).  Pixels
 * outside this shard are written as 0.  Blocking.  The image leaves the device through a pinned
 * staging buffer owned by the context (one DMA, then a parallel host copy into out_rgb). */
int pt_render(pt_ctx* ctx, const pt_params* params, const pt_camera* cam, float* out_rgb, pt_stats* stats);

/* Same into a DEVICE buffer d_out[W*H*3] on `stream` (a hipStream_t, NULL = default stream).
 * Only this shard's pixels are written; the caller zero-fills the buffer (a multi-GPU job
 * then sums the shards with one RCCL reduce).  Blocking (it waits for its own events). */
int pt_render_device(pt_ctx* ctx, const pt_params* params, const pt_camera* cam, float* d_out,
                     void* stream, pt_stats* stats);

/* pt_render_device in two halves: _async enqueues the whole render on `stream` and returns at once (up
 * to 2 renders in flight per context, each with its own work buffers: two renders on two streams may run
 * concurrently -- the next frame's blocks start while this one's last waves drain); pt_render_wait waits
 * for the OLDEST render in flight and returns its stats.  Frames queued back to back leave the GPU no
 * idle gap between them (the bench's frame loop).  pt_render_device = _async + wait, and refuses to run
 * while renders are in flight, as do pt_trace* and pt_tri_counts. */
int pt_render_device_async(pt_ctx* ctx, const pt_params* params, const pt_camera* cam, float* d_out, void* stream);
int pt_render_wait(pt_ctx* ctx, pt_stats* stats);

/* The reference's trace() (kernel.cu:112-161) for n rays given as rays[6n] = {o.xyz, d.xyz}
 * (host buffers): tri_out[i] = winning ORIGINAL triangle index or -1, t_out[i] = its closestT
 * (MAX_FLOAT = 1e5 on a miss).  flags: 0 = the render path's walk, PT_FLAG_REFERENCE_BVH = the
 * reference's own stack walk on its BVH.  Bit-identical to the reference for both.  Blocking. */
int pt_trace(pt_ctx* ctx, uint32_t n, const float* rays, int32_t* tri_out, float* t_out, uint32_t flags);

/* trace() as above, plus diagnostics (either may be NULL):
 *   tri_counts[num_tris]: every triangle test of the walk ADDED to tri_counts[original id] --
 *     the reference's test[k] += 1 (kernel.cu:133); with PT_FLAG_REFERENCE_BVH exactly the
 *     reference's counts for these rays, otherwise the tests the render path's walk performed;
 *   spill_entries: BVH4 stack entries pushed past the per-lane LDS ring into HBM. */
int pt_trace_counts(pt_ctx* ctx, uint32_t n, const float* rays, int32_t* tri_out, float* t_out, uint32_t flags,
                    uint32_t* tri_counts, uint64_t* spill_entries);

/* Per-triangle test counts (n = num_tris entries, by original triangle id) of the ctx's last
 * pt_render / pt_render_device with PT_FLAG_COUNT | PT_FLAG_TRI_COUNTS: the reference's bvhIntersection buffer
 * (kernel.cu:694-697, written to out.csv at :742-750).  With PT_FLAG_REFERENCE_TRAVERSAL |
 * PT_FLAG_NO_PRIMARY_CACHE | PT_FLAG_NO_DEAD_PATH_SKIP the render performs exactly the reference's
 * trace() calls, so these are the reference's counts (without its racy increments and with the
 * last triangle's slot, which the reference's numTris-1 buffer lacks). */
int pt_tri_counts(pt_ctx* ctx, uint32_t* counts, uint32_t n);

/* Output step on the GPU (kernel.cu:763-778, color.h:59-71): codes = pt_tonemap_u8(rgb) per
 * channel, identical to the host function (threshold table bisected with the host's libm at
 * pt_create).  _device: device pointers on `stream`, blocking; negative inputs (which the
 * integrator never produces) are written as INT32_MAX for the caller to redo on the host.
 * pt_tonemap: host buffers, negatives handled. */
int pt_tonemap_device(pt_ctx* ctx, const float* d_rgb, int width, int height, int32_t* d_codes, void* stream);
int pt_tonemap(pt_ctx* ctx, const float* rgb, int width, int height, int32_t* codes);

/* ----------------------------------------------------------- one process, N GPUs
 * A group of contexts on distinct devices with one RCCL communicator per device
 * (ncclCommInitAll).  pt_render_group renders shard i of N on context i -- image tiles dealt
 * round-robin, tile t -> context t % N (params' shard fields are ignored) -- concurrently, one
 * host thread and HIP stream per device, each into a zero-filled fp32 framebuffer, then ONE
 * ncclReduce(sum, root = ctxs[0]'s device) over xGMI and one copy of the image to out_rgb:
 * bit-identical to a single-GPU pt_render (every pixel is its shard's value plus zeros).  Stats
 * are summed over the shards; `seconds` is the job's wall time (renders + reduce + copy).
 * Replaces the reference's launch loop (kernel.cu:709-736) and its D2H copy (:760).
 * The group does not own the contexts; destroy it before them. */
/* The pixels shard `shard_index` of `shard_count` renders (tile_w x tile_h tiles, 0 = 8, dealt tile t ->
 * shard t % count): their scanline ids y*W + x, in the order the shard's work slots take them (8x8
 * blocks, Morton order within a block).  out = NULL: only *n_out.  Host-only; the kernels use the same
 * mapping function. */
int pt_shard_pixels(int width, int height, int shard_index, int shard_count, int tile_w, int tile_h, uint32_t* out,
                    uint32_t cap, uint32_t* n_out);

typedef struct pt_group pt_group;
pt_group* pt_group_create(pt_ctx* const* ctxs, int n, int* err);
int pt_group_size(const pt_group* group);
int pt_render_group(pt_group* group, const pt_params* params, const pt_camera* cam, float* out_rgb, pt_stats* stats);
void pt_group_destroy(pt_group* group);
/* create + render + destroy */
int pt_render_multi(pt_ctx* const* ctxs, int n, const pt_params* params, const pt_camera* cam, float* out_rgb,
                    pt_stats* stats);

void pt_destroy(pt_ctx* ctx);
const char* pt_last_error(void);
int pt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
