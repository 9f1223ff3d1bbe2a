// refgen.cpp -- golden-vector generator built from the REFERENCE's own sources.
//
// TEST INFRASTRUCTURE ONLY.  The reference headers are #included in place from
// /root/reference (nothing is copied into this repo).  The only adaptation is on the
// command line / below: CUDA's function-space qualifiers __host__/__device__ are
// defined empty (a host compile), and min/max/abs are brought in from <algorithm>/<cmath>
// as the reference's nvcc build got them from CUDA's math headers.  No header,
// library or generated file is substituted.  kernel.cu as a whole is NOT built (it needs
// cuda_runtime.h, cuRAND, NVML, windows.h and the broken triple.h -- see DESIGN.md); its
// trace() (kernel.cu:107-161: struct triIntersection + trace) needs none of those, so
// oracle/Makefile extracts exactly that span from /root/reference/kernel.cu at build time into
// oracle/_ref/ref_trace.inc (git-ignored, never committed) and it is #included below verbatim,
// with MAX_BVH_DEPTH = 64 as kernel.cu:35 defines it.
//
// Built by oracle/Makefile into oracle/_ref/refgen (git-ignored).  Driven by
// tools/make_golden.py, which writes tests/golden/*.
//
// Commands (all binary I/O little-endian, raw arrays):
//   refgen scene <out_prefix> <obj> <ox> <oy> <oz> <scale> <flip> [<obj> ...]   (cwd = dir holding models/)
//   refgen tri   <in.bin> <out.bin>   in: n x {o[3], d[3], v0[3], v1[3], v2[3]} f32 ; out: n x f32 t
//   refgen aabb  <in.bin> <out.bin>   in: n x {o[3], d[3], lo[3], hi[3]} f32     ; out: n x u8
//   refgen cam   <in.bin> <out.bin>   in: {cam 32 B} + n x {idx u32, u1 f32, u2 f32}; out: n x {o[3], d[3]} f32
//   refgen morton <out.bin> <n>       out: n x {x u16, y u16, back u32} for idx 0..n-1
//   refgen tone  <in.bin> <out.bin>   in: n x 3 f64 ; out: n x 3 i32 = (int)(gammaCorrect(normalized(c), 1/2.2)*255)
//   refgen trace <rays.bin> <out.bin> <counts.bin> <obj> <ox> <oy> <oz> <scale> <flip> [<obj> ...]  (cwd as for scene)
//                in: n x {o[3], d[3]} f32 ; out: n x {triIndex i32, t f32} from kernel.cu:112 trace() on the
//                scene's buildBVH() array; counts: numTris x u32, the trace()'s test[] increments summed
//                over all rays (kernel.cu:133; sized numTris here -- the reference's buffer has
//                bvh.size = numTris-1 entries, kernel.cu:696, so its last increment lands out of bounds)
//   refgen helpers <in.bin> <out.bin> in: n x {normal[3] f32, pad f32, albedo[3] f64}; out: n x {getTangent(normal)[3]
//                f32, pad, BRDF(albedo)[3] f64} -- kernel.cu:44-54 and :101-104, extracted verbatim into
//                oracle/_ref/ref_helpers.inc by oracle/Makefile
//   refgen ppm   <imgbuf.bin> <W> <H>  (writes ./image.ppm, as the reference does)
//                in: W*H x 3 f64, the reference's imgBuffer_host (Morton-indexed: kernel.cu:543,552); the
//                PPM is written by the reference's own output loop (kernel.cu:763-778, "save the file"),
//                extracted verbatim into oracle/_ref/ref_ppm.inc by oracle/Makefile, with IMAGE_WIDTH /
//                IMAGE_HEIGHT (kernel.cu:28-29 #defines) bound to W and H
#include <cstdint>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>
#include <string>
using std::min;
using std::max;
using std::abs;

#define __host__
#define __device__
#include "/root/reference/modelLoader.h"
#include "/root/reference/BVH.h"
#include "/root/reference/camera.h"
#ifdef REFGEN_HELPERS
#include REFGEN_HELPERS    // kernel.cu:44-54 getTangent and :101-104 BRDF, extracted verbatim by oracle/Makefile
#endif
#ifdef REFGEN_TRACE
#define MAX_BVH_DEPTH 64   // kernel.cu:35
#include REFGEN_TRACE      // kernel.cu:107-161, extracted verbatim by oracle/Makefile
#endif

static std::vector<char> slurp(const char* path)
{
    std::vector<char> buf;
    FILE* f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "refgen: cannot open %s\n", path); exit(2); }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    buf.resize((size_t)n);
    if (n && fread(buf.data(), 1, (size_t)n, f) != (size_t)n) { fprintf(stderr, "refgen: short read\n"); exit(2); }
    fclose(f);
    return buf;
}

static void spit(const char* path, const void* p, size_t n)
{
    FILE* f = fopen(path, "wb");
    if (!f) { fprintf(stderr, "refgen: cannot write %s\n", path); exit(2); }
    if (n) fwrite(p, 1, n, f);
    fclose(f);
}

static void spit_s(const std::string& path, const void* p, size_t n) { spit(path.c_str(), p, n); }

int main(int argc, char** argv)
{
    if (argc < 2) { fprintf(stderr, "usage: refgen <cmd> ...\n"); return 2; }
    std::string cmd = argv[1];
    if (cmd == "scene") {
        std::string pre = argv[2];
        for (int a = 3; a + 5 < argc; a += 6) {
            vec3 origin((float)atof(argv[a + 1]), (float)atof(argv[a + 2]), (float)atof(argv[a + 3]));
            loadOBJ(argv[a], origin, (float)atof(argv[a + 4]), atoi(argv[a + 5]) != 0);   // modelLoader.h:125
        }
        spit_s(pre + ".verts.bin", verts.data(), verts.size() * sizeof(vec3));
        spit_s(pre + ".tris.bin", tris.data(), tris.size() * sizeof(triangle));
        spit_s(pre + ".mats.bin", mats.data(), mats.size() * sizeof(materialDesc));
        spit_s(pre + ".lights.bin", lights.data(), lights.size() * sizeof(int32_t));
        float tla = totalLightArea;
        int32_t bvh_size = 0, bvh_depth = 0;
        if (tris.size() >= 2) {
            BVH_array bvh = buildBVH();                                                  // BVH.h:443
            bvh_size = bvh.size;
            bvh_depth = bvh.depth;
            spit_s(pre + ".bvh.bin", bvh.root, (size_t)bvh.size * sizeof(BVH_array_node));
        } else {
            spit_s(pre + ".bvh.bin", nullptr, 0);
        }
        FILE* f = fopen((pre + ".meta.txt").c_str(), "w");
        fprintf(f, "%zu %zu %zu %zu %.9g %a %d %d\n", verts.size(), tris.size(), mats.size(), lights.size(),
                (double)tla, (double)tla, bvh_size, bvh_depth);
        fclose(f);
        return 0;
    }
    if (cmd == "tri") {
        std::vector<char> in = slurp(argv[2]);
        size_t n = in.size() / (15 * 4);
        const float* p = (const float*)in.data();
        std::vector<float> out(n);
        for (size_t i = 0; i < n; ++i) {
            const float* r = p + i * 15;
            vec3 vs[3] = {vec3(r[6], r[7], r[8]), vec3(r[9], r[10], r[11]), vec3(r[12], r[13], r[14])};
            triangle t;
            t.v0 = 0; t.v1 = 1; t.v2 = 2; t.mat = 0;
            out[i] = triIntersect(vec3(r[0], r[1], r[2]), vec3(r[3], r[4], r[5]), vs, &t);  // modelLoader.h:49
        }
        spit(argv[3], out.data(), n * 4);
        return 0;
    }
    if (cmd == "aabb") {
        std::vector<char> in = slurp(argv[2]);
        size_t n = in.size() / (12 * 4);
        const float* p = (const float*)in.data();
        std::vector<uint8_t> out(n);
        for (size_t i = 0; i < n; ++i) {
            const float* r = p + i * 12;
            AABB b;
            b.lo = vec3(r[6], r[7], r[8]);
            b.hi = vec3(r[9], r[10], r[11]);
            out[i] = rayAABBIntersect(vec3(r[0], r[1], r[2]), vec3(r[3], r[4], r[5]), b) ? 1 : 0;  // BVH.h:51
        }
        spit(argv[3], out.data(), n);
        return 0;
    }
    if (cmd == "cam") {
        std::vector<char> in = slurp(argv[2]);
        camera cam;
        memcpy(&cam, in.data(), sizeof(camera));
        size_t n = (in.size() - sizeof(camera)) / 12;
        const char* q = in.data() + sizeof(camera);
        std::vector<float> out(n * 6);
        for (size_t i = 0; i < n; ++i) {
            uint32_t idx; float u1, u2;
            memcpy(&idx, q + i * 12, 4); memcpy(&u1, q + i * 12 + 4, 4); memcpy(&u2, q + i * 12 + 8, 4);
            ray r = cam.cameraRay((int)idx, u1, u2);                                         // camera.h:77
            out[i * 6 + 0] = r.o.x; out[i * 6 + 1] = r.o.y; out[i * 6 + 2] = r.o.z;
            out[i * 6 + 3] = r.dir.x; out[i * 6 + 4] = r.dir.y; out[i * 6 + 5] = r.dir.z;
        }
        spit(argv[3], out.data(), out.size() * 4);
        return 0;
    }
    if (cmd == "morton") {
        int n = atoi(argv[3]);
        camera cam;
        std::vector<uint32_t> out((size_t)n * 2);
        for (int i = 0; i < n; ++i) {
            uint16_t x, y;
            cam.mortonItoPxl(&x, &y, (uint32_t)i);                                          // camera.h:57
            out[(size_t)i * 2] = (uint32_t)x | ((uint32_t)y << 16);
            out[(size_t)i * 2 + 1] = cam.mortonPxltoI(x, y);                                 // camera.h:66
        }
        spit(argv[2], out.data(), out.size() * 4);
        return 0;
    }
    if (cmd == "tone") {
        std::vector<char> in = slurp(argv[2]);
        size_t n = in.size() / 24;
        const double* p = (const double*)in.data();
        std::vector<int32_t> out(n * 3);
        for (size_t i = 0; i < n; ++i) {
            color c = gammaCorrect(normalized(color(p[i * 3], p[i * 3 + 1], p[i * 3 + 2])), 1 / 2.2);  // kernel.cu:771
            out[i * 3 + 0] = (int)(c.r * 255);
            out[i * 3 + 1] = (int)(c.g * 255);
            out[i * 3 + 2] = (int)(c.b * 255);
        }
        spit(argv[3], out.data(), out.size() * 4);
        return 0;
    }
#ifdef REFGEN_TRACE
    if (cmd == "trace") {
        std::vector<char> in = slurp(argv[2]);
        const size_t n = in.size() / 24;
        for (int a = 5; a + 5 < argc; a += 6) {
            vec3 origin((float)atof(argv[a + 1]), (float)atof(argv[a + 2]), (float)atof(argv[a + 3]));
            loadOBJ(argv[a], origin, (float)atof(argv[a + 4]), atoi(argv[a + 5]) != 0);   // modelLoader.h:125
        }
        if (tris.size() < 2) { fprintf(stderr, "refgen trace: need >= 2 triangles\n"); return 2; }
        BVH_array bvh = buildBVH();                                                      // BVH.h:443
        if (bvh.depth >= MAX_BVH_DEPTH) { fprintf(stderr, "refgen trace: BVH depth too big\n"); return 2; }   // kernel.cu:627
        sceneDesc scene;                                                                 // kernel.cu:664-689
        scene.numVerts = (uint32_t)verts.size(); scene.verts = verts.data();
        scene.numTris = (uint32_t)tris.size(); scene.tris = tris.data();
        scene.numMats = (uint32_t)mats.size(); scene.mats = mats.data();
        scene.numLights = (uint32_t)lights.size(); scene.lights = (uint32_t*)lights.data();
        scene.totalLightArea = totalLightArea;
        std::vector<uint32_t> test(tris.size(), 0u);
        std::vector<char> out(n * 8);
        const float* p = (const float*)in.data();
        for (size_t i = 0; i < n; ++i) {
            ray r;
            r.o = vec3(p[6 * i], p[6 * i + 1], p[6 * i + 2]);
            r.dir = vec3(p[6 * i + 3], p[6 * i + 4], p[6 * i + 5]);
            triIntersection h = trace(r, scene, bvh, test.data());                          // kernel.cu:112
            memcpy(&out[8 * i], &h.triIndex, 4);
            memcpy(&out[8 * i + 4], &h.t, 4);
        }
        spit(argv[3], out.data(), out.size());
        spit(argv[4], test.data(), test.size() * 4);
        return 0;
    }
#endif
#ifdef REFGEN_HELPERS
    if (cmd == "helpers") {
        std::vector<char> in = slurp(argv[2]);
        const size_t n = in.size() / 40;
        std::vector<char> out(n * 40, 0);
        for (size_t i = 0; i < n; ++i) {
            float nv[3];
            double alb[3];
            memcpy(nv, &in[40 * i], 12);
            memcpy(alb, &in[40 * i + 16], 24);
            const vec3 t = getTangent(vec3(nv[0], nv[1], nv[2]));                          // kernel.cu:44
            materialDesc m;
            m.albedo = color(alb[0], alb[1], alb[2]);
            m.emmision = color(0.0, 0.0, 0.0);   // (the reference's spelling, modelLoader.h:21-25)
            const color b = BRDF(m, vec3(0, 0, 0), vec3(0, 0, 0));                         // kernel.cu:101
            const float tv[3] = {t.x, t.y, t.z};
            const double bv[3] = {b.r, b.g, b.b};
            memcpy(&out[40 * i], tv, 12);
            memcpy(&out[40 * i + 16], bv, 24);
        }
        spit(argv[3], out.data(), out.size());
        return 0;
    }
#endif
#ifdef REFGEN_PPM
    if (cmd == "ppm") {
        std::vector<char> in = slurp(argv[2]);
        const int img_w = atoi(argv[3]), img_h = atoi(argv[4]);
        if ((size_t)img_w * (size_t)img_h * 24 != in.size()) { fprintf(stderr, "refgen ppm: size mismatch\n"); return 2; }
        const double* p = (const double*)in.data();
        std::vector<color> imgBuffer_host_v((size_t)img_w * img_h);
        for (size_t i = 0; i < imgBuffer_host_v.size(); ++i)
            imgBuffer_host_v[i] = color(p[3 * i], p[3 * i + 1], p[3 * i + 2]);
        color* imgBuffer_host = imgBuffer_host_v.data();
        camera cam;   // (only mortonPxltoI is used, which reads no field)
        memset(&cam, 0, sizeof(cam));
#define IMAGE_WIDTH img_w
#define IMAGE_HEIGHT img_h
#include REFGEN_PPM   // kernel.cu:763-778, verbatim
#undef IMAGE_WIDTH
#undef IMAGE_HEIGHT
        return 0;
    }
#endif
    fprintf(stderr, "refgen: unknown command %s\n", cmd.c_str());
    return 2;
}
