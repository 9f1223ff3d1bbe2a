// scene.cpp -- the reference's scene globals and loadOBJ (modelLoader.h:43-47, 125-210),
// camera maps (camera.h:36-97) and the PPM writer (kernel.cu:763-778, color.h:59-71).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <new>
#include <thread>

#include "host_internal.h"

namespace pt {

namespace {
thread_local std::string g_error;

inline pt_vec3 v3(float x, float y, float z) { pt_vec3 r; r.x = x; r.y = y; r.z = z; return r; }
inline pt_vec3 vsub(pt_vec3 a, pt_vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline pt_vec3 vcross(pt_vec3 a, pt_vec3 b)
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline float vlen(pt_vec3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
inline pt_vec3 vunit(pt_vec3 v)
{
    float len = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    return v3(v.x / len, v.y / len, v.z / len);
}

// (int)x on the reference's x86 targets: truncation, "integer indefinite" INT_MIN for NaN
// and out-of-range values (cvttsd2si).  Made explicit so no C++ UB is involved.
inline int trunc_to_int(double x)
{
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
    return static_cast<int>(x);
}
}  // namespace

int fail(int code, const char* fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_error = buf;
    return code;
}

void clear_error() { g_error.clear(); }

const char* last_error_cstr() { return g_error.c_str(); }

}  // namespace pt

using namespace pt;

extern "C" {

const char* pt_last_error(void) { return pt::last_error_cstr(); }
int pt_abi_version(void) { return PT_ABI_VERSION; }

pt_host_scene* pt_scene_new(void) { return new (std::nothrow) pt_host_scene(); }

void pt_scene_free(pt_host_scene* s) { delete s; }

const char* pt_scene_last_warning(const pt_host_scene* s) { return s ? s->s.warning.c_str() : ""; }

int pt_scene_load_obj(pt_host_scene* hs, const char* obj_path, const char* mtl_basepath, pt_vec3 origin,
                      float scale, int flip_normals)
{
    if (!hs || !obj_path) return fail(PT_E_INVALID, "pt_scene_load_obj: null argument");
    HostScene& s = hs->s;
    ObjResult r = read_obj(obj_path, mtl_basepath ? mtl_basepath : "models/");
    s.warning = r.message;
    if (r.fatal) return fail(r.message.rfind("Cannot open", 0) == 0 ? PT_E_IO : PT_E_SCENE, "%s", r.message.c_str());
    // materials are appended twice; triangles index the second copy (modelLoader.h:138-159)
    auto to_mat = [](const ObjMaterial& m) {
        pt_material d;
        for (int c = 0; c < 3; ++c) {
            d.albedo[c] = static_cast<double>(m.diffuse[c]);
            d.emission[c] = static_cast<double>(m.emission[c]);
        }
        return d;
    };
    for (const ObjMaterial& m : r.materials) s.mats.push_back(to_mat(m));
    const uint32_t mat_base = static_cast<uint32_t>(s.mats.size());
    for (const ObjMaterial& m : r.materials) s.mats.push_back(to_mat(m));

    for (const ObjShape& sh : r.shapes) {
        const int32_t vbase = static_cast<int32_t>(s.verts.size());
        const size_t nv = sh.positions.size() / 3;
        for (size_t i = 0; i < nv; ++i) {                                       // :165-172
            s.verts.push_back(v3(sh.positions[3 * i + 0] * scale + origin.x,
                                 sh.positions[3 * i + 1] * scale + origin.y,
                                 sh.positions[3 * i + 2] * scale + origin.z));
        }
        const size_t nt = sh.indices.size() / 3;
        for (size_t i = 0; i < nt; ++i) {                                       // :175-205
            pt_triangle t;
            t.v0 = static_cast<int32_t>(sh.indices[3 * i + 0]) + vbase;
            t.v1 = static_cast<int32_t>(sh.indices[3 * i + 1]) + vbase;
            t.v2 = static_cast<int32_t>(sh.indices[3 * i + 2]) + vbase;
            const pt_vec3 a = s.verts[t.v0], b = s.verts[t.v1], c = s.verts[t.v2];
            // every triangle of a shape takes the shape's first material id (:186)
            t.mat = static_cast<int32_t>(static_cast<uint32_t>(sh.material_ids[0]) + mat_base);
            if (t.mat < 0 || static_cast<size_t>(t.mat) >= s.mats.size())
                return fail(PT_E_SCENE, "%s: triangle uses material %d but only %zu materials are loaded "
                            "(face without usemtl and no mtllib?)", obj_path, t.mat, s.mats.size());
            if (s.mats[t.mat].emission[0] != 0) {                               // :188-196
                s.lights.push_back(static_cast<uint32_t>(s.tris.size()));
                float area = vlen(vcross(vsub(b, a), vsub(c, a))) / 2;
                s.total_light_area += area;
            }
            t.norm = vunit(vcross(vsub(b, a), vsub(c, a)));                     // :198-200
            if (flip_normals) t.norm = v3(t.norm.x * -1, t.norm.y * -1, t.norm.z * -1);
            s.tris.push_back(t);
        }
    }
    s.bvh.clear();
    s.bvh_depth = 0;
    return PT_OK;
}

int pt_scene_add_sphere(pt_host_scene* hs, const pt_sphere* sp)
{
    if (!hs || !sp) return fail(PT_E_INVALID, "pt_scene_add_sphere: null argument");
    if (!(sp->rad > 0.0f) || !std::isfinite(sp->rad) || !std::isfinite(sp->pos.x) || !std::isfinite(sp->pos.y) ||
        !std::isfinite(sp->pos.z))
        return fail(PT_E_INVALID, "pt_scene_add_sphere: radius must be > 0 and the sphere finite");
    HostScene& s = hs->s;
    if (sp->emission[0] != 0) {
        s.lights.push_back(PT_LIGHT_SPHERE | static_cast<uint32_t>(s.spheres.size()));
        s.total_light_area += sphere_area(sp->rad);
    }
    s.spheres.push_back(*sp);
    return PT_OK;
}

int pt_scene_build_bvh(pt_host_scene* hs)
{
    if (!hs) return fail(PT_E_INVALID, "pt_scene_build_bvh: null scene");
    HostScene& s = hs->s;
    if (s.tris.empty() && !s.spheres.empty()) {   // spheres only: no triangle BVH (config C1)
        s.bvh.clear();
        s.bvh_depth = 0;
        return PT_OK;
    }
    int rc = build_bvh(s.verts, s.tris, &s.bvh, &s.bvh_depth);
    if (rc != PT_OK) return rc;
    if (s.bvh_depth >= PT_MAX_BVH_DEPTH)                                        // kernel.cu:627-631
        return fail(PT_E_BVH_DEPTH, "Critical Error: BVH depth is too big (%d >= %d)", s.bvh_depth, PT_MAX_BVH_DEPTH);
    return PT_OK;
}

int pt_scene_view(const pt_host_scene* hs, pt_scene* out)
{
    if (!hs || !out) return fail(PT_E_INVALID, "pt_scene_view: null argument");
    const HostScene& s = hs->s;
    out->num_verts = static_cast<uint32_t>(s.verts.size());
    out->num_tris = static_cast<uint32_t>(s.tris.size());
    out->num_mats = static_cast<uint32_t>(s.mats.size());
    out->num_lights = static_cast<uint32_t>(s.lights.size());
    out->verts = s.verts.data();
    out->tris = s.tris.data();
    out->mats = s.mats.data();
    out->lights = s.lights.data();
    out->total_light_area = s.total_light_area;
    out->bvh = s.bvh.data();
    out->bvh_size = static_cast<uint32_t>(s.bvh.size());
    out->bvh_depth = s.bvh_depth;
    out->spheres = s.spheres.data();
    out->num_spheres = static_cast<uint32_t>(s.spheres.size());
    return PT_OK;
}

// camera.h:66-75
uint32_t pt_morton_pxl_to_i(uint32_t x, uint32_t y)
{
    uint32_t r = 0;
    for (int b = 0; b < 16; ++b) {
        r |= ((x >> b) & 1u) << (2 * b);
        r |= ((y >> b) & 1u) << (2 * b + 1);
    }
    return r;
}

// camera.h:57-65 (outputs are uint16_t in the reference)
void pt_morton_i_to_pxl(uint32_t idx, uint32_t* x, uint32_t* y)
{
    uint32_t xx = 0, yy = 0;
    for (int b = 0; b < 16; ++b) {
        xx |= ((idx >> (2 * b)) & 1u) << b;
        yy |= ((idx >> (2 * b + 1)) & 1u) << b;
    }
    if (x) *x = xx & 0xffffu;
    if (y) *y = yy & 0xffffu;
}

// camera.h:77-97; the lens angle goes through the same deterministic sin/cos as the kernels.
void pt_camera_ray(const pt_camera* cam, uint32_t idx, int lens, float u1, float u2, pt_vec3* origin, pt_vec3* dir)
{
    uint32_t px, py;
    pt_morton_i_to_pxl(idx, &px, &py);
    pt_vec3 film = v3(static_cast<float>(px) / static_cast<float>(cam->pxl_width) - 0.5f,
                      static_cast<float>(py) / static_cast<float>(cam->pxl_height) - 0.5f, 0.0f);
    pt_vec3 o = v3(0.0f, 0.0f, 0.0f);
    if (lens) {
        float r = cam->radius * sqrtf(u1);
        float theta = static_cast<float>(2 * 3.14159 * static_cast<double>(u2));
        float sn, cs;
        pt::sincos_det(theta, &sn, &cs);
        o = v3(r * cs, r * sn, 0.0f);
    }
    film.z = cam->dist_from_film;
    const float k = -cam->focal_length;
    film = v3(film.x * k / cam->dist_from_film, film.y * k / cam->dist_from_film, film.z * k / cam->dist_from_film);
    *origin = v3(o.x + cam->pos.x, o.y + cam->pos.y, o.z + cam->pos.z);
    *dir = vunit(vsub(film, o));
}

// kernel.cu:771 -> color.h:59-62 normalized, color.h:68-71 gammaCorrect(c, 1/2.2), (int)(c*255)
int pt_tonemap_u8(double c)
{
    double n = c / (c + 1);
    double g = pow(n, static_cast<double>(static_cast<float>(1 / 2.2)));
    return trunc_to_int(g * 255);
}

}  // extern "C"

namespace {
template <typename T>
int write_ppm_any(const char* path, const T* rgb, int w, int h, int order = PT_ORDER_SCANLINE)
{
    if (!path || !rgb || w <= 0 || h <= 0) return fail(PT_E_INVALID, "pt_write_ppm: bad arguments");
    if (order != PT_ORDER_SCANLINE && order != PT_ORDER_MORTON) return fail(PT_E_INVALID, "pt_write_ppm: pixel order %d", order);
    if (order == PT_ORDER_MORTON && !pt::morton_size_ok(w, h))
        return fail(PT_E_INVALID, "pt_write_ppm: Morton order needs a square power-of-two image (%dx%d)", w, h);
    FILE* fp = fopen(path, "w");
    if (!fp) return fail(PT_E_IO, "pt_write_ppm: cannot open %s", path);
    fprintf(fp, "P3 %d %d 255\n", w, h);
    for (int y = 0; y < h; ++y) {
        for (int x = w - 1; x >= 0; --x) {                                     // mirrored, kernel.cu:766
            const size_t idx = order == PT_ORDER_MORTON ? pt_morton_pxl_to_i((uint32_t)x, (uint32_t)y)   // kernel.cu:771
                                                        : static_cast<size_t>(y) * w + x;
            const T* p = rgb + idx * 3;
            fprintf(fp, "%d %d %d ", pt_tonemap_u8(static_cast<double>(p[0])), pt_tonemap_u8(static_cast<double>(p[1])),
                    pt_tonemap_u8(static_cast<double>(p[2])));
        }
    }
    if (fclose(fp) != 0) return fail(PT_E_IO, "pt_write_ppm: write failed for %s", path);
    return PT_OK;
}
}  // namespace

extern "C" int pt_write_ppm(const char* path, const float* rgb, int width, int height)
{
    return write_ppm_any(path, rgb, width, height);
}

extern "C" int pt_write_ppm_order(const char* path, const float* rgb, int width, int height, int pixel_order)
{
    return write_ppm_any(path, rgb, width, height, pixel_order);
}

// The reference's PPM text (kernel.cu:763-778) from tone-mapped codes (pt_tonemap / GPU).
extern "C" int pt_write_ppm_codes(const char* path, const int32_t* codes, int w, int h)
{
    if (!path || !codes || w <= 0 || h <= 0) return fail(PT_E_INVALID, "pt_write_ppm_codes: bad arguments");
    FILE* fp = fopen(path, "w");
    if (!fp) return fail(PT_E_IO, "pt_write_ppm_codes: cannot open %s", path);
    fprintf(fp, "P3 %d %d 255\n", w, h);
    for (int y = 0; y < h; ++y)
        for (int x = w - 1; x >= 0; --x) {                                         // mirrored, kernel.cu:766
            const int32_t* p = codes + (static_cast<size_t>(y) * w + x) * 3;
            fprintf(fp, "%d %d %d ", p[0], p[1], p[2]);
        }
    if (fclose(fp) != 0) return fail(PT_E_IO, "pt_write_ppm_codes: write failed for %s", path);
    return PT_OK;
}

// Portable float map of the fp32 mean image (little-endian, scale -1, rows bottom-up per the
// PFM convention): the lossless dump for parity checks.
extern "C" int pt_write_pfm(const char* path, const float* rgb, int w, int h)
{
    if (!path || !rgb || w <= 0 || h <= 0) return fail(PT_E_INVALID, "pt_write_pfm: bad arguments");
    FILE* fp = fopen(path, "wb");
    if (!fp) return fail(PT_E_IO, "pt_write_pfm: cannot open %s", path);
    fprintf(fp, "PF\n%d %d\n-1.0\n", w, h);
    bool ok = true;
    for (int y = h - 1; y >= 0 && ok; --y)
        ok = fwrite(rgb + static_cast<size_t>(y) * w * 3, sizeof(float), static_cast<size_t>(w) * 3, fp) ==
             static_cast<size_t>(w) * 3;
    if (fclose(fp) != 0 || !ok) return fail(PT_E_IO, "pt_write_pfm: write failed for %s", path);
    return PT_OK;
}

namespace pt {
// the sizes for which the reference's Morton framebuffer (idx < W*H, camera.h:57-75) covers the
// image one-to-one: square powers of two
bool morton_size_ok(int w, int h)
{
    return w > 0 && w == h && (w & (w - 1)) == 0 && w <= 65536;
}

unsigned host_threads()
{
    for (const char* var : {"PT_HOST_THREADS", "OMP_NUM_THREADS"}) {
        if (const char* e = getenv(var)) {
            const int v = atoi(e);
            if (v > 0) return static_cast<unsigned>(v < 64 ? v : 64);
        }
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return hw == 0 ? 1u : (hw < 16 ? hw : 16u);
}

// Tone-map thresholds for the GPU output step: t[k] (k = 1..255) = the smallest non-negative
// float c with pt_tonemap_u8(c) >= k.  The map is monotone in c (c/(c+1), pow, *255 and the
// truncation all are), so for finite c >= 0 the code is the number of thresholds <= c, exactly
// as this host's libm computes it.  t[0] = 0.  Returns false if a bisection finds the map
// non-monotone at a boundary (then the device step must not be used).
bool tonemap_thresholds(float t[256])
{
    t[0] = 0.0f;
    bool ok = true;
    for (int k = 1; k < 256; ++k) {
        uint32_t lo = 0, hi = 0x7f7fffffu;   // [0, FLT_MAX]; f(FLT_MAX) = 255
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            float c;
            memcpy(&c, &mid, 4);
            if (pt_tonemap_u8(static_cast<double>(c)) >= k) hi = mid; else lo = mid + 1;
        }
        memcpy(&t[k], &lo, 4);
        if (pt_tonemap_u8(static_cast<double>(t[k])) < k) ok = false;
        if (lo > 0) {
            float below;
            const uint32_t b = lo - 1;
            memcpy(&below, &b, 4);
            if (pt_tonemap_u8(static_cast<double>(below)) >= k) ok = false;
        }
        if (k > 1 && t[k] < t[k - 1]) ok = false;
    }
    return ok;
}
}  // namespace pt

extern "C" int pt_write_ppm_f64(const char* path, const double* rgb, int width, int height)
{
    return write_ppm_any(path, rgb, width, height);
}
