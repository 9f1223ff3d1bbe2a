// host_internal.h -- shared declarations of the host surface (plain C++17, no HIP).
#pragma once

#include <cstdarg>
#include <cstdint>
#include <string>
#include <vector>

#include "pt/pt.h"

static_assert(sizeof(pt_vec3) == 12, "vec3 is 12 B (vec3.h:4-7)");
static_assert(sizeof(pt_triangle) == 28, "triangle is 28 B (modelLoader.h:14-19)");
static_assert(sizeof(pt_material) == 48, "materialDesc is 48 B (modelLoader.h:21-25)");
static_assert(sizeof(pt_sphere) == 64, "sphere.h sphere is 64 B");
static_assert(sizeof(pt_bvh_node) == 32, "BVH_array_node is 32 B (BVH.h:111-115)");
static_assert(sizeof(pt_camera) == 32, "camera is 32 B (camera.h:26-34)");

namespace pt {

// Thread-local error channel behind pt_last_error().
int fail(int code, const char* fmt, ...);
void clear_error();

// The HIP device ordinal a render context lives on (pt_render.hip; used by pt_multi.cpp).
int ctx_device(const pt_ctx* c);

// ---- OBJ/MTL ingest with tinyobj 0.9.13 semantics (tiny_obj_loader.cc) ------------------
// Only what loadOBJ (modelLoader.h:125-210) consumes is kept: positions, per-triangle
// indices, per-triangle material ids, material diffuse/emission.  Vertex dedupe keys still
// include the vt/vn indices, since they decide how many positions a shape gets.
struct ObjMaterial {
    std::string name;
    float diffuse[3];
    float emission[3];
};
struct ObjShape {
    std::string name;
    std::vector<float> positions;       // xyz per deduplicated vertex
    std::vector<uint32_t> indices;      // 3 per triangle
    std::vector<int> material_ids;      // 1 per triangle
};
struct ObjResult {
    std::vector<ObjShape> shapes;
    std::vector<ObjMaterial> materials;
    std::string message;                // tinyobj's returned error/warning string
    bool fatal = false;                 // file could not be opened / malformed index
};
ObjResult read_obj(const std::string& path, const std::string& mtl_basepath);

// Greedy decimal parser of tinyobj's tryParseDouble (tiny_obj_loader.cc:127-241).
bool parse_real(const char* s, const char* end, double* out);

// ---- scene (the reference's globals, modelLoader.h:43-47) -------------------------------
struct HostScene {
    std::vector<pt_vec3> verts;
    std::vector<pt_triangle> tris;
    std::vector<pt_material> mats;
    std::vector<uint32_t> lights;
    float total_light_area = 0.0f;
    std::vector<pt_bvh_node> bvh;
    int32_t bvh_depth = 0;
    std::vector<pt_sphere> spheres;
    std::string warning;
};

// Area of an emissive sphere light: 4*3.14159*r^2 evaluated in float, left to right.
inline float sphere_area(float r) { return 4.0f * 3.14159f * r * r; }

// Deterministic float sin/cos shared with the kernels (defined in hip/pt_render.hip).
void sincos_det(float theta, float* s, float* c);
bool tonemap_thresholds(float t[256]);
// host threads for the parallel builders: PT_HOST_THREADS, else OMP_NUM_THREADS, else the
// hardware concurrency, capped at 16
unsigned host_threads();
bool morton_size_ok(int w, int h);   // square power-of-two image (the reference's Morton imgBuff)
// Device -> host copy of a finished image through a pinned staging buffer (*pinned, grown as needed,
// owned by the caller's context / group; freed with free_pinned): one DMA on `stream` (a
// hipStream_t), then host_threads() threads copy the staging buffer into dst -- a pageable
// destination's first-touch page faults spread over the threads instead of serialising the DMA.
int copy_to_host(void* dst, const void* src_dev, size_t bytes, void* stream, void** pinned, size_t* pinned_bytes);
void free_pinned(void* pinned);

// ---- render-path acceleration structure (accel_build.cpp) --------------------------------
struct AccelNode {
    float box[2][6];       // child boxes (lo xyz, hi xyz), inflated by `margin`
    uint32_t child[2];     // inner node index, or a leaf: PT_BVH_LEAF_FLAG | (count - 1) << 29 | first slot
};
// a leaf of the render-path BVH holds 1..kAccelLeafMax triangles at consecutive leaf slots
constexpr uint32_t kAccelLeafMax = 2;
inline uint32_t accel_leaf_count(uint32_t ref) { return ((ref >> 29) & 3u) + 1u; }
inline uint32_t accel_leaf_slot(uint32_t ref) { return ref & 0x1fffffffu; }
struct AccelBvh {
    std::vector<AccelNode> nodes;        // node 0 = root
    std::vector<uint32_t> leaf_order;    // triangle id of each leaf slot
    float root_box[6];
    int depth = 0;
    float margin = 0.0f;
};
int build_accel(const pt_scene& sc, AccelBvh* out);
// SAH cost of the binary tree: the sum of its inner-node surface areas
double accel_sah_cost(const AccelBvh& acc);

// 4-wide collapse of the binary SAH BVH: each node holds up to 4 children (largest-area
// expansion, at most kAccel4LeafTris triangles in its leaf children), empty slots are
// kAccel4Empty; leaves keep their binary-BVH refs (count and first leaf slot).
constexpr uint32_t kAccel4Empty = 0xffffffffu;
constexpr uint32_t kAccel4LeafTris = 8;    // at most this many triangles in a node's leaf children (kLeafBits)
struct Accel4Node {
    float lo[3][4], hi[3][4];   // [axis][child]
    uint32_t child[4];          // inner node index, PT_BVH_LEAF_FLAG | slot, or kAccel4Empty
};
struct Accel4 {
    std::vector<Accel4Node> nodes;       // node 0 = root
    int depth = 0;
};
int collapse_accel4(const AccelBvh& bin, Accel4* out);
// c_node x inner-node surfaces + c_tri x leaf surfaces x triangles, over the root's (diagnostic)
double accel4_cost(const Accel4& t, const float* root_box, double cn, double ct);
// every node and leaf slot reached once, <= kAccel4LeafTris leaf triangles per node, nested boxes
int validate_accel4(const AccelBvh& bin, const Accel4& t);

// ---- BVH (BVH.h) ------------------------------------------------------------------------
int build_bvh(const std::vector<pt_vec3>& verts, const std::vector<pt_triangle>& tris,
              std::vector<pt_bvh_node>* out, int32_t* depth);

}  // namespace pt

struct pt_host_scene {
    pt::HostScene s;
};
