// pt_cli -- the reference's program (kernel.cu:565-790 `main`) as a command-line tool over the
// C-ABI of include/pt/pt.h: load OBJ models (loadOBJ, kernel.cu:589-599), build the BVH
// (:601, depth guard :627-631), render (:702-737), report rates (:753-757, in 64-bit), tone-map
// on the GPU and write the PPM (:763-778), optionally a PFM float dump.
//
//   pt_cli --obj models/CornellBox-Original.obj --obj models/teapot.obj@0.35,0.6,0.3@0.75 \
//          --width 512 --height 512 --spp 99 --bounces 3 --out image.ppm [--pfm image.pfm]
//
// --obj PATH[@ox,oy,oz[@scale[@flip]]]   loadOBJ(path, mtl dir, origin, scale, flipNormals)
// --num-samples N                         the reference's NUM_SAMPLES (renders N-1 samples);
//                                         --spp gives the sample count directly
// --gpus N                                shard image tiles over devices 0..N-1 (pt_render_multi:
//                                         one context per device, one RCCL reduce of the shards)
// --morton                                render into the reference's Morton-indexed framebuffer
//                                         (square power-of-two sizes); --tile WxH sets the shard tile
// --tri-counts out.csv                    per-triangle test counts (the reference's out.csv,
//                                         kernel.cu:742-750); --reference-walk makes them the
//                                         reference's own (its exact trace() sequence)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pt/pt.h"

namespace {

struct Obj {
    std::string path;
    pt_vec3 origin{0, 0, 0};
    float scale = 1.0f;
    int flip = 0;
};

[[noreturn]] void usage(const char* msg)
{
    if (msg) fprintf(stderr, "pt_cli: %s\n", msg);
    fprintf(stderr,
            "usage: pt_cli --obj PATH[@ox,oy,oz[@scale[@flip]]] [--obj ...] [--mtl-dir DIR]\n"
            "              [--width W] [--height H] [--spp N | --num-samples N] [--bounces D]\n"
            "              [--integrator unidir|head] [--seed S] [--cam X,Y,Z] [--dist D] [--focal F]\n"
            "              [--radius R] [--gpus N] [--out image.ppm] [--pfm image.pfm] [--quiet]\n"
            "              [--tri-counts out.csv [--reference-walk]] [--morton] [--tile WxH]\n");
    exit(2);
}

bool parse_vec3(const std::string& s, pt_vec3* v)
{
    return sscanf(s.c_str(), "%f,%f,%f", &v->x, &v->y, &v->z) == 3;
}

Obj parse_obj(const std::string& arg)
{
    Obj o;
    std::vector<std::string> parts;
    size_t b = 0;
    for (size_t e; (e = arg.find('@', b)) != std::string::npos; b = e + 1) parts.push_back(arg.substr(b, e - b));
    parts.push_back(arg.substr(b));
    o.path = parts[0];
    if (parts.size() > 1 && !parse_vec3(parts[1], &o.origin)) usage("bad --obj origin");
    if (parts.size() > 2) o.scale = strtof(parts[2].c_str(), nullptr);
    if (parts.size() > 3) o.flip = atoi(parts[3].c_str());
    return o;
}

std::string dir_of(const std::string& p)
{
    const size_t k = p.find_last_of('/');
    return k == std::string::npos ? std::string("./") : p.substr(0, k + 1);
}

int die(const char* what)
{
    fprintf(stderr, "pt_cli: %s: %s\n", what, pt_last_error());
    return 1;
}

}  // namespace

int main(int argc, char** argv)
{
    std::vector<Obj> objs;
    std::string mtl_dir, out = "image.ppm", pfm;
    pt_params p{};
    p.width = 512; p.height = 512; p.spp = 99; p.bounces = 3;   // kernel.cu:29-33 defaults
    p.integrator = PT_INTEGRATOR_UNIDIR; p.seed = 1234; p.shard_index = 0; p.shard_count = 1;
    pt_camera cam{{0, 1, 3}, 1, 3, 0, 0, 0};                      // kernel.cu:642-648
    int gpus = 1;
    bool quiet = false, ref_walk = false;
    std::string tri_csv;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) usage(("missing value for " + a).c_str());
            return argv[++i];
        };
        if (a == "--obj") objs.push_back(parse_obj(next()));
        else if (a == "--mtl-dir") mtl_dir = next();
        else if (a == "--width") p.width = atoi(next().c_str());
        else if (a == "--height") p.height = atoi(next().c_str());
        else if (a == "--spp") p.spp = atoi(next().c_str());
        else if (a == "--num-samples") p.spp = atoi(next().c_str()) - 1;   // kernel.cu:709-710
        else if (a == "--bounces") p.bounces = atoi(next().c_str());
        else if (a == "--integrator") {
            const std::string v = next();
            if (v == "unidir") p.integrator = PT_INTEGRATOR_UNIDIR;
            else if (v == "head") p.integrator = PT_INTEGRATOR_HEAD;
            else usage("--integrator is unidir or head");
        } else if (a == "--seed") p.seed = strtoull(next().c_str(), nullptr, 10);
        else if (a == "--cam") { if (!parse_vec3(next(), &cam.pos)) usage("bad --cam"); }
        else if (a == "--dist") cam.dist_from_film = strtof(next().c_str(), nullptr);
        else if (a == "--focal") cam.focal_length = strtof(next().c_str(), nullptr);
        else if (a == "--radius") cam.radius = strtof(next().c_str(), nullptr);
        else if (a == "--gpus") gpus = atoi(next().c_str());
        else if (a == "--out") out = next();
        else if (a == "--pfm") pfm = next();
        else if (a == "--quiet") quiet = true;
        else if (a == "--tri-counts") tri_csv = next();
        else if (a == "--reference-walk") ref_walk = true;
        else if (a == "--morton") p.pixel_order = PT_ORDER_MORTON;   // the reference's imgBuff order
        else if (a == "--tile") {
            if (sscanf(next().c_str(), "%dx%d", &p.tile_w, &p.tile_h) != 2) usage("--tile is WxH");
        }
        else if (a == "-h" || a == "--help") usage(nullptr);
        else usage(("unknown option " + a).c_str());
    }
    if (objs.empty()) usage("at least one --obj is required");
    if (gpus < 1) usage("--gpus must be >= 1");
    if (!tri_csv.empty() && gpus != 1) usage("--tri-counts needs --gpus 1");
    if (!tri_csv.empty()) p.flags |= PT_FLAG_COUNT | PT_FLAG_TRI_COUNTS;
    // --reference-walk: the reference's own trace() sequence for every sample (its node order, the
    // camera ray traced per sample, dead paths traced), so --tri-counts reproduces its out.csv
    if (ref_walk) p.flags |= PT_FLAG_REFERENCE_TRAVERSAL | PT_FLAG_NO_PRIMARY_CACHE | PT_FLAG_NO_DEAD_PATH_SKIP;
    cam.pxl_width = p.width;
    cam.pxl_height = p.height;

    const auto t0 = std::chrono::steady_clock::now();
    pt_host_scene* s = pt_scene_new();
    for (const Obj& o : objs) {
        const std::string md = mtl_dir.empty() ? dir_of(o.path) : mtl_dir;
        if (pt_scene_load_obj(s, o.path.c_str(), md.c_str(), o.origin, o.scale, o.flip) != PT_OK) return die("loadOBJ");
        const char* warn = pt_scene_last_warning(s);
        if (warn && *warn && !quiet) fprintf(stderr, "%s", warn);
    }
    if (pt_scene_build_bvh(s) != PT_OK) return die("buildBVH");
    pt_scene view;
    pt_scene_view(s, &view);
    const double t_load = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!quiet)
        printf("scene: %u triangles, %u lights, BVH depth %d (load + build %.3f s)\n", view.num_tris, view.num_lights,
               view.bvh_depth, t_load);

    const size_t n = (size_t)p.width * p.height * 3;
    std::vector<pt_ctx*> ctx(gpus, nullptr);
    for (int g = 0; g < gpus; ++g) {
        int err = 0;
        ctx[g] = pt_create(&view, g, &err);
        if (!ctx[g]) return die("pt_create");
    }
    std::vector<float> img(n, 0.0f);
    pt_stats st{};
    const auto t1 = std::chrono::steady_clock::now();
    // one GPU: pt_render; N GPUs: image-tile shards on devices 0..N-1 summed by one RCCL reduce
    const int rc = (gpus == 1) ? pt_render(ctx[0], &p, &cam, img.data(), &st)
                               : pt_render_multi(ctx.data(), gpus, &p, &cam, img.data(), &st);
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    if (rc != PT_OK) return die("pt_render");
    const uint64_t samples = st.samples, traced = st.rays_traced, reference = st.rays_reference;
    const uint64_t nominal = st.rays_nominal;   // (summed over the shards)
    if (!tri_csv.empty()) {
        // kernel.cu:742-750: one "count,\n" line per entry of the reference's test[] buffer, which
        // has bvh.size = numTris-1 entries (kernel.cu:696)
        std::vector<uint32_t> counts(view.num_tris);
        if (pt_tri_counts(ctx[0], counts.data(), view.num_tris) != PT_OK) return die("pt_tri_counts");
        FILE* f = fopen(tri_csv.c_str(), "w");
        if (!f) { fprintf(stderr, "pt_cli: cannot write %s\n", tri_csv.c_str()); return 1; }
        for (uint32_t k = 0; k + 1 < view.num_tris; ++k) fprintf(f, "%u,\n", counts[k]);
        fclose(f);
    }
    if (!quiet) {
        printf("%d GPU(s): %.3f s, %.1f Msamples/s, %.1f Mrays/s traced, %.1f Mrays/s reference-equivalent, "
               "%.1f Mrays/s nominal (kernel.cu:757)\n",
               gpus, secs, samples / secs / 1e6, traced / secs / 1e6, reference / secs / 1e6, nominal / secs / 1e6);
    }
    if (p.pixel_order == PT_ORDER_MORTON) {
        // the buffer as the reference holds it (imgBuff[mortonPxltoI(x,y)]): the PPM loop of
        // kernel.cu:763-778 reads it through the Morton map
        if (pt_write_ppm_order(out.c_str(), img.data(), p.width, p.height, PT_ORDER_MORTON) != PT_OK) return die("write PPM");
        if (!pfm.empty()) {
            std::vector<float> scan(n);
            for (int y = 0; y < p.height; ++y)
                for (int x = 0; x < p.width; ++x)
                    memcpy(&scan[((size_t)y * p.width + x) * 3], &img[(size_t)pt_morton_pxl_to_i(x, y) * 3], 12);
            if (pt_write_pfm(pfm.c_str(), scan.data(), p.width, p.height) != PT_OK) return die("write PFM");
        }
    } else {
        std::vector<int32_t> codes(n);
        if (pt_tonemap(ctx[0], img.data(), p.width, p.height, codes.data()) != PT_OK) return die("tone map");
        if (pt_write_ppm_codes(out.c_str(), codes.data(), p.width, p.height) != PT_OK) return die("write PPM");
        if (!pfm.empty() && pt_write_pfm(pfm.c_str(), img.data(), p.width, p.height) != PT_OK) return die("write PFM");
    }
    for (pt_ctx* c : ctx) pt_destroy(c);
    pt_scene_free(s);
    return 0;
}
