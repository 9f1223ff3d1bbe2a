// pt_multi.cpp -- one process driving N GPUs: image tiles are dealt round-robin to
// the devices (tile t -> device t % N), each device renders its shard into a zero-filled fp32
// framebuffer on its own HIP stream (one host thread per device, the renders run concurrently),
// and ONE RCCL reduce (sum, root = device 0) over xGMI assembles the image.  Disjoint shards make
// the sum exact: every pixel is x + 0 + ... + 0 = x, so the result is bit-identical to a single
// GPU's render.  This replaces the reference's single-device launch loop (kernel.cu:709-736) and
// its one D2H copy of imgBuffer (kernel.cu:760).
//
// Host code only (no kernels): compiled by hipcc for the HIP runtime API, linked against RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../host/host_internal.h"

struct pt_group {
    std::vector<pt_ctx*> ctx;       // not owned
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    std::vector<float*> fb;         // per device: its shard, zero elsewhere
    float* result = nullptr;        // on dev[0]: the reduced image
    size_t bytes = 0;               // current framebuffer size
    void* pinned = nullptr;         // pinned staging buffer of the image copy-out (pt::copy_to_host)
    size_t pinned_bytes = 0;
};

namespace {

int hip_fail(const char* what, hipError_t e)
{
    return pt::fail(PT_E_HIP, "%s failed: %s", what, hipGetErrorString(e));
}

int nccl_fail(const char* what, ncclResult_t r)
{
    return pt::fail(PT_E_HIP, "%s failed: %s", what, ncclGetErrorString(r));
}

void release(pt_group* g)
{
    for (size_t i = 0; i < g->dev.size(); ++i) {
        (void)hipSetDevice(g->dev[i]);
        if (i < g->fb.size() && g->fb[i]) (void)hipFree(g->fb[i]);
        if (i < g->stream.size() && g->stream[i]) (void)hipStreamDestroy(g->stream[i]);
    }
    if (g->result) {
        (void)hipSetDevice(g->dev[0]);
        (void)hipFree(g->result);
    }
    for (ncclComm_t c : g->comm)
        if (c) (void)ncclCommDestroy(c);
    g->fb.clear();
    g->stream.clear();
    g->comm.clear();
    g->result = nullptr;
    g->bytes = 0;
    pt::free_pinned(g->pinned);
    g->pinned = nullptr;
    g->pinned_bytes = 0;
}

// (re)allocate the per-device framebuffers and device 0's result buffer for `bytes`
int ensure_buffers(pt_group* g, size_t bytes)
{
    if (g->bytes >= bytes) return PT_OK;
    g->bytes = 0;   // (until every buffer below exists: a partial failure reallocates on the next call)
    for (size_t i = 0; i < g->dev.size(); ++i) {
        hipError_t e = hipSetDevice(g->dev[i]);
        if (e != hipSuccess) return hip_fail("hipSetDevice", e);
        if (g->fb[i]) (void)hipFree(g->fb[i]);
        g->fb[i] = nullptr;
        if ((e = hipMalloc(reinterpret_cast<void**>(&g->fb[i]), bytes)) != hipSuccess) return hip_fail("hipMalloc(framebuffer)", e);
    }
    hipError_t e = hipSetDevice(g->dev[0]);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    if (g->result) (void)hipFree(g->result);
    g->result = nullptr;
    if ((e = hipMalloc(reinterpret_cast<void**>(&g->result), bytes)) != hipSuccess) return hip_fail("hipMalloc(result)", e);
    g->bytes = bytes;
    return PT_OK;
}

// shard stats -> job stats: counts add up; times are the slowest device's
void add_stats(pt_stats* sum, const pt_stats& s)
{
    sum->seconds = std::max(sum->seconds, s.seconds);
    sum->kernel_ms = std::max(sum->kernel_ms, s.kernel_ms);
    sum->samples += s.samples;
    sum->rays_traced += s.rays_traced;
    sum->rays_reference += s.rays_reference;
    sum->rays_nominal += s.rays_nominal;
    sum->node_tests += s.node_tests;
    sum->tri_tests += s.tri_tests;
    sum->walk_lane_slots += s.walk_lane_slots;
    sum->leaf_steps += s.leaf_steps;
    sum->shade_lane_slots += s.shade_lane_slots;
    sum->accel_fallbacks += s.accel_fallbacks;
    sum->walk_cycles += s.walk_cycles;
    sum->shade_cycles += s.shade_cycles;
    sum->spill_entries += s.spill_entries;
    sum->lds_node_tests += s.lds_node_tests;
    sum->work_units += s.work_units;
    sum->split_pixels += s.split_pixels;
}

}  // namespace

extern "C" {

pt_group* pt_group_create(pt_ctx* const* ctxs, int n, int* err)
{
    pt::clear_error();
    auto bail = [&](int code) -> pt_group* { if (err) *err = code; return nullptr; };
    if (!ctxs || n < 1) return bail(pt::fail(PT_E_INVALID, "pt_group_create: need >= 1 context"));
    pt_group* g = new (std::nothrow) pt_group();
    if (!g) return bail(pt::fail(PT_E_OOM, "pt_group_create: out of host memory"));
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) { delete g; return bail(pt::fail(PT_E_INVALID, "pt_group_create: context %d is null", i)); }
        const int d = pt::ctx_device(ctxs[i]);
        if (std::find(g->dev.begin(), g->dev.end(), d) != g->dev.end()) {
            delete g;
            return bail(pt::fail(PT_E_INVALID, "pt_group_create: two contexts on device %d (one per device)", d));
        }
        g->ctx.push_back(ctxs[i]);
        g->dev.push_back(d);
    }
    g->comm.assign(n, nullptr);
    g->stream.assign(n, nullptr);
    g->fb.assign(n, nullptr);
    // one communicator per device, all in this process (ncclCommInitAll: no rendezvous needed)
    const ncclResult_t r = ncclCommInitAll(g->comm.data(), n, g->dev.data());
    if (r != ncclSuccess) {
        g->comm.assign(n, nullptr);
        const int code = nccl_fail("ncclCommInitAll", r);
        release(g);
        delete g;
        return bail(code);
    }
    for (int i = 0; i < n; ++i) {
        hipError_t e = hipSetDevice(g->dev[i]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->stream[i], hipStreamNonBlocking);
        if (e != hipSuccess) {
            const int code = hip_fail("hipStreamCreate", e);
            release(g);
            delete g;
            return bail(code);
        }
    }
    if (err) *err = PT_OK;
    return g;
}

void pt_group_destroy(pt_group* g)
{
    if (!g) return;
    release(g);
    delete g;
}

int pt_group_size(const pt_group* g) { return g ? (int)g->ctx.size() : 0; }

int pt_render_group(pt_group* g, const pt_params* params, const pt_camera* cam, float* out_rgb, pt_stats* stats)
{
    pt::clear_error();
    if (!g || !params || !cam || !out_rgb) return pt::fail(PT_E_INVALID, "pt_render_group: null argument");
    if (params->width <= 0 || params->height <= 0 || params->width > 65535 || params->height > 65535)
        return pt::fail(PT_E_INVALID, "pt_render_group: image size %dx%d out of range", params->width, params->height);
    const int n = (int)g->ctx.size();
    const size_t count = (size_t)params->width * (size_t)params->height * 3;
    const size_t bytes = count * sizeof(float);
    if (int rc = ensure_buffers(g, bytes)) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<int> rc(n, PT_OK);
    std::vector<std::string> msg(n);
    std::vector<pt_stats> st(n);
    auto shard = [&](int i) {
        hipError_t e = hipSetDevice(g->dev[i]);
        if (e == hipSuccess) e = hipMemsetAsync(g->fb[i], 0, bytes, g->stream[i]);
        if (e != hipSuccess) {
            rc[i] = PT_E_HIP;
            msg[i] = std::string("hipMemsetAsync: ") + hipGetErrorString(e);
            return;
        }
        pt_params q = *params;
        q.shard_index = i;
        q.shard_count = n;
        memset(&st[i], 0, sizeof(st[i]));
        rc[i] = pt_render_device(g->ctx[i], &q, cam, g->fb[i], g->stream[i], &st[i]);
        if (rc[i] != PT_OK) msg[i] = pt_last_error();   // (the error channel is per thread)
    };
    if (n == 1) {
        shard(0);
    } else {
        std::vector<std::thread> th;
        th.reserve(n);
        for (int i = 0; i < n; ++i) th.emplace_back(shard, i);
        for (std::thread& t : th) t.join();
    }
    for (int i = 0; i < n; ++i)
        if (rc[i] != PT_OK) return pt::fail(rc[i], "pt_render_group: device %d: %s", g->dev[i], msg[i].c_str());
    // the framebuffer sum over xGMI: one reduce, root = device 0
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_fail("ncclGroupStart", r);
    for (int i = 0; i < n; ++i) {
        r = ncclReduce(g->fb[i], i == 0 ? g->result : nullptr, count, ncclFloat, ncclSum, 0, g->comm[i], g->stream[i]);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return nccl_fail("ncclReduce", r);
        }
    }
    if ((r = ncclGroupEnd()) != ncclSuccess) return nccl_fail("ncclGroupEnd", r);
    for (int i = 1; i < n; ++i) {
        hipError_t e = hipSetDevice(g->dev[i]);
        if (e == hipSuccess) e = hipStreamSynchronize(g->stream[i]);
        if (e != hipSuccess) return hip_fail("hipStreamSynchronize", e);
    }
    // the image leaves device 0 behind its reduce on the same stream: one DMA into pinned staging,
    // then a parallel host copy into the caller's buffer (pt_render's path)
    hipError_t e = hipSetDevice(g->dev[0]);
    if (e != hipSuccess) return hip_fail("hipSetDevice", e);
    if (int rc0 = pt::copy_to_host(out_rgb, g->result, bytes, g->stream[0], &g->pinned, &g->pinned_bytes)) return rc0;
    if (stats) {
        pt_stats sum;
        memset(&sum, 0, sizeof(sum));
        for (int i = 0; i < n; ++i) add_stats(&sum, st[i]);
        // wall time of the whole job (concurrent shard renders + the reduce + the D2H copy)
        sum.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        *stats = sum;
    }
    return PT_OK;
}

int pt_render_multi(pt_ctx* const* ctxs, int n, const pt_params* params, const pt_camera* cam, float* out_rgb,
                    pt_stats* stats)
{
    int err = PT_OK;
    pt_group* g = pt_group_create(ctxs, n, &err);
    if (!g) return err;
    const int rc = pt_render_group(g, params, cam, out_rgb, stats);
    std::string keep = rc != PT_OK ? std::string(pt_last_error()) : std::string();
    pt_group_destroy(g);
    if (rc != PT_OK) return pt::fail(rc, "%s", keep.c_str());
    return PT_OK;
}

}  // extern "C"
