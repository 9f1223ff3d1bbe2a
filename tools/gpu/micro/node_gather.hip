// Node-fetch probe (gfx950): dependent gathers of 128-B BVH4-node records, as the walk step does them, in
// two forms --
//   lane:  every lane loads its own node with 7 global_load_dwordx4 (the render kernel's form: one L1 tag
//          lookup per lane per instruction, seven per node);
//   coop:  the wave's nodes are fetched cooperatively into LDS -- global_load_lds_dwordx4 where 8 lanes read
//          the 8 16-B chunks of one node (one lookup per node) -- and each lane then reads its node from LDS
//          with 7 ds_read_b128.
// Each lane chases a chain: the next node index comes from the node just read.  Table: TABLE_MB of nodes
// (the stand-in's BVH4 is ~10 MB).  Reports nodes per second and CU-cycles per wave-step.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kSteps = 256;

__device__ __forceinline__ uint32_t hash(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// active: lanes (lane % 64 < kAct) walk; the others issue nothing (lane form: exec-masked)
template <int kAct>
__global__ __launch_bounds__(256) void lane_form(const uint4* __restrict__ nodes, uint32_t nn, uint32_t* out)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    uint32_t idx = hash(g * 2654435761u + 7u) % nn, acc = 0;
    if ((int)lane < kAct) {
        for (int s = 0; s < kSteps; ++s) {
            const uint4* p = nodes + (size_t)idx * 8;
            uint4 v[7];
#pragma unroll
            for (int k = 0; k < 7; ++k) v[k] = p[k];
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 7; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
            acc += x;
            idx = (v[6].x ^ (lane * 0x9e3779b9u) ^ (uint32_t)s) % nn;   // dependent: from the node
        }
    }
    out[g] = acc;
}

// Cooperative form.  LDS per wave: 64 slots x 128 B staging + 64 slot words.
template <int kAct>
__global__ __launch_bounds__(256) void coop_form(const uint4* __restrict__ nodes, uint32_t nn, uint32_t* out)
{
    extern __shared__ uint4 lds[];
    const uint32_t g = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint4* stage = lds + wave * (64 * 8 + 16);              // 8 KiB staging
    uint32_t* slots = reinterpret_cast<uint32_t*>(stage + 64 * 8);   // 64 words, transposed
    uint32_t idx = hash(g * 2654435761u + 7u) % nn, acc = 0;
    const bool act = (int)lane < kAct;
    for (int s = 0; s < kSteps; ++s) {
        const uint64_t m = __ballot(act);
        const uint32_t nact = (uint32_t)__popcll(m);
        const uint32_t slot = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        // slot s's index at word (s % 8) * 8 + s / 8: a fetching lane j reads its 8 instructions' indices
        // (slots 8i + j/8, i = 0..7) as the 8 consecutive words (j/8) * 8 + i
        if (act) slots[(slot & 7u) * 8u + (slot >> 3)] = idx;
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        const uint32_t* row = slots + (lane >> 3) * 8;
        const uint4 i0 = *reinterpret_cast<const uint4*>(row), i1 = *reinterpret_cast<const uint4*>(row + 4);
        const uint32_t ids[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
        const uint32_t ninst = (nact + 7u) / 8u;
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            if (i < ninst) {   // (wave-uniform)
                const uint4* src = nodes + (size_t)ids[i] * 8 + (lane & 7u);
                __builtin_amdgcn_global_load_lds(src, stage + i * 64, 16, 0, 0);
            }
        }
        __builtin_amdgcn_s_waitcnt(0x0070 | 0xc00f);   // vmcnt(0) (expcnt/lgkm don't care)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t x = 0;
        uint4 v6 = make_uint4(0, 0, 0, 0);
        if (act) {
            const uint4* p = stage + slot * 8;
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                const uint4 v = p[k];
                x ^= v.x ^ v.y ^ v.z ^ v.w;
                if (k == 6) v6 = v;
            }
            acc += x;
            idx = (v6.x ^ (lane * 0x9e3779b9u) ^ (uint32_t)s) % nn;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next step's DMA overwrites
    }
    out[g] = acc;
}


// lane form with 64-B nodes (4 loads per visit): the lookup count halves
template <int kAct>
__global__ __launch_bounds__(256) void lane4_form(const uint4* __restrict__ nodes, uint32_t nn, uint32_t* out)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    uint32_t idx = hash(g * 2654435761u + 7u) % nn, acc = 0;
    if ((int)lane < kAct) {
        for (int s = 0; s < kSteps; ++s) {
            const uint4* p = nodes + (size_t)idx * 8;
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = p[k];
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
            acc += x;
            idx = (v[3].x ^ (lane * 0x9e3779b9u) ^ (uint32_t)s) % nn;
        }
    }
    out[g] = acc;
}


// lane form with buffer loads issued by EVERY lane, the inactive ones at an out-of-range offset (the render
// kernel's uniform walk-step loads): do out-of-range lanes cost address-path cycles?
template <int kAct>
__global__ __launch_bounds__(256) void lane_oor_form(const uint4* __restrict__ nodes, uint32_t nn, uint32_t* out)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    uint32_t idx = hash(g * 2654435761u + 7u) % nn, acc = 0;
    const bool act = (int)lane < kAct;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(nodes), 0, 0x7fffff00, 0x00020000);
    for (int s = 0; s < kSteps; ++s) {
        const uint32_t nb = act ? idx * 128u : 0x80000000u;
        uint4 v[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            const u4 w = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, nb + 16u * k, 0, 0));
            v[k] = make_uint4(w.x, w.y, w.z, w.w);
        }
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 7; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        acc += x;
        if (act) idx = (v[6].x ^ (lane * 0x9e3779b9u) ^ (uint32_t)s) % nn;
    }
    out[g] = acc;
}

// Per-instruction cost probe (round 5): 7 loads per step of width W bytes (4: dword, 16: dwordx4), kAct lanes
// active; kMask: the others exec-masked (true) or at an out-of-range buffer offset (false).  If the cost per
// wave-step stays ~constant as kAct falls to 1, the memory pipe charges per wave-instruction (not per lane).
template <int kAct, int kW, bool kMask>
__global__ __launch_bounds__(256) void width_form(const uint4* __restrict__ nodes, uint32_t nn, uint32_t* out)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    uint32_t idx = hash(g * 2654435761u + 7u) % nn, acc = 0;
    const bool act = (int)lane < kAct;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(nodes), 0, 0x7fffff00, 0x00020000);
    if (kMask && !act) { out[g] = 0; return; }
    for (int s = 0; s < kSteps; ++s) {
        const uint32_t nb = act ? idx * 128u : 0x80000000u;
        uint32_t x = 0, last = 0;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            if (kW == 16) {
                const u4 w = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, nb + 16u * k, 0, 0));
                x ^= w.x ^ w.y ^ w.z ^ w.w;
                last = w.x;
            } else {
                const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(rs, nb + 16u * k, 0, 0);
                x ^= w;
                last = w;
            }
        }
        acc += x;
        if (act) idx = (last ^ (lane * 0x9e3779b9u) ^ (uint32_t)s) % nn;
    }
    out[g] = acc;
}

template <class K>
static double timeit(K kern, dim3 grid, size_t lds, const uint4* nodes, uint32_t nn, uint32_t* out)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, grid, dim3(256), lds, 0, nodes, nn, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv)
{
    const double mb = argc > 1 ? atof(argv[1]) : 10.0;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t nn = (uint32_t)(mb * 1048576.0 / 128.0);
    std::vector<uint32_t> h((size_t)nn * 32);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;
    uint4* nodes; uint32_t* out;
    CK(hipMalloc(&nodes, h.size() * 4));
    CK(hipMemcpy(nodes, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    const size_t coop_lds = 4 * (64 * 8 + 16) * 16;   // per 256-thread block
    printf("table %.1f MB (%u nodes), %d CUs, %d dependent steps per lane\n", mb, nn, cus, kSteps);
    for (int bpc : {4, 5}) {
        const dim3 grid(cus * bpc);
        struct R { const char* name; double ms; int act; };
        std::vector<R> rs;
        rs.push_back({"lane 64 active", timeit(lane_form<64>, grid, 0, nodes, nn, out), 64});
        rs.push_back({"lane 40 active", timeit(lane_form<40>, grid, 0, nodes, nn, out), 40});
        rs.push_back({"lane4 40 active", timeit(lane4_form<40>, grid, 0, nodes, nn, out), 40});
        rs.push_back({"lane_oor 40 active", timeit(lane_oor_form<40>, grid, 0, nodes, nn, out), 40});
        rs.push_back({"lane_oor 20 active", timeit(lane_oor_form<20>, grid, 0, nodes, nn, out), 20});
        rs.push_back({"lane 20 active", timeit(lane_form<20>, grid, 0, nodes, nn, out), 20});
        rs.push_back({"lane_oor 64 active", timeit(lane_oor_form<64>, grid, 0, nodes, nn, out), 64});
        rs.push_back({"w16 oor 1 active", timeit(width_form<1, 16, false>, grid, 0, nodes, nn, out), 1});
        rs.push_back({"w16 exec 1 active", timeit(width_form<1, 16, true>, grid, 0, nodes, nn, out), 1});
        rs.push_back({"w16 oor 8 active", timeit(width_form<8, 16, false>, grid, 0, nodes, nn, out), 8});
        rs.push_back({"w16 oor 40 active", timeit(width_form<40, 16, false>, grid, 0, nodes, nn, out), 40});
        rs.push_back({"w4 oor 1 active", timeit(width_form<1, 4, false>, grid, 0, nodes, nn, out), 1});
        rs.push_back({"w4 oor 40 active", timeit(width_form<40, 4, false>, grid, 0, nodes, nn, out), 40});
        rs.push_back({"w4 oor 64 active", timeit(width_form<64, 4, false>, grid, 0, nodes, nn, out), 64});
        if (bpc == 4) {   // (32 KiB of staging per block: 4 blocks per CU)
            rs.push_back({"coop 64 active", timeit(coop_form<64>, grid, coop_lds, nodes, nn, out), 64});
            rs.push_back({"coop 40 active", timeit(coop_form<40>, grid, coop_lds, nodes, nn, out), 40});
        }
        for (auto& r : rs) {
            const double visits = (double)grid.x * 4 * r.act * kSteps;
            const double wave_steps_per_cu = (double)grid.x * 4 * kSteps / cus;
            printf("%d waves/CU  %-16s %8.3f ms  %8.1f Gnodes/s  %7.1f CU-cycles per wave-step\n", bpc * 4, r.name, r.ms,
                   visits / (r.ms * 1e-3) / 1e9, r.ms * 1e-3 * 2.4e9 / wave_steps_per_cu);
        }
    }
    return 0;
}
