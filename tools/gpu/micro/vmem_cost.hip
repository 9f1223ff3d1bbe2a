// Vector-memory cost model probe (gfx950): CU-cycles per wave-level load instruction for the access
// shapes of the path tracer (scattered 16-B node chunks, coalesced record words, partial exec), with
// an L1-resident footprint (pipeline cost) and an L2-resident one.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s\n", #x); return 1; } } while (0)
constexpr int kIters = 256, kLoads = 8;

__device__ __forceinline__ uint32_t hash(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// kShape: 0 scattered (a random line per lane, chunk k of it: a node's 7 loads), 1 eight lanes per
// line, 2 wave-coalesced (lane-contiguous).  kW: bytes per lane (4, 8, 16).  kAct: active lanes.
template <int kShape, int kW, int kAct>
__global__ __launch_bounds__(256) void probe(const uint4* __restrict__ buf, uint32_t nlines, uint32_t* out)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    uint32_t acc = 0, seed = hash(g * 7919u + 1u);
    if (lane % (64 / kAct) != 0) { out[g] = 0; return; }
    for (int it = 0; it < kIters; ++it) {
        seed = hash(seed + it);
        const uint32_t wseed = hash((g >> 6) * 131u + it);
        uint32_t line;
        if (kShape == 0) line = seed % nlines;
        else if (kShape == 1) line = hash((g >> 3) * 131u + it) % nlines;
        else line = (wseed % (nlines / 8)) * 8;
        const char* base = reinterpret_cast<const char*>(buf) + (size_t)line * 128;
#pragma unroll
        for (int k = 0; k < kLoads; ++k) {
            uint32_t off;
            if (kShape == 0) off = (k & 7) * 16;
            else if (kShape == 1) off = ((lane + k) & 7) * 16;
            else off = (k * 64 + lane) * kW;    // instruction k: the next 64*kW bytes
            if (kShape == 2) off %= 1024;        // stay inside the 8 lines
            if (kW == 4) acc ^= *reinterpret_cast<const uint32_t*>(base + off);
            else if (kW == 8) { const uint2 v = *reinterpret_cast<const uint2*>(base + off); acc ^= v.x ^ v.y; }
            else { const uint4 v = *reinterpret_cast<const uint4*>(base + off); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
        }
    }
    out[g] = acc;
}

template <int S, int W, int A>
static int run(const char* name, const uint4* buf, uint32_t nlines, uint32_t* out, int cus, hipEvent_t e0, hipEvent_t e1)
{
    const uint32_t blocks = cus * 5;   // 20 waves per CU
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((probe<S, W, A>), dim3(blocks), dim3(256), 0, 0, buf, nlines, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
    }
    const double instr_per_cu = (double)blocks * 4 * kIters * kLoads / cus;
    printf("%-34s lines=%-8u %8.3f ms %7.2f CU-cycles/instr\n", name, nlines, best, best * 1e-3 * 2.4e9 / instr_per_cu);
    return 0;
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t bytes = 64u << 20;
    uint4* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 1, bytes));
    CK(hipMalloc(&out, (size_t)cus * 5 * 256 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (uint32_t nl : {64u, 131072u}) {   // 8 KiB (L1-resident) / 16 MiB (L2/MALL)
        run<0, 16, 64>("scatter x4 64 lanes", buf, nl, out, cus, e0, e1);
        run<0, 16, 32>("scatter x4 32 lanes", buf, nl, out, cus, e0, e1);
        run<0, 16, 16>("scatter x4 16 lanes", buf, nl, out, cus, e0, e1);
        run<0, 8, 64>("scatter x2 64 lanes", buf, nl, out, cus, e0, e1);
        run<0, 4, 64>("scatter x1 64 lanes", buf, nl, out, cus, e0, e1);
        run<1, 16, 64>("x4 8 lanes per line", buf, nl, out, cus, e0, e1);
        run<2, 16, 64>("coalesced x4 (1 KiB)", buf, nl, out, cus, e0, e1);
        run<2, 8, 64>("coalesced x2 (512 B)", buf, nl, out, cus, e0, e1);
        run<2, 4, 64>("coalesced x1 (256 B)", buf, nl, out, cus, e0, e1);
    }
    return 0;
}
