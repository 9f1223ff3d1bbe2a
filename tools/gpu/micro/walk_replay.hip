// VALU issue time of the wavefront kernel's own instruction streams, replayed with no memory, SALU or
// branches at 1-5 waves per SIMD: one walk wave-step of render_unidir_wf<false,5,false> (walk_step.inc,
// its common path), and three shading sections of a PT_SEC_MARKERS build (sec_*.inc: the sampling block,
// the sample end, the trace begin with its root-first LDS visits; their static code, once).
// Generated includes: gen_walk_replay.py.  Priced against the kernel's cycles in DESIGN.md 6.3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "walk_step.inc"
#include "sec_COSINE.inc"
#include "sec_SAMPLE_END.inc"
#include "sec_BEGIN.inc"

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s\n", #x); return 1; } } while (0)

#define REPLAY_KERNEL(NAME, P)                                                       \
    __global__ __launch_bounds__(256) void NAME(int iters, uint32_t* sink)           \
    {                                                                                \
        for (int i = 0; i < iters; ++i) asm volatile(P##_ASM ::: P##_CLOBBERS);      \
        sink[blockIdx.x * 256 + threadIdx.x] = iters;                                \
    }
REPLAY_KERNEL(replay_walk, WALK_STEP)
REPLAY_KERNEL(replay_cosine, SEC_COSINE)
REPLAY_KERNEL(replay_sample_end, SEC_SAMPLE_END)
REPLAY_KERNEL(replay_begin, SEC_BEGIN)

static int run(const char* name, void (*k)(int, uint32_t*), int valu, int iters, int cus, uint32_t* sink,
               hipEvent_t e0, hipEvent_t e1)
{
    for (int wps = 1; wps <= 5; ++wps) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k, dim3(cus * wps), dim3(256), 0, 0, iters, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0 && ms < best) best = ms;
        }
        const double cyc = best * 1e-3 * 2.4e9 / ((double)wps * iters);
        printf("%-11s VALU %4d  waves/SIMD %d  %7.3f ms  %8.1f SIMD-cycles per replay @2.4 GHz  %5.2f per VALU\n", name,
               valu, wps, best, cyc, cyc / valu);
    }
    return 0;
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* sink;
    CK(hipMalloc(&sink, (size_t)cus * 8 * 256 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("CUs %d\n", cus);
    if (run("walk_step", replay_walk, WALK_STEP_VALU, 2000, cus, sink, e0, e1)) return 1;
    if (run("cosine", replay_cosine, SEC_COSINE_VALU, 800, cus, sink, e0, e1)) return 1;
    if (run("sample_end", replay_sample_end, SEC_SAMPLE_END_VALU, 1600, cus, sink, e0, e1)) return 1;
    if (run("begin", replay_begin, SEC_BEGIN_VALU, 400, cus, sink, e0, e1)) return 1;
    return 0;
}
