// Exhaustive check, on the GPU, that the refined hardware reciprocal
//     y0 = v_rcp_f32(a); e = fma(-a, y0, 1); y = fma(e, y0, y0)
// equals the correctly rounded 1/a (IEEE '/') for every float a with T <= |a| <= 2^64,
// T = 0x1.4f8b5ap-17 (the smallest float whose double is >= 1e-5: the triangle test's
// "|a| < 0.00001" cut-off).  The walk's Markstein quotients need y = RN(1/a) exactly.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/gpu/rcp_check.hip -o rcp_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__global__ void check(uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* first)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    for (int s = 0; s < 2; ++s) {
        const uint32_t bits = (lo + k) | (s ? 0x80000000u : 0u);
        const float a = __uint_as_float(bits);
        const float y0 = __builtin_amdgcn_rcpf(a);
        const float e = __builtin_fmaf(-a, y0, 1.0f);
        const float y = __builtin_fmaf(e, y0, y0);
        const float r = 1.0f / a;
        if (__float_as_uint(y) != __float_as_uint(r)) {
            if (atomicAdd(bad, 1ull) < 8ull) atomicExch(first + (atomicAdd(bad + 1, 1ull) & 7), bits);
        }
    }
}

int main(int argc, char** argv)
{
    // default: [T, 2^64]; `rcp_check LO HI` (hex float bits) checks another range
    uint32_t lo = 0x3727c5adu;   // T = 0x1.4f8b5ap-17
    uint32_t hi = 0x5f800000u;   // 2^64
    if (argc == 3) { lo = (uint32_t)strtoul(argv[1], nullptr, 16); hi = (uint32_t)strtoul(argv[2], nullptr, 16); }
    const uint32_t n = hi - lo + 1u;
    unsigned long long* bad;
    uint32_t* first;
    if (hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&first, 32) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 16);
    (void)hipMemset(first, 0, 32);
    hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, lo, n, bad, first);
    unsigned long long hb[2];
    uint32_t hf[8];
    if (hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost) != hipSuccess) { printf("hip error\n"); return 2; }
    (void)hipMemcpy(hf, first, 32, hipMemcpyDeviceToHost);
    printf("checked %llu floats (both signs) in [0x%08x, 0x%08x]: %llu mismatches\n",
           2ull * n, lo, hi, hb[0]);
    for (int i = 0; i < 8 && i < (int)hb[0]; ++i) printf("  a bits 0x%08x\n", hf[i]);
    return hb[0] ? 1 : 0;
}
