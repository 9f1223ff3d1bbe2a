// VALU issue-cost probe (gfx950): SIMD-cycles per wave64 vector instruction for the instruction classes the
// wavefront kernel's walk and shading use, at 1, 2, 4 and 8 waves per SIMD (independent chains, no memory).
// Cycles come from the shader clock read at the start and end of each wave; the event time cross-checks it.
// Used to price SQ_INSTS_VALU_* of the C3 launch (tools/valu_bound.py).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s\n", #x); return 1; } } while (0)
constexpr int kIters = 8192;   // ~0.3-3 ms per launch: dispatch amortised

enum Op { ADD_U32, FMA_F32, PK_FMA_F32, MIN3_F32, CNDMASK, CMP_F32, FMA_F64, ADD_F64, MUL_F64, MAD_U64_U32,
          LSHL_ADD_U64, RCP_F32, RCP_F64, CVT_F64_F32, AND_OR_B32, MUL_LO_U32, MOV_B32, MAX_U32, PK_MUL_F32, BITOP3,
          CNDMASK_SREG, CNDMASK_VCC_E64, CMP_CNDMASK, ADDC_VCC, CMP_SREG_CNDMASK, kNumOps };
static const char* kNames[kNumOps] = {"v_add_u32", "v_fma_f32", "v_pk_fma_f32", "v_min3_f32", "v_cndmask_b32",
                                      "v_cmp_lt_f32 (vcc)", "v_fma_f64", "v_add_f64", "v_mul_f64", "v_mad_u64_u32",
                                      "v_lshl_add_u64", "v_rcp_f32", "v_rcp_f64", "v_cvt_f64_f32", "v_and_or_b32",
                                      "v_mul_lo_u32", "v_mov_b32", "v_max_u32", "v_pk_mul_f32", "v_bitop3_b32",
                                      "v_cndmask_b32 (s[])", "v_cndmask_b32_e64 vcc", "v_cmp vcc + cndmask", "v_addc_co_u32 vcc",
                                      "v_cmp s[] + cndmask"};

// one instruction on chain register r (32-bit chains x, 64-bit chains d)
#define STEP32(ASM, r) asm volatile(ASM : "+v"(r) : "v"(k1), "v"(k2))
#define STEP64(ASM, r) asm volatile(ASM : "+v"(r) : "v"(q1), "v"(q2))

template <int kOp>
__device__ __forceinline__ void body(uint32_t (&x)[8], uint64_t (&d)[8], uint32_t k1, uint32_t k2, uint64_t q1, uint64_t q2, uint64_t sm)
{
#pragma unroll
    for (int rep = 0; rep < 2; ++rep)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (kOp == ADD_U32) STEP32("v_add_u32 %0, %0, %1", x[i]);
            else if constexpr (kOp == FMA_F32) STEP32("v_fma_f32 %0, %0, %1, %2", x[i]);
            else if constexpr (kOp == PK_FMA_F32) STEP64("v_pk_fma_f32 %0, %0, %1, %2", d[i]);
            else if constexpr (kOp == MIN3_F32) STEP32("v_min3_f32 %0, %0, %1, %2", x[i]);
            else if constexpr (kOp == CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(k1));
            else if constexpr (kOp == CMP_F32) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(x[i]), "v"(k1) : "vcc");
            else if constexpr (kOp == FMA_F64) STEP64("v_fma_f64 %0, %0, %1, %2", d[i]);
            else if constexpr (kOp == ADD_F64) STEP64("v_add_f64 %0, %0, %1", d[i]);
            else if constexpr (kOp == MUL_F64) STEP64("v_mul_f64 %0, %0, %1", d[i]);
            else if constexpr (kOp == MAD_U64_U32)
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(d[i]) : "v"(k1), "v"(k2) : "vcc");
            else if constexpr (kOp == LSHL_ADD_U64) STEP64("v_lshl_add_u64 %0, %0, 2, %1", d[i]);
            else if constexpr (kOp == RCP_F32) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i]));
            else if constexpr (kOp == RCP_F64) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[i]));
            else if constexpr (kOp == CVT_F64_F32) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[i]) : "v"(x[i]));
            else if constexpr (kOp == AND_OR_B32) STEP32("v_and_or_b32 %0, %0, %1, %2", x[i]);
            else if constexpr (kOp == MUL_LO_U32) STEP32("v_mul_lo_u32 %0, %0, %1", x[i]);
            else if constexpr (kOp == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 1) & 7]));
            else if constexpr (kOp == MAX_U32) STEP32("v_max_u32 %0, %0, %1", x[i]);
            else if constexpr (kOp == PK_MUL_F32) STEP64("v_pk_mul_f32 %0, %0, %1", d[i]);
            else if constexpr (kOp == BITOP3) STEP32("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x36", x[i]);
            else if constexpr (kOp == CNDMASK_VCC_E64) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(k1));
            else if constexpr (kOp == CMP_CNDMASK)   // two instructions: the pair the compiler emits for a select
                asm volatile("v_cmp_lt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(k1) : "vcc");
            else if constexpr (kOp == ADDC_VCC) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(x[i]) : "v"(k1) : "vcc");
            else if constexpr (kOp == CMP_SREG_CNDMASK) {
                uint64_t m;
                asm volatile("v_cmp_lt_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1" : "+v"(x[i]), "=s"(m) : "v"(k1));
            }
            else if constexpr (kOp == CNDMASK_SREG) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[i]) : "v"(k1), "s"(sm));
        }
}

template <int kOp>
__global__ __launch_bounds__(256) void probe(uint32_t seed, uint64_t* cyc, uint32_t* sink)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    uint32_t x[8];
    uint64_t d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = 0x3f800000u ^ (g * 2654435761u + i + seed) & 0x7fffu;
        d[i] = 0x3ff0000000000000ull ^ ((uint64_t)(g + i) << 8);
    }
    const uint32_t k1 = 0x3f7ff000u ^ (seed & 1u), k2 = 0x3a000000u;
    const uint64_t q1 = 0x3fefff0000000000ull + seed, q2 = 0x3e00000000000000ull;
    const uint64_t sm = __builtin_amdgcn_read_exec() & (0x5555555555555555ull ^ seed);   // a lane mask in an SGPR pair
    if constexpr (kOp == CNDMASK || kOp == CNDMASK_VCC_E64 || kOp == ADDC_VCC) asm volatile("v_cmp_lt_u32 vcc, %0, %1" : : "v"(x[0]), "v"(k1) : "vcc");
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) body<kOp>(x, d, k1, k2, q1, q2, sm);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= x[i] ^ (uint32_t)d[i] ^ (uint32_t)(d[i] >> 32);
    sink[g] = acc;
    if ((threadIdx.x & 63) == 0) cyc[g >> 6] = t1 - t0;
}

template <int kOp>
static int run(int cus, int wps, uint64_t* cyc, uint64_t* hcyc, uint32_t* sink, hipEvent_t e0, hipEvent_t e1)
{
    const uint32_t blocks = cus * wps;   // 4 waves per block: one per SIMD of a CU
    const uint32_t waves = blocks * 4;
    float best = 1e30f;
    double cyc_avg = 0;
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((probe<kOp>), dim3(blocks), dim3(256), 0, 0, (uint32_t)rep, cyc, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) {
            best = ms;
            CK(hipMemcpy(hcyc, cyc, waves * sizeof(uint64_t), hipMemcpyDeviceToHost));
            double s = 0;
            for (uint32_t w = 0; w < waves; ++w) s += (double)hcyc[w];
            cyc_avg = s / waves;
        }
    }
    const double per_wave = (double)kIters * 16;
    // wps waves share one SIMD: SIMD-cycles per instruction = wave elapsed / (wps * instructions per wave)
    printf("%-20s waves/SIMD %d  %7.3f ms  %6.2f SIMD-cycles/instr (clock)  %6.2f (event @2.4 GHz)\n", kNames[kOp],
           wps, best, cyc_avg / (wps * per_wave), best * 1e-3 * 2.4e9 / (wps * per_wave));
    return 0;
}

template <int kOp>
static int sweep(int cus, uint64_t* cyc, uint64_t* hcyc, uint32_t* sink, hipEvent_t e0, hipEvent_t e1)
{
    for (int wps : {1, 2, 4, 8})
        if (run<kOp>(cus, wps, cyc, hcyc, sink, e0, e1)) return 1;
    if constexpr (kOp + 1 < kNumOps) return sweep<kOp + 1>(cus, cyc, hcyc, sink, e0, e1);
    return 0;
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t waves = (size_t)cus * 8 * 4;
    uint64_t *cyc, *hcyc = new uint64_t[waves];
    uint32_t* sink;
    CK(hipMalloc(&cyc, waves * sizeof(uint64_t)));
    CK(hipMalloc(&sink, waves * 64 * sizeof(uint32_t)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("CUs %d, %d iterations x 16 instructions per wave\n", cus, kIters);
    const int rc = sweep<0>(cus, cyc, hcyc, sink, e0, e1);   // the pair ops count 16 pairs per iteration
    delete[] hcyc;
    return rc;
}
