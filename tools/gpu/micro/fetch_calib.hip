// FETCH_SIZE / WRITE_SIZE calibration for the path tracer's access shapes (gfx950).
//
// MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of the bytes of wide coalesced streaming reads; "other
// access widths are uncalibrated: calibrate on a known byte count in your own access pattern".  This
// probe runs kernels with a KNOWN number of distinct 128-B lines fetched from a buffer far larger
// than the 256 MiB Infinity Cache (every line is a first touch: no cache can serve it), so that
// rocprofv3 --pmc FETCH_SIZE (one pass) / WRITE_SIZE (another) per dispatch can be divided by the
// known bytes:
//   gather7 : one random 128-B line per lane, read as 7 x 16 B (a BVH4 node visit)
//   gather3 : one random line per lane, 36 B of it (a triangle record test: 2 x 16 B + 4 B)
//   stream  : lane-contiguous 16-B loads over the buffer (the guide's reference case, factor 2)
//   cells   : lane-major 16-B cells read then written (the shading record's pattern)
// Each kernel prints its known byte count; the profile pass supplies the counters.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("HIP error %s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                           \
        }                                                                       \
    } while (0)

// every lane of every launch touches distinct lines: line = permuted global index (a bijection
// on [0, nlines) for nlines a power of two: odd multiplier + xor-shift is invertible mod 2^k)
__device__ __forceinline__ uint32_t perm(uint32_t x, uint32_t mask)
{
    x = (x * 0x9E3779B1u) & mask;
    x ^= x >> 7;
    x = (x * 0x85EBCA77u) & mask;
    return x;
}

__global__ __launch_bounds__(256) void gather7(const uint4* __restrict__ buf, uint32_t mask, uint32_t* out)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    const char* base = reinterpret_cast<const char*>(buf) + (size_t)perm(g, mask) * 128;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const uint4 v = *reinterpret_cast<const uint4*>(base + 16 * k);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[g] = acc;
}

__global__ __launch_bounds__(256) void gather3(const uint4* __restrict__ buf, uint32_t mask, uint32_t* out)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    const char* base = reinterpret_cast<const char*>(buf) + (size_t)perm(g, mask) * 128;
    const uint4 a = *reinterpret_cast<const uint4*>(base);
    const uint4 b = *reinterpret_cast<const uint4*>(base + 16);
    const uint32_t c = *reinterpret_cast<const uint32_t*>(base + 32);
    out[g] = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c;
}

__global__ __launch_bounds__(256) void stream(const uint4* __restrict__ buf, size_t n16, uint32_t* out)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// 4 cells of 16 B per lane, cell-major with lane-contiguous cells (cell c of lane g at (c*n + g)*16):
// read all, write all back modified
__global__ __launch_bounds__(256) void cells(uint4* __restrict__ buf, uint32_t n)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    uint4 v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = buf[(size_t)c * n + g];
#pragma unroll
    for (int c = 0; c < 4; ++c) buf[(size_t)c * n + g] = make_uint4(v[c].y + 1u, v[c].z, v[c].w, v[c].x);
}

// The DRAM-request calibration (round 5): the same gather and cell shapes on tables that stay resident
// in a cache, so that TCC_EA0_RDREQ_DRAM / TCC_EA0_WRREQ_DRAM can be compared with TCC_EA0_RDREQ / WRREQ:
// a counter that excludes Infinity-Cache hits reads ~0 on the 32 MB table's measured launch (every line
// was brought in by the warm launch just before it); one that counts them reads like RDREQ.
template <int kTag>
__global__ __launch_bounds__(256) void gather7_res(const uint4* __restrict__ buf, uint32_t mask, uint32_t* out)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    const char* base = reinterpret_cast<const char*>(buf) + (size_t)perm(g, mask) * 128;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const uint4 v = *reinterpret_cast<const uint4*>(base + 16 * k);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[g] = acc;
}
template <int kTag>
__global__ __launch_bounds__(256) void cells_res(uint4* __restrict__ buf, uint32_t n)
{
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    uint4 v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = buf[(size_t)c * n + g];
#pragma unroll
    for (int c = 0; c < 4; ++c) buf[(size_t)c * n + g] = make_uint4(v[c].y + 1u, v[c].z, v[c].w, v[c].x);
}

int main()
{
    // 8 GiB of 128-B lines (>> 256 MiB Infinity Cache); 2^26 lines
    const uint32_t nlines = 1u << 26;
    const size_t bytes = (size_t)nlines * 128;
    uint4* buf = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 1, bytes));
    CK(hipMalloc(&out, 64u << 20));
    CK(hipDeviceSynchronize());
    const uint32_t lanes = 1u << 22;   // 4M lanes = 4M distinct lines per gather launch
    // flush: stream 8 GiB once so no earlier line is cached
    hipLaunchKernelGGL(stream, dim3(8192), dim3(256), 0, 0, buf, bytes / 16, out);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(gather7, dim3(lanes / 256), dim3(256), 0, 0, buf, nlines - 1, out);
    CK(hipDeviceSynchronize());
    printf("gather7 lines %u known_read_bytes %llu (7x16 B of each line; whole lines %llu)\n", lanes,
           (unsigned long long)lanes * 112, (unsigned long long)lanes * 128);
    hipLaunchKernelGGL(stream, dim3(8192), dim3(256), 0, 0, buf, bytes / 16, out);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(gather3, dim3(lanes / 256), dim3(256), 0, 0, buf + 1, nlines - 2, out);   // (other lines)
    CK(hipDeviceSynchronize());
    printf("gather3 lines %u known_read_bytes %llu (36 B of each line; whole lines %llu)\n", lanes,
           (unsigned long long)lanes * 36, (unsigned long long)lanes * 128);
    const size_t sbytes = (size_t)1 << 32;   // 4 GiB stream
    hipLaunchKernelGGL(stream, dim3(8192), dim3(256), 0, 0, buf + (bytes - sbytes) / 16, sbytes / 16, out);
    CK(hipDeviceSynchronize());
    printf("stream known_read_bytes %llu\n", (unsigned long long)sbytes);
    const uint32_t ncell = 1u << 24;   // 16M lanes x 64 B = 1 GiB read + 1 GiB written
    hipLaunchKernelGGL(cells, dim3(ncell / 256), dim3(256), 0, 0, buf, ncell);
    CK(hipDeviceSynchronize());
    printf("cells known_read_bytes %llu known_write_bytes %llu\n", (unsigned long long)ncell * 64,
           (unsigned long long)ncell * 64);
    // resident tables: warm launch (tag 0), then the measured launch (tag 1) on the same lines
    // 32 MB table = 2^18 lines (Infinity-Cache resident, 8x an XCD's L2); 4M lanes: each line 16 times
    hipLaunchKernelGGL(stream, dim3(8192), dim3(256), 0, 0, buf, bytes / 16, out);   // (flush)
    hipLaunchKernelGGL((gather7_res<0>), dim3(lanes / 256), dim3(256), 0, 0, buf, (1u << 18) - 1, out);
    hipLaunchKernelGGL((gather7_res<1>), dim3(lanes / 256), dim3(256), 0, 0, buf, (1u << 18) - 1, out);
    CK(hipDeviceSynchronize());
    printf("gather7_res<1> table 32 MiB (resident in the Infinity Cache after gather7_res<0>), %u lane-lines of 112 B "
           "(%llu B requested by lanes), distinct lines 2^18\n", lanes, (unsigned long long)lanes * 112);
    // 2 MB table = 2^14 lines: resident in every XCD's 4 MiB L2
    hipLaunchKernelGGL((gather7_res<2>), dim3(lanes / 256), dim3(256), 0, 0, buf, (1u << 14) - 1, out);
    hipLaunchKernelGGL((gather7_res<3>), dim3(lanes / 256), dim3(256), 0, 0, buf, (1u << 14) - 1, out);
    CK(hipDeviceSynchronize());
    printf("gather7_res<3> table 2 MiB (L2 resident after gather7_res<2>), %u lane-lines\n", lanes);
    // 32 MB of cells (2^19 lanes x 4 x 16 B) read and written twice: warm <0>, measured <1>
    const uint32_t ncr = 1u << 19;
    hipLaunchKernelGGL((cells_res<0>), dim3(ncr / 256), dim3(256), 0, 0, buf, ncr);
    hipLaunchKernelGGL((cells_res<1>), dim3(ncr / 256), dim3(256), 0, 0, buf, ncr);
    CK(hipDeviceSynchronize());
    printf("cells_res<1> 32 MiB read + 32 MiB written (resident after cells_res<0>) known_read_bytes %llu known_write_bytes %llu\n",
           (unsigned long long)ncr * 64, (unsigned long long)ncr * 64);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
