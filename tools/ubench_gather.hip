// Gather granularity microbenchmark: random rows read the way the MSM
// accumulation reads its window tables, at the row pitch it uses and at the next power of two.
//   g2: a 192-B G2 affine point read by a lane PAIR, each lane its half (48 B of x and 48 B of y at
//       offsets 48 l and 96 + 48 l: the c0 / c1 split of fq2pair.hpp), pitch 192 or 256
//   g1: a 96-B G1 affine point read by one lane (6 x 16 B), pitch 96 or 128 (the table's G1Slot)
// plus a 1 GiB contiguous streaming read (16 B per lane) to calibrate FETCH_SIZE's byte scale.
// Table: 2^24 rows (past the 256 MiB Infinity Cache); 2^22 random rows per launch.
// Timing by HIP events here; bytes per row from a rocprofv3 --pmc FETCH_SIZE pass over the same binary
// (tools/gather_granularity.sh). Usage: ubench_gather  -> one line per variant.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ void fold(uint4& a, const uint4& v) {
    a.x ^= v.x, a.y ^= v.y, a.z ^= v.z, a.w ^= v.w;
}

template <int PITCH>
__global__ __launch_bounds__(256) void k_gather_g2(const uint8_t* __restrict__ tab, uint32_t ntab, uint32_t nrows,
                                                   uint32_t seed, uint32_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, e = t >> 1, l = t & 1;
    if (e >= nrows) return;
    const uint8_t* row = tab + (size_t)(hash32(e ^ seed) % ntab) * PITCH;
    const uint4* x = (const uint4*)(row + 48 * l);
    const uint4* y = (const uint4*)(row + 96 + 48 * l);
    uint4 a = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 3; ++k) fold(a, x[k]), fold(a, y[k]);
    if ((a.x ^ a.y ^ a.z ^ a.w) == 0x9E3779B9u) out[t] = 1;  // keeps the loads; never true for the fill
}
template <int PITCH>
__global__ __launch_bounds__(256) void k_gather_g1(const uint8_t* __restrict__ tab, uint32_t ntab, uint32_t nrows,
                                                   uint32_t seed, uint32_t* __restrict__ out) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nrows) return;
    const uint4* p = (const uint4*)(tab + (size_t)(hash32(e ^ seed) % ntab) * PITCH);
    uint4 a = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 6; ++k) fold(a, p[k]);
    if ((a.x ^ a.y ^ a.z ^ a.w) == 0x9E3779B9u) out[e] = 1;
}
__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ a, size_t n, uint32_t* __restrict__ out) {
    uint4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) fold(acc, a[i]);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[threadIdx.x] = 1;
}

int main() {
    const uint32_t ntab = 1u << 24, nrows = 1u << 22;
    const size_t tab_bytes = (size_t)ntab * 256;  // the largest pitch
    uint8_t* tab;
    uint32_t* out;
    CK(hipMalloc(&tab, tab_bytes));
    CK(hipMalloc(&out, 4 * (size_t)2 * nrows));
    CK(hipMemset(tab, 0x5A, tab_bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, int pitch, int rowb, auto launch) {
        launch(1u);  // warm-up (page tables)
        CK(hipEventRecord(a));
        const int reps = 5;
        for (int r = 0; r < reps; ++r) launch(100u + r);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / reps;
        printf("%-10s pitch %3d row %3d B: %8.1f us per launch of %u rows, %6.2f G rows/s, %7.1f GB/s of row bytes\n", name,
               pitch, rowb, us, nrows, nrows / us / 1e3, (double)nrows * rowb / us / 1e3);
    };
    const unsigned g2b = (2 * nrows + 255) / 256, g1b = (nrows + 255) / 256;
    timeit("g2", 192, 192, [&](uint32_t s) { hipLaunchKernelGGL(k_gather_g2<192>, dim3(g2b), dim3(256), 0, 0, tab, ntab, nrows, s, out); });
    timeit("g2", 256, 192, [&](uint32_t s) { hipLaunchKernelGGL(k_gather_g2<256>, dim3(g2b), dim3(256), 0, 0, tab, ntab, nrows, s, out); });
    timeit("g1", 96, 96, [&](uint32_t s) { hipLaunchKernelGGL(k_gather_g1<96>, dim3(g1b), dim3(256), 0, 0, tab, ntab, nrows, s, out); });
    timeit("g1", 128, 96, [&](uint32_t s) { hipLaunchKernelGGL(k_gather_g1<128>, dim3(g1b), dim3(256), 0, 0, tab, ntab, nrows, s, out); });
    const size_t n16 = (1ull << 30) / 16;
    timeit("stream", 16, 16, [&](uint32_t) { hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)tab, n16, out); });
    printf("(stream line: 'rows' = 2^22 for the format; it reads 1 GiB = 2^26 x 16 B per launch)\n");
    CK(hipDeviceSynchronize());
    CK(hipFree(tab));
    CK(hipFree(out));
    return 0;
}
