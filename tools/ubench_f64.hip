// Issue cost of the double-precision FMA on gfx950 next to v_mad_u64_u32, by waves per SIMD: does a
// floating-point limb product (Emmart-Weems style: 50-bit limbs, hi/lo by two FMAs) issue faster per
// product bit than the 32x32->64 integer mad the MSM arithmetic uses today? Same method as
// tools/ubench_issue.hip: each thread runs CH independent chains of one instruction (inline asm),
// IT iterations unrolled by 8, W waves on every SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                          \
    do {                                                                \
        hipError_t e = (x);                                             \
        if (e != hipSuccess) {                                          \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                    \
        }                                                               \
    } while (0)

template <int OP>
__device__ __forceinline__ void step(double& a, double x, double y, uint64_t& m, uint32_t u, uint32_t v) {
    if constexpr (OP == 0) {
        asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y));
    } else if constexpr (OP == 1) {
        asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(x));
    } else if constexpr (OP == 2) {
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(x));
    } else {
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(m) : "v"(u), "v"(v) : "vcc");
    }
}

template <int OP, int W, int CH>
__global__ __launch_bounds__(256, W) void k_issue(double* out, uint64_t* out2, double seed, int iters) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    double a[CH];
    uint64_t m[CH];
    const double x = 1.0 + seed * 1e-9, y = 1.0 - seed * 1e-9;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        a[c] = t + c;
        m[c] = t + c;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) step<OP>(a[c], x, y, m[c], t, t ^ 0x55u);
    }
    double s = 0;
    uint64_t s2 = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        s += a[c];
        s2 ^= m[c];
    }
    out[t] = s;
    out2[t] = s2;
}

template <int OP, int W, int CH = 8>
static void run(const char* name, double* buf, uint64_t* buf2) {
    const int blocks = 256 * W;  // 256 threads = 4 waves (one per SIMD) per block
    const int iters = 2048;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_issue<OP, W, CH>), dim3(blocks), dim3(256), 0, 0, buf, buf2, 1.0, iters);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_issue<OP, W, CH>), dim3(blocks), dim3(256), 0, 0, buf, buf2, 2.0, iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double winst = (double)blocks * 4 * iters * 8 * CH;
    const double cyc = ms * 1e-3 * 2.4e9 * 1024.0 / winst;
    printf("%-14s x%2d chains waves/SIMD %d: %.3f ms, %.2f cycles per wave-instruction per SIMD (%.1f G wave-inst/s)\n",
           name, CH, W, ms, cyc, winst / (ms * 1e-3) / 1e9);
}

int main() {
    double* buf;
    uint64_t* buf2;
    CHK(hipMalloc(&buf, sizeof(double) * 256 * 256 * 8 + 64));
    CHK(hipMalloc(&buf2, sizeof(uint64_t) * 256 * 256 * 8 + 64));
    run<0, 1>("v_fma_f64", buf, buf2);
    run<0, 2>("v_fma_f64", buf, buf2);
    run<0, 4>("v_fma_f64", buf, buf2);
    run<1, 2>("v_mul_f64", buf, buf2);
    run<2, 2>("v_add_f64", buf, buf2);
    run<3, 1>("v_mad_u64_u32", buf, buf2);
    run<3, 2>("v_mad_u64_u32", buf, buf2);
    run<0, 2, 1>("v_fma_f64", buf, buf2);  // one dependent chain: latency
    CHK(hipFree(buf));
    CHK(hipFree(buf2));
    return 0;
}
