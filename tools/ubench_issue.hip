// VALU issue cost of the instructions the MSM field arithmetic is made of, on gfx950, by waves per SIMD.
// Each thread runs CH independent dependency chains of one instruction (inline asm, so the exact
// instruction is issued), IT iterations unrolled by 8. The grid puts W waves on every SIMD
// (256 CUs x 4 SIMDs x W waves of 64 lanes). cycles per wave-instruction per SIMD =
// elapsed x f_clk x 1024 SIMDs / wave-instructions, with f_clk measured from s_memtime/realtime.
// Used to price the VALU roofline of the MSM kernels: a G2 mixed addition is ~11 K
// v_mad_u64_u32 plus ~4 K other VALU per thread.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);             \
            exit(1);                                                                \
        }                                                                           \
    } while (0)


template <int OP>
__device__ __forceinline__ void step(uint64_t& a, uint32_t x, uint32_t y) {
    if constexpr (OP == 0) {  // v_mad_u64_u32 (carry-out to vcc)
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y) : "vcc");
    } else if constexpr (OP == 1) {  // v_add_u32
        uint32_t lo = (uint32_t)a;
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(lo) : "v"(x));
        a = (a & ~0xffffffffull) | lo;
    } else if constexpr (OP == 2) {  // v_mul_lo_u32
        uint32_t lo = (uint32_t)a;
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(lo) : "v"(x));
        a = (a & ~0xffffffffull) | lo;
    } else if constexpr (OP == 3) {  // v_add_co_u32 + v_addc_co_u32 (a 64-bit add), counted as 2
        uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                     : "+v"(lo), "+v"(hi)
                     : "v"(x), "v"(y)
                     : "vcc");
        a = ((uint64_t)hi << 32) | lo;
    } else {  // v_and_b32
        uint32_t lo = (uint32_t)a;
        asm volatile("v_and_b32 %0, %0, %1" : "+v"(lo) : "v"(x));
        a = (a & ~0xffffffffull) | lo;
    }
}

template <int OP, int W, int CH>
__global__ __launch_bounds__(256, W) void k_issue(uint64_t* out, uint32_t seed, int iters) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t a[CH];
    uint32_t x = seed ^ t, y = seed * 7 + t;
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = t + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) step<OP>(a[c], x, y);
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s ^= a[c];
    out[t] = s;
}

__global__ void k_clock(uint64_t* out, int spin) {
    uint64_t t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t a = 1;
    for (int i = 0; i < spin; ++i) a = a * 3 + 1;
    uint64_t t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = a;
    }
}

template <int OP, int W, int CH = 8>
static void run(const char* name, uint64_t* buf, double fclk) {
    const int blocks = 256 * W;  // 256 threads = 4 waves (one per SIMD) per block
    const int iters = 2048;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_issue<OP, W, CH>), dim3(blocks), dim3(256), 0, 0, buf, 1u, iters);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_issue<OP, W, CH>), dim3(blocks), dim3(256), 0, 0, buf, 2u, iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double per_inst = OP == 3 ? 2.0 : 1.0;
    const double winst = (double)blocks * 4 * iters * 8 * CH * per_inst;  // wave-instructions
    const double cyc = ms * 1e-3 * fclk * 1024.0 / winst;
    printf("%-14s x%2d chains waves/SIMD %d: %.3f ms, %.2f cycles per wave-instruction per SIMD (%.1f G wave-inst/s)\n", name, CH, W,
           ms, cyc, winst / (ms * 1e-3) / 1e9);
}

int main() {
    uint64_t* buf;
    CHK(hipMalloc(&buf, sizeof(uint64_t) * 256 * 256 * 8 + 64));
    // shader clock: cycle counter vs the 100 MHz realtime counter while the chip is busy
    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, buf, 1 << 22);
    uint64_t h[3];
    CHK(hipMemcpy(h, buf, 24, hipMemcpyDeviceToHost));
    double fclk = (double)h[0] / ((double)h[1] / 100e6);
    printf("shader clock (one wave, idle chip): %.0f MHz\n", fclk / 1e6);
    if (fclk < 1.0e9 || fclk > 3.0e9) fclk = 2.4e9;
    fclk = 2.4e9;  // price against the spec clock (MI355X_MICROARCH.md: 2400 MHz)
    run<0, 1, 1>("v_mad_u64_u32", buf, fclk);  // one dependent chain: latency
    run<0, 2, 1>("v_mad_u64_u32", buf, fclk);
    run<0, 4, 1>("v_mad_u64_u32", buf, fclk);
    run<0, 1, 2>("v_mad_u64_u32", buf, fclk);
    run<0, 2, 2>("v_mad_u64_u32", buf, fclk);
    run<0, 1, 16>("v_mad_u64_u32", buf, fclk);
    run<0, 1, 32>("v_mad_u64_u32", buf, fclk);
    run<1, 1, 16>("v_add_u32", buf, fclk);
    run<0, 1>("v_mad_u64_u32", buf, fclk);
    run<0, 2>("v_mad_u64_u32", buf, fclk);
    run<0, 4>("v_mad_u64_u32", buf, fclk);
    run<1, 1>("v_add_u32", buf, fclk);
    run<1, 2>("v_add_u32", buf, fclk);
    run<1, 4>("v_add_u32", buf, fclk);
    run<2, 1>("v_mul_lo_u32", buf, fclk);
    run<2, 2>("v_mul_lo_u32", buf, fclk);
    run<3, 1>("v_add_co+v_addc_co", buf, fclk);
    run<3, 2>("v_add_co+v_addc_co", buf, fclk);
    run<4, 1>("v_and_b32", buf, fclk);
    run<4, 2>("v_and_b32", buf, fclk);
    CHK(hipFree(buf));
    return 0;
}
