// Fr Montgomery product (ff_asm.hpp) issue rate on gfx950: one dependent chain of products per wave,
// two independent chains through fr_mul_asm (the compiler may only alternate whole per-column asm
// blocks), and two chains through fr_mul_x2_asm (the two products' multiply-accumulates interleaved
// instruction by instruction, carries in VCC and an SGPR pair). Register-resident, full grid, at 4 and 8
// waves per SIMD. Prints mismatches of fr_mul_x2_asm against fr_mul_asm, then cycles per product per
// SIMD for each form.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "ff_dev.hpp"

using namespace spx;

#define CHK(x)                                                          \
    do {                                                                \
        hipError_t e = (x);                                             \
        if (e != hipSuccess) {                                          \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                    \
        }                                                               \
    } while (0)

DEV void rnd(Fr& f, uint32_t& s) {
    for (int i = 0; i < 8; ++i) {
        s = s * 1664525u + 1013904223u;
        f.v[i] = s;
    }
    f.v[7] &= 0x3fffffffu;  // < r
}

__global__ void k_check(uint32_t* bad, uint32_t seed) {
    uint32_t s = seed ^ (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u;
    for (int it = 0; it < 32; ++it) {
        Fr a, b, c, d, r0, r1, q0, q1;
        rnd(a, s), rnd(b, s), rnd(c, s), rnd(d, s);
        fr_mul_asm(r0, a, b);
        fr_mul_asm(r1, c, d);
        fr_mul_x2_asm(q0, a, b, q1, c, d);
        for (int i = 0; i < 8; ++i)
            if (r0.v[i] != q0.v[i] || r1.v[i] != q1.v[i]) {
                atomicAdd(bad, 1u);
                break;
            }
    }
}

template <int KIND, int W>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W))) void k_loop(uint32_t* out, uint32_t seed, int iters) {
    uint32_t s = seed ^ (blockIdx.x * 64 + threadIdx.x) * 2654435761u;
    Fr x0, x1, y;
    rnd(x0, s), rnd(x1, s), rnd(y, s);
    for (int i = 0; i < iters; ++i) {
        if constexpr (KIND == 0) {
            fr_mul_asm(x0, x0, y);
            fr_mul_asm(x0, x0, y);
        } else if constexpr (KIND == 1) {
            fr_mul_asm(x0, x0, y);
            fr_mul_asm(x1, x1, y);
        } else {
            fr_mul_x2_asm(x0, x0, y, x1, x1, y);
        }
    }
    uint32_t h = 0;
    for (int k = 0; k < 8; ++k) h ^= x0.v[k] ^ x1.v[k];
    out[blockIdx.x * 64 + threadIdx.x] = h;
}

template <int KIND, int W>
static void run(uint32_t* buf, int iters) {
    const int blocks = 1024 * W * 4;  // 4 rounds of W waves on every SIMD
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_loop<KIND, W>), dim3(blocks), dim3(64), 0, 0, buf, 1u, 4);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_loop<KIND, W>), dim3(blocks), dim3(64), 0, 0, buf, 2u, iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double prods = (double)blocks * iters * 2;  // wave-products
    printf("%-28s waves/SIMD %d: %.0f cycles per product per SIMD (%.3f ms)\n",
           KIND == 0 ? "one chain" : (KIND == 1 ? "two chains, fr_mul_asm" : "two chains, fr_mul_x2_asm"), W,
           ms * 1e-3 * 2.4e9 * 1024.0 / prods, ms);
}

int main() {
    uint32_t *bad, *buf;
    CHK(hipMalloc(&bad, 4));
    CHK(hipMalloc(&buf, sizeof(uint32_t) * 1024 * 8 * 4 * 64));
    CHK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, 0, bad, 5u);
    uint32_t nbad = 0;
    CHK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
    printf("fr_mul_x2_asm vs fr_mul_asm: %u mismatches of %d\n", nbad, 256 * 256 * 32);
    if (nbad) return 1;
    for (int rep = 0; rep < 2; ++rep) {
        run<0, 4>(buf, 200);
        run<1, 4>(buf, 200);
        run<2, 4>(buf, 200);
        run<0, 8>(buf, 200);
        run<1, 8>(buf, 200);
        run<2, 8>(buf, 200);
    }
    return 0;
}
