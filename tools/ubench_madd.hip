// Cost of the G2 bucket-accumulation formula on gfx950, register-resident (no memory traffic):
//   k_madd: x29_madd (madd-2008-s, lane-pair Fq2) in a loop — the hot loop of k_accum_aff<Fq2>,
//           ~100 KB of straight-line code per iteration;
//   k_mul : the lane-pair Fq2 product alone, 10 per iteration in a non-unrolled loop (~5 KB of code).
// (Round 2 built this once per SPX_F29_CHAINS value; the chain variant was dropped: one chain.) The per-product cost of k_madd over
// that of k_mul separates the formula's own overhead (additions, selects, instruction supply) from
// the product's issue cost. Operands are random field-sized values, not curve points: the formula's
// cost does not depend on them (no exceptional branch is taken).
#ifndef SPX_F29_CHAINS
#define SPX_F29_CHAINS 1
#endif
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "curve29.hpp"
#include "fq2pair.hpp"

using namespace spx;

#define CHK(x)                                                          \
    do {                                                                \
        hipError_t e = (x);                                             \
        if (e != hipSuccess) {                                          \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                    \
        }                                                               \
    } while (0)

DEV void rnd(F29& f, uint32_t& s) {
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        s = s * 1664525u + 1013904223u;
        f.v[i] = (s >> 3) & Q29::M;
    }
    f.v[13] &= 0x7;  // < 2^380 < p
}

template <int W>
__global__ __launch_bounds__(64, W) void k_madd(uint32_t* out, uint32_t seed, int iters) {
    uint32_t s = seed ^ ((blockIdx.x * 64 + threadIdx.x) >> 1) * 2654435761u;
    X29<FP29A> acc;
    FP29A px, py;
    rnd(acc.x.v, s);
    rnd(acc.y.v, s);
    rnd(acc.zz.v, s);
    rnd(acc.zzz.v, s);
    rnd(px.v, s);
    rnd(py.v, s);
    for (int i = 0; i < iters; ++i) {
        x29_madd(acc, px, py, false);
        px.v.v[0] ^= (uint32_t)i & 1u;
    }
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 14; ++k) h ^= acc.x.v.v[k] ^ acc.y.v.v[k] ^ acc.zz.v.v[k] ^ acc.zzz.v.v[k];
    out[blockIdx.x * 64 + threadIdx.x] = h;
}

template <int W>
__global__ __launch_bounds__(64, W) void k_mul(uint32_t* out, uint32_t seed, int iters) {
    uint32_t s = seed ^ ((blockIdx.x * 64 + threadIdx.x) >> 1) * 2654435761u;
    FP29A a, b;
    rnd(a.v, s);
    rnd(b.v, s);
    for (int i = 0; i < iters; ++i) {
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            FP29A r;
            Ops29<FP29A>::mul(r, a, b);
            a = b;
            b = r;
        }
    }
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 14; ++k) h ^= a.v.v[k] ^ b.v.v[k];
    out[blockIdx.x * 64 + threadIdx.x] = h;
}

template <int KIND, int W>
static void run(uint32_t* buf, int iters, double per_iter_products) {
    const int blocks = 1024 * W * 4;  // 4 rounds of W waves on every SIMD
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto launch = [&](uint32_t seed, int it) {
        if (KIND == 0)
            hipLaunchKernelGGL(k_madd<W>, dim3(blocks), dim3(64), 0, 0, buf, seed, it);
        else
            hipLaunchKernelGGL(k_mul<W>, dim3(blocks), dim3(64), 0, 0, buf, seed, it);
    };
    launch(1u, 2);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    launch(2u, iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double wave_iters = (double)blocks * iters;  // one wave per block
    const double cyc_iter = ms * 1e-3 * 2.4e9 * 1024.0 / wave_iters;
    printf("chains %d %-6s waves/SIMD %d: %.3f ms, %.0f cycles per wave-iteration per SIMD, %.0f per Fq2 product, "
           "%.3f G iterations/s (x32 elements)\n",
           SPX_F29_CHAINS, KIND == 0 ? "madd" : "mul", W, ms, cyc_iter, cyc_iter / per_iter_products,
           wave_iters * 32 / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
    uint32_t* buf;
    CHK(hipMalloc(&buf, sizeof(uint32_t) * 1024 * 4 * 4 * 64));
    // k_madd: 8 products + 2 squares (a square ~ 2/3 of a product in lane-pair form) per iteration
    run<0, 2>(buf, 40, 8 + 2 * 2.0 / 3.0);
    run<0, 1>(buf, 40, 8 + 2 * 2.0 / 3.0);
    run<1, 2>(buf, 40, 10);
    run<1, 1>(buf, 40, 10);
    CHK(hipFree(buf));
    return 0;
}
