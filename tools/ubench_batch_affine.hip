// Batch-affine accumulation (Montgomery's trick) against madd-2008-s for the G2 bucket accumulation,
// measured on gfx950 in the lane-pair Fq2 form of the product kernels (fq2pair.hpp).
//
//   k_inv   : one Fq inversion per lane pair per iteration (Fermat, x^(p-2), 4-bit windows; both
//             lanes of the pair run it on the pair's norm, as a batch-affine step needs)
//   k_aff<K>: K independent affine accumulators per lane pair, one step = K affine additions sharing
//             ONE Fq2 inversion: prefix products of the K denominators (x_P - x_A), the inversion of
//             the last, the backward pass (2 products per k), then lambda, x3, y3 (1 product, 1 square,
//             1 product). Accumulators and prefix products live in global memory (they do not fit on
//             chip at two waves per SIMD), laid out [k][lane] so every access is lane-contiguous.
//   k_madd  : x29_madd in registers (the formula of k_accum_aff<Fq2>), for the same grid.
// Operands are random field-sized values (no exceptional branch is taken); the cost of the
// arithmetic does not depend on them. Output: additions per second at each K, and the break-even K.
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

// p - 2 (BLS12-381 base field), 32-bit words, little endian
__device__ __constant__ uint32_t kPm2[12] = {0xffffaaa9u, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                                             0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};

// x^(p-2) in the radix-2^29 Montgomery domain: 4-bit fixed window, 14 + 380 squarings + 95 products
DEV void f29_inv(F29& r, const F29& x) {
    F29 tab[16];
    f29_one(tab[0]);
    tab[1] = x;
#pragma unroll 1
    for (int i = 2; i < 16; ++i) f29_mul(tab[i], tab[i - 1], x);
    F29 acc;
    f29_one(acc);
#pragma unroll 1
    for (int w = 95; w >= 0; --w) {
        if (w != 95)
#pragma unroll 1
            for (int k = 0; k < 4; ++k) f29_mul(acc, acc, acc);
        const uint32_t d = (kPm2[w >> 3] >> (4 * (w & 7))) & 0xf;
        F29 t = tab[0];
#pragma unroll 1
        for (int i = 1; i < 16; ++i) t = f29_select(i == (int)d, tab[i], t);  // no divergent table index
        f29_mul(acc, acc, t);
    }
    r = acc;
}

// Fq2 inverse of a lane-pair value: conj(a) / (a0^2 + a1^2); both lanes invert the norm
DEV void pair_inv(FP29A& r, const FP29A& a) {
    F29 sq, nrm, inv;
    f29_mul(sq, a.v, a.v);
    f29_add(nrm, sq, pair_swap(sq));
    f29_inv(inv, nrm);
    F29 t;
    f29_mul(t, a.v, inv);  // even: a0 / N; odd: a1 / N, negated below
    if (pair_odd()) {
        F29 z;
        f29_zero(z);
        f29_sub<2>(t, z, t);
        f29_reduce<4>(t);
    }
    r.v = t;
}

template <int W>
__global__ __launch_bounds__(64, W) void k_inv(uint32_t* out, uint32_t seed, int iters) {
    uint32_t s = seed ^ ((blockIdx.x * 64 + threadIdx.x) >> 1) * 2654435761u;
    FP29A a;
    rnd(a.v, s);
    for (int i = 0; i < iters; ++i) {
        FP29A r;
        pair_inv(r, a);
        a = r;
        a.v.v[0] ^= (uint32_t)i & 1u;
    }
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 14; ++k) h ^= a.v.v[k];
    out[blockIdx.x * 64 + threadIdx.x] = h;
}

DEV void ldg(F29& r, const uint32_t* p, uint64_t stride) {
#pragma unroll
    for (int i = 0; i < 14; ++i) r.v[i] = p[i * stride];
}
DEV void stg(uint32_t* p, uint64_t stride, const F29& r) {
#pragma unroll
    for (int i = 0; i < 14; ++i) p[i * stride] = r.v[i];
}

// state: [3][K][14][lanes] words (acc x, acc y, prefix), lane-contiguous
template <int W, int K>
__global__ __launch_bounds__(64, W) void k_aff(uint32_t* st, uint32_t* out, uint32_t seed, int iters) {
    using O = Ops29<FP29A>;
    const uint64_t lanes = (uint64_t)gridDim.x * 64, lane = blockIdx.x * 64ull + threadIdx.x;
    uint32_t* AX = st + lane;
    uint32_t* AY = st + (uint64_t)K * 14 * lanes + lane;
    uint32_t* PR = st + 2ull * K * 14 * lanes + lane;
    auto at = [&](uint32_t* base, int k) { return base + (uint64_t)k * 14 * lanes; };
    uint32_t s = seed ^ (uint32_t)(lane >> 1) * 2654435761u;
    for (int k = 0; k < K; ++k) {
        F29 x, y;
        rnd(x, s);
        rnd(y, s);
        stg(at(AX, k), lanes, x);
        stg(at(AY, k), lanes, y);
    }
    FP29A px, py;  // the incoming point of accumulator k: (px + k, py + k), register-resident inputs
    rnd(px.v, s);
    rnd(py.v, s);
    for (int it = 0; it < iters; ++it) {
        // prefix products of d_k = x_P - x_A
        FP29A pre;
#pragma unroll 1
        for (int k = 0; k < K; ++k) {
            FP29A ax, d;
            ldg(ax.v, at(AX, k), lanes);
            FP29A xk = px;
            xk.v.v[0] += (uint32_t)k;
            O::template sub<2>(d, xk, ax);
            if (k == 0)
                pre = d;
            else
                O::mul(pre, pre, d);
            stg(at(PR, k), lanes, pre.v);
        }
        FP29A inv;
        pair_inv(inv, pre);
        // backward: inv_k = inv * pre_{k-1}; inv *= d_k; then the affine addition of accumulator k
#pragma unroll 1
        for (int k = K - 1; k >= 0; --k) {
            FP29A ax, ay, d, ik, lam, t, x3, y3;
            ldg(ax.v, at(AX, k), lanes);
            ldg(ay.v, at(AY, k), lanes);
            FP29A xk = px, yk = py;
            xk.v.v[0] += (uint32_t)k;
            yk.v.v[0] += (uint32_t)k;
            O::template sub<2>(d, xk, ax);
            if (k > 0) {
                FP29A pk;
                ldg(pk.v, at(PR, k - 1), lanes);
                O::mul(ik, inv, pk);
                O::mul(inv, inv, d);
            } else {
                ik = inv;
            }
            O::template sub<2>(t, yk, ay);
            O::mul(lam, t, ik);          // lambda = (y_P - y_A) / (x_P - x_A)
            O::sqr(t, lam);
            O::template sub<4>(x3, t, ax);
            O::template sub<4>(x3, x3, xk);
            O::template reduce<8>(x3);   // x3 = lambda^2 - x_A - x_P
            O::template sub<2>(t, ax, x3);
            O::mul(y3, lam, t);
            O::template sub<2>(y3, y3, ay);
            O::template reduce<4>(y3);   // y3 = lambda (x_A - x3) - y_A
            stg(at(AX, k), lanes, x3.v);
            stg(at(AY, k), lanes, y3.v);
        }
        px.v.v[1] ^= (uint32_t)it & 1u;
    }
    out[lane] = px.v.v[0];
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

static const int kBlocks = 1024 * 2 * 2;  // two rounds of two waves on every SIMD (64K lane pairs... x2)

template <class L>
static float timed(L launch) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0));
    launch();
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
}

template <int K>
static void run_aff(uint32_t* st, uint32_t* out, int iters, double madd_rate) {
    hipLaunchKernelGGL((k_aff<2, K>), dim3(kBlocks), dim3(64), 0, 0, st, out, 1u, 1);
    CHK(hipDeviceSynchronize());
    const float ms = timed([&] { hipLaunchKernelGGL((k_aff<2, K>), dim3(kBlocks), dim3(64), 0, 0, st, out, 2u, iters); });
    CHK(hipGetLastError());
    const double adds = (double)kBlocks * 32 * K * iters;  // lane pairs x K per step
    const double rate = adds / (ms * 1e-3);
    printf("batch-affine K=%3d: %.3f ms, %.3f G additions/s (%.2fx madd-2008-s register-resident), "
           "%.0f B global traffic per addition\n",
           K, ms, rate / 1e9, rate / madd_rate, (5.0 * 56 + 2 * 56) * 2);
}

int main() {
    uint32_t* out;
    CHK(hipMalloc(&out, sizeof(uint32_t) * kBlocks * 64));
    // madd-2008-s, register-resident
    hipLaunchKernelGGL(k_madd<2>, dim3(kBlocks), dim3(64), 0, 0, out, 1u, 2);
    CHK(hipDeviceSynchronize());
    const int mi = 40;
    const float mms = timed([&] { hipLaunchKernelGGL(k_madd<2>, dim3(kBlocks), dim3(64), 0, 0, out, 2u, mi); });
    const double madd_rate = (double)kBlocks * 32 * mi / (mms * 1e-3);
    printf("madd-2008-s (x29_madd, registers): %.3f ms, %.3f G additions/s\n", mms, madd_rate / 1e9);
    // one Fq2 inversion per lane pair
    hipLaunchKernelGGL(k_inv<2>, dim3(kBlocks), dim3(64), 0, 0, out, 1u, 1);
    CHK(hipDeviceSynchronize());
    const int ii = 4;
    const float ims = timed([&] { hipLaunchKernelGGL(k_inv<2>, dim3(kBlocks), dim3(64), 0, 0, out, 2u, ii); });
    const double inv_rate = (double)kBlocks * 32 * ii / (ims * 1e-3);
    printf("Fq2 inversion (pair, Fermat on the norm): %.3f ms, %.4f G inversions/s = %.1f madd-2008-s additions each\n",
           ims, inv_rate / 1e9, madd_rate / inv_rate);
    uint32_t* st;
    const size_t words = 3ull * 128 * 14 * kBlocks * 64;
    CHK(hipMalloc(&st, words * 4));
    run_aff<8>(st, out, 4, madd_rate);
    run_aff<16>(st, out, 4, madd_rate);
    run_aff<32>(st, out, 2, madd_rate);
    run_aff<64>(st, out, 2, madd_rate);
    run_aff<128>(st, out, 1, madd_rate);
    CHK(hipFree(st));
    CHK(hipFree(out));
    return 0;
}
