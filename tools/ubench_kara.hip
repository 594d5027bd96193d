// Limb-level Karatsuba for the radix-2^29 Fq product, measured
// against the product-scanning form the MSM kernels use (ff29.hpp f29_mul2: REDC(a b + c d), 14
// limbs, one 64-bit accumulator per column, 2 x 196 + 210 v_mad_u64_u32).
//
// f29_mul2_kara: the two products a b and c d by one Karatsuba level on 7-limb halves
//   L = aL bL + cL dL, H = aH bH + cH dH, S = (aL + aH)(bL + bH) + (cL + cH)(dL + dH)   (13 columns each,
//   3 x 98 limb products), then columns C_k = L_k + (S - L - H)_{k-7} + H_{k-14} (S - L - H = the cross
//   terms, non-negative column by column), then the same REDC scan over C (the m p products, 210).
// Normalized operands (< 2^29 limbs): S columns < 14 x 2^60; the REDC column sums C_k + m p can pass
// 2^64, so they are joined as f29_redc_sum4 does (low 29 bits and high parts separately).
// 504 multiply-adds instead of 602, paid for by the limb sums, the column combination (64-bit adds and
// subtracts, two instructions each) and the split join.
//
// Output: mismatches against f29_mul2 on random inputs (must be 0), then cycles per mul2 per SIMD at
// two waves per SIMD (the G2 kernels' occupancy) for both forms.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "ff29.hpp"

using namespace spx;

#define CHK(x)                                                          \
    do {                                                                \
        hipError_t e = (x);                                             \
        if (e != hipSuccess) {                                          \
            printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                    \
        }                                                               \
    } while (0)

DEV void f29_mul2_kara(F29& r, const F29& a, const F29& b, const F29& c, const F29& d) {
    uint32_t as[7], bs[7], cs[7], ds[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        as[i] = a.v[i] + a.v[i + 7];
        bs[i] = b.v[i] + b.v[i + 7];
        cs[i] = c.v[i] + c.v[i + 7];
        ds[i] = d.v[i] + d.v[i + 7];
    }
    uint64_t L[13], H[13], S[13];
#pragma unroll
    for (int k = 0; k < 13; ++k) {
        uint64_t l = 0, h = 0, s = 0;
        const int lo = k < 7 ? 0 : k - 6, hi = k < 7 ? k : 6;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            const int j = k - i;
            l += (uint64_t)a.v[i] * b.v[j];
            l += (uint64_t)c.v[i] * d.v[j];
            h += (uint64_t)a.v[i + 7] * b.v[j + 7];
            h += (uint64_t)c.v[i + 7] * d.v[j + 7];
            s += (uint64_t)as[i] * bs[j];
            s += (uint64_t)cs[i] * ds[j];
        }
        L[k] = f29_opaque(l);
        H[k] = f29_opaque(h);
        S[k] = f29_opaque(s);
    }
    uint32_t m[14], t[14];
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 27; ++k) {
        uint64_t ck = 0;
        if (k < 13) ck += L[k];
        if (k >= 14) ck += H[k - 14];
        if (k >= 7 && k < 20) ck += S[k - 7] - L[k - 7] - H[k - 7];
        uint64_t cb = 0;
        const int lo = k < 14 ? 0 : k - 13;
#pragma unroll
        for (int i = lo; i <= (k < 14 ? k - 1 : 13); ++i) cb += (uint64_t)m[i] * Q29::P[k - i];
        ck = f29_opaque(ck);
        cb = f29_opaque(cb);
        uint64_t low = (ck & Q29::M) + (cb & Q29::M) + (carry & Q29::M);
        const uint64_t high = (ck >> 29) + (cb >> 29) + (carry >> 29);
        if (k < 14) {
            m[k] = ((uint32_t)low * Q29::PINV) & Q29::M;
            low += (uint64_t)m[k] * Q29::P[0];
        } else {
            t[k - 14] = (uint32_t)low & Q29::M;
        }
        carry = high + (low >> 29);
    }
    t[13] = (uint32_t)carry;
#pragma unroll
    for (int i = 0; i < 14; ++i) r.v[i] = t[i];
}

DEV void rnd(F29& f, uint32_t& s) {
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        s = s * 1664525u + 1013904223u;
        f.v[i] = (s >> 3) & Q29::M;
    }
    f.v[13] &= 0x7;  // < 2^380 < p
}

__global__ void k_check(uint32_t* bad, uint32_t seed, int reps) {
    uint32_t s = seed ^ (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u;
    for (int it = 0; it < reps; ++it) {
        F29 a, b, c, d, r1, r2;
        rnd(a, s);
        rnd(b, s);
        rnd(c, s);
        rnd(d, s);
        if (it == 0) {  // extreme limbs: every limb 2^29 - 1 (above p: still within the bounds)
#pragma unroll
            for (int i = 0; i < 14; ++i) a.v[i] = b.v[i] = c.v[i] = d.v[i] = Q29::M;
            a.v[13] = b.v[13] = c.v[13] = d.v[13] = 0x7;
        }
        f29_mul2(r1, a, b, c, d);
        f29_mul2_kara(r2, a, b, c, d);
        for (int i = 0; i < 14; ++i)
            if (r1.v[i] != r2.v[i]) {
                atomicAdd(bad, 1u);
                break;
            }
    }
}

template <bool KARA>
__global__ __launch_bounds__(64, 2) void k_loop(uint32_t* out, uint32_t seed, int iters) {
    uint32_t s = seed ^ (blockIdx.x * 64 + threadIdx.x) * 2654435761u;
    F29 a, b, c, d;
    rnd(a, s);
    rnd(b, s);
    rnd(c, s);
    rnd(d, s);
    for (int i = 0; i < iters; ++i) {
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            F29 r;
            if constexpr (KARA)
                f29_mul2_kara(r, a, b, c, d);
            else
                f29_mul2(r, a, b, c, d);
            a = b;
            b = c;
            c = d;
            d = r;
        }
    }
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 14; ++k) h ^= a.v[k] ^ b.v[k] ^ c.v[k] ^ d.v[k];
    out[blockIdx.x * 64 + threadIdx.x] = h;
}

template <bool KARA>
static double run(uint32_t* buf, int iters) {
    const int blocks = 1024 * 2 * 4;  // 4 rounds of 2 waves on every SIMD
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_loop<KARA>, dim3(blocks), dim3(64), 0, 0, buf, 1u, 2);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_loop<KARA>, dim3(blocks), dim3(64), 0, 0, buf, 2u, iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double calls = (double)blocks * iters * 10;  // per wave
    return ms * 1e-3 * 2.4e9 * 1024.0 / calls;           // cycles per wave-call per SIMD
}

int main() {
    uint32_t *bad, *buf;
    CHK(hipMalloc(&bad, 4));
    CHK(hipMalloc(&buf, sizeof(uint32_t) * 1024 * 2 * 4 * 64));
    CHK(hipMemset(bad, 0, 4));
    hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, 0, bad, 7u, 16);
    uint32_t nbad = 0;
    CHK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
    printf("karatsuba vs product scanning: %u mismatching products of %d\n", nbad, 256 * 256 * 16);
    if (nbad) return 1;
    for (int rep = 0; rep < 3; ++rep) {
        const double ps = run<false>(buf, 40), ka = run<true>(buf, 40);
        printf("waves/SIMD 2: product scanning %.0f cycles per mul2, karatsuba %.0f (%.3fx)\n", ps, ka, ka / ps);
    }
    CHK(hipFree(buf));
    CHK(hipFree(bad));
    return 0;
}
