// BLS12-381 base field in unsaturated radix 2^29 (14 limbs, Montgomery R = 2^406), the arithmetic of
// the MSM's bucket accumulation and weighting kernels.
//
// Why: with 32-bit limbs every limb product's 64-bit carry-out needs its own instruction
// (v_mad_u64_u32 + v_addc, ~800 instructions per product; ff_asm.hpp). With 29-bit limbs a whole
// Montgomery column (<= 14 a*b + 14 c*d + 14 m*p products of < 2^58 each) fits one 64-bit
// accumulator, so each limb product is exactly one v_mad_u64_u32 and the column bookkeeping is
// 3 instructions: ~490 instructions per product, and a fused REDC(a*b + c*d) for the Fq2
// schoolbook product with lazy reduction (one reduction per output coefficient, no Karatsuba adds).
//
// Value bounds (lazy reduction): limbs are kept normalized (< 2^29), values are not. REDC of inputs
// below 2^392 returns < p + 2^378 < 2p. Callers track bounds in multiples of p:
//   add(a, b)        -> bound(a) + bound(b)
//   sub<K>(a, b)     -> a - b + K p, requires b < K p
//   reduce<K>(x)     -> x < K p  to  x < 2p   (log2(K) - 1 conditional subtractions)
// Values stored to memory are < 2p (< 2^382), packed into 12 x 32-bit words (pack / unpack).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace spx {

struct F29 {
    uint32_t v[14];
};

struct Q29 {  // constants (see tools/gen_mont_asm.py's sibling computation in DESIGN.md §4)
    static constexpr int N = 14;
    static constexpr uint32_t M = (1u << 29) - 1;
    static constexpr uint32_t PINV = 0x1ffcfffdu;  // -p^-1 mod 2^29
    static constexpr uint32_t P[14] = {0x1fffaaab, 0x0ff7ffff, 0x14ffffee, 0x17fffd62, 0x0f6241ea, 0x09507b58, 0x0afd9cc3,
                                       0x109e70a2, 0x1764774b, 0x121a5d66, 0x12c6e9ed, 0x12ffcd34, 0x00111ea3, 0x0000000d};
    static constexpr uint32_t P2[14] = {0x1fff5556, 0x1fefffff, 0x09ffffdc, 0x0ffffac5, 0x1ec483d5, 0x12a0f6b0, 0x15fb3986,
                                        0x013ce144, 0x0ec8ee97, 0x0434bacd, 0x058dd3db, 0x05ff9a69, 0x00223d47, 0x0000001a};
    static constexpr uint32_t P4[14] = {0x1ffeaaac, 0x1fdfffff, 0x13ffffb9, 0x1ffff58a, 0x1d8907aa, 0x0541ed61, 0x0bf6730d,
                                        0x0279c289, 0x1d91dd2e, 0x0869759a, 0x0b1ba7b6, 0x0bff34d2, 0x00447a8e, 0x00000034};
    static constexpr uint32_t P8[14] = {0x1ffd5558, 0x1fbfffff, 0x07ffff73, 0x1fffeb15, 0x1b120f55, 0x0a83dac3, 0x17ece61a,
                                        0x04f38512, 0x1b23ba5c, 0x10d2eb35, 0x16374f6c, 0x17fe69a4, 0x0088f51c, 0x00000068};
    static constexpr uint32_t P16[14] = {0x1ffaaab0, 0x1f7fffff, 0x0ffffee7, 0x1fffd62a, 0x16241eab, 0x1507b587,
                                         0x0fd9cc34, 0x09e70a25, 0x164774b8, 0x01a5d66b, 0x0c6e9ed9, 0x0ffcd349,
                                         0x0111ea39, 0x000000d0};
    // j p mod 2^29 = 2^29 - j 0x5555 (P[0] = 2^29 - 0x5555): INV5555 = 0x5555^-1 mod 2^32
    static constexpr uint32_t INV5555 = 0xfffcfffdu;
    // R2 mod p (Montgomery one), R1 = 2^384 mod p (REDC by it maps x R2 -> x R1), R2^2 / R1 mod p (x R1 -> x R2)
    static constexpr uint32_t ONE[14] = {0x03a9fb84, 0x0ba00690, 0x071288f1, 0x0f59bcc5, 0x126cb614, 0x0585bf36, 0x1b85ac3d,
                                         0x1cf856fa, 0x1891ecbd, 0x1a7eec05, 0x155a88f0, 0x0741ac6d, 0x1317c30f, 0x00000009};
    static constexpr uint32_t TO_R1[14] = {0x0002fffd, 0x10480000, 0x0300009d, 0x08001788, 0x158baebf, 0x0c2ba9e3, 0x1d157d22,
                                           0x0a6e0a4a, 0x0d77ce58, 0x1d12b763, 0x1701c6a5, 0x1501c926, 0x1f65ec3f, 0x0000000a};
    static constexpr uint32_t FROM_R1[14] = {0x1fddebbd, 0x1a4f5474, 0x0291f399, 0x14d03b3c, 0x0f6cad2c, 0x1b4cabca,
                                             0x1592827c, 0x021c6ac7, 0x1ec52a84, 0x16fd5ec4, 0x0c960da6, 0x0fd2af6b,
                                             0x13263591, 0x0000000b};
};

template <int K>
DEV constexpr uint32_t kp29(int i) {
    static_assert(K == 1 || K == 2 || K == 4 || K == 8 || K == 16, "multiple of p");
    return K == 1 ? Q29::P[i] : K == 2 ? Q29::P2[i] : K == 4 ? Q29::P4[i] : K == 8 ? Q29::P8[i] : Q29::P16[i];
}

DEV void f29_set(F29& r, const uint32_t (&c)[14]) {
#pragma unroll
    for (int i = 0; i < 14; ++i) r.v[i] = c[i];
}
DEV void f29_zero(F29& r) {
#pragma unroll
    for (int i = 0; i < 14; ++i) r.v[i] = 0;
}
DEV void f29_one(F29& r) { f29_set(r, Q29::ONE); }

// Each Montgomery column is one 64-bit accumulator (<= 42 products < 2^58). Splitting a column into 2-4
// independent chains was measured slower at two waves per SIMD: dependent-mad latency
// is not what bounds the G2 kernels.
// An empty asm on a partial sum: integer addition is associative, and without the barrier LLVM's
// reassociation folds separately summed chains back into one serial v_mad_u64_u32 chain.
DEV uint64_t f29_opaque(uint64_t x) {
    asm("" : "+v"(x));
    return x;
}

// REDC(sum of NP products a_j b_j): NP = 1 (f29_mul) or 2 (f29_mul2, lazy reduction)
template <int NP>
DEV void f29_redc_sum(F29& r, const F29* const (&a)[NP], const F29* const (&b)[NP]) {
    uint32_t m[14], t[14];
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 27; ++k) {
        const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
        uint64_t ch = 0;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
#pragma unroll
            for (int q = 0; q < NP; ++q) ch += (uint64_t)a[q]->v[i] * b[q]->v[k - i];
        }
#pragma unroll
        for (int i = lo; i <= (k < 14 ? k - 1 : 13); ++i) ch += (uint64_t)m[i] * Q29::P[k - i];
        uint64_t acc = ch + carry;
        if (k < 14) {
            m[k] = ((uint32_t)acc * Q29::PINV) & Q29::M;
            acc += (uint64_t)m[k] * Q29::P[0];
        } else {
            t[k - 14] = (uint32_t)acc & Q29::M;
        }
        carry = acc >> 29;
    }
    t[13] = (uint32_t)carry;
#pragma unroll
    for (int i = 0; i < 14; ++i) r.v[i] = t[i];
}

// r = REDC(a0 b0 + a1 b1 + a2 b2 + a3 b3): one reduction for four products. A column then holds up
// to 4 x 14 products and 14 m p terms, which can pass 2^64, so it is summed in two 64-bit chains
// (A: products 0, 1; B: products 2, 3 and m p). PRECONDITION: in each chain at most ONE of its two
// products may have a factor with limbs below 2^30 (limb products < 2^59, as the borrow-free
// lane-pair operands give); the other product must have both factors' limbs below 2^29 (< 2^58).
// Then A <= 14 x 2^59 + 14 x 2^58 = 42 x 2^58 and B <= 14 x 2^59 + 14 x 2^58 + 14 x 2^58 (m p)
// = 56 x 2^58, both below 2^64 = 64 x 2^58; two 2^30-limb products in one chain (70 x 2^58 with m p)
// would overflow. The only caller, PairOps<FP29A>::mul_sum (fq2pair.hpp), meets it. The chains are
// joined without a 65-bit sum: the column's low 29 bits come from the low parts, the carry from the
// high parts plus the low parts' overflow.
DEV void f29_redc_sum4(F29& r, const F29& a0, const F29& b0, const F29& a1, const F29& b1, const F29& a2,
                       const F29& b2, const F29& a3, const F29& b3) {
    uint32_t m[14], t[14];
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 27; ++k) {
        const int lo = k < 14 ? 0 : k - 13, hi = k < 14 ? k : 13;
        uint64_t ca = 0, cb = 0;
#pragma unroll
        for (int i = lo; i <= hi; ++i) {
            ca += (uint64_t)a0.v[i] * b0.v[k - i];
            ca += (uint64_t)a1.v[i] * b1.v[k - i];
            cb += (uint64_t)a2.v[i] * b2.v[k - i];
            cb += (uint64_t)a3.v[i] * b3.v[k - i];
        }
#pragma unroll
        for (int i = lo; i <= (k < 14 ? k - 1 : 13); ++i) cb += (uint64_t)m[i] * Q29::P[k - i];
        ca = f29_opaque(ca);
        cb = f29_opaque(cb);
        // low: < 3 x 2^29 (+ m p0 < 2^58 below); high: < 2^36 each
        uint64_t low = (ca & Q29::M) + (cb & Q29::M) + (carry & Q29::M);
        const uint64_t high = (ca >> 29) + (cb >> 29) + (carry >> 29);
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

// r = REDC(a b) = a b / 2^406 mod p, < 2p for inputs < 2^392
DEV void f29_mul(F29& r, const F29& a, const F29& b) {
    const F29* const pa[1] = {&a};
    const F29* const pb[1] = {&b};
    f29_redc_sum<1>(r, pa, pb);
}

// r = REDC(a b + c d): one reduction for a sum of two products (lazy reduction)
DEV void f29_mul2(F29& r, const F29& a, const F29& b, const F29& c, const F29& d) {
    const F29* const pa[2] = {&a, &c};
    const F29* const pb[2] = {&b, &d};
    f29_redc_sum<2>(r, pa, pb);
}

DEV void f29_add(F29& r, const F29& a, const F29& b) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) {
        const uint32_t t = a.v[i] + b.v[i] + c;
        r.v[i] = t & Q29::M;
        c = t >> 29;
    }
    r.v[13] = a.v[13] + b.v[13] + c;
}

// r = a - b + K p  (b < K p)
template <int K>
DEV void f29_sub(F29& r, const F29& a, const F29& b) {
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) {
        const int32_t t = (int32_t)a.v[i] - (int32_t)b.v[i] + (int32_t)kp29<K>(i) + c;
        r.v[i] = (uint32_t)t & Q29::M;
        c = t >> 29;  // arithmetic
    }
    r.v[13] = (uint32_t)((int32_t)a.v[13] - (int32_t)b.v[13] + (int32_t)kp29<K>(13) + c);
}

// x -= K p if x >= K p
template <int K>
DEV void f29_csub(F29& x) {
    uint32_t d[14];
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) {
        const int32_t t = (int32_t)x.v[i] - (int32_t)kp29<K>(i) + c;
        d[i] = (uint32_t)t & Q29::M;
        c = t >> 29;
    }
    const int32_t top = (int32_t)x.v[13] - (int32_t)kp29<K>(13) + c;
    d[13] = (uint32_t)top;
    const bool keep = top < 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) x.v[i] = keep ? x.v[i] : d[i];
}

// x < K p  ->  x < 2p
template <int K>
DEV void f29_reduce(F29& x) {
    if constexpr (K >= 16) f29_csub<8>(x);
    if constexpr (K >= 8) f29_csub<4>(x);
    if constexpr (K >= 4) f29_csub<2>(x);
}

template <int K>
DEV bool f29_eq_kp(const F29& x) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) acc |= x.v[i] ^ kp29<K>(i);
    return acc == 0;
}
DEV bool f29_is_zero_raw(const F29& x) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) acc |= x.v[i];
    return acc == 0;
}
// x == 0 mod p for x < 2p
DEV bool f29_zero2(const F29& x) { return f29_is_zero_raw(x) || f29_eq_kp<1>(x); }
// x == 0 mod p for x < 4p
DEV bool f29_zero4(const F29& x) {
    F29 y = x;
    f29_csub<2>(y);
    return f29_zero2(y);
}
// x == 0 mod p for x < K p (K <= 16). x == j p for some j < K exactly when limb 0 (x mod 2^29, limbs
// are normalized) is j p mod 2^29 = 2^29 - j 0x5555: a multiply and a compare reject every other
// value, and only a candidate pays for the reduction and the full comparison.
template <int K>
DEV bool f29_zero_lt(const F29& x) {
    const uint32_t v0 = x.v[0];
    const bool cand = v0 == 0 || ((1u << 29) - v0) * Q29::INV5555 < (uint32_t)K;
    if (!cand) return false;
    F29 y = x;
    f29_reduce<K>(y);
    return f29_zero2(y);
}
// canonical (< p) from < 2p
DEV void f29_canon(F29& x) { f29_csub<1>(x); }

// 12 x 32-bit words (value < 2^384) <-> 14 x 29-bit limbs
DEV void f29_unpack(F29& r, const uint32_t* w) {
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        const int o = 29 * i, k = o >> 5, s = o & 31;
        uint32_t v = w[k] >> s;
        if (s + 29 > 32 && k + 1 < 12) v |= w[k + 1] << (32 - s);
        r.v[i] = v & Q29::M;
    }
}
DEV void f29_pack(uint32_t* w, const F29& x) {
#pragma unroll
    for (int k = 0; k < 12; ++k) w[k] = 0;
#pragma unroll
    for (int i = 0; i < 14; ++i) {
        const int o = 29 * i, k = o >> 5, s = o & 31;
        w[k] |= x.v[i] << s;
        if (s + 29 > 32 && k + 1 < 12) w[k + 1] |= x.v[i] >> (32 - s);
    }
}

// ---------------------------------------------------------------- Fq2 = Fq[u] / (u^2 + 1)
struct F2_29 {
    F29 c0, c1;
};
// Operands of the products below may be up to 8p per coefficient (products stay far below 2^406 p).
// schoolbook with lazy reduction: c0 = REDC(a0 b0 + a1 (8p - b1)), c1 = REDC(a0 b1 + a1 b0)
DEV void f2_29_mul(F2_29& r, const F2_29& a, const F2_29& b) {
    F29 nb1, c0, c1;
    F29 z;
    f29_zero(z);
    f29_sub<8>(nb1, z, b.c1);
    f29_mul2(c0, a.c0, b.c0, a.c1, nb1);
    f29_mul2(c1, a.c0, b.c1, a.c1, b.c0);
    r.c0 = c0;
    r.c1 = c1;
}
// (a0 + a1 u)^2 = (a0 + a1)(a0 - a1) + 2 a0 a1 u
// KB: bound of a.c1 in multiples of p (the subtraction adds KB p)
template <int KB = 8>
DEV void f2_29_sqr(F2_29& r, const F2_29& a) {
    F29 s, d, t, c0, c1;
    f29_add(s, a.c0, a.c1);
    f29_sub<KB>(d, a.c0, a.c1);
    f29_add(t, a.c0, a.c0);
    f29_mul(c0, s, d);
    f29_mul(c1, t, a.c1);
    r.c0 = c0;
    r.c1 = c1;
}

// ---------------------------------------------------------------- uniform ops for the curve code
template <class F>
struct Ops29;
template <>
struct Ops29<F29> {
    static constexpr bool kFusedSum = true;  // mul_sum is one reduction
    static DEV void mul(F29& r, const F29& a, const F29& b) { f29_mul(r, a, b); }
    // r = a b + c d with one reduction (operands < 16p: the sum < 512 p^2 < 2^406 p), < 2p
    static DEV void mul_sum(F29& r, const F29& a, const F29& b, const F29& c, const F29& d) { f29_mul2(r, a, b, c, d); }
    static DEV void sqr(F29& r, const F29& a) { f29_mul(r, a, a); }
    static DEV void add(F29& r, const F29& a, const F29& b) { f29_add(r, a, b); }
    template <int K>
    static DEV void sub(F29& r, const F29& a, const F29& b) {
        f29_sub<K>(r, a, b);
    }
    template <int K>
    static DEV void reduce(F29& x) {
        f29_reduce<K>(x);
    }
    static DEV bool zero2(const F29& x) { return f29_zero2(x); }
    static DEV bool zero4(const F29& x) { return f29_zero4(x); }
    template <int K>
    static DEV bool zero_lt(const F29& x) {
        return f29_zero_lt<K>(x);
    }
    template <int KB>
    static DEV void sqr_b(F29& r, const F29& a) {
        f29_mul(r, a, a);
    }
    static DEV bool is_zero_raw(const F29& x) { return f29_is_zero_raw(x); }
    static DEV void zero(F29& r) { f29_zero(r); }
    static DEV void one(F29& r) { f29_one(r); }
};
template <>
struct Ops29<F2_29> {
    static constexpr bool kFusedSum = false;
    static DEV void mul(F2_29& r, const F2_29& a, const F2_29& b) { f2_29_mul(r, a, b); }
    static DEV void mul_sum(F2_29& r, const F2_29& a, const F2_29& b, const F2_29& c, const F2_29& d) {
        F2_29 x, y;
        f2_29_mul(x, a, b);
        f2_29_mul(y, c, d);
        f29_add(r.c0, x.c0, y.c0);  // < 4p
        f29_add(r.c1, x.c1, y.c1);
    }
    static DEV void sqr(F2_29& r, const F2_29& a) { f2_29_sqr(r, a); }
    static DEV void add(F2_29& r, const F2_29& a, const F2_29& b) {
        f29_add(r.c0, a.c0, b.c0);
        f29_add(r.c1, a.c1, b.c1);
    }
    template <int K>
    static DEV void sub(F2_29& r, const F2_29& a, const F2_29& b) {
        f29_sub<K>(r.c0, a.c0, b.c0);
        f29_sub<K>(r.c1, a.c1, b.c1);
    }
    template <int K>
    static DEV void reduce(F2_29& x) {
        f29_reduce<K>(x.c0);
        f29_reduce<K>(x.c1);
    }
    static DEV bool zero2(const F2_29& x) { return f29_zero2(x.c0) && f29_zero2(x.c1); }
    static DEV bool zero4(const F2_29& x) { return f29_zero4(x.c0) && f29_zero4(x.c1); }
    template <int K>
    static DEV bool zero_lt(const F2_29& x) {
        return f29_zero_lt<K>(x.c0) && f29_zero_lt<K>(x.c1);
    }
    template <int KB>
    static DEV void sqr_b(F2_29& r, const F2_29& a) {
        f2_29_sqr<KB>(r, a);
    }
    static DEV bool is_zero_raw(const F2_29& x) { return f29_is_zero_raw(x.c0) && f29_is_zero_raw(x.c1); }
    static DEV void zero(F2_29& r) {
        f29_zero(r.c0);
        f29_zero(r.c1);
    }
    static DEV void one(F2_29& r) {
        f29_one(r.c0);
        f29_zero(r.c1);
    }
};

}  // namespace spx
