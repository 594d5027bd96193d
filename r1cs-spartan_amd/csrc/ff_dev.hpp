// Device big-integer field arithmetic for BLS12-381 on CDNA4 (gfx950).
//
// Fr (scalar field, 255 bits) = 8 x u32 limbs, Fq (base field, 381 bits) = 12 x u32 limbs,
// both in Montgomery form with R = 2^256 / 2^384 — bit-identical to ark-ff's 4x/6x u64
// Montgomery representation, so device buffers and ark-serialize byte images convert with
// one Montgomery multiplication. Fq2 = Fq[u]/(u^2+1).
//
// Multiplication is CIOS on 32-bit limbs: every limb product is one v_mad_u64_u32 (32x32+64
// -> 64), the 64-bit VALU path of CDNA4; there is no MFMA anywhere (big-integer modular
// arithmetic is not a dense FP contraction). Both moduli leave spare top bits
// (r < 2^255, q < 2^381), so sums of two reduced values never carry out of the top limb.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

namespace spx {

// ---------------------------------------------------------------- constants
struct FrCfg {
    static constexpr int N = 8;
    static constexpr uint32_t INV = 0xffffffffu;  // -r^-1 mod 2^32
};
struct FqCfg {
    static constexpr int N = 12;
    static constexpr uint32_t INV = 0xfffcfffdu;  // -q^-1 mod 2^32
};

// r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
__device__ __constant__ constexpr uint32_t kFrP[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                                     0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
__device__ __constant__ constexpr uint32_t kFrOne[8] = {0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau,
                                                       0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u};
__device__ __constant__ constexpr uint32_t kFrR2[8] = {0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu,
                                                      0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u};
// q = 0x1a0111ea...ffffaaab
__device__ __constant__ constexpr uint32_t kFqP[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu,
                                                      0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, 0x64774b84u,
                                                      0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
__device__ __constant__ constexpr uint32_t kFqOne[12] = {0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu,
                                                        0x53c758bau, 0x5f489857u, 0x70525745u, 0x77ce5853u,
                                                        0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u};

template <class C>
struct PCfg;
template <>
struct PCfg<FrCfg> {
    static DEV uint32_t p(int i) { return kFrP[i]; }
    static DEV uint32_t one(int i) { return kFrOne[i]; }
};
template <>
struct PCfg<FqCfg> {
    static DEV uint32_t p(int i) { return kFqP[i]; }
    static DEV uint32_t one(int i) { return kFqOne[i]; }
};

template <class C>
struct Fe {
    uint32_t v[C::N];
};
using Fr = Fe<FrCfg>;
using Fq = Fe<FqCfg>;
struct Fq2 {
    Fq c0, c1;
};

// ---------------------------------------------------------------- primitives
template <class C>
DEV void fe_zero(Fe<C>& r) {
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = 0;
}
template <class C>
DEV void fe_one(Fe<C>& r) {
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = PCfg<C>::one(i);
}
template <class C>
DEV bool fe_is_zero(const Fe<C>& a) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) acc |= a.v[i];
    return acc == 0;
}
template <class C>
DEV bool fe_eq(const Fe<C>& a, const Fe<C>& b) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) acc |= a.v[i] ^ b.v[i];
    return acc == 0;
}

// Carry chains through __builtin_addc / __builtin_subc: one v_add_co/v_addc_co (v_sub_co/v_subb_co)
// per limb. The 64-bit-sum form these replace compiled to 64-bit shifts and adds per limb (~70 VALU
// instructions per Fr addition against ~25).
// r = t - p if t >= p (t < 2p, t has no extra top word)
template <class C>
DEV void fe_reduce_once(Fe<C>& r, const uint32_t (&t)[C::N]) {
    uint32_t d[C::N];
    unsigned br = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) d[i] = __builtin_subc(t[i], PCfg<C>::p(i), br, &br);
    // br == 1 -> t < p -> keep t
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = br ? t[i] : d[i];
}

template <class C>
DEV void fe_add(Fe<C>& r, const Fe<C>& a, const Fe<C>& b) {
    uint32_t t[C::N];
    unsigned c = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) t[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
    fe_reduce_once<C>(r, t);
}

template <class C>
DEV void fe_sub(Fe<C>& r, const Fe<C>& a, const Fe<C>& b) {
    uint32_t t[C::N];
    unsigned br = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) t[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
    const uint32_t mask = 0u - br;
    unsigned c = 0;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __builtin_addc(t[i], PCfg<C>::p(i) & mask, c, &c);
}

template <class C>
DEV void fe_neg(Fe<C>& r, const Fe<C>& a) {
    Fe<C> z;
    fe_zero(z);
    fe_sub(r, z, a);
}

template <class C>
DEV void fe_dbl(Fe<C>& r, const Fe<C>& a) {
    fe_add(r, a, a);
}

// Montgomery multiplication, CIOS, 32-bit limbs (portable form; the asm product-scanning form in
// ff_asm.hpp is the one the kernels use).
template <class C>
DEV void fe_mul_cios(Fe<C>& r, const Fe<C>& a, const Fe<C>& b) {
    constexpr int N = C::N;
    uint32_t t[N + 1];
#pragma unroll
    for (int i = 0; i <= N; ++i) t[i] = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t bi = b.v[i];
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            c = (uint64_t)a.v[j] * bi + t[j] + (c >> 32);
            t[j] = (uint32_t)c;
        }
        uint64_t s = (uint64_t)t[N] + (c >> 32);  // < 2^33 only transiently; top word small
        uint32_t tN = (uint32_t)s;
        uint32_t tN1 = (uint32_t)(s >> 32);
        const uint32_t m = t[0] * C::INV;
        c = (uint64_t)m * PCfg<C>::p(0) + t[0];
#pragma unroll
        for (int j = 1; j < N; ++j) {
            c = (uint64_t)m * PCfg<C>::p(j) + t[j] + (c >> 32);
            t[j - 1] = (uint32_t)c;
        }
        s = (uint64_t)tN + (c >> 32);
        t[N - 1] = (uint32_t)s;
        t[N] = tN1 + (uint32_t)(s >> 32);
    }
    // spare top bits: result < 2p and t[N] == 0
    uint32_t res[N];
#pragma unroll
    for (int i = 0; i < N; ++i) res[i] = t[i];
    fe_reduce_once<C>(r, res);
}

#include "ff_asm.hpp"

template <class C>
DEV void fe_mul(Fe<C>& r, const Fe<C>& a, const Fe<C>& b) {
    if constexpr (C::N == 8)
        fr_mul_asm(r, a, b);
    else
        fq_mul_asm(r, a, b);
}

// two independent Fr products: one instruction stream carrying both multiply-accumulate chains
// (ff_asm.hpp fr_mul_x2_asm). At 8 waves per SIMD one chain already issues at the VALU rate
// (tools/ubench_frmul.hip: 1175 vs 1171 cycles per product); the pair helps where a kernel runs
// fewer waves or stalls on loads (k_col_stream 167 -> 150 us; profiles/r04/r04q_ab.jsonl).
DEV void fr_mul_pair(Fr& r0, const Fr& a0, const Fr& b0, Fr& r1, const Fr& a1, const Fr& b1) {
    fr_mul_x2_asm(r0, a0, b0, r1, a1, b1);
}

template <class C>
DEV void fe_sqr(Fe<C>& r, const Fe<C>& a) {
    fe_mul(r, a, a);
}

// canonical <-> Montgomery
DEV void fr_to_mont(Fr& r, const Fr& canon) {
    Fr r2;
#pragma unroll
    for (int i = 0; i < 8; ++i) r2.v[i] = kFrR2[i];
    fe_mul(r, canon, r2);
}
template <class C>
DEV void fe_from_mont(Fe<C>& r, const Fe<C>& a) {
    Fe<C> one;
    fe_zero(one);
    one.v[0] = 1;
    fe_mul(r, a, one);
}
DEV bool fr_is_canonical(const Fr& a) {  // a < r
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t s = (uint64_t)a.v[i] - kFrP[i] - br;
        br = (uint32_t)(s >> 63);
    }
    return br != 0;
}

// a^e for a small public exponent list (Fermat inversion): e = p - 2
template <class C>
DEV void fe_inv(Fe<C>& r, const Fe<C>& a) {
    constexpr int N = C::N;
    Fe<C> acc;
    fe_one(acc);
    // exponent p - 2 (p odd, low limb >= 3 for both moduli)
#pragma unroll 1
    for (int i = N - 1; i >= 0; --i) {
        uint32_t e = PCfg<C>::p(i) - (i == 0 ? 2u : 0u);
#pragma unroll 1
        for (int b = 31; b >= 0; --b) {
            fe_sqr(acc, acc);
            if ((e >> b) & 1u) fe_mul(acc, acc, a);
        }
    }
    r = acc;
}

// ---------------------------------------------------------------- Fq2
// 32-bit-limb Fq2 (the PP loading / keygen / verifier-side kernels; the MSM hot path uses the
// radix-2^29 lane-pair form of fq2pair.hpp). Each Fq2 product / square is a call with its 3 (2) Fq
// products inline and independent: a fully inlined G2 point addition is ~30 inlined 12-limb products
// (~25k instructions), which overflows the instruction cache.
#define SPX_FQMUL(r, a, b) fe_mul((r), (a), (b))
DEV void f2_zero(Fq2& r) {
    fe_zero(r.c0);
    fe_zero(r.c1);
}
DEV void f2_one(Fq2& r) {
    fe_one(r.c0);
    fe_zero(r.c1);
}
DEV bool f2_is_zero(const Fq2& a) { return fe_is_zero(a.c0) && fe_is_zero(a.c1); }
DEV bool f2_eq(const Fq2& a, const Fq2& b) { return fe_eq(a.c0, b.c0) && fe_eq(a.c1, b.c1); }
DEV void f2_add(Fq2& r, const Fq2& a, const Fq2& b) {
    fe_add(r.c0, a.c0, b.c0);
    fe_add(r.c1, a.c1, b.c1);
}
DEV void f2_sub(Fq2& r, const Fq2& a, const Fq2& b) {
    fe_sub(r.c0, a.c0, b.c0);
    fe_sub(r.c1, a.c1, b.c1);
}
DEV void f2_neg(Fq2& r, const Fq2& a) {
    fe_neg(r.c0, a.c0);
    fe_neg(r.c1, a.c1);
}
DEV void f2_dbl(Fq2& r, const Fq2& a) { f2_add(r, a, a); }
DEV void f2_mul_inl(Fq2& r, const Fq2& a, const Fq2& b) {
    Fq t0, t1, s0, s1, m;
    SPX_FQMUL(t0, a.c0, b.c0);
    SPX_FQMUL(t1, a.c1, b.c1);
    fe_add(s0, a.c0, a.c1);
    fe_add(s1, b.c0, b.c1);
    SPX_FQMUL(m, s0, s1);
    fe_sub(r.c0, t0, t1);
    fe_sub(m, m, t0);
    fe_sub(r.c1, m, t1);
}
DEV void f2_sqr_inl(Fq2& r, const Fq2& a) {
    Fq s, d, p;
    fe_add(s, a.c0, a.c1);
    fe_sub(d, a.c0, a.c1);
    SPX_FQMUL(p, a.c0, a.c1);
    SPX_FQMUL(r.c0, s, d);
    fe_add(r.c1, p, p);
}
static __device__ __noinline__ Fq2 f2_mul_call(Fq2 a, Fq2 b) {
    Fq2 r;
    f2_mul_inl(r, a, b);
    return r;
}
static __device__ __noinline__ Fq2 f2_sqr_call(Fq2 a) {
    Fq2 r;
    f2_sqr_inl(r, a);
    return r;
}
DEV void f2_mul(Fq2& r, const Fq2& a, const Fq2& b) { r = f2_mul_call(a, b); }
DEV void f2_sqr(Fq2& r, const Fq2& a) { r = f2_sqr_call(a); }
DEV void f2_inv(Fq2& r, const Fq2& a) {
    Fq t0, t1, n;
    fe_sqr(t0, a.c0);
    fe_sqr(t1, a.c1);
    fe_add(n, t0, t1);
    fe_inv(n, n);
    fe_mul(r.c0, a.c0, n);
    fe_mul(t1, a.c1, n);
    fe_neg(r.c1, t1);
}

// ---------------------------------------------------------------- generic field ops used by curve code
template <class F>
struct FieldOps;
template <>
struct FieldOps<Fq> {
    static DEV void zero(Fq& r) { fe_zero(r); }
    static DEV void one(Fq& r) { fe_one(r); }
    static DEV bool is_zero(const Fq& a) { return fe_is_zero(a); }
    static DEV bool eq(const Fq& a, const Fq& b) { return fe_eq(a, b); }
    static DEV void add(Fq& r, const Fq& a, const Fq& b) { fe_add(r, a, b); }
    static DEV void sub(Fq& r, const Fq& a, const Fq& b) { fe_sub(r, a, b); }
    static DEV void neg(Fq& r, const Fq& a) { fe_neg(r, a); }
    static DEV void mul(Fq& r, const Fq& a, const Fq& b) { fe_mul(r, a, b); }
    static DEV void sqr(Fq& r, const Fq& a) { fe_sqr(r, a); }
    static DEV void inv(Fq& r, const Fq& a) { fe_inv(r, a); }
};
template <>
struct FieldOps<Fq2> {
    static DEV void zero(Fq2& r) { f2_zero(r); }
    static DEV void one(Fq2& r) { f2_one(r); }
    static DEV bool is_zero(const Fq2& a) { return f2_is_zero(a); }
    static DEV bool eq(const Fq2& a, const Fq2& b) { return f2_eq(a, b); }
    static DEV void add(Fq2& r, const Fq2& a, const Fq2& b) { f2_add(r, a, b); }
    static DEV void sub(Fq2& r, const Fq2& a, const Fq2& b) { f2_sub(r, a, b); }
    static DEV void neg(Fq2& r, const Fq2& a) { f2_neg(r, a); }
    static DEV void mul(Fq2& r, const Fq2& a, const Fq2& b) { f2_mul(r, a, b); }
    static DEV void sqr(Fq2& r, const Fq2& a) { f2_sqr(r, a); }
    static DEV void inv(Fq2& r, const Fq2& a) { f2_inv(r, a); }
};

// ---------------------------------------------------------------- vector memory helpers
template <class T>
DEV void load_vec(T& dst, const T* src) {
    static_assert(sizeof(T) % 16 == 0, "16-byte granules");
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(&dst);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 16); ++i) d[i] = s[i];
}
template <class T>
DEV void store_vec(T* dst, const T& src) {
    static_assert(sizeof(T) % 16 == 0, "16-byte granules");
    uint4* d = reinterpret_cast<uint4*>(dst);
    const uint4* s = reinterpret_cast<const uint4*>(&src);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 16); ++i) d[i] = s[i];
}

// wave64 shuffle of a whole field element
template <class C>
DEV Fe<C> shfl_xor(const Fe<C>& a, int mask) {
    Fe<C> r;
#pragma unroll
    for (int i = 0; i < C::N; ++i) r.v[i] = __shfl_xor(a.v[i], mask, 64);
    return r;
}

}  // namespace spx
