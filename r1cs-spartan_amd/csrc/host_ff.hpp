// Host-side BLS12-381 arithmetic for the prover's control path: Fiat-Shamir challenge
// handling, sumcheck message assembly (a few Fr ops per round), XYZZ -> affine conversion of
// MSM results, point compression (ark-serialize flags) and public-parameter parsing.
// 64-bit limbs with unsigned __int128, Montgomery form identical to the device's 32-bit limbs.
#pragma once
#include <stdint.h>
#include <string.h>

#include <array>
#include <stdexcept>
#include <vector>

namespace spx {
namespace host {

typedef unsigned __int128 u128;

template <int N>
struct Modulus {
    uint64_t p[N];
    uint64_t r2[N];
    uint64_t one[N];
    uint64_t inv;
};

static constexpr Modulus<4> kFr = {
    {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL},
    {0xc999e990f3f29c6dULL, 0x2b6cedcb87925c23ULL, 0x05d314967254398fULL, 0x0748d9d99f59ff11ULL},
    {0x00000001fffffffeULL, 0x5884b7fa00034802ULL, 0x998c4fefecbc4ff5ULL, 0x1824b159acc5056fULL},
    0xfffffffeffffffffULL};
static constexpr Modulus<6> kFq = {
    {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL, 0x64774b84f38512bfULL,
     0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL},
    {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL, 0x8de5476c4c95b6d5ULL, 0x67eb88a9939d83c0ULL,
     0x9a793e85b519952dULL, 0x11988fe592cae3aaULL},
    {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL, 0x77ce585370525745ULL,
     0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL},
    0x89f3fffcfffcfffdULL};

template <int N, const Modulus<N>& M>
struct Fp {
    uint64_t v[N];

    static Fp zero() {
        Fp r;
        memset(r.v, 0, sizeof r.v);
        return r;
    }
    static Fp one() {
        Fp r;
        memcpy(r.v, M.one, sizeof r.v);
        return r;
    }
    static bool geq_p(const uint64_t* a) {
        for (int i = N - 1; i >= 0; --i)
            if (a[i] != M.p[i]) return a[i] > M.p[i];
        return true;
    }
    static void sub_p(uint64_t* a) {
        uint64_t br = 0;
        for (int i = 0; i < N; ++i) {
            u128 d = (u128)a[i] - M.p[i] - br;
            a[i] = (uint64_t)d;
            br = (uint64_t)(d >> 64) & 1;
        }
    }
    friend Fp operator*(const Fp& a, const Fp& b) {
        uint64_t t[N + 2] = {0};
        for (int i = 0; i < N; ++i) {
            u128 c = 0;
            for (int j = 0; j < N; ++j) {
                c = (u128)a.v[j] * b.v[i] + t[j] + (c >> 64);
                t[j] = (uint64_t)c;
            }
            c = (u128)t[N] + (c >> 64);
            t[N] = (uint64_t)c;
            t[N + 1] = (uint64_t)(c >> 64);
            uint64_t m = t[0] * M.inv;
            c = (u128)m * M.p[0] + t[0];
            for (int j = 1; j < N; ++j) {
                c = (u128)m * M.p[j] + t[j] + (c >> 64);
                t[j - 1] = (uint64_t)c;
            }
            c = (u128)t[N] + (c >> 64);
            t[N - 1] = (uint64_t)c;
            t[N] = t[N + 1] + (uint64_t)(c >> 64);
        }
        if (t[N] || geq_p(t)) sub_p(t);
        Fp r;
        memcpy(r.v, t, sizeof r.v);
        return r;
    }
    friend Fp operator+(const Fp& a, const Fp& b) {
        Fp r;
        uint64_t c = 0;
        for (int i = 0; i < N; ++i) {
            u128 s = (u128)a.v[i] + b.v[i] + c;
            r.v[i] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
        if (c || geq_p(r.v)) sub_p(r.v);
        return r;
    }
    friend Fp operator-(const Fp& a, const Fp& b) {
        Fp r;
        uint64_t br = 0;
        for (int i = 0; i < N; ++i) {
            u128 d = (u128)a.v[i] - b.v[i] - br;
            r.v[i] = (uint64_t)d;
            br = (uint64_t)(d >> 64) & 1;
        }
        if (br) {
            uint64_t c = 0;
            for (int i = 0; i < N; ++i) {
                u128 s = (u128)r.v[i] + M.p[i] + c;
                r.v[i] = (uint64_t)s;
                c = (uint64_t)(s >> 64);
            }
        }
        return r;
    }
    Fp operator-() const { return zero() - *this; }
    Fp& operator+=(const Fp& b) { return *this = *this + b; }
    Fp& operator-=(const Fp& b) { return *this = *this - b; }
    Fp& operator*=(const Fp& b) { return *this = *this * b; }
    bool operator==(const Fp& b) const { return memcmp(v, b.v, sizeof v) == 0; }
    bool operator!=(const Fp& b) const { return !(*this == b); }
    bool is_zero() const {
        uint64_t a = 0;
        for (int i = 0; i < N; ++i) a |= v[i];
        return a == 0;
    }
    static Fp from_canon(const uint64_t* c) {
        Fp a, r2;
        memcpy(a.v, c, sizeof a.v);
        memcpy(r2.v, M.r2, sizeof r2.v);
        return a * r2;
    }
    void to_canon(uint64_t* c) const {
        Fp one_raw = zero();
        one_raw.v[0] = 1;
        Fp r = *this * one_raw;
        memcpy(c, r.v, sizeof r.v);
    }
    static Fp from_u64(uint64_t x) {
        uint64_t c[N] = {0};
        c[0] = x;
        return from_canon(c);
    }
    Fp pow(const uint64_t* e, int ne) const {
        Fp acc = one();
        for (int i = ne - 1; i >= 0; --i)
            for (int b = 63; b >= 0; --b) {
                acc = acc * acc;
                if ((e[i] >> b) & 1) acc = acc * *this;
            }
        return acc;
    }
    Fp inv() const {
        if (is_zero()) throw std::domain_error("inverse of zero");
        uint64_t e[N];
        memcpy(e, M.p, sizeof e);
        e[0] -= 2;
        return pow(e, N);
    }
    // canonical-integer comparison (ark-ff Ord)
    bool canon_gt(const Fp& b) const {
        uint64_t x[N], y[N];
        to_canon(x);
        b.to_canon(y);
        for (int i = N - 1; i >= 0; --i)
            if (x[i] != y[i]) return x[i] > y[i];
        return false;
    }
};

using Fr = Fp<4, kFr>;
using Fq = Fp<6, kFq>;

// ark-serialize Fr: 32-byte LE canonical
inline bool fr_from_bytes(Fr& r, const uint8_t* b) {
    uint64_t c[4];
    memcpy(c, b, 32);
    if (Fr::geq_p(c)) return false;
    r = Fr::from_canon(c);
    return true;
}
inline void fr_to_bytes(uint8_t* b, const Fr& a) {
    uint64_t c[4];
    a.to_canon(c);
    memcpy(b, c, 32);
}

struct Fq2 {
    Fq c0, c1;
    static Fq2 zero() { return {Fq::zero(), Fq::zero()}; }
    static Fq2 one() { return {Fq::one(), Fq::zero()}; }
    friend Fq2 operator+(const Fq2& a, const Fq2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
    friend Fq2 operator-(const Fq2& a, const Fq2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
    Fq2 operator-() const { return {-c0, -c1}; }
    friend Fq2 operator*(const Fq2& a, const Fq2& b) {
        Fq t0 = a.c0 * b.c0, t1 = a.c1 * b.c1;
        Fq m = (a.c0 + a.c1) * (b.c0 + b.c1);
        return {t0 - t1, m - t0 - t1};
    }
    bool operator==(const Fq2& b) const { return c0 == b.c0 && c1 == b.c1; }
    bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
    Fq2 inv() const {
        Fq n = (c0 * c0 + c1 * c1).inv();
        return {c0 * n, -(c1 * n)};
    }
    bool canon_gt(const Fq2& b) const {  // ark-ff Ord: c1 first, then c0
        if (!(c1 == b.c1)) return c1.canon_gt(b.c1);
        return c0.canon_gt(b.c0);
    }
};

// ---------------------------------------------------------------- points
template <class F>
struct Affine {
    F x, y;
    bool inf;
};
template <class F>
struct Jac {
    F x, y, z;
};

template <class F>
inline F curve_b();
template <>
inline Fq curve_b<Fq>() {
    return Fq::from_u64(4);
}
template <>
inline Fq2 curve_b<Fq2>() {
    return {Fq::from_u64(4), Fq::from_u64(4)};
}

template <class F>
inline bool on_curve(const Affine<F>& a) {
    if (a.inf) return true;
    return a.y * a.y == a.x * a.x * a.x + curve_b<F>();
}

template <class F>
inline Jac<F> jac_inf() {
    return {F::one(), F::one(), F::zero()};
}
template <class F>
inline Jac<F> jac_from(const Affine<F>& a) {
    if (a.inf) return jac_inf<F>();
    return {a.x, a.y, F::one()};
}
template <class F>
inline Jac<F> jac_dbl(const Jac<F>& p) {
    if (p.z.is_zero()) return p;
    F A = p.x * p.x, B = p.y * p.y, C = B * B;
    F t = p.x + B;
    F D = t * t - A - C;
    D = D + D;
    F E = A + A + A;
    F Fv = E * E;
    Jac<F> r;
    r.x = Fv - (D + D);
    F C8 = C + C;
    C8 = C8 + C8;
    C8 = C8 + C8;
    r.y = E * (D - r.x) - C8;
    F yz = p.y * p.z;
    r.z = yz + yz;
    return r;
}
template <class F>
inline Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
    if (p.z.is_zero()) return q;
    if (q.z.is_zero()) return p;
    F Z1Z1 = p.z * p.z, Z2Z2 = q.z * q.z;
    F U1 = p.x * Z2Z2, U2 = q.x * Z1Z1;
    F S1 = p.y * q.z * Z2Z2, S2 = q.y * p.z * Z1Z1;
    if (U1 == U2) return S1 == S2 ? jac_dbl(p) : jac_inf<F>();
    F H = U2 - U1;
    F I = (H + H) * (H + H);
    F J = H * I;
    F rr = S2 - S1;
    rr = rr + rr;
    F V = U1 * I;
    Jac<F> o;
    o.x = rr * rr - J - V - V;
    F s1j = S1 * J;
    o.y = rr * (V - o.x) - s1j - s1j;
    F zs = p.z + q.z;
    o.z = (zs * zs - Z1Z1 - Z2Z2) * H;
    return o;
}
template <class F>
inline Affine<F> jac_to_affine(const Jac<F>& p) {
    if (p.z.is_zero()) return {F::zero(), F::one(), true};
    F zi = p.z.inv(), zi2 = zi * zi;
    return {p.x * zi2, p.y * zi2 * zi, false};
}
// canonical 4x64 scalar
template <class F>
inline Jac<F> jac_mul(const Jac<F>& p, const uint64_t* k) {
    Jac<F> acc = jac_inf<F>();
    for (int i = 3; i >= 0; --i)
        for (int b = 63; b >= 0; --b) {
            acc = jac_dbl(acc);
            if ((k[i] >> b) & 1) acc = jac_add(acc, p);
        }
    return acc;
}

// XYZZ (device MSM output) -> affine: x = X/ZZ, y = Y/ZZZ
template <class F>
inline Affine<F> xyzz_to_affine(const F& X, const F& Y, const F& ZZ, const F& ZZZ) {
    if (ZZ.is_zero()) return {F::zero(), F::one(), true};
    F i = (ZZ * ZZZ).inv();
    F izz = i * ZZZ, izzz = i * ZZ;
    return {X * izz, Y * izzz, false};
}

// ---------------------------------------------------------------- ark-serialize of points
static const uint8_t kFlagInf = 0x40, kFlagPosY = 0x80;
inline void fq_to_bytes(uint8_t* out48, const Fq& x, uint8_t flags = 0) {
    uint64_t c[6];
    x.to_canon(c);
    memcpy(out48, c, 48);
    out48[47] |= flags;
}
inline bool fq_from_bytes(Fq& r, const uint8_t* b, uint8_t* flags) {
    uint64_t c[6];
    memcpy(c, b, 48);
    if (flags) *flags = (uint8_t)(c[5] >> 56) & 0xC0;
    c[5] &= 0x3FFFFFFFFFFFFFFFULL;
    if (Fq::geq_p(c)) return false;
    r = Fq::from_canon(c);
    return true;
}
inline void g1_compress(uint8_t* out48, const Affine<Fq>& a) {
    if (a.inf) return fq_to_bytes(out48, Fq::zero(), kFlagInf);
    fq_to_bytes(out48, a.x, a.y.canon_gt(-a.y) ? kFlagPosY : 0);
}
inline void g2_compress(uint8_t* out96, const Affine<Fq2>& a) {
    if (a.inf) {
        fq_to_bytes(out96, Fq::zero());
        fq_to_bytes(out96 + 48, Fq::zero(), kFlagInf);
        return;
    }
    fq_to_bytes(out96, a.x.c0);
    fq_to_bytes(out96 + 48, a.x.c1, a.y.canon_gt(-a.y) ? kFlagPosY : 0);
}
inline bool g1_from_uncompressed(Affine<Fq>& a, const uint8_t* b) {
    uint8_t f = 0;
    if (!fq_from_bytes(a.x, b, nullptr) || !fq_from_bytes(a.y, b + 48, &f)) return false;
    a.inf = (f & kFlagInf) != 0;
    return true;
}
inline bool g2_from_uncompressed(Affine<Fq2>& a, const uint8_t* b) {
    uint8_t f = 0;
    if (!fq_from_bytes(a.x.c0, b, nullptr) || !fq_from_bytes(a.x.c1, b + 48, nullptr) ||
        !fq_from_bytes(a.y.c0, b + 96, nullptr) || !fq_from_bytes(a.y.c1, b + 144, &f))
        return false;
    a.inf = (f & kFlagInf) != 0;
    return true;
}
inline void g1_to_uncompressed(uint8_t* b, const Affine<Fq>& a) {
    if (a.inf) {
        fq_to_bytes(b, Fq::zero());
        fq_to_bytes(b + 48, Fq::one(), kFlagInf);
        return;
    }
    fq_to_bytes(b, a.x);
    fq_to_bytes(b + 48, a.y);
}
inline void g2_to_uncompressed(uint8_t* b, const Affine<Fq2>& a) {
    if (a.inf) {
        fq_to_bytes(b, Fq::zero());
        fq_to_bytes(b + 48, Fq::zero());
        fq_to_bytes(b + 96, Fq::one());
        fq_to_bytes(b + 144, Fq::zero(), kFlagInf);
        return;
    }
    fq_to_bytes(b, a.x.c0);
    fq_to_bytes(b + 48, a.x.c1);
    fq_to_bytes(b + 96, a.y.c0);
    fq_to_bytes(b + 144, a.y.c1);
}

// generators (affine, Montgomery)
inline Affine<Fq> g1_generator() {
    static const uint64_t X[6] = {0x5cb38790fd530c16ULL, 0x7817fc679976fff5ULL, 0x154f95c7143ba1c1ULL,
                                  0xf0ae6acdf3d0e747ULL, 0xedce6ecc21dbf440ULL, 0x120177419e0bfb75ULL};
    static const uint64_t Y[6] = {0xbaac93d50ce72271ULL, 0x8c22631a7918fd8eULL, 0xdd595f13570725ceULL,
                                  0x51ac582950405194ULL, 0x0e1c8c3fad0059c0ULL, 0x0bbc3efc5008a26aULL};
    Affine<Fq> a;
    memcpy(a.x.v, X, 48);
    memcpy(a.y.v, Y, 48);
    a.inf = false;
    return a;
}
inline Affine<Fq2> g2_generator() {
    static const uint64_t X0[6] = {0xf5f28fa202940a10ULL, 0xb3f5fb2687b4961aULL, 0xa1a893b53e2ae580ULL,
                                   0x9894999d1a3caee9ULL, 0x6f67b7631863366bULL, 0x058191924350bcd7ULL};
    static const uint64_t X1[6] = {0xa5a9c0759e23f606ULL, 0xaaa0c59dbccd60c3ULL, 0x3bb17e18e2867806ULL,
                                   0x1b1ab6cc8541b367ULL, 0xc2b6ed0ef2158547ULL, 0x11922a097360edf3ULL};
    static const uint64_t Y0[6] = {0x4c730af860494c4aULL, 0x597cfa1f5e369c5aULL, 0xe7e6856caa0a635aULL,
                                   0xbbefb5e96e0d495fULL, 0x07d3a975f0ef25a2ULL, 0x0083fd8e7e80dae5ULL};
    static const uint64_t Y1[6] = {0xadc0fc92df64b05dULL, 0x18aa270a2b1461dcULL, 0x86adac6a3be4eba0ULL,
                                   0x79495c4ec93da33aULL, 0xe7175850a43ccaedULL, 0x0b2bc2a163de1bf2ULL};
    Affine<Fq2> a;
    memcpy(a.x.c0.v, X0, 48);
    memcpy(a.x.c1.v, X1, 48);
    memcpy(a.y.c0.v, Y0, 48);
    memcpy(a.y.c1.v, Y1, 48);
    a.inf = false;
    return a;
}

// batch inversion (Montgomery's trick); zeros stay zero
template <class F>
inline void batch_inverse(std::vector<F>& xs) {
    std::vector<F> pre(xs.size());
    F acc = F::one();
    for (size_t i = 0; i < xs.size(); ++i) {
        pre[i] = acc;
        if (!xs[i].is_zero()) acc = acc * xs[i];
    }
    F inv = acc.inv();
    for (size_t k = xs.size(); k-- > 0;) {
        if (xs[k].is_zero()) continue;
        F xi = inv * pre[k];
        inv = inv * xs[k];
        xs[k] = xi;
    }
}

}  // namespace host
}  // namespace spx
