// Host-side BLS12-381 pairing for the verifier's two mKZG checks (verify.rs:12-45,
// E::product_of_pairings [upstream ark-bls12-381]) and point decompression for proof parsing.
//
// Off the prover's hot path (the verifier is a host acceptance check; its O(nnz)
// part, eval_on_x, runs on the GPU). Representation chosen for simplicity over speed:
//   Fq12 = Fq[w] / (w^12 - 2 w^6 + 2), Fq2 embedded by u -> w^6 - 1, the sextic twist point
//   (x, y) of y^2 = x^3 + 4(u+1) maps to (x / w^2, y / w^3).
// Miller loop over |x| = 0xd201000000010000, run simultaneously for all pairs of a product (one
// Fq12 squaring per step, one batch inversion of the affine-step denominators per step), lines
// scaled by w^3 (killed by the final exponentiation), and one final exponentiation by
// (q^12 - 1) / r (pairing_consts.hpp). Ignoring the sign of x gives the inverse of the optimal-ate
// value: still bilinear and non-degenerate, which is all a product-equals-one check needs.
#pragma once
#include <utility>
#include <vector>

#include "host_ff.hpp"
#include "pairing_consts.hpp"

namespace spx {
namespace host {

struct Fq12 {
    Fq c[12];
};
inline Fq12 f12_one() {
    Fq12 r;
    for (auto& x : r.c) x = Fq::zero();
    r.c[0] = Fq::one();
    return r;
}
inline bool f12_is_one(const Fq12& a) {
    if (!(a.c[0] == Fq::one())) return false;
    for (int i = 1; i < 12; ++i)
        if (!a.c[i].is_zero()) return false;
    return true;
}
// zero coefficients of `a` are skipped (sparse line values go first)
inline Fq12 f12_mul(const Fq12& a, const Fq12& b) {
    Fq t[23];
    for (auto& x : t) x = Fq::zero();
    for (int i = 0; i < 12; ++i) {
        if (a.c[i].is_zero()) continue;
        for (int j = 0; j < 12; ++j) t[i + j] += a.c[i] * b.c[j];
    }
    for (int k = 22; k >= 12; --k) {  // w^12 = 2 w^6 - 2
        if (t[k].is_zero()) continue;
        const Fq d = t[k] + t[k];
        t[k - 6] += d;
        t[k - 12] -= d;
    }
    Fq12 r;
    for (int i = 0; i < 12; ++i) r.c[i] = t[i];
    return r;
}
inline Fq12 f12_pow(const Fq12& a, const uint64_t* e, int ne) {
    Fq12 tab[16];  // fixed 4-bit window
    tab[0] = f12_one();
    for (int i = 1; i < 16; ++i) tab[i] = f12_mul(tab[i - 1], a);
    Fq12 acc = f12_one();
    bool started = false;
    for (int i = ne - 1; i >= 0; --i)
        for (int nib = 15; nib >= 0; --nib) {
            if (started)
                for (int s = 0; s < 4; ++s) acc = f12_mul(acc, acc);
            const unsigned d = (unsigned)(e[i] >> (4 * nib)) & 15u;
            if (d) {
                acc = started ? f12_mul(acc, tab[d]) : tab[d];
                started = true;
            }
        }
    return acc;
}
inline Fq12 final_exp(const Fq12& f) { return f12_pow(f, kFinalExp, kFinalExpLimbs); }

// w^3 * [slope (xP - X1) - (yP - Y1)], slope = l w^-1, T1 = (x1 w^-2, y1 w^-3)
inline Fq12 line_value(const Fq2& l, const Fq2& x1, const Fq2& y1, const Affine<Fq>& P) {
    const Fq2 m = l * x1;
    Fq12 c;
    for (auto& x : c.c) x = Fq::zero();
    c.c[0] = (y1.c0 - y1.c1) - (m.c0 - m.c1);
    c.c[6] = y1.c1 - m.c1;
    c.c[2] = (l.c0 - l.c1) * P.x;
    c.c[8] = l.c1 * P.x;
    c.c[3] = -P.y;
    return c;
}

inline Fq2 f2_small(uint64_t k) { return {Fq::from_u64(k), Fq::zero()}; }

// prod_j e(P_j, Q_j) before the final exponentiation (pairs with an infinite point contribute 1)
inline Fq12 miller_loop_multi(const std::vector<std::pair<Affine<Fq>, Affine<Fq2>>>& pairs) {
    std::vector<Affine<Fq>> P;
    std::vector<Affine<Fq2>> Qs, T;
    for (auto& pq : pairs)
        if (!pq.first.inf && !pq.second.inf) {
            P.push_back(pq.first);
            Qs.push_back(pq.second);
        }
    T = Qs;
    const size_t k = P.size();
    const uint64_t ate = 0xd201000000010000ULL;
    Fq12 f = f12_one();
    std::vector<Fq2> den(k);
    const Fq2 three = f2_small(3);
    for (int i = 62; i >= 0; --i) {
        f = f12_mul(f, f);
        for (size_t j = 0; j < k; ++j) den[j] = T[j].y + T[j].y;
        batch_inverse(den);
        for (size_t j = 0; j < k; ++j) {
            const Fq2 x1 = T[j].x, y1 = T[j].y;
            const Fq2 lam = three * (x1 * x1) * den[j];
            f = f12_mul(line_value(lam, x1, y1, P[j]), f);
            const Fq2 x3 = lam * lam - (x1 + x1);
            T[j].y = lam * (x1 - x3) - y1;
            T[j].x = x3;
        }
        if ((ate >> i) & 1) {
            for (size_t j = 0; j < k; ++j) {
                den[j] = Qs[j].x - T[j].x;
                if (den[j].is_zero()) throw std::runtime_error("pairing: degenerate addition step");
            }
            batch_inverse(den);
            for (size_t j = 0; j < k; ++j) {
                const Fq2 x1 = T[j].x, y1 = T[j].y;
                const Fq2 lam = (Qs[j].y - y1) * den[j];
                f = f12_mul(line_value(lam, x1, y1, P[j]), f);
                const Fq2 x3 = lam * lam - x1 - Qs[j].x;
                T[j].y = lam * (x1 - x3) - y1;
                T[j].x = x3;
            }
        }
    }
    return f;
}
inline bool pairing_product_is_one(const std::vector<std::pair<Affine<Fq>, Affine<Fq2>>>& pairs) {
    return f12_is_one(final_exp(miller_loop_multi(pairs)));
}

// ---------------------------------------------------------------- decompression (ark-serialize flags)
inline void p_shifted(uint64_t* e, int shift, uint64_t add) {  // e = (p >> shift) + add
    for (int i = 0; i < 6; ++i) e[i] = (kFq.p[i] >> shift) | (i + 1 < 6 ? kFq.p[i + 1] << (64 - shift) : 0);
    for (int i = 0; i < 6 && add; ++i) {
        const uint64_t s = e[i] + add;
        add = s < e[i] ? 1 : 0;
        e[i] = s;
    }
}
inline Fq2 f2_pow(const Fq2& a, const uint64_t* e, int ne) {
    Fq2 acc = Fq2::one();
    for (int i = ne - 1; i >= 0; --i)
        for (int b = 63; b >= 0; --b) {
            acc = acc * acc;
            if ((e[i] >> b) & 1) acc = acc * a;
        }
    return acc;
}
inline bool fq_sqrt(const Fq& a, Fq& r) {  // q = 3 mod 4
    uint64_t e[6];
    p_shifted(e, 2, 1);  // (q + 1) / 4
    r = a.pow(e, 6);
    return r * r == a;
}
// Algorithm 9 of "Square root computation over even extension fields" (q = 3 mod 4)
inline bool f2_sqrt(const Fq2& a, Fq2& r) {
    uint64_t e1[6], e2[6];
    p_shifted(e1, 2, 0);  // (q - 3) / 4
    p_shifted(e2, 1, 0);  // (q - 1) / 2
    const Fq2 a1 = f2_pow(a, e1, 6);
    const Fq2 alpha = a1 * a1 * a;
    const Fq2 x0 = a1 * a;
    Fq2 x;
    if (alpha == Fq2{-Fq::one(), Fq::zero()})
        x = {-x0.c1, x0.c0};
    else
        x = f2_pow(Fq2::one() + alpha, e2, 6) * x0;
    r = x;
    return x * x == a;
}
inline bool g1_decompress(Affine<Fq>& a, const uint8_t* b48) {
    uint8_t f = 0;
    if (!fq_from_bytes(a.x, b48, &f)) return false;
    a.inf = (f & kFlagInf) != 0;
    if (a.inf) return true;
    Fq y;
    if (!fq_sqrt(a.x * a.x * a.x + curve_b<Fq>(), y)) return false;
    if (y.canon_gt(-y) != ((f & kFlagPosY) != 0)) y = -y;
    a.y = y;
    return true;
}
inline bool g2_decompress(Affine<Fq2>& a, const uint8_t* b96) {
    uint8_t f = 0;
    if (!fq_from_bytes(a.x.c0, b96, nullptr) || !fq_from_bytes(a.x.c1, b96 + 48, &f)) return false;
    a.inf = (f & kFlagInf) != 0;
    if (a.inf) return true;
    Fq2 y;
    if (!f2_sqrt(a.x * a.x * a.x + curve_b<Fq2>(), y)) return false;
    if (y.canon_gt(-y) != ((f & kFlagPosY) != 0)) y = -y;
    a.y = y;
    return true;
}

}  // namespace host
}  // namespace spx
