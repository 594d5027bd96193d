// Device elliptic-curve arithmetic for BLS12-381 G1 (over Fq) and G2 (over Fq2).
//
// Bucket accumulation runs in XYZZ ("extended Jacobian": x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2)
// coordinates: mixed add madd-2008-s = 8M + 2S, general add add-2008-s = 12M + 2S, doubling
// dbl-2008-s-1 — the curves have a = 0. Infinity is ZZ == 0. Affine points are stored
// AoS, 16-byte aligned: G1 = 96 B, G2 = 192 B (Montgomery limbs), so one point is one run of
// 16-byte vector loads.
#pragma once
#include "ff_dev.hpp"

namespace spx {

template <class F>
struct Aff {
    F x, y;
};
template <class F>
struct Xyzz {
    F x, y, zz, zzz;
};
using G1Aff = Aff<Fq>;
// A G1 point of the MSM window tables in a 128-byte slot: a 96-byte point at a 96-byte pitch
// straddles two 128-byte lines for two points in three, so every random gather fetched ~2x its bytes
// (profiles/r01_pmc_traffic.json); one slot per line fetches each point with one line.
struct G1Slot {
    G1Aff p;
    uint32_t pad[8];
};
static_assert(sizeof(G1Slot) == 128, "G1 table slot");
using G2Aff = Aff<Fq2>;
using G1Xyzz = Xyzz<Fq>;
using G2Xyzz = Xyzz<Fq2>;

template <class F>
DEV void xyzz_set_inf(Xyzz<F>& p) {
    FieldOps<F>::one(p.x);
    FieldOps<F>::one(p.y);
    FieldOps<F>::zero(p.zz);
    FieldOps<F>::zero(p.zzz);
}
template <class F>
DEV bool xyzz_is_inf(const Xyzz<F>& p) {
    return FieldOps<F>::is_zero(p.zz);
}

// affine doubling into XYZZ (mdbl-2008-s-1)
template <class F>
DEV void xyzz_from_aff_dbl(Xyzz<F>& r, const Aff<F>& a) {
    using O = FieldOps<F>;
    F U, V, W, S, M, t;
    O::add(U, a.y, a.y);
    O::sqr(V, U);
    O::mul(W, U, V);
    O::mul(S, a.x, V);
    O::sqr(M, a.x);
    O::add(t, M, M);
    O::add(M, M, t);
    O::sqr(r.x, M);
    O::sub(r.x, r.x, S);
    O::sub(r.x, r.x, S);
    O::sub(t, S, r.x);
    O::mul(t, M, t);
    O::mul(r.y, W, a.y);
    O::sub(r.y, t, r.y);
    r.zz = V;
    r.zzz = W;
}

// dbl-2008-s-1
template <class F>
DEV void xyzz_dbl(Xyzz<F>& r, const Xyzz<F>& p) {
    using O = FieldOps<F>;
    if (xyzz_is_inf(p)) {
        r = p;
        return;
    }
    F U, V, W, S, M, t;
    O::add(U, p.y, p.y);
    O::sqr(V, U);
    O::mul(W, U, V);
    O::mul(S, p.x, V);
    O::sqr(M, p.x);
    O::add(t, M, M);
    O::add(M, M, t);
    Xyzz<F> o;
    O::sqr(o.x, M);
    O::sub(o.x, o.x, S);
    O::sub(o.x, o.x, S);
    O::sub(t, S, o.x);
    O::mul(t, M, t);
    O::mul(o.y, W, p.y);
    O::sub(o.y, t, o.y);
    O::mul(o.zz, V, p.zz);
    O::mul(o.zzz, W, p.zzz);
    r = o;
}

// p += a (a affine, not infinity); `neg` adds -a. madd-2008-s.
template <class F>
DEV void xyzz_madd(Xyzz<F>& p, const Aff<F>& a, bool neg) {
    using O = FieldOps<F>;
    F ay = a.y;
    if (neg) O::neg(ay, a.y);
    if (xyzz_is_inf(p)) {
        p.x = a.x;
        p.y = ay;
        O::one(p.zz);
        O::one(p.zzz);
        return;
    }
    F U2, S2, P, R, PP, PPP, Q, t;
    O::mul(U2, a.x, p.zz);
    O::mul(S2, ay, p.zzz);
    O::sub(P, U2, p.x);
    O::sub(R, S2, p.y);
    if (O::is_zero(P)) {
        if (O::is_zero(R)) {
            Aff<F> aa{a.x, ay};
            xyzz_from_aff_dbl(p, aa);
        } else {
            xyzz_set_inf(p);
        }
        return;
    }
    O::sqr(PP, P);
    O::mul(PPP, P, PP);
    O::mul(Q, p.x, PP);
    O::sqr(t, R);
    O::sub(t, t, PPP);
    O::sub(t, t, Q);
    F x3;
    O::sub(x3, t, Q);
    O::sub(t, Q, x3);
    O::mul(t, R, t);
    O::mul(S2, p.y, PPP);
    O::sub(p.y, t, S2);
    p.x = x3;
    O::mul(p.zz, p.zz, PP);
    O::mul(p.zzz, p.zzz, PPP);
}

// p += q (both XYZZ). add-2008-s.
template <class F>
DEV void xyzz_add(Xyzz<F>& p, const Xyzz<F>& q) {
    using O = FieldOps<F>;
    if (xyzz_is_inf(q)) return;
    if (xyzz_is_inf(p)) {
        p = q;
        return;
    }
    F U1, U2, S1, S2, P, R, PP, PPP, Q, t;
    O::mul(U1, p.x, q.zz);
    O::mul(U2, q.x, p.zz);
    O::mul(S1, p.y, q.zzz);
    O::mul(S2, q.y, p.zzz);
    O::sub(P, U2, U1);
    O::sub(R, S2, S1);
    if (O::is_zero(P)) {
        if (O::is_zero(R)) {
            xyzz_dbl(p, p);
        } else {
            xyzz_set_inf(p);
        }
        return;
    }
    O::sqr(PP, P);
    O::mul(PPP, P, PP);
    O::mul(Q, U1, PP);
    O::sqr(t, R);
    O::sub(t, t, PPP);
    O::sub(t, t, Q);
    F x3;
    O::sub(x3, t, Q);
    O::sub(t, Q, x3);
    O::mul(t, R, t);
    O::mul(S1, S1, PPP);
    O::sub(p.y, t, S1);
    p.x = x3;
    O::mul(t, p.zz, q.zz);
    O::mul(p.zz, t, PP);
    O::mul(t, p.zzz, q.zzz);
    O::mul(p.zzz, t, PPP);
}

template <class F>
DEV void xyzz_neg(Xyzz<F>& p) {
    FieldOps<F>::neg(p.y, p.y);
}

// small-scalar multiple k * p (k < 2^32), double-and-add MSB first
template <class F>
DEV void xyzz_mul_small(Xyzz<F>& r, const Xyzz<F>& p, uint32_t k) {
    Xyzz<F> acc;
    xyzz_set_inf(acc);
    if (k == 0 || xyzz_is_inf(p)) {
        r = acc;
        return;
    }
    int top = 31 - __clz(k);
#pragma unroll 1
    for (int b = top; b >= 0; --b) {
        xyzz_dbl(acc, acc);
        if ((k >> b) & 1u) xyzz_add(acc, p);
    }
    r = acc;
}

}  // namespace spx
