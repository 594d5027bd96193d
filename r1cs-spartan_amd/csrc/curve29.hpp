// XYZZ point arithmetic over the radix-2^29 field (ff29.hpp) for the MSM hot kernels, with the
// value bounds of every intermediate (multiples of p) written next to it. Inputs and outputs of
// every formula are "reduced": each coordinate < 2p. Infinity is ZZ == 0 as a literal (every
// path that produces it sets it explicitly). Storage stays the 12 x 32-bit layout of curve_dev.hpp
// (Aff<Fq> / Xyzz<Fq2> ...): values there are in the R = 2^406 domain, < 2p, packed.
#pragma once
#include "curve_dev.hpp"
#include "ff29.hpp"

namespace spx {

template <class S>
struct R29;
template <>
struct R29<Fq> {
    using T = F29;
    static DEV void unpack(F29& r, const Fq& s) { f29_unpack(r, s.v); }
    static DEV void pack(Fq& s, const F29& r) { f29_pack(s.v, r); }
};
template <>
struct R29<Fq2> {
    using T = F2_29;
    static DEV void unpack(F2_29& r, const Fq2& s) {
        f29_unpack(r.c0, s.c0.v);
        f29_unpack(r.c1, s.c1.v);
    }
    static DEV void pack(Fq2& s, const F2_29& r) {
        f29_pack(s.c0.v, r.c0);
        f29_pack(s.c1.v, r.c1);
    }
};

template <class F>
struct A29 {
    F x, y;
};
template <class F>
struct X29 {
    F x, y, zz, zzz;
};

template <class S>
DEV void ld29(A29<typename R29<S>::T>& r, const Aff<S>* p) {
    Aff<S> a;
    load_vec(a, p);
    R29<S>::unpack(r.x, a.x);
    R29<S>::unpack(r.y, a.y);
}
template <class S>
DEV void ld29(X29<typename R29<S>::T>& r, const Xyzz<S>* p) {
    Xyzz<S> a;
    load_vec(a, p);
    R29<S>::unpack(r.x, a.x);
    R29<S>::unpack(r.y, a.y);
    R29<S>::unpack(r.zz, a.zz);
    R29<S>::unpack(r.zzz, a.zzz);
}
template <class S>
DEV void st29(Xyzz<S>* p, const X29<typename R29<S>::T>& r) {
    Xyzz<S> a;
    R29<S>::pack(a.x, r.x);
    R29<S>::pack(a.y, r.y);
    R29<S>::pack(a.zz, r.zz);
    R29<S>::pack(a.zzz, r.zzz);
    store_vec(p, a);
}

template <class F>
DEV void x29_set_inf(X29<F>& p) {
    using O = Ops29<F>;
    O::one(p.x);
    O::one(p.y);
    O::zero(p.zz);
    O::zero(p.zzz);
}
template <class F>
DEV bool x29_is_inf(const X29<F>& p) {
    return Ops29<F>::is_zero_raw(p.zz);
}

// 2 (x, y) into XYZZ (mdbl-2008-s-1); x, y < 2p
template <class F>
DEV void x29_from_aff_dbl(X29<F>& r, const F& ax, const F& ay) {
    using O = Ops29<F>;
    F U, V, W, S, X2, M, t, s2;
    O::add(U, ay, ay);     // < 4p
    O::sqr(V, U);          // < 2p
    O::mul(W, U, V);       // < 2p
    O::mul(S, ax, V);      // < 2p
    O::sqr(X2, ax);        // < 2p
    O::add(M, X2, X2);     // < 4p
    O::add(M, M, X2);      // < 6p
    O::sqr(t, M);          // < 2p
    O::add(s2, S, S);      // < 4p
    O::template sub<4>(r.x, t, s2);  // < 6p
    O::template reduce<8>(r.x);      // < 2p
    O::template sub<2>(t, S, r.x);  // < 4p
    if constexpr (O::kFusedSum) {   // M t + (2p - W) ay in one reduction, < 2p
        O::zero(s2);
        O::template sub<2>(s2, s2, W);
        O::mul_sum(r.y, M, t, s2, ay);
    } else {
        O::mul(t, M, t);                 // < 2p
        O::mul(s2, W, ay);               // < 2p
        O::template sub<2>(r.y, t, s2);  // < 4p
        O::template reduce<4>(r.y);
    }
    r.zz = V;
    r.zzz = W;
}

// dbl-2008-s-1
template <class F>
DEV void x29_dbl(X29<F>& p) {
    using O = Ops29<F>;
    if (x29_is_inf(p)) return;
    F U, V, W, S, X2, M, t, s2;
    O::add(U, p.y, p.y);
    O::sqr(V, U);
    O::mul(W, U, V);
    O::mul(S, p.x, V);
    O::sqr(X2, p.x);
    O::add(M, X2, X2);
    O::add(M, M, X2);  // < 6p
    O::sqr(t, M);
    O::add(s2, S, S);
    F x3;
    O::template sub<4>(x3, t, s2);
    O::template reduce<8>(x3);
    O::template sub<2>(t, S, x3);
    if constexpr (O::kFusedSum) {  // M t + (2p - W) Y in one reduction, < 2p
        O::zero(s2);
        O::template sub<2>(s2, s2, W);
        O::mul_sum(p.y, M, t, s2, p.y);
    } else {
        O::mul(t, M, t);
        O::mul(s2, W, p.y);
        O::template sub<2>(p.y, t, s2);
        O::template reduce<4>(p.y);
    }
    p.x = x3;
    O::mul(p.zz, V, p.zz);
    O::mul(p.zzz, W, p.zzz);
}

// p += (ax, ay) or (ax, -ay); affine coordinates canonical (< p). madd-2008-s.
// The accumulator of this chain is kept "loose": X < 8p, Y < 4p (ZZ, ZZZ < 2p as products), so the
// exits skip the conditional subtractions; every other formula and the packed storage (8p < 2^384)
// accept loose inputs, because they use X and Y only as product operands (x29_add, x29_dbl:
// 2Y < 8p) or map them through a product (k_tree_out).
template <class F>
DEV void x29_madd(X29<F>& p, const F& ax, const F& ay_in, bool neg) {
    using O = Ops29<F>;
    F ay = ay_in;
    if (neg) {
        F z;
        O::zero(z);
        O::template sub<2>(ay, z, ay_in);  // 2p - y < 2p
    }
    if (x29_is_inf(p)) {
        p.x = ax;
        p.y = ay;
        O::one(p.zz);
        O::one(p.zzz);
        return;
    }
    F U2, S2, P, R;
    O::mul(U2, ax, p.zz);
    O::mul(S2, ay, p.zzz);
    O::template sub<8>(P, U2, p.x);  // < 10p
    O::template sub<4>(R, S2, p.y);  // < 6p
    if (O::template zero_lt<16>(P)) {
        if (O::template zero_lt<8>(R))
            x29_from_aff_dbl(p, ax, ay);
        else
            x29_set_inf(p);
        return;
    }
    F PP, PPP, Q, t, w;
    O::template sqr_b<16>(PP, P);    // P.c1 < 10p
    O::mul(PPP, P, PP);
    O::mul(Q, p.x, PP);
    O::sqr(t, R);                    // R.c1 < 6p
    O::template sub<2>(w, t, PPP);   // < 4p
    O::add(t, Q, Q);                 // < 4p
    O::template sub<4>(w, w, t);     // X3 < 8p (loose)
    O::template sub<8>(t, Q, w);     // < 10p
    // Y3 = t R - Y1 PPP = t R + (4p - Y1) PPP in one reduction where the field form allows it
    // (mul_sum: < 2p fused, < 4p otherwise); R's and PPP's c1 stay < 8p as the products require
    O::zero(S2);
    O::template sub<4>(S2, S2, p.y);  // 4p - Y1 (Y1 < 4p), < 4p
    O::mul_sum(p.y, t, R, S2, PPP);   // Y3 < 4p (loose)
    p.x = w;
    O::mul(p.zz, p.zz, PP);
    O::mul(p.zzz, p.zzz, PPP);
}

// p += q, add-2008-s
template <class F>
DEV void x29_add(X29<F>& p, const X29<F>& q) {
    using O = Ops29<F>;
    if (x29_is_inf(q)) return;
    if (x29_is_inf(p)) {
        p = q;
        return;
    }
    F U1, U2, S1, S2, P, R;
    O::mul(U1, p.x, q.zz);
    O::mul(U2, q.x, p.zz);
    O::mul(S1, p.y, q.zzz);
    O::mul(S2, q.y, p.zzz);
    O::template sub<2>(P, U2, U1);
    O::template sub<2>(R, S2, S1);
    if (O::template zero_lt<4>(P)) {
        if (O::template zero_lt<4>(R))
            x29_dbl(p);
        else
            x29_set_inf(p);
        return;
    }
    F PP, PPP, Q, t, w;
    O::sqr(PP, P);
    O::mul(PPP, P, PP);
    O::mul(Q, U1, PP);
    O::sqr(t, R);
    O::template sub<2>(w, t, PPP);
    O::add(t, Q, Q);
    O::template sub<4>(w, w, t);
    O::template reduce<8>(w);
    O::template sub<2>(t, Q, w);
    if constexpr (O::kFusedSum) {  // R t + (2p - S1) PPP in one reduction, < 2p
        F n;
        O::zero(n);
        O::template sub<2>(n, n, S1);
        O::mul_sum(p.y, R, t, n, PPP);
    } else {
        O::mul(t, R, t);
        O::mul(S1, S1, PPP);
        O::template sub<2>(p.y, t, S1);
        O::template reduce<4>(p.y);
    }
    p.x = w;
    O::mul(t, p.zz, q.zz);
    O::mul(p.zz, t, PP);
    O::mul(t, p.zzz, q.zzz);
    O::mul(p.zzz, t, PPP);
}

// domain conversions for one coordinate (storage words in and out)
template <class F>
DEV void f29_map(F& r, const F& x, const uint32_t (&c)[14]);
template <>
DEV void f29_map<F29>(F29& r, const F29& x, const uint32_t (&c)[14]) {
    F29 k;
    f29_set(k, c);
    f29_mul(r, x, k);
    f29_canon(r);
}
template <>
DEV void f29_map<F2_29>(F2_29& r, const F2_29& x, const uint32_t (&c)[14]) {
    f29_map<F29>(r.c0, x.c0, c);
    f29_map<F29>(r.c1, x.c1, c);
}

}  // namespace spx
