// Fq2 = Fq[u] / (u^2 + 1) held by a PAIR of adjacent lanes: the even lane holds c0, the odd lane c1,
// each as one radix-2^29 Fq value (ff29.hpp). The G2 MSM kernels run one curve element per lane
// pair, so every lane carries half of a G2 point's state: the accumulation fits 256 registers and
// two waves share each SIMD. That is the point: a lone wave issues a v_mad_u64_u32 only every
// ~9 cycles, two waves per SIMD every ~5.2 (tools/ubench_issue.hip, profiles/r02_ubench_issue.txt),
// and the Fq2 products are where the limb products are.
//
// Products exchange operands with the partner lane through DPP (quad_perm [1,0,3,2]: lane i reads
// lane i^1), 14 moves per operand:
//   c0 = REDC(a0 b0 + a1 (8p - b1))     even lane: REDC(a b + a' (8p - b'))
//   c1 = REDC(a0 b1 + a1 b0)            odd lane:  REDC(a b' + a' b)
// (x' = the partner's value), i.e. REDC(a y1 + a' y2) with (y1, y2) = (b, 8p - b') on the even lane
// and (b', b) on the odd one: one fused two-product reduction per lane instead of two per element.
// Squares: c0 = (a0 + a1)(a0 - a1), c1 = 2 a0 a1: one product per lane.
// Every predicate (zero / infinity tests) is combined over the pair, so both lanes of a pair always
// take the same branch; a kernel must keep both lanes of every pair active together.
// Value bounds are those of ff29.hpp / curve29.hpp, per coefficient.
#pragma once
#include "ff29.hpp"

namespace spx {

struct FP29 {
    F29 v;  // this lane's coefficient: c0 on even lanes, c1 on odd lanes
};

DEV bool pair_odd() { return (__lane_id() & 1) != 0; }
DEV uint32_t pair_swap(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
DEV F29 pair_swap(const F29& a) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 14; ++i) r.v[i] = pair_swap(a.v[i]);
    return r;
}
DEV bool pair_all(bool b) {  // b on both lanes of the pair
    const uint32_t x = b ? 1u : 0u;
    return (x & pair_swap(x)) != 0;
}
DEV F29 f29_select(bool c, const F29& a, const F29& b) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 14; ++i) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}

template <>
struct Ops29<FP29> {
    // operands up to 8p per coefficient (the partner's b enters as 8p - b')
    static DEV void mul(FP29& r, const FP29& a, const FP29& b) {
        const bool odd = pair_odd();
        const F29 ap = pair_swap(a.v), bp = pair_swap(b.v);
        F29 z, nbp;
        f29_zero(z);
        f29_sub<8>(nbp, z, bp);
        const F29 y1 = f29_select(odd, bp, b.v);
        const F29 y2 = f29_select(odd, b.v, nbp);
        f29_mul2(r.v, a.v, y1, ap, y2);
    }
    // (a0 + a1)(a0 - a1 + KB p) on the even lane, (a0 + a0) a1 on the odd one; KB bounds c1
    template <int KB>
    static DEV void sqr_b(FP29& r, const FP29& a) {
        const bool odd = pair_odd();
        const F29 ap = pair_swap(a.v);
        F29 s, d, x, y;
        f29_add(s, a.v, ap);          // even: a0 + a1
        f29_sub<KB>(d, a.v, ap);      // even: a0 - a1 + KB p
        f29_add(x, ap, ap);           // odd: 2 a0
        y = f29_select(odd, a.v, d);  // odd: a1
        x = f29_select(odd, x, s);
        f29_mul(r.v, x, y);
    }
    static DEV void sqr(FP29& r, const FP29& a) { sqr_b<8>(r, a); }
    static DEV void add(FP29& r, const FP29& a, const FP29& b) { f29_add(r.v, a.v, b.v); }
    template <int K>
    static DEV void sub(FP29& r, const FP29& a, const FP29& b) {
        f29_sub<K>(r.v, a.v, b.v);
    }
    template <int K>
    static DEV void reduce(FP29& x) {
        f29_reduce<K>(x.v);
    }
    static DEV bool zero2(const FP29& x) { return pair_all(f29_zero2(x.v)); }
    static DEV bool zero4(const FP29& x) { return pair_all(f29_zero4(x.v)); }
    template <int K>
    static DEV bool zero_lt(const FP29& x) {
        return pair_all(f29_zero_lt<K>(x.v));
    }
    static DEV bool is_zero_raw(const FP29& x) { return pair_all(f29_is_zero_raw(x.v)); }
    static DEV void zero(FP29& r) { f29_zero(r.v); }
    static DEV void one(FP29& r) {
        if (pair_odd())
            f29_zero(r.v);
        else
            f29_one(r.v);
    }
};

// ---- storage: the lane's half of a packed (12 x 32-bit words per Fq) Fq2 coordinate
DEV void fp29_unpack(FP29& r, const Fq2& s) { f29_unpack(r.v, pair_odd() ? s.c1.v : s.c0.v); }
// ld / st of one lane's coefficient of coordinate k of a point at p (Fq2 coordinates, c0 then c1)
DEV void fp29_ld(FP29& r, const Fq2* coord) {
    Fq w;
    load_vec(w, pair_odd() ? &coord->c1 : &coord->c0);
    f29_unpack(r.v, w.v);
}
DEV void fp29_st(Fq2* coord, const FP29& r) {
    Fq w;
    f29_pack(w.v, r.v);
    store_vec(pair_odd() ? &coord->c1 : &coord->c0, w);
}

}  // namespace spx
