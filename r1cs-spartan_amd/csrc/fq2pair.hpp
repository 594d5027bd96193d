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

// b0 (the even lane's value) on both lanes of the pair: quad_perm [0,0,2,2]
DEV uint32_t pair_even(uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xA0, 0xF, 0xF, false); }
// b1 (the odd lane's value) on both lanes: quad_perm [1,1,3,3]
DEV uint32_t pair_odd_val(uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xF5, 0xF, 0xF, false); }

// 16p with every limb but the top raised by 2^29 (borrowed from the next limb): k_i - z_i is then
// non-negative and < 2^30 for every normalized z < 8p, so 16p - z needs no borrow chain
DEV constexpr uint32_t k16(int i) {
    return i == 0 ? Q29::P16[0] + (1u << 29) : i < 13 ? Q29::P16[i] + (1u << 29) - 1u : Q29::P16[13] - 1u;
}

// Two forms of the lane pair, identical in value and layout, differing only in how a product
// prepares the partner's operand:
//   FP29  (weighting and partial levels): y2 = 8p - b' by a borrow-chain subtraction;
//   FP29A (the bucket accumulation, k_accum_aff): y1 and b1 come straight from DPP quad-permutes and
//         y2 = 16p - b1 from the borrow-free k16 form (non-normalized limbs < 2^30). Columns stay below
//         2^64: 14 products < 2^58 (a y1) + 14 < 2^59 (a' y2) + 14 m p < 2^58 = 56 x 2^58; the REDC
//         input a0 b0 + a1 (16p - b1) < 192 p^2 < 2^406 p, so the result is < 2p as before.
// FP29A is 3% faster in the accumulation (profiles/r02_ab9_xad.jsonl); in the weighting kernels,
// which already spill at 256 registers, it spills more and is slower, so they keep FP29.
struct FP29A {
    F29 v;
};

template <class P, bool kBorrowFree>
struct PairOps {
    static constexpr bool kFusedSum = kBorrowFree;
    static DEV void mul(P& r, const P& a, const P& b) {
        const bool odd = pair_odd();
        if constexpr (kBorrowFree) {
            const uint32_t msk = odd ? 0u : 0xffffffffu;
            F29 ap, y1, y2;
#pragma unroll
            for (int i = 0; i < 14; ++i) {
                ap.v[i] = pair_swap(a.v.v[i]);
                y1.v[i] = pair_even(b.v.v[i]);
                const uint32_t z = pair_odd_val(b.v.v[i]);
                y2.v[i] = (z ^ msk) + (msk & (k16(i) + 1u));  // even: k_i - z_i; odd: z_i
            }
            f29_mul2(r.v, a.v, y1, ap, y2);
        } else {
            const F29 ap = pair_swap(a.v), bp = pair_swap(b.v);
            F29 z, nbp;
            f29_zero(z);
            f29_sub<8>(nbp, z, bp);
            const F29 y1 = f29_select(odd, bp, b.v);
            const F29 y2 = f29_select(odd, b.v, nbp);
            f29_mul2(r.v, a.v, y1, ap, y2);
        }
    }
    // r = a b + c d. Borrow-free form: one REDC of the lane's four products (f29_redc_sum4), < 2p;
    // otherwise two products and an addition, < 4p
    static DEV void mul_sum(P& r, const P& a, const P& b, const P& c, const P& d) {
        if constexpr (kBorrowFree) {
            const bool odd = pair_odd();
            const uint32_t msk = odd ? 0u : 0xffffffffu;
            F29 ap, y1, y2, cp, z1, z2;
#pragma unroll
            for (int i = 0; i < 14; ++i) {
                ap.v[i] = pair_swap(a.v.v[i]);
                y1.v[i] = pair_even(b.v.v[i]);
                const uint32_t yb = pair_odd_val(b.v.v[i]);
                y2.v[i] = (yb ^ msk) + (msk & (k16(i) + 1u));
                cp.v[i] = pair_swap(c.v.v[i]);
                z1.v[i] = pair_even(d.v.v[i]);
                const uint32_t zd = pair_odd_val(d.v.v[i]);
                z2.v[i] = (zd ^ msk) + (msk & (k16(i) + 1u));
            }
            // chains (a y1, ap y2) and (c z1, cp z2): one factor with 2^30 limbs (y2, z2) per chain, the
            // precondition of f29_redc_sum4
            f29_redc_sum4(r.v, a.v, y1, ap, y2, c.v, z1, cp, z2);
        } else {
            P x, y;
            mul(x, a, b);
            mul(y, c, d);
            f29_add(r.v, x.v, y.v);
        }
    }
    // (a0 + a1)(a0 - a1 + KB p) on the even lane, (a0 + a0) a1 on the odd one; KB bounds c1
    template <int KB>
    static DEV void sqr_b(P& r, const P& a) {
        const bool odd = pair_odd();
        const F29 ap = pair_swap(a.v);
        if constexpr (kBorrowFree) {
            // even: (a0 + a1) [limb sums, < 2^30, no carry] x (a0 - a1 + KB p) [normalized];
            // odd: a0 [normalized] x (a1 + a1) [limb sums, < 2^30]. One factor of every limb product
            // is < 2^29: columns <= 14 x 2^59 + 14 m p < 2^58 = 42 x 2^58. Same values as below.
            F29 d, x, y;
            f29_sub<KB>(d, a.v, ap);
#pragma unroll
            for (int i = 0; i < 14; ++i) {
                x.v[i] = odd ? ap.v[i] : a.v.v[i] + ap.v[i];
                y.v[i] = odd ? a.v.v[i] + a.v.v[i] : d.v[i];
            }
            f29_mul(r.v, x, y);
            return;
        }
        F29 s, d, x, y;
        f29_add(s, a.v, ap);          // even: a0 + a1
        f29_sub<KB>(d, a.v, ap);      // even: a0 - a1 + KB p
        f29_add(x, ap, ap);           // odd: 2 a0
        y = f29_select(odd, a.v, d);  // odd: a1
        x = f29_select(odd, x, s);
        f29_mul(r.v, x, y);
    }
    static DEV void sqr(P& r, const P& a) { sqr_b<8>(r, a); }
    static DEV void add(P& r, const P& a, const P& b) { f29_add(r.v, a.v, b.v); }
    template <int K>
    static DEV void sub(P& r, const P& a, const P& b) {
        f29_sub<K>(r.v, a.v, b.v);
    }
    template <int K>
    static DEV void reduce(P& x) {
        f29_reduce<K>(x.v);
    }
    static DEV bool zero2(const P& x) { return pair_all(f29_zero2(x.v)); }
    static DEV bool zero4(const P& x) { return pair_all(f29_zero4(x.v)); }
    template <int K>
    static DEV bool zero_lt(const P& x) {
        return pair_all(f29_zero_lt<K>(x.v));
    }
    static DEV bool is_zero_raw(const P& x) { return pair_all(f29_is_zero_raw(x.v)); }
    static DEV void zero(P& r) { f29_zero(r.v); }
    static DEV void one(P& r) {
        if (pair_odd())
            f29_zero(r.v);
        else
            f29_one(r.v);
    }
};
template <>
struct Ops29<FP29> : PairOps<FP29, false> {};
template <>
struct Ops29<FP29A> : PairOps<FP29A, true> {};

// ---- storage: the lane's half of a packed (12 x 32-bit words per Fq) Fq2 coordinate
template <class P>
DEV void fp29_unpack(P& r, const Fq2& s) {
    f29_unpack(r.v, pair_odd() ? s.c1.v : s.c0.v);
}
// ld / st of one lane's coefficient of coordinate k of a point at p (Fq2 coordinates, c0 then c1)
template <class P>
DEV void fp29_ld(P& r, const Fq2* coord) {
    Fq w;
    load_vec(w, pair_odd() ? &coord->c1 : &coord->c0);
    f29_unpack(r.v, w.v);
}
template <class P>
DEV void fp29_st(Fq2* coord, const P& r) {
    Fq w;
    f29_pack(w.v, r.v);
    store_vec(pair_odd() ? &coord->c1 : &coord->c0, w);
}

}  // namespace spx
