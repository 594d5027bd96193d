// Curve-templated MSM kernels and drivers; instantiated once per curve (msm_g1.hip, msm_g2.hip)
// so the heavy big-integer code of G1 and G2 compiles in parallel.
#pragma once
#include "curve29.hpp"
#include "fq2pair.hpp"
#include "msm_common.hpp"

namespace spx {

// Representation of the accumulation / weighting kernels per curve: G1 runs one point per lane
// (radix-2^29 Fq), G2 one point per lane PAIR (fq2pair.hpp: c0 on the even lane, c1 on the odd),
// so a G2 lane holds half a point and two waves fit each SIMD.
template <class F>
struct Acc;
// one lane's packed affine coordinates (G1: the point; G2: its half), as loaded from the table
struct AffRaw {
    Fq x, y;
};
template <>
struct Acc<Fq> {
    using Pt = G1Slot;  // window-table element: one 128-byte line per point
    using T = F29;
    using TA = F29;  // the accumulation kernel's element type
    static constexpr int kLanes = 1, kWaves = 1;
    static DEV void ld_raw(AffRaw& a, const G1Slot* p) { load_vec(*(Aff<Fq>*)&a, &p->p); }
    static DEV void unpack(T& x, T& y, const AffRaw& a) {
        f29_unpack(x, a.x.v);
        f29_unpack(y, a.y.v);
    }
    static DEV void ld_aff(T& x, T& y, const G1Slot* p) {
        AffRaw a;
        ld_raw(a, p);
        unpack(x, y, a);
    }
    static DEV bool aff_sentinel(const T& x, const T& y) { return f29_is_zero_raw(x) && f29_is_zero_raw(y); }
    static DEV void ld(X29<T>& r, const Xyzz<Fq>* p) { ld29<Fq>(r, p); }
    static DEV void st(Xyzz<Fq>* p, const X29<T>& r) { st29<Fq>(p, r); }
};
template <>
struct Acc<Fq2> {
    using Pt = Aff<Fq2>;  // 192 bytes: 1.5 lines, the lane pair's halves 96 bytes each
    // borrow-free operand preparation in the accumulation only (fq2pair.hpp); the weighting kernels,
    // at 256 registers already, keep the borrow-chain form (the borrow-free one spilled there)
    using T = FP29;
    using TA = FP29A;
    static constexpr int kLanes = 2, kWaves = 2;
    static DEV void ld_raw(AffRaw& a, const Aff<Fq2>* p) {
        const bool odd = pair_odd();
        load_vec(a.x, odd ? &p->x.c1 : &p->x.c0);
        load_vec(a.y, odd ? &p->y.c1 : &p->y.c0);
    }
    template <class P>
    static DEV void unpack(P& x, P& y, const AffRaw& a) {
        f29_unpack(x.v, a.x.v);
        f29_unpack(y.v, a.y.v);
    }
    template <class P>
    static DEV void ld_aff(P& x, P& y, const Aff<Fq2>* p) {
        fp29_ld(x, &p->x);
        fp29_ld(y, &p->y);
    }
    template <class P>
    static DEV bool aff_sentinel(const P& x, const P& y) {
        return pair_all(f29_is_zero_raw(x.v) && f29_is_zero_raw(y.v));
    }
    static DEV void ld(X29<T>& r, const Xyzz<Fq2>* p) {
        fp29_ld(r.x, &p->x);
        fp29_ld(r.y, &p->y);
        fp29_ld(r.zz, &p->zz);
        fp29_ld(r.zzz, &p->zzz);
    }
    template <class P>
    static DEV void st(Xyzz<Fq2>* p, const X29<P>& r) {
        fp29_st(&p->x, r.x);
        fp29_st(&p->y, r.y);
        fp29_st(&p->zz, r.zz);
        fp29_st(&p->zzz, r.zzz);
    }
};

// ---- split additions for the latency-bound weighting and partial kernels: two lane groups hold the
// same operands and split one addition's products (G2: two lane pairs = a quad, exchanged through DPP
// quad_perm [2,3,0,1]; G1: two lanes, exchanged through quad_perm [1,0,3,2]). 7 products on the
// dependent path of an addition instead of 14, 5 instead of 9 for a doubling, so one addition's
// latency (the whole cost of the weighting tree's upper levels) roughly halves. Both groups end with
// the identical result; group A = the lower, B = the upper.
template <class T>
struct Split;
template <>
struct Split<FP29> {
    static DEV bool half() { return (__lane_id() & 2) != 0; }
    static DEV FP29 swap(const FP29& a) {
        FP29 r;
#pragma unroll
        for (int i = 0; i < 14; ++i)
            r.v.v[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v.v[i], 0x4E, 0xF, 0xF, false);
        return r;
    }
    static DEV FP29 sel(bool h, const FP29& a, const FP29& b) {  // h ? b : a
        FP29 r;
        r.v = f29_select(h, b.v, a.v);
        return r;
    }
};
template <>
struct Split<F29> {
    static DEV bool half() { return pair_odd(); }
    static DEV F29 swap(const F29& a) { return pair_swap(a); }
    static DEV F29 sel(bool h, const F29& a, const F29& b) { return f29_select(h, b, a); }
};

// 2p (dbl-2008-s-1) split over two groups (the group that would square M computes M M as a
// product, so both groups run the same instruction stream)
template <class T>
DEV void x29_dbl_split(X29<T>& p) {
    using O = Ops29<T>;
    using S2 = Split<T>;
    if (x29_is_inf(p)) return;
    const bool h = S2::half();
    T U;
    O::add(U, p.y, p.y);  // < 8p
    T s1;
    O::sqr(s1, S2::sel(h, U, p.x));  // A: V = U^2, B: X2 = X^2 (c1 < 8p)
    const T s1o = S2::swap(s1);
    const T V = S2::sel(h, s1, s1o), X2 = S2::sel(h, s1o, s1);
    T M;
    O::add(M, X2, X2);
    O::add(M, M, X2);  // < 6p
    T a, b;
    O::mul(a, S2::sel(h, U, M), S2::sel(h, V, M));       // A: W = U V,  B: T = M M
    O::mul(b, S2::sel(h, p.x, V), S2::sel(h, V, p.zz));  // A: S = X V,  B: ZZ3 = V ZZ
    const T ao = S2::swap(a), bo = S2::swap(b);
    const T W = S2::sel(h, a, ao), Tm = S2::sel(h, ao, a);
    const T S = S2::sel(h, b, bo), ZZ3 = S2::sel(h, bo, b);
    T s2, x3, t2;
    O::add(s2, S, S);                 // < 4p
    O::template sub<4>(x3, Tm, s2);   // < 6p
    O::template reduce<8>(x3);        // < 2p
    O::template sub<2>(t2, S, x3);    // < 4p
    T c, d;
    O::mul(c, S2::sel(h, M, W), S2::sel(h, t2, p.y));  // A: M (S - X3),  B: W Y
    O::mul(d, W, p.zzz);                                // ZZZ3, both groups
    const T co = S2::swap(c);
    O::template sub<2>(p.y, S2::sel(h, c, co), S2::sel(h, co, c));
    O::template reduce<4>(p.y);
    p.x = x3;
    p.zz = ZZ3;
    p.zzz = d;
}

// p += q (add-2008-s) split over two groups; p and q identical on both; inputs and output as x29_add
// (< 2p, X may be loose < 8p, Y < 4p on input)
template <class T>
DEV void x29_add_split(X29<T>& p, const X29<T>& q) {
    using O = Ops29<T>;
    using S2 = Split<T>;
    if (x29_is_inf(q)) return;
    if (x29_is_inf(p)) {
        p = q;
        return;
    }
    const bool h = S2::half();
    // A: U1 = X1 ZZ2, S1 = Y1 ZZZ2, ZZ1 ZZ2;  B: U2 = X2 ZZ1, S2 = Y2 ZZZ1, ZZZ1 ZZZ2
    T u, s, z;
    O::mul(u, S2::sel(h, p.x, q.x), S2::sel(h, q.zz, p.zz));
    O::mul(s, S2::sel(h, p.y, q.y), S2::sel(h, q.zzz, p.zzz));
    O::mul(z, S2::sel(h, p.zz, p.zzz), S2::sel(h, q.zz, q.zzz));
    const T uo = S2::swap(u), so = S2::swap(s), zo = S2::swap(z);
    const T U1 = S2::sel(h, u, uo), U2 = S2::sel(h, uo, u);
    const T Sa = S2::sel(h, s, so), Sb = S2::sel(h, so, s);
    const T ZZ12 = S2::sel(h, z, zo), ZZZ12 = S2::sel(h, zo, z);
    T P, R;
    O::template sub<2>(P, U2, U1);
    O::template sub<2>(R, Sb, Sa);
    if (O::template zero_lt<4>(P)) {  // identical values on both groups: they branch together
        if (O::template zero_lt<4>(R))
            x29_dbl_split(p);
        else
            x29_set_inf(p);
        return;
    }
    // A: PP = P^2;  B: T = R^2  (P, R < 4p)
    T sq;
    O::sqr(sq, S2::sel(h, P, R));
    const T sqo = S2::swap(sq);
    const T PP = S2::sel(h, sq, sqo), Tr = S2::sel(h, sqo, sq);
    // A: PPP = P PP;  B: Q = U1 PP
    T m3;
    O::mul(m3, S2::sel(h, P, U1), PP);
    const T m3o = S2::swap(m3);
    const T PPP = S2::sel(h, m3, m3o), Q = S2::sel(h, m3o, m3);
    T w, t;
    O::template sub<2>(w, Tr, PPP);
    O::add(t, Q, Q);
    O::template sub<4>(w, w, t);
    O::template reduce<8>(w);       // X3 < 2p
    O::template sub<2>(t, Q, w);    // < 4p
    // A: R t, ZZ1 ZZ2 PP;  B: S1 PPP, ZZZ1 ZZZ2 PPP
    T y4, z4;
    O::mul(y4, S2::sel(h, R, Sa), S2::sel(h, t, PPP));
    O::mul(z4, S2::sel(h, ZZ12, ZZZ12), S2::sel(h, PP, PPP));
    const T y4o = S2::swap(y4), z4o = S2::swap(z4);
    O::template sub<2>(p.y, S2::sel(h, y4, y4o), S2::sel(h, y4o, y4));  // R t - S1 PPP
    O::template reduce<4>(p.y);
    p.x = w;
    p.zz = S2::sel(h, z4, z4o);
    p.zzz = S2::sel(h, z4o, z4);
}

// lanes per element in the weighting / partial kernels: G2 a quad, G1 a pair (split additions: the
// two halves of an element take different products of one addition)
template <class F>
struct TreeLanes {
    static constexpr int v = 2 * Acc<F>::kLanes;
};
template <class F>
DEV void tree_add(X29<typename Acc<F>::T>& p, const X29<typename Acc<F>::T>& q) {
    x29_add_split(p, q);
}
template <class F>
DEV void tree_dbl(X29<typename Acc<F>::T>& p) {
    x29_dbl_split(p);
}
template <class F>
DEV uint64_t tree_elem() {
    return (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / TreeLanes<F>::v;
}
template <class F>
static unsigned tree_blocks(uint64_t elems) {
    return (unsigned)((elems * TreeLanes<F>::v + kHeavy - 1) / kHeavy);
}

// element index of the calling lane (one element per Acc<F>::kLanes lanes)
template <class F>
DEV uint64_t acc_elem() {
    return (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / Acc<F>::kLanes;
}
template <class F>
static unsigned acc_blocks(uint64_t elems) {
    return (unsigned)((elems * Acc<F>::kLanes + kHeavy - 1) / kHeavy);
}

// ------------------------------------------------------------------ accumulation levels
// Accumulation and weighting run in the radix-2^29 domain (ff29.hpp / curve29.hpp): tables and
// partials in memory hold R = 2^406 Montgomery values (< 2p), packed into the 12-word layout.
// Load-balanced: thread t adds references [t seg1, (t+1) seg1) of the bucket-sorted array whatever
// the bucket boundaries, so every lane runs the same number of additions. A thread whose range
// crosses into the next (non-empty) bucket stores the finished partial and restarts; bucket b's
// partials are pfx[b] + (t - off[b] / seg1) for the threads t its range intersects.
template <class F>
__global__ __launch_bounds__(kHeavy, Acc<F>::kWaves) void k_accum_aff(const uint32_t* __restrict__ off, uint32_t nb,
                                                                      const uint32_t* __restrict__ pfx,
                                                                      const uint32_t* __restrict__ refs,
                                                                      const typename Acc<F>::Pt* __restrict__ pts,
                                                                      Xyzz<F>* __restrict__ out, uint32_t seg1) {
    using A = Acc<F>;
    using T = typename A::TA;
    const uint32_t t = (uint32_t)acc_elem<F>();
    const uint32_t total = off[nb];
    uint32_t e = t * seg1;
    if (e >= total) return;
    const uint32_t end = min(e + seg1, total);
    uint32_t b = find_bucket(off, nb, e);
    uint32_t bend = off[b + 1];
    uint32_t slot = pfx[b] + (t - off[b] / seg1);
    X29<T> acc;
    x29_set_inf(acc);
    for (; e < end; ++e) {
        if (e == bend) {  // bucket b is finished inside this range: the next one starts here
            A::st(out + slot, acc);
            x29_set_inf(acc);
            do {
                ++b;
            } while (off[b + 1] <= e);  // skip empty buckets
            bend = off[b + 1];
            slot = pfx[b];
        }
        // (issuing the next point's load before this addition measured within noise: DESIGN.md 4.1)
        const uint32_t r = refs[e];
        T px, py;
        A::ld_aff(px, py, pts + (r & 0x7fffffffu));
        if (A::aff_sentinel(px, py)) continue;
        x29_madd(acc, px, py, (r >> 31) != 0);
    }
    A::st(out + slot, acc);
}

template <class F>
__global__ __launch_bounds__(kHeavy, Acc<F>::kWaves) void k_accum_xyzz(const uint32_t* __restrict__ segoff, uint32_t nb,
                                                                       const uint32_t* __restrict__ off,
                                                                       const Xyzz<F>* __restrict__ in,
                                                                       Xyzz<F>* __restrict__ out) {
    using A = Acc<F>;
    using T = typename A::T;
    const uint32_t s = (uint32_t)tree_elem<F>();
    if (s >= segoff[nb]) return;
    const uint32_t b = find_bucket(segoff, nb, s);
    const uint32_t k = s - segoff[b];
    const uint32_t start = off[b] + k * kSeg;
    const uint32_t end = min(start + kSeg, off[b + 1]);  // bucket b's partials: [off[b], off[b + 1])
    X29<T> acc;
    A::ld(acc, in + start);
    for (uint32_t e = start + 1; e < end; ++e) {
        X29<T> p;
        A::ld(p, in + e);
        tree_add<F>(acc, p);
    }
    A::st(out + s, acc);
}

// ------------------------------------------------------------------ bucket weighting: chunks + tree
// Result = sum_j (j+1) S_j over the B = 2^(c-1) bucket sums of an instance. Node = (F, S, D) over a
// run of consecutive buckets, with F = sum_m (m+1) X_m (local index m), S = sum X_m, D = size * S.
// Leaf level, chunked (k_tree_chunk): one thread sums m = 2^lgm consecutive buckets by a running
// sum (from the top bucket down: run += X_j, F += run), giving the chunk's node (F, S, D = m S) in
// 2m additions + lgm doublings (a pairwise tree spends ~5 group operations per bucket on the
// levels this replaces). Above it, a binary tree over the chunks:
//   parent(l, r) = (F_l + D_r + F_r,  S_l + S_r,  2 (D_l + D_r))      (size(l) = size(r))
// one level per launch, one thread per (node, component), component-major so every wave runs one
// component (no divergence between the F / S / D formulas): 2 group operations of dependent
// depth per level (single-lane latency of a G2 addition is ~45 us on CDNA4).
// A missing right child (instances with fewer chunks) is the point at infinity: F and S pass
// through unchanged, so all instances of a batch run the same number of levels.
// lb = log2 of the instance's (local) buckets >= 1; chunks of 2^lgm buckets, lgm <= lb - 1
DEV uint32_t tree_chunk_log(uint32_t lb) { return lb - 1 < kTreeChunkLog ? lb - 1 : kTreeChunkLog; }

// Every partial a bucket still has is added here (the partial levels are planned from the expected
// occupancy, so a crowded bucket may arrive with several): run += X for each, then F += run.
template <class F>
__global__ __launch_bounds__(kHeavy, Acc<F>::kWaves) void k_tree_chunk(
    const MsmInst* __restrict__ insts, const uint64_t* __restrict__ wp, int ninst, const uint32_t* __restrict__ node_off,
    const uint32_t* __restrict__ off, const Xyzz<F>* __restrict__ P,
    Xyzz<F>* __restrict__ Fo, Xyzz<F>* __restrict__ So, Xyzz<F>* __restrict__ Do) {
    using A = Acc<F>;
    const uint64_t t = tree_elem<F>();
    if (t >= wp[ninst]) return;
    const int i = find_slot(wp, ninst, t);
    const uint32_t k = (uint32_t)(t - wp[i]);
    const MsmInst I = insts[i];
    const uint32_t lgm = tree_chunk_log(I.lb);
    const uint32_t b0 = I.bucket_off + (k << lgm);
    const uint32_t o = node_off[i] + k;
    // F accumulates in its output slot, and both kinds of step (run += X, F += run) go through one
    // addition site with two points live: a G2 XYZZ point is 112 registers in radix 2^29
    using T = typename A::T;
    X29<T> run;
    x29_set_inf(run);
    const int m = 1 << lgm;
    int j = m - 1;
    uint32_t u = 0, nu = off[b0 + j + 1] - off[b0 + j];  // partials of bucket j added so far / to add
#pragma unroll 1
    for (;;) {
        const bool bucket_step = u < nu;
        X29<T> a, b;
        if (bucket_step) {
            a = run;
            A::ld(b, P + off[b0 + j] + u);
            ++u;
        } else if (j == m - 1) {  // F = run for the top bucket
            A::st(Fo + o, run);
            if (j == 0) break;
            --j;
            u = 0;
            nu = off[b0 + j + 1] - off[b0 + j];
            continue;
        } else {
            A::ld(a, Fo + o);
            b = run;
        }
        tree_add<F>(a, b);
        if (bucket_step) {
            run = a;
        } else {
            A::st(Fo + o, a);
            if (j == 0) break;
            --j;
            u = 0;
            nu = off[b0 + j + 1] - off[b0 + j];
        }
    }
    A::st(So + o, run);
#pragma unroll 1
    for (uint32_t d = 0; d < lgm; ++d) tree_dbl<F>(run);
    A::st(Do + o, run);
}

template <class F>
__global__ __launch_bounds__(kHeavy, Acc<F>::kWaves) void k_tree_level(
    const uint64_t* __restrict__ wp, int ninst, const uint32_t* __restrict__ node_off, const uint32_t* __restrict__ cnt_in,
    const Xyzz<F>* __restrict__ Fi, const Xyzz<F>* __restrict__ Si, const Xyzz<F>* __restrict__ Di,
    Xyzz<F>* __restrict__ Fo, Xyzz<F>* __restrict__ So, Xyzz<F>* __restrict__ Do) {
    using A = Acc<F>;
    const uint64_t t = tree_elem<F>();
    const uint64_t N = wp[ninst];
    if (t >= 3 * N) return;
    const uint32_t comp = (uint32_t)(t / N);
    const uint64_t tn = t - comp * N;
    const int i = find_slot(wp, ninst, tn);
    const uint32_t k = (uint32_t)(tn - wp[i]);
    const uint32_t base = node_off[i], n = cnt_in[i];
    const bool has_r = 2 * k + 1 < n;
    X29<typename A::T> a, b;
    if (comp == 0) {  // F_l + D_r + F_r
        A::ld(a, Fi + base + 2 * k);
        if (has_r) {
            A::ld(b, Di + base + 2 * k + 1);
            tree_add<F>(a, b);
            A::ld(b, Fi + base + 2 * k + 1);
            tree_add<F>(a, b);
        }
        A::st(Fo + base + k, a);
    } else if (comp == 1) {
        A::ld(a, Si + base + 2 * k);
        if (has_r) {
            A::ld(b, Si + base + 2 * k + 1);
            tree_add<F>(a, b);
        }
        A::st(So + base + k, a);
    } else {
        A::ld(a, Di + base + 2 * k);
        if (has_r) {  // a lone root passes through (its D is never read again)
            A::ld(b, Di + base + 2 * k + 1);
            tree_add<F>(a, b);
            tree_dbl<F>(a);
        }
        A::st(Do + base + k, a);
    }
}

// The top levels of every instance's weighting tree in ONE launch: one workgroup per instance, its
// nodes in LDS (the levels whose input has <= kTopNodes = 32 nodes; each is 2 dependent additions, so
// launching them one by one cost a launch gap per level). Then, for an instance split over the ranks
// (this rank holds buckets u = sel + G k, G = 2^lg, as local buckets k, and the tree computed
// F = sum_k (k + 1) X_k, S = sum_k X_k), the rank's share sum_k (sel + G k + 1) X_k = G F - (G - 1 - sel) S;
// finally the R = 2^384 Montgomery output for the host.
static constexpr int kTopThreads = 128;
template <class F>
__global__ __launch_bounds__(kTopThreads, 1) void k_tree_top(const MsmInst* __restrict__ insts, int nact,
                                                             const uint32_t* __restrict__ node_off,
                                                             const uint32_t* __restrict__ cin_top, int lv0, int levels,
                                                             const Xyzz<F>* __restrict__ Fi, const Xyzz<F>* __restrict__ Si,
                                                             const Xyzz<F>* __restrict__ Di, Xyzz<F>* __restrict__ out) {
    using A = Acc<F>;
    using T = typename A::T;
    using O = Ops29<T>;
    constexpr int kL = TreeLanes<F>::v;
    __shared__ Xyzz<F> buf[2][3][kTopNodes];
    const int i = blockIdx.x;
    const MsmInst I = insts[i];
    const uint32_t base = node_off[i];
    const int grp = threadIdx.x / kL, ngrp = kTopThreads / kL;
    // the instance's node count after the leaf: its input at lv0 is max(1, cnt >> (lv0 - 1))
    uint32_t nin = cin_top[i];
    for (uint32_t t = threadIdx.x; t < 3 * nin; t += blockDim.x) {
        const uint32_t comp = t / nin, k = t % nin;
        const Xyzz<F>* src = comp == 0 ? Fi : (comp == 1 ? Si : Di);
        buf[0][comp][k] = src[base + k];
    }
    __syncthreads();
    int cur = 0;
    for (int lv = lv0; lv <= levels; ++lv) {
        const uint32_t nout = nin > 1 ? nin / 2 : 1;
        for (uint32_t task = grp; task < 3 * nout; task += ngrp) {
            const uint32_t comp = task / nout, k = task % nout;
            const bool has_r = 2 * k + 1 < nin;
            X29<T> a, b;
            A::ld(a, &buf[cur][comp][2 * k]);
            if (comp == 0) {  // F_l + D_r + F_r
                if (has_r) {
                    A::ld(b, &buf[cur][2][2 * k + 1]);
                    tree_add<F>(a, b);
                    A::ld(b, &buf[cur][0][2 * k + 1]);
                    tree_add<F>(a, b);
                }
            } else if (has_r) {  // S_l + S_r; 2 (D_l + D_r)
                A::ld(b, &buf[cur][comp][2 * k + 1]);
                tree_add<F>(a, b);
                if (comp == 2) tree_dbl<F>(a);
            }
            A::st(&buf[cur ^ 1][comp][k], a);
        }
        __syncthreads();
        cur ^= 1;
        nin = nout;
    }
    if (I.lg) {  // the rank's share of a split instance: G F - (G - 1 - sel) S, the two products side by side
        const uint32_t k = (1u << I.lg) - 1 - I.sel;
        if (grp == 0) {  // G F: lg doublings
            X29<T> f;
            A::ld(f, &buf[cur][0][0]);
#pragma unroll 1
            for (uint32_t d = 0; d < I.lg; ++d) tree_dbl<F>(f);
            A::st(&buf[cur][0][0], f);
        } else if (grp == 1 && k) {  // -(k S): double-and-add below the top bit, into the free slot
            X29<T> sv, acc;
            A::ld(sv, &buf[cur][1][0]);
            acc = sv;
#pragma unroll 1
            for (int b = 30 - __clz(k); b >= 0; --b) {
                tree_dbl<F>(acc);
                if ((k >> b) & 1u) tree_add<F>(acc, sv);
            }
            T z;
            O::zero(z);
            O::template sub<2>(acc.y, z, acc.y);  // y < 2p -> 2p - y < 2p
            A::st(&buf[cur][1][1], acc);
        }
        __syncthreads();
        if (grp == 0 && k) {
            X29<T> f, acc;
            A::ld(f, &buf[cur][0][0]);
            A::ld(acc, &buf[cur][1][1]);
            tree_add<F>(f, acc);
            A::st(&buf[cur][0][0], f);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // back to the R = 2^384 Montgomery domain, canonical, for the host
        using T1 = typename R29<F>::T;
        X29<T1> a, b;
        ld29<F>(a, &buf[cur][0][0]);
        f29_map(b.x, a.x, Q29::TO_R1);
        f29_map(b.y, a.y, Q29::TO_R1);
        f29_map(b.zz, a.zz, Q29::TO_R1);
        f29_map(b.zzz, a.zzz, Q29::TO_R1);
        st29<F>(out + I.out, b);
    }
}

// SPX_MSM_LEVELS=k (A/B): at most k XYZZ partial levels; the weighting leaf adds the rest
static int msm_levels_env() {
    static const int v = [] {
        const char* e = getenv("SPX_MSM_LEVELS");
        return e ? atoi(e) : -1;
    }();
    return v;
}
// SPX_MSM_SEG1=k (A/B): at most k references per accumulation thread
static int msm_seg1_env() {
    static const int v = [] {
        const char* e = getenv("SPX_MSM_SEG1");
        return e ? atoi(e) : 0;
    }();
    return v;
}

template <class F>
static void msm_run_t(MsmWorkspace* ws, const MsmInst* ih, int ninst, const typename Acc<F>::Pt* pts, const Fr* scalars,
                      void* out_dev, hipStream_t s, const MsmShard& sh) {
    if (ninst <= 0) return;
    const bool g2 = sizeof(F) == sizeof(Fq2);
    const size_t psz = sizeof(Xyzz<F>);
    const size_t ob = msm_out_bytes(g2, ninst);
    MsmPlan pl = msm_plan(ih, ninst, sh, ws->cap_scale);
    const int nact = (int)pl.insts.size();
    if (!nact) {  // nothing of this batch is this rank's: every output is infinity (all zero), status 0
        HIPCHK(hipMemsetAsync(out_dev, 0, ob, s));
        return;
    }
    msm_upload_plan(ws, pl, s);
    const uint32_t nb = pl.nb;
    const uint64_t tot_refs = pl.tot_refs;
    // level 1: affine references -> XYZZ partials, one per segment of kSeg1 references
    uint32_t kSeg1 = seg1_fit(seg1_len(g2), tot_refs, Acc<F>::kWaves, Acc<F>::kLanes);
    if (msm_seg1_env() > 0) kSeg1 = std::min<uint32_t>(kSeg1, (uint32_t)msm_seg1_env());
    // XYZZ partial levels, planned from the expected occupancy (no host round trip): a bucket with
    // mu references on average rarely exceeds mu + 6 sqrt(mu) + 16; the weighting leaf adds the
    // partials of any bucket that does (k_tree_chunk), so the plan decides speed, never correctness
    const double mu = pl.mu_max;
    int nlev = 0;
    for (uint32_t m = (uint32_t)std::ceil((mu + 6.0 * std::sqrt(mu) + 16.0) / kSeg1) + 1; m > 1; m = (m + kSeg - 1) / kSeg)
        ++nlev;  // partials per bucket, divided by kSeg per level
    if (msm_levels_env() >= 0) nlev = std::min(nlev, msm_levels_env());
    // the sort's first launch zeroes the outputs (infinity) and the status words
    MsmSorted so = msm_sort(ws, pl, scalars, out_dev, ob, s, kSeg1, nlev);
    const uint64_t max_segs = tot_refs / kSeg1 + nb + 1;
    auto* PA = (Xyzz<F>*)ws->pa.ensure(psz * max_segs);
    auto* PB = (Xyzz<F>*)ws->pb.ensure(psz * (max_segs / kSeg + nb + 1));
    uint32_t* cur_off = so.np_off;
    uint32_t* nxt_off = nullptr;
    const uint64_t nthr = (tot_refs + kSeg1 - 1) / kSeg1;
    kp_begin(g2 ? KP_ACC_G2 : KP_ACC_G1, s);
    hipLaunchKernelGGL(k_accum_aff<F>, dim3(acc_blocks<F>(nthr)), dim3(kHeavy), 0, s, so.offs, nb, cur_off, so.refs, pts, PA,
                       kSeg1);
    // algorithmic bytes: every reference (4 B) and its affine point once (96 / 192 B, not the slot's
    // padding), one XYZZ partial per segment
    kp_end((double)tot_refs * (4.0 + sizeof(Aff<F>)) + (double)(tot_refs / kSeg1) * psz, s, (double)tot_refs);
    Xyzz<F>* cur = PA;
    Xyzz<F>* nxt = PB;
    uint64_t cur_max_segs = max_segs;
    for (int l = 0; l < nlev; ++l) {
        nxt_off = so.lev[l];  // computed by the sort
        uint64_t nsegs = cur_max_segs / kSeg + nb + 1;
        kp_begin(g2 ? KP_ACCX_G2 : KP_ACCX_G1, s);
        hipLaunchKernelGGL(k_accum_xyzz<F>, dim3(tree_blocks<F>(nsegs)), dim3(kHeavy), 0, s, nxt_off, nb, cur_off, cur, nxt);
        kp_end((double)(cur_max_segs + nsegs) * psz, s, (double)cur_max_segs);
        std::swap(cur, nxt);
        std::swap(cur_off, nxt_off);
        cur_max_segs = nsegs;
    }
    // bucket weighting tree over each instance's 2^lb local buckets: leaf, middle levels, top
    uint32_t tot_nodes = 0;
    for (int i = 0; i < nact; ++i) tot_nodes += pl.cnt[i];
    auto* TA = (Xyzz<F>*)ws->tree_a.ensure(3 * psz * std::max<uint32_t>(tot_nodes, 1));
    auto* TB = (Xyzz<F>*)ws->tree_b.ensure(3 * psz * std::max<uint32_t>(tot_nodes, 1));
    Xyzz<F>* A3[3] = {TA, TA + tot_nodes, TA + 2 * (size_t)tot_nodes};
    Xyzz<F>* B3[3] = {TB, TB + tot_nodes, TB + 2 * (size_t)tot_nodes};
    kp_begin(g2 ? KP_RED_G2 : KP_RED_G1, s);
    {
        uint64_t work = pl.wp[nact];
        hipLaunchKernelGGL(k_tree_chunk<F>, dim3(tree_blocks<F>(work)), dim3(kHeavy), 0, s, pl.d_insts, pl.d_wp, nact,
                           pl.d_noff, cur_off, cur, A3[0], A3[1], A3[2]);
    }
    for (int lv = 1; lv < pl.top_from; ++lv) {
        uint64_t work = 3 * pl.wp[(size_t)lv * (nact + 1) + nact];
        hipLaunchKernelGGL(k_tree_level<F>, dim3(tree_blocks<F>(work)), dim3(kHeavy), 0, s,
                           pl.d_wp + (size_t)lv * (nact + 1), nact, pl.d_noff, pl.d_cin + (size_t)lv * nact, A3[0], A3[1],
                           A3[2], B3[0], B3[1], B3[2]);
        std::swap(A3, B3);
    }
    hipLaunchKernelGGL(k_tree_top<F>, dim3(nact), dim3(kTopThreads), 0, s, pl.d_insts, nact, pl.d_noff,
                       pl.d_cin + (size_t)pl.top_from * nact, pl.top_from, pl.levels, A3[0], A3[1], A3[2],
                       (Xyzz<F>*)out_dev);
    kp_end((double)nb * psz, s);
    HIPCHK(hipGetLastError());
}

// ------------------------------------------------------------------ PP preprocessing
template <class F>
DEV void xyzz_from_aff(Xyzz<F>& r, const Aff<F>& a) {
    if (aff_is_sentinel(a)) {
        xyzz_set_inf(r);
        return;
    }
    r.x = a.x;
    r.y = a.y;
    FieldOps<F>::one(r.zz);
    FieldOps<F>::one(r.zzz);
}

template <class F>
__global__ __launch_bounds__(kHeavy) void k_precompute(const Aff<F>* __restrict__ raw, uint64_t count, int pair_sum,
                                                       int c, int W, Xyzz<F>* __restrict__ tmp) {
    const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= count) return;
    Xyzz<F> P;
    if (pair_sum) {
        Aff<F> a, b;
        load_vec(a, raw + 2 * j);
        load_vec(b, raw + 2 * j + 1);
        xyzz_from_aff(P, a);
        if (!aff_is_sentinel(b)) xyzz_madd(P, b, false);
    } else {
        Aff<F> a;
        load_vec(a, raw + j);
        xyzz_from_aff(P, a);
    }
    for (int w = 0; w < W; ++w) {
        store_vec(tmp + (uint64_t)w * count + j, P);
        if (w + 1 < W)
            for (int k = 0; k < c; ++k) xyzz_dbl(P, P);
    }
}

// XYZZ -> affine with Montgomery's batch-inversion trick over chunks of kNormChunk points
static constexpr int kNormChunk = 32;
template <class F>
__global__ __launch_bounds__(kHeavy) void k_normalize(const Xyzz<F>* __restrict__ in, uint64_t n, Aff<F>* __restrict__ out) {
    using O = FieldOps<F>;
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t b = t * kNormChunk;
    if (b >= n) return;
    const uint64_t e = min(b + (uint64_t)kNormChunk, n);
    F acc;
    O::one(acc);
    for (uint64_t k = b; k < e; ++k) {
        Xyzz<F> p;
        load_vec(p, in + k);
        out[k].x = acc;  // prefix product parked in the output
        if (!xyzz_is_inf(p)) {
            F d;
            O::mul(d, p.zz, p.zzz);
            O::mul(acc, acc, d);
        }
    }
    F inv;
    O::inv(inv, acc);
    for (uint64_t k = e; k-- > b;) {
        Xyzz<F> p;
        load_vec(p, in + k);
        if (xyzz_is_inf(p)) {
            Aff<F> a;
            aff_set_sentinel(a);
            store_vec(out + k, a);
            continue;
        }
        F d, di, izz, izzz;
        O::mul(di, inv, out[k].x);
        O::mul(d, p.zz, p.zzz);
        O::mul(inv, inv, d);
        O::mul(izz, di, p.zzz);
        O::mul(izzz, di, p.zz);
        Aff<F> a;
        O::mul(a.x, p.x, izz);
        O::mul(a.y, p.y, izzz);
        store_vec(out + k, a);
    }
}

// affine table, R = 2^384 canonical -> R = 2^406 canonical (in place); the sentinel (0, 0) maps to itself
template <class F>
__global__ __launch_bounds__(kHeavy) void k_aff_to_r29(Aff<F>* __restrict__ a, uint64_t n) {
    using T = typename R29<F>::T;
    const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= n) return;
    Aff<F> p;
    load_vec(p, a + j);
    T x, y, mx, my;
    R29<F>::unpack(x, p.x);
    R29<F>::unpack(y, p.y);
    f29_map(mx, x, Q29::FROM_R1);
    f29_map(my, y, Q29::FROM_R1);
    R29<F>::pack(p.x, mx);
    R29<F>::pack(p.y, my);
    store_vec(a + j, p);
}

template <class F>
static void precompute_windows_t(const Aff<F>* raw, uint64_t count, bool pair_sum, int c, int W, Aff<F>* dst, void* tmp,
                               hipStream_t s) {
    if (!count) return;
    Xyzz<F>* t = (Xyzz<F>*)tmp;
    hipLaunchKernelGGL(k_precompute<F>, dim3((unsigned)((count + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, raw, count,
                       pair_sum ? 1 : 0, c, W, t);
    const uint64_t n = count * (uint64_t)W;
    const uint64_t nt = (n + kNormChunk - 1) / kNormChunk;
    hipLaunchKernelGGL(k_normalize<F>, dim3((unsigned)((nt + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, t, n, dst);
    hipLaunchKernelGGL(k_aff_to_r29<F>, dim3((unsigned)((n + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, dst, n);
    HIPCHK(hipGetLastError());
}
// ------------------------------------------------------------------ fixed-base (keygen)
template <class F>
__global__ __launch_bounds__(kHeavy) void k_fixed_base(const Aff<F>* __restrict__ table, const Fr* __restrict__ scalars,
                                                       uint64_t n, Xyzz<F>* __restrict__ tmp) {
    const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= n) return;
    Fr m, s;
    load_vec(m, scalars + j);
    fe_from_mont(s, m);
    Xyzz<F> acc;
    xyzz_set_inf(acc);
    for (int w = 0; w < 32; ++w) {
        const uint32_t d = (s.v[w >> 2] >> (8 * (w & 3))) & 0xffu;
        if (d) {
            Aff<F> a;
            load_vec(a, table + w * 256 + d);
            xyzz_madd(acc, a, false);
        }
    }
    store_vec(tmp + j, acc);
}
template <class F>
static void fixed_base_t(const Aff<F>* table, const Fr* scalars, uint64_t n, Aff<F>* out, void* tmp, hipStream_t s) {
    if (!n) return;
    Xyzz<F>* t = (Xyzz<F>*)tmp;
    hipLaunchKernelGGL(k_fixed_base<F>, dim3((unsigned)((n + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, table, scalars,
                       n, t);
    const uint64_t nt = (n + kNormChunk - 1) / kNormChunk;
    hipLaunchKernelGGL(k_normalize<F>, dim3((unsigned)((nt + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, t, n, out);
    HIPCHK(hipGetLastError());
}
}  // namespace spx
