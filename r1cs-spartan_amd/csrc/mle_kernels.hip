// HBM-streaming Fr kernels of the hot path:
//   * canonical <-> Montgomery conversion of witness / matrix values,
//   * sum_over_y  = three CSR SpMVs Az, Bz, Cz (r1cs_reader.rs:75-85),
//   * eval_on_x   = A(r_x, .) as a CSC gather against eq(r_x), combined over A,B,C with the
//                   verifier's r_A, r_B, r_C (r1cs_reader.rs:91-117 + prover.rs:239-245),
//   * eq tables   (eq.rs:5-20 in product form),
//   * sumcheck rounds (AHPForMLSumcheck::prove_round [upstream]) fused with the binding of the
//     previous challenge, and the mKZG quotient/fold levels of open.rs:37-45.
// Every kernel is a grid-stride stream over 32-byte Fr elements (two 16-byte loads per element),
// with per-block partial sums reduced by wave64 shuffles + LDS and, in the last block to finish,
// over the blocks (field addition is exact, so results are deterministic). A sumcheck round is ONE
// launch: the previous challenge arrives as a kernel argument and the round's three sums are written
// straight into the host's pinned memory.
#include "kernels.hpp"

#include <algorithm>
#include <stdexcept>

namespace spx {

thread_local KProf* g_kprof = nullptr;
static constexpr int kThreads = 256;

DEV Fr ld_fr(const Fr* p) {
    Fr r;
    load_vec(r, p);
    return r;
}
DEV void st_fr(Fr* p, const Fr& v) { store_vec(p, v); }
// folded sumcheck tables: written once, read by the next round (SPX_FOLD_NT=1: non-temporal stores)
#ifndef SPX_FOLD_NT
#define SPX_FOLD_NT 0
#endif
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
DEV void st_fr_fold(Fr* p, const Fr& v) {
    if constexpr (SPX_FOLD_NT) {
        u32x4* d = reinterpret_cast<u32x4*>(p);
        __builtin_nontemporal_store((u32x4){v.v[0], v.v[1], v.v[2], v.v[3]}, d);
        __builtin_nontemporal_store((u32x4){v.v[4], v.v[5], v.v[6], v.v[7]}, d + 1);
    } else {
        store_vec(p, v);
    }
}

// ------------------------------------------------------------------ block reduction of K Fr values
template <int K>
DEV void block_reduce_store(Fr (&acc)[K], Fr* out /* K entries for this block */) {
    __shared__ Fr lds[K][kThreads / 64];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            Fr o = shfl_xor(acc[k], m);
            fe_add(acc[k], acc[k], o);
        }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) lds[k][wid] = acc[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            Fr s = lds[k][0];
            for (int w = 1; w < (int)(blockDim.x / 64); ++w) fe_add(s, s, lds[k][w]);
            st_fr(out + k, s);
        }
    }
}

// out[k] = sum over blocks of partial[b*K + k]  (one block)
template <int K>
__global__ __launch_bounds__(kThreads) void k_reduce_partials(const Fr* __restrict__ partial, int nblk,
                                                              Fr* __restrict__ out) {
    Fr acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) fe_zero(acc[k]);
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
#pragma unroll
        for (int k = 0; k < K; ++k) fe_add(acc[k], acc[k], ld_fr(partial + (size_t)b * K + k));
    }
    block_reduce_store<K>(acc, out);
}

// Last-block reduction (one launch per sumcheck round instead of two). The per-XCD L2s are not
// coherent, and a __threadfence() per block (an L2 write-back + L1 invalidate, several us each) cost
// more than the launch it saves; so the hand-off follows the guide's write-through form
// (cdna_hip_programming.md §6 G16): each block's thread 0 stores its K partials with agent-scope
// (sc1, write-through) stores, drains them (s_waitcnt vmcnt(0)), then takes a ticket; the block that
// draws the last ticket reads every partial with agent-scope (sc1) loads, sums them in block order
// (field addition is exact: the same element as a separate reduction launch) into `out` (may be
// host-mapped pinned memory, read after the stream sync) and resets the ticket.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
template <int K>
DEV void block_reduce(Fr (&acc)[K]) {  // result valid in thread 0
    __shared__ Fr lds[K][kThreads / 64];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            Fr o = shfl_xor(acc[k], m);
            fe_add(acc[k], acc[k], o);
        }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) lds[k][wid] = acc[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            Fr s = lds[k][0];
            for (int w = 1; w < (int)(blockDim.x / 64); ++w) fe_add(s, s, lds[k][w]);
            acc[k] = s;
        }
    }
    __syncthreads();  // lds may be reused by the caller's next reduction
}
template <int K>
DEV void grid_reduce_last(Fr (&acc)[K], Fr* __restrict__ partial, uint32_t* __restrict__ ticket, Fr* __restrict__ out) {
    block_reduce<K>(acc);
    __shared__ bool last;
    if (threadIdx.x == 0) {
        gu64* dst = (gu64*)(partial + (size_t)blockIdx.x * K);
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int w = 0; w < 4; ++w)
                __hip_atomic_store(dst + 4 * k + w, (unsigned long long)acc[k].v[2 * w] | ((unsigned long long)acc[k].v[2 * w + 1] << 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial has left this CU before the ticket
        last = __hip_atomic_fetch_add((gu32*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
#pragma unroll
    for (int k = 0; k < K; ++k) fe_zero(acc[k]);
    for (uint32_t b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
        const gu64* src = (const gu64*)(partial + (size_t)b * K);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            Fr v;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const unsigned long long x = __hip_atomic_load(src + 4 * k + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v.v[2 * w] = (uint32_t)x;
                v.v[2 * w + 1] = (uint32_t)(x >> 32);
            }
            fe_add(acc[k], acc[k], v);
        }
    }
    block_reduce<K>(acc);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) st_fr(out + k, acc[k]);
        *ticket = 0u;
    }
}

// ------------------------------------------------------------------ conversions
__global__ void k_to_mont(Fr* __restrict__ data, size_t n, int* __restrict__ err) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        Fr c = ld_fr(data + i);
        if (!fr_is_canonical(c)) atomicOr(err, 1);
        Fr m;
        fr_to_mont(m, c);
        st_fr(data + i, m);
    }
}
__global__ void k_from_mont(Fr* __restrict__ out, const Fr* __restrict__ in, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        Fr m = ld_fr(in + i), c;
        fe_from_mont(c, m);
        st_fr(out + i, c);
    }
}

// ------------------------------------------------------------------ sparse products
// Short rows: one thread per output index x (local), three matrices at once. Rows flagged
// long (row length > kLongRow) contribute nothing here and are added by the chunk kernels.
// MODE 0 (sum_over_y): out_m[x] = sum_k val_m[k] * vec[col_m[k]] for m = A,B,C.
// MODE 1 (eval_on_x, combined): out[x] = sum_m scale_m * sum_k val_m[k] * vec[col_m[k]].
template <int MODE>
__global__ __launch_bounds__(kThreads) void k_sparse3(SparseView3 mv, const Fr* __restrict__ vec, Fr* out0,
                                                      Fr* out1, Fr* out2, const Fr* __restrict__ scale,
                                                      uint64_t count) {
    Fr s[3];
    if (MODE == 1) {
#pragma unroll
        for (int m = 0; m < 3; ++m) s[m] = ld_fr(scale + m);
    }
    for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < count;
         x += (uint64_t)gridDim.x * blockDim.x) {
        Fr tot;
        fe_zero(tot);
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            const uint64_t b = mv.ptr[m][x], e = mv.ptr[m][x + 1];
            Fr acc;
            fe_zero(acc);
            if (e - b <= kLongRow) {
                for (uint64_t k = b; k < e; ++k) {
                    Fr v = ld_fr(mv.val[m] + k), zv = ld_fr(vec + mv.idx[m][k]), t;
                    fe_mul(t, v, zv);
                    fe_add(acc, acc, t);
                }
            }
            if (MODE == 0) {
                st_fr(m == 0 ? out0 + x : (m == 1 ? out1 + x : out2 + x), acc);
            } else {
                Fr t;
                fe_mul(t, acc, s[m]);
                fe_add(tot, tot, t);
            }
        }
        if (MODE == 1) st_fr(out0 + x, tot);
    }
}

// Long rows: one block per chunk of <= kChunk entries; partial[chunk] = sum val * vec[idx].
__global__ __launch_bounds__(kThreads) void k_sparse_chunks(SparseView3 mv, const Fr* __restrict__ vec,
                                                            const LongChunk* __restrict__ chunks,
                                                            Fr* __restrict__ partial) {
    const LongChunk ch = chunks[blockIdx.x];
    const Fr* val = mv.val[ch.m];
    const uint32_t* idx = mv.idx[ch.m];
    Fr acc[1];
    fe_zero(acc[0]);
    for (uint64_t k = ch.begin + threadIdx.x; k < ch.end; k += blockDim.x) {
        Fr v = ld_fr(val + k), zv = ld_fr(vec + idx[k]), t;
        fe_mul(t, v, zv);
        fe_add(acc[0], acc[0], t);
    }
    block_reduce_store<1>(acc, partial + blockIdx.x);
}

// Single thread, fixed order: fold the chunk partials of every long (matrix, row) into the outputs.
template <int MODE>
__global__ void k_sparse_long_finish(const LongRow* __restrict__ rows, int nrows, const Fr* __restrict__ partial,
                                     Fr* out0, Fr* out1, Fr* out2, const Fr* __restrict__ scale) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int r = 0; r < nrows; ++r) {
        const LongRow lr = rows[r];
        Fr acc;
        fe_zero(acc);
        for (uint32_t c = lr.chunk_begin; c < lr.chunk_end; ++c) fe_add(acc, acc, ld_fr(partial + c));
        Fr* o;
        if (MODE == 0) {
            o = (lr.m == 0 ? out0 : (lr.m == 1 ? out1 : out2)) + lr.x;
        } else {
            Fr t;
            fe_mul(t, acc, ld_fr(scale + lr.m));
            acc = t;
            o = out0 + lr.x;
        }
        Fr cur = ld_fr(o);
        fe_add(cur, cur, acc);
        st_fr(o, cur);
    }
}

// ------------------------------------------------------------------ eq tables
// One block: tab[x] = prod_{j<k} eq(r_j, x_j) for x < 2^k (k <= 12), variable 0 = LSB.
__global__ __launch_bounds__(kThreads) void k_eq_small(const Fr* __restrict__ r, int k, Fr* __restrict__ tab) {
    if (threadIdx.x == 0) {
        Fr one;
        fe_one(one);
        st_fr(tab, one);
    }
    __syncthreads();
    // step j: tab[x + 2^j] = tab[x] * r_j, tab[x] *= (1 - r_j) for x < 2^j. Each thread touches
    // only its own x and x + 2^j, so a barrier between steps is the only ordering needed.
    for (int j = 0; j < k; ++j) {
        const uint32_t half = 1u << j;
        Fr rj = ld_fr(r + j), one, om;
        fe_one(one);
        fe_sub(om, one, rj);
        for (uint32_t x = threadIdx.x; x < half; x += blockDim.x) {
            Fr v = ld_fr(tab + x), a, b;
            fe_mul(a, v, om);
            fe_mul(b, v, rj);
            st_fr(tab + x, a);
            st_fr(tab + x + half, b);
        }
        __syncthreads();
    }
}

// out[i] = lo[(i + base) & mask] * hi[(i + base) >> klo],  i < count
__global__ __launch_bounds__(kThreads) void k_eq_expand(const Fr* __restrict__ lo, const Fr* __restrict__ hi, int klo,
                                                        uint64_t base, uint64_t count, Fr* __restrict__ out) {
    const uint64_t mask = (1ull << klo) - 1;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t x = i + base;
        Fr a = ld_fr(lo + (x & mask)), b = ld_fr(hi + (x >> klo)), t;
        fe_mul(t, a, b);
        st_fr(out + i, t);
    }
}

// ------------------------------------------------------------------ sumcheck #1 round
// FOLD == false (round 1): X_t = in[2b + t];            e = E[b]
// FOLD == true  (round >= 2): X'[2b+u] = in[4b+2u] + r*(in[4b+2u+1] - in[4b+2u]) stored to out,
//                             e = Ein[2b] + Ein[2b+1] stored to Eout[b]
// partial[blk] = (G(0), G(1), G(2)) with G(t) = sum_b (A_t B_t - C_t) e,  X_2 = 2 X_1 - X_0.
// need1 == 0: G(1) is left 0 (the host derives it from the previous round's claim: P(0) + P(1) = claim).
template <bool FOLD, bool FUSED>
__global__ __launch_bounds__(kThreads) void k_sc1_round(Tables3 in, Tables3 out, const Fr* __restrict__ Ein,
                                                        Fr* __restrict__ Eout, const Fr r, uint64_t half,
                                                        Fr* __restrict__ partial, uint32_t* __restrict__ ticket,
                                                        Fr* __restrict__ result3, int need1) {
    Fr g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fe_zero(g[k]);
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < half; b += (uint64_t)gridDim.x * blockDim.x) {
        Fr x0[3], x1[3], e;
        if (FOLD) {
            // every load of the pair is issued before the first store (the in/out tables may not alias,
            // but the compiler cannot know): one memory round trip per element instead of four
            Fr a[3][4], e0, e1;
#pragma unroll
            for (int m = 0; m < 3; ++m)
#pragma unroll
                for (int k = 0; k < 4; ++k) a[m][k] = ld_fr(in.t[m] + 4 * b + k);
            e0 = ld_fr(Ein + 2 * b);
            e1 = ld_fr(Ein + 2 * b + 1);
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                Fr d;
                fe_sub(d, a[m][1], a[m][0]);
                fe_mul(d, d, r);
                fe_add(x0[m], a[m][0], d);
                fe_sub(d, a[m][3], a[m][2]);
                fe_mul(d, d, r);
                fe_add(x1[m], a[m][2], d);
            }
            fe_add(e, e0, e1);
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                st_fr_fold(out.t[m] + 2 * b, x0[m]);
                st_fr_fold(out.t[m] + 2 * b + 1, x1[m]);
            }
            if (Eout) st_fr_fold(Eout + b, e);
        } else {
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                x0[m] = ld_fr(in.t[m] + 2 * b);
                x1[m] = ld_fr(in.t[m] + 2 * b + 1);
            }
            e = ld_fr(Ein + b);
        }
        Fr t, u;
        // t = 0
        fe_mul(t, x0[0], x0[1]);
        fe_sub(t, t, x0[2]);
        fe_mul(t, t, e);
        fe_add(g[0], g[0], t);
        // t = 1
        if (need1) {
            fe_mul(t, x1[0], x1[1]);
            fe_sub(t, t, x1[2]);
            fe_mul(t, t, e);
            fe_add(g[1], g[1], t);
        }
        // t = 2
        Fr y[3];
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            fe_add(u, x1[m], x1[m]);
            fe_sub(y[m], u, x0[m]);
        }
        fe_mul(t, y[0], y[1]);
        fe_sub(t, t, y[2]);
        fe_mul(t, t, e);
        fe_add(g[2], g[2], t);
    }
    if constexpr (FUSED)
        grid_reduce_last<3>(g, partial, ticket, result3);
    else
        block_reduce_store<3>(g, partial + (size_t)blockIdx.x * 3);
}

// ------------------------------------------------------------------ sumcheck #2 round
// tables M (= sum_m r_m M(r_x, .)) and Z; partial = (P(0), P(1), P(2)), P(t) = sum_b M_t Z_t
// (need1 == 0: P(1) left 0, derived on the host).
template <bool FOLD, bool FUSED>
__global__ __launch_bounds__(kThreads) void k_sc2_round(const Fr* __restrict__ Min, const Fr* __restrict__ Zin,
                                                        Fr* __restrict__ Mout, Fr* __restrict__ Zout, const Fr r,
                                                        uint64_t half, Fr* __restrict__ partial,
                                                        uint32_t* __restrict__ ticket, Fr* __restrict__ result3, int need1) {
    Fr g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fe_zero(g[k]);
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < half; b += (uint64_t)gridDim.x * blockDim.x) {
        Fr m0, m1, z0, z1;
        if (FOLD) {
            Fr d, a[4], c[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                a[k] = ld_fr(Min + 4 * b + k);
                c[k] = ld_fr(Zin + 4 * b + k);
            }
            fe_sub(d, a[1], a[0]);
            fe_mul(d, d, r);
            fe_add(m0, a[0], d);
            fe_sub(d, a[3], a[2]);
            fe_mul(d, d, r);
            fe_add(m1, a[2], d);
            fe_sub(d, c[1], c[0]);
            fe_mul(d, d, r);
            fe_add(z0, c[0], d);
            fe_sub(d, c[3], c[2]);
            fe_mul(d, d, r);
            fe_add(z1, c[2], d);
            st_fr_fold(Mout + 2 * b, m0);
            st_fr_fold(Mout + 2 * b + 1, m1);
            st_fr_fold(Zout + 2 * b, z0);
            st_fr_fold(Zout + 2 * b + 1, z1);
        } else {
            m0 = ld_fr(Min + 2 * b);
            m1 = ld_fr(Min + 2 * b + 1);
            z0 = ld_fr(Zin + 2 * b);
            z1 = ld_fr(Zin + 2 * b + 1);
        }
        Fr t, u, v;
        fe_mul(t, m0, z0);
        fe_add(g[0], g[0], t);
        if (need1) {
            fe_mul(t, m1, z1);
            fe_add(g[1], g[1], t);
        }
        fe_add(u, m1, m1);
        fe_sub(u, u, m0);
        fe_add(v, z1, z1);
        fe_sub(v, v, z0);
        fe_mul(t, u, v);
        fe_add(g[2], g[2], t);
    }
    if constexpr (FUSED)
        grid_reduce_last<3>(g, partial, ticket, result3);
    else
        block_reduce_store<3>(g, partial + (size_t)blockIdx.x * 3);
}

// ------------------------------------------------------------------ mKZG open level (open.rs:42-45)
// q[b] = r[2b+1] - r[2b];  r'[b] = r[2b] + p * q[b]   ( = r[2b](1-p) + r[2b+1] p )
// q may be null (fold only: the commitment-stubbed mode evaluates z without quotients)
__global__ __launch_bounds__(kThreads) void k_open_level(const Fr* __restrict__ rin, Fr* __restrict__ rout,
                                                         Fr* __restrict__ q, const Fr p, uint64_t half) {
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < half; b += (uint64_t)gridDim.x * blockDim.x) {
        Fr a0 = ld_fr(rin + 2 * b), a1 = ld_fr(rin + 2 * b + 1), d, t;
        fe_sub(d, a1, a0);
        if (q) st_fr(q + b, d);
        if (!rout) continue;  // quotient only (the shared level 0 of the openings)
        fe_mul(t, d, p);
        fe_add(t, a0, t);
        st_fr(rout + b, t);
    }
}

// NF consecutive levels of an opening in one launch: thread b takes the 2^NF entries
// rin[2^NF b ..] and runs the NF folds in registers, writing level j's 2^(NF-1-j) quotients to
// q_j = q + qoff[j] (j's quotients of this thread are contiguous; qoff[j] = ~0: not written) and the
// last level's value to rout[b]. The intermediate tables never go to HBM (open.rs:42-45 per level).
template <int NF>
struct FoldArgs {
    Fr p[NF];
    uint64_t qoff[NF];
};
template <int NF>
__global__ __launch_bounds__(kThreads) void k_open_fold(const Fr* __restrict__ rin, Fr* __restrict__ rout, Fr* __restrict__ q,
                                                        FoldArgs<NF> a, uint64_t nout) {
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nout; b += (uint64_t)gridDim.x * blockDim.x) {
        Fr v[1 << NF];
#pragma unroll
        for (int k = 0; k < (1 << NF); ++k) v[k] = ld_fr(rin + ((uint64_t)b << NF) + k);
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            const int m = 1 << (NF - 1 - j);  // this thread's pairs at level j
#pragma unroll
            for (int k = 0; k < m; ++k) {
                Fr d, t;
                fe_sub(d, v[2 * k + 1], v[2 * k]);
                if (a.qoff[j] != ~0ull) st_fr(q + a.qoff[j] + (uint64_t)b * m + k, d);
                fe_mul(t, d, a.p[j]);
                fe_add(v[k], v[2 * k], t);
            }
        }
        st_fr(rout + b, v[0]);
    }
}

// The last levels of an opening in ONE launch (one block, the table in LDS): level j folds
// half = h0 >> j pairs, q_j = the level's quotients (q + qoff_j, contiguous), r' as k_open_level.
// The final one-entry table goes to `last`. (Launched per level these small folds were latency: one
// launch gap each.)
static constexpr int kTailMax = 512;  // largest first half of the tail (LDS: 2 x 512 Fr)
struct TailPoints {
    Fr p[kTailMax <= 512 ? 10 : 20];
};
__global__ __launch_bounds__(kTailMax) void k_open_tail(const Fr* __restrict__ rin, Fr* __restrict__ q, uint32_t h0,
                                                        int nlev, TailPoints pts, Fr* __restrict__ last) {
    __shared__ Fr buf[2 * kTailMax];
    for (uint32_t b = threadIdx.x; b < 2 * h0; b += blockDim.x) buf[b] = ld_fr(rin + b);
    __syncthreads();
    uint32_t half = h0;
    Fr* qj = q;
    for (int j = 0; j < nlev; ++j) {
        Fr t;
        const uint32_t b = threadIdx.x;
        if (b < half) {
            const Fr a0 = buf[2 * b], a1 = buf[2 * b + 1];
            Fr d;
            fe_sub(d, a1, a0);
            if (q) st_fr(qj + b, d);
            fe_mul(t, d, pts.p[j]);
            fe_add(t, a0, t);
        }
        __syncthreads();
        if (b < half) buf[b] = t;
        __syncthreads();
        qj += half;
        half >>= 1;
    }
    if (threadIdx.x == 0) st_fr(last, buf[0]);
}

// ------------------------------------------------------------------ launchers
static inline int grid_for(uint64_t n, int cap = 2048) {
    uint64_t g = (n + kThreads - 1) / kThreads;
    if (g < 1) g = 1;
    if (g > (uint64_t)cap) g = cap;
    return (int)g;
}

void launch_to_mont(Fr* d, size_t n, int* err, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_to_mont, dim3(grid_for(n, 4096)), dim3(kThreads), 0, s, d, n, err);
}
void launch_from_mont(Fr* out, const Fr* in, size_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_from_mont, dim3(grid_for(n, 4096)), dim3(kThreads), 0, s, out, in, n);
}

void launch_sparse3(int mode, const SparseView3& mv, const Fr* vec, Fr* o0, Fr* o1, Fr* o2, const Fr* scale,
                    uint64_t count, const LongChunk* chunks, int nchunks, const LongRow* lrows, int nlrows,
                    Fr* partial, hipStream_t s) {
    if (count) {
        if (mode == 0)
            hipLaunchKernelGGL(k_sparse3<0>, dim3(grid_for(count, 8192)), dim3(kThreads), 0, s, mv, vec, o0, o1, o2,
                               scale, count);
        else
            hipLaunchKernelGGL(k_sparse3<1>, dim3(grid_for(count, 8192)), dim3(kThreads), 0, s, mv, vec, o0, o1, o2,
                               scale, count);
    }
    if (nchunks > 0) {
        hipLaunchKernelGGL(k_sparse_chunks, dim3(nchunks), dim3(kThreads), 0, s, mv, vec, chunks, partial);
        if (mode == 0)
            hipLaunchKernelGGL(k_sparse_long_finish<0>, dim3(1), dim3(64), 0, s, lrows, nlrows, partial, o0, o1, o2,
                               scale);
        else
            hipLaunchKernelGGL(k_sparse_long_finish<1>, dim3(1), dim3(64), 0, s, lrows, nlrows, partial, o0, o1, o2,
                               scale);
    }
}

void launch_eq_table(const Fr* r_dev, int k, uint64_t base, uint64_t count, Fr* out, Fr* scratch_lo,
                     Fr* scratch_hi, hipStream_t s) {
    // split k = klo + khi, each <= 13 (k <= 26): the scratch halves hold 2^13 entries
    int klo = (k + 1) / 2, khi = k - klo;
    if (k < 0 || klo > 13) throw std::invalid_argument("launch_eq_table: more than 26 variables");
    hipLaunchKernelGGL(k_eq_small, dim3(1), dim3(kThreads), 0, s, r_dev, klo, scratch_lo);
    hipLaunchKernelGGL(k_eq_small, dim3(1), dim3(kThreads), 0, s, r_dev + klo, khi, scratch_hi);
    kp_begin(KP_EQ, s);
    hipLaunchKernelGGL(k_eq_expand, dim3(grid_for(count, 8192)), dim3(kThreads), 0, s, scratch_lo, scratch_hi, klo, base,
                       count, out);
    kp_end(32.0 * (double)count, s);
}

int sc_grid(uint64_t half) { return grid_for(half, 1024); }

// Rounds whose grid has few blocks reduce in their last block (one launch); large grids keep a
// separate one-block reduction launch, so the streaming kernel's own duration carries no serial tail.
static constexpr int kFuseMaxBlocks = 64;
template <bool FOLD>
static void sc1_launch(int g, const Tables3& in, const Tables3& out, const Fr* Ein, Fr* Eout, const Fr& r, uint64_t half,
                       Fr* partial, uint32_t* ticket, Fr* result3, int need1, hipStream_t s) {
    if (g <= kFuseMaxBlocks)
        hipLaunchKernelGGL((k_sc1_round<FOLD, true>), dim3(g), dim3(kThreads), 0, s, in, out, Ein, Eout, r, half, partial,
                           ticket, result3, need1);
    else
        hipLaunchKernelGGL((k_sc1_round<FOLD, false>), dim3(g), dim3(kThreads), 0, s, in, out, Ein, Eout, r, half, partial,
                           ticket, result3, need1);
}
template <bool FOLD>
static void sc2_launch(int g, const Fr* Min, const Fr* Zin, Fr* Mout, Fr* Zout, const Fr& r, uint64_t half, Fr* partial,
                       uint32_t* ticket, Fr* result3, int need1, hipStream_t s) {
    if (g <= kFuseMaxBlocks)
        hipLaunchKernelGGL((k_sc2_round<FOLD, true>), dim3(g), dim3(kThreads), 0, s, Min, Zin, Mout, Zout, r, half, partial,
                           ticket, result3, need1);
    else
        hipLaunchKernelGGL((k_sc2_round<FOLD, false>), dim3(g), dim3(kThreads), 0, s, Min, Zin, Mout, Zout, r, half,
                           partial, ticket, result3, need1);
}

void launch_sc1_round(bool fold, const Tables3& in, const Tables3& out, const Fr* Ein, Fr* Eout, const Fr& r,
                      uint64_t half, Fr* partial, uint32_t* ticket, Fr* result3, bool need1, hipStream_t s) {
    int g = sc_grid(half);
    kp_begin(KP_SC1, s);
    if (fold)
        sc1_launch<true>(g, in, out, Ein, Eout, r, half, partial, ticket, result3, need1 ? 1 : 0, s);
    else
        sc1_launch<false>(g, in, out, Ein, Eout, r, half, partial, ticket, result3, need1 ? 1 : 0, s);
    // algorithmic bytes: fold reads 4 Fr x 3 tables + 2 E, writes 2 x 3 + 1 E; no fold reads 2 x 3 + 1
    kp_end(32.0 * (double)half * (fold ? (14.0 + 6.0 + (Eout ? 1.0 : 0.0)) : 7.0), s);
    if (g > kFuseMaxBlocks) hipLaunchKernelGGL(k_reduce_partials<3>, dim3(1), dim3(kThreads), 0, s, partial, g, result3);
}

void launch_sc2_round(bool fold, const Fr* Min, const Fr* Zin, Fr* Mout, Fr* Zout, const Fr& r, uint64_t half,
                      Fr* partial, uint32_t* ticket, Fr* result3, bool need1, hipStream_t s) {
    int g = sc_grid(half);
    kp_begin(KP_SC2, s);
    if (fold)
        sc2_launch<true>(g, Min, Zin, Mout, Zout, r, half, partial, ticket, result3, need1 ? 1 : 0, s);
    else
        sc2_launch<false>(g, Min, Zin, Mout, Zout, r, half, partial, ticket, result3, need1 ? 1 : 0, s);
    kp_end(32.0 * (double)half * (fold ? 12.0 : 4.0), s);
    if (g > kFuseMaxBlocks) hipLaunchKernelGGL(k_reduce_partials<3>, dim3(1), dim3(kThreads), 0, s, partial, g, result3);
}

int open_tail_levels(uint64_t half, int remaining) {
    if (half > (uint64_t)kTailMax || remaining < 2) return 0;
    int k = 0;
    while ((half >> k) >= 1 && k < remaining) ++k;
    return std::min(k, (int)(sizeof(TailPoints) / sizeof(Fr)));
}
void launch_open_tail(const Fr* rin, Fr* q, uint64_t half, int nlev, const Fr* points, Fr* last, hipStream_t s) {
    TailPoints tp{};
    if (nlev < 1 || nlev > (int)(sizeof(TailPoints) / sizeof(Fr)) || half > (uint64_t)kTailMax || (half >> (nlev - 1)) < 1)
        throw std::invalid_argument("launch_open_tail: bad level range");
    for (int j = 0; j < nlev; ++j) tp.p[j] = points[j];
    kp_begin(KP_OPEN, s);
    hipLaunchKernelGGL(k_open_tail, dim3(1), dim3(kTailMax), 0, s, rin, q, (uint32_t)half, nlev, tp, last);
    kp_end(32.0 * 4.0 * (double)half, s);  // read 2, write q and r' per pair, over the levels: <= 4 x half
}

void launch_open_fold(const Fr* rin, Fr* rout, Fr* q, int nf, const Fr* points, const uint64_t* qoffs, uint64_t nout,
                      hipStream_t s) {
    kp_begin(KP_OPEN, s);
    const int g = grid_for(nout, 8192);
    double qw = 0;
    for (int j = 0; j < nf; ++j) qw += qoffs[j] != ~0ull ? (double)(nout << (nf - 1 - j)) : 0.0;
    if (nf == 3) {
        FoldArgs<3> a;
        for (int j = 0; j < 3; ++j) a.p[j] = points[j], a.qoff[j] = qoffs[j];
        hipLaunchKernelGGL(k_open_fold<3>, dim3(g), dim3(kThreads), 0, s, rin, rout, q, a, nout);
    } else if (nf == 2) {
        FoldArgs<2> a;
        for (int j = 0; j < 2; ++j) a.p[j] = points[j], a.qoff[j] = qoffs[j];
        hipLaunchKernelGGL(k_open_fold<2>, dim3(g), dim3(kThreads), 0, s, rin, rout, q, a, nout);
    } else {
        throw std::invalid_argument("launch_open_fold: 2 or 3 levels");
    }
    kp_end(32.0 * ((double)(nout << nf) + qw + (double)nout), s);  // read 2^nf per output, write quotients + 1
}

void launch_open_level(const Fr* rin, Fr* rout, Fr* q, const Fr& point, uint64_t half, hipStream_t s) {
    kp_begin(KP_OPEN, s);
    hipLaunchKernelGGL(k_open_level, dim3(grid_for(half, 8192)), dim3(kThreads), 0, s, rin, rout, q, point, half);
    kp_end(32.0 * (2.0 + (q ? 1.0 : 0.0) + (rout ? 1.0 : 0.0)) * (double)half, s);  // read 2, write q and/or r'
}

}  // namespace spx
