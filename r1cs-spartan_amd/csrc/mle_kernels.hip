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
#include <type_traits>
#include <vector>
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
// folded sumcheck tables: written once, read by the next round (non-temporal stores measured no gain)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
DEV void st_fr_fold(Fr* p, const Fr& v) { store_vec(p, v); }

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
// one block per proof of a lockstep group: proof blockIdx.x's partials into its result
template <class Group>
__global__ __launch_bounds__(kThreads) void k_reduce_partials_group(Group g, int nblk) {
    const auto& j = g.j[blockIdx.x];
    Fr acc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fe_zero(acc[k]);
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
#pragma unroll
        for (int k = 0; k < 3; ++k) fe_add(acc[k], acc[k], ld_fr(j.partial + (size_t)b * 3 + k));
    }
    block_reduce_store<3>(acc, j.result3);
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
    if (gridDim.x == 1) {  // one block: its sum is the result (no hand-off)
        if (threadIdx.x == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) st_fr(out + k, acc[k]);
        }
        return;
    }
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

// sum_over_y over the column-sorted entry list (kernels.hpp: SpmvSlicedView). The list is cut into 8
// equal contiguous ranges, one per XCD: workgroup b works on range b % 8 (the dispatcher deals
// workgroups to the 8 XCDs round-robin; placement decides locality only, never correctness), chunks q,
// q + Q, ... of it (q = b / 8, Q = grid / 8). A range is 1/8 of the entries in column order, so the z
// it gathers is a contiguous ~1/8 of z, read nearly sequentially and held in that XCD's L2, instead of
// every XCD fetching a whole 128-byte line of z per 32-byte read (the CSR kernel: 2.0x its algorithmic
// bytes). Entry e: out_m[row] = val[e] * z[col[e]]; exactly one entry per (row, matrix), so products
// are stored, never accumulated. No atomics, no counters.
static constexpr uint32_t kSpmvPer = 4;  // entries per thread per chunk
DEV void k_spmv_sliced_body(SpmvSlicedView v, const Fr* __restrict__ z, Fr* o0, Fr* o1,
                            Fr* o2, uint64_t entries) {
    constexpr uint64_t kChunkE = kThreads * kSpmvPer;
    const uint64_t d = blockIdx.x & 7u, q = blockIdx.x >> 3, Q = gridDim.x >> 3;
    const uint64_t r0 = entries * d / 8, r1 = entries * (d + 1) / 8;
    for (uint64_t c0 = r0 + q * kChunkE; c0 < r1; c0 += Q * kChunkE) {
        // the chunk's kSpmvPer entries per thread: all stream loads first, then all gathers, then the
        // products (independent loads in flight together; an index past the range is clamped for the
        // loads and its store skipped)
        uint32_t col[kSpmvPer], dst[kSpmvPer];
        Fr a[kSpmvPer], zv[kSpmvPer];
#pragma unroll
        for (uint32_t j = 0; j < kSpmvPer; ++j) {
            const uint64_t i = min(c0 + j * kThreads + threadIdx.x, r1 - 1);
            col[j] = v.col[i];
            dst[j] = v.dst[i];
            a[j] = ld_fr(v.val + i);
        }
#pragma unroll
        for (uint32_t j = 0; j < kSpmvPer; ++j) zv[j] = ld_fr(z + col[j]);
#pragma unroll
        for (uint32_t j = 0; j < kSpmvPer; ++j) {
            if (c0 + j * kThreads + threadIdx.x < r1) {
                Fr t;
                fe_mul(t, a[j], zv[j]);
                const uint32_t m = dst[j] >> 30, x = dst[j] & 0x3FFFFFFFu;
                st_fr((m == 0 ? o0 : (m == 1 ? o1 : o2)) + x, t);
            }
        }
    }
}
__global__ __launch_bounds__(kThreads) void k_spmv_sliced(SpmvSlicedView v, const Fr* __restrict__ z, Fr* o0, Fr* o1,
                                                          Fr* o2, uint64_t entries) {
    k_spmv_sliced_body(v, z, o0, o1, o2, entries);
}


// eval_on_x over the column stream (kernels.hpp: ColStreamView). eq(r_x, x) is never materialised:
// it factors as lo[x & (2^klo - 1)] * hi[x >> klo] over the low and high variables (eq.rs:5-20 in
// product form), with the matrix scale r_M folded into three copies of hi (EqFactors, nf = 2:
// hi3[m << khi | x_hi] = r_M hi[x_hi]); the two tables (<= 2^13 entries each) stay in L2. An entry
// then costs one streamed 36 B (value, row | matrix), two cache-resident gathers and two Montgomery
// products, where a materialised n-entry table costs a random 32 B HBM gather plus the table's write.
// One block of 4 waves per window of 16 slices of 64 columns sorted by length (the window's output
// lines are written by one CU); wave w takes slices w, w + 4, w + 8, w + 12, so the waves of a block get
// similar totals. Lane l of a slice owns one column: its entries sit at off + 64 j + l (lane-contiguous
// loads per step), and a lane idles only for the steps between its own length and the slice's longest.
// Two Montgomery products per entry at the product's measured issue rate (~4 cycles per instruction)
// put the floor near 72 us at 2^20, well above the 19 us of its HBM bytes; loading the
// row words a step ahead measured no gain.
DEV void k_col_stream_body(ColStreamView cv, EqFactors ef, Fr* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const Fr* __restrict__ lo = ef.t[0];
    const Fr* __restrict__ hi3 = ef.t[1];
    const int klo = ef.k[0], khi = ef.k[1];
    const uint32_t mask = (1u << klo) - 1;
    auto hidx = [&](uint32_t rm) { return ((rm >> 30) << khi) | ((rm & 0x3FFFFFFFu) >> klo); };
    for (uint32_t k = wid; k < kColWindow; k += kThreads / 64) {
        const uint32_t si = blockIdx.x * kColWindow + k;
        if (si >= cv.nslices) break;
        const ColSlice sl = cv.slices[si];
        const uint32_t info = cv.lanes[(size_t)si * 64 + lane];
        const uint32_t len = info == kColNone ? 0u : info >> 26;
        Fr acc;
        fe_zero(acc);
        const uint32_t* rp = cv.rowm + sl.off + lane;
        const Fr* vp = cv.val + sl.off + lane;
        uint32_t j = 0;
        // two entries at a time: both entries' loads are in flight before the first product, and the
        // two products are independent chains
        for (; j + 1 < len; j += 2) {
            const uint32_t r0 = rp[(size_t)j * 64], r1 = rp[(size_t)(j + 1) * 64];
            Fr v0 = ld_fr(vp + (size_t)j * 64), v1 = ld_fr(vp + (size_t)(j + 1) * 64);
            Fr a0 = ld_fr(lo + (r0 & mask)), a1 = ld_fr(lo + (r1 & mask));
            Fr b0 = ld_fr(hi3 + hidx(r0)), b1 = ld_fr(hi3 + hidx(r1)), t0, t1;
            fr_mul_pair(t0, v0, a0, t1, v1, a1);
            fr_mul_pair(t0, t0, b0, t1, t1, b1);
            fe_add(acc, acc, t0);
            fe_add(acc, acc, t1);
        }
        if (j < len) {
            const uint32_t r0 = rp[(size_t)j * 64];
            Fr v0 = ld_fr(vp + (size_t)j * 64), a0 = ld_fr(lo + (r0 & mask)), b0 = ld_fr(hi3 + hidx(r0)), t0;
            fe_mul(t0, v0, a0);
            fe_mul(t0, t0, b0);
            fe_add(acc, acc, t0);
        }
        if (info != kColNone) st_fr(out + (info & 0x3FFFFFFu), acc);
    }
}
__global__ __launch_bounds__(kThreads) void k_col_stream(ColStreamView cv, EqFactors ef, Fr* __restrict__ out) {
    k_col_stream_body(cv, ef, out);
}


// long columns: one block per chunk of <= kChunk entries of one matrix; partial[chunk] = sum over the
// chunk of val * eq(r_x, row) * r_m, the factor tables read from global memory (EqFactors)
__global__ __launch_bounds__(kThreads) void k_col_chunks(SparseView3 mv, EqFactors ef, const LongChunk* __restrict__ chunks,
                                                         Fr* __restrict__ partial) {
    const LongChunk ch = chunks[blockIdx.x];
    const Fr* val = mv.val[ch.m];
    const uint32_t* idx = mv.idx[ch.m];
    const int last = ef.nf - 1;
    Fr acc[1];
    fe_zero(acc[0]);
    for (uint64_t k = ch.begin + threadIdx.x; k < ch.end; k += blockDim.x) {
        uint32_t r = idx[k];
        Fr t = ld_fr(val + k);
        for (int f = 0; f < ef.nf; ++f) {
            const uint32_t i = f == last ? ((uint32_t)ch.m << ef.k[f]) | r : r & ((1u << ef.k[f]) - 1);
            fe_mul(t, t, ld_fr(ef.t[f] + i));
            r >>= ef.k[f];
        }
        fe_add(acc[0], acc[0], t);
    }
    block_reduce_store<1>(acc, partial + blockIdx.x);
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
// eq tables of <= 13 variables, variable 0 = LSB: tab[x] = prod_{j<k} eq(r_j, x_j), eq(r, 1) = r,
// eq(r, 0) = 1 - r (eq.rs:5-20). Block f builds the table of the f-th field of ef.k (variables
// sum_{g<f} k_g ..) into ef.t[f]; the last block, if scale, writes the three scaled copies
// scale[m] tab[x] at m 2^k + x instead. Each table is the outer product of two sub-tables of <= 7
// variables computed directly in LDS (k / 2 + 1 dependent products deep, no per-variable barrier),
// one product per output entry.
static constexpr int kEqThreads = 1024;
DEV void k_eq_factors_body(const Fr* __restrict__ r, EqFactors ef,
                           const Fr* __restrict__ scale) {
    __shared__ Fr A[64], B[128 * 3];
    const int f = blockIdx.x;
    const int k = ef.k[f];
    int off = 0;
    for (int g = 0; g < f; ++g) off += ef.k[g];
    const Fr* rr = r + off;
    const int a = k / 2, b = k - a;
    const int nsc = (f == ef.nf - 1 && scale) ? 3 : 1;
    const uint32_t t = threadIdx.x;
    Fr one;
    fe_one(one);
    if (t < (1u << a) + (1u << b)) {
        const bool isA = t < (1u << a);
        const uint32_t i = isA ? t : t - (1u << a);
        const int o = isA ? 0 : a, nb = isA ? a : b;
        Fr acc = one;
        for (int j = 0; j < nb; ++j) {
            Fr rj = ld_fr(rr + o + j), fj;
            if ((i >> j) & 1)
                fj = rj;
            else
                fe_sub(fj, one, rj);
            fe_mul(acc, acc, fj);
        }
        if (isA) {
            A[i] = acc;
        } else if (nsc == 1) {
            B[i] = acc;
        } else {
            for (int m = 0; m < 3; ++m) {
                Fr sm;
                fe_mul(sm, acc, ld_fr(scale + m));
                B[m * 128 + i] = sm;
            }
        }
    }
    __syncthreads();
    const uint32_t cnt = 1u << k, amask = (1u << a) - 1;
    Fr* dst = const_cast<Fr*>(ef.t[f]);
    for (uint32_t x = t; x < cnt; x += blockDim.x) {
        const Fr ax = A[x & amask];
        for (int m = 0; m < nsc; ++m) {
            Fr v;
            fe_mul(v, ax, B[m * 128 + (x >> a)]);
            st_fr(dst + (size_t)m * cnt + x, v);
        }
    }
}
__global__ __launch_bounds__(kEqThreads) void k_eq_factors(const Fr* __restrict__ r, EqFactors ef,
                                                           const Fr* __restrict__ scale) {
    k_eq_factors_body(r, ef, scale);
}


// out[i] = lo[(i + base) & mask] * hi[(i + base) >> klo],  i < count
DEV void k_eq_expand_body(const Fr* __restrict__ lo, const Fr* __restrict__ hi, int klo,
                          uint64_t base, uint64_t count, Fr* __restrict__ out) {
    const uint64_t mask = (1ull << klo) - 1;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t x = i + base;
        Fr a = ld_fr(lo + (x & mask)), b = ld_fr(hi + (x >> klo)), t;
        fe_mul(t, a, b);
        st_fr(out + i, t);
    }
}
__global__ __launch_bounds__(kThreads) void k_eq_expand(const Fr* __restrict__ lo, const Fr* __restrict__ hi, int klo,
                                                        uint64_t base, uint64_t count, Fr* __restrict__ out) {
    k_eq_expand_body(lo, hi, klo, base, count, out);
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

// ------------------------------------------------------------------ small fold rounds, split over lanes
// The rounds of a few thousand pairs or fewer are latency: a lane's 10 (sumcheck 1) or 6 (sumcheck 2)
// dependent Fr products at one wave per SIMD. Here one pair is spread over a quad (sumcheck 1: lanes
// 0, 1, 2 fold A, B, C, lane 3 sums E; then lane 0 adds x0_A x0_B e to G(0), lane 1 adds y_A y_B e to
// G(2), lane 2 subtracts x0_C e and y_C e: 4 dependent products per lane) or a lane pair (sumcheck 2:
// lane 0 folds M, lane 1 folds Z; lane 0 adds m0 z0, lane 1 adds (2 m1 - m0)(2 z1 - z0): 3 products),
// with 4x / 2x the waves. Every lane accumulates its own share; field addition is exact, so the sums
// equal k_sc1_round's / k_sc2_round's. (For the large rounds this form measured slower than the
// per-lane one: the wave-transposed kernels below take those.)
template <int SEL>  // quad_perm: lane i of a quad reads lane SEL[2i+1:2i]
DEV Fr dpp_fr(const Fr& a) {
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v[i], SEL, 0xF, 0xF, false);
    return r;
}
DEV Fr sel_fr(bool c, const Fr& a, const Fr& b) {
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}
DEV void fold2(Fr& x0, Fr& x1, const Fr* p, const Fr& r) {  // p[0..3] -> (p0 + r(p1-p0), p2 + r(p3-p2))
    const Fr a0 = ld_fr(p), a1 = ld_fr(p + 1), a2 = ld_fr(p + 2), a3 = ld_fr(p + 3);
    Fr d;
    fe_sub(d, a1, a0);
    fe_mul(d, d, r);
    fe_add(x0, a0, d);
    fe_sub(d, a3, a2);
    fe_mul(d, d, r);
    fe_add(x1, a2, d);
}
template <bool FUSED>
DEV void sc1_fold_quad_body(const Tables3& in, const Tables3& out, const Fr* __restrict__ Ein, Fr* __restrict__ Eout,
                            const Fr& r, uint64_t half, Fr* __restrict__ partial, uint32_t* __restrict__ ticket,
                            Fr* __restrict__ result3) {
    Fr g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fe_zero(g[k]);
    const int k = threadIdx.x & 3;
    const Fr* src = k == 0 ? in.t[0] : k == 1 ? in.t[1] : k == 2 ? in.t[2] : Ein;
    Fr* dst = k == 0 ? out.t[0] : k == 1 ? out.t[1] : k == 2 ? out.t[2] : Eout;
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) >> 2;
    for (uint64_t b = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 2; b < half; b += stride) {
        Fr x0, x1;
        if (k < 3) {
            fold2(x0, x1, src + 4 * b, r);
            st_fr_fold(dst + 2 * b, x0);
            st_fr_fold(dst + 2 * b + 1, x1);
        } else {
            const Fr e0 = ld_fr(src + 2 * b), e1 = ld_fr(src + 2 * b + 1);
            fe_add(x0, e0, e1);
            x1 = x0;
            if (dst) st_fr_fold(dst + b, x0);
        }
        Fr y, P, Q;
        fe_add(y, x1, x1);
        fe_sub(y, y, x0);
        const Fr e = dpp_fr<0xFF>(x0);                       // [3,3,3,3]: lane 3's e
        const Fr recv = dpp_fr<0xB1>(sel_fr(k == 0, y, x0));  // [1,0,3,2]: lane 0 gets x0_B, lane 1 y_A
        fe_mul(P, sel_fr(k == 1, y, x0), sel_fr(k == 2, e, recv));
        fe_mul(Q, sel_fr(k == 2, y, P), e);
        if (k == 0) {
            fe_add(g[0], g[0], Q);
        } else if (k == 1) {
            fe_add(g[2], g[2], Q);
        } else if (k == 2) {
            fe_sub(g[0], g[0], P);
            fe_sub(g[2], g[2], Q);
        }
    }
    if constexpr (FUSED)
        grid_reduce_last<3>(g, partial, ticket, result3);
    else
        block_reduce_store<3>(g, partial + (size_t)blockIdx.x * 3);
}
template <bool FUSED>
__global__ __launch_bounds__(kThreads) void k_sc1_fold_quad(Tables3 in, Tables3 out, const Fr* __restrict__ Ein,
                                                            Fr* __restrict__ Eout, const Fr r, uint64_t half,
                                                            Fr* __restrict__ partial, uint32_t* __restrict__ ticket,
                                                            Fr* __restrict__ result3) {
    sc1_fold_quad_body<FUSED>(in, out, Ein, Eout, r, half, partial, ticket, result3);
}
// the same round of a lockstep group of proofs: proof blockIdx.y's job (its tables, challenge,
// partials, ticket and result), gridDim.x blocks per proof
__global__ __launch_bounds__(kThreads) void k_sc1_fold_quad_group(Sc1Group g, uint64_t half) {
    const Sc1Job& j = g.j[blockIdx.y];
    sc1_fold_quad_body<true>(j.in, j.out, j.Ein, j.Eout, j.r, half, j.partial, j.ticket, j.result3);
}
template <bool FUSED>
DEV void sc2_fold_pair_body(const Fr* __restrict__ Min, const Fr* __restrict__ Zin, Fr* __restrict__ Mout,
                            Fr* __restrict__ Zout, const Fr& r, uint64_t half, Fr* __restrict__ partial,
                            uint32_t* __restrict__ ticket, Fr* __restrict__ result3) {
    Fr g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fe_zero(g[k]);
    const int k = threadIdx.x & 1;
    const Fr* src = k ? Zin : Min;
    Fr* dst = k ? Zout : Mout;
    const uint64_t stride = ((uint64_t)gridDim.x * blockDim.x) >> 1;
    for (uint64_t b = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 1; b < half; b += stride) {
        Fr x0, x1, u, t;
        fold2(x0, x1, src + 4 * b, r);
        st_fr_fold(dst + 2 * b, x0);
        st_fr_fold(dst + 2 * b + 1, x1);
        fe_add(u, x1, x1);
        fe_sub(u, u, x0);
        const Fr recv = dpp_fr<0xB1>(sel_fr(k == 0, u, x0));  // lane 0 gets z0, lane 1 gets 2 m1 - m0
        fe_mul(t, sel_fr(k == 0, x0, u), recv);
        if (k == 0)
            fe_add(g[0], g[0], t);
        else
            fe_add(g[2], g[2], t);
    }
    if constexpr (FUSED)
        grid_reduce_last<3>(g, partial, ticket, result3);
    else
        block_reduce_store<3>(g, partial + (size_t)blockIdx.x * 3);
}
template <bool FUSED>
__global__ __launch_bounds__(kThreads) void k_sc2_fold_pair(const Fr* __restrict__ Min, const Fr* __restrict__ Zin,
                                                            Fr* __restrict__ Mout, Fr* __restrict__ Zout, const Fr r,
                                                            uint64_t half, Fr* __restrict__ partial,
                                                            uint32_t* __restrict__ ticket, Fr* __restrict__ result3) {
    sc2_fold_pair_body<FUSED>(Min, Zin, Mout, Zout, r, half, partial, ticket, result3);
}
__global__ __launch_bounds__(kThreads) void k_sc2_fold_pair_group(Sc2Group g, uint64_t half) {
    const Sc2Job& j = g.j[blockIdx.y];
    sc2_fold_pair_body<true>(j.Min, j.Zin, j.Mout, j.Zout, j.r, half, j.partial, j.ticket, j.result3);
}

// ------------------------------------------------------------------ wave-transposed fold rounds
// The large fold rounds of both sumchecks (round >= 2, P(1) derived on the host). In k_sc1_round a
// lane reads its own 128-byte runs of every table, so each 16-byte load instruction touches 64
// different cache lines and reuses each line over 8 instructions; with ~28 KB of lines in flight
// per wave the L1 cannot hold them, and the lines are fetched again from L2. Here every global load
// and store instruction is lane-contiguous (one wave covers 1 KB): a wave moves its 64 pairs'
// inputs through a wave-private LDS region (rows padded to (R + 1) x 16 B, conflict-free) and each
// lane then reads its own row. Only the wave itself touches its region, so there is no block
// barrier: LDS operations of one wave complete in order, and `wave_lds_sync` keeps the compiler from
// moving them across each other.
// 4 waves per SIMD (a few spilled registers) so a 2^20 round's 4096 waves fit one round
#define SPX_WAVE_OCC __attribute__((amdgpu_waves_per_eu(4)))
static constexpr int kWaveLdsChunks = 64 * 9;  // 16-byte chunks per wave: 64 rows of up to 8 + 1 pad
DEV Fr shfl_fr(const Fr& a, int src) {
    Fr r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = (uint32_t)__shfl((int)a.v[i], src, 64);
    return r;
}
DEV void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// a wave's block of 64 * R chunks (global, contiguous) -> registers, chunk 64 k + lane in t[k]
// (lane-contiguous loads; split from the transposition so a kernel can issue the next table's loads
// before it works on the current one)
template <int R>
DEV void wave_load(const uint4* __restrict__ g, uint4 (&t)[R], int lane) {
#pragma unroll
    for (int k = 0; k < R; ++k) t[k] = g[64 * k + lane];
}
// the loaded chunks -> lane l's row l (R chunks), through the wave's LDS region
template <int R>
DEV void wave_transpose(const uint4 (&t)[R], uint4* lds, uint4 (&row)[R], int lane) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int c = 64 * k + lane;
        lds[(c / R) * (R + 1) + c % R] = t[k];
    }
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < R; ++j) row[j] = lds[lane * (R + 1) + j];
    wave_lds_sync();
}
// a wave's block of 64 * R chunks (global, contiguous) -> lane l's row l (R chunks)
template <int R>
DEV void wave_rows_in(const uint4* __restrict__ g, uint4* lds, uint4 (&row)[R], int lane) {
    uint4 t[R];
    wave_load<R>(g, t, lane);
    wave_transpose<R>(t, lds, row, lane);
}
// lane l's row l (R chunks) -> the wave's block of 64 * R chunks (global, contiguous)
template <int R>
DEV void wave_rows_out(uint4* __restrict__ g, uint4* lds, const uint4 (&row)[R], int lane) {
#pragma unroll
    for (int j = 0; j < R; ++j) lds[lane * (R + 1) + j] = row[j];
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int c = 64 * k + lane;
        g[64 * k + lane] = lds[(c / R) * (R + 1) + c % R];
    }
    wave_lds_sync();
}
DEV Fr fr_of(const uint4& lo, const uint4& hi) {
    Fr r;
    r.v[0] = lo.x, r.v[1] = lo.y, r.v[2] = lo.z, r.v[3] = lo.w;
    r.v[4] = hi.x, r.v[5] = hi.y, r.v[6] = hi.z, r.v[7] = hi.w;
    return r;
}
DEV void fr_to(uint4& lo, uint4& hi, const Fr& a) {
    lo = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
    hi = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
// one table's 4 inputs of this lane's pair b -> (x0, x1) = (T[4b] + r (T[4b+1] - T[4b]), ...) and
// the folded pair stored to out[2b], out[2b+1]; `base` = the wave's first pair
// the same from this table's chunks already loaded by wave_load<8>
DEV void wave_fold_loaded(const uint4 (&raw)[8], Fr* __restrict__ out, uint64_t base, const Fr& r, uint4* lds, int lane,
                          Fr& x0, Fr& x1) {
    uint4 a[8];
    wave_transpose<8>(raw, lds, a, lane);
    const Fr a0 = fr_of(a[0], a[1]), a1 = fr_of(a[2], a[3]), a2 = fr_of(a[4], a[5]), a3 = fr_of(a[6], a[7]);
    Fr d0, d1;
    fe_sub(d0, a1, a0);
    fe_sub(d1, a3, a2);
    fr_mul_pair(d0, d0, r, d1, d1, r);
    fe_add(x0, a0, d0);
    fe_add(x1, a2, d1);
    uint4 o[4];
    fr_to(o[0], o[1], x0);
    fr_to(o[2], o[3], x1);
    wave_rows_out<4>(reinterpret_cast<uint4*>(out + 2 * base), lds, o, lane);
}
DEV void wave_fold(const Fr* __restrict__ in, Fr* __restrict__ out, uint64_t base, const Fr& r, uint4* lds, int lane,
                   Fr& x0, Fr& x1) {
    uint4 raw[8];
    wave_load<8>(reinterpret_cast<const uint4*>(in + 4 * base), raw, lane);
    wave_fold_loaded(raw, out, base, r, lds, lane, x0, x1);
}

// this lane's pair of one table without a fold (round 1): (T[2b], T[2b+1])
DEV void wave_pair(const Fr* __restrict__ in, uint64_t base, uint4* lds, int lane, Fr& x0, Fr& x1) {
    uint4 a[4];
    wave_rows_in<4>(reinterpret_cast<const uint4*>(in + 2 * base), lds, a, lane);
    x0 = fr_of(a[0], a[1]);
    x1 = fr_of(a[2], a[3]);
}

// sumcheck #1 round (FOLD: round >= 2 with the fold of r_{i-1}; NEED1: also G(1)), one wave per 64
// consecutive pairs (half a multiple of 64); the sums as k_sc1_round
template <bool FOLD, bool NEED1, bool FUSED>
DEV void sc1_wave_body(const Tables3& in, const Tables3& out, const Fr* __restrict__ Ein, Fr* __restrict__ Eout,
                       const Fr& r, uint64_t half, Fr* __restrict__ partial, uint32_t* __restrict__ ticket,
                       Fr* __restrict__ result3) {
    __shared__ uint4 lds_all[kThreads / 64][kWaveLdsChunks];
    uint4* lds = lds_all[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    Fr g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fe_zero(g[k]);
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < (half >> 6); w += waves) {
        const uint64_t base = w << 6;
        Fr x0[3], x1[3], e;
        if constexpr (FOLD) {
            // one table at a time: the software-pipelined form (the next table's loads issued before
            // the current one's fold) spills to 400 B of scratch per lane at 4 waves per SIMD and ran
            // 81-86 us against 59-61 (profiles/r04/r04ab_ab_pipelined.jsonl); with the products taken as
            // soon as their factors exist (only A B live) still 352 B and 73-74 us against 62-65
            // (r04ag_ab_sc1_early_products.jsonl). Sumcheck 2 and the opening folds keep it (two tables
            // / two halves: no extra spills)
#pragma unroll
            for (int m = 0; m < 3; ++m) wave_fold(in.t[m], out.t[m], base, r, lds, lane, x0[m], x1[m]);
            uint4 ev[4];
            wave_rows_in<4>(reinterpret_cast<const uint4*>(Ein + 2 * base), lds, ev, lane);
            fe_add(e, fr_of(ev[0], ev[1]), fr_of(ev[2], ev[3]));
            if (Eout) st_fr(Eout + base + lane, e);
        } else {
#pragma unroll
            for (int m = 0; m < 3; ++m) wave_pair(in.t[m], base, lds, lane, x0[m], x1[m]);
            uint4 ev[2];
            wave_rows_in<2>(reinterpret_cast<const uint4*>(Ein + base), lds, ev, lane);
            e = fr_of(ev[0], ev[1]);
        }
        Fr t, t2, u, y[3];
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            fe_add(u, x1[m], x1[m]);
            fe_sub(y[m], u, x0[m]);
        }
        // G(0) and G(2) terms as product pairs (two independent chains per wave)
        fr_mul_pair(t, x0[0], x0[1], t2, y[0], y[1]);
        fe_sub(t, t, x0[2]);
        fe_sub(t2, t2, y[2]);
        fr_mul_pair(t, t, e, t2, t2, e);
        fe_add(g[0], g[0], t);
        fe_add(g[2], g[2], t2);
        if constexpr (NEED1) {
            fe_mul(t, x1[0], x1[1]);
            fe_sub(t, t, x1[2]);
            fe_mul(t, t, e);
            fe_add(g[1], g[1], t);
        }
    }
    if constexpr (FUSED)
        grid_reduce_last<3>(g, partial, ticket, result3);
    else
        block_reduce_store<3>(g, partial + (size_t)blockIdx.x * 3);
}
template <bool FOLD, bool NEED1, bool FUSED>
__global__ __launch_bounds__(kThreads) SPX_WAVE_OCC void k_sc1_wave(Tables3 in, Tables3 out, const Fr* __restrict__ Ein,
                                                                   Fr* __restrict__ Eout, const Fr r, uint64_t half,
                                                                   Fr* __restrict__ partial, uint32_t* __restrict__ ticket,
                                                                   Fr* __restrict__ result3) {
    sc1_wave_body<FOLD, NEED1, FUSED>(in, out, Ein, Eout, r, half, partial, ticket, result3);
}
template <bool FOLD, bool NEED1, bool FUSED>
__global__ __launch_bounds__(kThreads) SPX_WAVE_OCC void k_sc1_wave_group(Sc1Group g, uint64_t half) {
    const Sc1Job& j = g.j[blockIdx.y];
    sc1_wave_body<FOLD, NEED1, FUSED>(j.in, j.out, j.Ein, j.Eout, j.r, half, j.partial, j.ticket, j.result3);
}

// sumcheck #2 round, one wave per 64 consecutive pairs; the sums as k_sc2_round
template <bool FOLD, bool NEED1, bool FUSED>
DEV void sc2_wave_body(const Fr* __restrict__ Min, const Fr* __restrict__ Zin, Fr* __restrict__ Mout,
                       Fr* __restrict__ Zout, const Fr& r, uint64_t half, Fr* __restrict__ partial,
                       uint32_t* __restrict__ ticket, Fr* __restrict__ result3) {
    __shared__ uint4 lds_all[kThreads / 64][kWaveLdsChunks];
    uint4* lds = lds_all[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    Fr g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) fe_zero(g[k]);
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < (half >> 6); w += waves) {
        const uint64_t base = w << 6;
        Fr m0, m1, z0, z1, t, u, v;
        if constexpr (FOLD) {  // Z's loads in flight while M is folded
            uint4 rm[8], rz[8];
            wave_load<8>(reinterpret_cast<const uint4*>(Min + 4 * base), rm, lane);
            wave_load<8>(reinterpret_cast<const uint4*>(Zin + 4 * base), rz, lane);
            wave_fold_loaded(rm, Mout, base, r, lds, lane, m0, m1);
            wave_fold_loaded(rz, Zout, base, r, lds, lane, z0, z1);
        } else {
            wave_pair(Min, base, lds, lane, m0, m1);
            wave_pair(Zin, base, lds, lane, z0, z1);
        }
        Fr t2;
        fe_add(u, m1, m1);
        fe_sub(u, u, m0);
        fe_add(v, z1, z1);
        fe_sub(v, v, z0);
        fr_mul_pair(t, m0, z0, t2, u, v);
        fe_add(g[0], g[0], t);
        fe_add(g[2], g[2], t2);
        if constexpr (NEED1) {
            fe_mul(t, m1, z1);
            fe_add(g[1], g[1], t);
        }
    }
    if constexpr (FUSED)
        grid_reduce_last<3>(g, partial, ticket, result3);
    else
        block_reduce_store<3>(g, partial + (size_t)blockIdx.x * 3);
}
template <bool FOLD, bool NEED1, bool FUSED>
__global__ __launch_bounds__(kThreads) SPX_WAVE_OCC void k_sc2_wave(const Fr* __restrict__ Min, const Fr* __restrict__ Zin,
                                                                   Fr* __restrict__ Mout, Fr* __restrict__ Zout, const Fr r,
                                                                   uint64_t half, Fr* __restrict__ partial,
                                                                   uint32_t* __restrict__ ticket, Fr* __restrict__ result3) {
    sc2_wave_body<FOLD, NEED1, FUSED>(Min, Zin, Mout, Zout, r, half, partial, ticket, result3);
}
template <bool FOLD, bool NEED1, bool FUSED>
__global__ __launch_bounds__(kThreads) SPX_WAVE_OCC void k_sc2_wave_group(Sc2Group g, uint64_t half) {
    const Sc2Job& j = g.j[blockIdx.y];
    sc2_wave_body<FOLD, NEED1, FUSED>(j.Min, j.Zin, j.Mout, j.Zout, j.r, half, j.partial, j.ticket, j.result3);
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
DEV void k_open_level_body(const Fr* __restrict__ rin, Fr* __restrict__ rout,
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
__global__ __launch_bounds__(kThreads) void k_open_level(const Fr* __restrict__ rin, Fr* __restrict__ rout,
                                                         Fr* __restrict__ q, const Fr p, uint64_t half) {
    k_open_level_body(rin, rout, q, p, half);
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
DEV void k_open_fold_body(const Fr* __restrict__ rin, Fr* __restrict__ rout, Fr* __restrict__ q,
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
template <int NF>
__global__ __launch_bounds__(kThreads) void k_open_fold(const Fr* __restrict__ rin, Fr* __restrict__ rout, Fr* __restrict__ q,
                                                        FoldArgs<NF> a, uint64_t nout) {
    k_open_fold_body<NF>(rin, rout, q, a, nout);
}


// k_open_fold with every global access lane-contiguous (the wave-transposed form of the sumcheck
// rounds above). A lane folds one group of 4 consecutive entries through two levels (2 + 1
// quotients, one output u): NF = 2 takes the wave's 64 outputs directly; NF = 3 takes the 128 groups
// behind its 64 outputs in two halves, and the third level combines the u of lanes 2k, 2k+1 (DPP).
DEV void fold_group4(const uint4 (&a)[8], const FoldArgs<3>& fa, int j0, Fr (&q0)[2], Fr& q1, Fr& u) {
    Fr v[4], t;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = fr_of(a[2 * k], a[2 * k + 1]);
    Fr t1;
    fe_sub(q0[0], v[1], v[0]);
    fe_sub(q0[1], v[3], v[2]);
    fr_mul_pair(t, q0[0], fa.p[j0], t1, q0[1], fa.p[j0]);  // the level's two folds: one pair
    fe_add(v[0], v[0], t);
    fe_add(v[1], v[2], t1);
    fe_sub(q1, v[1], v[0]);
    fe_mul(t, q1, fa.p[j0 + 1]);
    fe_add(u, v[0], t);
}
DEV void wave_store_q(Fr* __restrict__ q, uint64_t qoff, uint64_t first, const Fr (&q0)[2], uint4* lds, int lane) {
    uint4 o[4];
    fr_to(o[0], o[1], q0[0]);
    fr_to(o[2], o[3], q0[1]);
    wave_rows_out<4>(reinterpret_cast<uint4*>(q + qoff + 2 * first), lds, o, lane);
}
DEV void wave_store_1(Fr* __restrict__ dst, const Fr& x, uint4* lds, int lane) {
    uint4 o[2];
    fr_to(o[0], o[1], x);
    wave_rows_out<2>(reinterpret_cast<uint4*>(dst), lds, o, lane);
}
template <int NF>
DEV void k_open_fold_wave_body(const Fr* __restrict__ rin, Fr* __restrict__ rout,
                               Fr* __restrict__ q, FoldArgs<NF> a, uint64_t nout) {
    static_assert(NF == 2 || NF == 3, "2 or 3 levels");
    __shared__ uint4 lds_all[kThreads / 64][kWaveLdsChunks];
    uint4* lds = lds_all[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    FoldArgs<3> fa;  // levels j0, j0 + 1 of fold_group4
#pragma unroll
    for (int j = 0; j < NF; ++j) fa.p[j] = a.p[j];
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < (nout >> 6); w += waves) {
        const uint64_t base = w << 6;  // first output of this wave
        if constexpr (NF == 2) {
            uint4 in[8];
            wave_rows_in<8>(reinterpret_cast<const uint4*>(rin + 4 * base), lds, in, lane);
            Fr q0[2], q1, u;
            fold_group4(in, fa, 0, q0, q1, u);
            if (a.qoff[0] != ~0ull) wave_store_q(q, a.qoff[0], base, q0, lds, lane);
            if (a.qoff[1] != ~0ull) wave_store_1(q + a.qoff[1] + base, q1, lds, lane);
            wave_store_1(rout + base, u, lds, lane);
        } else {
            Fr q2 = {}, r = {};
            // both halves' loads issued up front: the second half's are in flight during the first's work
            uint4 raw0[8], raw1[8];
            wave_load<8>(reinterpret_cast<const uint4*>(rin + 4 * (2 * base)), raw0, lane);
            wave_load<8>(reinterpret_cast<const uint4*>(rin + 4 * (2 * base + 64)), raw1, lane);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint64_t grp = 2 * base + 64 * h;  // first group of this half (group = 4 entries)
                uint4 in[8];
                wave_transpose<8>(h ? raw1 : raw0, lds, in, lane);
                Fr q0[2], q1, u, t;
                fold_group4(in, fa, 0, q0, q1, u);
                if (a.qoff[0] != ~0ull) wave_store_q(q, a.qoff[0], grp, q0, lds, lane);
                if (a.qoff[1] != ~0ull) wave_store_1(q + a.qoff[1] + grp, q1, lds, lane);
                const Fr un = dpp_fr<0xB1>(u);  // [1,0,3,2]: the pair partner's u
                Fr d;
                fe_sub(d, un, u);  // even lane: u_odd - u_even = level 2's quotient
                fe_mul(t, d, a.p[2]);
                fe_add(t, u, t);
                // gather the even lanes' results of this half into lanes 32 h .. 32 h + 31
                const int src = 2 * (lane & 31);
                const Fr dq = shfl_fr(d, src), dr = shfl_fr(t, src);
                if ((lane >> 5) == h) {
                    q2 = dq;
                    r = dr;
                }
            }
            if (a.qoff[2] != ~0ull) st_fr(q + a.qoff[2] + base + lane, q2);
            st_fr(rout + base + lane, r);
        }
    }
}
template <int NF>
__global__ __launch_bounds__(kThreads) void k_open_fold_wave(const Fr* __restrict__ rin, Fr* __restrict__ rout,
                                                             Fr* __restrict__ q, FoldArgs<NF> a, uint64_t nout) {
    k_open_fold_wave_body<NF>(rin, rout, q, a, nout);
}


// The last levels of an opening in ONE launch (one block, the table in LDS): level j folds
// half = h0 >> j pairs, q_j = the level's quotients (q + qoff_j, contiguous), r' as k_open_level.
// The final one-entry table goes to `last`. (Launched per level these small folds were latency: one
// launch gap each.)
static constexpr int kTailMax = 512;  // largest first half of the tail (LDS: 2 x 512 Fr)
struct TailPoints {
    Fr p[kTailMax <= 512 ? 10 : 20];
};
DEV void k_open_tail_body(const Fr* __restrict__ rin, Fr* __restrict__ q, uint32_t h0,
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
__global__ __launch_bounds__(kTailMax) void k_open_tail(const Fr* __restrict__ rin, Fr* __restrict__ q, uint32_t h0,
                                                        int nlev, TailPoints pts, Fr* __restrict__ last) {
    k_open_tail_body(rin, q, h0, nlev, pts, last);
}


// ------------------------------------------------------------------ lockstep groups: the other steps
// The same kernels for the k proofs of a lockstep group in one launch: proof j's blocks at blockIdx.y
// = j with its own job (pointers, points), everything else shared. The bodies see blockIdx.x and
// gridDim.x of their own proof, as in the per-proof launch (k_spmv_sliced's XCD eighths included: the
// per-proof grid is a multiple of 8, so the linear workgroup id keeps blockIdx.x mod 8).
template <class J, int N = kGroupMax>
struct GroupOf {
    J j[N];
};
struct SpmvJob {
    const Fr* z;
    Fr* o[3];
};
struct EqfJob {
    const Fr* r;
    EqFactors ef;
    const Fr* scale;
};
struct EqxJob {
    const Fr* lo;
    const Fr* hi;
    Fr* out;
};
struct ColJob {
    EqFactors ef;
    Fr* out;
};
template <int NF>
struct FoldJob {
    const Fr* rin;
    Fr* rout;
    FoldArgs<NF> a;
};
struct LevelJob {
    const Fr* rin;
    Fr* rout;
    Fr p;
};
struct TailJob {
    const Fr* rin;
    Fr* last;
    TailPoints pts;
};
struct CopyJob {  // up to 3 runs of `per` Fr -> dst, back to back
    const Fr* src[3];
    Fr* dst;
};
// The group's SpMVs share one index: each entry (value, column, row | matrix: 40 B) is streamed ONCE
// and applied to the k proofs' z in turn (gather, product, store per proof), instead of once per
// proof (blockIdx.y = proof). Same XCD eighths and chunking as k_spmv_sliced_body; per proof the same
// products land in the same slots, so every proof's Az, Bz, Cz are its own launch's.
__global__ __launch_bounds__(kThreads) void k_spmv_sliced_group(SpmvSlicedView v, GroupOf<SpmvJob> g, int k,
                                                                uint64_t entries) {
    constexpr uint64_t kChunkE = kThreads * kSpmvPer;
    const uint64_t d = blockIdx.x & 7u, q = blockIdx.x >> 3, Q = gridDim.x >> 3;
    const uint64_t r0 = entries * d / 8, r1 = entries * (d + 1) / 8;
    for (uint64_t c0 = r0 + q * kChunkE; c0 < r1; c0 += Q * kChunkE) {
        uint32_t col[kSpmvPer], dst[kSpmvPer];
        Fr a[kSpmvPer];
#pragma unroll
        for (uint32_t j = 0; j < kSpmvPer; ++j) {
            const uint64_t i = min(c0 + j * kThreads + threadIdx.x, r1 - 1);
            col[j] = v.col[i];
            dst[j] = v.dst[i];
            a[j] = ld_fr(v.val + i);
        }
        // two proofs at a time: both proofs' gathers are issued before the first product (the stores of
        // one proof could otherwise alias the next proof's z as far as the compiler knows, which would
        // serialise every gather behind the previous proof's stores)
        for (int p = 0; p < k; p += 2) {
            const bool two = p + 1 < k;
            const SpmvJob& J0 = g.j[p];
            const SpmvJob& J1 = g.j[two ? p + 1 : p];
            Fr z0[kSpmvPer], z1[kSpmvPer];
#pragma unroll
            for (uint32_t j = 0; j < kSpmvPer; ++j) {
                z0[j] = ld_fr(J0.z + col[j]);
                z1[j] = ld_fr(J1.z + col[j]);
            }
#pragma unroll
            for (uint32_t j = 0; j < kSpmvPer; ++j) {
                if (c0 + j * kThreads + threadIdx.x < r1) {
                    const uint32_t m = dst[j] >> 30, x = dst[j] & 0x3FFFFFFFu;
                    Fr t0, t1;
                    if (two) {
                        fr_mul_pair(t0, a[j], z0[j], t1, a[j], z1[j]);
                        st_fr((m == 0 ? J1.o[0] : (m == 1 ? J1.o[1] : J1.o[2])) + x, t1);
                    } else {
                        fe_mul(t0, a[j], z0[j]);
                    }
                    st_fr((m == 0 ? J0.o[0] : (m == 1 ? J0.o[1] : J0.o[2])) + x, t0);
                }
            }
        }
    }
}
__global__ __launch_bounds__(kEqThreads) void k_eq_factors_group(GroupOf<EqfJob> g) {
    const EqfJob& j = g.j[blockIdx.y];
    k_eq_factors_body(j.r, j.ef, j.scale);
}
__global__ __launch_bounds__(kThreads) void k_eq_expand_group(GroupOf<EqxJob> g, int klo, uint64_t base, uint64_t count) {
    const EqxJob& j = g.j[blockIdx.y];
    k_eq_expand_body(j.lo, j.hi, klo, base, count, j.out);
}
__global__ __launch_bounds__(kThreads) void k_col_stream_group(ColStreamView cv, GroupOf<ColJob> g) {
    const ColJob& j = g.j[blockIdx.y];
    k_col_stream_body(cv, j.ef, j.out);
}
template <int NF>
__global__ __launch_bounds__(kThreads) void k_open_fold_group(GroupOf<FoldJob<NF>> g, uint64_t nout) {
    const FoldJob<NF>& j = g.j[blockIdx.y];
    k_open_fold_body<NF>(j.rin, j.rout, nullptr, j.a, nout);
}
template <int NF>
__global__ __launch_bounds__(kThreads) void k_open_fold_wave_group(GroupOf<FoldJob<NF>> g, uint64_t nout) {
    const FoldJob<NF>& j = g.j[blockIdx.y];
    k_open_fold_wave_body<NF>(j.rin, j.rout, nullptr, j.a, nout);
}
__global__ __launch_bounds__(kThreads) void k_open_level_group(GroupOf<LevelJob> g, uint64_t half) {
    const LevelJob& j = g.j[blockIdx.y];
    k_open_level_body(j.rin, j.rout, nullptr, j.p, half);
}
// (a tail job carries its points by value: 336 B, so a tail launch takes at most kTailGroup proofs and
// its arguments stay below 4 KiB)
static constexpr int kTailGroup = 8;
__global__ __launch_bounds__(kTailMax) void k_open_tail_group(GroupOf<TailJob, kTailGroup> g, uint32_t h0, int nlev) {
    const TailJob& j = g.j[blockIdx.y];
    k_open_tail_body(j.rin, nullptr, h0, nlev, j.pts, j.last);
}
static_assert(sizeof(GroupOf<TailJob, kTailGroup>) <= 4096 && sizeof(GroupOf<FoldJob<3>>) <= 4096 &&
                  sizeof(GroupOf<ColJob>) <= 4096 && sizeof(GroupOf<EqfJob>) <= 4096 && sizeof(Sc1Group) <= 4096 &&
                  sizeof(Sc2Group) <= 4096,
              "a group launch's arguments stay below 4 KiB");
// proof blockIdx.x: n runs of `per` Fr (src[i][0 .. per)) -> dst[per i ..] (host-mapped pinned memory:
// a group's small device-to-host results in one launch instead of a copy per run)
__global__ void k_copy_runs_group(GroupOf<CopyJob> g, int n, int per) {
    const CopyJob& j = g.j[blockIdx.x];
    for (int t = threadIdx.x; t < n * per; t += blockDim.x) st_fr(j.dst + t, ld_fr(j.src[t / per] + t % per));
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

void launch_spmv_sliced(const SpmvSlicedView& v, const Fr* z, Fr* o0, Fr* o1, Fr* o2, uint64_t entries, hipStream_t s) {
    // 8 x Q workgroups (a multiple of the 8 XCDs), at most 2 chunks' worth of workgroups per range
    const uint64_t per_xcd = (entries / 8 + kThreads * kSpmvPer - 1) / (kThreads * kSpmvPer);
    const unsigned Q = (unsigned)std::min<uint64_t>(256, std::max<uint64_t>(1, (per_xcd + 1) / 2));
    hipLaunchKernelGGL(k_spmv_sliced, dim3(8 * Q), dim3(kThreads), 0, s, v, z, o0, o1, o2, entries);
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

EqFactors eq_factors_for(int L, Fr* scratch) {
    EqFactors ef{};
    if (L < 1 || L > 26) throw std::invalid_argument("eq_factors_for: 1..26 variables");
    ef.nf = 2;  // lo (<= 2^13 entries) + 3 scaled copies of hi: <= kEqScratch entries, L2-resident
    ef.k[0] = (L + 1) / 2;
    ef.k[1] = L - ef.k[0];
    ef.t[0] = scratch;
    ef.t[1] = scratch + (1u << ef.k[0]);
    return ef;
}

void launch_col_stream(const ColStreamView& cv, const Fr* r_x, int L, const Fr* scale, Fr* out, Fr* eq_scratch,
                       const SparseView3& lv, const LongChunk* chunks, int nchunks, const LongRow* lrows, int nlrows,
                       Fr* partial, hipStream_t s) {
    const EqFactors ef = eq_factors_for(L, eq_scratch);
    hipLaunchKernelGGL(k_eq_factors, dim3(ef.nf), dim3(kEqThreads), 0, s, r_x, ef, scale);
    if (cv.nslices) {
        const uint32_t nwin = (cv.nslices + kColWindow - 1) / kColWindow;
        hipLaunchKernelGGL(k_col_stream, dim3(nwin), dim3(kThreads), 0, s, cv, ef, out);
    }
    if (nchunks > 0) {
        hipLaunchKernelGGL(k_col_chunks, dim3(nchunks), dim3(kThreads), 0, s, lv, ef, chunks, partial);
        hipLaunchKernelGGL(k_sparse_long_finish<0>, dim3(1), dim3(64), 0, s, lrows, nlrows, partial, out, out, out,
                           nullptr);
    }
}

void launch_eq_table(const Fr* r_dev, int k, uint64_t base, uint64_t count, Fr* out, Fr* scratch_lo,
                     Fr* scratch_hi, hipStream_t s) {
    // split k = klo + khi, each <= 13 (k <= 26): the scratch halves hold 2^13 entries
    int klo = (k + 1) / 2, khi = k - klo;
    if (k < 0 || klo > 13) throw std::invalid_argument("launch_eq_table: more than 26 variables");
    EqFactors ef{};
    ef.nf = 2;
    ef.k[0] = klo;
    ef.k[1] = khi;
    ef.t[0] = scratch_lo;
    ef.t[1] = scratch_hi;
    hipLaunchKernelGGL(k_eq_factors, dim3(2), dim3(kEqThreads), 0, s, r_dev, ef, nullptr);
    kp_begin(KP_EQ, s);
    hipLaunchKernelGGL(k_eq_expand, dim3(grid_for(count, 8192)), dim3(kThreads), 0, s, scratch_lo, scratch_hi, klo, base,
                       count, out);
    kp_end(32.0 * (double)count, s);
}

int sc_grid(uint64_t half) { return grid_for(half, 1024); }

// Rounds whose grid has few blocks reduce in their last block (one launch); large grids keep a
// separate one-block reduction launch, so the streaming kernel's own duration carries no serial tail.
static constexpr int kFuseMaxBlocks = 64;
// wave-transposed fold rounds (k_sc1_fold_wave, k_sc2_fold_wave) for the large rounds only (whole
// waves of 64 pairs; grids of <= kFuseMaxBlocks blocks reduce in their last block, as k_sc1_round)
static constexpr uint64_t kWaveMinHalf = 1u << 14;
static constexpr int kWaveMaxBlocks = (int)(kRoundPartials / 3);
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

template <bool FOLD, bool NEED1>
static void sc1_wave_launch(int g, const Tables3& in, const Tables3& out, const Fr* Ein, Fr* Eout, const Fr& r,
                            uint64_t half, Fr* partial, uint32_t* ticket, Fr* result3, hipStream_t s) {
    if (g <= kFuseMaxBlocks)
        hipLaunchKernelGGL((k_sc1_wave<FOLD, NEED1, true>), dim3(g), dim3(kThreads), 0, s, in, out, Ein, Eout, r, half,
                           partial, ticket, result3);
    else
        hipLaunchKernelGGL((k_sc1_wave<FOLD, NEED1, false>), dim3(g), dim3(kThreads), 0, s, in, out, Ein, Eout, r, half,
                           partial, ticket, result3);
}
template <bool FOLD, bool NEED1>
static void sc2_wave_launch(int g, const Fr* Min, const Fr* Zin, Fr* Mout, Fr* Zout, const Fr& r, uint64_t half,
                            Fr* partial, uint32_t* ticket, Fr* result3, hipStream_t s) {
    if (g <= kFuseMaxBlocks)
        hipLaunchKernelGGL((k_sc2_wave<FOLD, NEED1, true>), dim3(g), dim3(kThreads), 0, s, Min, Zin, Mout, Zout, r, half,
                           partial, ticket, result3);
    else
        hipLaunchKernelGGL((k_sc2_wave<FOLD, NEED1, false>), dim3(g), dim3(kThreads), 0, s, Min, Zin, Mout, Zout, r,
                           half, partial, ticket, result3);
}

void launch_sc1_round(bool fold, const Tables3& in, const Tables3& out, const Fr* Ein, Fr* Eout, const Fr& r,
                      uint64_t half, Fr* partial, uint32_t* ticket, Fr* result3, bool need1, hipStream_t s) {
    int g = sc_grid(half);
    kp_begin(KP_SC1, s);
    if (half >= kWaveMinHalf) {
        g = grid_for(half, kWaveMaxBlocks);
        if (fold && need1)
            sc1_wave_launch<true, true>(g, in, out, Ein, Eout, r, half, partial, ticket, result3, s);
        else if (fold)
            sc1_wave_launch<true, false>(g, in, out, Ein, Eout, r, half, partial, ticket, result3, s);
        else if (need1)
            sc1_wave_launch<false, true>(g, in, out, Ein, Eout, r, half, partial, ticket, result3, s);
        else
            sc1_wave_launch<false, false>(g, in, out, Ein, Eout, r, half, partial, ticket, result3, s);
    } else if (fold && !need1) {  // small fold round: quad per pair, last-block reduction
        g = grid_for(4 * half, kFuseMaxBlocks);
        hipLaunchKernelGGL(k_sc1_fold_quad<true>, dim3(g), dim3(kThreads), 0, s, in, out, Ein, Eout, r, half, partial,
                           ticket, result3);
    } else if (fold)
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
    if (half >= kWaveMinHalf) {
        g = grid_for(half, kWaveMaxBlocks);
        if (fold && need1)
            sc2_wave_launch<true, true>(g, Min, Zin, Mout, Zout, r, half, partial, ticket, result3, s);
        else if (fold)
            sc2_wave_launch<true, false>(g, Min, Zin, Mout, Zout, r, half, partial, ticket, result3, s);
        else if (need1)
            sc2_wave_launch<false, true>(g, Min, Zin, Mout, Zout, r, half, partial, ticket, result3, s);
        else
            sc2_wave_launch<false, false>(g, Min, Zin, Mout, Zout, r, half, partial, ticket, result3, s);
    } else if (fold && !need1) {  // small fold round: lane pair per pair
        g = grid_for(2 * half, kFuseMaxBlocks);
        hipLaunchKernelGGL(k_sc2_fold_pair<true>, dim3(g), dim3(kThreads), 0, s, Min, Zin, Mout, Zout, r, half, partial,
                           ticket, result3);
    } else if (fold)
        sc2_launch<true>(g, Min, Zin, Mout, Zout, r, half, partial, ticket, result3, need1 ? 1 : 0, s);
    else
        sc2_launch<false>(g, Min, Zin, Mout, Zout, r, half, partial, ticket, result3, need1 ? 1 : 0, s);
    kp_end(32.0 * (double)half * (fold ? 12.0 : 4.0), s);
    if (g > kFuseMaxBlocks) hipLaunchKernelGGL(k_reduce_partials<3>, dim3(1), dim3(kThreads), 0, s, partial, g, result3);
}

// ---- lockstep groups: the launch decisions of launch_sc1_round / launch_sc2_round, one launch for k
// proofs (grid gridDim.x per proof, blockIdx.y = proof). Round shapes without a group kernel (small
// rounds that need G(1), or a round 1 below kWaveMinHalf) launch per proof.
template <class Group, class Job>
static Group group_of(int k, const Job* jobs) {
    if (k < 1 || k > kGroupMax) throw std::invalid_argument("lockstep group size out of range");
    Group g{};
    for (int i = 0; i < k; ++i) g.j[i] = jobs[i];
    return g;
}
template <bool FOLD, bool NEED1>
static void sc1_wave_group_launch(int k, int g, const Sc1Group& G, uint64_t half, hipStream_t s) {
    if (g <= kFuseMaxBlocks)
        hipLaunchKernelGGL((k_sc1_wave_group<FOLD, NEED1, true>), dim3(g, k), dim3(kThreads), 0, s, G, half);
    else
        hipLaunchKernelGGL((k_sc1_wave_group<FOLD, NEED1, false>), dim3(g, k), dim3(kThreads), 0, s, G, half);
}
template <bool FOLD, bool NEED1>
static void sc2_wave_group_launch(int k, int g, const Sc2Group& G, uint64_t half, hipStream_t s) {
    if (g <= kFuseMaxBlocks)
        hipLaunchKernelGGL((k_sc2_wave_group<FOLD, NEED1, true>), dim3(g, k), dim3(kThreads), 0, s, G, half);
    else
        hipLaunchKernelGGL((k_sc2_wave_group<FOLD, NEED1, false>), dim3(g, k), dim3(kThreads), 0, s, G, half);
}
void launch_sc1_round_group(int k, bool fold, const Sc1Job* jobs, uint64_t half, bool need1, hipStream_t s) {
    const Sc1Group G = group_of<Sc1Group>(k, jobs);
    if (half < kWaveMinHalf && !(fold && !need1)) {
        for (int i = 0; i < k; ++i)
            launch_sc1_round(fold, jobs[i].in, jobs[i].out, jobs[i].Ein, jobs[i].Eout, jobs[i].r, half, jobs[i].partial,
                             jobs[i].ticket, jobs[i].result3, need1, s);
        return;
    }
    int g;
    kp_begin(KP_SC1, s);
    if (half >= kWaveMinHalf) {
        g = grid_for(half, kWaveMaxBlocks);
        if (fold && need1)
            sc1_wave_group_launch<true, true>(k, g, G, half, s);
        else if (fold)
            sc1_wave_group_launch<true, false>(k, g, G, half, s);
        else if (need1)
            sc1_wave_group_launch<false, true>(k, g, G, half, s);
        else
            sc1_wave_group_launch<false, false>(k, g, G, half, s);
    } else {  // small fold round without G(1)
        g = grid_for(4 * half, kFuseMaxBlocks);
        hipLaunchKernelGGL(k_sc1_fold_quad_group, dim3(g, k), dim3(kThreads), 0, s, G, half);
    }
    kp_end(32.0 * (double)k * (double)half * (fold ? (14.0 + 6.0 + (jobs[0].Eout ? 1.0 : 0.0)) : 7.0), s);
    if (g > kFuseMaxBlocks)
        hipLaunchKernelGGL(k_reduce_partials_group<Sc1Group>, dim3(k), dim3(kThreads), 0, s, G, g);
}
void launch_sc2_round_group(int k, bool fold, const Sc2Job* jobs, uint64_t half, bool need1, hipStream_t s) {
    const Sc2Group G = group_of<Sc2Group>(k, jobs);
    if (half < kWaveMinHalf && !(fold && !need1)) {
        for (int i = 0; i < k; ++i)
            launch_sc2_round(fold, jobs[i].Min, jobs[i].Zin, jobs[i].Mout, jobs[i].Zout, jobs[i].r, half, jobs[i].partial,
                             jobs[i].ticket, jobs[i].result3, need1, s);
        return;
    }
    int g;
    kp_begin(KP_SC2, s);
    if (half >= kWaveMinHalf) {
        g = grid_for(half, kWaveMaxBlocks);
        if (fold && need1)
            sc2_wave_group_launch<true, true>(k, g, G, half, s);
        else if (fold)
            sc2_wave_group_launch<true, false>(k, g, G, half, s);
        else if (need1)
            sc2_wave_group_launch<false, true>(k, g, G, half, s);
        else
            sc2_wave_group_launch<false, false>(k, g, G, half, s);
    } else {  // small fold round without P(1)
        g = grid_for(2 * half, kFuseMaxBlocks);
        hipLaunchKernelGGL(k_sc2_fold_pair_group, dim3(g, k), dim3(kThreads), 0, s, G, half);
    }
    kp_end(32.0 * (double)k * (double)half * (fold ? 12.0 : 4.0), s);
    if (g > kFuseMaxBlocks)
        hipLaunchKernelGGL(k_reduce_partials_group<Sc2Group>, dim3(k), dim3(kThreads), 0, s, G, g);
}

// ---- the other steps of a lockstep group (prove_group), one launch per step for the k proofs
template <class J>
static GroupOf<J> group_check(int k) {
    if (k < 1 || k > kGroupMax) throw std::invalid_argument("lockstep group size out of range");
    return GroupOf<J>{};
}
void launch_spmv_sliced_group(int k, const SpmvSlicedView& v, const Fr* const* z, const Tables3* out, uint64_t entries,
                              hipStream_t s) {
    GroupOf<SpmvJob> g = group_check<SpmvJob>(k);
    for (int i = 0; i < k; ++i) g.j[i] = SpmvJob{z[i], {out[i].t[0], out[i].t[1], out[i].t[2]}};
    const uint64_t per_xcd = (entries / 8 + kThreads * kSpmvPer - 1) / (kThreads * kSpmvPer);
    // k proofs per entry: as many workgroups as one proof's launch has, each doing k proofs' products
    const uint32_t Q = (uint32_t)std::min<uint64_t>(256, std::max<uint64_t>(1, per_xcd));
    hipLaunchKernelGGL(k_spmv_sliced_group, dim3(8 * Q), dim3(kThreads), 0, s, v, g, k, entries);
}
void launch_eq_table_group(int k, const Fr* const* r_dev, int nvar, uint64_t base, uint64_t count, Fr* const* out,
                           Fr* const* lo, Fr* const* hi, hipStream_t s) {
    const int klo = (nvar + 1) / 2, khi = nvar - klo;
    if (nvar < 0 || klo > 13) throw std::invalid_argument("launch_eq_table_group: more than 26 variables");
    GroupOf<EqfJob> gf = group_check<EqfJob>(k);
    GroupOf<EqxJob> gx = group_check<EqxJob>(k);
    for (int i = 0; i < k; ++i) {
        EqFactors ef{};
        ef.nf = 2;
        ef.k[0] = klo;
        ef.k[1] = khi;
        ef.t[0] = lo[i];
        ef.t[1] = hi[i];
        gf.j[i] = EqfJob{r_dev[i], ef, nullptr};
        gx.j[i] = EqxJob{lo[i], hi[i], out[i]};
    }
    hipLaunchKernelGGL(k_eq_factors_group, dim3(2, k), dim3(kEqThreads), 0, s, gf);
    kp_begin(KP_EQ, s);
    hipLaunchKernelGGL(k_eq_expand_group, dim3(grid_for(count, 8192), k), dim3(kThreads), 0, s, gx, klo, base, count);
    kp_end(32.0 * (double)count * k, s);
}
void launch_col_stream_group(int k, const ColStreamView& cv, const Fr* const* r_x, int L, const Fr* const* scale,
                             Fr* const* out, Fr* const* eq_scratch, hipStream_t s) {
    GroupOf<EqfJob> gf = group_check<EqfJob>(k);
    GroupOf<ColJob> gc = group_check<ColJob>(k);
    int nf = 0;
    for (int i = 0; i < k; ++i) {
        const EqFactors ef = eq_factors_for(L, eq_scratch[i]);
        nf = ef.nf;
        gf.j[i] = EqfJob{r_x[i], ef, scale[i]};
        gc.j[i] = ColJob{ef, out[i]};
    }
    hipLaunchKernelGGL(k_eq_factors_group, dim3(nf, k), dim3(kEqThreads), 0, s, gf);
    if (cv.nslices) {
        const uint32_t nwin = (cv.nslices + kColWindow - 1) / kColWindow;
        hipLaunchKernelGGL(k_col_stream_group, dim3(nwin, k), dim3(kThreads), 0, s, cv, gc);
    }
}
void launch_open_eval_group(int k, const Fr* const* z, Fr* const* bufA, Fr* const* bufB, const Fr* points, int L,
                            uint64_t n, Fr* const* last, hipStream_t s) {
    group_check<LevelJob>(k);
    std::vector<const Fr*> rin(z, z + k);
    kp_begin(KP_OPEN, s);
    bool tail = false;
    int nb = 0;
    for (int i = 0; i < L;) {
        Fr* const* rout = (nb++ & 1) ? bufB : bufA;
        const uint64_t half = n >> (i + 1);
        if (open_tail_levels(half, L - i) == L - i) {  // the remaining levels, straight into `last`
            for (int j0 = 0; j0 < k; j0 += kTailGroup) {
                const int kk = std::min(kTailGroup, k - j0);
                GroupOf<TailJob, kTailGroup> g{};
                for (int j = 0; j < kk; ++j) {
                    g.j[j].rin = rin[j0 + j];
                    g.j[j].last = last[j0 + j];
                    for (int q = i; q < L; ++q) g.j[j].pts.p[q - i] = points[(size_t)(j0 + j) * L + q];
                }
                hipLaunchKernelGGL(k_open_tail_group, dim3(1, kk), dim3(kTailMax), 0, s, g, (uint32_t)half, L - i);
            }
            tail = true;
            break;
        }
        const int nf = L - i >= 3 && (half >> 2) >= 1 ? 3 : (L - i >= 2 && (half >> 1) >= 1 ? 2 : 1);
        const uint64_t nout = n >> (i + nf);
        if (nf == 3 || nf == 2) {
            auto run = [&](auto tag) {
                constexpr int NF = decltype(tag)::value;
                GroupOf<FoldJob<NF>> g{};
                for (int j = 0; j < k; ++j) {
                    g.j[j].rin = rin[j];
                    g.j[j].rout = rout[j];
                    for (int q = 0; q < NF; ++q) g.j[j].a.p[q] = points[(size_t)j * L + i + q], g.j[j].a.qoff[q] = ~0ull;
                }
                if (nout >= kWaveMinHalf)
                    hipLaunchKernelGGL(k_open_fold_wave_group<NF>, dim3(grid_for(nout, 8192), k), dim3(kThreads), 0, s, g,
                                       nout);
                else
                    hipLaunchKernelGGL(k_open_fold_group<NF>, dim3(grid_for(nout, 8192), k), dim3(kThreads), 0, s, g, nout);
            };
            if (nf == 3)
                run(std::integral_constant<int, 3>{});
            else
                run(std::integral_constant<int, 2>{});
        } else {
            GroupOf<LevelJob> g{};
            for (int j = 0; j < k; ++j) g.j[j] = LevelJob{rin[j], rout[j], points[(size_t)j * L + i]};
            hipLaunchKernelGGL(k_open_level_group, dim3(grid_for(half, 8192), k), dim3(kThreads), 0, s, g, half);
        }
        for (int j = 0; j < k; ++j) rin[j] = rout[j];
        i += nf;
    }
    kp_end(32.0 * 2.0 * (double)n * k, s);  // reads ~2n over the levels, writes ~n
    if (!tail) {  // the chain ended on a fold: its one-entry table to `last`
        GroupOf<CopyJob> g{};
        for (int j = 0; j < k; ++j) g.j[j] = CopyJob{{rin[j], nullptr, nullptr}, last[j]};
        hipLaunchKernelGGL(k_copy_runs_group, dim3(k), dim3(64), 0, s, g, 1, 1);
    }
}
void launch_copy_runs_group(int k, const Tables3* src, int nruns, int per, Fr* const* dst, hipStream_t s) {
    GroupOf<CopyJob> g = group_check<CopyJob>(k);
    if (nruns < 1 || nruns > 3 || per < 1 || nruns * per > 4096) throw std::invalid_argument("launch_copy_runs_group");
    for (int j = 0; j < k; ++j) g.j[j] = CopyJob{{src[j].t[0], src[j].t[1], src[j].t[2]}, dst[j]};
    hipLaunchKernelGGL(k_copy_runs_group, dim3(k), dim3(256), 0, s, g, nruns, per);
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
    const bool wave = nout >= kWaveMinHalf;  // whole waves of 64 outputs
    if (nf == 3) {
        FoldArgs<3> a;
        for (int j = 0; j < 3; ++j) a.p[j] = points[j], a.qoff[j] = qoffs[j];
        if (wave)
            hipLaunchKernelGGL(k_open_fold_wave<3>, dim3(grid_for(nout, 8192)), dim3(kThreads), 0, s, rin, rout, q, a, nout);
        else
            hipLaunchKernelGGL(k_open_fold<3>, dim3(g), dim3(kThreads), 0, s, rin, rout, q, a, nout);
    } else if (nf == 2) {
        FoldArgs<2> a;
        for (int j = 0; j < 2; ++j) a.p[j] = points[j], a.qoff[j] = qoffs[j];
        if (wave)
            hipLaunchKernelGGL(k_open_fold_wave<2>, dim3(grid_for(nout, 8192)), dim3(kThreads), 0, s, rin, rout, q, a, nout);
        else
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
