// Pippenger multi-scalar multiplication for G1 (commit, commit.rs:25) and G2 (opening proofs,
// open.rs:49), plus the public-parameter preprocessing and fixed-base keygen kernels.
//
// Design (MI355X-first, HBM capacity traded for latency):
//  * PP preprocessing stores, for every base B_j, the W window copies 2^(c w) B_j as affine
//    points, so all windows of an MSM share ONE set of 2^(c-1) signed-digit buckets and no
//    window-combination doubling chain is ever run (that chain is a ~255-step serial dependency
//    on a single lane). G2 bases of open level i are pre-summed pairs raw[2b] + raw[2b+1],
//    because open.rs:46 feeds every quotient scalar twice (q_k[x >> 1]); the MSM result is
//    identical and half the size.
//  * Signed c-bit digits -> (bucket, reference) pairs placed in bucket order by a hand-written
//    two-level counting sort with LDS histograms (k_sort_*: five launches, no global atomic per pair,
//    no library kernel), which also yields every partial level's offsets. References are 32-bit
//    point indices with the sign in bit 31. Order inside a bucket is irrelevant: group addition is
//    exact and commutative, the affine result is unique.
//  * Proof-sharded ranks split every instance by BUCKET range (MsmShard, kernels.hpp): each rank
//    digitises all scalars but keeps only its range's digits (compacted), so every stage after the
//    digit pass divides by the world size, the bucket weighting included.
//  * Bucket accumulation in XYZZ coordinates: the affine level gives every thread the same number
//    of consecutive references of the sorted array across bucket boundaries (a thread crossing a
//    boundary stores a partial and restarts), then XYZZ levels over the partials of each bucket,
//    as many as the expected occupancy needs; the weighting leaf adds whatever partials remain.
//  * Bucket weighting sum_j j S_j as a low-depth (F, S, D) tree (msm_impl.hpp).
// Many MSMs run as one batch (all nv levels of an opening), and nothing in it waits for the host.
#include "msm_common.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdlib>

namespace spx {

__device__ __constant__ constexpr uint32_t kFqR2[12] = {0x1c341746u, 0xf4df1f34u, 0x09d104f1u, 0x0a76e6a6u,
                                                       0x4c95b6d5u, 0x8de5476cu, 0x939d83c0u, 0x67eb88a9u,
                                                       0xb519952du, 0x9a793e85u, 0x92cae3aau, 0x11988fe5u};

// ------------------------------------------------------------------ digits -> (bucket, reference) keys
// Signed c-bit digits of a canonical scalar, least significant window first.
struct Digits {
    uint32_t s[8];
    uint32_t carry = 0;
    DEV int32_t next(uint32_t c) {
        const uint32_t full = 1u << c, half = full >> 1;
        uint32_t v = (s[0] & (full - 1)) + carry;
#pragma unroll
        for (int k = 0; k < 7; ++k) s[k] = (s[k] >> c) | (s[k + 1] << (32 - c));
        s[7] >>= c;
        carry = v > half;
        return carry ? (int32_t)v - (int32_t)full : (int32_t)v;
    }
    // c = 16 (every MSM of >= 2^14 points): window w is half-word w of the scalar, so nothing is
    // shifted (w a constant in the unrolled loops); the same signed digits as next(16) in order
    DEV int32_t at16(uint32_t w) {
        const uint32_t v = ((s[w >> 1] >> (16 * (w & 1))) & 0xFFFFu) + carry;
        carry = v > 0x8000u;
        return carry ? (int32_t)v - 0x10000 : (int32_t)v;
    }
};
// the digit's bucket if it is one of this rank's (local index in the batch), else ~0u
DEV uint32_t digit_key(const MsmInst& I, int32_t d) {
    if (!d) return ~0u;
    const uint32_t u = (uint32_t)(d < 0 ? -d : d) - 1;  // 0 .. 2^(c-1) - 1
    if ((u & ((1u << I.lg) - 1)) != I.sel) return ~0u;
    return I.bucket_off + (u >> I.lg);
}
DEV uint32_t digit_ref(const MsmInst& I, uint32_t w, uint64_t j, int32_t d) {
    return (uint32_t)(I.pts_off + (uint64_t)w * I.stride + j) | (d < 0 ? 0x80000000u : 0u);
}
// The digits of batch scalar g that land in one of this rank's buckets. c = 16 with 16 windows (every
// MSM of >= 2^14 points): all 16 keys and references into registers (unrolled: static indices), so a
// caller can issue their 16 LDS atomics back to back; otherwise f(key, ref) per digit.
struct Keys16 {
    uint32_t key[16], ref[16];  // key ~0u: not this rank's / zero digit
};
template <class Fn>
DEV bool scalar_keys(const MsmInst* __restrict__ insts, const uint64_t* __restrict__ prefix, int nact,
                     const Fr* __restrict__ scalars, uint64_t g, Keys16& k16, Fn&& f) {
    const int i = find_slot(prefix, nact, g);
    const uint64_t j = g - prefix[i];
    const MsmInst I = insts[i];
    Fr m, sc;
    load_vec(m, scalars + I.scalar_off + j);
    fe_from_mont(sc, m);
    Digits d;
#pragma unroll
    for (int k = 0; k < 8; ++k) d.s[k] = sc.v[k];
    if (I.c == 16 && I.W == 16) {
#pragma unroll
        for (uint32_t w = 0; w < 16; ++w) {
            const int32_t dg = d.at16(w);
            k16.key[w] = digit_key(I, dg);
            k16.ref[w] = digit_ref(I, w, j, dg);
        }
        return true;
    }
    for (uint32_t w = 0; w < I.W; ++w) {
        const int32_t dg = d.next(I.c);
        const uint32_t key = digit_key(I, dg);
        if (key != ~0u) f(key, digit_ref(I, w, j, dg));
    }
    return false;
}

// ------------------------------------------------------------------ the bucket sort (hand-written)
// The (bucket, reference) pairs of a batch are placed in bucket order by a two-level counting sort
// whose histograms live in LDS; no global atomic is taken per pair (per-lane global atomics to
// scattered words run at ~0.08 TB/s on this chip, MI355X_MICROARCH.md "Global float atomics"), and
// both scatter passes stage their pairs in LDS so that the global writes are contiguous runs (a wave
// store to 64 different lines is what bounded the first, unstaged form):
//   bins    = ranges of 2^sb consecutive buckets (the batch's nb buckets in nbin <= kMaxBins bins),
//             sized so that a bin's expected pairs fit k_sort_bins's LDS staging;
//   tiles   = ranges of kTileThreads x spt consecutive batch scalars (one workgroup each).
//   K1 k_sort_count  : per tile, digits -> LDS histogram over bins -> column `tile` of cnt[bin][tile];
//                      block 0 also zeroes the batch's outputs and status words (no fill launch)
//   K2 k_sort_scan   : per bin, the exclusive scan of its row over the tiles (in place) and the bin's
//                      total; the last block to finish scans the totals into binbase and checks the
//                      capacity (compacted keys of a sharded rank: overflow -> empty buckets, rerun)
//   K3 k_sort_scatter: per tile, the same digits again, kTileThreads scalars at a time: LDS ranks per
//                      bin, the pairs ordered by bin in LDS, then written (reference, in-bin bucket)
//                      as runs at binbase[bin] + row prefix into the bin-partitioned staging
//   K4 k_sort_bins   : per bin, an LDS histogram over its <= 256 buckets, their offsets, and every
//                      partial level's per-bucket counts (they depend on the bucket's global offset,
//                      which is known here) scanned inside the bin; the references ordered by bucket
//                      in LDS and written back contiguously; the last block scans the bins' partial totals
//   K5 k_sort_final  : each partial level's offsets += the bin's base.
// Order inside a bucket follows LDS atomics and may differ between runs: group addition is exact and
// the affine result unique, so every output is identical.
static constexpr int kTileThreads = 1024;     // K1, K3: one workgroup per tile
static constexpr int kRowThreads = 1024;      // K2
static constexpr int kScanThreads = 256;      // K5
static constexpr int kBinThreads = 1024;      // K4: one workgroup per bin
static constexpr uint32_t kMaxBins = 2048;    // K1 / K3: LDS words per bin
static constexpr uint32_t kStagePairs = (uint32_t)kTileThreads * 16;  // K3: one iteration's pairs (<= 16 per scalar)
static constexpr uint32_t kBinStage = 36864;  // K4: a bin's references ordered in LDS (144 KB); larger bins write directly
static constexpr int kMaxLev = 8;             // XYZZ partial levels the sort prepares offsets for
typedef __attribute__((address_space(1))) unsigned int gu32;

struct SortGeom {
    uint32_t nb, sb, nbin;  // buckets; in-bin bits (<= 8); bins = ceil(nb / 2^sb)
    uint32_t spt, ntile;    // scalars per thread; tiles of (sub x kCountThreads) x spt scalars
    uint32_t sub;           // K1 workgroups per tile: kSub (staged form) or 1 (direct form)
    uint64_t tot_sc;
};

// block-wide exclusive scan of one value per thread (NT threads); agg = the block's total.
// `sh` holds >= NT / 64 words of LDS; reusable after the call returns.
template <int NT>
DEV uint32_t block_excl_scan(uint32_t v, uint32_t& agg, uint32_t* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint32_t pre = 0;
    agg = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        const uint32_t t = sh[k];
        pre += k < w ? t : 0u;
        agg += t;
    }
    __syncthreads();
    return pre + x - v;
}
// hand-off to the launch's last block (cdna_hip_programming.md §6 G16, write-through form, as
// grid_reduce_last in mle_kernels.hip): thread 0 stores the block's words with agent-scope (sc1)
// stores, drains them, and takes a ticket; true in every thread of the block that drew the last one
DEV bool handoff_last(uint32_t* __restrict__ ticket, uint32_t ntickets, bool* flag) {
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *flag = __hip_atomic_fetch_add((gu32*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ntickets - 1;
    }
    __syncthreads();
    return *flag;
}
DEV void st_agent(uint32_t* p, uint32_t v) { __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV uint32_t ld_agent(const uint32_t* p) { return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// K1 runs kSub workgroups of kCountThreads per tile (more, smaller workgroups than K3's: K1 is the
// digit extraction alone); sub-unit u counts scalars [u, u + 1) x kCountThreads x spt, so the kSub
// sub-units of tile t cover exactly its scalars, and column kSub t of a scanned row is the tile's prefix
static constexpr int kCountThreads = 256, kSub = kTileThreads / kCountThreads;
static constexpr int kDirectThreads = kCountThreads;  // K3 / K4 of the direct form
__global__ __launch_bounds__(kCountThreads) void k_sort_count(const MsmInst* __restrict__ insts, const uint64_t* __restrict__ prefix,
                                                              int nact, const Fr* __restrict__ scalars, SortGeom g,
                                                              uint32_t* __restrict__ cnt, uint32_t* __restrict__ zero_dst,
                                                              uint32_t zero_words) {
    __shared__ uint32_t h[kMaxBins];
    for (uint32_t b = threadIdx.x; b < g.nbin; b += kCountThreads) h[b] = 0;
    if (blockIdx.x == 0)
        for (uint32_t i = threadIdx.x; i < zero_words; i += kCountThreads) zero_dst[i] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kCountThreads * g.spt + threadIdx.x;
    for (uint32_t k = 0; k < g.spt; ++k) {
        const uint64_t gi = t0 + (uint64_t)k * kCountThreads;
        if (gi >= g.tot_sc) break;
        Keys16 kk;
        auto add = [&](uint32_t key, uint32_t) { atomicAdd(&h[key >> g.sb], 1u); };
        if (scalar_keys(insts, prefix, nact, scalars, gi, kk, add)) {
#pragma unroll
            for (int w = 0; w < 16; ++w)
                if (kk.key[w] != ~0u) add(kk.key[w], 0u);
        }
    }
    __syncthreads();
    const uint32_t ncol = g.ntile * g.sub;
    for (uint32_t b = threadIdx.x; b < g.nbin; b += kCountThreads) cnt[(size_t)b * ncol + blockIdx.x] = h[b];
}

template <int NT>
__global__ __launch_bounds__(NT) void k_sort_scan(uint32_t* __restrict__ cnt, SortGeom g, uint32_t* __restrict__ bintot,
                                                            uint32_t* __restrict__ binbase, uint32_t* __restrict__ ticket,
                                                            uint32_t cap, uint32_t* __restrict__ st,
                                                            uint32_t* __restrict__ offs_end) {
    __shared__ uint32_t sh[NT / 64];
    __shared__ bool last;
    const uint32_t ncol = g.ntile * g.sub;
    uint32_t* row = cnt + (size_t)blockIdx.x * ncol;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < ncol; base += NT) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < ncol ? row[i] : 0u;
        uint32_t agg;
        const uint32_t e = block_excl_scan<NT>(v, agg, sh);
        if (i < ncol) row[i] = carry + e;
        carry += agg;
    }
    if (threadIdx.x == 0) st_agent(bintot + blockIdx.x, carry);
    if (!handoff_last(ticket, g.nbin, &last)) return;
    carry = 0;
    for (uint32_t base = 0; base < g.nbin; base += NT) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < g.nbin ? ld_agent(bintot + i) : 0u;
        uint32_t agg;
        const uint32_t e = block_excl_scan<NT>(v, agg, sh);
        if (i < g.nbin) binbase[i] = carry + e;
        carry += agg;
    }
    if (threadIdx.x == 0) {
        binbase[g.nbin] = carry;
        const bool over = carry > cap;
        if (over) atomicOr(&st[0], kMsmOverflow);
        *offs_end = over ? 0u : carry;
        *ticket = 0u;
    }
}

// K3. Per iteration (kTileThreads scalars, one per thread): every c = 16 scalar's <= 16 pairs take an
// LDS rank in their bin (lcnt), the counts are scanned over the bins (lst = this iteration's run
// start of each bin), the pairs are placed in bin order in LDS (sk, sr), and thread i writes pair i
// to pos[bin] + (i - lst[bin]): consecutive threads, consecutive addresses inside a bin's run. A
// scalar of another window size writes its pairs directly (pos[bin] atomics) before the runs.
struct ScatterLds {
    uint32_t pos[kMaxBins];   // this tile's next global slot in each bin
    uint32_t lst[kMaxBins];   // this iteration's counts, then run starts
    uint32_t sk[kStagePairs], sr[kStagePairs];
    uint32_t sh[kTileThreads / 64];
};
__global__ __launch_bounds__(kTileThreads) void k_sort_scatter(const MsmInst* __restrict__ insts, const uint64_t* __restrict__ prefix,
                                                               int nact, const Fr* __restrict__ scalars, SortGeom g,
                                                               const uint32_t* __restrict__ cnt,
                                                               const uint32_t* __restrict__ binbase,
                                                               const uint32_t* __restrict__ st,
                                                               uint32_t* __restrict__ sref, uint8_t* __restrict__ sfine) {
    if (st[0] & kMsmOverflow) return;  // compacted capacity exceeded: the batch reruns dense
    __shared__ ScatterLds L;
    const uint32_t tid = threadIdx.x, fmask = (1u << g.sb) - 1;
    for (uint32_t b = tid; b < g.nbin; b += kTileThreads) L.pos[b] = binbase[b] + cnt[((size_t)b * g.ntile + blockIdx.x) * kSub];  // (staged form: sub = kSub)
    const uint64_t t0 = (uint64_t)blockIdx.x * kTileThreads * g.spt + tid;
    for (uint32_t it = 0; it < g.spt; ++it) {
        const uint64_t gi = t0 + (uint64_t)it * kTileThreads;
        if (gi - tid >= g.tot_sc) break;  // block-uniform: no scalar of this iteration is in the batch
        for (uint32_t b = tid; b < g.nbin; b += kTileThreads) L.lst[b] = 0;
        __syncthreads();  // (also orders the previous iteration's pos updates before the direct writes)
        Keys16 kk;
        bool fast = false;
        uint32_t rk[16];
        if (gi < g.tot_sc) {
            auto direct = [&](uint32_t key, uint32_t ref) {
                const uint32_t q = atomicAdd(&L.pos[key >> g.sb], 1u);
                sref[q] = ref;
                sfine[q] = (uint8_t)(key & fmask);
            };
            fast = scalar_keys(insts, prefix, nact, scalars, gi, kk, direct);
            if (fast) {
#pragma unroll
                for (int w = 0; w < 16; ++w) rk[w] = kk.key[w] != ~0u ? atomicAdd(&L.lst[kk.key[w] >> g.sb], 1u) : 0u;
            }
        }
        __syncthreads();
        // run starts: exclusive scan of the counts over the bins
        uint32_t carry = 0;
        for (uint32_t base = 0; base < g.nbin; base += kTileThreads) {
            const uint32_t b = base + tid;
            const uint32_t v = b < g.nbin ? L.lst[b] : 0u;
            uint32_t agg;
            const uint32_t e = block_excl_scan<kTileThreads>(v, agg, L.sh);
            if (b < g.nbin) L.lst[b] = carry + e;
            carry += agg;
        }
        const uint32_t total = carry;  // this iteration's staged pairs (<= kStagePairs)
        __syncthreads();
        if (fast) {
#pragma unroll
            for (int w = 0; w < 16; ++w)
                if (kk.key[w] != ~0u) {
                    const uint32_t q = L.lst[kk.key[w] >> g.sb] + rk[w];
                    L.sk[q] = kk.key[w];
                    L.sr[q] = kk.ref[w];
                }
        }
        __syncthreads();
        for (uint32_t i = tid; i < total; i += kTileThreads) {
            const uint32_t key = L.sk[i], b = key >> g.sb;
            const uint32_t q = L.pos[b] + (i - L.lst[b]);
            sref[q] = L.sr[i];
            sfine[q] = (uint8_t)(key & fmask);
        }
        __syncthreads();
        for (uint32_t b = tid; b < g.nbin; b += kTileThreads) {  // advance by this iteration's run lengths
            const uint32_t e = b + 1 < g.nbin ? L.lst[b + 1] : total;
            L.pos[b] += e - L.lst[b];
        }
        __syncthreads();  // lst is cleared for the next iteration
    }
}

// K3, direct form (tiles of kDirectThreads x spt scalars, sub = 1): the pairs of a scalar take their
// slots from LDS atomics on pos (the 16 returning atomics issued back to back) and are written where
// they land. Chosen for sparse batches (a sharded rank keeps 1/G of the digits): per bin and tile
// too few pairs for runs, and the staged form's 144 KB workgroups would hold whole CUs.
__global__ __launch_bounds__(kDirectThreads) void k_sort_scatter_direct(const MsmInst* __restrict__ insts,
                                                                        const uint64_t* __restrict__ prefix, int nact,
                                                                        const Fr* __restrict__ scalars, SortGeom g,
                                                                        const uint32_t* __restrict__ cnt,
                                                                        const uint32_t* __restrict__ binbase,
                                                                        const uint32_t* __restrict__ st,
                                                                        uint32_t* __restrict__ sref, uint8_t* __restrict__ sfine) {
    if (st[0] & kMsmOverflow) return;
    __shared__ uint32_t pos[kMaxBins];
    for (uint32_t b = threadIdx.x; b < g.nbin; b += kDirectThreads) pos[b] = binbase[b] + cnt[(size_t)b * g.ntile + blockIdx.x];
    __syncthreads();
    const uint32_t fmask = (1u << g.sb) - 1;
    const uint64_t t0 = (uint64_t)blockIdx.x * kDirectThreads * g.spt + threadIdx.x;
    for (uint32_t k = 0; k < g.spt; ++k) {
        const uint64_t gi = t0 + (uint64_t)k * kDirectThreads;
        if (gi >= g.tot_sc) break;
        Keys16 kk;
        auto put = [&](uint32_t key, uint32_t ref) {
            const uint32_t q = atomicAdd(&pos[key >> g.sb], 1u);
            sref[q] = ref;
            sfine[q] = (uint8_t)(key & fmask);
        };
        if (scalar_keys(insts, prefix, nact, scalars, gi, kk, put)) {
            uint32_t q[16];
#pragma unroll
            for (int w = 0; w < 16; ++w) q[w] = kk.key[w] != ~0u ? atomicAdd(&pos[kk.key[w] >> g.sb], 1u) : 0u;
#pragma unroll
            for (int w = 0; w < 16; ++w)
                if (kk.key[w] != ~0u) {
                    sref[q[w]] = kk.ref[w];
                    sfine[q[w]] = (uint8_t)(kk.key[w] & fmask);
                }
        }
    }
}

// K4: per bin (one workgroup): bucket offsets, the partial levels' counts (affine level: the
// seg1-reference thread ranges [o, o + c) meets; XYZZ level l: ceil(previous / kSeg)) scanned inside
// the bin into lev[l], the bin's totals handed to the last block, which scans them into
// binpfx[l][bin]; then the bin's references ordered by bucket in LDS and written back contiguously
// (a bin larger than the staging: each reference written to its slot directly)
template <int NT, uint32_t STAGE>
struct BinLds {
    uint32_t out[STAGE ? STAGE : 1];
    uint32_t h[256], sh[NT / 64];
};
struct LevPtrs {
    uint32_t* p[kMaxLev + 1];  // [0]: the affine level's partial offsets; [l]: XYZZ level l
};
// NT threads (>= 256: one per in-bin bucket); STAGE: LDS staging capacity (0: every reference written directly)
template <int NT, uint32_t STAGE>
__global__ __launch_bounds__(NT) void k_sort_bins(SortGeom g, const uint32_t* __restrict__ binbase,
                                                            const uint32_t* __restrict__ st, const uint32_t* __restrict__ sref,
                                                            const uint8_t* __restrict__ sfine, uint32_t* __restrict__ offs,
                                                            uint32_t* __restrict__ refs, uint32_t seg1, int nlev, LevPtrs lev,
                                                            uint32_t* __restrict__ binsum, uint32_t* __restrict__ binpfx,
                                                            uint32_t* __restrict__ ticket) {
    __shared__ BinLds<NT, STAGE> L;
    __shared__ bool last;
    const uint32_t bin = blockIdx.x, f = threadIdx.x;
    const uint32_t b0 = bin << g.sb, nbk = min(1u << g.sb, g.nb - b0);
    const bool over = (st[0] & kMsmOverflow) != 0;
    const uint32_t base = binbase[bin], n = over ? 0u : binbase[bin + 1] - base;
    // the bin's pairs read as aligned quads: element e of quad q is pair a0 + 4 q + e, valid in
    // [head, head + n) (the staging buffers have 16 bytes of slack past their capacity)
    const uint32_t a0 = base & ~3u, head = base - a0, nq = (head + n + 3) / 4;
    if (f < 256) L.h[f] = 0;
    __syncthreads();
    for (uint32_t q = f; q < nq; q += NT) {
        const uint32_t w4 = *(const uint32_t*)(sfine + a0 + 4 * q);
#pragma unroll
        for (uint32_t e = 0; e < 4; ++e)
            if (4 * q + e - head < n) atomicAdd(&L.h[(w4 >> (8 * e)) & 0xFFu], 1u);
    }
    __syncthreads();
    const uint32_t c = f < nbk ? L.h[f] : 0u;
    uint32_t agg;
    const uint32_t lo = block_excl_scan<NT>(c, agg, L.sh);  // in-bin offset of bucket f
    const uint32_t o = base + lo;
    if (f < nbk) offs[b0 + f] = over ? 0u : o;
    // the partial levels: counts from (c, o), scanned inside the bin
    uint32_t v = c ? (o + c - 1) / seg1 - o / seg1 + 1 : 0u;
    for (int l = 0; l <= nlev; ++l) {
        if (l) v = (v + kSeg - 1) / kSeg;
        const uint32_t e = block_excl_scan<NT>(v, agg, L.sh);
        if (f < nbk) lev.p[l][b0 + f] = e;
        if (f == 0) st_agent(binsum + (size_t)l * (g.nbin + 1) + bin, agg);
    }
    const bool staged = n <= STAGE;
    if (f < 256) L.h[f] = staged ? lo : o;  // each bucket's next slot (in LDS / in refs)
    __syncthreads();
    for (uint32_t q = f; q < nq; q += NT) {
        const uint32_t w4 = *(const uint32_t*)(sfine + a0 + 4 * q);
        const uint4 r4 = *(const uint4*)(sref + a0 + 4 * q);
        const uint32_t rr[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
        for (uint32_t e = 0; e < 4; ++e)
            if (4 * q + e - head < n) {
                const uint32_t slot = atomicAdd(&L.h[(w4 >> (8 * e)) & 0xFFu], 1u);
                if (staged)
                    L.out[slot] = rr[e];
                else
                    refs[slot] = rr[e];
            }
    }
    if (staged) {
        __syncthreads();
        for (uint32_t i = f; i < n; i += NT) refs[base + i] = L.out[i];
    }
    if (!handoff_last(ticket, g.nbin, &last)) return;
    for (int l = 0; l <= nlev; ++l) {
        uint32_t carry = 0;
        const uint32_t* src = binsum + (size_t)l * (g.nbin + 1);
        uint32_t* dst = binpfx + (size_t)l * (g.nbin + 1);
        for (uint32_t b = 0; b < g.nbin; b += NT) {
            const uint32_t i = b + f;
            const uint32_t x = i < g.nbin ? ld_agent(src + i) : 0u;
            const uint32_t e = block_excl_scan<NT>(x, agg, L.sh);
            if (i < g.nbin) dst[i] = carry + e;
            carry += agg;
        }
        if (f == 0) dst[g.nbin] = carry;
    }
    if (f == 0) *ticket = 0u;
}

// K5: lev[l][b] += the bin's base; lev[l][nb] = the level's total
__global__ __launch_bounds__(kScanThreads) void k_sort_final(SortGeom g, int nlev, LevPtrs lev, const uint32_t* __restrict__ binpfx) {
    const uint64_t t = blockIdx.x * (uint64_t)kScanThreads + threadIdx.x;
    const uint32_t l = (uint32_t)(t / (g.nb + 1)), b = (uint32_t)(t % (g.nb + 1));
    if ((int)l > nlev) return;
    const uint32_t* pf = binpfx + (size_t)l * (g.nbin + 1);
    lev.p[l][b] = b < g.nb ? lev.p[l][b] + pf[b >> g.sb] : pf[g.nbin];
}

uint32_t seg1_len(bool) { return kSeg1Default; }

// The accumulation kernel's threads all run the same number of additions, so its duration is
// (rounds of resident waves) x (one wave's chain of seg1 additions). A grid of 4.02 rounds takes as
// long as 5: seg1 is lowered to the smallest value that keeps the round count, so the last round is
// full (the fixed length measured 1.5% slower: profiles/r02_ab8_seg1fit.jsonl, r02_ab20_seg.jsonl).
uint32_t seg1_fit(uint32_t seg1, uint64_t refs, int waves_per_simd, int lanes_per_elem) {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            n = 0;
        return n;
    }();
    if (cus <= 0 || refs == 0) return seg1;
    const uint64_t slots = (uint64_t)cus * 4 * waves_per_simd * 64 / lanes_per_elem;  // resident elements
    const uint64_t nthr = (refs + seg1 - 1) / seg1;
    const uint64_t rounds = (nthr + slots - 1) / slots;
    if (rounds > 16) return seg1;
    const uint64_t fit = (refs + rounds * slots - 1) / (rounds * slots);
    // floor 8: below one round the grid cannot fill the GPU anyway, and every reference moved out of
    // the mixed-addition chains costs a full XYZZ addition in the partial levels instead
    return (uint32_t)std::min<uint64_t>(seg1, std::max<uint64_t>(fit, std::min<uint32_t>(seg1, 8)));
}

MsmWorkspace* msm_ws_create() { return new MsmWorkspace(); }
void msm_ws_destroy(MsmWorkspace* ws) { delete ws; }
void msm_ws_staging_reset(MsmWorkspace* ws) {
    if (ws) ws->pin.reset();
}
void msm_ws_note_overflow(MsmWorkspace* ws) {
    if (ws) ws->cap_scale = std::min(ws->cap_scale * 1.5, 64.0);
}

static double msm_cap_env() {  // SPX_MSM_CAP_SCALE (tests): scales the compacted-key capacity, e.g. 0.5 forces overflow
    const char* e = getenv("SPX_MSM_CAP_SCALE");
    const double v = e ? atof(e) : 1.0;
    return v > 0 ? v : 1.0;
}

MsmPlan msm_plan(const MsmInst* ih, int ninst, const MsmShard& sh, double cap_scale) {
    MsmPlan o;
    const int G = std::max(1, sh.world);
    int g = 0;
    while ((1 << g) < G) ++g;
    if ((1 << g) != G || sh.rank < 0 || sh.rank >= G) throw std::runtime_error("MSM shard: bad rank / world");
    o.compact = G > 1 && !sh.dense;
    uint64_t tot_refs = 0;
    double split_refs = 0, whole_refs = 0;
    int nsplit = 0;
    for (int i = 0; i < ninst; ++i) {
        MsmInst I = ih[i];
        if (!I.size) continue;  // empty MSM: infinity
        if (I.c < 3 || I.c > 24) throw std::runtime_error("MSM window bits out of range");
        const uint32_t lbf = I.c - 1;  // log2 of the instance's buckets
        if (G > 1 && (int)lbf - g >= 2) {  // split: buckets dealt round-robin over the ranks
            I.lb = lbf - g;
            I.lg = (uint32_t)g;
            I.sel = (uint32_t)sh.rank;
            split_refs += (double)I.size * I.W / G;
            ++nsplit;
        } else if (i % G == sh.rank) {  // whole, on its owner
            I.lb = lbf;
            I.lg = 0;
            I.sel = 0;
            whole_refs += (double)I.size * I.W;
        } else {
            continue;
        }
        I.out = (uint32_t)i;
        I.bucket_off = o.nb;
        I.ref_off = (uint32_t)tot_refs;
        o.nb += 1u << I.lb;
        o.prefix.push_back(o.tot_sc);
        o.tot_sc += I.size;
        tot_refs += (uint64_t)I.size * I.W;
        o.mu_max = std::max(o.mu_max, (double)I.size * I.W / (double)(1u << lbf));
        o.any_split |= I.lg != 0;
        o.insts.push_back(I);
    }
    const int nact = (int)o.insts.size();
    o.prefix.push_back(o.tot_sc);
    if (tot_refs >= 0xffffffffull) throw std::runtime_error("MSM batch too large");
    if (o.compact) {
        // expected own digits plus a margin: ~8 standard deviations of the uniform case and a fixed
        // slack per split instance
        const double cap = whole_refs + (split_refs + 8.0 * std::sqrt(split_refs) + 2048.0 * nsplit) * cap_scale * msm_cap_env();
        tot_refs = std::min<uint64_t>(tot_refs, (uint64_t)std::ceil(cap));
    }
    o.tot_refs = tot_refs;
    // weighting tree: nodes after the chunked leaf level, 2^lb / 2^lgm per instance
    o.node_off.resize(nact);
    o.cnt.resize(nact);
    uint32_t tot_nodes = 0;
    for (int i = 0; i < nact; ++i) {
        o.node_off[i] = tot_nodes;
        const int lg = (int)o.insts[i].lb - (int)std::min<uint32_t>(kTreeChunkLog, o.insts[i].lb - 1);
        o.cnt[i] = 1u << lg;
        tot_nodes += o.cnt[i];
        o.levels = std::max(o.levels, lg);
    }
    o.wp.assign((size_t)(o.levels + 1) * (nact + 1), 0);
    o.cin.assign((size_t)(o.levels + 1) * nact, 0);
    uint32_t maxc = 1;
    for (int i = 0; i < nact; ++i) maxc = std::max(maxc, o.cnt[i]);
    o.top_from = o.levels + 1;
    for (int lv = 0; lv <= o.levels; ++lv) {
        uint64_t acc = 0;
        for (int i = 0; i < nact; ++i) {
            uint32_t nin = lv == 0 ? (o.cnt[i] * 2) : std::max(1u, o.cnt[i] >> (lv - 1));
            uint32_t nout = lv == 0 ? o.cnt[i] : std::max(1u, o.cnt[i] >> lv);
            o.cin[(size_t)lv * nact + i] = nin;
            o.wp[(size_t)lv * (nact + 1) + i] = acc;
            acc += nout;
        }
        o.wp[(size_t)lv * (nact + 1) + nact] = acc;
        if (lv >= 1 && o.top_from > o.levels && std::max(1u, maxc >> (lv - 1)) <= kTopNodes) o.top_from = lv;
    }
    return o;
}

void msm_upload_plan(MsmWorkspace* ws, MsmPlan& p, hipStream_t s) {
    // [insts | prefix | wp | cin | node_off], 16-byte aligned parts, one pinned staging copy
    const int nact = (int)p.insts.size();
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t b0 = al(sizeof(MsmInst) * nact), b1 = al(8 * p.prefix.size()), b2 = al(8 * p.wp.size()),
                 b3 = al(4 * p.cin.size()), b4 = al(4 * p.node_off.size());
    std::vector<uint8_t> h(b0 + b1 + b2 + b3 + b4, 0);
    size_t o = 0;
    memcpy(h.data() + o, p.insts.data(), sizeof(MsmInst) * nact), o += b0;
    memcpy(h.data() + o, p.prefix.data(), 8 * p.prefix.size()), o += b1;
    memcpy(h.data() + o, p.wp.data(), 8 * p.wp.size()), o += b2;
    memcpy(h.data() + o, p.cin.data(), 4 * p.cin.size()), o += b3;
    memcpy(h.data() + o, p.node_off.data(), 4 * p.node_off.size());
    uint8_t* d = (uint8_t*)ws->tables.ensure(h.size());
    // pinned staging: the copy may run after this returns; the arena is reset after a covering sync
    HIPCHK(hipMemcpyAsync(d, ws->pin.stage(h.data(), h.size()), h.size(), hipMemcpyHostToDevice, s));
    p.d_insts = (MsmInst*)d;
    p.d_prefix = (uint64_t*)(d + b0);
    p.d_wp = (uint64_t*)(d + b0 + b1);
    p.d_cin = (uint32_t*)(d + b0 + b1 + b2);
    p.d_noff = (uint32_t*)(d + b0 + b1 + b2 + b3);
}

// Sort geometry, by the batch's expected pairs per scalar (rho: 16 dense, ~16 / G on a rank of a
// G-rank proof):
//  * staged form (rho >= kStagedRho): bins as few as the in-bin staging allows (long runs in K3),
//    i.e. 2^sb buckets of the batch's most crowded instance expected to fill <= 80% of kBinStage;
//    tiles of kTileThreads x spt scalars, about 2^8 of them (one workgroup per CU);
//  * direct form: about 2^9 bins and 2^9 tiles of kDirectThreads x spt scalars.
// Either way at most kMaxBins bins. SPX_SORT_FORM=staged|direct (A/B) forces a form.
static constexpr double kStagedRho = 6.0;
static constexpr size_t kTicketBytes = 128;
static int sort_form_env() {  // -1: by rho; 0: direct; 1: staged
    static const int v = [] {
        const char* e = getenv("SPX_SORT_FORM");
        if (!e) return -1;
        return std::string(e) == "staged" ? 1 : std::string(e) == "direct" ? 0 : -1;
    }();
    return v;
}
static SortGeom sort_geom(const MsmPlan& p, bool& staged) {
    SortGeom g;
    g.nb = p.nb;
    g.tot_sc = p.tot_sc;
    const double rho = p.tot_sc ? (double)p.tot_refs / (double)p.tot_sc : 0.0;
    staged = sort_form_env() >= 0 ? sort_form_env() == 1 : rho >= kStagedRho;
    int lnb = 0;
    while ((1ull << lnb) < p.nb) ++lnb;
    int sb = 8;
    if (staged)
        while (sb > 0 && (double)(1u << sb) * std::max(p.mu_max, 1.0) > 0.8 * kBinStage) --sb;
    else
        sb = std::min(8, std::max(0, lnb - 9));
    while (sb < 8 && ((uint64_t)p.nb + (1u << sb) - 1) >> sb > kMaxBins) ++sb;
    g.sb = (uint32_t)sb;
    g.nbin = (p.nb + (1u << g.sb) - 1) >> g.sb;
    if (g.nbin > kMaxBins) throw std::runtime_error("MSM batch: too many buckets for the sort");
    const int threads = staged ? kTileThreads : kDirectThreads, tiles_log = staged ? 8 : 9;
    const uint64_t tile_sc = (uint64_t)threads << tiles_log;
    g.spt = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, (p.tot_sc + tile_sc - 1) / tile_sc));
    const uint64_t ts = (uint64_t)threads * g.spt;
    const uint64_t nt = (p.tot_sc + ts - 1) / ts;
    if (nt > 0x7fffffffull / kSub) throw std::runtime_error("MSM batch: too many tiles");
    g.ntile = (uint32_t)std::max<uint64_t>(1, nt);
    g.sub = staged ? kSub : 1;
    return g;
}

MsmSorted msm_sort(MsmWorkspace* ws, const MsmPlan& p, const Fr* scalars, void* out_dev, size_t out_bytes, hipStream_t s,
                   uint32_t seg1, int nlev) {
    if (nlev > kMaxLev) throw std::runtime_error("MSM: too many partial levels");
    if (out_bytes % 4) throw std::runtime_error("MSM: output bytes not a multiple of 4");
    MsmSorted o;
    bool staged = false;
    const SortGeom g = sort_geom(p, staged);
    const uint32_t nb = p.nb;
    const uint64_t cap = std::max<uint64_t>(p.tot_refs, 1);
    uint32_t* st = (uint32_t*)((uint8_t*)out_dev + out_bytes - 16);
    o.offs = (uint32_t*)ws->offs.ensure(4 * (size_t)(nb + 1));
    o.refs = (uint32_t*)ws->refs.ensure(4 * cap);
    uint32_t* cnt = (uint32_t*)ws->cnt.ensure(4 * (size_t)g.nbin * g.ntile * g.sub);
    uint32_t* bintot = (uint32_t*)ws->bintot.ensure(4 * (size_t)g.nbin);
    uint32_t* binbase = (uint32_t*)ws->binbase.ensure(4 * (size_t)(g.nbin + 1));
    // binsum: per level the bins' partial totals; binpfx (after it): their exclusive prefixes
    uint32_t* binsum = (uint32_t*)ws->binsum.ensure(4 * 2 * (size_t)(kMaxLev + 1) * (g.nbin + 1));
    uint32_t* binpfx = binsum + (size_t)(kMaxLev + 1) * (g.nbin + 1);
    uint32_t* sref = (uint32_t*)ws->stage_ref.ensure(4 * cap + 16);  // + 16: k_sort_bins reads aligned quads
    uint8_t* sfine = (uint8_t*)ws->stage_fine.ensure(cap + 16);
    uint32_t* lv = (uint32_t*)ws->lvl.ensure(4 * (size_t)(nb + 1) * (nlev + 1));
    // two tickets on 64-byte lines of their own: [0] k_sort_scan, [16] k_sort_bins
    uint32_t* tk = (uint32_t*)ws->tickets.ensure(kTicketBytes);
    if (!ws->tickets_zeroed) {  // once per workspace: every hand-off's last block resets its ticket
        HIPCHK(hipMemsetAsync(tk, 0, kTicketBytes, s));
        ws->tickets_zeroed = true;
    }
    LevPtrs lp{};
    for (int l = 0; l <= nlev; ++l) lp.p[l] = lv + (size_t)l * (nb + 1);
    const int nact = (int)p.insts.size();
    kp_begin(KP_SORT, s);
    hipLaunchKernelGGL(k_sort_count, dim3(g.ntile * g.sub), dim3(kCountThreads), 0, s, p.d_insts, p.d_prefix, nact, scalars, g,
                       cnt, (uint32_t*)out_dev, (uint32_t)(out_bytes / 4));
    const uint32_t cap32 = (uint32_t)std::min<uint64_t>(cap, 0xffffffffu);
    if (staged) {
        hipLaunchKernelGGL(k_sort_scan<kRowThreads>, dim3(g.nbin), dim3(kRowThreads), 0, s, cnt, g, bintot, binbase, tk, cap32,
                           st, o.offs + nb);
        hipLaunchKernelGGL(k_sort_scatter, dim3(g.ntile), dim3(kTileThreads), 0, s, p.d_insts, p.d_prefix, nact, scalars, g, cnt,
                           binbase, st, sref, sfine);
        hipLaunchKernelGGL((k_sort_bins<kBinThreads, kBinStage>), dim3(g.nbin), dim3(kBinThreads), 0, s, g, binbase, st, sref,
                           sfine, o.offs, o.refs, seg1, nlev, lp, binsum, binpfx, tk + 16);
    } else {
        hipLaunchKernelGGL(k_sort_scan<kDirectThreads>, dim3(g.nbin), dim3(kDirectThreads), 0, s, cnt, g, bintot, binbase, tk,
                           cap32, st, o.offs + nb);
        hipLaunchKernelGGL(k_sort_scatter_direct, dim3(g.ntile), dim3(kDirectThreads), 0, s, p.d_insts, p.d_prefix, nact, scalars,
                           g, cnt, binbase, st, sref, sfine);
        hipLaunchKernelGGL((k_sort_bins<kDirectThreads, 0>), dim3(g.nbin), dim3(kDirectThreads), 0, s, g, binbase, st, sref,
                           sfine, o.offs, o.refs, seg1, nlev, lp, binsum, binpfx, tk + 16);
    }
    const uint64_t nfin = (uint64_t)(nlev + 1) * (nb + 1);
    hipLaunchKernelGGL(k_sort_final, dim3((unsigned)((nfin + kScanThreads - 1) / kScanThreads)), dim3(kScanThreads), 0, s, g,
                       nlev, lp, binpfx);
    // algorithmic bytes: every scalar read twice (32 B), every kept pair staged (5 B), re-read (5 B)
    // and placed (4 B); the count matrix written, scanned and read (16 B per entry)
    kp_end(64.0 * p.tot_sc + 14.0 * p.tot_refs + 16.0 * g.nbin * g.ntile * g.sub, s, (double)p.tot_refs);
    o.np_off = lp.p[0];
    for (int l = 1; l <= nlev; ++l) o.lev.push_back(lp.p[l]);
    return o;
}

// ------------------------------------------------------------------ byte images <-> device points
DEV bool fq_canon_to_mont(Fq& r, const Fq& c) {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        uint64_t d = (uint64_t)c.v[i] - kFqP[i] - br;
        br = (uint32_t)(d >> 63);
    }
    Fq r2;
#pragma unroll
    for (int i = 0; i < 12; ++i) r2.v[i] = kFqR2[i];
    fe_mul(r, c, r2);
    return br != 0;  // c < q
}

template <int NF>  // NF = number of Fq coordinates per point (2 for G1, 4 for G2)
__global__ void k_points_from_bytes(Fq* pts, uint64_t n, int* err) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        Fq* p = pts + j * NF;
        Fq last;
        load_vec(last, p + NF - 1);
        const uint32_t flags = last.v[11] >> 30;
        bool ok = true;
        if (flags & 1u) {  // bit 6 of the last byte: point at infinity
            Fq z;
            fe_zero(z);
#pragma unroll
            for (int k = 0; k < NF; ++k) store_vec(p + k, z);
            continue;
        }
        Fq m[NF];
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            Fq c;
            load_vec(c, p + k);
            if (k == NF - 1) c.v[11] &= 0x3fffffffu;
            ok &= fq_canon_to_mont(m[k], c);
            store_vec(p + k, m[k]);
        }
        if (!ok) {
            atomicOr(err, 1);
            continue;
        }
        // on the curve: y^2 = x^3 + b, b = 4 (G1) or 4 (1 + u) (G2); ark's CanonicalDeserialize of the
        // PublicParameter rejects such points too (the subgroup check is not repeated: the PP is trusted
        // input from setup, as in the reference's cache, commitment/mod.rs:41-62)
        if constexpr (NF == 2) {
            Fq y2, x3, b;
            fe_sqr(y2, m[1]);
            fe_sqr(x3, m[0]);
            fe_mul(x3, x3, m[0]);
            fe_one(b);
            fe_add(b, b, b);
            fe_add(b, b, b);
            fe_add(x3, x3, b);
            if (!fe_eq(y2, x3)) atomicOr(err, 2);
        } else {
            Fq2 x, y, y2, x3, b;
            x.c0 = m[0], x.c1 = m[1], y.c0 = m[2], y.c1 = m[3];
            f2_sqr(y2, y);
            f2_sqr(x3, x);
            f2_mul(x3, x3, x);
            fe_one(b.c0);
            fe_add(b.c0, b.c0, b.c0);
            fe_add(b.c0, b.c0, b.c0);
            b.c1 = b.c0;
            f2_add(x3, x3, b);
            if (!f2_eq(y2, x3)) atomicOr(err, 2);
        }
    }
}
template <int NF>
__global__ void k_points_to_canon(Fq* pts, uint64_t n) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        Fq* p = pts + j * NF;
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            Fq m, c;
            load_vec(m, p + k);
            fe_from_mont(c, m);
            store_vec(p + k, c);
        }
    }
}
static unsigned pgrid(uint64_t n) { return (unsigned)std::min<uint64_t>((n + 255) / 256, 8192); }
void launch_points_from_bytes_g1(G1Aff* pts, uint64_t n, int* err, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_points_from_bytes<2>, dim3(pgrid(n)), dim3(256), 0, s, (Fq*)pts, n, err);
}
void launch_points_from_bytes_g2(G2Aff* pts, uint64_t n, int* err, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_points_from_bytes<4>, dim3(pgrid(n)), dim3(256), 0, s, (Fq*)pts, n, err);
}
void launch_points_to_canon_g1(G1Aff* pts, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_points_to_canon<2>, dim3(pgrid(n)), dim3(256), 0, s, (Fq*)pts, n);
}
void launch_points_to_canon_g2(G2Aff* pts, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_points_to_canon<4>, dim3(pgrid(n)), dim3(256), 0, s, (Fq*)pts, n);
}

}  // namespace spx
