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
//  * Signed c-bit digits -> (bucket, reference) pairs written window-major, hipCUB LSD radix sort
//    on the bucket bits, run boundaries -> per-bucket counts and offsets. References are 32-bit
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

#include <rocprim/device/device_radix_sort.hpp>

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

// One thread per scalar. Dense: a (key, reference) pair for every (scalar, window), window-major
// within each instance so the stores coalesce; digits that are zero or not this rank's get the key
// nb and sort last. Compact (proof-sharded ranks): only this rank's digits, appended through a
// block-level scan and one atomic per block (st[1]); pairs past `cap` are dropped and flag st[0].
// Compact with HIST (the counting sort): each kept digit also takes its rank inside its bucket from
// the bucket's counter (hist[key]++, returned into posv); otherwise the last block to finish (ticket
// st[2]) fills the unused key slots with ~0 (sorts last in the radix sort).
template <bool COMPACT, bool HIST>
__global__ __launch_bounds__(kLight) void k_msm_keys(const MsmInst* __restrict__ insts, const uint64_t* __restrict__ prefix,
                                                     int ninst, uint64_t total, uint32_t nb, const Fr* __restrict__ scalars,
                                                     uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t cap,
                                                     uint32_t* __restrict__ st, uint32_t* __restrict__ hist,
                                                     uint32_t* __restrict__ posv) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const bool live = g < total;
    if (!COMPACT && !live) return;
    MsmInst I{};
    uint64_t j = 0;
    Digits d0;
    if (live) {
        const int i = find_slot(prefix, ninst, g);
        j = g - prefix[i];
        I = insts[i];
        Fr m, s;
        load_vec(m, scalars + I.scalar_off + j);
        fe_from_mont(s, m);
#pragma unroll
        for (int k = 0; k < 8; ++k) d0.s[k] = s.v[k];
    }
    if constexpr (!COMPACT) {
        for (uint32_t w = 0; w < I.W; ++w) {
            const int32_t d = d0.next(I.c);
            const uint32_t key = digit_key(I, d);
            const uint64_t o = I.ref_off + (uint64_t)w * I.size + j;
            keys[o] = key == ~0u ? nb : key;
            vals[o] = digit_ref(I, w, j, d);
        }
    } else {
        // the digits are extracted once: for up to kKeep windows (c >= 16 at the sizes that matter) the
        // counting pass keeps every window's key and reference in registers (the window loop unrolled,
        // so the arrays are indexed statically); more windows recompute them in the writing pass
        constexpr uint32_t kKeep = 16;
        uint32_t cnt = 0, kkey[kKeep], kref[kKeep], kpos[kKeep];
        if (live && I.c == 16 && I.W == kKeep) {
            Digits d = d0;
#pragma unroll
            for (uint32_t w = 0; w < kKeep; ++w) {
                const int32_t dg = d.at16(w);
                kkey[w] = digit_key(I, dg);
                kref[w] = digit_ref(I, w, j, dg);
                cnt += kkey[w] != ~0u;
                // independent returning atomics, issued back to back (their latency overlaps)
                if constexpr (HIST) kpos[w] = kkey[w] != ~0u ? atomicAdd(&hist[kkey[w]], 1u) : 0u;
            }
        } else if (live && I.W <= kKeep) {
            Digits d = d0;
#pragma unroll
            for (uint32_t w = 0; w < kKeep; ++w) {
                kkey[w] = ~0u;
                if (w < I.W) {
                    const int32_t dg = d.next(I.c);
                    kkey[w] = digit_key(I, dg);
                    kref[w] = digit_ref(I, w, j, dg);
                }
                cnt += kkey[w] != ~0u;
                if constexpr (HIST) kpos[w] = kkey[w] != ~0u ? atomicAdd(&hist[kkey[w]], 1u) : 0u;
            }
        } else if (live) {
            Digits d = d0;
            for (uint32_t w = 0; w < I.W; ++w) cnt += digit_key(I, d.next(I.c)) != ~0u;
        }
        using Scan = hipcub::BlockScan<uint32_t, kLight>;
        __shared__ typename Scan::TempStorage tmp;
        __shared__ uint32_t base;
        __shared__ bool last;
        uint32_t pre, agg;
        Scan(tmp).ExclusiveSum(cnt, pre, agg);
        if (threadIdx.x == 0) {
            base = agg ? atomicAdd(&st[1], agg) : 0u;
            if ((uint64_t)base + agg > cap) atomicOr(&st[0], kMsmOverflow);
        }
        __syncthreads();
        if (cnt && I.W <= kKeep) {
            uint64_t pos = (uint64_t)base + pre;
#pragma unroll
            for (uint32_t w = 0; w < kKeep; ++w)
                if (kkey[w] != ~0u) {
                    if (pos < cap) {
                        keys[pos] = kkey[w];
                        vals[pos] = kref[w];
                        if constexpr (HIST) posv[pos] = kpos[w];
                    }
                    ++pos;
                }
        } else if (cnt) {
            uint64_t pos = (uint64_t)base + pre;
            Digits d = d0;
            for (uint32_t w = 0; w < I.W; ++w) {
                const int32_t dg = d.next(I.c);
                const uint32_t key = digit_key(I, dg);
                if (key == ~0u) continue;
                const uint32_t rk = HIST ? atomicAdd(&hist[key], 1u) : 0u;
                if (pos < cap) {
                    keys[pos] = key;
                    vals[pos] = digit_ref(I, w, j, dg);
                    if constexpr (HIST) posv[pos] = rk;
                }
                ++pos;
            }
        }
        if constexpr (HIST) return;  // the counting sort places the pairs itself: no fillers
        if (threadIdx.x == 0)  // (its cursor add has returned: every block's slots are taken when the last ticket is)
            last = atomicAdd(&st[2], 1u) == gridDim.x - 1;
        __syncthreads();
        if (last) {  // every block has taken its slots: fill the rest
            const uint32_t used = min(atomicAdd(&st[1], 0u), cap);
            for (uint32_t i = used + threadIdx.x; i < cap; i += blockDim.x) keys[i] = ~0u;
        }
    }
}

// ------------------------------------------------------------------ counting sort (compacted batches)
// A proof-sharded rank keeps 1/G of the digits (G = 8 at 2^20: ~2 M pairs per batch into 2^12..2^16
// local buckets). Their order is: keys pass (hist[key]++ gives each pair its rank in its bucket) ->
// ONE workgroup derives every offset array from the counts -> one scatter pass. Three launches, no
// device-wide look-back scans, no fill kernels; the radix sort stays for dense batches and for
// 2-rank sharding (MsmPlan::counting).
static constexpr int kScanThreads = 1024;
static constexpr int kMaxLev = 8;
struct LevPtrs {
    uint32_t* p[kMaxLev + 1];  // [0]: the affine level's partial offsets; [l]: XYZZ level l
};
// The offsets kernel runs in ONE workgroup of kScanThreads threads and goes through the counts in
// tiles of kScanThreads x kScanPer buckets (thread t: kScanPer consecutive buckets). Every array it
// writes is an exclusive scan of a per-bucket count that follows from the bucket's own reference
// count c and its offset o: the affine level's partials p = c ? (o + c - 1) / seg1 - o / seg1 + 1 : 0
// (the seg1-reference thread ranges [o, o + c) meets), and each XYZZ level's segments
// ceil(previous count / kSeg). So a tile needs two block scans (offsets, then all partial arrays
// at once as one vector) and the counts are read once.
static constexpr int kScanPer = 8;
struct ScanVec {
    uint32_t v[kMaxLev + 1];
};
struct ScanVecSum {
    DEV ScanVec operator()(const ScanVec& a, const ScanVec& b) const {
        ScanVec r;
#pragma unroll
        for (int k = 0; k <= kMaxLev; ++k) r.v[k] = a.v[k] + b.v[k];
        return r;
    }
};
// hist (nb counts) -> offs (nb + 1), lev.p[0] (partials of seg1-reference thread ranges) and
// lev.p[1..nlev] (segments of kSeg partials), exactly the arrays scan_partials / scan_segs give the
// dense path; hist is cleared for the next batch. If the counted pairs exceed the capacity (the
// compaction dropped some), the batch is flagged kMsmOverflow and every offset is 0: later kernels see
// empty buckets, never read an unwritten slot, and the driver reruns the batch dense.
__global__ __launch_bounds__(kScanThreads) void k_msm_offsets(uint32_t* __restrict__ hist, uint32_t nb, uint32_t cap,
                                                              uint32_t* __restrict__ st, uint32_t* __restrict__ offs,
                                                              uint32_t seg1, int nlev, LevPtrs lev) {
    using Red = hipcub::BlockReduce<uint32_t, kScanThreads>;
    using Scan1 = hipcub::BlockScan<uint32_t, kScanThreads>;
    using ScanV = hipcub::BlockScan<ScanVec, kScanThreads>;
    __shared__ union {
        typename Red::TempStorage r;
        typename Scan1::TempStorage a;
        typename ScanV::TempStorage v;
    } tmp;
    __shared__ uint32_t s_total;
    {  // pass 1: the total, to decide overflow before anything is written
        uint32_t sum = 0;
        for (uint32_t b = threadIdx.x; b < nb; b += kScanThreads) sum += hist[b];
        const uint32_t t = Red(tmp.r).Sum(sum);
        if (threadIdx.x == 0) s_total = t;
        __syncthreads();
    }
    const bool over = s_total > cap;
    if (over && threadIdx.x == 0) atomicOr(&st[0], kMsmOverflow);
    const uint32_t n = nb + 1;  // offs[nb] / lev[l][nb]: the totals
    uint32_t carry0 = 0;
    ScanVec carry;
#pragma unroll
    for (int l = 0; l <= kMaxLev; ++l) carry.v[l] = 0;
    for (uint32_t base = 0; base < n; base += kScanThreads * kScanPer) {
        const uint32_t b0 = base + threadIdx.x * kScanPer;
        uint32_t c[kScanPer], s = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            c[k] = b0 + k < nb ? hist[b0 + k] : 0u;
            s += c[k];
        }
#pragma unroll
        for (int k = 0; k < kScanPer; ++k)
            if (b0 + k < nb) hist[b0 + k] = 0u;
        uint32_t e0, agg0;
        Scan1(tmp.a).ExclusiveSum(s, e0, agg0);
        __syncthreads();
        // this thread's partial-array counts, summed per array
        ScanVec sv;
#pragma unroll
        for (int l = 0; l <= kMaxLev; ++l) sv.v[l] = 0;
        uint32_t o = carry0 + e0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            uint32_t v = c[k] ? (o + c[k] - 1) / seg1 - o / seg1 + 1 : 0u;
            sv.v[0] += v;
            for (int l = 1; l <= nlev; ++l) {
                v = (v + kSeg - 1) / kSeg;
                sv.v[l] += v;
            }
            o += c[k];
        }
        ScanVec ev, aggv;
        ScanV(tmp.v).ExclusiveScan(sv, ev, carry, ScanVecSum(), aggv);  // carry as the initial value
        __syncthreads();
        o = carry0 + e0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const uint32_t b = b0 + k;
            if (b < n) {
                offs[b] = over ? 0u : o;
                uint32_t v = c[k] ? (o + c[k] - 1) / seg1 - o / seg1 + 1 : 0u;
                lev.p[0][b] = over ? 0u : ev.v[0];
                ev.v[0] += v;
                for (int l = 1; l <= nlev; ++l) {
                    v = (v + kSeg - 1) / kSeg;
                    lev.p[l][b] = over ? 0u : ev.v[l];
                    ev.v[l] += v;
                }
            }
            o += c[k];
        }
        carry0 += agg0;
        carry = ScanVecSum()(carry, aggv);
    }
}
// compacted pair i -> refs[offs[key] + its rank in the bucket] (skipped when the batch overflowed)
__global__ __launch_bounds__(kLight) void k_msm_scatter(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                        const uint32_t* __restrict__ posv, const uint32_t* __restrict__ st,
                                                        uint32_t cap, const uint32_t* __restrict__ offs,
                                                        uint32_t* __restrict__ refs) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (st[0] & kMsmOverflow) return;
    if (i >= min(st[1], cap)) return;
    refs[offs[keys[i]] + posv[i]] = vals[i];
}

// sorted keys -> offs[b] = first index with key >= b, for b = 0..nb (offs[nb] = the references;
// an empty bucket shares the next bucket's offset)
__global__ __launch_bounds__(kLight) void k_bucket_bounds(const uint32_t* __restrict__ keys, uint64_t n, uint32_t nb,
                                                          uint32_t* __restrict__ offs) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nb) return;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (keys[mid] < b)
            lo = mid + 1;
        else
            hi = mid;
    }
    offs[b] = (uint32_t)lo;
}

// Exclusive offsets of a per-bucket count derived from the previous offsets (device-wide hipCUB
// scan over a transform iterator: no count array, no extra launch). Counts are off[b + 1] - off[b].
struct PartialsOp {  // the seg-length thread ranges bucket b's references [off[b], off[b + 1]) meet
    const uint32_t* off;
    uint32_t nb, seg;
    __host__ __device__ uint32_t operator()(uint32_t b) const {
        if (b >= nb) return 0u;
        const uint32_t o = off[b], c = off[b + 1] - o;
        return c ? (o + c - 1) / seg - o / seg + 1 : 0u;
    }
};
struct SegsOp {  // segments of `seg` partials for bucket b's partials [off[b], off[b + 1])
    const uint32_t* off;
    uint32_t nb, seg;
    __host__ __device__ uint32_t operator()(uint32_t b) const {
        return b < nb ? (off[b + 1] - off[b] + seg - 1) / seg : 0u;
    }
};
template <class Op>
static void scan_op(MsmWorkspace* ws, const Op& op, uint32_t nb, uint32_t* out, hipStream_t s) {
    hipcub::CountingInputIterator<uint32_t> cit(0u);
    hipcub::TransformInputIterator<uint32_t, Op, hipcub::CountingInputIterator<uint32_t>> it(cit, op);
    size_t tb = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, it, out, (int)nb + 1, s));
    void* t = ws->cub.ensure(tb);
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(t, tb, it, out, (int)nb + 1, s));
}
void scan_partials(MsmWorkspace* ws, const uint32_t* offs, uint32_t nb, uint32_t seg, uint32_t* np_off, hipStream_t s) {
    scan_op(ws, PartialsOp{offs, nb, seg}, nb, np_off, s);
}
void scan_segs(MsmWorkspace* ws, const uint32_t* off, uint32_t nb, uint32_t seg, uint32_t* seg_off, hipStream_t s) {
    scan_op(ws, SegsOp{off, nb, seg}, nb, seg_off, s);
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
    // the counting sort for 4 and more ranks (2^20: 2-3.5% more proofs per second than the radix sort
    // at G = 8, equal at G = 4); at G = 2 a rank keeps half the digits (~8 M pairs per opening batch
    // into ~10^5 buckets) and the returning bucket atomics and the one-workgroup offsets cost more than
    // the radix sort does (105 vs 114 M constraints/s): profiles/r05/r05l_*.jsonl, r05m_*.jsonl
    o.counting = o.compact && G >= 4;
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

MsmSorted msm_sort(MsmWorkspace* ws, const MsmPlan& p, const Fr* scalars, uint32_t* st, hipStream_t s, uint32_t seg1,
                   int nlev) {
    MsmSorted o;
    const uint32_t nb = p.nb;
    const uint64_t n = p.tot_refs;
    const int nact = (int)p.insts.size();
    o.offs = (uint32_t*)ws->offs.ensure(4 * (nb + 1));
    o.refs = (uint32_t*)ws->refs.ensure(4 * std::max<uint64_t>(n, 1));
    if (p.counting) {  // counting sort: keys + counts, every offset array in one workgroup, scatter
        if (nlev > kMaxLev) throw std::runtime_error("MSM: too many partial levels");
        uint32_t* hist = (uint32_t*)ws->hist.ensure(4 * (size_t)std::max<uint32_t>(nb, 1));
        if (ws->hist_zeroed != ws->hist.cap) {  // fresh allocation: zero once; the offsets kernel keeps it zero
            HIPCHK(hipMemsetAsync(hist, 0, ws->hist.cap, s));
            ws->hist_zeroed = ws->hist.cap;
        }
        uint32_t* ka = (uint32_t*)ws->keys_a.ensure(4 * std::max<uint64_t>(n, 1));
        uint32_t* va = (uint32_t*)ws->vals_a.ensure(4 * std::max<uint64_t>(n, 1));
        uint32_t* pv = (uint32_t*)ws->posv.ensure(4 * std::max<uint64_t>(n, 1));
        uint32_t* lv = (uint32_t*)ws->lvl.ensure(4 * (size_t)(nb + 1) * (nlev + 1));
        LevPtrs lp{};
        for (int l = 0; l <= nlev; ++l) lp.p[l] = lv + (size_t)l * (nb + 1);
        const int gsc = (int)((p.tot_sc + kLight - 1) / kLight);
        kp_begin(KP_SORT, s);
        hipLaunchKernelGGL((k_msm_keys<true, true>), dim3(gsc), dim3(kLight), 0, s, p.d_insts, p.d_prefix, nact, p.tot_sc, nb,
                           scalars, ka, va, (uint32_t)n, st, hist, pv);
        hipLaunchKernelGGL(k_msm_offsets, dim3(1), dim3(kScanThreads), 0, s, hist, nb, (uint32_t)n, st, o.offs, seg1, nlev,
                           lp);
        hipLaunchKernelGGL(k_msm_scatter, dim3((unsigned)((n + kLight - 1) / kLight)), dim3(kLight), 0, s, ka, va, pv, st,
                           (uint32_t)n, o.offs, o.refs);
        kp_end(32.0 * p.tot_sc + 4.0 * 6 * n, s);
        o.np_off = lp.p[0];
        for (int l = 1; l <= nlev; ++l) o.lev.push_back(lp.p[l]);
        return o;
    }
    // (bucket, reference) pairs, LSD radix sort on the bucket bits, bucket bounds by binary search
    int bits = 1;
    while ((1ull << bits) <= nb) ++bits;  // keys 0..nb; the compact filler ~0 has all these bits set
    uint32_t* ka = (uint32_t*)ws->keys_a.ensure(4 * std::max<uint64_t>(n, 1));
    uint32_t* kb = (uint32_t*)ws->keys_b.ensure(4 * std::max<uint64_t>(n, 1));
    uint32_t* va = (uint32_t*)ws->vals_a.ensure(4 * std::max<uint64_t>(n, 1));
    const int gsc = (int)((p.tot_sc + kLight - 1) / kLight);
    // (a counting sort, histogram atomics in the keys pass + scan + scatter, measured 10% slower end to
    // end: profiles/r03/r03t_ab.jsonl; 11-bit onesweep digits no faster: r03at_ab_sort_bits.jsonl)
    kp_begin(KP_SORT, s);
    if (p.compact)
        hipLaunchKernelGGL((k_msm_keys<true, false>), dim3(gsc), dim3(kLight), 0, s, p.d_insts, p.d_prefix, nact, p.tot_sc,
                           nb, scalars, ka, va, (uint32_t)n, st, nullptr, nullptr);
    else
        hipLaunchKernelGGL((k_msm_keys<false, false>), dim3(gsc), dim3(kLight), 0, s, p.d_insts, p.d_prefix, nact, p.tot_sc,
                           nb, scalars, ka, va, 0u, st, nullptr, nullptr);
    {
        hipcub::DoubleBuffer<uint32_t> dk(ka, kb), dv(va, o.refs);
        size_t tb = 0;
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dv, (int)n, 0, bits, s));
        void* t = ws->cub.ensure(tb);
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(t, tb, dk, dv, (int)n, 0, bits, s));
        o.refs = dv.Current();
        const uint32_t* sorted = dk.Current();
        hipLaunchKernelGGL(k_bucket_bounds, dim3((nb + 1 + kLight - 1) / kLight), dim3(kLight), 0, s, sorted, n, nb,
                           o.offs);
    }
    kp_end(32.0 * p.tot_sc + 4.0 * 8 * n, s);
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
