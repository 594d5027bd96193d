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
//  * Signed c-bit digits -> counting sort by bucket (atomic histogram, hipCUB scan, atomic
//    scatter of 32-bit point references with the sign in bit 31). Order inside a bucket is
//    irrelevant: group addition is exact and commutative, the affine result is unique.
//  * Bucket accumulation in XYZZ coordinates over fixed segments of kSeg references per thread
//    (load-balanced whatever the scalar distribution), repeated on the partial sums until every
//    bucket has one value (log_kSeg(max bucket) levels: one host sync to read the max count).
//  * Bucket weighting sum_j j S_j with per-thread running sums over L buckets plus one small
//    scalar multiple, then a per-instance block reduction. Result: one XYZZ point per MSM.
// Many MSMs run as one batch (all nv levels of an opening): one pipeline, one sync.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.hpp"

namespace spx {

static constexpr uint32_t kSeg = 32;
static constexpr int kLight = 256;  // threads for bookkeeping kernels
static constexpr int kHeavy = 64;   // threads for curve kernels (register-heavy)

#define HIPCHK(x)                                                                                     \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + \
                                                       " at " __FILE__ ":" + std::to_string(__LINE__)); \
    } while (0)

__device__ __constant__ constexpr uint32_t kFqR2[12] = {0x1c341746u, 0xf4df1f34u, 0x09d104f1u, 0x0a76e6a6u,
                                                       0x4c95b6d5u, 0x8de5476cu, 0x939d83c0u, 0x67eb88a9u,
                                                       0xb519952du, 0x9a793e85u, 0x92cae3aau, 0x11988fe5u};

// ------------------------------------------------------------------ helpers
template <class F>
DEV bool aff_is_sentinel(const Aff<F>& a) {
    return FieldOps<F>::is_zero(a.x) && FieldOps<F>::is_zero(a.y);
}
template <class F>
DEV void aff_set_sentinel(Aff<F>& a) {
    FieldOps<F>::zero(a.x);
    FieldOps<F>::zero(a.y);
}

DEV int find_slot(const uint64_t* prefix, int n, uint64_t g) {  // largest i with prefix[i] <= g
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (prefix[mid] <= g)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}
DEV uint32_t find_bucket(const uint32_t* off, uint32_t nb, uint32_t s) {  // largest b with off[b] <= s
    uint32_t lo = 0, hi = nb - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi + 1) >> 1;
        if (off[mid] <= s)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

// ------------------------------------------------------------------ digits: count / scatter
template <bool SCATTER>
__global__ __launch_bounds__(kLight) void k_msm_digits(const MsmInst* __restrict__ insts,
                                                       const uint64_t* __restrict__ prefix, int ninst,
                                                       uint64_t total, const Fr* __restrict__ scalars,
                                                       uint32_t* __restrict__ counts, uint32_t* __restrict__ cursor,
                                                       uint32_t* __restrict__ refs) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (g >= total) return;
    const int i = find_slot(prefix, ninst, g);
    const uint64_t j = g - prefix[i];
    const MsmInst I = insts[i];
    Fr m, s;
    load_vec(m, scalars + I.scalar_off + j);
    fe_from_mont(s, m);
    const uint32_t c = I.c, full = 1u << c, half = full >> 1, mask = full - 1;
    uint32_t carry = 0;
    for (uint32_t w = 0; w < I.W; ++w) {
        uint32_t v = (s.v[0] & mask) + carry;
#pragma unroll
        for (int k = 0; k < 7; ++k) s.v[k] = (s.v[k] >> c) | (s.v[k + 1] << (32 - c));
        s.v[7] >>= c;
        int32_t d;
        if (v > half) {
            d = (int32_t)v - (int32_t)full;
            carry = 1;
        } else {
            d = (int32_t)v;
            carry = 0;
        }
        if (d != 0) {
            const uint32_t b = I.bucket_off + (uint32_t)(d < 0 ? -d : d) - 1;
            if (!SCATTER) {
                atomicAdd(&counts[b], 1u);
            } else {
                const uint32_t pos = atomicAdd(&cursor[b], 1u);
                refs[pos] = (uint32_t)(I.pts_off + (uint64_t)w * I.stride + j) | (d < 0 ? 0x80000000u : 0u);
            }
        }
    }
}

__global__ void k_seg_counts(const uint32_t* __restrict__ cnt, uint32_t nb, uint32_t* __restrict__ segcnt) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) segcnt[b] = (cnt[b] + kSeg - 1) / kSeg;
    if (b == nb) segcnt[b] = 0;
}

// ------------------------------------------------------------------ accumulation levels
template <class F>
__global__ __launch_bounds__(kHeavy) void k_accum_aff(const uint32_t* __restrict__ segoff, uint32_t nb,
                                                      const uint32_t* __restrict__ off,
                                                      const uint32_t* __restrict__ cnt,
                                                      const uint32_t* __restrict__ refs,
                                                      const Aff<F>* __restrict__ pts, Xyzz<F>* __restrict__ out) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= segoff[nb]) return;
    const uint32_t b = find_bucket(segoff, nb, s);
    const uint32_t k = s - segoff[b];
    const uint32_t start = off[b] + k * kSeg;
    const uint32_t end = min(start + kSeg, off[b] + cnt[b]);
    Xyzz<F> acc;
    xyzz_set_inf(acc);
    for (uint32_t e = start; e < end; ++e) {
        const uint32_t r = refs[e];
        Aff<F> p;
        load_vec(p, pts + (r & 0x7fffffffu));
        if (aff_is_sentinel(p)) continue;
        xyzz_madd(acc, p, (r >> 31) != 0);
    }
    store_vec(out + s, acc);
}

template <class F>
__global__ __launch_bounds__(kHeavy) void k_accum_xyzz(const uint32_t* __restrict__ segoff, uint32_t nb,
                                                       const uint32_t* __restrict__ off,
                                                       const uint32_t* __restrict__ cnt,
                                                       const Xyzz<F>* __restrict__ in, Xyzz<F>* __restrict__ out) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= segoff[nb]) return;
    const uint32_t b = find_bucket(segoff, nb, s);
    const uint32_t k = s - segoff[b];
    const uint32_t start = off[b] + k * kSeg;
    const uint32_t end = min(start + kSeg, off[b] + cnt[b]);
    Xyzz<F> acc;
    load_vec(acc, in + start);
    for (uint32_t e = start + 1; e < end; ++e) {
        Xyzz<F> p;
        load_vec(p, in + e);
        xyzz_add(acc, p);
    }
    store_vec(out + s, acc);
}

// ------------------------------------------------------------------ bucket weighting
template <class F>
__global__ __launch_bounds__(kHeavy) void k_bucket_reduce(const MsmInst* __restrict__ insts,
                                                          const uint64_t* __restrict__ redp, int ninst,
                                                          uint64_t total, const uint32_t* __restrict__ cnt,
                                                          const uint32_t* __restrict__ off,
                                                          const Xyzz<F>* __restrict__ P, Xyzz<F>* __restrict__ red) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= total) return;
    const int i = find_slot(redp, ninst, t);
    const uint32_t tt = (uint32_t)(t - redp[i]);
    const MsmInst I = insts[i];
    const uint32_t lo = tt * I.red_L;
    Xyzz<F> run, acc;
    xyzz_set_inf(run);
    xyzz_set_inf(acc);
    for (int j = (int)I.red_L - 1; j >= 0; --j) {
        const uint32_t b = I.bucket_off + lo + (uint32_t)j;
        if (cnt[b]) {
            Xyzz<F> p;
            load_vec(p, P + off[b]);
            xyzz_add(run, p);
        }
        xyzz_add(acc, run);
    }
    // acc = sum_j (j + 1) S_{lo + j}; the buckets' true weights are lo + j + 1
    Xyzz<F> t2;
    xyzz_mul_small(t2, run, lo);
    xyzz_add(acc, t2);
    store_vec(red + I.red_off + tt, acc);
}

template <class F>
__global__ __launch_bounds__(64) void k_final_reduce(const MsmInst* __restrict__ insts, const Xyzz<F>* __restrict__ red,
                                                     Xyzz<F>* __restrict__ out) {
    __shared__ Xyzz<F> lds[64];
    const MsmInst I = insts[blockIdx.x];
    Xyzz<F> acc;
    xyzz_set_inf(acc);
    for (uint32_t t = threadIdx.x; t < I.red_T; t += 64) {
        Xyzz<F> p;
        load_vec(p, red + I.red_off + t);
        xyzz_add(acc, p);
    }
    lds[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 32; w >= 1; w >>= 1) {
        if ((int)threadIdx.x < w) {
            Xyzz<F> o = lds[threadIdx.x + w];
            xyzz_add(acc, o);
            lds[threadIdx.x] = acc;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) store_vec(out + blockIdx.x, acc);
}

// ------------------------------------------------------------------ workspace
struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    void* ensure(size_t bytes) {
        if (bytes > cap) {
            if (p) HIPCHK(hipFree(p));
            size_t nb = std::max(bytes, cap + cap / 2);
            HIPCHK(hipMalloc(&p, nb));
            cap = nb;
        }
        return p;
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
};

struct MsmWorkspace {
    DBuf insts, prefix, redp, counts, offs, cursor, refs, segcnt, segoff_a, segoff_b, pa, pb, red, cub, maxv;
    uint32_t* h_max = nullptr;
    MsmWorkspace() { HIPCHK(hipHostMalloc((void**)&h_max, sizeof(uint32_t))); }
    ~MsmWorkspace() {
        if (h_max) (void)hipHostFree(h_max);
    }
};
MsmWorkspace* msm_ws_create() { return new MsmWorkspace(); }
void msm_ws_destroy(MsmWorkspace* ws) { delete ws; }

static void exclusive_scan(MsmWorkspace* ws, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s) {
    size_t tb = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, s));
    void* t = ws->cub.ensure(tb);
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(t, tb, in, out, n, s));
}

template <class F>
static void msm_run(MsmWorkspace* ws, const MsmInst* ih, int ninst, const Aff<F>* pts, const Fr* scalars,
                    void* out_dev, hipStream_t s) {
    if (ninst <= 0) return;
    std::vector<MsmInst> insts(ih, ih + ninst);
    std::vector<uint64_t> prefix(ninst + 1), redp(ninst + 1);
    uint64_t tot_sc = 0, tot_red = 0, tot_refs = 0;
    uint32_t nb = 0;
    for (int i = 0; i < ninst; ++i) {
        MsmInst& I = insts[i];
        I.bucket_off = nb;
        nb += 1u << (I.c - 1);
        prefix[i] = tot_sc;
        tot_sc += I.size;
        tot_refs += (uint64_t)I.size * I.W;
        uint32_t B = 1u << (I.c - 1);
        I.red_L = std::min<uint32_t>(B, 8);
        I.red_T = B / I.red_L;
        I.red_off = (uint32_t)tot_red;
        redp[i] = tot_red;
        tot_red += I.red_T;
    }
    prefix[ninst] = tot_sc;
    redp[ninst] = tot_red;
    if (tot_refs >= 0xffffffffull) throw std::runtime_error("MSM batch too large");

    auto* d_insts = (MsmInst*)ws->insts.ensure(sizeof(MsmInst) * ninst);
    auto* d_prefix = (uint64_t*)ws->prefix.ensure(8 * (ninst + 1));
    auto* d_redp = (uint64_t*)ws->redp.ensure(8 * (ninst + 1));
    HIPCHK(hipMemcpyAsync(d_insts, insts.data(), sizeof(MsmInst) * ninst, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_prefix, prefix.data(), 8 * (ninst + 1), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_redp, redp.data(), 8 * (ninst + 1), hipMemcpyHostToDevice, s));

    auto* counts = (uint32_t*)ws->counts.ensure(4 * (nb + 1));
    auto* offs = (uint32_t*)ws->offs.ensure(4 * (nb + 1));
    auto* cursor = (uint32_t*)ws->cursor.ensure(4 * (nb + 1));
    auto* refs = (uint32_t*)ws->refs.ensure(4 * std::max<uint64_t>(tot_refs, 1));
    auto* segcnt = (uint32_t*)ws->segcnt.ensure(4 * (nb + 1));
    auto* soa = (uint32_t*)ws->segoff_a.ensure(4 * (nb + 1));
    auto* sob = (uint32_t*)ws->segoff_b.ensure(4 * (nb + 1));
    auto* d_max = (uint32_t*)ws->maxv.ensure(4);

    HIPCHK(hipMemsetAsync(counts, 0, 4 * (nb + 1), s));
    const int gsc = (int)((tot_sc + kLight - 1) / kLight);
    const bool g2 = sizeof(F) == sizeof(Fq2);
    kp_begin(KP_SORT, s);
    hipLaunchKernelGGL(k_msm_digits<false>, dim3(gsc), dim3(kLight), 0, s, d_insts, d_prefix, ninst, tot_sc, scalars,
                       counts, nullptr, nullptr);
    kp_end(32.0 * tot_sc, s);
    exclusive_scan(ws, counts, offs, nb + 1, s);
    HIPCHK(hipMemcpyAsync(cursor, offs, 4 * (nb + 1), hipMemcpyDeviceToDevice, s));
    kp_begin(KP_SORT, s);
    hipLaunchKernelGGL(k_msm_digits<true>, dim3(gsc), dim3(kLight), 0, s, d_insts, d_prefix, ninst, tot_sc, scalars,
                       nullptr, cursor, refs);
    kp_end(32.0 * tot_sc + 4.0 * tot_refs, s);
    {
        size_t tb = 0;
        HIPCHK(hipcub::DeviceReduce::Max(nullptr, tb, counts, d_max, nb, s));
        void* t = ws->cub.ensure(tb);
        HIPCHK(hipcub::DeviceReduce::Max(t, tb, counts, d_max, nb, s));
    }
    HIPCHK(hipMemcpyAsync(ws->h_max, d_max, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    uint32_t maxc = *ws->h_max;

    // level 1: affine references -> XYZZ partials, one per segment
    const size_t psz = sizeof(Xyzz<F>);
    const uint64_t max_segs = tot_refs / kSeg + nb + 1;
    auto* PA = (Xyzz<F>*)ws->pa.ensure(psz * max_segs);
    auto* PB = (Xyzz<F>*)ws->pb.ensure(psz * (max_segs / kSeg + nb + 1));
    const int gb = (int)((nb + 1 + kLight - 1) / kLight);
    hipLaunchKernelGGL(k_seg_counts, dim3(gb), dim3(kLight), 0, s, counts, nb, segcnt);
    exclusive_scan(ws, segcnt, soa, nb + 1, s);
    kp_begin(g2 ? KP_ACC_G2 : KP_ACC_G1, s);
    hipLaunchKernelGGL(k_accum_aff<F>, dim3((unsigned)((max_segs + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, soa,
                       nb, offs, counts, refs, pts, PA);
    // algorithmic bytes: every reference (4 B) and its affine point once, one XYZZ partial per segment
    kp_end((double)tot_refs * (4.0 + sizeof(Aff<F>)) + (double)(tot_refs / kSeg) * psz, s);
    // the per-bucket counts of PA are segcnt, offsets soa
    uint32_t* cur_cnt = segcnt;
    uint32_t* cur_off = soa;
    uint32_t* nxt_off = sob;
    uint32_t* spare_cnt = cursor;  // cursor no longer needed
    Xyzz<F>* cur = PA;
    Xyzz<F>* nxt = PB;
    uint64_t cur_max_segs = max_segs;
    uint32_t m = (maxc + kSeg - 1) / kSeg;
    while (m > 1) {
        hipLaunchKernelGGL(k_seg_counts, dim3(gb), dim3(kLight), 0, s, cur_cnt, nb, spare_cnt);
        exclusive_scan(ws, spare_cnt, nxt_off, nb + 1, s);
        uint64_t nsegs = cur_max_segs / kSeg + nb + 1;
        kp_begin(g2 ? KP_ACCX_G2 : KP_ACCX_G1, s);
        hipLaunchKernelGGL(k_accum_xyzz<F>, dim3((unsigned)((nsegs + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s,
                           nxt_off, nb, cur_off, cur_cnt, cur, nxt);
        kp_end((double)(cur_max_segs + nsegs) * psz, s);
        std::swap(cur, nxt);
        std::swap(cur_off, nxt_off);
        std::swap(cur_cnt, spare_cnt);
        cur_max_segs = nsegs;
        m = (m + kSeg - 1) / kSeg;
    }
    // weighting
    auto* red = (Xyzz<F>*)ws->red.ensure(psz * std::max<uint64_t>(tot_red, 1));
    kp_begin(g2 ? KP_RED_G2 : KP_RED_G1, s);
    hipLaunchKernelGGL(k_bucket_reduce<F>, dim3((unsigned)((tot_red + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s,
                       d_insts, d_redp, ninst, tot_red, cur_cnt, cur_off, cur, red);
    hipLaunchKernelGGL(k_final_reduce<F>, dim3(ninst), dim3(64), 0, s, d_insts, red, (Xyzz<F>*)out_dev);
    kp_end((double)nb * psz, s);
    HIPCHK(hipGetLastError());
}

void msm_run_g1(MsmWorkspace* ws, const MsmInst* insts, int ninst, const G1Aff* pts, const Fr* scalars, void* out,
                hipStream_t s) {
    msm_run<Fq>(ws, insts, ninst, pts, scalars, out, s);
}
void msm_run_g2(MsmWorkspace* ws, const MsmInst* insts, int ninst, const G2Aff* pts, const Fr* scalars, void* out,
                hipStream_t s) {
    msm_run<Fq2>(ws, insts, ninst, pts, scalars, out, s);
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

template <class F>
static void precompute_windows(const Aff<F>* raw, uint64_t count, bool pair_sum, int c, int W, Aff<F>* dst, void* tmp,
                               hipStream_t s) {
    if (!count) return;
    Xyzz<F>* t = (Xyzz<F>*)tmp;
    hipLaunchKernelGGL(k_precompute<F>, dim3((unsigned)((count + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, raw, count,
                       pair_sum ? 1 : 0, c, W, t);
    const uint64_t n = count * (uint64_t)W;
    const uint64_t nt = (n + kNormChunk - 1) / kNormChunk;
    hipLaunchKernelGGL(k_normalize<F>, dim3((unsigned)((nt + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, t, n, dst);
    HIPCHK(hipGetLastError());
}
void precompute_windows_g1(const G1Aff* raw, uint64_t count, bool pair_sum, int c, int W, G1Aff* dst, void* tmp,
                           hipStream_t s) {
    precompute_windows<Fq>(raw, count, pair_sum, c, W, dst, tmp, s);
}
void precompute_windows_g2(const G2Aff* raw, uint64_t count, bool pair_sum, int c, int W, G2Aff* dst, void* tmp,
                           hipStream_t s) {
    precompute_windows<Fq2>(raw, count, pair_sum, c, W, dst, tmp, s);
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
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            Fq c, m;
            load_vec(c, p + k);
            if (k == NF - 1) c.v[11] &= 0x3fffffffu;
            ok &= fq_canon_to_mont(m, c);
            store_vec(p + k, m);
        }
        if (!ok) atomicOr(err, 1);
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
static void fixed_base(const Aff<F>* table, const Fr* scalars, uint64_t n, Aff<F>* out, void* tmp, hipStream_t s) {
    if (!n) return;
    Xyzz<F>* t = (Xyzz<F>*)tmp;
    hipLaunchKernelGGL(k_fixed_base<F>, dim3((unsigned)((n + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, table, scalars,
                       n, t);
    const uint64_t nt = (n + kNormChunk - 1) / kNormChunk;
    hipLaunchKernelGGL(k_normalize<F>, dim3((unsigned)((nt + kHeavy - 1) / kHeavy)), dim3(kHeavy), 0, s, t, n, out);
    HIPCHK(hipGetLastError());
}
void fixed_base_g1(const G1Aff* table, const Fr* scalars, uint64_t n, G1Aff* out, void* tmp, hipStream_t s) {
    fixed_base<Fq>(table, scalars, n, out, tmp, s);
}
void fixed_base_g2(const G2Aff* table, const Fr* scalars, uint64_t n, G2Aff* out, void* tmp, hipStream_t s) {
    fixed_base<Fq2>(table, scalars, n, out, tmp, s);
}

}  // namespace spx
