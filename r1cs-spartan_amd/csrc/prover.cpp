// MI355X prover orchestration: the reference's `MLArgumentForR1CS::prove`
// (/root/reference/src/lib.rs:58-146) with the AHP rounds of src/ahp/prover.rs:109-281 run as
// HIP kernels (mle_kernels.hip, msm.hip) and the Fiat-Shamir transcript on the host.
//
// Sharding: G = 2^g ranks own contiguous blocks of the hypercube (top g bits of x
// or y) for the SpMV, eval_on_x and both sumchecks. Variables bind LSB first, so every rank folds
// locally for the first L - g rounds; each round exchanges 3 Fr per rank, and the last g rounds run
// on the gathered G-entry tables. The MSMs (commitment, openings) split every instance by bucket
// range instead (MsmShard, kernels.hpp): z is replicated, every rank folds the opening tables in
// full (HBM-streaming) and weights 1/G of the buckets; each MSM exchanges one XYZZ point per rank.
// Every rank replays the same transcript, so no challenge broadcast.
#include "prover.hpp"
#include "sc_message.hpp"
#include "pairing.hpp"

#include <type_traits>

#include <algorithm>
#include <sys/prctl.h>

#include <chrono>
#include <thread>
#include <cstdlib>
#include <cstring>

namespace spx {

using host::Affine;
using HFr = host::Fr;
using HFq = host::Fq;
using HFq2 = host::Fq2;

// ====================================================================== context
Ctx::Ctx(int dev) : device(dev) {
    // SPX_BLOCKING_SYNC=1: host waits sleep instead of spinning (frees cores for the transcript
    // hashing pool when many proofs are in flight); must precede the device's first use
    static const bool blocking = [] {
        const char* e = getenv("SPX_BLOCKING_SYNC");
        return e && e[0] == '1';
    }();
    if (blocking) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    SPX_HIP(hipSetDevice(dev));
    SPX_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    SPX_HIP(hipHostMalloc((void**)&pin, kPinBytes));
    SPX_HIP(hipHostGetDevicePointer((void**)&pin_dev_base, pin, 0));
    SPX_HIP(hipMalloc((void**)&ticket, 64));
    SPX_HIP(hipMemset(ticket, 0, 64));
    msm = msm_ws_create();
    comm.reset(new LocalComm());
}
// SPX_SYNC_POLL_US (see Ctx::wait_stream): 0 = hipStreamSynchronize
static int sync_poll_us() {
    static const int v = [] {
        const char* e = getenv("SPX_SYNC_POLL_US");
        return e ? std::max(0, atoi(e)) : 0;
    }();
    return v;
}
void Ctx::wait_stream(hipStream_t s) {
    const int pu = poll_us.load(std::memory_order_relaxed);
    const int us = pu >= 0 ? pu : sync_poll_us();
    if (us <= 0) {
        SPX_HIP(hipStreamSynchronize(s));
        return;
    }
    // one event per (thread, device): waits on this context from different threads (a prove worker,
    // an uploader) never record or query the same event
    struct TlEvents {
        std::vector<hipEvent_t> ev;
        ~TlEvents() {
            for (hipEvent_t e : ev)
                if (e) (void)hipEventDestroy(e);
        }
    };
    thread_local TlEvents tl;
    if ((int)tl.ev.size() <= device) tl.ev.resize(device + 1, nullptr);
    hipEvent_t& ev = tl.ev[device];
    if (!ev) SPX_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    SPX_HIP(hipEventRecord(ev, s));
    // sleeps of tens of microseconds, not the default 50 us timer slack on top: the calling thread's
    // slack is lowered for the poll loop and restored after it
    const int old_slack = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
    (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
    struct Restore {
        int v;
        ~Restore() {
            if (v > 0) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)v, 0, 0, 0);
        }
    } restore{old_slack};
    for (int i = 0;; ++i) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) SPX_HIP(e);
        if (i < 4)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(us));
    }
}
void Ctx::ensure_side() {
    if (side) return;
    SPX_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    SPX_HIP(hipEventCreateWithFlags(&side_ev, hipEventDisableTiming));
    msm_side = msm_ws_create();
}
Ctx::~Ctx() {
    (void)hipSetDevice(device);
    if (msm_side) msm_ws_destroy(msm_side);
    if (side_ev) (void)hipEventDestroy(side_ev);
    if (side) (void)hipStreamDestroy(side);
    msm_ws_destroy(msm);
    scratch.release();
    if (ticket) (void)hipFree(ticket);
    if (pin) (void)hipHostFree(pin);
    if (stream) (void)hipStreamDestroy(stream);
}
uint8_t* Ctx::pin_at(size_t off, size_t bytes, size_t region) {
    if (bytes > region || off + region > kPinBytes) throw SpxError(kDevice, "pinned staging region too small");
    return pin + off;
}


// ====================================================================== public parameters
// Pippenger window bits: 16 for >= 2^14 points (wider windows for >= 2^18 and narrower ones for
// 2^14-2^17 measured slower or equal: profiles/r02_ab6_window_bits.jsonl, r02_ab7_window_mid.jsonl)
int window_bits_for(uint64_t size) {
    const int k = size ? ilog2(size) : 0;
    return k >= 14 ? 16 : std::max(3, k - 2);
}
static int windows_for(int c) { return (256 + c - 1) / c; }

// dst: G2Aff rows, or G1Slot rows (128-byte slots) for G1
template <class A, class D>
static void precompute_level(Ctx& C, const A* raw, uint64_t count, bool pair, int c, int W, D* dst) {
    // chunked to bound the XYZZ temporary: tmp XYZZ [W][chunk] -> affine [W][chunk] -> dst rows (pitch count)
    const uint64_t chunk = std::min<uint64_t>(count, 1ull << 18);
    const size_t xyzz_sz = 2 * sizeof(A);
    DevMem tmp(xyzz_sz * chunk * W), aff(sizeof(A) * chunk * W);
    for (uint64_t j0 = 0; j0 < count; j0 += chunk) {
        const uint64_t cn = std::min(chunk, count - j0);
        const A* src = raw + (pair ? 2 * j0 : j0);
        if constexpr (sizeof(A) == sizeof(G1Aff))
            precompute_windows_g1((const G1Aff*)src, cn, pair, c, W, aff.as<G1Aff>(), tmp.p, C.stream);
        else
            precompute_windows_g2((const G2Aff*)src, cn, pair, c, W, aff.as<G2Aff>(), tmp.p, C.stream);
        if constexpr (sizeof(D) == sizeof(A)) {
            SPX_HIP(hipMemcpy2DAsync(dst + j0, sizeof(A) * count, aff.p, sizeof(A) * cn, sizeof(A) * cn, W,
                                     hipMemcpyDeviceToDevice, C.stream));
        } else {  // one point per slot: a 2-D copy per window, rows = points (pitch 96 -> 128 bytes)
            for (int w = 0; w < W; ++w)
                SPX_HIP(hipMemcpy2DAsync(dst + (uint64_t)w * count + j0, sizeof(D), aff.as<A>() + (uint64_t)w * cn,
                                         sizeof(A), sizeof(A), cn, hipMemcpyDeviceToDevice, C.stream));
        }
    }
    C.sync();
}

void pp_preprocess(Ctx& C, PP& P) {
    const int nv = P.nv;
    const uint64_t n = 1ull << nv;
    P.g1_c = window_bits_for(n);
    P.g1_W = windows_for(P.g1_c);
    P.g1_pre.alloc(sizeof(G1Slot) * n * P.g1_W);
    precompute_level(C, P.g1_level(0), n, false, P.g1_c, P.g1_W, P.g1_pre.as<G1Slot>());
    P.g2_off.assign(nv + 1, 0);
    P.g2_c.assign(nv, 0);
    P.g2_W.assign(nv, 0);
    uint64_t tot = 0;
    for (int i = 0; i < nv; ++i) {
        uint64_t cnt = 1ull << (nv - i - 1);
        P.g2_c[i] = window_bits_for(cnt);
        P.g2_W[i] = windows_for(P.g2_c[i]);
        P.g2_off[i] = tot;
        tot += cnt * P.g2_W[i];
    }
    P.g2_off[nv] = tot;
    P.g2_pre.alloc(sizeof(G2Aff) * std::max<uint64_t>(tot, 1));
    for (int i = 0; i < nv; ++i) {
        uint64_t cnt = 1ull << (nv - i - 1);
        precompute_level(C, P.g2_level(i), cnt, true, P.g2_c[i], P.g2_W[i], P.g2_pre.as<G2Aff>() + P.g2_off[i]);
    }
}

static void pp_alloc_raw(PP& P, int nv) {
    P.nv = nv;
    P.lvl_off.assign(nv + 1, 0);
    uint64_t tot = 0;
    for (int i = 0; i < nv; ++i) {
        P.lvl_off[i] = tot;
        tot += 1ull << (nv - i);
    }
    P.lvl_off[nv] = tot;
    P.g1_raw_mem.alloc(sizeof(G1Aff) * std::max<uint64_t>(tot, 1));
    P.g2_raw_mem.alloc(sizeof(G2Aff) * std::max<uint64_t>(tot, 1));
}

std::unique_ptr<PP> pp_load(Ctx& C, const uint8_t* b, size_t len) {
    auto P = std::make_unique<PP>();
    size_t pos = 0;
    auto need = [&](size_t k) {
        if (pos + k > len) throw SpxError(kSerialization, "truncated public parameter bytes");
    };
    auto u64 = [&]() {
        need(8);
        uint64_t v;
        memcpy(&v, b + pos, 8);
        pos += 8;
        return v;
    };
    uint64_t nv = u64();
    if (nv < 1 || nv > (uint64_t)kMaxLogN) throw SpxError(kSerialization, "bad public parameter nv (1..26 supported)");
    if (u64() != nv) throw SpxError(kSerialization, "powers_of_g length != nv");
    pp_alloc_raw(*P, (int)nv);
    std::vector<size_t> g1_pos(nv), g2_pos(nv);
    for (uint64_t i = 0; i < nv; ++i) {
        if (u64() != (1ull << (nv - i))) throw SpxError(kSerialization, "powers_of_g level size");
        need(96ull << (nv - i));
        g1_pos[i] = pos;
        pos += 96ull << (nv - i);
    }
    if (u64() != nv) throw SpxError(kSerialization, "powers_of_h length != nv");
    for (uint64_t i = 0; i < nv; ++i) {
        if (u64() != (1ull << (nv - i))) throw SpxError(kSerialization, "powers_of_h level size");
        need(192ull << (nv - i));
        g2_pos[i] = pos;
        pos += 192ull << (nv - i);
    }
    need(96 + 192);
    if (!host::g1_from_uncompressed(P->g, b + pos) || !host::g2_from_uncompressed(P->h, b + pos + 96))
        throw SpxError(kSerialization, "bad g / h");
    for (uint64_t i = 0; i < nv; ++i) {
        SPX_HIP(hipMemcpyAsync(P->g1_level((int)i), b + g1_pos[i], 96ull << (nv - i), hipMemcpyHostToDevice, C.stream));
        SPX_HIP(hipMemcpyAsync(P->g2_level((int)i), b + g2_pos[i], 192ull << (nv - i), hipMemcpyHostToDevice, C.stream));
    }
    DevMem err(sizeof(int));
    SPX_HIP(hipMemsetAsync(err.p, 0, sizeof(int), C.stream));
    launch_points_from_bytes_g1(P->g1_raw_mem.as<G1Aff>(), P->lvl_off[nv], err.as<int>(), C.stream);
    launch_points_from_bytes_g2(P->g2_raw_mem.as<G2Aff>(), P->lvl_off[nv], err.as<int>(), C.stream);
    int herr = 0;
    SPX_HIP(hipMemcpyAsync(&herr, err.p, sizeof(int), hipMemcpyDeviceToHost, C.stream));
    C.sync();
    if (herr & 1) throw SpxError(kSerialization, "non-canonical coordinate in public parameters");
    if (herr & 2) throw SpxError(kSerialization, "public parameter point not on the curve");
    pp_preprocess(C, *P);
    return P;
}

// SplitMix64 (the synthetic-input / keygen PRNG shared with oracle/c/oracle.c)
struct SplitMix64 {
    uint64_t s;
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ULL;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    HFr fr() {
        for (;;) {
            uint64_t c[4] = {next(), next(), next(), next() & 0x7FFFFFFFFFFFFFFFULL};
            if (!HFr::geq_p(c)) return HFr::from_canon(c);
        }
    }
};

template <class F>
static std::vector<Affine<F>> fixed_base_table(const Affine<F>& base) {
    std::vector<host::Jac<F>> jac(32 * 256);
    host::Jac<F> outer = host::jac_from(base);
    for (int w = 0; w < 32; ++w) {
        host::Jac<F> acc = host::jac_inf<F>();
        jac[w * 256] = acc;
        for (int d = 1; d < 256; ++d) {
            acc = host::jac_add(acc, outer);
            jac[w * 256 + d] = acc;
        }
        for (int k = 0; k < 8; ++k) outer = host::jac_dbl(outer);
    }
    std::vector<F> zs(jac.size());
    for (size_t i = 0; i < jac.size(); ++i) zs[i] = jac[i].z;
    host::batch_inverse(zs);
    std::vector<Affine<F>> out(jac.size());
    for (size_t i = 0; i < jac.size(); ++i) {
        if (jac[i].z.is_zero()) {
            out[i] = {F::zero(), F::zero(), true};  // device sentinel (0,0)
            continue;
        }
        F zi2 = zs[i] * zs[i];
        out[i] = {jac[i].x * zi2, jac[i].y * zi2 * zs[i], false};
    }
    return out;
}
template <class F, class A>
static void upload_affine(const std::vector<Affine<F>>& v, A* dst, hipStream_t s) {
    static_assert(sizeof(A) == 2 * sizeof(F), "layout");
    std::vector<A> tmp(v.size());
    for (size_t i = 0; i < v.size(); ++i) {
        memcpy((uint8_t*)&tmp[i], &v[i].x, sizeof(F));
        memcpy((uint8_t*)&tmp[i] + sizeof(F), &v[i].y, sizeof(F));
    }
    SPX_HIP(hipMemcpyAsync(dst, tmp.data(), sizeof(A) * v.size(), hipMemcpyHostToDevice, s));
    SPX_HIP(hipStreamSynchronize(s));
}

std::unique_ptr<PP> pp_generate(Ctx& C, int nv, uint64_t seed) {
    if (nv < 1 || nv > kMaxLogN) invalid("keygen: nv out of range (1..26 supported)");
    auto P = std::make_unique<PP>();
    SplitMix64 rng{seed};
    HFr gs = rng.fr(), hs = rng.fr();
    P->t.resize(nv);
    for (int i = 0; i < nv; ++i) P->t[i] = rng.fr();
    P->has_t = true;
    uint64_t c[4];
    gs.to_canon(c);
    P->g = host::jac_to_affine(host::jac_mul(host::jac_from(host::g1_generator()), c));
    hs.to_canon(c);
    P->h = host::jac_to_affine(host::jac_mul(host::jac_from(host::g2_generator()), c));
    pp_alloc_raw(*P, nv);
    const uint64_t tot = P->lvl_off[nv];
    // eq(t[i..], x) scalars for every level (setup.rs:37-60), Montgomery
    DevMem tdev(32 * nv), scal(32 * tot), lo(32 << 14), hi(32 << 14);
    SPX_HIP(hipMemcpyAsync(tdev.p, P->t.data(), 32 * nv, hipMemcpyHostToDevice, C.stream));
    for (int i = 0; i < nv; ++i)
        launch_eq_table(tdev.as<Fr>() + i, nv - i, 0, 1ull << (nv - i), scal.as<Fr>() + P->lvl_off[i], lo.as<Fr>(),
                        hi.as<Fr>(), C.stream);
    {
        auto tg = fixed_base_table(P->g);
        DevMem tab(sizeof(G1Aff) * tg.size()), tmp(2 * sizeof(G1Aff) * tot);
        upload_affine(tg, tab.as<G1Aff>(), C.stream);
        fixed_base_g1(tab.as<G1Aff>(), scal.as<Fr>(), tot, P->g1_raw_mem.as<G1Aff>(), tmp.p, C.stream);
        C.sync();
    }
    {
        auto th = fixed_base_table(P->h);
        DevMem tab(sizeof(G2Aff) * th.size()), tmp(2 * sizeof(G2Aff) * tot);
        upload_affine(th, tab.as<G2Aff>(), C.stream);
        fixed_base_g2(tab.as<G2Aff>(), scal.as<Fr>(), tot, P->g2_raw_mem.as<G2Aff>(), tmp.p, C.stream);
        C.sync();
    }
    pp_preprocess(C, *P);
    return P;
}

std::vector<uint8_t> pp_serialize(Ctx& C, const PP& P) {
    const int nv = P.nv;
    const uint64_t tot = P.lvl_off[nv];
    size_t need = 8 + 8 + 8 + 96 + 192;
    for (int i = 0; i < nv; ++i) need += 16 + (96 + 192) * (1ull << (nv - i));
    std::vector<uint8_t> out(need);
    DevMem t1(sizeof(G1Aff) * tot), t2(sizeof(G2Aff) * tot);
    SPX_HIP(hipMemcpyAsync(t1.p, P.g1_raw_mem.p, sizeof(G1Aff) * tot, hipMemcpyDeviceToDevice, C.stream));
    SPX_HIP(hipMemcpyAsync(t2.p, P.g2_raw_mem.p, sizeof(G2Aff) * tot, hipMemcpyDeviceToDevice, C.stream));
    launch_points_to_canon_g1(t1.as<G1Aff>(), tot, C.stream);
    launch_points_to_canon_g2(t2.as<G2Aff>(), tot, C.stream);
    std::vector<uint8_t> h1(sizeof(G1Aff) * tot), h2(sizeof(G2Aff) * tot);
    SPX_HIP(hipMemcpyAsync(h1.data(), t1.p, h1.size(), hipMemcpyDeviceToHost, C.stream));
    SPX_HIP(hipMemcpyAsync(h2.data(), t2.p, h2.size(), hipMemcpyDeviceToHost, C.stream));
    C.sync();
    auto fix_inf = [](uint8_t* p, size_t bytes) {  // (0,0) sentinel -> ark-serialize infinity (x=0, y=1, flag)
        for (size_t k = 0; k < bytes; ++k)
            if (p[k]) return;
        HFq zero = HFq::zero(), one = HFq::one();
        if (bytes == 96) {
            host::fq_to_bytes(p, zero);
            host::fq_to_bytes(p + 48, one, host::kFlagInf);
        } else {
            host::fq_to_bytes(p, zero);
            host::fq_to_bytes(p + 48, zero);
            host::fq_to_bytes(p + 96, one);
            host::fq_to_bytes(p + 144, zero, host::kFlagInf);
        }
    };
    uint8_t* p = out.data();
    uint64_t u = (uint64_t)nv;
    memcpy(p, &u, 8), p += 8;
    memcpy(p, &u, 8), p += 8;
    for (int i = 0; i < nv; ++i) {
        uint64_t k = 1ull << (nv - i);
        memcpy(p, &k, 8), p += 8;
        memcpy(p, h1.data() + 96 * P.lvl_off[i], 96 * k);
        for (uint64_t j = 0; j < k; ++j) fix_inf(p + 96 * j, 96);
        p += 96 * k;
    }
    memcpy(p, &u, 8), p += 8;
    for (int i = 0; i < nv; ++i) {
        uint64_t k = 1ull << (nv - i);
        memcpy(p, &k, 8), p += 8;
        memcpy(p, h2.data() + 192 * P.lvl_off[i], 192 * k);
        for (uint64_t j = 0; j < k; ++j) fix_inf(p + 192 * j, 192);
        p += 192 * k;
    }
    host::g1_to_uncompressed(p, P.g), p += 96;
    host::g2_to_uncompressed(p, P.h), p += 192;
    return out;
}

// ====================================================================== index
static void check_csr(const HostCsr& m, uint64_t n) {
    if (m.n != n) invalid("matrix size is inconsistent with number of constraints");
    if (m.rp.size() != n + 1 || m.rp[0] != 0) invalid("malformed row_ptr");
    for (uint64_t x = 0; x < n; ++x)
        if (m.rp[x + 1] < m.rp[x]) invalid("malformed row_ptr");
    const uint64_t nnz = m.rp[n];
    if (m.col.size() < nnz || m.val.size() < 32 * nnz) invalid("malformed CSR arrays");
    for (uint64_t k = 0; k < nnz; ++k)
        if (m.col[k] >= n) invalid("sparse index out of bound");
}

// upload a rank-local block [lo, lo + cnt) of `ptr`-indexed segments, with long-row chunking
static void upload_sparse(Ctx& C, DevSparse& D, const std::vector<uint64_t>* ptrs, const std::vector<uint32_t>* idxs,
                          const std::vector<uint8_t>* vals, uint64_t lo, uint64_t cnt, int* err_dev) {
    std::vector<LongChunk> chunks;
    std::vector<LongRow> lrows;
    for (int m = 0; m < 3; ++m) {
        const uint64_t base = ptrs[m][lo], end = ptrs[m][lo + cnt], nnz = end - base;
        std::vector<uint64_t> p(cnt + 1);
        for (uint64_t x = 0; x <= cnt; ++x) p[x] = ptrs[m][lo + x] - base;
        D.ptr[m].alloc(8 * (cnt + 1));
        D.idx[m].alloc(4 * std::max<uint64_t>(nnz, 1));
        D.val[m].alloc(32 * std::max<uint64_t>(nnz, 1));
        SPX_HIP(hipMemcpyAsync(D.ptr[m].p, p.data(), 8 * (cnt + 1), hipMemcpyHostToDevice, C.stream));
        if (nnz) {
            SPX_HIP(hipMemcpyAsync(D.idx[m].p, idxs[m].data() + base, 4 * nnz, hipMemcpyHostToDevice, C.stream));
            SPX_HIP(hipMemcpyAsync(D.val[m].p, vals[m].data() + 32 * base, 32 * nnz, hipMemcpyHostToDevice, C.stream));
            launch_to_mont(D.val[m].as<Fr>(), nnz, err_dev, C.stream);
        }
        for (uint64_t x = 0; x < cnt; ++x) {
            if (p[x + 1] - p[x] <= kLongRow) continue;
            LongRow lr{};
            lr.m = (uint32_t)m;
            lr.x = x;
            lr.chunk_begin = (uint32_t)chunks.size();
            for (uint64_t k = p[x]; k < p[x + 1]; k += kChunk) {
                LongChunk ch{};
                ch.m = (uint32_t)m;
                ch.begin = k;
                ch.end = std::min(k + kChunk, p[x + 1]);
                chunks.push_back(ch);
            }
            lr.chunk_end = (uint32_t)chunks.size();
            lrows.push_back(lr);
        }
        C.sync();  // host vectors go out of scope
    }
    D.nchunks = (int)chunks.size();
    D.nlrows = (int)lrows.size();
    if (D.nchunks) {
        D.chunks.alloc(sizeof(LongChunk) * chunks.size());
        D.lrows.alloc(sizeof(LongRow) * lrows.size());
        SPX_HIP(hipMemcpyAsync(D.chunks.p, chunks.data(), sizeof(LongChunk) * chunks.size(), hipMemcpyHostToDevice, C.stream));
        SPX_HIP(hipMemcpyAsync(D.lrows.p, lrows.data(), sizeof(LongRow) * lrows.size(), hipMemcpyHostToDevice, C.stream));
        C.sync();
    }
}

// Rows [lo, lo + cnt) of A, B, C as the column-sorted entry list (kernels.hpp: SpmvSlicedView) when
// every one of them has at most one entry: the entries by column, within a column in (matrix, row)
// order; an empty (row, matrix) is a zero entry whose column is the row (a product of 0 without a
// branch). Returns false, uploading nothing, otherwise (the CSR path then serves the SpMV).
static bool upload_sliced(Ctx& C, DevSliced& S, const HostCsr* mats, uint64_t n, uint64_t lo, uint64_t cnt,
                          int* err_dev) {
    if (n < (1ull << 12)) return false;
    for (int m = 0; m < 3; ++m)
        for (uint64_t x = lo; x < lo + cnt; ++x)
            if (mats[m].rp[x + 1] - mats[m].rp[x] > 1) return false;
    auto col_of = [&](int m, uint64_t x) -> uint32_t {
        const uint64_t k = mats[m].rp[x];
        return mats[m].rp[x + 1] > k ? mats[m].col[k] : (uint32_t)x;
    };
    std::vector<uint64_t> start(n + 1, 0);  // counting sort by column
    for (int m = 0; m < 3; ++m)
        for (uint64_t x = lo; x < lo + cnt; ++x) ++start[col_of(m, x) + 1];
    for (uint64_t c = 0; c < n; ++c) start[c + 1] += start[c];
    const uint64_t E = start[n];
    std::vector<uint32_t> col(E), dst(E);
    std::vector<uint8_t> val(32 * E, 0);
    for (int m = 0; m < 3; ++m)
        for (uint64_t x = lo; x < lo + cnt; ++x) {
            const uint32_t c = col_of(m, x);
            const uint64_t e = start[c]++;
            col[e] = c;
            dst[e] = (uint32_t)(x - lo) | ((uint32_t)m << 30);
            const uint64_t k = mats[m].rp[x];
            if (mats[m].rp[x + 1] > k) memcpy(val.data() + 32 * e, mats[m].val.data() + 32 * k, 32);
        }
    S.val.alloc(32 * E);
    S.col.alloc(4 * E);
    S.dst.alloc(4 * E);
    SPX_HIP(hipMemcpyAsync(S.val.p, val.data(), 32 * E, hipMemcpyHostToDevice, C.stream));
    SPX_HIP(hipMemcpyAsync(S.col.p, col.data(), 4 * E, hipMemcpyHostToDevice, C.stream));
    SPX_HIP(hipMemcpyAsync(S.dst.p, dst.data(), 4 * E, hipMemcpyHostToDevice, C.stream));
    launch_to_mont(S.val.as<Fr>(), E, err_dev, C.stream);
    C.sync();  // host vectors go out of scope
    S.entries = E;
    S.on = true;
    return true;
}

// CSC copy of M for eval_on_x (rows ascending within a column). The reference inserts every
// (xy_combine(x, y), value) pair into a SparseMLExtensionMap (r1cs_reader.rs:98-108), so when a
// row repeats a column only the LAST entry of that row survives; sum_over_y (r1cs_reader.rs:75-85)
// keeps adding every entry, so only this copy drops the superseded ones.
static void build_csc(const HostCsr& M, uint64_t n, std::vector<uint64_t>& cp, std::vector<uint32_t>& rows,
                      std::vector<uint8_t>& vals) {
    const uint64_t nnz = M.rp[n];
    std::vector<uint8_t> dead(nnz, 0);
    std::vector<uint64_t> last_row(n, ~0ull), last_k(n, 0);
    uint64_t live = 0;
    for (uint64_t x = 0; x < n; ++x)
        for (uint64_t k = M.rp[x]; k < M.rp[x + 1]; ++k) {
            const uint32_t y = M.col[k];
            if (last_row[y] == x)
                dead[last_k[y]] = 1;
            else
                ++live;
            last_row[y] = x;
            last_k[y] = k;
        }
    cp.assign(n + 1, 0);
    for (uint64_t k = 0; k < nnz; ++k)
        if (!dead[k]) cp[M.col[k] + 1]++;
    for (uint64_t y = 0; y < n; ++y) cp[y + 1] += cp[y];
    std::vector<uint64_t> cur(cp.begin(), cp.end() - 1);
    rows.assign(live, 0);
    vals.assign(32 * live, 0);
    for (uint64_t x = 0; x < n; ++x)
        for (uint64_t k = M.rp[x]; k < M.rp[x + 1]; ++k) {
            if (dead[k]) continue;
            const uint64_t pos = cur[M.col[k]]++;
            rows[pos] = (uint32_t)x;
            memcpy(&vals[32 * pos], &M.val[32 * k], 32);
        }
}

// The column stream of the rank-local columns [lo, lo + cnt) of (up to) three CSC matrices for
// k_col_stream (kernels.hpp: ColStreamView). A column's entries are A's, then B's, then C's (rows
// ascending); columns are sorted by entry count, longest first, inside windows of 64 kColWindow columns and
// dealt to the lanes of 64-column slices, so a wave's lanes run columns of nearly equal length (the
// per-column loop left lanes of Poisson-length columns idle for most of a wave's steps). Columns with
// more than kLongCol entries take the chunked long path instead.
static void upload_cols(Ctx& C, DevColStream& D, const std::vector<uint64_t>* cps, const std::vector<uint32_t>* rws,
                        const std::vector<uint8_t>* vals, uint64_t lo, uint64_t cnt, int* err_dev) {
    std::vector<uint32_t> len(cnt);
    std::vector<uint64_t> long_cols;
    uint64_t live = 0;
    for (uint64_t y = 0; y < cnt; ++y) {
        uint64_t L = 0;
        for (int m = 0; m < 3; ++m) L += cps[m][lo + y + 1] - cps[m][lo + y];
        live += L;
        len[y] = L > kLongCol ? 0u : (uint32_t)L;
        if (L > kLongCol) long_cols.push_back(y);
    }
    D.entries = live;
    const uint64_t win = 64ull * kColWindow, nslices = (cnt + 63) / 64;
    D.nslices = (uint32_t)nslices;
    std::vector<ColSlice> sl(nslices);
    std::vector<uint32_t> lanes(64 * nslices, kColNone);
    std::vector<uint64_t> order;
    uint64_t tot = 0;
    for (uint64_t w0 = 0; w0 < cnt; w0 += win) {
        const uint64_t wn = std::min(win, cnt - w0);
        order.resize(wn);
        for (uint64_t i = 0; i < wn; ++i) order[i] = w0 + i;
        std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return len[a] > len[b]; });
        for (uint64_t s0 = 0; s0 < wn; s0 += 64) {
            const uint64_t si = (w0 + s0) / 64;
            uint32_t mx = 0;
            for (uint64_t l = 0; l < 64 && s0 + l < wn; ++l) {
                const uint64_t y = order[s0 + l];
                lanes[64 * si + l] = (uint32_t)y | (len[y] << 26);
                mx = std::max(mx, len[y]);
            }
            sl[si].off = tot;
            sl[si].len = mx;
            tot += 64ull * mx;
        }
    }
    std::vector<uint32_t> rowm(std::max<uint64_t>(tot, 1), 0);
    std::vector<uint8_t> val(32 * std::max<uint64_t>(tot, 1), 0);
    for (uint64_t si = 0; si < nslices; ++si)
        for (uint64_t l = 0; l < 64; ++l) {
            const uint32_t info = lanes[64 * si + l];
            if (info == kColNone) continue;
            const uint64_t y = info & 0x3FFFFFFu;
            if (!len[y]) continue;
            uint64_t j = 0;
            for (uint32_t m = 0; m < 3; ++m)
                for (uint64_t k = cps[m][lo + y]; k < cps[m][lo + y + 1]; ++k, ++j) {
                    const uint64_t e = sl[si].off + 64 * j + l;
                    rowm[e] = rws[m][k] | (m << 30);
                    memcpy(&val[32 * e], &vals[m][32 * k], 32);
                }
        }
    D.slices.alloc(sizeof(ColSlice) * std::max<uint64_t>(nslices, 1));
    D.lanes.alloc(4 * std::max<uint64_t>(lanes.size(), 1));
    D.rowm.alloc(4 * rowm.size());
    D.val.alloc(val.size());
    if (nslices) {
        SPX_HIP(hipMemcpyAsync(D.slices.p, sl.data(), sizeof(ColSlice) * nslices, hipMemcpyHostToDevice, C.stream));
        SPX_HIP(hipMemcpyAsync(D.lanes.p, lanes.data(), 4 * lanes.size(), hipMemcpyHostToDevice, C.stream));
    }
    SPX_HIP(hipMemcpyAsync(D.rowm.p, rowm.data(), 4 * rowm.size(), hipMemcpyHostToDevice, C.stream));
    SPX_HIP(hipMemcpyAsync(D.val.p, val.data(), val.size(), hipMemcpyHostToDevice, C.stream));
    launch_to_mont(D.val.as<Fr>(), val.size() / 32, err_dev, C.stream);
    C.sync();  // host vectors go out of scope
    // long columns: per-matrix entry arrays holding only their entries, chunked (k_sparse_chunks)
    std::vector<uint32_t> li[3];
    std::vector<uint8_t> lvv[3];
    std::vector<LongChunk> chunks;
    std::vector<LongRow> lrows;
    for (uint32_t m = 0; m < 3; ++m)
        for (uint64_t y : long_cols) {
            const uint64_t b = cps[m][lo + y], e = cps[m][lo + y + 1];
            if (b == e) continue;
            LongRow lr{};
            lr.m = m;
            lr.x = y;
            lr.chunk_begin = (uint32_t)chunks.size();
            const uint64_t base = li[m].size();
            for (uint64_t k = 0; k < e - b; k += kChunk) {
                LongChunk ch{};
                ch.m = m;
                ch.begin = base + k;
                ch.end = base + std::min<uint64_t>(k + kChunk, e - b);
                chunks.push_back(ch);
            }
            lr.chunk_end = (uint32_t)chunks.size();
            lrows.push_back(lr);
            li[m].insert(li[m].end(), rws[m].begin() + b, rws[m].begin() + e);
            lvv[m].insert(lvv[m].end(), vals[m].begin() + 32 * b, vals[m].begin() + 32 * e);
        }
    DevSparse& L = D.longc;
    for (int m = 0; m < 3; ++m) {
        L.ptr[m].alloc(8);
        L.idx[m].alloc(4 * std::max<size_t>(li[m].size(), 1));
        L.val[m].alloc(std::max<size_t>(lvv[m].size(), 32));
        if (!li[m].empty()) {
            SPX_HIP(hipMemcpyAsync(L.idx[m].p, li[m].data(), 4 * li[m].size(), hipMemcpyHostToDevice, C.stream));
            SPX_HIP(hipMemcpyAsync(L.val[m].p, lvv[m].data(), lvv[m].size(), hipMemcpyHostToDevice, C.stream));
            launch_to_mont(L.val[m].as<Fr>(), li[m].size(), err_dev, C.stream);
        }
    }
    L.nchunks = (int)chunks.size();
    L.nlrows = (int)lrows.size();
    if (L.nchunks) {
        L.chunks.alloc(sizeof(LongChunk) * chunks.size());
        L.lrows.alloc(sizeof(LongRow) * lrows.size());
        SPX_HIP(hipMemcpyAsync(L.chunks.p, chunks.data(), sizeof(LongChunk) * chunks.size(), hipMemcpyHostToDevice, C.stream));
        SPX_HIP(hipMemcpyAsync(L.lrows.p, lrows.data(), sizeof(LongRow) * lrows.size(), hipMemcpyHostToDevice, C.stream));
    }
    C.sync();
}

// sink: update(data, len) of one state or of a group of states absorbing the same bytes
template <class Sink>
static void feed_matrix(Sink&& h, const HostCsr& m) {
    // CanonicalSerialize of MatrixExtension { constraint: Vec<Vec<(F, usize)>>, num_constraints: usize },
    // streamed through a 64 KiB staging block (u64 lengths, then (32-byte Fr, u64 column) per entry)
    constexpr size_t kBlk = 1 << 16;
    alignas(64) uint8_t buf[kBlk];
    size_t len = 0;
    auto put64 = [&](uint64_t v) {
        if (len + 8 > kBlk) h.update(buf, len), len = 0;
        memcpy(buf + len, &v, 8);
        len += 8;
    };
    put64(m.n);
    const uint8_t* val = m.val.data();
    const uint32_t* col = m.col.data();
    for (uint64_t x = 0; x < m.n; ++x) {
        put64(m.rp[x + 1] - m.rp[x]);
        for (uint64_t k = m.rp[x]; k < m.rp[x + 1]; ++k) {
            if (len + 40 > kBlk) h.update(buf, len), len = 0;
            memcpy(buf + len, val + 32 * k, 32);
            const uint64_t c = col[k];
            memcpy(buf + len + 32, &c, 8);
            len += 40;
        }
    }
    put64(m.n);
    h.update(buf, len);
}

Blake2s absorb_matrices(const Index& I) {
    Blake2s h;
    for (int m = 0; m < 3; ++m) feed_matrix(h, I.m[m]);
    return h;
}

void absorb_matrices_lanes(const Index& I, Blake2s* out, int k) {
    for (int l = 0; l < k; ++l) out[l].reset();
    struct Lanes {
        Blake2s* st;
        int k;
        void update(const void* d, size_t n) { blake2s_update_lanes(st, k, d, n); }
    } sink{out, k};
    for (int m = 0; m < 3; ++m) feed_matrix(sink, I.m[m]);
}

std::unique_ptr<Index> index_build(Ctx& C, const HostCsr* mats) {
    auto I = std::make_unique<Index>();
    const uint64_t n = mats[0].n;
    if (!is_pow2(n)) invalid("Matrix width should be a power of 2.");  // indexer.rs:49-51
    if (n < 2) invalid("at least 2 constraints are required");
    if (n > (1ull << kMaxLogN)) invalid("more than 2^26 constraints are not supported");
    for (int m = 0; m < 3; ++m) check_csr(mats[m], n);
    I->n = n;
    I->log_n = ilog2(n);
    for (int m = 0; m < 3; ++m) I->m[m] = mats[m];
    const int G = C.comm->size(), rank = C.comm->rank();
    if (!is_pow2((uint64_t)G) || (uint64_t)G > n / 2) invalid("world size must be a power of two <= n / 2");
    I->G = G;
    I->rank = rank;
    const uint64_t nl = n / G, lo = (uint64_t)rank * nl;
    DevMem err(sizeof(int));
    SPX_HIP(hipMemsetAsync(err.p, 0, sizeof(int), C.stream));
    // rows (CSR) for sum_over_y
    std::vector<uint64_t> rps[3];
    std::vector<uint32_t> cols[3];
    std::vector<uint8_t> vals[3];
    for (int m = 0; m < 3; ++m) rps[m] = mats[m].rp;
    if (!upload_sliced(C, I->rows_sliced, mats, n, lo, nl, err.as<int>())) {
        const std::vector<uint32_t>* ci[3] = {&mats[0].col, &mats[1].col, &mats[2].col};
        const std::vector<uint8_t>* vi[3] = {&mats[0].val, &mats[1].val, &mats[2].val};
        std::vector<uint32_t> c3[3];
        std::vector<uint8_t> v3[3];
        for (int m = 0; m < 3; ++m) c3[m] = *ci[m], v3[m] = *vi[m];
        upload_sparse(C, I->rows, rps, c3, v3, lo, nl, err.as<int>());
    }
    // columns (CSC, last entry of a repeated (x, y) kept) for eval_on_x
    for (int m = 0; m < 3; ++m) build_csc(mats[m], n, rps[m], cols[m], vals[m]);
    upload_cols(C, I->cols, rps, cols, vals, lo, nl, err.as<int>());
    {
        double e_rows = 0;
        for (int m = 0; m < 3; ++m) e_rows += (double)(mats[m].rp[lo + nl] - mats[m].rp[lo]);
        if (I->rows_sliced.on) {
            // column-sorted list: 40 B per entry (value, column, row | matrix), z read once (each XCD
            // its contiguous eighth), one 32 B output per local row and matrix
            I->rows_index_bytes = 40.0 * (double)I->rows_sliced.entries;
            I->rows_bytes = I->rows_index_bytes + 32.0 * n + 3.0 * 32.0 * nl;
        } else {  // CSR: value + column + a 32 B gather of z per entry, row pointers, 3 outputs
            I->rows_index_bytes = 36.0 * e_rows + 3.0 * 8.0 * nl;
            I->rows_bytes = 68.0 * e_rows + 3.0 * 8.0 * nl + 3.0 * 32.0 * nl;
        }
        // column stream: 32 B value + 4 B row|matrix per entry (eq(r_x) is gathered from its two
        // cache-resident factor tables, not from HBM); 4 B lane word and one 32 B output per column
        I->cols_bytes = 36.0 * (double)I->cols.entries + 4.0 * nl + 32.0 * nl;
    }
    int herr = 0;
    SPX_HIP(hipMemcpyAsync(&herr, err.p, sizeof(int), hipMemcpyDeviceToHost, C.stream));
    C.sync();
    if (herr) throw SpxError(kSerialization, "non-canonical field element in matrix");
    // witness-independent transcript prefix (lib.rs:61-64), absorbed once
    for (int m = 0; m < 3; ++m) feed_matrix(I->cache, mats[m]);
    I->has_cache = true;
    return I;
}

std::unique_ptr<Witness> witness_upload(Ctx& C, const uint8_t* v, size_t nv, const uint8_t* w, size_t nw) {
    if (!is_pow2(nv)) invalid("public input should be power of two");  // prover.rs:114-116
    auto W = std::make_unique<Witness>();
    W->n = nv + nw;
    W->v.assign(v, v + 32 * nv);
    W->z.alloc(32 * std::max<uint64_t>(W->n, 1));
    SPX_HIP(hipMemcpyAsync(W->z.p, v, 32 * nv, hipMemcpyHostToDevice, C.stream));
    if (nw) SPX_HIP(hipMemcpyAsync(W->z.as<uint8_t>() + 32 * nv, w, 32 * nw, hipMemcpyHostToDevice, C.stream));
    DevMem err(sizeof(int));
    SPX_HIP(hipMemsetAsync(err.p, 0, sizeof(int), C.stream));
    launch_to_mont(W->z.as<Fr>(), W->n, err.as<int>(), C.stream);
    int herr = 0;
    SPX_HIP(hipMemcpyAsync(&herr, err.p, sizeof(int), hipMemcpyDeviceToHost, C.stream));
    C.sync();
    if (herr) throw SpxError(kSerialization, "non-canonical field element in witness");
    return W;
}

// ====================================================================== prove helpers
struct Ser {
    std::vector<uint8_t> b;
    void u64(uint64_t v) {
        uint8_t t[8];
        memcpy(t, &v, 8);
        b.insert(b.end(), t, t + 8);
    }
    void fr(const HFr& x) {
        uint8_t t[32];
        host::fr_to_bytes(t, x);
        b.insert(b.end(), t, t + 32);
    }
    void raw(const uint8_t* p, size_t k) { b.insert(b.end(), p, p + k); }
};

static HFr ld_hfr(const uint8_t* p) {  // device Montgomery bytes -> host Fr
    HFr r;
    memcpy(r.v, p, 32);
    return r;
}
static Fr dev_fr(const HFr& x) {  // host Fr -> device Fr (same Montgomery bytes), e.g. a kernel argument
    Fr r;
    memcpy(&r, x.v, 32);
    return r;
}
static HFr eq1(const HFr& tau, const HFr& t) {  // eq(tau, t) = 1 - tau - t + 2 tau t  (eq.rs:14)
    HFr tt = tau * t;
    return HFr::one() - tau - t + tt + tt;
}

size_t proof_size(int L) {
    const size_t open = 32 + 96 + 8 + 96 * (size_t)L;
    return 56 + open + 16 + 8 + (size_t)L * (8 + 32 * (size_t)(L + 3)) + 96 + 16 + 8 + (size_t)L * (8 + 96) + open;
}

struct Timer {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    double us() const {
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
};

// Host CPU of the proving threads by phase, process-wide (spx_host_phase_stats): the calling thread's
// CPU time (CLOCK_THREAD_CPUTIME_ID) between prove()'s phase marks, with the wall time and the count.
// A rank of a G-rank proof replays the whole transcript and host arithmetic of every proof while its
// device work is 1/G, so this host work is what does not divide when proofs are sharded.
static uint64_t thread_cpu_ns() {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
static const char* const kPhaseNames[kHostPhases] = {"transcript_matrices", "commit", "open_rv", "sumcheck1",
                                                     "eval_on_x", "sumcheck2", "open_ry"};
static std::atomic<uint64_t> g_phase_cpu[kHostPhases], g_phase_wall[kHostPhases], g_phase_cnt[kHostPhases];
void host_phase_stats(uint64_t* out) {  // [phase][cpu ns, wall ns, count]
    for (int i = 0; i < kHostPhases; ++i) {
        out[3 * i] = g_phase_cpu[i].load();
        out[3 * i + 1] = g_phase_wall[i].load();
        out[3 * i + 2] = g_phase_cnt[i].load();
    }
}

// device MSM output (XYZZ, R = 2^384 Montgomery limbs) -> host Jacobian without an inversion:
// Z = ZZ ZZZ, X = x Z^2 = X ZZ ZZZ^2, Y = y Z^3 = Y ZZ^3 ZZZ^2 (ZZ = 0: infinity)
template <class F>
static host::Jac<F> xyzz_bytes_to_jac(const uint8_t* p) {
    F X, Y, ZZ, ZZZ;
    memcpy(&X, p, sizeof(F));
    memcpy(&Y, p + sizeof(F), sizeof(F));
    memcpy(&ZZ, p + 2 * sizeof(F), sizeof(F));
    memcpy(&ZZZ, p + 3 * sizeof(F), sizeof(F));
    if (ZZ.is_zero()) return host::jac_inf<F>();
    const F z3s = ZZZ * ZZZ;
    return {X * ZZ * z3s, Y * (ZZ * ZZ * ZZ) * z3s, ZZ * ZZZ};
}
template <class F>
static std::vector<Affine<F>> jac_to_affine_batch(const std::vector<host::Jac<F>>& v) {
    std::vector<F> zi(v.size());
    for (size_t k = 0; k < v.size(); ++k) zi[k] = v[k].z;
    host::batch_inverse(zi);
    std::vector<Affine<F>> out(v.size());
    for (size_t k = 0; k < v.size(); ++k) {
        if (v[k].z.is_zero()) {
            out[k] = {F::zero(), F::one(), true};
            continue;
        }
        const F z2 = zi[k] * zi[k];
        out[k] = {v[k].x * z2, v[k].y * z2 * zi[k], false};
    }
    return out;
}

// Outputs of an MSM batch (`cnt` instances, this rank's bucket ranges) -> the affine MSM results:
// every rank's partial of every instance, gathered over the communicator and summed.
template <class F>
static std::vector<Affine<F>> msm_results(Comm& comm, const uint8_t* xyzz, int cnt) {
    const size_t psz = 4 * sizeof(F);
    const int G = comm.size();
    std::vector<uint8_t> all;
    const uint8_t* src = xyzz;
    if (G > 1) {
        all.resize(psz * cnt * G);
        comm.allgather(xyzz, all.data(), psz * cnt);
        src = all.data();
    }
    std::vector<host::Jac<F>> sum(cnt, host::jac_inf<F>());
    for (int r = 0; r < G; ++r)
        for (int k = 0; k < cnt; ++k) sum[k] = host::jac_add(sum[k], xyzz_bytes_to_jac<F>(src + psz * ((size_t)r * cnt + k)));
    return jac_to_affine_batch(sum);
}

static uint32_t msm_status(const uint8_t* h, bool g2, int cnt) {
    uint32_t st;
    memcpy(&st, h + msm_out_bytes(g2, cnt) - 16, 4);
    return st;
}

static MsmShard shard_of(const Comm& comm) {
    MsmShard sh;
    sh.rank = comm.rank();
    sh.world = comm.size();
    return sh;
}

static std::vector<HFr> allgather_fr(Comm& comm, const std::vector<HFr>& mine) {
    const int G = comm.size();
    std::vector<HFr> all(mine.size() * G);
    comm.allgather(mine.data(), all.data(), sizeof(HFr) * mine.size());
    return all;
}

// ---------------------------------------------------------------- commit (commit.rs:17-29)
// Split in two so the MSM runs while the host absorbs the matrices into the transcript: launch
// enqueues the MSM and the copy of its XYZZ result into pinned memory; finish waits and decodes.
// Proof-sharded (world > 1): every rank holds all of z and weights its range of the buckets.
static void commit_launch(Ctx& C, PP& P, const Fr* z, uint64_t n, const MsmShard& sh) {
    MsmInst inst{};
    inst.pts_off = 0;
    inst.stride = (uint32_t)n;
    inst.scalar_off = 0;
    inst.size = (uint32_t)n;
    inst.c = (uint32_t)P.g1_c;
    inst.W = (uint32_t)P.g1_W;
    const size_t ob = msm_out_bytes(false, 1);
    void* out = C.buf(Ctx::kSlotCommit, ob);
    msm_run_g1(C.msm, &inst, 1, P.g1_pre.as<G1Slot>(), z, out, C.stream, sh);
    SPX_HIP(hipMemcpyAsync(C.pin_at(Ctx::kPinCommit, ob, 4 << 10), out, ob, hipMemcpyDeviceToHost, C.stream));
}
static Affine<HFq> commit_finish(Ctx& C, PP& P, const Fr* z, uint64_t n, Comm& comm) {
    C.sync();
    const uint8_t* h = C.pin_at(Ctx::kPinCommit, msm_out_bytes(false, 1), 4 << 10);
    if (msm_status(h, false, 1) & kMsmOverflow) {  // compacted keys overflowed: once more with a slot per digit
        msm_ws_note_overflow(C.msm);
        ++C.msm_reruns;
        MsmShard sh = shard_of(comm);
        sh.dense = true;
        commit_launch(C, P, z, n, sh);
        C.sync();
    }
    return msm_results<HFq>(comm, h, 1)[0];
}

// ---------------------------------------------------------------- level 0 of both openings
// open.rs:37-49 at i = 0 reads only the table itself: q_L[b] = z[2b+1] - z[2b] does not depend on
// the opening point, so pi_0 = MSM(powers_of_h[0], q_L) is the same group element in the opening at
// (r_v, 0..0) (prover.rs:152) and in the one at r_y (prover.rs:275). It is computed once per proof,
// launched right behind the commitment (before any challenge exists, overlapping the host's
// absorption of the matrices) and handed to both open_z calls: a quarter of the proof's G2 work.
// on_side: on the context's second stream (ordered after the main stream's work so far), without
// kernel statistics (they time the main stream only)
static void lvl0_launch(Ctx& C, PP& P, const Fr* z, int L, const MsmShard& sh, bool on_side = false) {
    const uint64_t half = (1ull << L) / 2;
    hipStream_t st = C.stream;
    MsmWorkspace* ws = C.msm;
    struct KpRestore {
        KProf* kp = g_kprof;
        ~KpRestore() { g_kprof = kp; }
    } restore;
    if (on_side) {  // C.side_ev: recorded on the main stream once z is in place (prove)
        SPX_HIP(hipStreamWaitEvent(C.side, C.side_ev, 0));
        st = C.side;
        ws = C.msm_side;
        g_kprof = nullptr;
    }
    Fr* q = C.buf<Fr>(Ctx::kSlotLvl0Q, 32 * half);
    launch_open_level(z, nullptr, q, Fr{}, half, st);
    MsmInst I{};
    I.pts_off = P.g2_off[0];
    I.stride = (uint32_t)half;
    I.scalar_off = 0;
    I.size = (uint32_t)half;
    I.c = (uint32_t)P.g2_c[0];
    I.W = (uint32_t)P.g2_W[0];
    const size_t ob = msm_out_bytes(true, 1);
    void* out = C.buf(Ctx::kSlotLvl0Out, ob);
    msm_run_g2(ws, &I, 1, P.g2_pre.as<G2Aff>(), q, out, st, sh);
    SPX_HIP(hipMemcpyAsync(C.pin_at(Ctx::kPinLvl0, ob, 4 << 10), out, ob, hipMemcpyDeviceToHost, st));
}
static Affine<HFq2> lvl0_finish(Ctx& C, PP& P, const Fr* z, int L, Comm& comm, bool on_side = false) {
    if (on_side)
        C.side_sync();
    else
        C.sync();
    const uint8_t* h = C.pin_at(Ctx::kPinLvl0, msm_out_bytes(true, 1), 4 << 10);
    if (msm_status(h, true, 1) & kMsmOverflow) {
        msm_ws_note_overflow(on_side ? C.msm_side : C.msm);
        ++C.msm_reruns;
        MsmShard sh = shard_of(comm);
        sh.dense = true;
        lvl0_launch(C, P, z, L, sh, on_side);
        if (on_side)
            C.side_sync();
        else
            C.sync();
    }
    return msm_results<HFq2>(comm, h, 1)[0];
}

// ---------------------------------------------------------------- open (open.rs:19-58)
struct OpenOut {
    HFr eval;
    std::vector<Affine<HFq2>> proofs;
};
// Every level's quotient and fold run here on the whole table (also on proof-sharded ranks, which
// all hold z: the folds are HBM-streaming and cheap, and the bucket-range MSM needs every scalar);
// all MSMs of the opening are one batch. proof0: the shared level-0 proof (lvl0_launch /
// lvl0_finish), or null to compute every level here.
static OpenOut open_z(Ctx& C, PP& P, const Fr* z, int L, const std::vector<HFr>& point, Comm& comm,
                      const Affine<HFq2>* proof0 = nullptr) {
    const uint64_t n = 1ull << L;
    const int first = proof0 ? 1 : 0;  // first level whose MSM runs here
    OpenOut res;
    res.proofs.resize(L);
    if (proof0) res.proofs[0] = *proof0;
    Fr* q = C.buf<Fr>(Ctx::kSlotOpenQ, 32 * n);
    Fr* bufs[2] = {C.buf<Fr>(Ctx::kSlotOpenA, 32 * std::max<uint64_t>(n / 2, 1)),
                   C.buf<Fr>(Ctx::kSlotOpenB, 32 * std::max<uint64_t>(n / 4, 1))};
    std::vector<MsmInst> insts(L - first);
    const Fr* rin = z;
    uint64_t qoff = 0;
    // folds: groups of up to 3 levels per launch while the tables are large, then the last levels
    // (<= 512 pairs) in one single-block launch; the fold-only level 0 (proof0 given) writes no quotient
    std::vector<uint64_t> lvl_qoff(L, ~0ull);  // level i's quotients: q + lvl_qoff[i] (~0: not kept)
    {
        uint64_t o = 0;
        for (int i = first; i < L; ++i) lvl_qoff[i] = o, o += n >> (i + 1);
    }
    int pp = 0;  // ping-pong: the next output buffer
    for (int i = 0; i < L;) {
        const uint64_t half = n >> (i + 1);
        if (i >= first && open_tail_levels(half, L - i) == L - i) {
            std::vector<Fr> pts(L - i);
            for (int j = i; j < L; ++j) pts[j - i] = dev_fr(point[j]);
            Fr* last = bufs[pp];
            launch_open_tail(rin, q + lvl_qoff[i], half, L - i, pts.data(), last, C.stream);
            rin = last;
            break;
        }
        int nf = 1;  // levels in this launch: stop before the tail's start
        while (nf < 3 && i + nf < L && open_tail_levels(n >> (i + nf + 1), L - i - nf) != L - i - nf) ++nf;
        Fr* rout = bufs[pp];
        pp ^= 1;
        if (nf >= 2) {
            Fr pts[3];
            uint64_t qo[3];
            for (int j = 0; j < nf; ++j) pts[j] = dev_fr(point[i + j]), qo[j] = lvl_qoff[i + j];
            launch_open_fold(rin, rout, q, nf, pts, qo, n >> (i + nf), C.stream);
        } else {
            launch_open_level(rin, rout, lvl_qoff[i] != ~0ull ? q + lvl_qoff[i] : q, dev_fr(point[i]), half, C.stream);
        }
        rin = rout;
        i += nf;
    }
    for (int i = 0; i < L; ++i) {
        const uint64_t half = n >> (i + 1);
        if (i < first) continue;  // the level's proof is proof0
        MsmInst& I = insts[i - first];
        I.pts_off = P.g2_off[i];
        I.stride = (uint32_t)half;
        I.scalar_off = qoff;
        I.size = (uint32_t)half;
        I.c = (uint32_t)P.g2_c[i];
        I.W = (uint32_t)P.g2_W[i];
        qoff += half;
    }
    const int nm = L - first;  // MSMs of this batch
    const size_t ob = msm_out_bytes(true, nm);
    void* out = C.buf(Ctx::kSlotOpenOut, ob);
    uint8_t* h = C.pin_at(Ctx::kPinOpen, ob + 32, 56 << 10);
    for (int attempt = 0;; ++attempt) {
        MsmShard sh = shard_of(comm);
        sh.dense = attempt > 0;
        if (nm) {
            msm_run_g2(C.msm, insts.data(), nm, P.g2_pre.as<G2Aff>(), q, out, C.stream, sh);
            SPX_HIP(hipMemcpyAsync(h, out, ob, hipMemcpyDeviceToHost, C.stream));
        }
        if (!attempt) SPX_HIP(hipMemcpyAsync(h + ob, rin, 32, hipMemcpyDeviceToHost, C.stream));
        C.sync();
        if (!nm || !(msm_status(h, true, nm) & kMsmOverflow)) break;
        msm_ws_note_overflow(C.msm);  // compacted keys overflowed: once more with a slot per digit
        ++C.msm_reruns;
    }
    res.eval = ld_hfr(h + ob);
    std::vector<Affine<HFq2>> part = msm_results<HFq2>(comm, h, nm);
    for (int k = 0; k < nm; ++k) res.proofs[first + k] = part[k];
    return res;
}

// BASELINE config C2 (commitment stubbed): the opening under the all-identity public parameter.
// The evaluation z(point) is computed exactly as open_z computes it (the same folds, no quotients,
// no MSM); h and every level's proof are the identity.
static OpenOut open_stub(Ctx& C, const Fr* z_local, int L, const std::vector<HFr>& point, int G) {
    const int g = ilog2((uint64_t)G);
    const uint64_t nl = (1ull << L) / G;
    const int nloc = L - g;
    OpenOut res;
    res.proofs.assign(L, Affine<HFq2>{HFq2::zero(), HFq2::zero(), true});
    Fr* bufs[2] = {C.buf<Fr>(Ctx::kSlotOpenA, 32 * std::max<uint64_t>(nl / 2, 1)),
                   C.buf<Fr>(Ctx::kSlotOpenB, 32 * std::max<uint64_t>(nl / 4, 1))};
    uint8_t* h = C.pin_at(Ctx::kPinOpen, 32 * (L + 1), 56 << 10);
    const Fr* rin = z_local;
    // z(point) only (no quotients): three levels per launch while the table is large, then the tail
    // in one launch (level by level this was ~L launches per opening: C2's proofs are launch-bound)
    int nb = 0;
    for (int i = 0; i < nloc;) {
        Fr* rout = bufs[nb++ & 1];
        const uint64_t half = nl >> (i + 1);
        if (open_tail_levels(half, nloc - i) == nloc - i) {  // the remaining levels in one launch
            std::vector<Fr> pts(nloc - i);
            for (int j = i; j < nloc; ++j) pts[j - i] = dev_fr(point[j]);
            launch_open_tail(rin, nullptr, half, nloc - i, pts.data(), rout, C.stream);
            rin = rout;
            break;
        }
        const int nf = nloc - i >= 3 && (half >> 2) >= 1 ? 3 : (nloc - i >= 2 && (half >> 1) >= 1 ? 2 : 1);
        if (nf >= 2) {
            Fr pts[3];
            uint64_t qoffs[3] = {~0ull, ~0ull, ~0ull};
            for (int j = 0; j < nf; ++j) pts[j] = dev_fr(point[i + j]);
            launch_open_fold(rin, rout, nullptr, nf, pts, qoffs, nl >> (i + nf), C.stream);
        } else {
            launch_open_level(rin, rout, nullptr, dev_fr(point[i]), half, C.stream);
        }
        rin = rout;
        i += nf;
    }
    SPX_HIP(hipMemcpyAsync(h + 32 * L, rin, 32, hipMemcpyDeviceToHost, C.stream));
    C.sync();
    HFr rlast = ld_hfr(h + 32 * L);
    if (G == 1) {
        res.eval = rlast;
        return res;
    }
    std::vector<HFr> rg = allgather_fr(*C.comm, {rlast});
    for (int i = nloc; i < L; ++i) {
        std::vector<HFr> nr(rg.size() / 2);
        for (size_t b = 0; b < nr.size(); ++b) nr[b] = rg[2 * b] + point[i] * (rg[2 * b + 1] - rg[2 * b]);
        rg.swap(nr);
    }
    res.eval = rg[0];
    return res;
}
static Affine<HFq2> h_of(const PP* P) { return P ? P->h : Affine<HFq2>{HFq2::zero(), HFq2::zero(), true}; }

static void ser_open(Ser& s, const HFr& eval, const Affine<HFq2>& h, const std::vector<Affine<HFq2>>& proofs) {
    s.fr(eval);
    uint8_t b[96];
    host::g2_compress(b, h);
    s.raw(b, 96);
    s.u64(proofs.size());
    for (auto& p : proofs) {
        host::g2_compress(b, p);
        s.raw(b, 96);
    }
}

// the quadratic through (0, g0), (1, g1), (2, g2) at t
static HFr quad_at(const HFr g[3], const HFr& t) {
    static const HFr inv2 = HFr::from_u64(2).inv();
    const HFr one = HFr::one(), two = HFr::from_u64(2);
    return g[0] * ((t - one) * (t - two) * inv2) - g[1] * (t * (t - two)) + g[2] * (t * (t - one) * inv2);
}

// ====================================================================== prove
std::vector<uint8_t> prove(Ctx& C, Index& I, Witness& W, PP* P, const ProveOpts& o) {
    CtxClaim claim;
    if (!o.claimed) claim.take(C);  // before anything is queued: a refused prove touches nothing
    // A prove that throws may leave work queued on both streams that still reads W.z and writes the
    // context's slots: drain them while unwinding, so the caller may free the witness and the next
    // proof on this context starts from idle streams.
    struct UnwindDrain {
        Ctx& C;
        int pending = std::uncaught_exceptions();
        ~UnwindDrain() {
            if (std::uncaught_exceptions() <= pending) return;
            (void)hipStreamSynchronize(C.stream);
            if (C.side) (void)hipStreamSynchronize(C.side);
            msm_ws_staging_reset(C.msm);
            if (C.msm_side) msm_ws_staging_reset(C.msm_side);
        }
    } drain{C};
    Timer tall;
    C.timings.clear();
    int phase = 0;
    uint64_t cpu0 = thread_cpu_ns();
    auto mark = [&](const char* name, Timer& t) {
        const double us = t.us();
        C.timings.emplace_back(name, us);
        t = Timer();
        const uint64_t c1 = thread_cpu_ns();
        if (phase < kHostPhases) {
            g_phase_cpu[phase] += c1 - cpu0;
            g_phase_wall[phase] += (uint64_t)(us * 1e3);
            g_phase_cnt[phase] += 1;
        }
        ++phase;
        cpu0 = c1;
    };
    Timer tp;
    const int L = I.log_n;
    const uint64_t n = I.n;
    Comm& comm = *C.comm;
    const int G = comm.size(), rank = comm.rank();
    if (G != I.G || rank != I.rank) invalid("index was built for a different communicator");
    const int g = ilog2((uint64_t)G);
    const uint64_t nl = n / G, lo = (uint64_t)rank * nl;
    const uint64_t nvv = W.v.size() / 32;
    if (!is_pow2(nvv)) invalid("public input should be power of two");
    if (W.n != n) invalid("|v| + |w| != number of variables");  // prover.rs:117-119
    if (!o.stub && !P) invalid("null public parameter");
    C.side_sync();  // a proof that threw may have left its level-0 MSM running on the second stream
    if (P && P->nv != L) invalid("public parameter nv != log_n");
    const int log_v = ilog2(nvv);
    const Fr* z = W.z.as<Fr>();
    const Fr* zl = z + lo;
    // scratch layout (Fr units)
    const uint64_t n2 = std::max<uint64_t>(nl / 2, 1), n4 = std::max<uint64_t>(nl / 4, 1);
    const uint64_t need = 3 * nl        // Az Bz Cz
                          + 3 * n2 + 3 * n4  // fold ping-pong
                          + n2 + n4 + std::max<uint64_t>(nl / 8, 1)  // E tables
                          + nl + n2 + n4     // Mrx + fold
                          + n2 + n4          // z fold
                          + std::max<uint64_t>(kRoundPartials, std::max(I.rows.nchunks, I.cols.longc.nchunks))
                          + 8192 * 2 + kEqScratch + 64 + 8 * L;  // partials, eq scratch, challenges
    C.scratch.ensure(32 * need);
    Fr* base = C.scratch.as<Fr>();
    uint64_t cur_off = 0;
    auto take = [&](uint64_t k) {
        Fr* p = base + cur_off;
        cur_off += k;
        return p;
    };
    Fr *Az = take(nl), *Bz = take(nl), *Cz = take(nl);
    Fr* F1[3] = {take(n2), take(n2), take(n2)};
    Fr* F2[3] = {take(n4), take(n4), take(n4)};
    Fr *E1 = take(n2), *Ea = take(n4), *Eb = take(std::max<uint64_t>(nl / 8, 1));
    Fr *M0 = take(nl), *M1 = take(n2), *M2 = take(n4);
    Fr *Z1 = take(n2), *Z2 = take(n4);
    Fr* partial = take(std::max<uint64_t>(kRoundPartials, std::max(I.rows.nchunks, I.cols.longc.nchunks)));
    Fr *eqlo = take(8192), *eqhi = take(8192), *eqf = take(kEqScratch);
    Fr* chdev = take(8 * L);  // tau, r_x, (r_a, r_b, r_c), ...
    uint8_t* hp = C.pin_at(Ctx::kPinHp, 1 << 16, 64 << 10);

    // ---- SpMV Az, Bz, Cz (challenge-independent: queued first, overlaps the commit's host work)
    {
        kp_begin(KP_SPMV, C.stream);
        if (I.rows_sliced.on)
            launch_spmv_sliced(I.rows_sliced.view(), z, Az, Bz, Cz, I.rows_sliced.entries, C.stream);
        else
            launch_sparse3(0, I.rows.view(), z, Az, Bz, Cz, nullptr, nl, I.rows.chunks.as<LongChunk>(), I.rows.nchunks,
                           I.rows.lrows.as<LongRow>(), I.rows.nlrows, partial, C.stream);
        kp_end(I.rows_bytes, C.stream);
    }
    // The shared level-0 opening proof is launched right behind the commitment, before any challenge,
    // when the host has the matrix absorption to do meanwhile. With the index-cached transcript there
    // is nothing to hide it behind: a sharded proof then runs it on the context's second stream, beside
    // the commitment and the first opening (reused by the second opening); an unsharded one puts it in
    // the first opening's batch (below). (Both forms give every rank the same
    // batches, so the exchanges of a proof-sharded prove line up.)
    // SPX_LVL0=batch (A/B; must be the same on every rank of a proof-sharded prove): level 0 inside the
    // first opening's MSM batch instead, one MSM pipeline (sort, weighting tree) less per proof
    static const bool lvl0_batch_env = [] {
        const char* e = getenv("SPX_LVL0");
        return e && std::string(e) == "batch";
    }();
    // Unsharded index-cached proofs default to the batch form: with no absorption to hide level 0
    // behind, one MSM pipeline less measured +2% index-cached at N = 1 (profiles/r06/r06zq_ab_lvl0_n1.jsonl)
    const bool lvl0_batch =
        C.lvl0_mode >= 0 ? C.lvl0_mode == 1 : (lvl0_batch_env || (G == 1 && o.cached && I.has_cache && !o.coins));
    // SPX_CHECK_DERIVED=1 (tests): from round 2 on, a sumcheck round's value at 1 is derived from the
    // previous claim on the host (P(0) + P(1) = claim); with this set the device computes it too and the
    // prove fails with SPX_SUMCHECK if they differ (the identity pinned round by round, every rank count)
    const bool check_derived = [] {
        const char* e = getenv("SPX_CHECK_DERIVED");
        return e && e[0] == '1';
    }();
    if (G > 1 && !C.knobs_agreed) {
        // the level-0 mode decides the order and sizes of a proof's exchanges: every rank of the
        // communicator must read the same SPX_LVL0 (one exchange on a context's first sharded proof)
        const uint32_t mine = lvl0_batch ? 1u : 0u;
        std::vector<uint32_t> all(G);
        comm.allgather(&mine, all.data(), sizeof mine);
        for (int r = 0; r < G; ++r)
            if (all[r] != mine) invalid("SPX_LVL0 / level-0 mode differs between the ranks of this communicator");
        C.knobs_agreed = true;
    }
    const bool share0 = !o.stub;
    const bool early0 = share0 && !lvl0_batch && !(o.cached && I.has_cache);
    const bool side0 = share0 && !lvl0_batch && !early0;
    const MsmShard sh = shard_of(comm);
    if (side0) {  // z is in place: the second stream may start
        C.ensure_side();
        SPX_HIP(hipEventRecord(C.side_ev, C.stream));
    }
    // ---- round 1: commitment (prover.rs:123-141); the MSM runs while the host absorbs A, B, C
    if (!o.stub) commit_launch(C, *P, z, n, sh);
    if (early0) lvl0_launch(C, *P, z, L, sh);
    if (side0) lvl0_launch(C, *P, z, L, sh, true);
    Transcript T(o.mode == 1, o.seed, o.coins);
    const uint64_t ctr = C.prove_seq++;
    const uint64_t seq = o.seq >= 0 ? (uint64_t)o.seq : ctr;
    const Blake2s* absorbed = o.await_absorbed ? o.await_absorbed() : o.absorbed;
    if (o.coins) {
        // interactive: the caller is the verifier; nothing is absorbed
    } else if (o.cached && I.has_cache)
        T.set_state(I.cache);
    else if (G == 1) {
        T.set_state(absorbed ? *absorbed : absorb_matrices(I));
    } else {
        // the (sequential, ~150 MB at 2^20) absorption of A, B, C is done once per proof, by one rank
        // in turn; the others take its Blake2s state from the allgather (bit-identical transcript)
        static_assert(std::is_trivially_copyable<Blake2s>::value, "Blake2s state is shipped as bytes");
        const int owner = (int)(seq % (uint64_t)G);
        Blake2s h;
        if (rank == owner) h = absorbed ? *absorbed : absorb_matrices(I);
        std::vector<uint8_t> all(sizeof(Blake2s) * G);
        comm.allgather(&h, all.data(), sizeof(Blake2s));
        memcpy(&h, all.data() + sizeof(Blake2s) * owner, sizeof(Blake2s));
        T.set_state(h);
    }
    {
        Ser s;
        s.u64(nvv);
        s.raw(W.v.data(), W.v.size());
        T.absorb(s.b.data(), s.b.size());
    }
    mark("transcript_matrices", tp);
    Affine<HFq> com = o.stub ? Affine<HFq>{HFq::zero(), HFq::zero(), true} : commit_finish(C, *P, z, n, comm);
    Affine<HFq2> proof0{};
    if (early0) proof0 = lvl0_finish(C, *P, z, L, comm);
    Ser proof;
    {
        size_t m0 = proof.b.size();
        proof.u64((uint64_t)L);
        uint8_t b[48];
        host::g1_compress(b, com);
        proof.raw(b, 48);
        T.feed(proof.b.data() + m0, proof.b.size() - m0);
    }
    mark("commit", tp);
    // ---- round 2: open at (r_v, 0...0) (prover.rs:143-160)
    std::vector<HFr> pt1(L, HFr::zero());
    for (int i = 0; i < log_v; ++i) pt1[i] = T.rand_fr();
    {
        OpenOut op = o.stub ? open_stub(C, zl, L, pt1, G)
                            : open_z(C, *P, z, L, pt1, comm, (early0 || side0) ? &proof0 : nullptr);
        if (side0) op.proofs[0] = proof0 = lvl0_finish(C, *P, z, L, comm, true);
        if (share0 && !early0 && !side0) proof0 = op.proofs[0];
        size_t m0 = proof.b.size();
        ser_open(proof, op.eval, h_of(P), op.proofs);
        T.feed(proof.b.data() + m0, proof.b.size() - m0);
    }
    mark("open_rv", tp);
    // ---- round 3: tau, eq, sumcheck #1 setup (prover.rs:163-196)
    std::vector<HFr> tau(L);
    for (int i = 0; i < L; ++i) tau[i] = T.rand_fr();
    memcpy(hp, tau.data(), 32 * L);
    SPX_HIP(hipMemcpyAsync(chdev, hp, 32 * L, hipMemcpyHostToDevice, C.stream));
    // E_1[b] = eq(tau_1..tau_{L-1}, b) on this rank's block of b
    if (L >= 2)
        launch_eq_table(chdev + 1, L - 1, (uint64_t)rank * (nl / 2), nl / 2, E1, eqlo, eqhi, C.stream);
    else {
        const HFr one = HFr::one();
        memcpy(hp + 4096, &one, 32);
        SPX_HIP(hipMemcpyAsync(E1, hp + 4096, 32, hipMemcpyHostToDevice, C.stream));
    }
    {
        size_t m0 = proof.b.size();
        proof.u64((uint64_t)(L + 2));  // IndexInfo.max_multiplicands (reconstructed field order)
        proof.u64((uint64_t)L);        // IndexInfo.num_variables
        T.feed(proof.b.data() + m0, proof.b.size() - m0);
    }
    // ---- sumcheck #1 (lib.rs:86-103)
    proof.u64((uint64_t)L);
    std::vector<HFr> r_x;
    HFr Cc = HFr::one(), claim1 = HFr::zero();
    Fr* res_dev = C.pin_dev<Fr>(hp);  // the rounds' sums land in pinned host memory (hp)
    Tables3 cur{{Az, Bz, Cz}};
    const Fr* Ecur = E1;
    Fr* Ebuf[2] = {Ea, Eb};
    // The last ht1 rounds of each sumcheck run on the host, as in prove_group: each rank binds its local
    // tables (<= 64 entries) and, sharded, the ranks' tables are gathered in rank order (the g high
    // variables) before the last g + ht1 rounds. Unsharded: one proof at a time 22.5 vs 22.6 ms
    // index-cached, throughput equal (profiles/r05/r05zt_ab_hosttail1.jsonl); a rank of an 8-rank proof
    // +2.3% (r05zu_ab_shardtail_G8.jsonl: 10 fewer launches and exchanges per proof). Fixed, so every
    // rank of a communicator agrees.
    const int ht1 = std::max(0, std::min(kGroupHostTail, L - g - 1));
    const uint32_t tn = 2u << ht1;  // entries per table after the device rounds
    for (int i = 1; i <= L - g - ht1; ++i) {
        const uint64_t half = nl >> i;
        const bool fold = i >= 2;
        Tables3 out{{nullptr, nullptr, nullptr}};
        Fr* Eout = nullptr;
        if (fold) {
            Fr** fb = (i % 2 == 0) ? F1 : F2;
            out = Tables3{{fb[0], fb[1], fb[2]}};
            if (i < L - g) Eout = Ebuf[i & 1];
        }
        // from round 2 on, P_i(0) + P_i(1) = P_{i-1}(r_{i-1}) (the claim) is an identity of the folded
        // tables, so G(1) follows from G(0): Cc (1 - tau) G(0) + Cc tau G(1) = claim; the kernel skips it
        // (2 of its 12 Fr products per pair). Exact field arithmetic: the same message bytes.
        const HFr ct = Cc * tau[i - 1];
        const bool derive1 = fold && !ct.is_zero();
        launch_sc1_round(fold, cur, out, Ecur, Eout, fold ? dev_fr(r_x[i - 2]) : Fr{}, half, partial, C.ticket, res_dev,
                         !derive1 || check_derived, C.stream);
        C.sync();
        HFr gs[3] = {ld_hfr(hp), ld_hfr(hp + 32), ld_hfr(hp + 64)};
        if (G > 1) {
            std::vector<HFr> all = allgather_fr(comm, {gs[0], gs[1], gs[2]});
            gs[0] = gs[1] = gs[2] = HFr::zero();
            for (int r = 0; r < G; ++r)
                for (int k = 0; k < 3; ++k) gs[k] += all[3 * r + k];
        }
        if (derive1) {
            const HFr d1 = (claim1 - (Cc - ct) * gs[0]) * ct.inv();
            if (check_derived && !(d1 == gs[1]))
                throw SpxError(kSumcheck, "sumcheck 1 round " + std::to_string(i) + ": derived G(1) differs from the device's");
            gs[1] = d1;
        }
        std::vector<HFr> msg = sc1_message(Cc, tau[i - 1], gs, L);
        size_t m0 = proof.b.size();
        proof.u64(msg.size());
        for (auto& e : msg) proof.fr(e);
        T.feed(proof.b.data() + m0, proof.b.size() - m0);
        HFr ch = T.rand_fr();
        r_x.push_back(ch);
        const HFr eqc = eq1(tau[i - 1], ch);
        claim1 = Cc * eqc * quad_at(gs, ch);  // P_i(r_i)
        Cc = Cc * eqc;
        if (fold) {
            cur = out;
            if (Eout) Ecur = Eout;
        }
    }
    // local tables now hold tn entries each (2 when sharded; folded up to r_{L-g-ht1-1}); bind r_{L-g-ht1}
    // on the host
    HFr va, vb, vc;
    {
        for (int m = 0; m < 3; ++m)
            SPX_HIP(hipMemcpyAsync(hp + 32 * tn * m, cur.t[m], 32 * tn, hipMemcpyDeviceToHost, C.stream));
        C.sync();
        const HFr r = r_x.back();
        // this rank's tables bound at r: 3 x tn / 2 entries; gathered in rank order (rank = the high
        // variables), the remaining g + ht1 variables' tables
        const uint32_t hn = tn / 2;
        std::vector<HFr> mine(3 * hn);
        for (int m = 0; m < 3; ++m)
            for (uint32_t b = 0; b < hn; ++b) {
                const HFr a0 = ld_hfr(hp + 32 * (tn * m + 2 * b)), a1 = ld_hfr(hp + 32 * (tn * m + 2 * b + 1));
                mine[m * hn + b] = a0 + r * (a1 - a0);
            }
        std::vector<HFr> tabs[3];
        const std::vector<HFr> all = G == 1 ? mine : allgather_fr(comm, mine);
        for (int m = 0; m < 3; ++m)
            for (int r2 = 0; r2 < G; ++r2)
                for (uint32_t b = 0; b < hn; ++b) tabs[m].push_back(all[(size_t)3 * hn * r2 + m * hn + b]);
        // last g (+ ht1) rounds on the gathered tables (size 2^g, or 2^ht1 unsharded), same message formula
        for (int i = L - g - ht1 + 1; i <= L; ++i) {
            const size_t half = tabs[0].size() / 2;
            const int c = i - 1;
            HFr gs[3] = {HFr::zero(), HFr::zero(), HFr::zero()};
            for (size_t b = 0; b < half; ++b) {
                HFr e = HFr::one();  // eq(tau_{c+1..L-1}, b)
                for (int j = c + 1; j < L; ++j) e *= ((b >> (j - c - 1)) & 1) ? tau[j] : HFr::one() - tau[j];
                HFr x0[3], x1[3], y[3];
                for (int m = 0; m < 3; ++m) {
                    x0[m] = tabs[m][2 * b];
                    x1[m] = tabs[m][2 * b + 1];
                    y[m] = x1[m] + x1[m] - x0[m];
                }
                gs[0] += (x0[0] * x0[1] - x0[2]) * e;
                gs[1] += (x1[0] * x1[1] - x1[2]) * e;
                gs[2] += (y[0] * y[1] - y[2]) * e;
            }
            std::vector<HFr> msg = sc1_message(Cc, tau[c], gs, L);
            size_t m0 = proof.b.size();
            proof.u64(msg.size());
            for (auto& e : msg) proof.fr(e);
            T.feed(proof.b.data() + m0, proof.b.size() - m0);
            HFr ch = T.rand_fr();
            r_x.push_back(ch);
            Cc = Cc * eq1(tau[c], ch);
            for (int m = 0; m < 3; ++m) {
                std::vector<HFr> nt(half);
                for (size_t b = 0; b < half; ++b) nt[b] = tabs[m][2 * b] + ch * (tabs[m][2 * b + 1] - tabs[m][2 * b]);
                tabs[m].swap(nt);
            }
        }
        va = tabs[0][0];
        vb = tabs[1][0];
        vc = tabs[2][0];
    }
    mark("sumcheck1", tp);
    // ---- round 4 (prover.rs:210-228)
    {
        size_t m0 = proof.b.size();
        proof.fr(va);
        proof.fr(vb);
        proof.fr(vc);
        T.feed(proof.b.data() + m0, proof.b.size() - m0);
    }
    HFr rabc[3] = {T.rand_fr(), T.rand_fr(), T.rand_fr()};
    // ---- round 5: M_rx = sum_m r_m M(r_x, .) on this rank's columns (prover.rs:230-255)
    Fr* rxdev = chdev + 2 * L;  // r_x (L) then r_abc (3)
    memcpy(hp, r_x.data(), 32 * L);
    memcpy(hp + 32 * L, rabc, 96);
    SPX_HIP(hipMemcpyAsync(rxdev, hp, 32 * (L + 3), hipMemcpyHostToDevice, C.stream));
    {
        kp_begin(KP_MTV, C.stream);
        I.cols.launch(rxdev, L, rxdev + L, M0, eqf, partial, C.stream);
        kp_end(I.cols_bytes, C.stream);
    }
    {
        size_t m0 = proof.b.size();
        proof.u64(2);
        proof.u64((uint64_t)L);
        T.feed(proof.b.data() + m0, proof.b.size() - m0);
    }
    mark("eval_on_x", tp);
    // ---- sumcheck #2 (lib.rs:114-131)
    proof.u64((uint64_t)L);
    std::vector<HFr> r_y;
    HFr claim2 = HFr::zero();
    const Fr* Mc = M0;
    const Fr* Zc = zl;
    Fr* Mb[2] = {M1, M2};
    Fr* Zb[2] = {Z1, Z2};
    for (int i = 1; i <= L - g - ht1; ++i) {
        const uint64_t half = nl >> i;
        const bool fold = i >= 2;
        Fr* Mo = fold ? Mb[i & 1] : nullptr;
        Fr* Zo = fold ? Zb[i & 1] : nullptr;
        // from round 2 on, P(1) = claim - P(0) (the folded tables' identity): the kernel skips it
        launch_sc2_round(fold, Mc, Zc, Mo, Zo, fold ? dev_fr(r_y[i - 2]) : Fr{}, half, partial, C.ticket, res_dev,
                         !fold || check_derived, C.stream);
        C.sync();
        HFr ps[3] = {ld_hfr(hp), ld_hfr(hp + 32), ld_hfr(hp + 64)};
        if (G > 1) {
            std::vector<HFr> all = allgather_fr(comm, {ps[0], ps[1], ps[2]});
            ps[0] = ps[1] = ps[2] = HFr::zero();
            for (int r = 0; r < G; ++r)
                for (int k = 0; k < 3; ++k) ps[k] += all[3 * r + k];
        }
        if (fold) {
            const HFr d1 = claim2 - ps[0];
            if (check_derived && !(d1 == ps[1]))
                throw SpxError(kSumcheck, "sumcheck 2 round " + std::to_string(i) + ": derived P(1) differs from the device's");
            ps[1] = d1;
        }
        size_t m0 = proof.b.size();
        proof.u64(3);
        for (int k = 0; k < 3; ++k) proof.fr(ps[k]);
        T.feed(proof.b.data() + m0, proof.b.size() - m0);
        HFr ch = T.rand_fr();
        r_y.push_back(ch);
        claim2 = quad_at(ps, ch);  // P_i(r_i)
        if (fold) {
            Mc = Mo;
            Zc = Zo;
        }
    }
    if (g + ht1 > 0) {
        SPX_HIP(hipMemcpyAsync(hp, Mc, 32 * tn, hipMemcpyDeviceToHost, C.stream));
        SPX_HIP(hipMemcpyAsync(hp + 32 * tn, Zc, 32 * tn, hipMemcpyDeviceToHost, C.stream));
        C.sync();
        const HFr r = r_y.back();
        const uint32_t hn = tn / 2;
        std::vector<HFr> mine(2 * hn);
        for (uint32_t b = 0; b < hn; ++b) {
            const HFr m0v = ld_hfr(hp + 32 * (2 * b)), m1v = ld_hfr(hp + 32 * (2 * b + 1));
            const HFr z0 = ld_hfr(hp + 32 * (tn + 2 * b)), z1 = ld_hfr(hp + 32 * (tn + 2 * b + 1));
            mine[b] = m0v + r * (m1v - m0v);
            mine[hn + b] = z0 + r * (z1 - z0);
        }
        const std::vector<HFr> all = G == 1 ? mine : allgather_fr(comm, mine);
        std::vector<HFr> Mt, Zt;
        for (int r2 = 0; r2 < G; ++r2)
            for (uint32_t b = 0; b < hn; ++b) {
                Mt.push_back(all[(size_t)2 * hn * r2 + b]);
                Zt.push_back(all[(size_t)2 * hn * r2 + hn + b]);
            }
        for (int i = L - g - ht1 + 1; i <= L; ++i) {
            const size_t half = Mt.size() / 2;
            HFr ps[3] = {HFr::zero(), HFr::zero(), HFr::zero()};
            for (size_t b = 0; b < half; ++b) {
                HFr m0v = Mt[2 * b], m1v = Mt[2 * b + 1], z0 = Zt[2 * b], z1 = Zt[2 * b + 1];
                ps[0] += m0v * z0;
                ps[1] += m1v * z1;
                ps[2] += (m1v + m1v - m0v) * (z1 + z1 - z0);
            }
            size_t m0 = proof.b.size();
            proof.u64(3);
            for (int k = 0; k < 3; ++k) proof.fr(ps[k]);
            T.feed(proof.b.data() + m0, proof.b.size() - m0);
            HFr ch = T.rand_fr();
            r_y.push_back(ch);
            std::vector<HFr> nm(half), nz(half);
            for (size_t b = 0; b < half; ++b) {
                nm[b] = Mt[2 * b] + ch * (Mt[2 * b + 1] - Mt[2 * b]);
                nz[b] = Zt[2 * b] + ch * (Zt[2 * b + 1] - Zt[2 * b]);
            }
            Mt.swap(nm);
            Zt.swap(nz);
        }
    }
    mark("sumcheck2", tp);
    // ---- round 6: open at r_y (prover.rs:268-281)
    {
        OpenOut op = o.stub ? open_stub(C, zl, L, r_y, G) : open_z(C, *P, z, L, r_y, comm, share0 ? &proof0 : nullptr);
        ser_open(proof, op.eval, h_of(P), op.proofs);
    }
    mark("open_ry", tp);
    C.timings.emplace_back("total", tall.us());
    return proof.b;
}

// ====================================================================== lockstep groups
// prove() for k stubbed-commitment proofs of one index on one rank (BASELINE C2), interleaved step by
// step. A C2 proof is ~55 small launches and ~40 host waits: with 32 proofs in flight on the context
// streams' 4 hardware queues the GPU ran ~1 kernel at a time and was idle 65% of the time (trace
// profiles/r05/r05zg_c2_busy.txt), each proof waiting its turn in a queue. Here the k proofs' sumcheck
// rounds are one launch each (launch_sc1_round_group: blockIdx.y = proof) with one wait, and the other
// steps queue the k proofs' launches back to back before one wait. Every value is computed by the same
// kernels and host formulas as prove(), so each proof's bytes are its own prove()'s.
std::vector<std::vector<uint8_t>> prove_group(Ctx& C, Index& I, Witness* const* Ws, int k, const ProveOpts* os) {
    static_assert(kGroupMax <= 16, "one sumcheck ticket per proof of a group: Ctx::ticket holds 16 counters");
    if (k < 1 || k > kGroupMax) invalid("lockstep group size must be 1.." + std::to_string(kGroupMax));
    CtxClaim claim;
    claim.take(C);
    struct UnwindDrain {
        Ctx& C;
        int pending = std::uncaught_exceptions();
        ~UnwindDrain() {
            if (std::uncaught_exceptions() <= pending) return;
            (void)hipStreamSynchronize(C.stream);
        }
    } drain{C};
    // a group records no per-phase marks (its phases interleave k proofs): spx_last_timings reports
    // its total alone, and the host-phase counters (spx_host_phase_stats) count prove() calls only
    C.timings.clear();
    Timer tgroup;
    Comm& comm = *C.comm;
    if (comm.size() != 1 || I.G != 1) invalid("lockstep groups need an unsharded context and index");
    const int L = I.log_n;
    const uint64_t n = I.n, nl = n;
    for (int j = 0; j < k; ++j) {
        if (!Ws[j]) invalid("null witness");
        if (!os[j].stub || os[j].coins || os[j].claimed) invalid("lockstep groups prove stubbed-commitment proofs only");
        if (!is_pow2(Ws[j]->v.size() / 32)) invalid("public input should be power of two");
        if (Ws[j]->n != n) invalid("|v| + |w| != number of variables");  // prover.rs:117-119
    }
    const bool check_derived = [] {
        const char* e = getenv("SPX_CHECK_DERIVED");
        return e && e[0] == '1';
    }();
    // per-proof scratch, prove()'s layout at G = 1
    const uint64_t n2 = std::max<uint64_t>(nl / 2, 1), n4 = std::max<uint64_t>(nl / 4, 1);
    const uint64_t npart = std::max<uint64_t>(kRoundPartials, std::max(I.rows.nchunks, I.cols.longc.nchunks));
    // (plus the opening folds' two buffers per proof: the group's fold chains run side by side)
    const uint64_t need = 3 * nl + 3 * n2 + 3 * n4 + n2 + n4 + std::max<uint64_t>(nl / 8, 1) + nl + n2 + n4 + n2 + n4 +
                          npart + 8192 * 2 + kEqScratch + 64 + n2 + n4;
    // the group's challenges: proof j's tau, r_x, r_abc at chg + 8 L j (one host-to-device copy each time)
    C.scratch.ensure(32 * (need + 8 * (uint64_t)L) * (uint64_t)k);
    Fr* chg = C.scratch.as<Fr>() + need * k;
    static_assert(kGroupMax * 8192 <= (128 << 10), "per-proof pinned regions");
    if (32 * (L + 3) > 4096 || 32 * 8 * L * kGroupMax > (128 << 10)) invalid("log_n too large for a lockstep group");
    uint8_t* hp0 = C.pin_at(Ctx::kPinHp, kGroupMax * 8192, 128 << 10);
    uint8_t* ho0 = C.pin_at(Ctx::kPinOpen, kGroupMax * 2048, 56 << 10);
    uint8_t* stage = C.pin_at(Ctx::kPinStage, (size_t)32 * 8 * L * k, 128 << 10);
    struct P {
        Fr *Az, *Bz, *Cz, *F1[3], *F2[3], *E1, *Ea, *Eb, *M0, *M1, *M2, *Z1, *Z2, *partial, *eqlo, *eqhi, *eqf, *chdev;
        Fr *oA, *oB;
        uint8_t *hp, *ho;
        Fr* res_dev;
        const Fr* z;
        int log_v;
        Transcript T;
        Ser proof;
        std::vector<HFr> tau, r_x, r_y;
        HFr Cc, claim1, claim2;
        Tables3 cur;
        const Fr* Ecur;
        const Fr *Mc, *Zc;
    };
    std::vector<P> ps;
    ps.reserve(k);
    for (int j = 0; j < k; ++j) {
        Fr* base = C.scratch.as<Fr>() + need * j;
        uint64_t off = 0;
        auto take = [&](uint64_t c) {
            Fr* q = base + off;
            off += c;
            return q;
        };
        P p;
        p.Az = take(nl), p.Bz = take(nl), p.Cz = take(nl);
        for (int m = 0; m < 3; ++m) p.F1[m] = take(n2);
        for (int m = 0; m < 3; ++m) p.F2[m] = take(n4);
        p.E1 = take(n2), p.Ea = take(n4), p.Eb = take(std::max<uint64_t>(nl / 8, 1));
        p.M0 = take(nl), p.M1 = take(n2), p.M2 = take(n4);
        p.Z1 = take(n2), p.Z2 = take(n4);
        p.partial = take(npart);
        p.eqlo = take(8192), p.eqhi = take(8192), p.eqf = take(kEqScratch);
        p.oA = take(n2), p.oB = take(n4);
        p.chdev = chg + (uint64_t)8 * L * j;
        p.hp = hp0 + 8192 * j;
        p.ho = ho0 + 2048 * j;
        p.res_dev = C.pin_dev<Fr>(p.hp);
        p.z = Ws[j]->z.as<Fr>();
        p.log_v = ilog2(Ws[j]->v.size() / 32);
        p.T = Transcript(os[j].mode == 1, os[j].seed, nullptr);
        ps.push_back(std::move(p));
    }
    // per-proof pointer arrays for the group launchers
    auto each = [&](auto f) {
        using T = decltype(f(ps[0]));
        std::vector<T> v;
        for (auto& p : ps) v.push_back(f(p));
        return v;
    };
    // ---- SpMV Az, Bz, Cz of every proof (challenge-independent)
    if (I.rows_sliced.on) {
        kp_begin(KP_SPMV, C.stream);
        const auto zs = each([](P& p) -> const Fr* { return p.z; });
        const auto outs = each([](P& p) { return Tables3{{p.Az, p.Bz, p.Cz}}; });
        launch_spmv_sliced_group(k, I.rows_sliced.view(), zs.data(), outs.data(), I.rows_sliced.entries, C.stream);
        // one index stream for the group (k_spmv_sliced_group), z and the outputs per proof
        kp_end(I.rows_index_bytes + (I.rows_bytes - I.rows_index_bytes) * k, C.stream);
    } else {
        for (auto& p : ps)
            launch_sparse3(0, I.rows.view(), p.z, p.Az, p.Bz, p.Cz, nullptr, nl, I.rows.chunks.as<LongChunk>(),
                           I.rows.nchunks, I.rows.lrows.as<LongRow>(), I.rows.nlrows, p.partial, C.stream);
    }
    // ---- transcripts: A, B, C (cached or absorbed), v; round 1 with the stubbed commitment
    for (int j = 0; j < k; ++j) {
        P& p = ps[j];
        const ProveOpts& o = os[j];
        C.prove_seq++;
        if (o.cached && I.has_cache)
            p.T.set_state(I.cache);
        else {
            const Blake2s* absorbed = o.await_absorbed ? o.await_absorbed() : o.absorbed;
            p.T.set_state(absorbed ? *absorbed : absorb_matrices(I));
        }
        Ser s;
        s.u64(Ws[j]->v.size() / 32);
        s.raw(Ws[j]->v.data(), Ws[j]->v.size());
        p.T.absorb(s.b.data(), s.b.size());
        const Affine<HFq> com{HFq::zero(), HFq::zero(), true};
        p.proof.u64((uint64_t)L);
        uint8_t b[48];
        host::g1_compress(b, com);
        p.proof.raw(b, 48);
        p.T.feed(p.proof.b.data(), p.proof.b.size());
    }
    // stubbed openings: every proof's z(point) by open_stub's fold chain, one launch per step for the
    // group, the values written straight into pinned memory; one wait
    auto open_all = [&](const std::vector<std::vector<HFr>>& pts) {
        std::vector<Fr> flat((size_t)k * L);
        for (int j = 0; j < k; ++j)
            for (int i = 0; i < L; ++i) flat[(size_t)j * L + i] = dev_fr(pts[j][i]);
        const auto zs = each([](P& p) -> const Fr* { return p.z; });
        const auto as = each([](P& p) { return p.oA; });
        const auto bs = each([](P& p) { return p.oB; });
        const auto last = each([&](P& p) { return C.pin_dev<Fr>(p.ho); });
        launch_open_eval_group(k, zs.data(), as.data(), bs.data(), flat.data(), L, nl, last.data(), C.stream);
        C.sync();
        const std::vector<Affine<HFq2>> none(L, Affine<HFq2>{HFq2::zero(), HFq2::zero(), true});
        for (int j = 0; j < k; ++j) {
            P& p = ps[j];
            const size_t m0 = p.proof.b.size();
            ser_open(p.proof, ld_hfr(p.ho), h_of(nullptr), none);
            p.T.feed(p.proof.b.data() + m0, p.proof.b.size() - m0);
        }
    };
    {  // round 2: open at (r_v, 0...0)
        std::vector<std::vector<HFr>> pts(k);
        for (int j = 0; j < k; ++j) {
            pts[j].assign(L, HFr::zero());
            for (int i = 0; i < ps[j].log_v; ++i) pts[j][i] = ps[j].T.rand_fr();
        }
        open_all(pts);
    }
    // ---- round 3: tau (one copy for the group), eq tables (one launch pair); sumcheck 1 setup
    for (int j = 0; j < k; ++j) {
        P& p = ps[j];
        p.tau.resize(L);
        for (int i = 0; i < L; ++i) p.tau[i] = p.T.rand_fr();
        memcpy(stage + (size_t)32 * 8 * L * j, p.tau.data(), 32 * L);
    }
    SPX_HIP(hipMemcpyAsync(chg, stage, (size_t)32 * 8 * L * k, hipMemcpyHostToDevice, C.stream));
    if (L >= 2) {
        const auto rs = each([](P& p) -> const Fr* { return p.chdev + 1; });
        const auto outs = each([](P& p) { return p.E1; });
        const auto lo = each([](P& p) { return p.eqlo; });
        const auto hi = each([](P& p) { return p.eqhi; });
        launch_eq_table_group(k, rs.data(), L - 1, 0, nl / 2, outs.data(), lo.data(), hi.data(), C.stream);
    }
    for (auto& p : ps) {
        if (L < 2) {
            const HFr one = HFr::one();
            memcpy(p.hp + 4096, &one, 32);
            SPX_HIP(hipMemcpyAsync(p.E1, p.hp + 4096, 32, hipMemcpyHostToDevice, C.stream));
        }
        const size_t m0 = p.proof.b.size();
        p.proof.u64((uint64_t)(L + 2));
        p.proof.u64((uint64_t)L);
        p.T.feed(p.proof.b.data() + m0, p.proof.b.size() - m0);
        p.proof.u64((uint64_t)L);
        p.Cc = HFr::one();
        p.claim1 = HFr::zero();
        p.cur = Tables3{{p.Az, p.Bz, p.Cz}};
        p.Ecur = p.E1;
    }
    // The last ht rounds of each sumcheck run on the host (the tables are then <= 2^(ht+1) entries: a few
    // microseconds of host arithmetic per round, against a ~30 us launch that holds one of the 4 hardware
    // queues), with prove()'s formulas for the gathered tables of a sharded proof: the same field values.
    // (2,216 - 2,221 M index-cached against 2,138 - 2,155 M with every round on the device, 3 or 4 rounds
    // between: profiles/r05/r05zs_hosttail.jsonl)
    static_assert(kGroupHostTail >= 0 && kGroupHostTail <= 5, "3 x 2^(ht+1) Fr fit each proof's 8 KiB pinned region");
    const int ht = std::min(kGroupHostTail, L - 1);
    // ---- sumcheck 1: one launch and one wait per round for the group
    std::vector<Sc1Job> j1(k);
    std::vector<char> derive(k);
    for (int i = 1; i <= L - ht; ++i) {
        const uint64_t half = nl >> i;
        const bool fold = i >= 2;
        bool need1 = check_derived;
        for (int j = 0; j < k; ++j) {
            P& p = ps[j];
            Sc1Job& jb = j1[j];
            jb.in = p.cur;
            jb.out = Tables3{{nullptr, nullptr, nullptr}};
            jb.Ein = p.Ecur;
            jb.Eout = nullptr;
            if (fold) {
                Fr** fb = (i % 2 == 0) ? p.F1 : p.F2;
                jb.out = Tables3{{fb[0], fb[1], fb[2]}};
                if (i < L) jb.Eout = (i & 1) ? p.Eb : p.Ea;
            }
            jb.r = fold ? dev_fr(p.r_x[i - 2]) : Fr{};
            jb.partial = p.partial;
            jb.ticket = C.ticket + j;
            jb.result3 = p.res_dev;
            const HFr ct = p.Cc * p.tau[i - 1];
            derive[j] = fold && !ct.is_zero();
            need1 = need1 || !derive[j];
        }
        launch_sc1_round_group(k, fold, j1.data(), half, need1, C.stream);
        C.sync();
        for (int j = 0; j < k; ++j) {
            P& p = ps[j];
            HFr gs[3] = {ld_hfr(p.hp), ld_hfr(p.hp + 32), ld_hfr(p.hp + 64)};
            const HFr ct = p.Cc * p.tau[i - 1];
            if (derive[j]) {
                const HFr d1 = (p.claim1 - (p.Cc - ct) * gs[0]) * ct.inv();
                if (check_derived && !(d1 == gs[1]))
                    throw SpxError(kSumcheck, "sumcheck 1 round " + std::to_string(i) + ": derived G(1) differs from the device's");
                gs[1] = d1;
            }
            std::vector<HFr> msg = sc1_message(p.Cc, p.tau[i - 1], gs, L);
            const size_t m0 = p.proof.b.size();
            p.proof.u64(msg.size());
            for (auto& e : msg) p.proof.fr(e);
            p.T.feed(p.proof.b.data() + m0, p.proof.b.size() - m0);
            const HFr ch = p.T.rand_fr();
            p.r_x.push_back(ch);
            const HFr eqc = eq1(p.tau[i - 1], ch);
            p.claim1 = p.Cc * eqc * quad_at(gs, ch);
            p.Cc = p.Cc * eqc;
            if (fold) {
                p.cur = j1[j].out;
                if (j1[j].Eout) p.Ecur = j1[j].Eout;
            }
        }
    }
    // the tables hold tn = 2^(ht+1) entries each: bind r_{L-ht} on the host, then the host rounds
    const uint32_t tn = 2u << ht;
    {
        const auto src = each([](P& p) { return p.cur; });
        const auto dst = each([&](P& p) { return C.pin_dev<Fr>(p.hp); });
        launch_copy_runs_group(k, src.data(), 3, (int)tn, dst.data(), C.stream);
    }
    C.sync();
    for (auto& p : ps) {
        std::vector<HFr> tabs[3];
        {
            const HFr r = p.r_x.back();
            for (int m = 0; m < 3; ++m)
                for (uint32_t b = 0; b < tn / 2; ++b) {
                    const HFr a0 = ld_hfr(p.hp + 32 * (m * tn + 2 * b)), a1 = ld_hfr(p.hp + 32 * (m * tn + 2 * b + 1));
                    tabs[m].push_back(a0 + r * (a1 - a0));
                }
        }
        for (int i = L - ht + 1; i <= L; ++i) {  // prove()'s rounds on gathered tables
            const size_t half = tabs[0].size() / 2;
            const int c = i - 1;
            HFr gs[3] = {HFr::zero(), HFr::zero(), HFr::zero()};
            for (size_t b = 0; b < half; ++b) {
                HFr e = HFr::one();  // eq(tau_{c+1..L-1}, b)
                for (int jj = c + 1; jj < L; ++jj) e *= ((b >> (jj - c - 1)) & 1) ? p.tau[jj] : HFr::one() - p.tau[jj];
                HFr x0[3], x1[3], y[3];
                for (int m = 0; m < 3; ++m) {
                    x0[m] = tabs[m][2 * b];
                    x1[m] = tabs[m][2 * b + 1];
                    y[m] = x1[m] + x1[m] - x0[m];
                }
                gs[0] += (x0[0] * x0[1] - x0[2]) * e;
                gs[1] += (x1[0] * x1[1] - x1[2]) * e;
                gs[2] += (y[0] * y[1] - y[2]) * e;
            }
            std::vector<HFr> msg = sc1_message(p.Cc, p.tau[c], gs, L);
            const size_t m1 = p.proof.b.size();
            p.proof.u64(msg.size());
            for (auto& e : msg) p.proof.fr(e);
            p.T.feed(p.proof.b.data() + m1, p.proof.b.size() - m1);
            const HFr ch = p.T.rand_fr();
            p.r_x.push_back(ch);
            p.Cc = p.Cc * eq1(p.tau[c], ch);
            for (int m = 0; m < 3; ++m) {
                std::vector<HFr> nt(half);
                for (size_t b = 0; b < half; ++b) nt[b] = tabs[m][2 * b] + ch * (tabs[m][2 * b + 1] - tabs[m][2 * b]);
                tabs[m].swap(nt);
            }
        }
        const HFr v[3] = {tabs[0][0], tabs[1][0], tabs[2][0]};
        // ---- round 4
        size_t m0 = p.proof.b.size();
        for (int m = 0; m < 3; ++m) p.proof.fr(v[m]);
        p.T.feed(p.proof.b.data() + m0, p.proof.b.size() - m0);
        HFr rabc[3] = {p.T.rand_fr(), p.T.rand_fr(), p.T.rand_fr()};
        // ---- round 5's challenges, staged for one copy (the waits above cover the stage's earlier copy)
        uint8_t* st = stage + (size_t)32 * (8 * L * (&p - ps.data()) + 2 * L);
        memcpy(st, p.r_x.data(), 32 * L);
        memcpy(st + 32 * L, rabc, 96);
        m0 = p.proof.b.size();
        p.proof.u64(2);
        p.proof.u64((uint64_t)L);
        p.T.feed(p.proof.b.data() + m0, p.proof.b.size() - m0);
        p.proof.u64((uint64_t)L);
        p.claim2 = HFr::zero();
        p.Mc = p.M0;
        p.Zc = p.z;
    }
    // ---- round 5: M_rx = sum_m r_m M(r_x, .) of every proof
    SPX_HIP(hipMemcpyAsync(chg, stage, (size_t)32 * 8 * L * k, hipMemcpyHostToDevice, C.stream));
    kp_begin(KP_MTV, C.stream);
    if (I.cols.longc.nchunks == 0) {
        const auto rx = each([&](P& p) -> const Fr* { return p.chdev + 2 * L; });
        const auto sc = each([&](P& p) -> const Fr* { return p.chdev + 3 * L; });
        const auto outs = each([](P& p) { return p.M0; });
        const auto eqs = each([](P& p) { return p.eqf; });
        launch_col_stream_group(k, I.cols.view(), rx.data(), L, sc.data(), outs.data(), eqs.data(), C.stream);
    } else {
        for (auto& p : ps) I.cols.launch(p.chdev + 2 * L, L, p.chdev + 3 * L, p.M0, p.eqf, p.partial, C.stream);
    }
    kp_end(I.cols_bytes * k, C.stream);
    // ---- sumcheck 2
    std::vector<Sc2Job> j2(k);
    for (int i = 1; i <= L - ht; ++i) {
        const uint64_t half = nl >> i;
        const bool fold = i >= 2;
        for (int j = 0; j < k; ++j) {
            P& p = ps[j];
            Sc2Job& jb = j2[j];
            jb.Min = p.Mc;
            jb.Zin = p.Zc;
            jb.Mout = fold ? ((i & 1) ? p.M2 : p.M1) : nullptr;
            jb.Zout = fold ? ((i & 1) ? p.Z2 : p.Z1) : nullptr;
            jb.r = fold ? dev_fr(p.r_y[i - 2]) : Fr{};
            jb.partial = p.partial;
            jb.ticket = C.ticket + j;
            jb.result3 = p.res_dev;
        }
        launch_sc2_round_group(k, fold, j2.data(), half, !fold || check_derived, C.stream);
        C.sync();
        for (int j = 0; j < k; ++j) {
            P& p = ps[j];
            HFr q[3] = {ld_hfr(p.hp), ld_hfr(p.hp + 32), ld_hfr(p.hp + 64)};
            if (fold) {
                const HFr d1 = p.claim2 - q[0];
                if (check_derived && !(d1 == q[1]))
                    throw SpxError(kSumcheck, "sumcheck 2 round " + std::to_string(i) + ": derived P(1) differs from the device's");
                q[1] = d1;
            }
            const size_t m0 = p.proof.b.size();
            p.proof.u64(3);
            for (int t = 0; t < 3; ++t) p.proof.fr(q[t]);
            p.T.feed(p.proof.b.data() + m0, p.proof.b.size() - m0);
            const HFr ch = p.T.rand_fr();
            p.r_y.push_back(ch);
            p.claim2 = quad_at(q, ch);
            if (fold) {
                p.Mc = j2[j].Mout;
                p.Zc = j2[j].Zout;
            }
        }
    }
    if (ht > 0) {  // M and Z hold tn entries each: bind r_{L-ht}, then the host rounds
        {
            const auto src = each([](P& p) { return Tables3{{const_cast<Fr*>(p.Mc), const_cast<Fr*>(p.Zc), nullptr}}; });
            const auto dst = each([&](P& p) { return C.pin_dev<Fr>(p.hp); });
            launch_copy_runs_group(k, src.data(), 2, (int)tn, dst.data(), C.stream);
        }
        C.sync();
        for (auto& p : ps) {
            const HFr r = p.r_y.back();
            std::vector<HFr> Mt, Zt;
            for (uint32_t b = 0; b < tn / 2; ++b) {
                const HFr m0v = ld_hfr(p.hp + 32 * (2 * b)), m1v = ld_hfr(p.hp + 32 * (2 * b + 1));
                const HFr z0 = ld_hfr(p.hp + 32 * (tn + 2 * b)), z1 = ld_hfr(p.hp + 32 * (tn + 2 * b + 1));
                Mt.push_back(m0v + r * (m1v - m0v));
                Zt.push_back(z0 + r * (z1 - z0));
            }
            for (int i = L - ht + 1; i <= L; ++i) {  // prove()'s rounds on gathered tables
                const size_t half = Mt.size() / 2;
                HFr q[3] = {HFr::zero(), HFr::zero(), HFr::zero()};
                for (size_t b = 0; b < half; ++b) {
                    const HFr m0v = Mt[2 * b], m1v = Mt[2 * b + 1], z0 = Zt[2 * b], z1 = Zt[2 * b + 1];
                    q[0] += m0v * z0;
                    q[1] += m1v * z1;
                    q[2] += (m1v + m1v - m0v) * (z1 + z1 - z0);
                }
                const size_t m1 = p.proof.b.size();
                p.proof.u64(3);
                for (int t = 0; t < 3; ++t) p.proof.fr(q[t]);
                p.T.feed(p.proof.b.data() + m1, p.proof.b.size() - m1);
                const HFr ch = p.T.rand_fr();
                p.r_y.push_back(ch);
                std::vector<HFr> nm(half), nz(half);
                for (size_t b = 0; b < half; ++b) {
                    nm[b] = Mt[2 * b] + ch * (Mt[2 * b + 1] - Mt[2 * b]);
                    nz[b] = Zt[2 * b] + ch * (Zt[2 * b + 1] - Zt[2 * b]);
                }
                Mt.swap(nm);
                Zt.swap(nz);
            }
        }
    }
    // ---- round 6: open at r_y
    {
        std::vector<std::vector<HFr>> pts(k);
        for (int j = 0; j < k; ++j) pts[j] = ps[j].r_y;
        open_all(pts);
    }
    std::vector<std::vector<uint8_t>> out(k);
    for (int j = 0; j < k; ++j) out[j] = std::move(ps[j].proof.b);
    C.timings.emplace_back("total_group", tgroup.us());
    return out;
}

// ====================================================================== kernel-level entry points
// ====================================================================== verifier
// lib.rs:147-212 with verifier.rs:143-512. The transcript is replayed on the host; the O(nnz) matrix
// evaluation (A, B, C)(r_x, r_y) runs on the GPU with the prover's kernels (eq table, CSC gather into
// sum_M r_M M(r_x, .), then L fold levels at r_y); the two mKZG checks (verify.rs:12-45) use the
// host pairing of pairing.hpp.
VP vp_load(const uint8_t* b, size_t len) {
    VP V;
    size_t pos = 0;
    auto take = [&](size_t k) {
        if (pos + k > len) throw SpxError(kSerialization, "truncated verifier parameter");
        const uint8_t* p = b + pos;
        pos += k;
        return p;
    };
    uint64_t nv, cnt;
    memcpy(&nv, take(8), 8);
    if (nv > (uint64_t)kMaxLogN) throw SpxError(kSerialization, "bad verifier parameter nv (<= 26 supported)");
    V.nv = (int)nv;
    if (!host::g1_from_uncompressed(V.g, take(96)) || !host::g2_from_uncompressed(V.h, take(192)))
        throw SpxError(kSerialization, "bad verifier parameter point");
    memcpy(&cnt, take(8), 8);
    if (cnt != nv) throw SpxError(kSerialization, "g_mask_random length != nv");
    V.g_mask.resize(cnt);
    for (auto& g : V.g_mask)
        if (!host::g1_from_uncompressed(g, take(96))) throw SpxError(kSerialization, "bad g_mask_random point");
    if (pos != len) throw SpxError(kSerialization, "trailing bytes in verifier parameter");
    return V;
}
std::vector<uint8_t> vp_serialize(const VP& V) {
    Ser s;
    s.u64((uint64_t)V.nv);
    uint8_t b[192];
    host::g1_to_uncompressed(b, V.g);
    s.raw(b, 96);
    host::g2_to_uncompressed(b, V.h);
    s.raw(b, 192);
    s.u64(V.g_mask.size());
    for (auto& g : V.g_mask) {
        host::g1_to_uncompressed(b, g);
        s.raw(b, 96);
    }
    return s.b;
}
VP vp_from_pp(const PP& P) {
    if (!P.has_t) invalid("verifier parameter needs a keygen-generated PP (trapdoor unknown)");
    VP V;
    V.nv = P.nv;
    V.g = P.g;
    V.h = P.h;
    for (int i = 0; i < P.nv; ++i) {  // setup.rs:91-101: g_mask_random[i] = g^{t_i}
        uint64_t k[4];
        P.t[i].to_canon(k);
        V.g_mask.push_back(host::jac_to_affine(host::jac_mul(host::jac_from(P.g), k)));
    }
    return V;
}

namespace {
struct ProofReader {
    const uint8_t* b;
    size_t len, pos = 0;
    const uint8_t* take(size_t k) {
        if (pos + k > len) throw SpxError(kSerialization, "truncated proof");
        const uint8_t* p = b + pos;
        pos += k;
        return p;
    }
    uint64_t u64() {
        uint64_t v;
        memcpy(&v, take(8), 8);
        return v;
    }
    HFr fr() {
        HFr r;
        if (!host::fr_from_bytes(r, take(32))) throw SpxError(kSerialization, "non-canonical field element");
        return r;
    }
    host::Affine<HFq> g1() {
        host::Affine<HFq> a;
        if (!host::g1_decompress(a, take(48))) throw SpxError(kSerialization, "invalid G1 point");
        return a;
    }
    host::Affine<HFq2> g2() {
        host::Affine<HFq2> a;
        if (!host::g2_decompress(a, take(96))) throw SpxError(kSerialization, "invalid G2 point");
        return a;
    }
};
struct OpenProof {
    HFr eval;
    host::Affine<HFq2> h;
    std::vector<host::Affine<HFq2>> proofs;
};
OpenProof read_open(ProofReader& R) {
    OpenProof o;
    o.eval = R.fr();
    o.h = R.g2();
    const uint64_t k = R.u64();
    if (k > 64) throw SpxError(kSerialization, "bad opening proof length");
    for (uint64_t i = 0; i < k; ++i) o.proofs.push_back(R.g2());
    return o;
}
std::vector<std::vector<HFr>> read_msgs(ProofReader& R, std::vector<std::pair<size_t, size_t>>& spans) {
    const uint64_t rounds = R.u64();
    if (rounds > 64) throw SpxError(kSerialization, "bad sumcheck round count");
    std::vector<std::vector<HFr>> m(rounds);
    for (auto& e : m) {
        const size_t start = R.pos;
        const uint64_t k = R.u64();
        if (k > 1024) throw SpxError(kSerialization, "bad sumcheck message length");
        for (uint64_t i = 0; i < k; ++i) e.push_back(R.fr());
        spans.emplace_back(start, R.pos - start);
    }
    return m;
}
// linear-sumcheck interpolate_uni_poly: value at x of the polynomial through (i, ev[i])
HFr interpolate(const std::vector<HFr>& ev, const HFr& x) {
    const size_t n = ev.size();
    HFr total = HFr::zero();
    for (size_t i = 0; i < n; ++i) {
        HFr num = HFr::one(), den = HFr::one();
        for (size_t j = 0; j < n; ++j) {
            if (j == i) continue;
            num = num * (x - HFr::from_u64(j));
            den = den * (HFr::from_u64(i) - HFr::from_u64(j));
        }
        total = total + ev[i] * num * den.inv();
    }
    return total;
}
// linear-sumcheck check_and_generate_subclaim; its errors surface as Error::SumCheckError
HFr check_subclaim(const std::vector<std::vector<HFr>>& msgs, const std::vector<HFr>& rnd, HFr expected, int nv,
                   uint64_t max_mult) {
    if ((int)msgs.size() != nv) throw SpxError(kSumcheck, "insufficient rounds");
    for (size_t i = 0; i < msgs.size(); ++i) {
        if (msgs[i].size() != max_mult + 1) throw SpxError(kSumcheck, "wrong number of evaluations");
        if (!(msgs[i][0] + msgs[i][1] == expected))
            throw SpxError(kSumcheck, "Prover message is not consistent with the claim.");
        expected = interpolate(msgs[i], rnd[i]);
    }
    return expected;
}
// MLPolyCommit::verify (verify.rs:12-45), vp.h on the left as in the reference
bool mkzg_check(const VP& V, const host::Affine<HFq>& com, const std::vector<HFr>& point, const HFr& value,
                const OpenProof& op) {
    if ((int)op.proofs.size() < V.nv || (int)point.size() < V.nv) return false;
    using host::jac_add;
    using host::jac_from;
    using host::jac_mul;
    using host::jac_to_affine;
    auto neg = [](host::Affine<HFq> a) {
        a.y = -a.y;
        return a;
    };
    uint64_t k[4];
    value.to_canon(k);
    std::vector<std::pair<host::Affine<HFq>, host::Affine<HFq2>>> pairs;
    pairs.push_back({jac_to_affine(jac_add(jac_from(com), jac_from(neg(jac_to_affine(jac_mul(jac_from(V.g), k)))))),
                     V.h});
    for (int i = 0; i < V.nv; ++i) {
        point[i].to_canon(k);
        host::Affine<HFq> li = jac_to_affine(
            jac_add(jac_from(V.g_mask[i]), jac_from(neg(jac_to_affine(jac_mul(jac_from(V.g), k))))));
        if (!li.inf) li = neg(li);
        pairs.push_back({li, op.proofs[i]});
    }
    return host::pairing_product_is_one(pairs);
}
HFr mle_eval_host(std::vector<HFr> t, const std::vector<HFr>& point) {
    for (const HFr& r : point) {
        std::vector<HFr> nt(t.size() / 2);
        for (size_t b = 0; b < nt.size(); ++b) nt[b] = t[2 * b] + r * (t[2 * b + 1] - t[2 * b]);
        t.swap(nt);
    }
    return t[0];
}
}  // namespace

// sum_M r_M M(r_x, r_y) on the GPU: eq(r_x) table, CSC gather (the prover's eval_on_x pass), L folds
static HFr eval_matrices_at(Ctx& C, Index& I, const std::vector<HFr>& r_x, const HFr rabc[3],
                            const std::vector<HFr>& r_y) {
    const int L = I.log_n;
    const uint64_t n = I.n;
    const uint64_t parts = std::max<uint64_t>(3 * 2048, (uint64_t)I.cols.longc.nchunks);
    C.scratch.ensure(32 * (n + n + n / 2 + 2 + parts + kEqScratch + 4 * L + 8));
    Fr* base = C.scratch.as<Fr>();
    Fr *EQ = base, *M0 = EQ + n, *Mb = M0 + n, *partial = Mb + n / 2 + 2, *eqf = partial + parts;
    Fr* ch = eqf + kEqScratch;  // r_x (L), r_abc (3), r_y (L)
    std::vector<HFr> hch(r_x);
    hch.insert(hch.end(), rabc, rabc + 3);
    hch.insert(hch.end(), r_y.begin(), r_y.end());
    uint8_t* hs = C.pin_at(Ctx::kPinStage, 32 * hch.size(), 64 << 10);
    memcpy(hs, hch.data(), 32 * hch.size());
    SPX_HIP(hipMemcpyAsync(ch, hs, 32 * hch.size(), hipMemcpyHostToDevice, C.stream));
    I.cols.launch(ch, L, ch + L, M0, eqf, partial, C.stream);
    // fold at r_y (variable 0 = LSB): M0 -> EQ (as q scratch) / Mb ping-pong
    const Fr* rin = M0;
    Fr* bufs[2] = {Mb, M0};
    for (int i = 0; i < L; ++i) {
        const uint64_t half = n >> (i + 1);
        Fr* rout = bufs[i & 1];
        launch_open_level(rin, rout, EQ, dev_fr(r_y[i]), half, C.stream);
        rin = rout;
    }
    uint8_t* hp = C.pin_at(Ctx::kPinOpen, 32, 56 << 10);
    SPX_HIP(hipMemcpyAsync(hp, rin, 32, hipMemcpyDeviceToHost, C.stream));
    C.sync();
    return ld_hfr(hp);
}

void verify(Ctx& C, Index& I, const uint8_t* v, size_t nv, const uint8_t* proof, size_t len, const VP& V,
            const ProveOpts& o) {
    if (I.G != 1) invalid("verify needs an index built on a single-rank context");
    const int L = I.log_n;
    const uint64_t n = I.n;
    // verifier_init (verifier.rs:143-146)
    if (!is_pow2(nv) || nv > n)
        invalid("public input should be power of two and has size smaller than number of constraints");
    const int log_v = ilog2(nv);
    std::vector<HFr> vv(nv);
    for (size_t i = 0; i < nv; ++i)
        if (!host::fr_from_bytes(vv[i], v + 32 * i)) invalid("public input is not a canonical field element");
    // parse (proof.rs:10-20 field order); remember each message's byte span for the transcript
    ProofReader R{proof, len};
    const size_t pm1_at = R.pos;
    const uint64_t com_nv = R.u64();
    const host::Affine<HFq> com = R.g1();
    const size_t pm1_len = R.pos - pm1_at, pm2_at = R.pos;
    const OpenProof op1 = read_open(R);
    const size_t pm2_len = R.pos - pm2_at, pm3_at = R.pos;
    const uint64_t mm1 = R.u64(), nv1 = R.u64();
    std::vector<std::pair<size_t, size_t>> sp1, sp2;
    const auto sc1 = read_msgs(R, sp1);
    const size_t pm4_at = R.pos;
    const HFr va = R.fr(), vb = R.fr(), vc = R.fr();
    const size_t pm5_at = R.pos;
    const uint64_t mm2 = R.u64(), nv2 = R.u64();
    const auto sc2 = read_msgs(R, sp2);
    const size_t pm6_at = R.pos;
    const OpenProof op2 = read_open(R);
    const size_t pm6_len = R.pos - pm6_at;
    if (R.pos != len) throw SpxError(kSerialization, "trailing bytes in proof");
    (void)com_nv;
    // transcript (lib.rs:152-212 feed order)
    Transcript T(o.mode == 1, o.seed);
    if (o.cached && I.has_cache)
        T.set_state(I.cache);
    else {
        Blake2s h;
        for (int m = 0; m < 3; ++m) feed_matrix(h, I.m[m]);
        T.set_state(h);
    }
    {
        Ser s;
        s.u64(nv);
        s.raw(v, 32 * nv);
        T.feed(s.b.data(), s.b.size());
    }
    T.feed(proof + pm1_at, pm1_len);
    std::vector<HFr> r_v(log_v);
    for (auto& r : r_v) r = T.rand_fr();
    T.feed(proof + pm2_at, pm2_len);
    std::vector<HFr> tau(L);
    for (auto& t : tau) t = T.rand_fr();
    if (nv1 != (uint64_t)L) invalid("invalid sumcheck proposal");
    T.feed(proof + pm3_at, 16);
    if ((int)sc1.size() != L || (int)sc2.size() != L) invalid("malformed sumcheck message");
    std::vector<HFr> rand1, rand2;
    for (auto& sp : sp1) {
        T.feed(proof + sp.first, sp.second);
        rand1.push_back(T.rand_fr());
    }
    T.feed(proof + pm4_at, 96);
    const HFr r_a = T.rand_fr(), r_b = T.rand_fr(), r_c = T.rand_fr();
    if (nv2 != (uint64_t)L) invalid("invalid sumcheck proposal");
    T.feed(proof + pm5_at, 16);
    for (auto& sp : sp2) {
        T.feed(proof + sp.first, sp.second);
        rand2.push_back(T.rand_fr());
    }
    T.feed(proof + pm6_at, pm6_len);
    // verify_sixth_round (verifier.rs:443-512)
    if (V.nv != L) invalid("verifier parameter nv != log_n");
    std::vector<HFr> r_v0(L, HFr::zero());
    for (int i = 0; i < log_v; ++i) r_v0[i] = r_v[i];
    if (!mkzg_check(V, com, r_v0, op1.eval, op1)) invalid("public witness failed in commitment check");
    if (!(mle_eval_host(vv, r_v) == op1.eval)) invalid("public witness is inconsistent with proof");
    const HFr expected1 = check_subclaim(sc1, rand1, HFr::zero(), L, mm1);
    HFr eq_rx = HFr::one();
    for (int i = 0; i < L; ++i) eq_rx = eq_rx * eq1(tau[i], rand1[i]);
    if (!((va * vb - vc) * eq_rx == expected1)) throw SpxError(kWrongWitness, "first sumcheck has wrong subclaim");
    const HFr claimed2 = r_a * va + r_b * vb + r_c * vc;
    const HFr expected2 = check_subclaim(sc2, rand2, claimed2, L, mm2);
    const HFr rabc[3] = {r_a, r_b, r_c};
    const HFr actual = eval_matrices_at(C, I, rand1, rabc, rand2) * op2.eval;
    if (!(expected2 == actual)) throw SpxError(kWrongWitness, "Cannot verify matrix A, B, C");
    if (!mkzg_check(V, com, rand2, op2.eval, op2)) throw SpxError(kWrongWitness, "Cannot verify z_ry");
}

static HostCsr single(const HostCsr& m) { return m; }

std::vector<uint8_t> k_sum_over_y(Ctx& C, const HostCsr& m, const uint8_t* z) {
    const uint64_t n = m.n;
    check_csr(m, n);
    HostCsr empty;
    empty.n = n;
    empty.rp.assign(n + 1, 0);
    HostCsr mats[3] = {single(m), empty, empty};
    DevSparse D;
    std::vector<uint64_t> rps[3] = {mats[0].rp, mats[1].rp, mats[2].rp};
    std::vector<uint32_t> cols[3] = {mats[0].col, mats[1].col, mats[2].col};
    std::vector<uint8_t> vals[3] = {mats[0].val, mats[1].val, mats[2].val};
    DevMem err(sizeof(int)), zd(32 * n), out(32 * n * 3), part(32 * 4096);
    SPX_HIP(hipMemsetAsync(err.p, 0, 4, C.stream));
    DevSliced S;  // the same two paths as prove(): sliced entries for single-entry rows, else CSR
    if (!upload_sliced(C, S, mats, n, 0, n, err.as<int>())) upload_sparse(C, D, rps, cols, vals, 0, n, err.as<int>());
    SPX_HIP(hipMemcpyAsync(zd.p, z, 32 * n, hipMemcpyHostToDevice, C.stream));
    launch_to_mont(zd.as<Fr>(), n, err.as<int>(), C.stream);
    Fr* o = out.as<Fr>();
    if (D.nchunks > (int)4096) part.alloc(32 * D.nchunks);
    if (S.on)
        launch_spmv_sliced(S.view(), zd.as<Fr>(), o, o + n, o + 2 * n, S.entries, C.stream);
    else
        launch_sparse3(0, D.view(), zd.as<Fr>(), o, o + n, o + 2 * n, nullptr, n, D.chunks.as<LongChunk>(), D.nchunks,
                       D.lrows.as<LongRow>(), D.nlrows, part.as<Fr>(), C.stream);
    launch_from_mont(o + n, o, n, C.stream);
    std::vector<uint8_t> res(32 * n);
    SPX_HIP(hipMemcpyAsync(res.data(), o + n, 32 * n, hipMemcpyDeviceToHost, C.stream));
    C.sync();
    return res;
}

std::vector<uint8_t> k_eval_on_x(Ctx& C, const HostCsr& m, const uint8_t* r_x) {
    const uint64_t n = m.n;
    check_csr(m, n);
    if (!is_pow2(n)) invalid("2^(r_x) should have size: num_constraints");
    const int L = ilog2(n);
    // CSC of m (matrices B, C empty), scale (1, 0, 0)
    std::vector<uint64_t> cp;
    std::vector<uint32_t> rows;
    std::vector<uint8_t> vals;
    build_csc(m, n, cp, rows, vals);
    std::vector<uint64_t> rps[3] = {cp, std::vector<uint64_t>(n + 1, 0), std::vector<uint64_t>(n + 1, 0)};
    std::vector<uint32_t> cols[3] = {rows, {}, {}};
    std::vector<uint8_t> vv[3] = {vals, {}, {}};
    DevColStream D;
    DevMem err(sizeof(int)), rx(32 * L + 96), out(32 * n * 2), part(32 * std::max(4096, 1)), eqf(32 * kEqScratch);
    SPX_HIP(hipMemsetAsync(err.p, 0, 4, C.stream));
    upload_cols(C, D, rps, cols, vv, 0, n, err.as<int>());
    std::vector<uint8_t> hr(32 * L + 96, 0);
    memcpy(hr.data(), r_x, 32 * L);
    HFr one = HFr::one();
    uint64_t onec[4];
    one.to_canon(onec);
    memcpy(hr.data() + 32 * L, onec, 32);  // canonical 1, 0, 0
    SPX_HIP(hipMemcpyAsync(rx.p, hr.data(), hr.size(), hipMemcpyHostToDevice, C.stream));
    launch_to_mont(rx.as<Fr>(), L + 3, err.as<int>(), C.stream);
    if (D.longc.nchunks > 4096) part.alloc(32 * D.longc.nchunks);
    Fr* o = out.as<Fr>();
    D.launch(rx.as<Fr>(), L, rx.as<Fr>() + L, o, eqf.as<Fr>(), part.as<Fr>(), C.stream);
    launch_from_mont(o + n, o, n, C.stream);
    std::vector<uint8_t> res(32 * n);
    SPX_HIP(hipMemcpyAsync(res.data(), o + n, 32 * n, hipMemcpyDeviceToHost, C.stream));
    int herr = 0;
    SPX_HIP(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, C.stream));
    C.sync();
    if (herr) throw SpxError(kSerialization, "non-canonical field element");
    return res;
}

// One AHPForMLSumcheck::prove_round [upstream linear-sumcheck] of sum_b f(b) g(b) (the second sumcheck's
// product shape [r_M M(r_x, .), z], prover.rs:239-247) through the product's round kernels: with r_prev
// the tables are first bound at variable 0 (T'[b] = T[2b] + r (T[2b+1] - T[2b]), n/2 entries out), then
// P(t) = sum_b f'(b, t) g'(b, t) at t = 0, 1, 2. Canonical bytes in and out.
void k_sumcheck_round(Ctx& C, const uint8_t* f, const uint8_t* g, uint64_t n, const uint8_t* r_prev,
                      uint8_t* evals_out, uint8_t* f_out, uint8_t* g_out) {
    if (!is_pow2(n) || n < (r_prev ? 4u : 2u)) invalid("table size must be a power of two (>= 2, >= 4 with a challenge)");
    const bool fold = r_prev != nullptr;
    const uint64_t half = fold ? n / 4 : n / 2;
    DevMem err(sizeof(int)), tabs(32 * 2 * n), outs(32 * (fold ? n : 2)), res(32 * (3 + std::max<uint64_t>(n, 3))),
        part(32 * kRoundPartials);
    SPX_HIP(hipMemsetAsync(err.p, 0, 4, C.stream));
    Fr* F = tabs.as<Fr>();
    Fr* Gt = F + n;
    SPX_HIP(hipMemcpyAsync(F, f, 32 * n, hipMemcpyHostToDevice, C.stream));
    SPX_HIP(hipMemcpyAsync(Gt, g, 32 * n, hipMemcpyHostToDevice, C.stream));
    launch_to_mont(F, 2 * n, err.as<int>(), C.stream);
    Fr r{};
    if (fold) {
        uint64_t c[4];
        memcpy(c, r_prev, 32);
        if (HFr::geq_p(c)) throw SpxError(kSerialization, "non-canonical challenge");
        r = dev_fr(HFr::from_canon(c));
    }
    Fr* Fo = fold ? outs.as<Fr>() : nullptr;
    Fr* Go = fold ? Fo + n / 2 : nullptr;
    Fr* ev = res.as<Fr>();
    launch_sc2_round(fold, F, Gt, Fo, Go, r, half, part.as<Fr>(), C.ticket, ev, true, C.stream);
    Fr* canon = ev + 3;
    launch_from_mont(canon, ev, 3, C.stream);
    int herr = 0;
    SPX_HIP(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, C.stream));
    SPX_HIP(hipMemcpyAsync(evals_out, canon, 96, hipMemcpyDeviceToHost, C.stream));
    C.sync();
    if (herr) throw SpxError(kSerialization, "non-canonical field element");
    if (fold) {
        launch_from_mont(canon, Fo, n, C.stream);  // f' then g' (n / 2 each, contiguous)
        if (f_out) SPX_HIP(hipMemcpyAsync(f_out, canon, 16 * n, hipMemcpyDeviceToHost, C.stream));
        if (g_out) SPX_HIP(hipMemcpyAsync(g_out, canon + n / 2, 16 * n, hipMemcpyDeviceToHost, C.stream));
        C.sync();
    }
}

std::vector<uint8_t> k_msm(Ctx& C, bool g2, const uint8_t* bases, const uint8_t* scalars, size_t n) {
    if (n == 0) invalid("empty MSM");
    const size_t ps = g2 ? 192 : 96;
    DevMem raw(ps * n), sc(32 * n), err(sizeof(int));
    SPX_HIP(hipMemsetAsync(err.p, 0, 4, C.stream));
    SPX_HIP(hipMemcpyAsync(raw.p, bases, ps * n, hipMemcpyHostToDevice, C.stream));
    SPX_HIP(hipMemcpyAsync(sc.p, scalars, 32 * n, hipMemcpyHostToDevice, C.stream));
    launch_to_mont(sc.as<Fr>(), n, err.as<int>(), C.stream);
    if (g2)
        launch_points_from_bytes_g2(raw.as<G2Aff>(), n, err.as<int>(), C.stream);
    else
        launch_points_from_bytes_g1(raw.as<G1Aff>(), n, err.as<int>(), C.stream);
    MsmInst I{};
    I.c = (uint32_t)window_bits_for(n);
    I.W = (uint32_t)windows_for((int)I.c);
    I.size = (uint32_t)n;
    I.stride = (uint32_t)n;
    DevMem pre((g2 ? sizeof(G2Aff) : sizeof(G1Slot)) * n * I.W), out(msm_out_bytes(g2, 1));
    if (g2)
        precompute_level(C, raw.as<G2Aff>(), n, false, (int)I.c, (int)I.W, pre.as<G2Aff>());
    else
        precompute_level(C, raw.as<G1Aff>(), n, false, (int)I.c, (int)I.W, pre.as<G1Slot>());
    if (g2)
        msm_run_g2(C.msm, &I, 1, pre.as<G2Aff>(), sc.as<Fr>(), out.p, C.stream);
    else
        msm_run_g1(C.msm, &I, 1, pre.as<G1Slot>(), sc.as<Fr>(), out.p, C.stream);
    std::vector<uint8_t> h(out.bytes);
    int herr = 0;
    SPX_HIP(hipMemcpyAsync(h.data(), out.p, out.bytes, hipMemcpyDeviceToHost, C.stream));
    SPX_HIP(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, C.stream));
    C.sync();
    if (herr & 1) throw SpxError(kSerialization, "non-canonical input");
    if (herr & 2) throw SpxError(kSerialization, "base point not on the curve");
    std::vector<uint8_t> res(ps);
    LocalComm local;
    if (g2)
        host::g2_to_uncompressed(res.data(), msm_results<HFq2>(local, h.data(), 1)[0]);
    else
        host::g1_to_uncompressed(res.data(), msm_results<HFq>(local, h.data(), 1)[0]);
    return res;
}

std::vector<uint8_t> k_commit(Ctx& C, PP& P, const uint8_t* table, int nv) {
    if (nv != P.nv) invalid("table size != 2^nv of the public parameters");
    auto W = witness_upload(C, table, 1, table + 32, (1ull << nv) - 1);
    LocalComm local;
    commit_launch(C, P, W->z.as<Fr>(), 1ull << nv, MsmShard());
    Affine<HFq> a = commit_finish(C, P, W->z.as<Fr>(), 1ull << nv, local);
    std::vector<uint8_t> out(56);
    uint64_t u = (uint64_t)nv;
    memcpy(out.data(), &u, 8);
    host::g1_compress(out.data() + 8, a);
    return out;
}

std::vector<uint8_t> k_open(Ctx& C, PP& P, const uint8_t* table, int nv, const uint8_t* point) {
    if (nv != P.nv) invalid("table size != 2^nv of the public parameters");
    auto W = witness_upload(C, table, 1, table + 32, (1ull << nv) - 1);
    std::vector<HFr> pt(nv);
    for (int i = 0; i < nv; ++i)
        if (!host::fr_from_bytes(pt[i], point + 32 * i)) throw SpxError(kSerialization, "non-canonical point");
    LocalComm local;
    OpenOut op = open_z(C, P, W->z.as<Fr>(), nv, pt, local);
    Ser s;
    ser_open(s, op.eval, P.h, op.proofs);
    return s.b;
}

}  // namespace spx
