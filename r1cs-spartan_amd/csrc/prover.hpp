// Host-side state of the MI355X prover: contexts (one per GPU / rank), communicators,
// device-resident public parameters, prover keys, witnesses.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "host_ff.hpp"
#include "kernels.hpp"
#include "transcript.hpp"

namespace spx {

struct SpxError : std::runtime_error {
    int code;
    SpxError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
enum { kOk = 0, kInvalidArgument = 1, kSumcheck = 2, kWrongWitness = 3, kSerialization = 4, kDevice = 5 };

#define SPX_HIP(x)                                                                                   \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess)                                                                        \
            throw ::spx::SpxError(::spx::kDevice, std::string("HIP: ") + hipGetErrorString(e_) + " (" #x ") at " + \
                                                     __FILE__ + ":" + std::to_string(__LINE__));    \
    } while (0)

inline void invalid(const std::string& m) { throw SpxError(kInvalidArgument, m); }
inline int ilog2(uint64_t x) { return 63 - __builtin_clzll(x); }
inline bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

// Largest supported log_n / nv. Bounded by the MSM references (31-bit point index: n x 16 window
// copies < 2^31 up to n = 2^26) and by the eq-table scratch (two halves of <= 2^13 entries each).
static constexpr int kMaxLogN = 26;

// owning device allocation
struct DevMem {
    void* p = nullptr;
    size_t bytes = 0;
    DevMem() = default;
    explicit DevMem(size_t b) { alloc(b); }
    void alloc(size_t b) {
        release();
        if (b) SPX_HIP(hipMalloc(&p, b));
        bytes = b;
    }
    void ensure(size_t b) {
        if (b > bytes) alloc(b);
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
    ~DevMem() { release(); }
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
};

// ---------------------------------------------------------------- communicators
struct Comm {
    virtual ~Comm() {}
    virtual int rank() const = 0;
    virtual int size() const = 0;
    // host buffers; every rank contributes `bytes`, recv holds size() * bytes in rank order
    virtual void allgather(const void* send, void* recv, size_t bytes) = 0;
};
struct LocalComm : Comm {
    int rank() const override { return 0; }
    int size() const override { return 1; }
    void allgather(const void* s, void* r, size_t b) override { memcpy(r, s, b); }
};
// Rehearsal of ONE rank of a proof-sharded prove on a GPU of its own (bench / scaling estimates):
// every allgather returns this rank's contribution in all `world` slots, so the rank does exactly a
// real rank's device and host work without its peers. The proofs it outputs are NOT valid proofs.
// SPX_REHEARSAL_EXCHANGE_NS (read when the comm is set): each allgather then also takes that long,
// the latency of a real exchange charged to the rank (bench.py measures it among world CPU processes
// over the shared-memory transport): a short spin, as comm_shm.cpp's, then a sleep for the rest.
struct SoloComm : Comm {
    int r, w;
    int64_t delay_ns = 0;
    SoloComm(int rank, int world) : r(rank), w(world) {
        if (const char* e = getenv("SPX_REHEARSAL_EXCHANGE_NS")) delay_ns = std::max<int64_t>(0, atoll(e));
    }
    int rank() const override { return r; }
    int size() const override { return w; }
    void allgather(const void* s, void* rv, size_t b) override {
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < w; ++k) memcpy((uint8_t*)rv + k * b, s, b);
        if (delay_ns <= 0) return;
        const auto until = t0 + std::chrono::nanoseconds(delay_ns);
        const auto spin_until = t0 + std::chrono::nanoseconds(std::min<int64_t>(delay_ns, 4000));
        while (std::chrono::steady_clock::now() < spin_until) {
        }
        const auto now = std::chrono::steady_clock::now();
        if (now < until) std::this_thread::sleep_for(until - now);
    }
};
struct GroupState {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::vector<uint8_t>> slots;
    int arrived = 0;
    uint64_t gen = 0;
    explicit GroupState(int w) : world(w), slots(w) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};
struct GroupComm : Comm {
    std::shared_ptr<GroupState> st;
    int r;
    GroupComm(std::shared_ptr<GroupState> s, int rk) : st(std::move(s)), r(rk) {}
    int rank() const override { return r; }
    int size() const override { return st->world; }
    void allgather(const void* s, void* rv, size_t b) override {
        {
            std::lock_guard<std::mutex> lk(st->mu);
            st->slots[r].assign((const uint8_t*)s, (const uint8_t*)s + b);
        }
        st->barrier();
        for (int k = 0; k < st->world; ++k) memcpy((uint8_t*)rv + k * b, st->slots[k].data(), b);
        st->barrier();
    }
};
std::unique_ptr<Comm> make_shm_comm(const char* name, int rank, int world);
std::unique_ptr<Comm> make_rccl_comm(const uint8_t id[128], int rank, int world, int device, hipStream_t s);
// ordered exchange hub (comm_hub.cpp): one transport per process shared by many proofs in flight,
// each context on its own channel (0..63)
struct OrderedHub;
std::shared_ptr<OrderedHub> make_hub(std::unique_ptr<Comm> base);
std::unique_ptr<Comm> make_hub_channel(const std::shared_ptr<OrderedHub>& hub, int channel);
void hub_allgather(OrderedHub& hub, int channel, const void* send, void* recv, size_t bytes);
void hub_stats(OrderedHub& hub, uint64_t out[5]);  // rounds, data rounds, exchanges served, largest batch, idle rounds

// ---------------------------------------------------------------- context
struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    MsmWorkspace* msm = nullptr;
    // second stream + MSM workspace (created on first use): the shared level-0 opening MSM of an
    // index-cached-transcript proof runs there, beside the commitment and the first opening
    hipStream_t side = nullptr;
    MsmWorkspace* msm_side = nullptr;
    hipEvent_t side_ev = nullptr;
    void ensure_side();
    std::unique_ptr<Comm> comm;
    void set_comm(std::unique_ptr<Comm> c) {
        comm = std::move(c);
        knobs_agreed = false;
    }
    // Pinned host staging, one fixed carve-out per context (allocated once, never moved: a region a
    // caller holds stays valid while its async copies run). Every region is reused only after a
    // stream sync that covers the copies issued from it.
    enum : size_t {
        kPinHp = 0,                 // prove(): challenges up, round results down (128 KiB: 8 KiB per proof of a group)
        kPinCommit = 128 << 10,     // commitment MSM result + status (4 KiB)
        kPinLvl0 = 132 << 10,       // shared level-0 opening proof + status (4 KiB)
        kPinOpen = 136 << 10,       // opening results + status / evaluations (56 KiB)
        kPinStage = 192 << 10,      // small host-to-device staging (opening points, constants, a group's challenges) (128 KiB)
        kPinBytes = 320 << 10
    };
    uint8_t* pin = nullptr;
    uint8_t* pin_dev_base = nullptr;  // the carve-out's device address (kernels write round results there)
    template <class T>
    T* pin_dev(const uint8_t* host_ptr) const {
        return reinterpret_cast<T*>(pin_dev_base + (host_ptr - pin));
    }
    uint32_t* ticket = nullptr;  // device counter of the one-launch sumcheck rounds (0 between launches)
    // per-prove scratch (grow-only: no hipMalloc/hipFree, which synchronise the device, while proofs
    // on other contexts are in flight)
    DevMem scratch;
    enum { kSlotCommit, kSlotOpenQ, kSlotOpenA, kSlotOpenB, kSlotOpenOut, kSlotLvl0Q, kSlotLvl0Out, kSlots };
    DevMem slot[kSlots];
    template <class T = void>
    T* buf(int id, size_t bytes) {
        slot[id].ensure(bytes);
        return static_cast<T*>(slot[id].p);
    }
    std::vector<std::pair<std::string, double>> timings;
    KProf kprof;
    uint64_t prove_seq = 0;  // proofs started on this context (identical on every rank of its communicator)
    bool knobs_agreed = false;  // exchange-shaping knobs checked equal across the communicator
    int lvl0_mode = -1;         // shared level-0 opening MSM: 1 inside the first opening's batch, 0 beside
                                // the commitment, -1 the process default (SPX_LVL0=batch -> 1)
    std::atomic<uint64_t> msm_reruns{0};  // MSM batches rerun dense after a compacted-key overflow
    // one prove or round-level session at a time: both own the streams, the scratch tables, the pinned
    // carve-out and the sumcheck ticket (CtxClaim)
    std::atomic<bool> in_use{false};
    Ctx(int dev);
    ~Ctx();
    // region [off, off + bytes) of the pinned carve-out (throws if it does not fit its region)
    uint8_t* pin_at(size_t off, size_t bytes, size_t region);
    // Waits for a stream's queued work. hipStreamSynchronize under the blocking-sync flag still spins
    // in the HSA runtime before it sleeps (~0.2 ms of a core per wait): with 64 proofs in flight per
    // rank and ~45 waits per proof that spinning was most of a proof's host CPU. With SPX_SYNC_POLL_US
    // = t > 0 the wait records an event of the calling thread's own and polls it, sleeping t us between
    // polls (wait_stream).
    // this context's wait: -1 = SPX_SYNC_POLL_US (default 0), 0 = hipStreamSynchronize (atomic: the
    // setter may run beside a worker's waits; spx_ctx_set_sync_poll refuses a context in use)
    std::atomic<int> poll_us{-1};
    // spx_prove_many on this context proves its stubbed-commitment, unsharded proofs in lockstep groups
    // of this many (prove_group; 1 = one at a time)
    std::atomic<int> group{1};
    void wait_stream(hipStream_t s);
    void sync() {  // the main stream's work is done: its MSM staging may be reused
        wait_stream(stream);
        msm_ws_staging_reset(msm);
        if (kprof.on) kprof.harvest();
    }
    void side_sync() {
        if (!side) return;
        wait_stream(side);
        msm_ws_staging_reset(msm_side);
    }
};

// Claims a context for one prove or one round-level session; a second claim while one is held fails
// with SPX_INVALID_ARGUMENT instead of overwriting the holder's device tables.
struct CtxClaim {
    Ctx* c = nullptr;
    CtxClaim() = default;
    explicit CtxClaim(Ctx& C) { take(C); }
    CtxClaim(const CtxClaim&) = delete;
    CtxClaim& operator=(const CtxClaim&) = delete;
    ~CtxClaim() { release(); }
    void take(Ctx& C) {
        bool want = false;
        if (!C.in_use.compare_exchange_strong(want, true))
            throw SpxError(kInvalidArgument, "context is in use by another prove or round-level prover session");
        c = &C;
    }
    void release() {
        if (c) c->in_use.store(false);
        c = nullptr;
    }
};

// ---------------------------------------------------------------- public parameters
struct PP {
    int nv = 0;
    DevMem g1_raw_mem, g2_raw_mem;            // all levels, contiguous
    std::vector<uint64_t> lvl_off;            // point offset of level i (2^(nv-i) points)
    host::Affine<host::Fq> g;
    host::Affine<host::Fq2> h;
    // window copies (device, affine): commit bases (level 0 of G1)
    DevMem g1_pre;
    int g1_c = 0, g1_W = 0;
    // G2 opening bases: level i pair-summed (2^(nv-i-1) points), copies [W_i][size_i]
    DevMem g2_pre;
    std::vector<uint64_t> g2_off;
    std::vector<int> g2_c, g2_W;
    bool has_t = false;
    std::vector<host::Fr> t;  // trapdoor (keygen only; tests)
    G1Aff* g1_level(int i) const { return g1_raw_mem.as<G1Aff>() + lvl_off[i]; }
    G2Aff* g2_level(int i) const { return g2_raw_mem.as<G2Aff>() + lvl_off[i]; }
};
void pp_preprocess(Ctx& C, PP& P);
int window_bits_for(uint64_t size);

// ---------------------------------------------------------------- index
struct HostCsr {
    uint64_t n = 0;
    std::vector<uint64_t> rp;
    std::vector<uint32_t> col;
    std::vector<uint8_t> val;  // canonical bytes
};
struct DevSparse {  // rank-local block of 3 matrices (CSR rows or CSC columns)
    DevMem ptr[3], idx[3], val[3];
    DevMem chunks, lrows;
    int nchunks = 0, nlrows = 0;
    SparseView3 view() const {
        SparseView3 v;
        for (int m = 0; m < 3; ++m) {
            v.ptr[m] = ptr[m].as<uint64_t>();
            v.idx[m] = idx[m].as<uint32_t>();
            v.val[m] = val[m].as<Fr>();
        }
        return v;
    }
};
struct DevSliced {  // rank-local rows of A, B, C as the column-sorted entry list (kernels.hpp: SpmvSlicedView)
    DevMem val, col, dst;
    uint64_t entries = 0;
    bool on = false;  // every local row of every matrix has at most one entry
    SpmvSlicedView view() const { return SpmvSlicedView{val.as<Fr>(), col.as<uint32_t>(), dst.as<uint32_t>()}; }
};
struct DevColStream {  // rank-local columns of A, B, C for eval_on_x (kernels.hpp: ColStreamView)
    DevMem slices, lanes, rowm, val;
    uint32_t nslices = 0;
    DevSparse longc;  // columns of more than kLongCol entries: per-matrix entry arrays + chunks
    uint64_t entries = 0;  // live entries (algorithmic bytes)
    ColStreamView view() const {
        return ColStreamView{slices.as<ColSlice>(), lanes.as<uint32_t>(), rowm.as<uint32_t>(), val.as<Fr>(), nslices};
    }
    // out = sum_m scale[m] M(r_x, .) (eq_scratch: kEqScratch Fr)
    void launch(const Fr* r_x, int L, const Fr* scale, Fr* out, Fr* eq_scratch, Fr* partial, hipStream_t s) const {
        launch_col_stream(view(), r_x, L, scale, out, eq_scratch, longc.view(), longc.chunks.as<LongChunk>(),
                          longc.nchunks, longc.lrows.as<LongRow>(), longc.nlrows, partial, s);
    }
};
struct Index {
    int log_n = 0;
    uint64_t n = 0;
    HostCsr m[3];
    DevSparse rows;      // local rows (SpMV), when rows_sliced is off
    DevSliced rows_sliced;  // local rows as the column-sorted entry list (single-entry rows)
    DevColStream cols;   // local columns (eval_on_x)
    bool has_cache = false;
    Blake2s cache;  // transcript state after feeding A, B, C
    double rows_bytes = 0, cols_bytes = 0;  // algorithmic bytes of one SpMV / eval_on_x pass (local)
    double rows_index_bytes = 0;            // of rows_bytes: the index stream (shared by a lockstep group)
    int G = 1, rank = 0;
};

struct Witness {
    uint64_t n = 0;
    std::vector<uint8_t> v;  // canonical bytes (transcript)
    DevMem z;                // Montgomery, full n
};

struct ProveOpts {
    int mode = 0;
    uint64_t seed = 0;
    bool cached = false;
    bool stub = false;  // BASELINE config C2: commitment and opening proofs = identity, no MSM (pp unused)
    // scheduling hooks used by spx_prove_many (neither changes the proof):
    int64_t seq = -1;                 // proof number deciding which rank absorbs A, B, C (default: ctx counter)
    const Blake2s* absorbed = nullptr;  // this proof's A, B, C absorption, already computed by the caller
    // or, when set, called once the challenge-independent device work (SpMV, commitment MSM, shared
    // level-0 opening MSM) is queued, and returns that absorption (waiting for it if needed)
    std::function<const Blake2s*()> await_absorbed;
    // interactive prove (round-level API, interactive.cpp): messages out, verifier coins in; no
    // Fiat-Shamir absorption at all
    ExternalCoins* coins = nullptr;
    bool claimed = false;  // the caller already holds the context's CtxClaim (a round-level session)
};
// Blake2s state after absorbing A, B, C (lib.rs:61-64): the per-proof sequential host work
Blake2s absorb_matrices(const Index& I);
// the same absorption for k proofs at once (multi-buffer BLAKE2s: k equal states in vector lanes)
void absorb_matrices_lanes(const Index& I, Blake2s* out, int k);

// host CPU of prove()'s phases, process-wide: out[3 i .. 3 i + 2] = CPU ns, wall ns, count of phase i
static constexpr int kHostPhases = 7;
void host_phase_stats(uint64_t* out);

// entry points used by the C ABI
std::unique_ptr<PP> pp_load(Ctx& C, const uint8_t* b, size_t len);
std::unique_ptr<PP> pp_generate(Ctx& C, int nv, uint64_t seed);
std::vector<uint8_t> pp_serialize(Ctx& C, const PP& P);
std::unique_ptr<Index> index_build(Ctx& C, const HostCsr* mats);
std::unique_ptr<Witness> witness_upload(Ctx& C, const uint8_t* v, size_t nv, const uint8_t* w, size_t nw);
// P may be null only when o.stub
std::vector<uint8_t> prove(Ctx& C, Index& I, Witness& W, PP* P, const ProveOpts& o);
// k (<= kGroupMax) proofs of one index in lockstep (BASELINE C2's form: commitment stubbed, one rank):
// the same steps as prove() for each, with every sumcheck round of the k proofs in one launch and one
// host wait, and the other steps' launches of the k proofs queued back to back before one wait. Each
// proof's bytes equal its own prove()'s; o[j] are proof j's options (all stubbed, none interactive).
std::vector<std::vector<uint8_t>> prove_group(Ctx& C, Index& I, Witness* const* W, int k, const ProveOpts* o);
size_t proof_size(int log_n);

// verifier (lib.rs:147-212 with verifier.rs:143-512); VerifierParameter: data_structures.rs:19-26
struct VP {
    int nv = 0;
    host::Affine<host::Fq> g;
    host::Affine<host::Fq2> h;
    std::vector<host::Affine<host::Fq>> g_mask;  // g^{t_i}
};
VP vp_load(const uint8_t* b, size_t len);
std::vector<uint8_t> vp_serialize(const VP& V);
VP vp_from_pp(const PP& P);  // keygen-generated PP only (keeps the trapdoor)
// throws SpxError(kInvalidArgument / kSumcheck / kWrongWitness / kSerialization) on rejection, as the
// reference's Err(...); returns normally on acceptance (Ok(true))
void verify(Ctx& C, Index& I, const uint8_t* v, size_t nv, const uint8_t* proof, size_t len, const VP& V,
            const ProveOpts& o);

std::vector<uint8_t> k_sum_over_y(Ctx& C, const HostCsr& m, const uint8_t* z);
std::vector<uint8_t> k_eval_on_x(Ctx& C, const HostCsr& m, const uint8_t* r_x);
void k_sumcheck_round(Ctx& C, const uint8_t* f, const uint8_t* g, uint64_t n, const uint8_t* r_prev,
                      uint8_t* evals_out, uint8_t* f_out, uint8_t* g_out);
std::vector<uint8_t> k_msm(Ctx& C, bool g2, const uint8_t* bases, const uint8_t* scalars, size_t n);
std::vector<uint8_t> k_commit(Ctx& C, PP& P, const uint8_t* table, int nv);
std::vector<uint8_t> k_open(Ctx& C, PP& P, const uint8_t* table, int nv, const uint8_t* point);

}  // namespace spx
