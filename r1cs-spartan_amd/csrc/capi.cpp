// extern "C" boundary (include/spartan_hip.h). Exceptions never cross it: every entry point
// maps them to an spx_status and a thread-local message (the reference's Error::Display is
// todo!(), /root/reference/src/error.rs:23-27).
#include "../../include/spartan_hip.h"

#include <atomic>
#include <chrono>
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <condition_variable>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "hash_sched.hpp"
#include "interactive.hpp"
#include "pairing.hpp"
#include "prover.hpp"

extern "C" int spx_comm_unique_id_impl(uint8_t out[128]);

struct spx_ctx {
    std::unique_ptr<spx::Ctx> c;
};
struct spx_pp {
    spx_ctx* ctx;
    std::unique_ptr<spx::PP> p;
};
struct spx_pk {
    spx_ctx* ctx;
    std::unique_ptr<spx::Index> i;
};
struct spx_witness {
    spx_ctx* ctx;
    std::unique_ptr<spx::Witness> w;
};
struct spx_prover {
    spx_ctx* ctx;
    std::unique_ptr<spx::Interactive> s;
};

namespace {
thread_local std::string g_err;
// host time spent absorbing A, B, C in spx_prove_many's hashing pools, and the proofs absorbed
std::atomic<uint64_t> g_hash_ns{0}, g_hash_proofs{0}, g_hash_wait_ns{0};
template <class F>
int guard(F&& f) {
    try {
        f();
        g_err.clear();
        return SPX_OK;
    } catch (const spx::SpxError& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "out of memory";
        return SPX_DEVICE;
    } catch (const std::exception& e) {
        g_err = e.what();
        return SPX_DEVICE;
    }
}
spx::HostCsr to_host(const spx_csr* m) {
    if (!m || !m->row_ptr) spx::invalid("null matrix");
    spx::HostCsr h;
    h.n = m->n;
    h.rp.assign(m->row_ptr, m->row_ptr + m->n + 1);
    const uint64_t nnz = h.rp[m->n];
    if (nnz && (!m->col || !m->val)) spx::invalid("null matrix arrays");
    h.col.assign(m->col, m->col + nnz);
    h.val.assign(m->val, m->val + 32 * nnz);
    return h;
}
void set_dev(spx_ctx* c) {
    if (!c) spx::invalid("null context");
    SPX_HIP(hipSetDevice(c->c->device));
    spx::g_kprof = &c->c->kprof;  // kernel statistics of this ctx for the calling thread
}
spx::ProveOpts opts_of(const spx_prove_opts* o) {
    spx::ProveOpts p;
    if (o) {
        if (o->mode != SPX_FS && o->mode != SPX_INJECTED) spx::invalid("bad mode");
        p.mode = o->mode;
        p.seed = o->inj_seed;
        p.cached = o->cached_matrix_transcript != 0;
        p.stub = o->commitment_stub != 0;
    }
    return p;
}
spx::PP* pp_of(spx_pp* pp, const spx::ProveOpts& o) {
    if (pp) return pp->p.get();
    if (!o.stub) spx::invalid("null public parameter");
    return nullptr;
}
int copy_out(const std::vector<uint8_t>& v, uint8_t* out, size_t cap, size_t* len) {
    if (len) *len = v.size();
    if (out) {
        if (cap < v.size()) spx::invalid("output buffer too small");
        memcpy(out, v.data(), v.size());
    }
    return 0;
}
template <class F>
int prover_step(spx_prover* p, uint8_t* msg, size_t cap, size_t* len, F&& f) {
    return guard([&] {
        if (!p) spx::invalid("null prover");
        set_dev(p->ctx);
        copy_out(f(*p->s), msg, cap, len);
    });
}
spx::PP* need_pp(spx_pp* pp) {
    if (!pp) spx::invalid("null public parameter");
    return pp->p.get();
}
}  // namespace

extern "C" {

const char* spx_last_error(void) { return g_err.c_str(); }
const char* spx_version(void) { return "spartan_hip 0.1 (gfx950)"; }

int spx_ctx_create(int device, spx_ctx** out) {
    return guard([&] {
        if (!out) spx::invalid("null out");
        int ndev = 0;
        SPX_HIP(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) spx::invalid("no such HIP device");
        auto* c = new spx_ctx();
        c->c.reset(new spx::Ctx(device));
        *out = c;
    });
}
int spx_ctx_destroy(spx_ctx* ctx) {
    return guard([&] { delete ctx; });
}
int spx_comm_unique_id(uint8_t id_out[128]) {
    return guard([&] {
        if (spx_comm_unique_id_impl(id_out)) throw spx::SpxError(spx::kDevice, "ncclGetUniqueId failed");
    });
}
int spx_ctx_set_comm_rccl(spx_ctx* ctx, const uint8_t id[128], int rank, int world) {
    return guard([&] {
        set_dev(ctx);
        if (world < 1 || rank < 0 || rank >= world) spx::invalid("bad rank / world");
        // a private hub on channel 0: the same ordered path as spx_comm_hub_create_rccl
        ctx->c->set_comm(spx::make_hub_channel(spx::make_hub(spx::make_rccl_comm(id, rank, world, ctx->c->device, nullptr)), 0));
    });
}
int spx_ctx_set_comm_shm(spx_ctx* ctx, const char* name, int rank, int world) {
    return guard([&] {
        if (!ctx) spx::invalid("null context");
        ctx->c->set_comm(spx::make_shm_comm(name, rank, world));
    });
}
int spx_comm_shm_create(const char* name, int rank, int world, void** comm_out) {
    return guard([&] {
        if (!comm_out) spx::invalid("null output");
        *comm_out = spx::make_shm_comm(name, rank, world).release();
    });
}
int spx_comm_shm_allgather(void* comm, const void* send, void* recv, size_t bytes) {
    return guard([&] {
        if (!comm || (bytes && (!send || !recv))) spx::invalid("null argument");
        static_cast<spx::Comm*>(comm)->allgather(send, recv, bytes);
    });
}
int spx_comm_shm_destroy(void* comm) {
    return guard([&] { delete static_cast<spx::Comm*>(comm); });
}
int spx_comm_group_create(int world, void** group_out) {
    return guard([&] {
        if (world < 1) spx::invalid("bad world");
        *group_out = new std::shared_ptr<spx::GroupState>(std::make_shared<spx::GroupState>(world));
    });
}
int spx_comm_group_destroy(void* group) {
    return guard([&] { delete static_cast<std::shared_ptr<spx::GroupState>*>(group); });
}
int spx_ctx_set_comm_group(spx_ctx* ctx, void* group, int rank) {
    return guard([&] {
        auto& st = *static_cast<std::shared_ptr<spx::GroupState>*>(group);
        if (rank < 0 || rank >= st->world) spx::invalid("bad rank");
        ctx->c->set_comm(std::unique_ptr<spx::Comm>(new spx::GroupComm(st, rank)));
    });
}

// ordered exchange hubs: a handle owns a shared_ptr; contexts attached to it keep it alive
int spx_comm_hub_create_rccl(const uint8_t id[128], int rank, int world, int device, void** hub_out) {
    return guard([&] {
        if (!hub_out || !id) spx::invalid("null argument");
        if (world < 1 || rank < 0 || rank >= world) spx::invalid("bad rank / world");
        *hub_out = new std::shared_ptr<spx::OrderedHub>(spx::make_hub(spx::make_rccl_comm(id, rank, world, device, nullptr)));
    });
}
int spx_comm_hub_create_shm(const char* name, int rank, int world, void** hub_out) {
    return guard([&] {
        if (!hub_out) spx::invalid("null output");
        *hub_out = new std::shared_ptr<spx::OrderedHub>(spx::make_hub(spx::make_shm_comm(name, rank, world)));
    });
}
namespace spx {
// a caller-provided allgather (spx_comm_hub_create_callback)
struct CallbackComm : Comm {
    spx_allgather_fn fn;
    void* user;
    int r, w;
    CallbackComm(spx_allgather_fn f, void* u, int rank, int world) : fn(f), user(u), r(rank), w(world) {}
    int rank() const override { return r; }
    int size() const override { return w; }
    void allgather(const void* s, void* rv, size_t b) override {
        const int rc = fn(user, s, rv, b);
        if (rc != 0) throw SpxError(kDevice, "caller-provided allgather failed (" + std::to_string(rc) + ")");
    }
};
}  // namespace spx
int spx_comm_hub_create_callback(spx_allgather_fn fn, void* user, int rank, int world, void** hub_out) {
    return guard([&] {
        if (!hub_out || !fn) spx::invalid("null argument");
        if (world < 1 || rank < 0 || rank >= world) spx::invalid("bad rank / world");
        *hub_out = new std::shared_ptr<spx::OrderedHub>(
            spx::make_hub(std::unique_ptr<spx::Comm>(new spx::CallbackComm(fn, user, rank, world))));
    });
}
int spx_comm_hub_create_group(void* group, int rank, void** hub_out) {
    return guard([&] {
        if (!hub_out || !group) spx::invalid("null argument");
        auto& st = *static_cast<std::shared_ptr<spx::GroupState>*>(group);
        if (rank < 0 || rank >= st->world) spx::invalid("bad rank");
        *hub_out = new std::shared_ptr<spx::OrderedHub>(spx::make_hub(std::unique_ptr<spx::Comm>(new spx::GroupComm(st, rank))));
    });
}
int spx_comm_hub_allgather(void* hub, int channel, const void* send, void* recv, size_t bytes) {
    return guard([&] {
        if (!hub || (bytes && (!send || !recv))) spx::invalid("null argument");
        spx::hub_allgather(**static_cast<std::shared_ptr<spx::OrderedHub>*>(hub), channel, send, recv, bytes);
    });
}
int spx_comm_hub_stats(void* hub, uint64_t out[5]) {
    return guard([&] {
        if (!hub || !out) spx::invalid("null argument");
        spx::hub_stats(**static_cast<std::shared_ptr<spx::OrderedHub>*>(hub), out);
    });
}
int spx_comm_hub_destroy(void* hub) {
    return guard([&] { delete static_cast<std::shared_ptr<spx::OrderedHub>*>(hub); });
}
int spx_ctx_set_comm_hub(spx_ctx* ctx, void* hub, int channel) {
    return guard([&] {
        if (!ctx || !hub) spx::invalid("null argument");
        ctx->c->set_comm(spx::make_hub_channel(*static_cast<std::shared_ptr<spx::OrderedHub>*>(hub), channel));
    });
}

int spx_ctx_set_comm_rehearsal(spx_ctx* ctx, int rank, int world) {
    return guard([&] {
        if (!ctx) spx::invalid("null context");
        if (world < 1 || rank < 0 || rank >= world) spx::invalid("bad rank / world");
        ctx->c->set_comm(std::unique_ptr<spx::Comm>(new spx::SoloComm(rank, world)));
    });
}

int spx_ctx_set_lvl0_batch(spx_ctx* ctx, int mode) {
    return guard([&] {
        if (!ctx) spx::invalid("null context");
        if (mode < -1 || mode > 1) spx::invalid("level-0 mode must be -1, 0 or 1");
        ctx->c->lvl0_mode = mode;
        ctx->c->knobs_agreed = false;
    });
}

int spx_ctx_comm_allgather(spx_ctx* ctx, const void* send, void* recv, size_t bytes) {
    return guard([&] {
        set_dev(ctx);
        if (bytes && (!send || !recv)) spx::invalid("null argument");
        ctx->c->comm->allgather(send, recv, bytes);
    });
}

int spx_pp_load(spx_ctx* ctx, const uint8_t* bytes, size_t len, spx_pp** out) {
    return guard([&] {
        set_dev(ctx);
        auto* p = new spx_pp{ctx, spx::pp_load(*ctx->c, bytes, len)};
        *out = p;
    });
}
int spx_pp_generate(spx_ctx* ctx, int nv, uint64_t seed, spx_pp** out) {
    return guard([&] {
        set_dev(ctx);
        auto* p = new spx_pp{ctx, spx::pp_generate(*ctx->c, nv, seed)};
        *out = p;
    });
}
int spx_pp_serialize(spx_pp* pp, uint8_t* out, size_t cap, size_t* len) {
    return guard([&] {
        set_dev(pp->ctx);
        copy_out(spx::pp_serialize(*pp->ctx->c, *pp->p), out, cap, len);
    });
}
int spx_pp_free(spx_pp* pp) {
    return guard([&] {
        if (pp) set_dev(pp->ctx);
        delete pp;
    });
}

int spx_index(spx_ctx* ctx, const spx_csr* a, const spx_csr* b, const spx_csr* c, spx_pk** out) {
    return guard([&] {
        set_dev(ctx);
        spx::HostCsr m[3] = {to_host(a), to_host(b), to_host(c)};
        *out = new spx_pk{ctx, spx::index_build(*ctx->c, m)};
    });
}
int spx_index_free(spx_pk* idx) {
    return guard([&] {
        if (idx) set_dev(idx->ctx);
        delete idx;
    });
}
int spx_witness_upload(spx_ctx* ctx, const uint8_t* v, size_t nv, const uint8_t* w, size_t nw, spx_witness** out) {
    return guard([&] {
        set_dev(ctx);
        *out = new spx_witness{ctx, spx::witness_upload(*ctx->c, v, nv, w, nw)};
    });
}
int spx_witness_free(spx_witness* wit) {
    return guard([&] {
        if (wit) set_dev(wit->ctx);
        delete wit;
    });
}
size_t spx_proof_size(int log_n, int /*log_v*/) { return spx::proof_size(log_n); }

int spx_prove(spx_ctx* ctx, spx_pk* idx, const uint8_t* v, size_t nv, const uint8_t* w, size_t nw, spx_pp* pp,
              const spx_prove_opts* opts, uint8_t* out, size_t cap, size_t* len) {
    return guard([&] {
        set_dev(ctx);
        if (!idx) spx::invalid("null prover key");
        const spx::ProveOpts o = opts_of(opts);
        spx::PP* P = pp_of(pp, o);
        auto W = spx::witness_upload(*ctx->c, v, nv, w, nw);
        copy_out(spx::prove(*ctx->c, *idx->i, *W, P, o), out, cap, len);
    });
}
// ---- round-level prover (interactive.cpp; prover.rs:109-281)
int spx_prover_init(spx_ctx* ctx, spx_pk* idx, const uint8_t* v, size_t nv, const uint8_t* w, size_t nw,
                    spx_prover** out) {
    return guard([&] {
        set_dev(ctx);
        if (!idx || !out) spx::invalid("null prover key / out");
        if (!spx::is_pow2(nv)) spx::invalid("public input should be power of two");  // prover.rs:114-116
        if (nv + nw != idx->i->n) spx::invalid("|v| + |w| != number of variables");  // prover.rs:117-119
        // a session freed mid-way cancels its worker at its next coin; on a sharded context the peer
        // ranks would then wait in their next exchange with no error, so sessions are unsharded
        if (ctx->c->comm->size() > 1) spx::invalid("round-level prover sessions need an unsharded context (comm size 1)");
        auto W = spx::witness_upload(*ctx->c, v, nv, w, nw);
        *out = new spx_prover{ctx, std::make_unique<spx::Interactive>(*ctx->c, *idx->i, std::move(W))};
    });
}
int spx_prover_free(spx_prover* p) {
    return guard([&] { delete p; });
}
int spx_prover_first_round(spx_prover* p, spx_pp* pp, uint8_t* msg, size_t cap, size_t* len) {
    return prover_step(p, msg, cap, len, [&](spx::Interactive& s) { return s.first_round(need_pp(pp)); });
}
int spx_prover_second_round(spx_prover* p, const uint8_t* r_v, size_t n, spx_pp* pp, uint8_t* msg, size_t cap,
                            size_t* len) {
    return prover_step(p, msg, cap, len, [&](spx::Interactive& s) { return s.second_round(r_v, n, need_pp(pp)); });
}
int spx_prover_third_round(spx_prover* p, const uint8_t* tau, size_t n, uint8_t* msg, size_t cap, size_t* len) {
    return prover_step(p, msg, cap, len, [&](spx::Interactive& s) { return s.third_round(tau, n); });
}
int spx_prove_first_sumcheck_round(spx_prover* p, const uint8_t* challenge, uint8_t* msg, size_t cap, size_t* len) {
    return prover_step(p, msg, cap, len,
                       [&](spx::Interactive& s) { return s.sumcheck_round(spx::Interactive::kSumcheck1, challenge); });
}
int spx_prove_fourth_round(spx_prover* p, const uint8_t* last_point, uint8_t* msg, size_t cap, size_t* len) {
    return prover_step(p, msg, cap, len, [&](spx::Interactive& s) { return s.fourth_round(last_point); });
}
int spx_prove_fifth_round(spx_prover* p, const uint8_t* r_abc, uint8_t* msg, size_t cap, size_t* len) {
    return prover_step(p, msg, cap, len, [&](spx::Interactive& s) { return s.fifth_round(r_abc); });
}
int spx_prove_second_sumcheck_round(spx_prover* p, const uint8_t* challenge, uint8_t* msg, size_t cap, size_t* len) {
    return prover_step(p, msg, cap, len,
                       [&](spx::Interactive& s) { return s.sumcheck_round(spx::Interactive::kSumcheck2, challenge); });
}
int spx_prove_sixth_round(spx_prover* p, const uint8_t* last_point, spx_pp* pp, uint8_t* msg, size_t cap, size_t* len) {
    return prover_step(p, msg, cap, len, [&](spx::Interactive& s) { return s.sixth_round(last_point, need_pp(pp)); });
}

int spx_prove_witness(spx_ctx* ctx, spx_pk* idx, spx_witness* wit, spx_pp* pp, const spx_prove_opts* opts,
                      uint8_t* out, size_t cap, size_t* len) {
    return guard([&] {
        set_dev(ctx);
        if (!idx || !wit) spx::invalid("null prover key / witness");
        const spx::ProveOpts o = opts_of(opts);
        copy_out(spx::prove(*ctx->c, *idx->i, *wit->w, pp_of(pp, o), o), out, cap, len);
    });
}
int spx_prove_many(spx_ctx** ctxs, int nctx, spx_pk* idx, spx_witness** wits, int nproofs, spx_pp* pp,
                   const spx_prove_opts* opts, uint8_t* out, size_t stride, size_t* lens) {
    if (!ctxs || nctx < 1 || !idx || !wits || nproofs < 0 || !out || !lens) {
        g_err = "spx_prove_many: bad arguments";
        return SPX_INVALID_ARGUMENT;
    }
    for (int k = 0; k < nctx; ++k)
        if (!ctxs[k]) {
            g_err = "spx_prove_many: null context";
            return SPX_INVALID_ARGUMENT;
        }
    for (int i = 0; i < nproofs; ++i)
        if (!wits[i]) {
            g_err = "spx_prove_many: null witness";
            return SPX_INVALID_ARGUMENT;
        }
    spx::ProveOpts base;
    spx::PP* P = nullptr;
    try {
        base = opts_of(opts);
        P = pp_of(pp, base);
    } catch (const spx::SpxError& e) {
        g_err = e.what();
        return e.code;
    }
    // Proof i is absorbed (A, B, C into its transcript) by rank i mod G, on a pool of host threads
    // that runs ahead of the GPU workers: the sequential ~150 MB Blake2s pass of each proof overlaps
    // the device work of earlier proofs instead of sitting in front of its own. Every proof is still
    // absorbed exactly once; only the schedule changes.
    const int G = ctxs[0]->c->comm->size(), rank = ctxs[0]->c->comm->rank();
    struct Slot {
        std::atomic<int> state{0};  // 0 pending, 1 ready, 2 failed
        spx::Blake2s h;
    };
    std::vector<Slot> slots(base.cached ? 0 : nproofs);
    std::vector<int> owned;
    if (!base.cached)
        for (int i = 0; i < nproofs; ++i)
            if (i % G == rank) owned.push_back(i);
    std::mutex mu;
    std::condition_variable cv;
    std::string pool_err;
    // A job absorbs A, B, C for `lanes` consecutive proofs at once: multi-buffer BLAKE2s, one proof's
    // state per vector lane (blake2s_lanes.cpp; 16 lanes with AVX-512, 8 with AVX2). Every proof's
    // transcript still absorbs the matrices itself (lib.rs:61-64); the lanes share the instructions.
    // Schedule (hash_sched.hpp). The first in-flight proofs wait for their absorption before their
    // first challenge: one scalar absorption takes 0.15-0.17 s, a full-width job ~0.3 s at best, so
    // with full-width jobs from the start the early waves of proofs waited for theirs (34 ms per proof
    // and 56.2 vs 59.6-60.3 M constraints/s for an all-scalar pool; profiles/r04/r04u_ab_hash_wait.jsonl).
    // The first two waves are scalar; a few full-width jobs for the next waves start beside them. With
    // the commitment stubbed (C2), all full width: 277 -> 370 M constraints/s at 2^18 in the same A/B
    // (profiles/r04/r04ae_ab_c2_schedule.jsonl).
    // Pool size: the hashers run ahead as fast as they can, so a pool larger than the cores it needs
    // starves the proof threads of their host work (solo G = 8 rank, 64 in flight on 16 cores: 64
    // hashers 332 M, 8 hashers 381 M constraints/s; profiles/r03/r03am_hash_threads.jsonl). A rank of a
    // G-rank proof absorbs 1/G of the proofs: half the core budget for G >= 4, all of it otherwise.
    // Budget: SPX_HASH_THREADS, else OMP_NUM_THREADS (the box's CPU share), else the hardware threads.
    int budget = (int)std::thread::hardware_concurrency();
    if (const char* e = getenv("OMP_NUM_THREADS")) budget = atoi(e);
    budget = std::max(1, budget);
    // proofs in flight: one per context, or its lockstep group (spx_ctx_set_group) for stubbed proofs
    int nfly = 0;
    for (int k = 0; k < nctx; ++k) nfly += (base.stub && G == 1) ? std::max(1, ctxs[k]->c->group.load()) : 1;
    const int nbase = std::min(nfly, G >= 4 ? std::max(1, budget / 2) : budget);
    const int lanes = std::max(1, spx::blake2s_lane_width());
    using clk = std::chrono::steady_clock;
    // SPX_HASH_THREADS replaces the pool size (lead jobs included) and with it the scalar cap
    int nh_env = 0;
    if (const char* e = getenv("SPX_HASH_THREADS")) nh_env = std::max(1, atoi(e));
    const size_t nsize = nh_env ? (size_t)nh_env : (size_t)nbase + spx::HashSched::kLead;
    spx::HashSched sched(owned.size(), (size_t)(nfly + G - 1) / G, lanes, base.stub ? 0 : 2,
                         2 * (size_t)(nh_env ? nh_env : nbase), nsize);
    const size_t njobs = sched.size();
    auto hasher = [&] {
        std::vector<spx::Blake2s> tmp(lanes);
        for (;;) {
            const size_t j = sched.claim();
            if (j >= njobs) return;
            const size_t b = sched.jobs[j].first, e = sched.jobs[j].second;
            int st = 1;
            try {
                const auto t0 = clk::now();
                spx::absorb_matrices_lanes(*idx->i, tmp.data(), (int)(e - b));
                for (size_t i = b; i < e; ++i) slots[owned[i]].h = tmp[i - b];
                g_hash_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
                g_hash_proofs += e - b;
            } catch (const std::exception& ex) {
                std::lock_guard<std::mutex> lk(mu);
                pool_err = ex.what();
                st = 2;
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                for (size_t i = b; i < e; ++i) slots[owned[i]].state.store(st);
            }
            cv.notify_all();
        }
    };
    int nh = nh_env ? nh_env : nbase + (int)sched.nlead;
    nh = std::min<int>(nh, (int)njobs);
    std::vector<std::thread> pool;
    for (int t = 0; t < nh; ++t) pool.emplace_back(hasher);

    std::vector<int> st(nctx, SPX_OK);
    std::vector<std::string> msg(nctx);
    auto opts_for = [&](int i) {
        spx::ProveOpts o = base;
        o.seq = i;
        if (!base.cached && i % G == rank)  // waited for inside prove, behind the proof's first kernels
            o.await_absorbed = [&, i]() -> const spx::Blake2s* {
                const auto w0 = clk::now();
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return slots[i].state.load() != 0; });
                g_hash_wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - w0).count();
                if (slots[i].state.load() == 2)
                    throw spx::SpxError(spx::kDevice, "absorption failed: " + pool_err);
                return &slots[i].h;
            };
        return o;
    };
    auto emit = [&](int i, const std::vector<uint8_t>& p) {
        if (p.size() > stride) spx::invalid("proof buffer too small");
        memcpy(out + (size_t)i * stride, p.data(), p.size());
        lens[i] = p.size();
    };
    auto work = [&](int k) {
        // lockstep groups (spx_ctx_set_group): the context's proofs k, k + nctx, ... in groups of K
        const int K = ctxs[k]->c->group.load();
        const bool grouped = K > 1 && base.stub && G == 1;
        std::vector<int> mine;
        for (int i = k; i < nproofs; i += nctx) mine.push_back(i);
        for (size_t a = 0; a < mine.size(); a += grouped ? (size_t)K : 1) {
            int rc = guard([&] {
                set_dev(ctxs[k]);
                if (!grouped) {
                    const int i = mine[a];
                    emit(i, spx::prove(*ctxs[k]->c, *idx->i, *wits[i]->w, P, opts_for(i)));
                    return;
                }
                const int cnt = (int)std::min<size_t>((size_t)K, mine.size() - a);
                std::vector<spx::ProveOpts> os;
                std::vector<spx::Witness*> ws;
                for (int q = 0; q < cnt; ++q) {
                    os.push_back(opts_for(mine[a + q]));
                    ws.push_back(wits[mine[a + q]]->w.get());
                }
                auto ps = spx::prove_group(*ctxs[k]->c, *idx->i, ws.data(), cnt, os.data());
                for (int q = 0; q < cnt; ++q) emit(mine[a + q], ps[q]);
            });
            if (rc != SPX_OK) {
                st[k] = rc;
                msg[k] = g_err;
                return;
            }
        }
    };
    const int nw = std::min(nctx, std::max(nproofs, 1));
    std::vector<std::thread> th;
    for (int k = 1; k < nw; ++k) th.emplace_back(work, k);
    work(0);
    for (auto& t : th) t.join();
    sched.stop();  // stop a pool still running after a worker failure
    for (auto& t : pool) t.join();
    for (int k = 0; k < nw; ++k)
        if (st[k] != SPX_OK) {
            g_err = msg[k];
            return st[k];
        }
    g_err.clear();
    return SPX_OK;
}
int spx_hash_stats(uint64_t out[4]) {
    return guard([&] {
        if (!out) spx::invalid("null argument");
        out[0] = g_hash_ns.load();
        out[1] = g_hash_proofs.load();
        out[2] = (uint64_t)std::max(1, spx::blake2s_lane_width());
        out[3] = g_hash_wait_ns.load();
    });
}
int spx_host_phase_stats(uint64_t out[21]) {
    return guard([&] {
        if (!out) spx::invalid("null argument");
        spx::host_phase_stats(out);
    });
}
int spx_vp_from_pp(spx_pp* pp, uint8_t* out, size_t cap, size_t* len) {
    return guard([&] {
        if (!pp) spx::invalid("null public parameter");
        copy_out(spx::vp_serialize(spx::vp_from_pp(*pp->p)), out, cap, len);
    });
}
int spx_verify(spx_ctx* ctx, spx_pk* idx, const uint8_t* v, size_t nv, const uint8_t* proof, size_t len,
               const uint8_t* vp, size_t vp_len, const spx_prove_opts* opts) {
    return guard([&] {
        if (!idx || (nv && !v) || (len && !proof) || !vp) spx::invalid("null argument");
        set_dev(ctx);
        spx::CtxClaim claim(*ctx->c);
        spx::verify(*ctx->c, *idx->i, v, nv, proof, len, spx::vp_load(vp, vp_len), opts_of(opts));
    });
}
int spx_pairing_check(const uint8_t* g1, const uint8_t* g2, size_t n, int* is_one) {
    return guard([&] {
        if ((n && (!g1 || !g2)) || !is_one) spx::invalid("null argument");
        std::vector<std::pair<spx::host::Affine<spx::host::Fq>, spx::host::Affine<spx::host::Fq2>>> pairs(n);
        for (size_t i = 0; i < n; ++i)
            if (!spx::host::g1_from_uncompressed(pairs[i].first, g1 + 96 * i) ||
                !spx::host::g2_from_uncompressed(pairs[i].second, g2 + 192 * i))
                throw spx::SpxError(spx::kSerialization, "bad point encoding");
        *is_one = spx::host::pairing_product_is_one(pairs) ? 1 : 0;
    });
}
int spx_last_timings(spx_ctx* ctx, double* out, int cap, int* n) {
    return guard([&] {
        auto& t = ctx->c->timings;
        if (n) *n = (int)t.size();
        for (int i = 0; i < (int)t.size() && i < cap; ++i) out[i] = t[i].second;
    });
}

int spx_kernel_stats_enable(spx_ctx* ctx, int on) {
    return guard([&] {
        set_dev(ctx);
        ctx->c->sync();
        ctx->c->kprof.on = on != 0;
        ctx->c->kprof.reset();
    });
}
int spx_kernel_stats(spx_ctx* ctx, int id, uint64_t* launches, double* ms, double* bytes) {
    return guard([&] {
        if (id < 0 || id >= SPX_K_COUNT) spx::invalid("bad kernel id");
        set_dev(ctx);
        ctx->c->sync();
        auto& k = ctx->c->kprof;
        if (launches) *launches = k.launches[id];
        if (ms) *ms = k.ms[id];
        if (bytes) *bytes = k.bytes[id];
    });
}

int spx_kernel_stats_largest(spx_ctx* ctx, int id, uint64_t* launches, double* ms, double* bytes) {
    return guard([&] {
        if (id < 0 || id >= SPX_K_COUNT) spx::invalid("bad kernel id");
        set_dev(ctx);
        ctx->c->sync();
        auto& k = ctx->c->kprof;
        if (launches) *launches = k.big_launches[id];
        if (ms) *ms = k.big_ms[id];
        if (bytes) *bytes = k.big_bytes[id];
    });
}
int spx_kernel_ops(spx_ctx* ctx, int id, double* ops) {
    return guard([&] {
        if (id < 0 || id >= SPX_K_COUNT) spx::invalid("bad kernel id");
        set_dev(ctx);
        ctx->c->sync();
        if (ops) *ops = ctx->c->kprof.ops[id];
    });
}
int spx_ctx_set_sync_poll(spx_ctx* ctx, int us) {
    return guard([&] {
        if (!ctx) spx::invalid("null context");
        if (ctx->c->in_use.load()) spx::invalid("context in use by a prove or session");
        ctx->c->poll_us = us < 0 ? -1 : us;
    });
}
int spx_ctx_set_group(spx_ctx* ctx, int k) {
    return guard([&] {
        if (!ctx) spx::invalid("null context");
        if (k < 1 || k > spx::kGroupMax) spx::invalid("lockstep group size must be 1.." + std::to_string(spx::kGroupMax));
        if (ctx->c->in_use.load()) spx::invalid("context in use by a prove or session");
        ctx->c->group = k;
    });
}
int spx_ctx_mem_info(spx_ctx* ctx, uint64_t* free_bytes, uint64_t* total_bytes) {
    return guard([&] {
        if (!free_bytes || !total_bytes) spx::invalid("null argument");
        set_dev(ctx);
        size_t f = 0, t = 0;
        SPX_HIP(hipMemGetInfo(&f, &t));
        *free_bytes = f;
        *total_bytes = t;
    });
}
int spx_msm_reruns(spx_ctx* ctx, uint64_t* reruns) {
    return guard([&] {
        if (!ctx || !reruns) spx::invalid("null argument");
        *reruns = ctx->c->msm_reruns.load();
    });
}
int spx_sum_over_y(spx_ctx* ctx, const spx_csr* m, const uint8_t* z, uint8_t* out) {
    return guard([&] {
        set_dev(ctx);
        spx::CtxClaim claim(*ctx->c);
        auto r = spx::k_sum_over_y(*ctx->c, to_host(m), z);
        memcpy(out, r.data(), r.size());
    });
}
int spx_eval_on_x(spx_ctx* ctx, const spx_csr* m, const uint8_t* r_x, uint8_t* out) {
    return guard([&] {
        set_dev(ctx);
        spx::CtxClaim claim(*ctx->c);
        auto r = spx::k_eval_on_x(*ctx->c, to_host(m), r_x);
        memcpy(out, r.data(), r.size());
    });
}
int spx_sumcheck_round(spx_ctx* ctx, const uint8_t* f, const uint8_t* g, size_t n, const uint8_t* r_prev,
                       uint8_t* evals_out, uint8_t* f_out, uint8_t* g_out) {
    return guard([&] {
        set_dev(ctx);
        if (!f || !g || !evals_out) spx::invalid("null argument");
        spx::CtxClaim claim(*ctx->c);
        spx::k_sumcheck_round(*ctx->c, f, g, n, r_prev, evals_out, f_out, g_out);
    });
}
int spx_msm_g1(spx_ctx* ctx, const uint8_t* bases, const uint8_t* scalars, size_t n, uint8_t* out96) {
    return guard([&] {
        set_dev(ctx);
        spx::CtxClaim claim(*ctx->c);
        auto r = spx::k_msm(*ctx->c, false, bases, scalars, n);
        memcpy(out96, r.data(), r.size());
    });
}
int spx_msm_g2(spx_ctx* ctx, const uint8_t* bases, const uint8_t* scalars, size_t n, uint8_t* out192) {
    return guard([&] {
        set_dev(ctx);
        spx::CtxClaim claim(*ctx->c);
        auto r = spx::k_msm(*ctx->c, true, bases, scalars, n);
        memcpy(out192, r.data(), r.size());
    });
}
int spx_commit(spx_ctx* ctx, spx_pp* pp, const uint8_t* table, int nv, uint8_t* out56) {
    return guard([&] {
        set_dev(ctx);
        spx::CtxClaim claim(*ctx->c);
        auto r = spx::k_commit(*ctx->c, *pp->p, table, nv);
        memcpy(out56, r.data(), r.size());
    });
}
int spx_open(spx_ctx* ctx, spx_pp* pp, const uint8_t* table, int nv, const uint8_t* point, uint8_t* eval_out,
             uint8_t* proof_out) {
    return guard([&] {
        set_dev(ctx);
        spx::CtxClaim claim(*ctx->c);
        auto r = spx::k_open(*ctx->c, *pp->p, table, nv, point);
        memcpy(eval_out, r.data(), 32);
        memcpy(proof_out, r.data() + 32, r.size() - 32);
    });
}

}  // extern "C"
