// Kernel-launch interface shared by the device translation units and the host prover.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "curve_dev.hpp"

namespace spx {

// rows longer than this go to the chunked long-row path (nnz skew, e.g. the dense row of
// the reference's TestSynthesizer at density 0, constraints.rs:77-88)
static constexpr uint64_t kLongRow = 64;
static constexpr uint64_t kChunk = 4096;

struct SparseView3 {            // three CSR (or CSC) matrices, local index space
    const uint64_t* ptr[3];     // [count + 1]
    const uint32_t* idx[3];     // column (CSR) / row (CSC) indices, global
    const Fr* val[3];           // Montgomery values
};
struct LongChunk {
    uint32_t m;
    uint32_t pad;
    uint64_t begin, end;
};
struct LongRow {
    uint32_t m;
    uint32_t chunk_begin, chunk_end;
    uint32_t pad;
    uint64_t x;  // local output index
};
// eval_on_x column stream (k_col_stream): the A, B, C entries of each column concatenated, columns
// sorted by length inside windows of 64 x kColWindow columns and dealt to the 64 lanes of a slice (SELL-64),
// so the lanes of a wave run columns of (nearly) equal length. Columns with more than kLongCol
// entries go to the chunked long path (a lane's length is a 6-bit field).
static constexpr uint32_t kLongCol = 62;
static constexpr uint32_t kColNone = 0xFFFFFFFFu;  // lane slot without a column
static constexpr uint32_t kColWindow = 16;         // slices per sorting window (1024 columns)
struct ColSlice {
    uint64_t off;  // first entry slot of the slice: entry j of lane l at off + 64 j + l
    uint32_t len;  // the slice's longest column (steps)
    uint32_t pad;
};
struct ColStreamView {
    const ColSlice* slices;  // [nslices]
    const uint32_t* lanes;   // [64 nslices]: local column | entries << 26, or kColNone
    const uint32_t* rowm;    // entry slots: row | matrix << 30
    const Fr* val;           // entry slots: Montgomery values
    uint32_t nslices;
};
// sum_over_y for matrices whose every row has at most one entry (the R1CS multiplication-gate form;
// the benchmark generators): the entries of the rank's rows of A, B and C, with an explicit zero entry
// for an empty (row, matrix), sorted by column. Workgroups of XCD d take the d-th eighth of the list
// (k_spmv_sliced), so each XCD gathers a contiguous eighth of z through its own L2, nearly in order,
// instead of every XCD fetching whole 128-byte lines of z for 32-byte reads (k_sparse3<0>: 2.0x its
// algorithmic bytes).
struct SpmvSlicedView {
    const Fr* val;        // [entries] Montgomery values
    const uint32_t* col;  // [entries] global column, ascending
    const uint32_t* dst;  // [entries] local row | matrix << 30
};
// per-block partial sums of one sumcheck round (3 Fr per block, up to 8192 blocks)
static constexpr uint64_t kRoundPartials = 3 * 8192;

struct Tables3 {
    Fr* t[3];
};

// Lockstep groups (spx_ctx_set_group): one launch runs the same sumcheck round of up to kGroupMax
// proofs of one index, proof j's blocks at blockIdx.y = j, each with its own tables, challenge,
// partials, ticket and result (the per-proof launches' arguments, passed by value)
static constexpr int kGroupMax = 16;
// the last rounds of each sumcheck a lockstep group runs on the host (prove_group): <= 5 (the tables
// then fit each proof's 8 KiB pinned region)
static constexpr int kGroupHostTail = 5;
struct Sc1Job {
    Tables3 in, out;
    const Fr* Ein;
    Fr* Eout;
    Fr r;
    Fr* partial;  // kRoundPartials Fr of this proof
    uint32_t* ticket;
    Fr* result3;
};
struct Sc2Job {
    const Fr* Min;
    const Fr* Zin;
    Fr* Mout;
    Fr* Zout;
    Fr r;
    Fr* partial;
    uint32_t* ticket;
    Fr* result3;
};
struct Sc1Group {
    Sc1Job j[kGroupMax];
};
struct Sc2Group {
    Sc2Job j[kGroupMax];
};

// ---- live kernel statistics (HIP events around selected launches; off unless enabled)
struct KProf {
    bool on = false;
    struct Rec {
        int id;
        hipEvent_t a, b;
        double bytes, ops;
    };
    std::vector<Rec> open;  // recorded, not yet harvested
    std::vector<hipEvent_t> pool;
    uint64_t launches[16] = {0};
    double ms[16] = {0}, bytes[16] = {0}, ops[16] = {0};
    // the launches moving the most algorithmic bytes per id (e.g. round 1 of a sumcheck: the
    // HBM-streaming case; later rounds are small and cache-resident)
    uint64_t big_launches[16] = {0};
    double big_ms[16] = {0}, big_bytes[16] = {0};
    int cur_id = -1;
    hipEvent_t cur_a = nullptr;
    hipEvent_t get() {
        if (pool.empty()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    void begin(int id, hipStream_t s) {
        if (!on) return;
        cur_id = id;
        cur_a = get();
        (void)hipEventRecord(cur_a, s);
    }
    void end(double algo_bytes, hipStream_t s, double n_ops) {
        if (!on || cur_id < 0) return;
        hipEvent_t b = get();
        (void)hipEventRecord(b, s);
        open.push_back({cur_id, cur_a, b, algo_bytes, n_ops});
        cur_id = -1;
    }
    void harvest() {  // call after a stream sync
        for (auto& r : open) {
            float t = 0;
            if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
                launches[r.id] += 1;
                ms[r.id] += t;
                bytes[r.id] += r.bytes;
                ops[r.id] += r.ops;
                const double top = big_launches[r.id] ? big_bytes[r.id] / big_launches[r.id] : 0.0;
                if (r.bytes > top * 1.0001) {
                    big_launches[r.id] = 0, big_ms[r.id] = 0, big_bytes[r.id] = 0;
                }
                if (r.bytes >= top * 0.9999) {
                    big_launches[r.id] += 1;
                    big_ms[r.id] += t;
                    big_bytes[r.id] += r.bytes;
                }
            }
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
        open.clear();
    }
    void reset() {
        for (int i = 0; i < 16; ++i)
            launches[i] = 0, ms[i] = 0, bytes[i] = 0, ops[i] = 0, big_launches[i] = 0, big_ms[i] = 0, big_bytes[i] = 0;
    }
};
extern thread_local KProf* g_kprof;  // set by the host for the calling thread
inline void kp_begin(int id, hipStream_t s) {
    if (g_kprof) g_kprof->begin(id, s);
}
// bytes: algorithmic bytes of the launch; ops: its unit operations (curve additions for the MSM
// levels, table entries elsewhere; 0 where no op count is defined)
inline void kp_end(double bytes, hipStream_t s, double ops = 0) {
    if (g_kprof) g_kprof->end(bytes, s, ops);
}
enum { KP_SC1 = 0, KP_SC2, KP_SPMV, KP_MTV, KP_OPEN, KP_EQ, KP_SORT, KP_ACC_G1, KP_ACC_G2, KP_ACCX_G1, KP_ACCX_G2,
       KP_RED_G1, KP_RED_G2 };

// ---- mle_kernels.hip
void launch_to_mont(Fr* d, size_t n, int* err, hipStream_t s);
void launch_from_mont(Fr* out, const Fr* in, size_t n, hipStream_t s);
void launch_spmv_sliced(const SpmvSlicedView& v, const Fr* z, Fr* o0, Fr* o1, Fr* o2, uint64_t entries, hipStream_t s);
void launch_sparse3(int mode, const SparseView3& mv, const Fr* vec, Fr* o0, Fr* o1, Fr* o2, const Fr* scale,
                    uint64_t count, const LongChunk* chunks, int nchunks, const LongRow* lrows, int nlrows,
                    Fr* partial, hipStream_t s);
// eq(r_x, .) over L variables as the product of nf tables over consecutive bit fields of x (variable
// 0 = LSB): t[f] has 2^k[f] entries, the last one three copies scaled by r_A, r_B, r_C (m 2^k + x).
// eq_factors_for: nf = 2 (k[0] = ceil(L / 2) <= 13)
struct EqFactors {
    const Fr* t[3];
    int k[3];
    int nf;
};
// the split used for L variables, tables carved from `scratch` (kEqScratch Fr)
static constexpr uint64_t kEqScratch = 4 * 8192;
EqFactors eq_factors_for(int L, Fr* scratch);
// out[y] = sum_m scale[m] sum_x eq(r_x, x) M[x][y] over the column stream (r_x: L device Fr, scale: 3),
// then the long columns' chunks (over `lv`'s per-matrix entry arrays) added in
void launch_col_stream(const ColStreamView& cv, const Fr* r_x, int L, const Fr* scale, Fr* out, Fr* eq_scratch,
                       const SparseView3& lv, const LongChunk* chunks, int nchunks, const LongRow* lrows, int nlrows,
                       Fr* partial, hipStream_t s);
void launch_eq_table(const Fr* r_dev, int k, uint64_t base, uint64_t count, Fr* out, Fr* scratch_lo,
                     Fr* scratch_hi, hipStream_t s);
int sc_grid(uint64_t half);
// A round: fold with the previous challenge r (by value; unused in round 1), evaluate the round
// polynomial at 0, 1, 2 (at 1 only if need1: otherwise result3[1] = 0 and the caller derives it from
// the previous claim), and reduce over the blocks into result3 (3 Fr; device or host-mapped pinned
// memory) - in the last block for small grids, by a second one-block launch otherwise.
// partial: sc_grid(half) x 3 Fr of scratch; ticket: a device counter that is 0 (left 0).
void launch_sc1_round(bool fold, const Tables3& in, const Tables3& out, const Fr* Ein, Fr* Eout, const Fr& r,
                      uint64_t half, Fr* partial, uint32_t* ticket, Fr* result3, bool need1, hipStream_t s);
void launch_sc2_round(bool fold, const Fr* Min, const Fr* Zin, Fr* Mout, Fr* Zout, const Fr& r, uint64_t half,
                      Fr* partial, uint32_t* ticket, Fr* result3, bool need1, hipStream_t s);
// launch_sc1_round / launch_sc2_round for the k (<= kGroupMax) proofs of a lockstep group, in ONE launch
// (and one reduction launch for large grids): the same kernels' arithmetic, so each proof's result3
// equals its own launch's. need1 applies to every proof of the group.
void launch_sc1_round_group(int k, bool fold, const Sc1Job* jobs, uint64_t half, bool need1, hipStream_t s);
void launch_sc2_round_group(int k, bool fold, const Sc2Job* jobs, uint64_t half, bool need1, hipStream_t s);
// the other steps of a lockstep group, one launch per step for the k proofs (each proof's arguments as
// its own launch would take them; outputs bit-identical to the per-proof launchers):
// SpMV over the column-sorted entry list into out[j] = (Az, Bz, Cz);
void launch_spmv_sliced_group(int k, const SpmvSlicedView& v, const Fr* const* z, const Tables3* out, uint64_t entries,
                              hipStream_t s);
// launch_eq_table per proof (nvar variables at r_dev[j], scratch tables lo[j], hi[j]);
void launch_eq_table_group(int k, const Fr* const* r_dev, int nvar, uint64_t base, uint64_t count, Fr* const* out,
                           Fr* const* lo, Fr* const* hi, hipStream_t s);
// launch_col_stream per proof, for an index without long columns (the caller checks);
void launch_col_stream_group(int k, const ColStreamView& cv, const Fr* const* r_x, int L, const Fr* const* scale,
                             Fr* const* out, Fr* const* eq_scratch, hipStream_t s);
// z_j(points_j) by the stubbed opening's fold chain (no quotients), the value written to last[j]
// (host-mapped pinned memory allowed); bufA / bufB: n/2 and n/4 Fr per proof; points: k x L Fr
void launch_open_eval_group(int k, const Fr* const* z, Fr* const* bufA, Fr* const* bufB, const Fr* points, int L,
                            uint64_t n, Fr* const* last, hipStream_t s);
// per proof j: nruns (<= 3) runs of `per` Fr (nruns x per <= 4096) from src[j].t[i] to dst[j] back to back,
// one launch
void launch_copy_runs_group(int k, const Tables3* src, int nruns, int per, Fr* const* dst, hipStream_t s);
void launch_open_level(const Fr* rin, Fr* rout, Fr* q, const Fr& point, uint64_t half, hipStream_t s);
// the last levels of an opening in one launch: how many of the `remaining` levels starting at a level
// of `half` pairs it takes (0: none), and the launch (points[j] folds level j; q receives the levels'
// quotients contiguously; `last` the final value)
int open_tail_levels(uint64_t half, int remaining);
// nf (2 or 3) consecutive levels in one launch: nout = the last level's table size; level j's
// quotients go to q + qoffs[j] (~0: not written), points[j] folds level j
void launch_open_fold(const Fr* rin, Fr* rout, Fr* q, int nf, const Fr* points, const uint64_t* qoffs, uint64_t nout,
                      hipStream_t s);
void launch_open_tail(const Fr* rin, Fr* q, uint64_t half, int nlev, const Fr* points, Fr* last, hipStream_t s);

// ---- msm.hip
// One MSM inside a batch. Bases are the PRECOMPUTED window copies of a base set:
// pts[pts_off + w * stride + j] = 2^(c w) * B_j (affine), so every window shares one bucket set.
struct MsmInst {
    uint64_t pts_off;     // first precomputed point of this base set
    uint64_t scalar_off;  // first scalar (Montgomery Fr) in the batch scalar array
    uint32_t size;        // number of (base, scalar) pairs
    uint32_t c, W;        // window bits, windows
    uint32_t stride;      // points per window copy of the base set (>= size)
    // filled in by the MSM driver:
    uint32_t bucket_off;  // first local bucket of this instance
    uint32_t ref_off;     // first (bucket, reference) slot of this instance (dense key layout)
    uint32_t lb;          // log2 of the buckets this rank weights: c - 1 (whole) or c - 1 - lg (split)
    uint32_t lg;          // split: this rank weights buckets u = sel + 2^lg k (u = |digit| - 1); whole: 0
    uint32_t sel;
    uint32_t out;         // output slot (index in the caller's instance list)
};

// Bucket partition of a batch over the ranks of a proof-sharded prove: every rank
// reads ALL scalars of an instance and keeps the digits whose bucket is one of its own, so the
// accumulation, the partial levels and the bucket weighting all divide by the world size. Buckets
// are dealt round-robin (rank r: u = r, r + G, r + 2G, ...): the digits of the top windows, which
// crowd the low buckets (scalars < r < 2^255), spread evenly over the ranks. Rank r's result for an
// instance is sum_{its u} (u + 1) S_u; the ranks' results sum to the MSM. Instances too small to
// split (fewer than 4 buckets per rank) go whole to rank (index mod world).
struct MsmShard {
    int rank = 0, world = 1;
    bool dense = false;  // world > 1: one key slot per (scalar, window), as at world 1 (never overflows)
};
static constexpr uint32_t kMsmOverflow = 1;  // status bit: compacted keys exceeded their capacity

struct MsmWorkspace;  // opaque, owned by the host side (msm.hip)
MsmWorkspace* msm_ws_create();
void msm_ws_destroy(MsmWorkspace* ws);
// the pinned staging of the small per-batch tables: call only after a sync covering the workspace's stream
void msm_ws_staging_reset(MsmWorkspace* ws);
// a batch of this workspace reported kMsmOverflow: raise its compacted-key capacity for later batches
void msm_ws_note_overflow(MsmWorkspace* ws);

// bytes of a batch's output buffer: one XYZZ point per instance (G1: 4 x 48 B, G2: 4 x 96 B,
// Montgomery limbs; infinity = all zero), then a 16-byte status word (kMsmOverflow)
inline size_t msm_out_bytes(bool g2, int ninst) { return (size_t)ninst * (g2 ? 4 * 96 : 4 * 48) + 16; }
// Enqueues a batch of MSMs on `s` without any host synchronisation. With world > 1 and !dense the
// keys are compacted into a capacity planned from the expected bucket occupancy; if the status word
// reads kMsmOverflow afterwards, the outputs are invalid and the batch must be rerun with dense = true.
void msm_run_g1(MsmWorkspace* ws, const MsmInst* insts_host, int ninst, const G1Slot* pts, const Fr* scalars,
                void* out_dev, hipStream_t s, const MsmShard& sh = MsmShard());
void msm_run_g2(MsmWorkspace* ws, const MsmInst* insts_host, int ninst, const G2Aff* pts, const Fr* scalars,
                void* out_dev, hipStream_t s, const MsmShard& sh = MsmShard());

// PP preprocessing: for each base B_j (raw affine, level array), write the W window copies
// 2^(c w) B_j (affine) to dst[w * count + j]. pair_sum: B_j := raw[2j] + raw[2j+1].
void precompute_windows_g1(const G1Aff* raw, uint64_t count, bool pair_sum, int c, int W, G1Aff* dst, void* tmp,
                           hipStream_t s);
void precompute_windows_g2(const G2Aff* raw, uint64_t count, bool pair_sum, int c, int W, G2Aff* dst, void* tmp,
                           hipStream_t s);
// raw ark-serialize uncompressed points (canonical, flags) -> device affine Montgomery, in place.
// Infinity (flag bit 6) becomes the (0,0) sentinel. err |= 1 on malformed input.
void launch_points_from_bytes_g1(G1Aff* pts, uint64_t n, int* err, hipStream_t s);
void launch_points_from_bytes_g2(G2Aff* pts, uint64_t n, int* err, hipStream_t s);
void launch_points_to_canon_g1(G1Aff* pts, uint64_t n, hipStream_t s);
void launch_points_to_canon_g2(G2Aff* pts, uint64_t n, hipStream_t s);
// keygen: out[i] = scalar_i * base, with table[w * 256 + d] = d * 2^(8 w) * base (affine, 32 windows)
void fixed_base_g1(const G1Aff* table, const Fr* scalars, uint64_t n, G1Aff* out, void* tmp, hipStream_t s);
void fixed_base_g2(const G2Aff* table, const Fr* scalars, uint64_t n, G2Aff* out, void* tmp, hipStream_t s);

}  // namespace spx
