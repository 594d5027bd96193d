// Shared pieces of the MSM translation units (msm_common.hip, msm_g1.hip, msm_g2.hip).
#pragma once
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.hpp"

namespace spx {

static constexpr uint32_t kSeg1Default = 64;  // references per thread, affine accumulation level (A/B: profiles/r02_ab19_seg.jsonl, r02_ab20_seg.jsonl)
uint32_t seg1_len(bool g2);                      // kSeg1Default for both curves
// seg1 lowered so the accumulation grid fills whole rounds of resident waves (no near-empty last round)
uint32_t seg1_fit(uint32_t seg1, uint64_t refs, int waves_per_simd, int lanes_per_elem);
// partials per thread, XYZZ accumulation levels (4: shallow levels; 8 measured -0.6% for a G = 8 rank,
// -0.4% at N = 1: profiles/r05/r05zza_ab_seg_chunk_*.jsonl)
static constexpr uint32_t kSeg = 4;
// buckets per running-sum chunk of the weighting leaf: 4 (8: within noise, r05zza_ab_seg_chunk_*.jsonl)
static constexpr uint32_t kTreeChunkLog = 2;
// k_tree_top: the levels whose input has <= 32 nodes, one launch (one level launch fewer per batch
// than 16: G = 8 rank +1.0%, N = 1 +1.4%; 64: +0.8% / +0.4%, 147 KB of LDS; profiles/r05/r05zz_ab_topnodes_*.jsonl)
static constexpr uint32_t kTopNodes = 32;
static constexpr int kLight = 256;  // threads for bookkeeping kernels
static constexpr int kHeavy = 64;   // threads for curve kernels (register-heavy)

#define HIPCHK(x)                                                                                     \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + \
                                                       " at " __FILE__ ":" + std::to_string(__LINE__)); \
    } while (0)

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

// Pinned host staging for the small per-batch tables an MSM uploads (instance descriptors, scalar
// prefixes, weighting-tree prefixes). A hipMemcpyAsync from pageable memory may read its source
// after the call returns, so the source must outlive the copy: regions are bump-allocated and the
// arena is reset only by the workspace's owner, right after a stream synchronisation that covers
// every copy issued from it (msm_ws_staging_reset). Fixed capacity: nothing is ever reallocated
// under an in-flight copy.
struct PinArena {
    static constexpr size_t kCap = 512 << 10;
    uint8_t* p = nullptr;
    size_t used = 0;
    PinArena() { HIPCHK(hipHostMalloc((void**)&p, kCap)); }
    ~PinArena() {
        if (p) (void)hipHostFree(p);
    }
    template <class T>
    T* stage(const T* src, size_t count) {  // copy `count` items into the arena; returns the pinned copy
        const size_t o = (used + 255) & ~(size_t)255, b = sizeof(T) * count;
        if (o + b > kCap) throw std::runtime_error("MSM pinned staging arena exhausted");
        used = o + b;
        memcpy(p + o, src, b);
        return (T*)(p + o);
    }
    void reset() { used = 0; }  // only after a sync covering every copy from the arena
};

struct MsmWorkspace {
    DBuf tables, offs, refs, pa, pb, tree_a, tree_b;
    // bucket sort (msm_sort): per-(bin, tile) counts and their row prefixes, per-bin totals and
    // bases, the bin-partitioned staging (reference + in-bin bucket), the partial-level offsets and
    // their per-bin sums / prefixes, and the two hand-off tickets (zero between launches: the last
    // block of each hand-off resets its ticket)
    DBuf cnt, bintot, binbase, binsum, stage_ref, stage_fine, lvl, tickets;
    bool tickets_zeroed = false;
    // compacted-key capacity factor: raised after an overflow, so a workload whose scalars crowd some
    // rank's buckets (e.g. many equal values) stops overflowing after its first batch
    double cap_scale = 1.0;
    PinArena pin;
};

// Host plan of a batch: the instances this rank works on (driver fields filled in), the key slots,
// the weighting tree's shape, and their device copy (ONE staged upload per batch).
struct MsmPlan {
    std::vector<MsmInst> insts;   // active instances
    std::vector<uint64_t> prefix;  // scalar prefix over the active instances (nact + 1)
    uint32_t nb = 0;              // local buckets in the batch
    uint64_t tot_sc = 0;          // scalars digitised
    uint64_t tot_refs = 0;        // key slots: upper bound of the references with a digit in range
    bool compact = false;         // proof-sharded keys (only in-range digits, capacity tot_refs)
    double mu_max = 0;            // largest expected references per bucket over the active instances
    bool any_split = false;
    // weighting tree: per instance, node offset and node count after the chunked leaf; levels above it
    std::vector<uint32_t> node_off, cnt;
    int levels = 0;     // tree levels above the leaf (max over instances)
    int top_from = 1;   // first level done by k_tree_top (all levels >= it); levels below run one launch each
    std::vector<uint64_t> wp;   // per level: work prefixes (levels + 1) x (nact + 1)
    std::vector<uint32_t> cin;  // per level: input node counts (levels + 1) x nact
    // device copies
    MsmInst* d_insts = nullptr;
    uint64_t *d_prefix = nullptr, *d_wp = nullptr;
    uint32_t *d_cin = nullptr, *d_noff = nullptr;
};
MsmPlan msm_plan(const MsmInst* ih, int ninst, const MsmShard& sh, double cap_scale);
void msm_upload_plan(MsmWorkspace* ws, MsmPlan& p, hipStream_t s);

// status words after a batch's outputs (zeroed with them by the sort's first launch): [0] status bits
// Digit / sort stage: references sorted by bucket, per-bucket offsets (offs[nb] = references), and
// the offsets of the affine level's partials (np_off: the seg1-reference thread ranges each bucket
// meets) and of every planned XYZZ level (lev[l]: segments of kSeg partials per bucket).
struct MsmSorted {
    uint32_t *offs, *refs, *np_off;
    std::vector<uint32_t*> lev;
};
// seg1 / nlev: the affine level's references per thread and the number of XYZZ partial levels the
// driver will run. out_dev / out_bytes: the batch's outputs and status words, zeroed by the first
// launch. Five launches, no host synchronisation, no library kernels (msm_common.hip).
MsmSorted msm_sort(MsmWorkspace* ws, const MsmPlan& p, const Fr* scalars, void* out_dev, size_t out_bytes, hipStream_t s,
                   uint32_t seg1, int nlev);

}  // namespace spx
