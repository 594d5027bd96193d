// Job plan of spx_prove_many's hashing pool (capi.cpp): which owned proofs each absorption job covers,
// in the order the pool threads claim them. Host-only, no HIP: tests/native/hash_sched_check.cpp
// runs it on threads and checks that every proof is absorbed exactly once for any pool size.
//
// Owned proofs are proved in waves of `wave` (the rank's share of one proof per context in flight:
// ceil(nctx / G) when proof i is absorbed by rank i mod G). The first `scalar_waves` waves (2 for
// full proofs) are absorbed one proof per job (scalar: ready after one absorption's time, as their
// proofs reach their first challenge); every later proof in full-width multi-buffer jobs (`lanes`
// proofs each). With the commitment stubbed (BASELINE C2) a proof's device work is ~1% of one
// absorption, so there is nothing to overlap and only the pool's throughput counts: 0 scalar waves.
// The first kLead full-width jobs are claimed before the scalar ones, so they run from the start on
// their own threads (kLead threads beyond the scalar part's) and are done before their waves start.
// With a pool of `threads` threads at most threads - 1 jobs lead, so at least one thread starts on the
// scalar jobs of the first wave (a pool of 1 or 2 threads would otherwise spend its first ~0.3 s on
// later waves' full-width jobs while the first proofs wait).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace spx {

struct HashSched {
    static constexpr size_t kLead = 4;
    std::vector<std::pair<size_t, size_t>> jobs;  // [first, last) owned indices per job, in claim order
    size_t nlead = 0;                             // full-width jobs claimed ahead of the scalar ones
    std::atomic<size_t> next{0};

    // max_scalar caps the scalar part (two rounds of the pool's threads: with many proofs in flight a
    // wave is wider than the pool, and the full-width jobs beside it are ready as early)
    HashSched(size_t owned, size_t wave, int lanes, int scalar_waves = 2, size_t max_scalar = SIZE_MAX,
              size_t threads = SIZE_MAX) {
        size_t nscalar = lanes > 1 ? std::min(owned, (size_t)std::max(scalar_waves, 0) * std::max<size_t>(wave, 1)) : owned;
        if (lanes > 1) nscalar = std::min(nscalar, max_scalar);
        std::vector<std::pair<size_t, size_t>> wide;
        for (size_t b = nscalar; b < owned; b += (size_t)lanes) wide.emplace_back(b, std::min(owned, b + (size_t)lanes));
        nlead = std::min(kLead, wide.size());
        if (nscalar > 0) nlead = std::min(nlead, threads > 0 ? threads - 1 : 0);
        jobs.assign(wide.begin(), wide.begin() + nlead);
        for (size_t b = 0; b < nscalar; ++b) jobs.emplace_back(b, b + 1);
        jobs.insert(jobs.end(), wide.begin() + nlead, wide.end());
    }
    size_t size() const { return jobs.size(); }
    // the next job in claim order, or size() when none is left
    size_t claim() { return std::min(next.fetch_add(1), size()); }
    void stop() { next.store(size()); }  // no job is handed out after this
};

}  // namespace spx
