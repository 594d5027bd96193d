// spx_prove_many's hashing-pool plan (r1cs-spartan_amd/csrc/hash_sched.hpp) on real threads: for
// every pool size, context count, lane width and proof count, each owned proof is absorbed by exactly
// one job, the first scalar waves (0, 1 or 2 waves of nctx proofs) one per job, the lead full-width jobs first, and
// every thread terminates (a proof whose
// job is never claimed would leave its prove waiting forever).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

#include "hash_sched.hpp"

int main() {
    int cases = 0;
    for (int owned : {0, 1, 5, 16, 31, 32, 33, 64, 192, 320, 1000})
        for (int nctx : {1, 4, 16, 64})
            for (int nh0 : {1, 2, 3, 4, 5, 8, 16, 32})
                for (int lanes : {1, 8, 16})
                    for (int sw : {0, 1, 2})
                    for (size_t cap : {(size_t)SIZE_MAX, (size_t)4, (size_t)32}) {
                        spx::HashSched s(owned, (size_t)nctx, lanes, sw, cap, (size_t)nh0);
                        std::vector<std::atomic<int>> done(owned);
                        for (auto& d : done) d = 0;
                        const int nh = std::min<int>(nh0, (int)s.size());
                        std::vector<std::thread> pool;
                        for (int t = 0; t < nh; ++t)
                            pool.emplace_back([&] {
                                for (size_t j; (j = s.claim()) < s.size();)
                                    for (size_t i = s.jobs[j].first; i < s.jobs[j].second; ++i) done[i]++;
                            });
                        for (auto& p : pool) p.join();
                        for (int i = 0; i < owned; ++i)
                            if (done[i] != 1) {
                                printf("FAIL owned %d nctx %d threads %d lanes %d: proof %d absorbed %d times\n", owned,
                                       nctx, nh0, lanes, i, (int)done[i]);
                                return 1;
                            }
                        // claim order: the lead full-width jobs, the scalar jobs of the first two waves, the rest
                        const size_t scalar = lanes > 1 ? std::min({(size_t)owned, (size_t)sw * nctx, cap}) : owned;
                        // a pool of nh0 threads leads with at most nh0 - 1 full-width jobs when there are
                        // scalar jobs, so one thread starts on the first wave
                        if (scalar > 0 && s.nlead + 1 > (size_t)nh0) {
                            printf("FAIL owned %d nctx %d threads %d: %zu lead jobs\n", owned, nctx, nh0, s.nlead);
                            return 1;
                        }
                        for (size_t j = 0; j < s.size(); ++j) {
                            const size_t w = s.jobs[j].second - s.jobs[j].first;
                            const bool is_scalar = j >= s.nlead && j < s.nlead + scalar;
                            if ((is_scalar && (w != 1 || s.jobs[j].first != j - s.nlead)) ||
                                (!is_scalar && (w < 1 || w > (size_t)lanes || s.jobs[j].first < scalar))) {
                                printf("FAIL owned %d nctx %d lanes %d: job %zu covers %zu proofs\n", owned, nctx, lanes, j, w);
                                return 1;
                            }
                        }
                        // after stop() nothing more is handed out
                        s.stop();
                        for (int t = 0; t < 8; ++t)
                            if (s.claim() < s.size()) {
                                printf("FAIL: a job claimed after stop()\n");
                                return 1;
                            }
                        ++cases;
                    }
    printf("ok %d cases\n", cases);
    return 0;
}
