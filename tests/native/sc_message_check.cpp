// Host check of the sumcheck-1 message stepping (r1cs-spartan_amd/csrc/sc_message.hpp): the
// finite-difference form equals the point-by-point Lagrange form on random inputs. Prints "ok".
#include <cstdio>
#include <random>

#include "sc_message.hpp"

int main() {
    using F = spx::host::Fr;
    std::mt19937_64 rng(20260417);
    int bad = 0;
    for (int it = 0; it < 3000; ++it) {
        F v[5];
        for (auto& x : v) x = F::from_u64(rng()) * F::from_u64(rng()) + F::from_u64(rng());
        if (it == 0) v[1] = F::zero();  // tau = 0 and tau = 1: the eq factor vanishes at one end
        if (it == 1) v[1] = F::one();
        const F g[3] = {v[2], v[3], v[4]};
        const int L = 1 + it % 26;
        const auto a = spx::sc1_message(v[0], v[1], g, L), b = spx::sc1_message_lagrange(v[0], v[1], g, L);
        for (size_t i = 0; i < a.size(); ++i) bad += !(a[i] == b[i]);
    }
    if (bad) {
        printf("mismatches: %d\n", bad);
        return 1;
    }
    printf("ok\n");
    return 0;
}
