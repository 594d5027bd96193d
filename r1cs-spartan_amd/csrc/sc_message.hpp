// Host side of a sumcheck-1 round (prover.rs:199-207): the prover message from the device's three
// sums. Header-only so tests/native/sc_message_check.cpp can check it on the host.
#pragma once
#include <vector>

#include "host_ff.hpp"

namespace spx {

// sumcheck #1 message from G(0), G(1), G(2): P(t) = C eq(tau_c, t) G(t), t = 0..L+2. G is quadratic
// and C eq(tau_c, t) = C (1 - tau) + t C (2 tau - 1) is linear in t, so both are stepped by finite
// differences and every point costs one product (exact field arithmetic: the same bytes as evaluating
// each point by Lagrange, sc1_message_lagrange).
inline std::vector<host::Fr> sc1_message(const host::Fr& Cc, const host::Fr& tau, const host::Fr g[3], int L) {
    using F = host::Fr;
    std::vector<F> P(L + 3);
    const F one = F::one();
    F Gt = g[0], d = g[1] - g[0];
    const F dd = g[2] - g[1] - d;  // second difference
    F Ce = Cc * (one - tau);
    const F Cs = Cc * (tau + tau - one);
    for (int t = 0; t <= L + 2; ++t) {
        P[t] = Ce * Gt;
        Gt = Gt + d;
        d = d + dd;
        Ce = Ce + Cs;
    }
    return P;
}

// the same message point by point: Lagrange through (0, g0), (1, g1), (2, g2), times
// C eq(tau, t) = C (1 - tau - t + 2 tau t) (eq.rs:14)
inline std::vector<host::Fr> sc1_message_lagrange(const host::Fr& Cc, const host::Fr& tau, const host::Fr g[3], int L) {
    using F = host::Fr;
    const F inv2 = F::from_u64(2).inv();
    std::vector<F> P(L + 3);
    const F one = F::one(), two = F::from_u64(2);
    for (int t = 0; t <= L + 2; ++t) {
        const F T = F::from_u64((uint64_t)t);
        const F l0 = (T - one) * (T - two) * inv2, l1 = T * (T - two), l2 = T * (T - one) * inv2;
        const F Gt = g[0] * l0 - g[1] * l1 + g[2] * l2;
        P[t] = Cc * (one - tau - T + (tau + tau) * T) * Gt;
    }
    return P;
}

}  // namespace spx
