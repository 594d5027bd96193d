// Host-only check of the multi-buffer BLAKE2s (r1cs-spartan_amd/csrc/blake2s_lanes.cpp): k states
// absorbing the same bytes in pieces of odd sizes end equal, word for word, to k separate scalar
// streams, for k below, at and above the lane width and with states at different positions (the
// one-by-one fallback). Prints "ok <lane width> <scalar MB/s> <lanes MB/s per proof stream x k>".
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "transcript.hpp"

static bool same(const spx::Blake2s& a, const spx::Blake2s& b) {
    uint8_t x[32], y[32];
    a.peek(x);
    b.peek(y);
    return memcmp(x, y, 32) == 0;
}

int main() {
    std::vector<uint8_t> buf((8u << 20) + 101);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 167 + 3);
    const size_t piece[] = {1, 63, 64, 65, 40, 8, 4096, 65536, 127};
    for (int k : {1, 3, 8, 13, 16, 20, 33}) {
        std::vector<spx::Blake2s> st(k);
        spx::Blake2s ref;
        size_t off = 0, pi = 0;
        while (off < buf.size()) {
            size_t n = std::min(piece[pi++ % 9], buf.size() - off);
            spx::blake2s_update_lanes(st.data(), k, buf.data() + off, n);
            ref.update(buf.data() + off, n);
            off += n;
        }
        for (int l = 0; l < k; ++l)
            if (!same(st[l], ref)) {
                printf("lane %d of %d differs\n", l, k);
                return 1;
            }
    }
    {   // states at different positions: each one advances by itself
        std::vector<spx::Blake2s> st(5);
        st[2].update("x", 1);
        spx::blake2s_update_lanes(st.data(), 5, buf.data(), 1000);
        spx::Blake2s a, b;
        a.update(buf.data(), 1000);
        b.update("x", 1);
        b.update(buf.data(), 1000);
        if (!same(st[0], a) || !same(st[4], a) || !same(st[2], b)) {
            printf("diverged states wrong\n");
            return 1;
        }
    }
    // throughput: one scalar stream vs lane-width streams on one core
    const int w = spx::blake2s_lane_width();
    std::vector<uint8_t> big(64u << 20);
    for (size_t i = 0; i < big.size(); ++i) big[i] = (uint8_t)i;
    auto t0 = std::chrono::steady_clock::now();
    spx::Blake2s s;
    s.update(big.data(), big.size());
    auto t1 = std::chrono::steady_clock::now();
    std::vector<spx::Blake2s> st(w);
    spx::blake2s_update_lanes(st.data(), w, big.data(), big.size());
    auto t2 = std::chrono::steady_clock::now();
    if (!same(st[w - 1], s)) {
        printf("throughput run differs\n");
        return 1;
    }
    const double mb = big.size() / 1e6;
    printf("ok %d %.0f %.0f\n", w, mb / std::chrono::duration<double>(t1 - t0).count(),
           w * mb / std::chrono::duration<double>(t2 - t1).count());
    return 0;
}
