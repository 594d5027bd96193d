// Multi-buffer BLAKE2s for the per-proof matrix absorption (lib.rs:61-64: every proof's transcript
// absorbs ark-serialize(A), ark-serialize(B), ark-serialize(C) before anything else).
//
// One BLAKE2s stream is latency-bound: every G step depends on the previous one, so a
// core hashing one proof's ~150 MB at 2^20 leaves most of its vector width idle. The absorptions of
// several proofs are the same bytes into states that are equal up to that point, so they run in
// lockstep: lane i of a 32-bit vector holds proof i's state word, and one compression advances W
// proofs' transcripts (W = 16 with AVX-512, 8 with AVX2, chosen at run time). Every lane still does
// its proof's complete absorption; only the instructions are shared across W proofs.
//
// Host-only translation unit (plain C++, built by the host compiler: the target attributes below
// have no meaning for the device pass of a HIP compile).
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "transcript.hpp"

namespace spx {

struct Blake2sLanes {
#define SPX_AI inline __attribute__((always_inline))
    template <int W>
    struct VT;
    template <int W>
    using V = typename VT<W>::type;

    template <int W>
    static SPX_AI V<W> rotr(V<W> x, int n) {
        return (x >> n) | (x << (32 - n));
    }

    // W lanes, one 64-byte block common to all of them (same counter, same flags)
    template <int W>
    static SPX_AI void compress(V<W> (&h)[8], const uint8_t* blk, uint32_t t0, uint32_t t1, bool last) {
        uint32_t m[16];
        memcpy(m, blk, 64);
        V<W> v[16];
        for (int i = 0; i < 8; ++i) {
            v[i] = h[i];
            v[i + 8] = (V<W>){} + Blake2s::kIV[i];
        }
        v[12] ^= t0;
        v[13] ^= t1;
        if (last) v[14] = ~v[14];
#pragma GCC unroll 10
        for (int r = 0; r < 10; ++r) {
            const uint8_t* s = Blake2s::kSigma[r];
#define SPX_GV(a, b, c, d, x, y)               \
    v[a] += v[b] + (x);                        \
    v[d] = rotr<W>(v[d] ^ v[a], 16);           \
    v[c] += v[d];                              \
    v[b] = rotr<W>(v[b] ^ v[c], 12);           \
    v[a] += v[b] + (y);                        \
    v[d] = rotr<W>(v[d] ^ v[a], 8);            \
    v[c] += v[d];                              \
    v[b] = rotr<W>(v[b] ^ v[c], 7);
            SPX_GV(0, 4, 8, 12, m[s[0]], m[s[1]])
            SPX_GV(1, 5, 9, 13, m[s[2]], m[s[3]])
            SPX_GV(2, 6, 10, 14, m[s[4]], m[s[5]])
            SPX_GV(3, 7, 11, 15, m[s[6]], m[s[7]])
            SPX_GV(0, 5, 10, 15, m[s[8]], m[s[9]])
            SPX_GV(1, 6, 11, 12, m[s[10]], m[s[11]])
            SPX_GV(2, 7, 8, 13, m[s[12]], m[s[13]])
            SPX_GV(3, 4, 9, 14, m[s[14]], m[s[15]])
#undef SPX_GV
        }
        for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
    }

    // the update of Blake2s::update, for W states that share counter, buffer and buffer length
    template <int W>
    static SPX_AI void update_group(Blake2s* st, const uint8_t* p, size_t len) {
        V<W> h[8];
        for (int i = 0; i < 8; ++i)
            for (int l = 0; l < W; ++l) h[i][l] = st[l].h_[i];
        Blake2s& s0 = st[0];
        uint32_t t0 = s0.t0_, t1 = s0.t1_;
        uint8_t buf[64];
        size_t buflen = s0.buflen_;
        memcpy(buf, s0.buf_, buflen);
        auto inc = [&](uint32_t k) {
            t0 += k;
            if (t0 < k) t1++;
        };
        while (len > 0) {
            if (buflen == 64) {
                inc(64);
                compress<W>(h, buf, t0, t1, false);
                buflen = 0;
            }
            if (buflen == 0 && len > 64) {
                inc(64);
                compress<W>(h, p, t0, t1, false);
                p += 64;
                len -= 64;
                continue;
            }
            size_t k = std::min<size_t>(64 - buflen, len);
            memcpy(buf + buflen, p, k);
            buflen += k;
            p += k;
            len -= k;
        }
        for (int l = 0; l < W; ++l) {
            for (int i = 0; i < 8; ++i) st[l].h_[i] = h[i][l];
            st[l].t0_ = t0;
            st[l].t1_ = t1;
            memcpy(st[l].buf_, buf, buflen);
            st[l].buflen_ = buflen;
        }
    }

    __attribute__((target("avx512f"))) static void update16(Blake2s* st, const uint8_t* p, size_t len) {
        update_group<16>(st, p, len);
    }
    __attribute__((target("avx2"))) static void update8(Blake2s* st, const uint8_t* p, size_t len) {
        update_group<8>(st, p, len);
    }

    static bool same_position(const Blake2s* st, int k) {
        for (int l = 1; l < k; ++l)
            if (st[l].t0_ != st[0].t0_ || st[l].t1_ != st[0].t1_ || st[l].buflen_ != st[0].buflen_ ||
                memcmp(st[l].buf_, st[0].buf_, st[0].buflen_) != 0)
                return false;
        return true;
    }
};

int blake2s_lane_width() {
    static const int w = __builtin_cpu_supports("avx512f") ? 16 : (__builtin_cpu_supports("avx2") ? 8 : 1);
    return w;
}

void blake2s_update_lanes(Blake2s* st, int k, const void* data, size_t len) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    if (k <= 0) return;
    if (!Blake2sLanes::same_position(st, k)) {  // not in lockstep: one stream each
        for (int l = 0; l < k; ++l) st[l].update(p, len);
        return;
    }
    const int w = blake2s_lane_width();
    if (w == 1) {
        for (int l = 0; l < k; ++l) st[l].update(p, len);
        return;
    }
    for (int l = 0; l < k;) {
        // groups of 16 (AVX-512) while at least 9 states remain, then 8 (AVX2, also on AVX-512
        // machines); a short last group runs at full width on copies (the extra lanes are dropped)
        const int gw = (w == 16 && k - l > 8) ? 16 : 8;
        Blake2s tmp[16];
        const int n = std::min(gw, k - l);
        if (n <= 2) {  // one or two states: scalar streams (a padded vector group costs more, and the
                       // scalar code shares a core's SMT siblings far better; spx_prove_many's first waves)
            for (int i = 0; i < n; ++i) st[l + i].update(p, len);
            l += n;
            continue;
        }
        Blake2s* g = st + l;
        if (n < gw) {
            for (int i = 0; i < gw; ++i) tmp[i] = st[l + std::min(i, n - 1)];
            g = tmp;
        }
        if (gw == 16)
            Blake2sLanes::update16(g, p, len);
        else
            Blake2sLanes::update8(g, p, len);
        if (n < gw)
            for (int i = 0; i < n; ++i) st[l + i] = tmp[i];
        l += n;
    }
}

template <>
struct Blake2sLanes::VT<8> {
    typedef uint32_t type __attribute__((vector_size(32)));
};
template <>
struct Blake2sLanes::VT<16> {
    typedef uint32_t type __attribute__((vector_size(64)));
};

}  // namespace spx
