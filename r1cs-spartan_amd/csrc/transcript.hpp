// Fiat-Shamir transcript of the reference, `linear_sumcheck::data_structures::Blake2s512Rng`
// [upstream arkworks-rs/sumcheck, unpinned; SURVEY §8(c)] as driven by /root/reference/src/lib.rs:61-131:
//   feed(m)   = Blake2s.update(ark-serialize(m))
//   fill(d)   = out = finalize(clone); copy out; every 32 consumed bytes: update(out), refresh;
//               at the end update(out)
//   Fr::rand  = 4 x next_u64 (LE), top limb & (2^63 - 1), retry while >= r; the accepted bigint is the
//               Montgomery REPRESENTATION (ark-ff Fp256 sampling).
// The Blake2s state is copyable, so a witness-independent prefix (the three matrices) can be
// absorbed once at index time and resumed per proof (bit-identical).
#pragma once
#include <stdint.h>
#include <string.h>

#include "host_ff.hpp"

namespace spx {

class Blake2s {
   public:
    Blake2s() { reset(); }
    void reset() {
        static const uint32_t iv[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                       0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
        memcpy(h_, iv, sizeof h_);
        h_[0] ^= 0x01010000u ^ 32u;
        t0_ = t1_ = 0;
        buflen_ = 0;
    }
    void update(const void* data, size_t len) {
        const uint8_t* p = static_cast<const uint8_t*>(data);
        // fast path: whole blocks while more input follows
        while (len > 0) {
            if (buflen_ == 64) {
                inc(64);
                compress(buf_, false);
                buflen_ = 0;
            }
            if (buflen_ == 0 && len > 64) {
                inc(64);
                compress(p, false);
                p += 64;
                len -= 64;
                continue;
            }
            size_t k = 64 - buflen_;
            if (k > len) k = len;
            memcpy(buf_ + buflen_, p, k);
            buflen_ += k;
            p += k;
            len -= k;
        }
    }
    // digest of a copy of the state (state unchanged)
    void peek(uint8_t out[32]) const {
        Blake2s s = *this;
        s.inc((uint32_t)s.buflen_);
        memset(s.buf_ + s.buflen_, 0, 64 - s.buflen_);
        s.compress(s.buf_, true);
        memcpy(out, s.h_, 32);  // little-endian host
    }

   private:
    static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
    void inc(uint32_t k) {
        t0_ += k;
        if (t0_ < k) t1_++;
    }
    // The matrix absorption (~150 MB per proof at 2^20) is the prover's largest sequential host work.
    // BLAKE2s is latency-bound on one stream (every G step depends on the previous one), so the gain
    // is in the fully unrolled rounds with compile-time message indices (1.5x over a table-indexed
    // loop); 128-bit SIMD forms of the four G functions measured no faster.
    void compress(const uint8_t* blk, bool last) { compress_scalar(blk, last); }

   public:
    static constexpr uint8_t kSigma[10][16] = {
        {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
        {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
        {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
        {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
        {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
    static constexpr uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                        0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
    void compress_scalar(const uint8_t* blk, bool last) {
        uint32_t m[16], v[16];
        memcpy(m, blk, 64);
        for (int i = 0; i < 8; ++i) v[i] = h_[i], v[i + 8] = kIV[i];
        v[12] ^= t0_;
        v[13] ^= t1_;
        if (last) v[14] = ~v[14];
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            const uint8_t* s = kSigma[r];
#define SPX_G(a, b, c, d, x, y)           \
    v[a] += v[b] + (x);                   \
    v[d] = rotr(v[d] ^ v[a], 16);         \
    v[c] += v[d];                         \
    v[b] = rotr(v[b] ^ v[c], 12);         \
    v[a] += v[b] + (y);                   \
    v[d] = rotr(v[d] ^ v[a], 8);          \
    v[c] += v[d];                         \
    v[b] = rotr(v[b] ^ v[c], 7);
            SPX_G(0, 4, 8, 12, m[s[0]], m[s[1]])
            SPX_G(1, 5, 9, 13, m[s[2]], m[s[3]])
            SPX_G(2, 6, 10, 14, m[s[4]], m[s[5]])
            SPX_G(3, 7, 11, 15, m[s[6]], m[s[7]])
            SPX_G(0, 5, 10, 15, m[s[8]], m[s[9]])
            SPX_G(1, 6, 11, 12, m[s[10]], m[s[11]])
            SPX_G(2, 7, 8, 13, m[s[12]], m[s[13]])
            SPX_G(3, 4, 9, 14, m[s[14]], m[s[15]])
#undef SPX_G
        }
        for (int i = 0; i < 8; ++i) h_[i] ^= v[i] ^ v[i + 8];
    }
   private:
    friend struct Blake2sLanes;
    uint32_t h_[8];
    uint32_t t0_, t1_;
    uint8_t buf_[64];
    size_t buflen_;
};

// Multi-buffer update (blake2s_lanes.cpp): st[0..k) absorb the same bytes; states at the same
// position (counter, buffered bytes) advance together in the lanes of one vector (16 with AVX-512,
// 8 with AVX2), others one by one. Results equal k separate update() calls.
int blake2s_lane_width();
void blake2s_update_lanes(Blake2s* st, int k, const void* data, size_t len);

// The verifier of an interactive prove (the reference's round-level API, prover.rs:109-281 driven as
// in ahp/tests.rs:8-70): every prover message goes to message(), every challenge comes from draw()
// (a verifier coin supplied by the caller).
struct ExternalCoins {
    virtual ~ExternalCoins() = default;
    virtual void message(const void* d, size_t n) = 0;
    virtual host::Fr draw() = 0;
};

class Transcript {
   public:
    explicit Transcript(bool injected = false, uint64_t seed = 0, ExternalCoins* ext = nullptr)
        : injected_(injected), sm_(seed), ext_(ext) {}
    // a prover message (lib.rs:74-129 feeds each one before the next challenge)
    void feed(const void* d, size_t n) {
        if (ext_)
            ext_->message(d, n);
        else if (!injected_)
            h_.update(d, n);
    }
    // absorption that is not a prover message (the public input v, lib.rs:65)
    void absorb(const void* d, size_t n) {
        if (!ext_ && !injected_) h_.update(d, n);
    }
    bool external() const { return ext_ != nullptr; }
    void set_state(const Blake2s& b) { h_ = b; }
    const Blake2s& state() const { return h_; }
    host::Fr rand_fr() {
        if (ext_) return ext_->draw();
        if (injected_) return sm_fr();
        for (;;) {
            uint64_t l[4];
            for (int i = 0; i < 4; ++i) {
                uint8_t b[8];
                fill(b, 8);
                memcpy(&l[i], b, 8);
            }
            l[3] &= 0x7FFFFFFFFFFFFFFFULL;
            if (!host::Fr::geq_p(l)) {
                host::Fr r;
                memcpy(r.v, l, 32);  // Montgomery representation
                return r;
            }
        }
    }

   private:
    void fill(uint8_t* dest, size_t n) {
        uint8_t out[32];
        h_.peek(out);
        size_t ptr = 0;
        for (size_t i = 0; i < n; ++i) {
            dest[i] = out[ptr++];
            if (ptr == 32) {
                h_.update(out, 32);
                h_.peek(out);
                ptr = 0;
            }
        }
        h_.update(out, 32);
    }
    uint64_t sm_next() {
        sm_ += 0x9E3779B97F4A7C15ULL;
        uint64_t z = sm_;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    host::Fr sm_fr() {  // canonical SplitMix64 Fr (injected-challenge mode)
        for (;;) {
            uint64_t c[4] = {sm_next(), sm_next(), sm_next(), sm_next() & 0x7FFFFFFFFFFFFFFFULL};
            if (!host::Fr::geq_p(c)) return host::Fr::from_canon(c);
        }
    }
    bool injected_;
    uint64_t sm_;
    ExternalCoins* ext_;
    Blake2s h_;
};

}  // namespace spx
