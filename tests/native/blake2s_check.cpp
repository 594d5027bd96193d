// Host-only check of the product's Blake2s (r1cs-spartan_amd/csrc/transcript.hpp): the digest matches
// the RFC 7693 known answer for "abc", and the streaming update over odd-sized pieces equals block-wise
// compression. Prints "ok <MB/s compress> <MB/s update>".
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "transcript.hpp"

struct Scalar : spx::Blake2s {};

int main() {
    // RFC 7693 Appendix B: BLAKE2s-256("abc")
    static const uint8_t kat[32] = {0x50, 0x8C, 0x5E, 0x8C, 0x32, 0x7C, 0x14, 0xE2, 0xE1, 0xA7, 0x2B,
                                    0xA3, 0x4E, 0xEB, 0x45, 0x2F, 0x37, 0x45, 0x8B, 0x20, 0x9E, 0xD6,
                                    0x3A, 0x29, 0x4D, 0x99, 0x9B, 0x4C, 0x86, 0x67, 0x59, 0x82};
    spx::Blake2s h;
    h.update("abc", 3);
    uint8_t out[32];
    h.peek(out);
    if (memcmp(out, kat, 32)) {
        printf("KAT mismatch\n");
        return 1;
    }
    std::vector<uint8_t> buf((64u << 20) + 37);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 131 + 7);
    uint8_t one[32], pieces[32];
    spx::Blake2s s1;
    auto t0 = std::chrono::steady_clock::now();
    s1.update(buf.data(), buf.size());
    const double mbs = buf.size() / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 1e6;
    s1.peek(one);
    spx::Blake2s s2;  // the same bytes in odd-sized pieces (the serializer's flush pattern)
    for (size_t o = 0, k = 1; o < buf.size(); k = k * 7 % 65521 + 1) {
        const size_t n = std::min(k, buf.size() - o);
        s2.update(buf.data() + o, n);
        o += n;
    }
    s2.peek(pieces);
    if (memcmp(one, pieces, 32)) {
        printf("piecewise update mismatch\n");
        return 1;
    }
    printf("ok %.0f\n", mbs);
    return 0;
}
