/* ORACLE — TEST INFRASTRUCTURE ONLY.
 * BLAKE2s-256 (RFC 7693), incremental, copyable state — the hash behind
 * linear-sumcheck's Blake2s512Rng [upstream] (see oracle/py/transcript.py for the
 * reconstructed RNG semantics restated in oracle.c).
 */
#ifndef ORACLE_BLAKE2S_H
#define ORACLE_BLAKE2S_H
#include <stddef.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    uint32_t h[8];
    uint32_t t[2];
    uint8_t buf[64];
    size_t buflen;
} ob2s_t;

static const uint32_t OB2S_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                    0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t OB2S_SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

static inline uint32_t ob2s_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static inline void ob2s_compress(ob2s_t *s, const uint8_t *blk, int last) {
    uint32_t m[16], v[16];
    for (int i = 0; i < 16; ++i)
        m[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) | ((uint32_t)blk[4 * i + 2] << 16) |
               ((uint32_t)blk[4 * i + 3] << 24);
    for (int i = 0; i < 8; ++i) {
        v[i] = s->h[i];
        v[i + 8] = OB2S_IV[i];
    }
    v[12] ^= s->t[0];
    v[13] ^= s->t[1];
    if (last) v[14] = ~v[14];
#define OB2S_G(a, b, c, d, x, y)                 \
    do {                                         \
        v[a] = v[a] + v[b] + (x);                \
        v[d] = ob2s_rotr(v[d] ^ v[a], 16);       \
        v[c] = v[c] + v[d];                      \
        v[b] = ob2s_rotr(v[b] ^ v[c], 12);       \
        v[a] = v[a] + v[b] + (y);                \
        v[d] = ob2s_rotr(v[d] ^ v[a], 8);        \
        v[c] = v[c] + v[d];                      \
        v[b] = ob2s_rotr(v[b] ^ v[c], 7);        \
    } while (0)
    for (int r = 0; r < 10; ++r) {
        const uint8_t *sg = OB2S_SIGMA[r];
        OB2S_G(0, 4, 8, 12, m[sg[0]], m[sg[1]]);
        OB2S_G(1, 5, 9, 13, m[sg[2]], m[sg[3]]);
        OB2S_G(2, 6, 10, 14, m[sg[4]], m[sg[5]]);
        OB2S_G(3, 7, 11, 15, m[sg[6]], m[sg[7]]);
        OB2S_G(0, 5, 10, 15, m[sg[8]], m[sg[9]]);
        OB2S_G(1, 6, 11, 12, m[sg[10]], m[sg[11]]);
        OB2S_G(2, 7, 8, 13, m[sg[12]], m[sg[13]]);
        OB2S_G(3, 4, 9, 14, m[sg[14]], m[sg[15]]);
    }
#undef OB2S_G
    for (int i = 0; i < 8; ++i) s->h[i] ^= v[i] ^ v[i + 8];
}

static inline void ob2s_init(ob2s_t *s) {
    memcpy(s->h, OB2S_IV, sizeof s->h);
    s->h[0] ^= 0x01010000u ^ 32u; /* key length 0, digest length 32 */
    s->t[0] = s->t[1] = 0;
    s->buflen = 0;
}

static inline void ob2s_inc(ob2s_t *s, uint32_t k) {
    s->t[0] += k;
    if (s->t[0] < k) s->t[1]++;
}

static inline void ob2s_update(ob2s_t *s, const void *data, size_t len) {
    const uint8_t *p = (const uint8_t *)data;
    while (len > 0) {
        if (s->buflen == 64) {
            ob2s_inc(s, 64);
            ob2s_compress(s, s->buf, 0);
            s->buflen = 0;
        }
        size_t k = 64 - s->buflen;
        if (k > len) k = len;
        memcpy(s->buf + s->buflen, p, k);
        s->buflen += k;
        p += k;
        len -= k;
    }
}

/* finalize a COPY of the state (the state itself is unchanged) */
static inline void ob2s_peek(const ob2s_t *s0, uint8_t out[32]) {
    ob2s_t s = *s0;
    ob2s_inc(&s, (uint32_t)s.buflen);
    memset(s.buf + s.buflen, 0, 64 - s.buflen);
    ob2s_compress(&s, s.buf, 1);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)s.h[i];
        out[4 * i + 1] = (uint8_t)(s.h[i] >> 8);
        out[4 * i + 2] = (uint8_t)(s.h[i] >> 16);
        out[4 * i + 3] = (uint8_t)(s.h[i] >> 24);
    }
}
#endif
