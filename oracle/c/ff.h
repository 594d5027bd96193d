/* ORACLE — TEST INFRASTRUCTURE ONLY (C restatement; CPU baseline + large-size checker).
 *
 * BLS12-381 field arithmetic as in ark-ff / ark-bls12-381 [upstream, not in container]:
 * Fr = 4 x u64 Montgomery (R = 2^256), Fq = 6 x u64 Montgomery (R = 2^384),
 * Fq2 = Fq[u]/(u^2 + 1). Single-threaded CIOS Montgomery multiplication (the reference runs
 * ark-ff's portable code single-threaded, /root/reference/Cargo.toml:10-27: no `asm`,
 * no `parallel`). Constants generated from the moduli by oracle/py/bls12_381.py.
 */
#ifndef ORACLE_FF_H
#define ORACLE_FF_H
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;

typedef struct { uint64_t v[4]; } fr_t;
typedef struct { uint64_t v[6]; } fq_t;
typedef struct { fq_t c0, c1; } fq2_t;

static const uint64_t FR_P[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL};
static const uint64_t FR_R2[4] = {0xc999e990f3f29c6dULL, 0x2b6cedcb87925c23ULL, 0x05d314967254398fULL, 0x0748d9d99f59ff11ULL};
static const uint64_t FR_ONE[4] = {0x00000001fffffffeULL, 0x5884b7fa00034802ULL, 0x998c4fefecbc4ff5ULL, 0x1824b159acc5056fULL};
static const uint64_t FR_INV = 0xfffffffeffffffffULL;
static const uint64_t FQ_P[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL, 0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const uint64_t FQ_R2[6] = {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL, 0x8de5476c4c95b6d5ULL, 0x67eb88a9939d83c0ULL, 0x9a793e85b519952dULL, 0x11988fe592cae3aaULL};
static const uint64_t FQ_ONE[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL, 0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
static const uint64_t FQ_INV = 0x89f3fffcfffcfffdULL;

/* ---- generic N-limb helpers, instantiated for N = 4 (Fr) and 6 (Fq) ---- */
#define DEFINE_FIELD(T, N, P, R2, ONE, INV)                                                   \
    static inline int T##_geq_p(const uint64_t *a) {                                       \
        for (int i = N - 1; i >= 0; --i) {                                                   \
            if (a[i] != P[i]) return a[i] > P[i];                                            \
        }                                                                                    \
        return 1;                                                                            \
    }                                                                                        \
    static inline void T##_sub_p(uint64_t *a) {                                              \
        uint64_t br = 0;                                                                     \
        for (int i = 0; i < N; ++i) {                                                        \
            u128 d = (u128)a[i] - P[i] - br;                                                 \
            a[i] = (uint64_t)d;                                                              \
            br = (uint64_t)(d >> 64) & 1;                                                    \
        }                                                                                    \
    }                                                                                        \
    static inline void T##_mul(T##_t *r, const T##_t *a, const T##_t *b) {                 \
        uint64_t t[N + 2];                                                                   \
        memset(t, 0, sizeof(t));                                                             \
        for (int i = 0; i < N; ++i) {                                                        \
            u128 c = 0;                                                                      \
            uint64_t bi = b->v[i];                                                           \
            for (int j = 0; j < N; ++j) {                                                    \
                c = (u128)a->v[j] * bi + t[j] + (c >> 64);                                   \
                t[j] = (uint64_t)c;                                                          \
            }                                                                                \
            c = (u128)t[N] + (c >> 64);                                                      \
            t[N] = (uint64_t)c;                                                              \
            t[N + 1] = (uint64_t)(c >> 64);                                                  \
            uint64_t m = t[0] * INV;                                                         \
            c = (u128)m * P[0] + t[0];                                                       \
            for (int j = 1; j < N; ++j) {                                                    \
                c = (u128)m * P[j] + t[j] + (c >> 64);                                       \
                t[j - 1] = (uint64_t)c;                                                      \
            }                                                                                \
            c = (u128)t[N] + (c >> 64);                                                      \
            t[N - 1] = (uint64_t)c;                                                          \
            t[N] = t[N + 1] + (uint64_t)(c >> 64);                                           \
        }                                                                                    \
        if (t[N] || T##_geq_p(t)) T##_sub_p(t);                                              \
        memcpy(r->v, t, 8 * N);                                                              \
    }                                                                                        \
    static inline void T##_sqr(T##_t *r, const T##_t *a) { T##_mul(r, a, a); }               \
    static inline void T##_add(T##_t *r, const T##_t *a, const T##_t *b) {                   \
        uint64_t t[N];                                                                       \
        uint64_t c = 0;                                                                      \
        for (int i = 0; i < N; ++i) {                                                        \
            u128 s = (u128)a->v[i] + b->v[i] + c;                                            \
            t[i] = (uint64_t)s;                                                              \
            c = (uint64_t)(s >> 64);                                                         \
        }                                                                                    \
        if (c || T##_geq_p(t)) T##_sub_p(t);                                                 \
        memcpy(r->v, t, 8 * N);                                                              \
    }                                                                                        \
    static inline void T##_sub(T##_t *r, const T##_t *a, const T##_t *b) {                   \
        uint64_t t[N];                                                                       \
        uint64_t br = 0;                                                                     \
        for (int i = 0; i < N; ++i) {                                                        \
            u128 d = (u128)a->v[i] - b->v[i] - br;                                           \
            t[i] = (uint64_t)d;                                                              \
            br = (uint64_t)(d >> 64) & 1;                                                    \
        }                                                                                    \
        if (br) {                                                                            \
            uint64_t c = 0;                                                                  \
            for (int i = 0; i < N; ++i) {                                                    \
                u128 s = (u128)t[i] + P[i] + c;                                              \
                t[i] = (uint64_t)s;                                                          \
                c = (uint64_t)(s >> 64);                                                     \
            }                                                                                \
        }                                                                                    \
        memcpy(r->v, t, 8 * N);                                                              \
    }                                                                                        \
    static inline int T##_is_zero(const T##_t *a) {                                          \
        uint64_t acc = 0;                                                                    \
        for (int i = 0; i < N; ++i) acc |= a->v[i];                                          \
        return acc == 0;                                                                     \
    }                                                                                        \
    static inline int T##_eq(const T##_t *a, const T##_t *b) {                               \
        return memcmp(a->v, b->v, 8 * N) == 0;                                               \
    }                                                                                        \
    static inline void T##_neg(T##_t *r, const T##_t *a) {                                   \
        T##_t z;                                                                             \
        memset(&z, 0, sizeof z);                                                             \
        T##_sub(r, &z, a);                                                                   \
    }                                                                                        \
    static inline void T##_zero(T##_t *r) { memset(r, 0, sizeof *r); }                       \
    static inline void T##_one(T##_t *r) { memcpy(r->v, ONE, 8 * N); }                       \
    /* canonical little-endian integer (< p) -> Montgomery */                                \
    static inline void T##_from_canon(T##_t *r, const uint64_t *c) {                         \
        T##_t a, r2;                                                                         \
        memcpy(a.v, c, 8 * N);                                                               \
        memcpy(r2.v, R2, 8 * N);                                                             \
        T##_mul(r, &a, &r2);                                                                 \
    }                                                                                        \
    static inline void T##_to_canon(uint64_t *c, const T##_t *a) {                           \
        T##_t one_raw, r;                                                                    \
        memset(&one_raw, 0, sizeof one_raw);                                                 \
        one_raw.v[0] = 1;                                                                    \
        T##_mul(&r, a, &one_raw);                                                            \
        memcpy(c, r.v, 8 * N);                                                               \
    }                                                                                        \
    static inline void T##_from_u64(T##_t *r, uint64_t x) {                                  \
        uint64_t c[N];                                                                       \
        memset(c, 0, sizeof c);                                                              \
        c[0] = x;                                                                            \
        T##_from_canon(r, c);                                                                \
    }                                                                                        \
    static inline void T##_pow(T##_t *r, const T##_t *a, const uint64_t *e, int ne) {        \
        T##_t acc;                                                                           \
        T##_one(&acc);                                                                       \
        for (int i = ne - 1; i >= 0; --i)                                                    \
            for (int b = 63; b >= 0; --b) {                                                  \
                T##_sqr(&acc, &acc);                                                         \
                if ((e[i] >> b) & 1) T##_mul(&acc, &acc, a);                                 \
            }                                                                                \
        *r = acc;                                                                            \
    }                                                                                        \
    static inline void T##_inv(T##_t *r, const T##_t *a) {                                   \
        uint64_t e[N];                                                                       \
        memcpy(e, P, 8 * N);                                                                 \
        e[0] -= 2; /* p is odd and > 2: no borrow */                                         \
        T##_pow(r, a, e, N);                                                                 \
    }

DEFINE_FIELD(fr, 4, FR_P, FR_R2, FR_ONE, FR_INV)
DEFINE_FIELD(fq, 6, FQ_P, FQ_R2, FQ_ONE, FQ_INV)

/* ---- Fr byte I/O: 32-B LE canonical (ark-serialize) ---- */
static inline int fr_from_bytes(fr_t *r, const uint8_t *b) {
    uint64_t c[4];
    memcpy(c, b, 32);
    if (fr_geq_p(c)) return -1;
    fr_from_canon(r, c);
    return 0;
}
static inline void fr_to_bytes(uint8_t *b, const fr_t *a) {
    uint64_t c[4];
    fr_to_canon(c, a);
    memcpy(b, c, 32);
}
/* compare canonical integers: a > b */
static inline int fq_canon_gt(const fq_t *a, const fq_t *b) {
    uint64_t x[6], y[6];
    fq_to_canon(x, a);
    fq_to_canon(y, b);
    for (int i = 5; i >= 0; --i)
        if (x[i] != y[i]) return x[i] > y[i];
    return 0;
}

/* ---- Fq2 ---- */
static inline void fq2_add(fq2_t *r, const fq2_t *a, const fq2_t *b) {
    fq_add(&r->c0, &a->c0, &b->c0);
    fq_add(&r->c1, &a->c1, &b->c1);
}
static inline void fq2_sub(fq2_t *r, const fq2_t *a, const fq2_t *b) {
    fq_sub(&r->c0, &a->c0, &b->c0);
    fq_sub(&r->c1, &a->c1, &b->c1);
}
static inline void fq2_neg(fq2_t *r, const fq2_t *a) {
    fq_neg(&r->c0, &a->c0);
    fq_neg(&r->c1, &a->c1);
}
static inline void fq2_mul(fq2_t *r, const fq2_t *a, const fq2_t *b) {
    fq_t t0, t1, s0, s1, m;
    fq_mul(&t0, &a->c0, &b->c0);
    fq_mul(&t1, &a->c1, &b->c1);
    fq_add(&s0, &a->c0, &a->c1);
    fq_add(&s1, &b->c0, &b->c1);
    fq_mul(&m, &s0, &s1);
    fq_sub(&r->c0, &t0, &t1);
    fq_sub(&m, &m, &t0);
    fq_sub(&r->c1, &m, &t1);
}
static inline void fq2_sqr(fq2_t *r, const fq2_t *a) {
    fq_t s, d, p;
    fq_add(&s, &a->c0, &a->c1);
    fq_sub(&d, &a->c0, &a->c1);
    fq_mul(&p, &a->c0, &a->c1);
    fq_mul(&r->c0, &s, &d);
    fq_add(&r->c1, &p, &p);
}
static inline int fq2_is_zero(const fq2_t *a) { return fq_is_zero(&a->c0) && fq_is_zero(&a->c1); }
static inline int fq2_eq(const fq2_t *a, const fq2_t *b) { return fq_eq(&a->c0, &b->c0) && fq_eq(&a->c1, &b->c1); }
static inline void fq2_zero(fq2_t *r) { fq_zero(&r->c0); fq_zero(&r->c1); }
static inline void fq2_one(fq2_t *r) { fq_one(&r->c0); fq_zero(&r->c1); }
static inline void fq2_inv(fq2_t *r, const fq2_t *a) {
    fq_t t0, t1, n;
    fq_sqr(&t0, &a->c0);
    fq_sqr(&t1, &a->c1);
    fq_add(&n, &t0, &t1);
    fq_inv(&n, &n);
    fq_mul(&r->c0, &a->c0, &n);
    fq_mul(&t1, &a->c1, &n);
    fq_neg(&r->c1, &t1);
}
/* ark-ff Ord on QuadExtField: c1 first, then c0 */
static inline int fq2_canon_gt(const fq2_t *a, const fq2_t *b) {
    if (!fq_eq(&a->c1, &b->c1)) return fq_canon_gt(&a->c1, &b->c1);
    return fq_canon_gt(&a->c0, &b->c0);
}

#endif
