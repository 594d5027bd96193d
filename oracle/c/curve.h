/* ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Short-Weierstrass Jacobian arithmetic for BLS12-381 G1 (over Fq, b = 4) and G2
 * (over Fq2, b = 4(u+1)), restating ark-ec's `short_weierstrass_jacobian` [upstream]:
 * doubling dbl-2009-l, addition add-2007-bl, mixed addition madd-2007-bl; affine points
 * carry an `infinity` flag. Instantiated twice by DEFINE_CURVE below.
 */
#ifndef ORACLE_CURVE_H
#define ORACLE_CURVE_H
#include "ff.h"

#define DEFINE_CURVE(G, F)                                                                  \
    typedef struct { F##_t x, y; int inf; } G##_aff;                                         \
    typedef struct { F##_t x, y, z; } G##_jac;                                               \
    static inline void G##_set_inf(G##_jac *p) {                                             \
        F##_one(&p->x); F##_one(&p->y); F##_zero(&p->z);                                     \
    }                                                                                        \
    static inline int G##_is_inf(const G##_jac *p) { return F##_is_zero(&p->z); }            \
    static inline void G##_from_aff(G##_jac *r, const G##_aff *a) {                          \
        if (a->inf) { G##_set_inf(r); return; }                                              \
        r->x = a->x; r->y = a->y; F##_one(&r->z);                                            \
    }                                                                                        \
    static inline void G##_dbl(G##_jac *r, const G##_jac *p) {                               \
        if (G##_is_inf(p)) { *r = *p; return; }                                              \
        F##_t A, B, C, D, E, Fv, t, X3, Y3, Z3;                                              \
        F##_sqr(&A, &p->x);                                                                  \
        F##_sqr(&B, &p->y);                                                                  \
        F##_sqr(&C, &B);                                                                     \
        F##_add(&t, &p->x, &B); F##_sqr(&t, &t); F##_sub(&t, &t, &A); F##_sub(&t, &t, &C);   \
        F##_add(&D, &t, &t);                                                                 \
        F##_add(&E, &A, &A); F##_add(&E, &E, &A);                                            \
        F##_sqr(&Fv, &E);                                                                    \
        F##_add(&t, &D, &D); F##_sub(&X3, &Fv, &t);                                          \
        F##_add(&C, &C, &C); F##_add(&C, &C, &C); F##_add(&C, &C, &C);                       \
        F##_sub(&t, &D, &X3); F##_mul(&t, &E, &t); F##_sub(&Y3, &t, &C);                     \
        F##_mul(&Z3, &p->y, &p->z); F##_add(&Z3, &Z3, &Z3);                                  \
        r->x = X3; r->y = Y3; r->z = Z3;                                                     \
    }                                                                                        \
    static inline void G##_add(G##_jac *r, const G##_jac *p, const G##_jac *q) {             \
        if (G##_is_inf(p)) { *r = *q; return; }                                              \
        if (G##_is_inf(q)) { *r = *p; return; }                                              \
        F##_t Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, rr, V, t;                                 \
        F##_sqr(&Z1Z1, &p->z); F##_sqr(&Z2Z2, &q->z);                                        \
        F##_mul(&U1, &p->x, &Z2Z2); F##_mul(&U2, &q->x, &Z1Z1);                              \
        F##_mul(&S1, &p->y, &q->z); F##_mul(&S1, &S1, &Z2Z2);                                \
        F##_mul(&S2, &q->y, &p->z); F##_mul(&S2, &S2, &Z1Z1);                                \
        if (F##_eq(&U1, &U2)) {                                                              \
            if (F##_eq(&S1, &S2)) { G##_dbl(r, p); return; }                                 \
            G##_set_inf(r); return;                                                          \
        }                                                                                    \
        F##_sub(&H, &U2, &U1);                                                               \
        F##_add(&I, &H, &H); F##_sqr(&I, &I);                                                \
        F##_mul(&J, &H, &I);                                                                 \
        F##_sub(&rr, &S2, &S1); F##_add(&rr, &rr, &rr);                                      \
        F##_mul(&V, &U1, &I);                                                                \
        G##_jac o;                                                                           \
        F##_sqr(&o.x, &rr); F##_sub(&o.x, &o.x, &J); F##_sub(&o.x, &o.x, &V);                \
        F##_sub(&o.x, &o.x, &V);                                                             \
        F##_sub(&t, &V, &o.x); F##_mul(&o.y, &rr, &t);                                       \
        F##_mul(&S1, &S1, &J); F##_add(&S1, &S1, &S1); F##_sub(&o.y, &o.y, &S1);             \
        F##_add(&t, &p->z, &q->z); F##_sqr(&t, &t); F##_sub(&t, &t, &Z1Z1);                  \
        F##_sub(&t, &t, &Z2Z2); F##_mul(&o.z, &t, &H);                                       \
        *r = o;                                                                              \
    }                                                                                        \
    static inline void G##_madd(G##_jac *r, const G##_jac *p, const G##_aff *q) {            \
        if (q->inf) { *r = *p; return; }                                                     \
        if (G##_is_inf(p)) { G##_from_aff(r, q); return; }                                   \
        F##_t Z1Z1, U2, S2, H, HH, I, J, rr, V, t;                                           \
        F##_sqr(&Z1Z1, &p->z);                                                               \
        F##_mul(&U2, &q->x, &Z1Z1);                                                          \
        F##_mul(&S2, &q->y, &p->z); F##_mul(&S2, &S2, &Z1Z1);                                \
        if (F##_eq(&U2, &p->x)) {                                                            \
            if (F##_eq(&S2, &p->y)) { G##_dbl(r, p); return; }                               \
            G##_set_inf(r); return;                                                          \
        }                                                                                    \
        F##_sub(&H, &U2, &p->x);                                                             \
        F##_sqr(&HH, &H);                                                                    \
        F##_add(&I, &HH, &HH); F##_add(&I, &I, &I);                                          \
        F##_mul(&J, &H, &I);                                                                 \
        F##_sub(&rr, &S2, &p->y); F##_add(&rr, &rr, &rr);                                    \
        F##_mul(&V, &p->x, &I);                                                              \
        G##_jac o;                                                                           \
        F##_sqr(&o.x, &rr); F##_sub(&o.x, &o.x, &J); F##_sub(&o.x, &o.x, &V);                \
        F##_sub(&o.x, &o.x, &V);                                                             \
        F##_sub(&t, &V, &o.x); F##_mul(&o.y, &rr, &t);                                       \
        F##_mul(&t, &p->y, &J); F##_add(&t, &t, &t); F##_sub(&o.y, &o.y, &t);                \
        F##_add(&t, &p->z, &H); F##_sqr(&t, &t); F##_sub(&t, &t, &Z1Z1);                     \
        F##_sub(&o.z, &t, &HH);                                                              \
        *r = o;                                                                              \
    }                                                                                        \
    static inline void G##_neg_jac(G##_jac *r, const G##_jac *p) {                           \
        *r = *p; F##_neg(&r->y, &p->y);                                                      \
    }                                                                                        \
    static inline void G##_to_aff(G##_aff *r, const G##_jac *p) {                            \
        if (G##_is_inf(p)) { F##_zero(&r->x); F##_one(&r->y); r->inf = 1; return; }          \
        F##_t zi, zi2;                                                                       \
        F##_inv(&zi, &p->z); F##_sqr(&zi2, &zi);                                             \
        F##_mul(&r->x, &p->x, &zi2); F##_mul(&zi2, &zi2, &zi); F##_mul(&r->y, &p->y, &zi2);  \
        r->inf = 0;                                                                          \
    }                                                                                        \
    /* ark-ec batch_normalization_into_affine: one inversion per batch */                   \
    static inline void G##_batch_to_aff(G##_aff *out, const G##_jac *in, size_t n) {         \
        F##_t *pre = (F##_t *)malloc(sizeof(F##_t) * (n ? n : 1));                           \
        F##_t acc, inv, zi, zi2;                                                             \
        F##_one(&acc);                                                                       \
        for (size_t i = 0; i < n; ++i) {                                                     \
            pre[i] = acc;                                                                    \
            if (!G##_is_inf(&in[i])) F##_mul(&acc, &acc, &in[i].z);                          \
        }                                                                                    \
        F##_inv(&inv, &acc);                                                                 \
        for (size_t k = n; k-- > 0;) {                                                       \
            if (G##_is_inf(&in[k])) {                                                        \
                F##_zero(&out[k].x); F##_one(&out[k].y); out[k].inf = 1; continue;           \
            }                                                                                \
            F##_mul(&zi, &inv, &pre[k]);                                                     \
            F##_mul(&inv, &inv, &in[k].z);                                                   \
            F##_sqr(&zi2, &zi);                                                              \
            F##_mul(&out[k].x, &in[k].x, &zi2);                                              \
            F##_mul(&zi2, &zi2, &zi);                                                        \
            F##_mul(&out[k].y, &in[k].y, &zi2);                                              \
            out[k].inf = 0;                                                                  \
        }                                                                                    \
        free(pre);                                                                           \
    }                                                                                        \
    /* scalar given as canonical 4 x u64 */                                                  \
    static inline void G##_mul_canon(G##_jac *r, const G##_jac *p, const uint64_t *k) {      \
        G##_jac acc;                                                                         \
        G##_set_inf(&acc);                                                                   \
        for (int i = 3; i >= 0; --i)                                                         \
            for (int b = 63; b >= 0; --b) {                                                  \
                G##_dbl(&acc, &acc);                                                         \
                if ((k[i] >> b) & 1) G##_add(&acc, &acc, p);                                 \
            }                                                                                \
        *r = acc;                                                                            \
    }

#include <stdlib.h>
DEFINE_CURVE(g1, fq)
DEFINE_CURVE(g2, fq2)

#endif
