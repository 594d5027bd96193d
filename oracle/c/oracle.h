/* ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * C-ABI of the reference-faithful C CPU prover (liboracle.so). Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may load it — as the CHECKER / the timed CPU
 * baseline, never as the product path.
 *
 * Byte conventions (same as the product ABI, include/spartan_hip.h):
 *   Fr      32-byte little-endian canonical (ark-serialize)
 *   G1/G2   96/192-byte ark-serialize UNCOMPRESSED affine points
 *   CSR     row_ptr[n+1] (u64), col[nnz] (u32), val[nnz] (Fr bytes); row order and the order
 *           of entries inside a row are the `Matrix<F>` order (they are hashed).
 */
#ifndef ORACLE_H
#define ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint64_t n;
    const uint64_t *row_ptr;
    const uint32_t *col;
    const uint8_t *val;
} orc_csr;

typedef struct orc_inst orc_inst;
typedef struct orc_pp orc_pp;

/* ---- synthetic instances (oracle/py/gen.py, draw for draw) ---- */
enum { ORC_GEN_UNIFORM_3N = 0, ORC_GEN_REF_SHAPED = 1, ORC_GEN_RAGGED = 2, ORC_GEN_CIRCUIT_3N = 3 /* param = witness seed */ };
orc_inst *orc_gen(int kind, int log_n, int log_v, uint64_t seed, uint64_t param);
uint64_t orc_inst_nnz(const orc_inst *I, int m);
int orc_inst_log_v(const orc_inst *I);
void orc_inst_export(const orc_inst *I, int m, uint64_t *row_ptr, uint32_t *col, uint8_t *val);
void orc_inst_z(const orc_inst *I, uint8_t *z_out);
void orc_inst_free(orc_inst *I);

/* ---- public parameters (commitment/setup.rs:27-105) ---- */
orc_pp *orc_keygen(int nv, uint64_t seed);
orc_pp *orc_pp_load(const uint8_t *bytes, size_t len);
size_t orc_pp_serialize(const orc_pp *pp, uint8_t *out, size_t cap);
void orc_pp_trapdoor(const orc_pp *pp, uint8_t *t_out);
void orc_pp_free(orc_pp *pp);

/* ---- hot-path functions (kernel-level checkers) ---- */
void orc_sum_over_y(const orc_csr *M, const uint8_t *z, uint8_t *out);
void orc_eval_on_x(const orc_csr *M, const uint8_t *r_x, uint8_t *out);
void orc_msm_g1(const uint8_t *bases, const uint8_t *scalars, size_t n, uint8_t *out96);
void orc_msm_g2(const uint8_t *bases, const uint8_t *scalars, size_t n, uint8_t *out192);
void orc_commit(const orc_pp *pp, const uint8_t *table, int nv, uint8_t *out56);
/* proof_out receives Proof{h, proofs} compressed: 96 + 8 + 96 nv bytes */
void orc_open(const orc_pp *pp, const uint8_t *table, int nv, const uint8_t *point, uint8_t *eval_out,
              uint8_t *proof_out);

/* ---- full-size checkers (tests): final matrix claim, openings against the keygen trapdoor ---- */
void orc_matrix_eval(const orc_csr *M, const uint8_t *r_x, const uint8_t *r_y, uint8_t *out);
void orc_open_trapdoor(const uint8_t *table, int nv, const uint8_t *point, const uint8_t *t, uint8_t *qv_out,
                       uint8_t *eval_out);
void orc_mle_eval(const uint8_t *table, int nv, const uint8_t *point, uint8_t *out);

/* ---- full argument (lib.rs:58-146) ----
 * mode 0 = Fiat-Shamir (Blake2s512Rng transcript), 1 = injected challenges (SplitMix64(inj_seed));
 * OR 2 = commitment stubbed (BASELINE config C2: identity commitment and opening proofs, no MSM,
 * pp may be NULL).
 * Returns 0 on success, else an error code (1 = InvalidArgument ...); *out_len = proof length. */
int orc_prove(const orc_csr *A, const orc_csr *B, const orc_csr *C, const uint8_t *v, size_t nv_len,
              const uint8_t *w, size_t nw_len, const orc_pp *pp, int mode, uint64_t inj_seed, uint8_t *out,
              size_t cap, size_t *out_len);
const char *orc_last_error(void);
/* OpenMP threads for the MSM windows and sumcheck rounds (default 1: the reference is single-threaded) */
void orc_set_threads(int k);
int orc_get_threads(void);

#ifdef __cplusplus
}
#endif
#endif
