/* spartan_hip — MI355X-native drop-in for the proving hot path of tsunrise/r1cs-spartan.
 *
 * C ABI of libspartan_hip.so. Every entry point returns an spx_status; on failure
 * spx_last_error() holds a thread-local message. No torch / HIP types cross this boundary:
 * plain pointers, sizes and byte images.
 *
 * Byte conventions (ark-serialize, the reference's own wire format):
 *   Fr        32-byte little-endian canonical integer (`into_repr` bytes)
 *   G1 / G2   96 / 192-byte UNCOMPRESSED affine points (public-parameter files),
 *             48 / 96-byte COMPRESSED points inside proofs
 *   Matrix    CSR: row_ptr[n+1] (u64), col[nnz] (u32), val[nnz] (Fr bytes); the row order and
 *             the order of entries inside a row are the `ark_relations::r1cs::Matrix<F>` order
 *             (they are hashed into the Fiat-Shamir transcript, /root/reference/src/lib.rs:61-64).
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   spx_index            MLArgumentForR1CS::index                 src/lib.rs:45-51 -> src/ahp/indexer.rs:41-64
 *   spx_prove            MLArgumentForR1CS::prove                 src/lib.rs:58-146
 *   spx_verify           MLArgumentForR1CS::verify                src/lib.rs:147-212
 *   spx_pp_load          PublicParameter (CanonicalDeserialize)   src/commitment/data_structures.rs:9-17
 *   spx_pp_generate      MLProofForR1CS::setup / MLPolyCommit::keygen  src/ahp/setup.rs:13-16, src/commitment/setup.rs:27-105
 *   spx_commit           MLPolyCommit::commit                     src/commitment/commit.rs:17-29
 *   spx_open             MLPolyCommit::open                       src/commitment/open.rs:19-58
 *   spx_sum_over_y       MatrixExtension::sum_over_y              src/data_structures/r1cs_reader.rs:75-85
 *   spx_eval_on_x        MatrixExtension::eval_on_x               src/data_structures/r1cs_reader.rs:91-117
 *   spx_msm_g1 / _g2     ark-ec VariableBaseMSM::multi_scalar_mul (called at commit.rs:25, open.rs:49)
 *   spx_prover_*, spx_prove_*_round   the round-level prover API  src/ahp/prover.rs:109-281
 *   spx_sumcheck_round   AHPForMLSumcheck::prove_round [linear-sumcheck] (called at prover.rs:204, 263)
 * Errors mirror src/error.rs:5-14 (Display is todo!() there; here a message string).
 */
#ifndef SPARTAN_HIP_H
#define SPARTAN_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SPX_OK = 0,
    SPX_INVALID_ARGUMENT = 1, /* Error::InvalidArgument */
    SPX_SUMCHECK = 2,         /* Error::SumCheckError */
    SPX_WRONG_WITNESS = 3,    /* Error::WrongWitness */
    SPX_SERIALIZATION = 4,    /* Error::SerializationError */
    SPX_DEVICE = 5            /* HIP / RCCL failure (no reference counterpart) */
} spx_status;

typedef struct spx_ctx spx_ctx;         /* one GPU (one rank): stream, workspaces, communicator */
typedef struct spx_pp spx_pp;           /* device-resident public parameters (+ window tables) */
typedef struct spx_pk spx_pk;           /* prover key (IndexPK): matrices on host (transcript) and device */
typedef struct spx_witness spx_witness; /* z = v || w resident in HBM */

typedef struct {
    uint64_t n;               /* rows (= number of constraints) */
    const uint64_t *row_ptr;  /* n + 1 */
    const uint32_t *col;      /* nnz */
    const uint8_t *val;       /* 32 * nnz */
} spx_csr;

typedef enum { SPX_FS = 0, SPX_INJECTED = 1 } spx_mode;

typedef struct {
    int mode;            /* SPX_FS: Blake2s512Rng Fiat-Shamir (reference); SPX_INJECTED: SplitMix64(inj_seed) */
    uint64_t inj_seed;
    int cached_matrix_transcript; /* 1: resume the Blake2s state absorbed at spx_index time (bit-identical) */
    int commitment_stub; /* 1: BASELINE config C2, "sumcheck-only, commitment stubbed": the proof prove()
                            gives under a public parameter whose every group element is the identity
                            (commitment, h and opening proofs = infinity; the z evaluations are still
                            computed). No MSM runs and pp may be NULL. Not a sound proof: benchmark /
                            parity mode of the sumcheck half of lib.rs:58-146. */
} spx_prove_opts;

const char *spx_last_error(void);
const char *spx_version(void);

/* ---- context / multi-GPU ---- */
int spx_ctx_create(int device, spx_ctx **out);
int spx_ctx_destroy(spx_ctx *ctx);
/* RCCL (one process per GPU): rank 0 calls spx_comm_unique_id, broadcasts the 128 bytes out of band
 * (e.g. torch.distributed), then every rank creates ONE hub on it (spx_comm_hub_create_rccl) and
 * attaches each of its contexts to a channel (spx_ctx_set_comm_hub): context j of every rank on
 * channel j (0..63). The hub's thread is the only caller of the communicator and matches the
 * channels' exchanges across ranks in rounds every rank runs identically, so any number of proofs in
 * flight share one communicator without collective-ordering deadlocks.
 * spx_ctx_set_comm_rccl is the one-context shorthand (a private hub, channel 0).
 * Replaces the reference's single-threaded prove (/root/reference/src/lib.rs:58-146), which has
 * no exchange; the exchange schedule is DESIGN.md §6. */
int spx_comm_unique_id(uint8_t id_out[128]);
int spx_ctx_set_comm_rccl(spx_ctx *ctx, const uint8_t id[128], int rank, int world);
int spx_comm_hub_create_rccl(const uint8_t id[128], int rank, int world, int device, void **hub_out);
/* the same hub over the shared-memory transport (one segment per rank set instead of one per
 * context), and over the in-process test group (virtual ranks as host threads; spx_comm_group_create) */
int spx_comm_hub_create_shm(const char *name, int rank, int world, void **hub_out);
int spx_comm_hub_create_group(void *group, int rank, void **hub_out);
/* ... and over a caller-provided collective (e.g. a torch.distributed process group: gloo on the CPU,
 * RCCL = backend "nccl" on MI355X): fn(user, send, recv, bytes) must gather `bytes` from every rank of
 * the caller's group into recv in rank order and return 0 (non-zero fails the exchange with
 * SPX_DEVICE); rank / world are the caller's group's. Only the hub's thread calls fn, in the same
 * sequence on every rank. */
typedef int (*spx_allgather_fn)(void *user, const void *send, void *recv, size_t bytes);
int spx_comm_hub_create_callback(spx_allgather_fn fn, void *user, int rank, int world, void **hub_out);
int spx_ctx_set_comm_hub(spx_ctx *ctx, void *hub, int channel);
/* one exchange on `channel` without a context (transport tests); blocks until every rank posted it */
int spx_comm_hub_allgather(void *hub, int channel, const void *send, void *recv, size_t bytes);
/* out[0] control rounds, out[1] data rounds, out[2] exchanges served, out[3] largest batch per round,
 * out[4] idle rounds (matched nothing: a peer had not reached the exchange yet; each is followed by a
 * 50 us back-off or the next local request) */
int spx_comm_hub_stats(void *hub, uint64_t out[5]);
int spx_comm_hub_destroy(void *hub); /* contexts attached keep the hub alive until they are destroyed */
/* On-node shared-memory communicator (default for one process per GPU on one host): every rank
 * passes the same `name` (rank 0 makes it unique, e.g. "spx_<random hex>_<k>", and distributes it
 * out of band), one name per context. The exchanges of a sharded proof are host-side and tiny, so
 * no GPU queue is involved (multi-GPU). The standalone form is a host-only
 * allgather (tests, other transports' validation). */
int spx_ctx_set_comm_shm(spx_ctx *ctx, const char *name, int rank, int world);
int spx_comm_shm_create(const char *name, int rank, int world, void **comm_out);
int spx_comm_shm_allgather(void *comm, const void *send, void *recv, size_t bytes);
int spx_comm_shm_destroy(void *comm);
/* In-process test communicator: `world` contexts sharing one exchange object (shards of one proof
 * driven by `world` host threads). group_create returns a handle; each ctx joins with its rank. */
int spx_comm_group_create(int world, void **group_out);
int spx_comm_group_destroy(void *group);
int spx_ctx_set_comm_group(spx_ctx *ctx, void *group, int rank);
/* Rehearsal: this context acts as rank `rank` of a `world`-rank proof-sharded prove WITHOUT peers
 * (every exchange returns its own contribution in all slots): the device and host work of one rank
 * on a GPU of its own, for throughput estimates of an N-GPU node. Its proofs are not valid. */
int spx_ctx_set_comm_rehearsal(spx_ctx *ctx, int rank, int world);
/* Where the shared level-0 opening MSM of a proof runs (no effect on the proof bytes): 0 = beside the
 * commitment (its own MSM pipeline, the default), 1 = inside the first opening's MSM batch (one MSM
 * pipeline less per proof: sort, weighting tree), -1 = the process default (SPX_LVL0=batch -> 1).
 * Every rank of a proof-sharded prove must use the same mode (checked on the context's first sharded
 * proof: SPX_INVALID_ARGUMENT otherwise). */
int spx_ctx_set_lvl0_batch(spx_ctx *ctx, int mode);
/* one allgather on the context's communicator (whatever its transport): every rank passes `bytes`,
 * recv receives world * bytes in rank order. For transport tests. */
int spx_ctx_comm_allgather(spx_ctx *ctx, const void *send, void *recv, size_t bytes);

/* How this context's host waits for its stream (no effect on the proof bytes): us > 0 polls an event
 * every us microseconds (frees the host cores the HSA runtime's spinning wait would take: BASELINE C2
 * with matrices absorbed per proof, sharded ranks), 0 = hipStreamSynchronize, -1 = the process default
 * (SPX_SYNC_POLL_US, else 0). */
int spx_ctx_set_sync_poll(spx_ctx *ctx, int us);
/* Lockstep groups for spx_prove_many (no effect on the proof bytes): with k > 1 (at most 16) the
 * context's stubbed-commitment proofs on an unsharded context (BASELINE C2) run k at a time in
 * lockstep: each sumcheck round of the k proofs is one launch (blockIdx.y = proof) with one host wait,
 * and the other steps queue the k proofs' launches before one wait. Other proofs, and
 * k = 1 (the default), run one at a time. Replaces nothing in the reference (its prove is one proof,
 * /root/reference/src/lib.rs:58-146); each proof's bytes are that prove's. */
int spx_ctx_set_group(spx_ctx *ctx, int k);
/* free and total bytes of the context's device (hipMemGetInfo): bench.py sizes the proofs in flight
 * per rank from it (each context keeps grow-only scratch and an MSM workspace) */
int spx_ctx_mem_info(spx_ctx *ctx, uint64_t *free_bytes, uint64_t *total_bytes);

/* ---- public parameters ---- */
int spx_pp_load(spx_ctx *ctx, const uint8_t *bytes, size_t len, spx_pp **out);
int spx_pp_generate(spx_ctx *ctx, int nv, uint64_t seed, spx_pp **out);
int spx_pp_serialize(spx_pp *pp, uint8_t *out, size_t cap, size_t *len);
int spx_pp_free(spx_pp *pp);

/* ---- index / witness / prove ---- */
int spx_index(spx_ctx *ctx, const spx_csr *a, const spx_csr *b, const spx_csr *c, spx_pk **out);
int spx_index_free(spx_pk *idx);
int spx_witness_upload(spx_ctx *ctx, const uint8_t *v, size_t nv, const uint8_t *w, size_t nw, spx_witness **out);
int spx_witness_free(spx_witness *wit);
size_t spx_proof_size(int log_n, int log_v);
/* host buffers in, proof bytes out (the reference's prove(pk, v, w, &pp) -> Proof, serialized) */
int spx_prove(spx_ctx *ctx, spx_pk *idx, const uint8_t *v, size_t nv, const uint8_t *w, size_t nw, spx_pp *pp,
              const spx_prove_opts *opts, uint8_t *out, size_t cap, size_t *len);
/* witness already resident in HBM (the benchmarked form) */
int spx_prove_witness(spx_ctx *ctx, spx_pk *idx, spx_witness *wit, spx_pp *pp, const spx_prove_opts *opts,
                      uint8_t *out, size_t cap, size_t *len);
/* Proves nproofs witnesses of one index concurrently: worker k drives ctxs[k] (its own HIP stream,
 * MSM workspace and communicator) and proves witnesses k, k + nctx, ... in order. Every proof does
 * the complete per-proof work of spx_prove_witness (transcript absorption of A, B, C included unless
 * opts->cached_matrix_transcript). Proof i is written to out + i * stride, its length to lens[i].
 * All contexts must be on the device (and communicator rank) the index was built for. Throughput
 * form of lib.rs:58-146 for a prover serving many witnesses; returns the first failure's status. */
int spx_prove_many(spx_ctx **ctxs, int nctx, spx_pk *idx, spx_witness **wits, int nproofs, spx_pp *pp,
                   const spx_prove_opts *opts, uint8_t *out, size_t stride, size_t *lens);
/* ---- round-level prover: the reference's interactive API (src/ahp/prover.rs:109-281), driven with
 * verifier coins supplied by the caller as src/ahp/tests.rs:8-70 drives it. Each call takes the
 * verifier message of its step (canonical Fr, 32 B each) and returns the prover message, ark-serialize
 * compressed as the reference's message types (ProverFirstMessage .. ProverSixthMessage, the
 * linear-sumcheck ProverMsg / IndexInfo). The session runs the same kernels as spx_prove: with the
 * challenges a Fiat-Shamir prove would draw, the messages concatenate to spx_prove's proof (plus the
 * two sumchecks' u64 round counts). One session or prove per context at a time, enforced: from
 * spx_prover_init until the session's last round (or spx_prover_free) the context is claimed, and a
 * prove, verify, kernel-level call or second session on it fails with SPX_INVALID_ARGUMENT (so do
 * two concurrent proves on one context). Sessions need an unsharded context (comm size 1).
 *   spx_prover_init                  prover_init              prover.rs:109-121 (|v| power of two, |v|+|w| = n)
 *   spx_prover_first_round           prover_first_round       prover.rs:123-141 (commitment)
 *   spx_prover_second_round          prover_second_round      prover.rs:143-160 (r_v: log2|v| coins)
 *   spx_prover_third_round           prover_third_round       prover.rs:163-196 (tau: log_n coins)
 *   spx_prove_first_sumcheck_round   prove_first_sumcheck_round prover.rs:199-207 (NULL first, then r_{i-1})
 *   spx_prove_fourth_round           prove_fourth_round       prover.rs:210-228 (last point of r_x)
 *   spx_prove_fifth_round            prove_fifth_round        prover.rs:230-255 (r_a, r_b, r_c: 96 B)
 *   spx_prove_second_sumcheck_round  prove_second_sumcheck_round prover.rs:258-266 (NULL first, then r_{i-1})
 *   spx_prove_sixth_round            prove_sixth_round        prover.rs:268-281 (last point of r_y)
 * Out-of-order calls fail with SPX_INVALID_ARGUMENT; a sumcheck round given a challenge first, or
 * none later, or called past log_n rounds fails with SPX_SUMCHECK (linear-sumcheck's errors). */
typedef struct spx_prover spx_prover;
int spx_prover_init(spx_ctx *ctx, spx_pk *idx, const uint8_t *v, size_t nv, const uint8_t *w, size_t nw,
                    spx_prover **out);
int spx_prover_first_round(spx_prover *p, spx_pp *pp, uint8_t *msg, size_t cap, size_t *len);
int spx_prover_second_round(spx_prover *p, const uint8_t *r_v, size_t n, spx_pp *pp, uint8_t *msg, size_t cap,
                            size_t *len);
int spx_prover_third_round(spx_prover *p, const uint8_t *tau, size_t n, uint8_t *msg, size_t cap, size_t *len);
int spx_prove_first_sumcheck_round(spx_prover *p, const uint8_t *challenge, uint8_t *msg, size_t cap, size_t *len);
int spx_prove_fourth_round(spx_prover *p, const uint8_t *last_point, uint8_t *msg, size_t cap, size_t *len);
int spx_prove_fifth_round(spx_prover *p, const uint8_t *r_abc, uint8_t *msg, size_t cap, size_t *len);
int spx_prove_second_sumcheck_round(spx_prover *p, const uint8_t *challenge, uint8_t *msg, size_t cap, size_t *len);
int spx_prove_sixth_round(spx_prover *p, const uint8_t *last_point, spx_pp *pp, uint8_t *msg, size_t cap, size_t *len);
int spx_prover_free(spx_prover *p);

/* host time spent by spx_prove_many's hashing pools absorbing A, B, C (lib.rs:61-64), process-wide:
 * out[0] nanoseconds (summed over the pool threads), out[1] proofs absorbed, out[2] the multi-buffer
 * lane width (proofs hashed per vector instruction: 16 AVX-512, 8 AVX2, 1 scalar), out[3] nanoseconds
 * the proof workers waited for a proof's absorption (summed over the workers) */
int spx_hash_stats(uint64_t out[4]);
/* host CPU of the proving threads by prove() phase, process-wide since load: out[3 i], out[3 i + 1],
 * out[3 i + 2] = thread CPU ns, wall ns and count of phase i in the order transcript_matrices, commit,
 * open_rv, sumcheck1, eval_on_x, sumcheck2, open_ry (the phases of spx_last_timings) */
int spx_host_phase_stats(uint64_t out[21]);
/* MLArgumentForR1CS::verify (src/lib.rs:147-212, verifier.rs:143-512): SPX_OK = accepted (the
 * reference's Ok(true)); a rejection returns the reference's error kind (SPX_INVALID_ARGUMENT,
 * SPX_SUMCHECK, SPX_WRONG_WITNESS, SPX_SERIALIZATION) with its message in spx_last_error.
 * vp = VerifierParameter (commitment/data_structures.rs:19-26) in ark-serialize uncompressed form.
 * The matrix evaluation runs on the ctx's GPU; the index must be built on a single-rank context. */
int spx_verify(spx_ctx *ctx, spx_pk *idx, const uint8_t *v, size_t nv, const uint8_t *proof, size_t len,
               const uint8_t *vp, size_t vp_len, const spx_prove_opts *opts);
/* VerifierParameter of a keygen-generated PP (spx_pp_generate; setup.rs:91-101), uncompressed bytes */
int spx_vp_from_pp(spx_pp *pp, uint8_t *out, size_t cap, size_t *len);
/* prod_i e(P_i, Q_i) == 1 over n pairs (uncompressed G1 96 B / G2 192 B each); host only, no GPU
 * (E::product_of_pairings as used by verify.rs:12-45) */
int spx_pairing_check(const uint8_t *g1, const uint8_t *g2, size_t n, int *is_one);
/* per-phase device timings of the last prove on this ctx, microseconds */
int spx_last_timings(spx_ctx *ctx, double *out, int cap, int *n);

/* ---- R1CS front-end: ark-relations ConstraintSystem semantics ----
 * Variable 0 is the constant One; spx_cs_new_input returns instance variables (Variable::Instance,
 * numbered before witnesses in z = v || w), spx_cs_new_witness returns witness variables (bit 63
 * set). Linear combinations are compactified on export (sorted, merged, zeros dropped:
 * LinearCombination::compactify / inline_all_lcs). spx_cs_make_square follows test_utils.rs:81-102.
 * spx_cs_matrices exports CSR rows (constraints) over columns z and v / w value bytes, valid until
 * the next change to the system; they feed spx_index and spx_prove directly. Host only. */
typedef struct spx_cs spx_cs;
typedef struct {
    const uint64_t *vars;    /* len variables */
    const uint8_t *coeffs;   /* len canonical Fr, 32 B each */
    size_t len;
} spx_lc;
const char *spx_cs_last_error(void);
int spx_cs_create(spx_cs **out);
int spx_cs_free(spx_cs *cs);
int spx_cs_new_input(spx_cs *cs, const uint8_t value[32], uint64_t *var);
int spx_cs_new_witness(spx_cs *cs, const uint8_t value[32], uint64_t *var);
int spx_cs_enforce(spx_cs *cs, const spx_lc *a, const spx_lc *b, const spx_lc *c);
int spx_cs_make_square(spx_cs *cs, uint64_t num_formatted_variables);
int spx_cs_counts(const spx_cs *cs, uint64_t *constraints, uint64_t *instance, uint64_t *witness);
int spx_cs_is_satisfied(spx_cs *cs, int *ok);
int spx_cs_matrices(spx_cs *cs, spx_csr *a, spx_csr *b, spx_csr *c, const uint8_t **v, const uint8_t **w);

/* ---- synthetic instances (SURVEY §8(d) generators; SplitMix64, same draws as the test oracle) ----
 * kind 0 = uniform-3n (satisfiable, nnz = 3n), 1 = ref-shaped (TestSynthesizer, param = density),
 * 3 = circuit-3n (fixed index, nnz = 3n, many witnesses: param = witness seed of spx_synth_z).
 * spx_synth_csr fills views into the handle (valid until spx_synth_free). */
typedef struct spx_synth spx_synth;
int spx_synth_create(int kind, int log_n, int log_v, uint64_t seed, uint64_t param, spx_synth **out);
uint64_t spx_synth_nnz(const spx_synth *s, int m);
int spx_synth_csr(const spx_synth *s, int m, spx_csr *out);
const uint8_t *spx_synth_z(const spx_synth *s);
/* kind 3 only: the witnesses (z = v || w, canonical, 32 n bytes each) of seeds wseed0 .. wseed0 + count - 1 */
int spx_synth_witnesses(const spx_synth *s, uint64_t wseed0, int count, uint8_t *z_out);
int spx_synth_free(spx_synth *s);

/* ---- live kernel statistics (HIP events on the library's stream, enabled per ctx) ----
 * ids: see SPX_K_* below; per id: launches, summed device ms, summed algorithmic bytes. */
enum {
    SPX_K_SC1 = 0,      /* sumcheck #1 round (fold + evaluate) */
    SPX_K_SC2 = 1,      /* sumcheck #2 round */
    SPX_K_SPMV = 2,     /* Az, Bz, Cz */
    SPX_K_MTV = 3,      /* sum_m r_m M(r_x, .) */
    SPX_K_OPEN = 4,     /* mKZG quotient / fold level */
    SPX_K_EQ = 5,       /* eq tables */
    SPX_K_MSM_SORT = 6, /* the bucket sort: k_sort_count .. k_sort_final (both curves) */
    SPX_K_ACC_G1 = 7,   /* bucket accumulation, affine level, G1 */
    SPX_K_ACC_G2 = 8,   /* bucket accumulation, affine level, G2 */
    SPX_K_ACCX_G1 = 9,  /* bucket accumulation, XYZZ levels, G1 */
    SPX_K_ACCX_G2 = 10, /* bucket accumulation, XYZZ levels, G2 */
    SPX_K_RED_G1 = 11,  /* bucket weighting + final reduction, G1 */
    SPX_K_RED_G2 = 12,  /* bucket weighting + final reduction, G2 */
    SPX_K_COUNT = 13
};
int spx_kernel_stats_enable(spx_ctx *ctx, int on);
int spx_kernel_stats(spx_ctx *ctx, int id, uint64_t *launches, double *ms, double *bytes);
/* the same, restricted to the launches of `id` with the largest algorithmic bytes (e.g. round 1 of a
 * sumcheck, where the tables stream from HBM) */
int spx_kernel_stats_largest(spx_ctx *ctx, int id, uint64_t *launches, double *ms, double *bytes);
/* unit operations counted for a kernel id: curve additions (upper bound: zero digits included) for
 * SPX_K_ACC_* (mixed) and SPX_K_ACCX_* (XYZZ); 0 for the others */
int spx_kernel_ops(spx_ctx *ctx, int id, double *ops);
/* MSM batches of this context rerun with one key slot per digit because a proof-sharded rank's
 * compacted keys overflowed their planned capacity (scalars crowding one rank's buckets); a
 * diagnostic: the results are exact either way */
int spx_msm_reruns(spx_ctx *ctx, uint64_t *reruns);

/* ---- kernel-level entry points (parity tests) ---- */
int spx_sum_over_y(spx_ctx *ctx, const spx_csr *m, const uint8_t *z, uint8_t *out);
int spx_eval_on_x(spx_ctx *ctx, const spx_csr *m, const uint8_t *r_x, uint8_t *out);
/* one AHPForMLSumcheck::prove_round [linear-sumcheck] of sum_b f(b) g(b) over n = 2^k canonical Fr
 * (the second sumcheck's product shape, prover.rs:239-247): r_prev = NULL is the first round; with
 * r_prev both tables are first bound at variable 0 to it (f_out / g_out receive the n / 2 bound
 * entries, either may be NULL) and the round runs on the bound tables. evals_out = P(0), P(1), P(2). */
int spx_sumcheck_round(spx_ctx *ctx, const uint8_t *f, const uint8_t *g, size_t n, const uint8_t *r_prev,
                       uint8_t *evals_out, uint8_t *f_out, uint8_t *g_out);
int spx_msm_g1(spx_ctx *ctx, const uint8_t *bases, const uint8_t *scalars, size_t n, uint8_t *out96);
int spx_msm_g2(spx_ctx *ctx, const uint8_t *bases, const uint8_t *scalars, size_t n, uint8_t *out192);
int spx_commit(spx_ctx *ctx, spx_pp *pp, const uint8_t *table, int nv, uint8_t *out56);
/* proof_out: Proof{h, proofs} compressed = 96 + 8 + 96 * nv bytes */
int spx_open(spx_ctx *ctx, spx_pp *pp, const uint8_t *table, int nv, const uint8_t *point, uint8_t *eval_out,
             uint8_t *proof_out);

#ifdef __cplusplus
}
#endif
#endif
