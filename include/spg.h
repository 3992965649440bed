/*
 * spg.h — C-ABI of the MI355X-native Spartan prover hot path (libspg.so).
 *
 * Drop-in boundary for scroll-tech/spartan-parallel (reference snapshot under /root/reference).
 * Every entry point replaces one internal seam of the Rust crate; the seam is cited per function.
 * A Rust maintainer binds these with a `#[link(name = "spg")] extern "C"` block.
 *
 * Conventions
 *   - Scalars cross as the reference's in-memory layout of `Scalar`: four little-endian u64 limbs in
 *     Montgomery form with R = 2^256 (src/scalar/ristretto255.rs:193-199), i.e. `uint64_t[4]`.
 *   - Group elements cross only as 32-byte CompressedRistretto encodings (src/group.rs:7).
 *   - Every function returns 0 on success or a negative SPG_E_* code; spg_last_error() describes it.
 *   - All calls on one spg_ctx are issued on that context's HIP stream and return after their
 *     results are in the caller's buffers. Distinct contexts may be used from different threads.
 *   - The library never draws randomness; callers own all host buffers.
 */
#ifndef SPG_H
#define SPG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPG_OK 0
#define SPG_E_ARG -1       /* bad size / null pointer / inconsistent shapes */
#define SPG_E_NOMEM -2     /* device allocation failed */
#define SPG_E_HIP -3       /* HIP runtime error */
#define SPG_E_POINT -4     /* invalid compressed point (ProofVerifyError::DecompressionError) */
#define SPG_E_NODEVICE -5  /* no usable gfx950 device */
#define SPG_E_VERIFY -6    /* a proof did not verify (spg_last_error names the failed check) */
#define SPG_E_CALLBACK -7  /* a caller-provided transcript callback returned non-zero */

typedef struct spg_ctx spg_ctx;
typedef struct spg_gens spg_gens;

/* ---- context ------------------------------------------------------------------------------- */
int spg_init(int device, spg_ctx** out);
int spg_free(spg_ctx* ctx);
const char* spg_last_error(const spg_ctx* ctx);
/* device-side wall time of the most recent compute call, in microseconds (HIP events on the stream) */
double spg_last_kernel_us(const spg_ctx* ctx);

/* Multi-process proving: one process (and context) per GPU; with nranks > 1 the calls below become SPMD
 * collectives (every rank makes the same call with the same public arguments and runs the same Fiat-Shamir
 * transcript; every exchange carries each rank's status, so a failure on one rank fails all of them):
 *  - spg_r1cs_prove is sharded by instance p: rank r holds instances [b(r), b(r+1)) with
 *    b(r) = r*floor(P/n) + min(r, P mod n) (spg.shard_range); the argument check is allgathered first.
 *  - spg_spark_commit / spg_spark_prove (every rank holds the whole dense representation): Hyrax rows are
 *    split, product trees are interleaved by the low lg n index bits (n a power of two; otherwise they stay
 *    whole), layer rounds and hash-layer evaluations sum partials; every rank returns the same bytes.
 *  - spg_r1cs_multi_evaluate splits every matrix's rows and sums the 3P partial evaluations.
 * fn(user, send, bytes, recv) must place the `bytes` sent by rank k at recv + k*bytes on every rank (an
 * allgather, e.g. RCCL / torch.distributed); it returns 0 on success. nranks == 1 clears it. */
typedef int (*spg_allgather_fn)(void* user, const void* send, size_t bytes, void* recv);
int spg_set_comm(spg_ctx* ctx, int rank, int nranks, spg_allgather_fn fn, void* user);
/* The same with libspg's own transport: RCCL (librccl.so.1, opened at first use) on the context's stream, one
 * process per GPU; no caller code runs per exchange. Rank 0 makes the 128-byte id with spg_rccl_unique_id and
 * hands it to every rank by any channel of the caller's (e.g. a torch.distributed broadcast); every rank then calls
 * spg_set_comm_rccl (collective: it returns once all nranks have joined). An exchange that a dead peer never
 * completes fails after SPG_RCCL_TIMEOUT_S seconds (default 600) instead of hanging; the communicator is then
 * aborted and stays unusable (every later exchange on it fails): install a new transport to continue. */
int spg_rccl_unique_id(uint8_t id[128]);
int spg_set_comm_rccl(spg_ctx* ctx, const uint8_t id[128], int rank, int nranks);
/* one allgather over the context's transport (callback or RCCL): the `bytes` of rank k land at recv + k*bytes */
int spg_comm_allgather(spg_ctx* ctx, const void* send, size_t bytes, void* recv);

/* per-kernel timing on the context stream (events; off by default). spg_prof_read resolves them and
 * returns up to `max` records (name[32], launches, total microseconds, algorithmic HBM bytes moved
 * by those launches as modelled in DESIGN.md, 0 where not modelled); reset != 0 clears the tallies.
 * The record named "(device_busy)" (0 launches) holds the union of the timed intervals: the device's busy time,
 * which the per-kernel totals overstate where the context's two streams ran kernels at once. */
int spg_prof_enable(spg_ctx* ctx, int on);
int spg_prof_read(spg_ctx* ctx, char* names, long* launches, double* total_us, double* bytes, int max, int reset);
/* the same plus the modelled VALU work of those launches in curve mixed additions (ops; 0 where not modelled):
 * one per nonzero signed window digit of the MSM kernels */
int spg_prof_read2(spg_ctx* ctx, char* names, long* launches, double* total_us, double* bytes, double* ops, int max,
                   int reset);
/* the same plus the modelled VALU work in Fq (scalar-field Montgomery) products (fqm; 0 where not modelled): the
 * sumcheck evaluations and SPARK layer rounds, priced against the measured whole-GPU Fq product rate */
int spg_prof_read3(spg_ctx* ctx, char* names, long* launches, double* total_us, double* bytes, double* ops,
                   double* fqm, int max, int reset);
/* Fixed-base precomputation of this process: the HBM bytes of the comb tables currently allocated
 * for every live generator set, the number of comb tables built so far and their total build time in seconds (device
 * build + synchronisation, wall clock), and the HBM bytes of the 2^k G_i tables every generator set keeps (254 rows of
 * n + 1 Niels points, built by spg_gens_derive / spg_gens_upload). Comb tables are built on first use of a generator
 * set and live until spg_gens_free; the figures let a caller (bench.py) disclose the precomputation behind an
 * MSM-throughput number. Any pointer may be NULL. */
int spg_comb_stats(uint64_t* bytes, int* tables_built, double* build_seconds, uint64_t* gens_table_bytes);
/* on = 0: this context's MSMs and row commitments skip the comb tables and run the bucket Pippenger pipelines (over
 * the 2^k G_i generator tables only); on = 1 (default) restores them. Results are identical either way. */
int spg_set_comb(spg_ctx* ctx, int on);

/* ---- device-resident scalar vectors (HBM) ----------------------------------------------------
 * Tables the prover keeps resident between calls (witness polynomials, sumcheck tables). */
typedef struct spg_buf spg_buf;
int spg_buf_upload(spg_ctx* ctx, const uint64_t* scalars_mont, size_t n, spg_buf** out);
int spg_buf_download(spg_ctx* ctx, const spg_buf* b, uint64_t* scalars_mont);
size_t spg_buf_len(const spg_buf* b);
int spg_buf_free(spg_ctx* ctx, spg_buf* b);
/* EqPolynomial::new(r).evals() (src/dense_mlpoly.rs:76-92): the 2^ell table prod_j (b_j ? r_j : 1 - r_j),
 * r[0] the most significant bit of the index, computed on the device into a new spg_buf (ell <= 30). The
 * prover's sumchecks and SPARK build the same tables internally; this entry point exposes them. */
int spg_eq_evals(spg_ctx* ctx, const uint64_t* r_mont, size_t ell, spg_buf** out);

/* ---- per-operation seams on device vectors (csrc/seams.hip) ---------------------------------
 * The reference's dense-polynomial and cubic-sumcheck operations one call at a time, for a caller that drives its
 * own protocol around them. Scalars are Montgomery [u64; 4]; each call returns when its result is ready. */
/* DensePolynomial::bound_poly_var_top (src/dense_mlpoly.rs:267-275): Z[i] += r (Z[i + n/2] - Z[i]) for i < n/2,
 * then the length halves (spg_buf_len); n even and >= 2, else SPG_E_ARG */
int spg_buf_bound_top(spg_ctx* ctx, spg_buf* b, const uint64_t* r_mont);
/* DensePolynomial::bound_poly_var_bot (src/dense_mlpoly.rs:350-358): Z[i] = Z[2i] + r (Z[2i+1] - Z[2i]), length halves */
int spg_buf_bound_bot(spg_ctx* ctx, spg_buf* b, const uint64_t* r_mont);
/* DensePolynomial::evaluate (src/dense_mlpoly.rs:361-367): sum_i Z[i] chi_i(r), r[0] the index's most significant
 * bit; b holds exactly 2^ell scalars (the reference asserts the same) and is left unchanged */
int spg_buf_evaluate(spg_ctx* ctx, const spg_buf* b, const uint64_t* r_mont, size_t ell, uint64_t* out_mont);
/* One round of SumcheckInstanceProof::prove_cubic with the product-circuit comb A B C (src/sumcheck.rs:207-236,
 * src/product_tree.rs:185-189): out3 = (eval_point_0, eval_point_2, eval_point_3) over A, B, C of one even length */
int spg_cubic_round_evals(spg_ctx* ctx, const spg_buf* A, const spg_buf* B, const spg_buf* C, uint64_t* out3_mont);
/* SumcheckInstanceProof::prove_cubic (src/sumcheck.rs:193-262) with comb A B C on A, B, C of 2^k scalars each
 * (k >= num_rounds; bound in place, their lengths halve every round) against transcript t: polys receives
 * num_rounds CompressedUniPoly (3 scalars each: the coefficients without the linear term), r the num_rounds
 * challenges, claims (A[0], B[0], C[0]) after the last round */
int spg_prove_cubic(spg_ctx* ctx, const uint64_t* claim_mont, size_t num_rounds, spg_buf* A, spg_buf* B, spg_buf* C,
                    struct spg_transcript* t, uint64_t* polys_mont, uint64_t* r_mont, uint64_t* claims_mont);
/* DensePolynomialPqx (src/custom_dense_mlpoly.rs:22-359), the ragged (p, q_rev, w, x_rev) table of the R1CS proof,
 * resident in HBM. spg_pqx_new = DensePolynomialPqx::new (:45-64) on z_mat already in (p, q_rev, w, x_rev) order:
 * instance p's num_proofs[p] x num_witness_secs x num_inputs[p] scalars row-major, instances one after another
 * (num_proofs[p], num_inputs[p] powers of two <= the maxima, which are powers of two; < 2^31 scalars in all). */
typedef struct spg_pqx spg_pqx;
int spg_pqx_new(spg_ctx* ctx, const uint64_t* z_mont, size_t num_instances, const size_t* num_proofs,
                size_t max_num_proofs, size_t num_witness_secs, const size_t* num_inputs, size_t max_num_inputs,
                spg_pqx** out);
int spg_pqx_free(spg_ctx* ctx, spg_pqx* h);
/* bound_poly(r, mode) (:180-289): mode 1 = first p variable, 2 = q, 3 = w, 4 = x; mode 1 before every q and x
 * variable is bound is SPG_E_ARG (the reference's assert_eq! in bound_poly_p, :206-207) */
int spg_pqx_bound(spg_ctx* ctx, spg_pqx* h, const uint64_t* r_mont, int mode);
/* evaluate(r_p, r_q, r_w, r_x) (:320-333): a clone bound by r_x, r_w, r_q, r_p, then index(0, 0, 0, 0) */
int spg_pqx_evaluate(spg_ctx* ctx, const spg_pqx* h, const uint64_t* rp, size_t np, const uint64_t* rq, size_t nq,
                     const uint64_t* rw, size_t nw, const uint64_t* rx, size_t nx, uint64_t* out_mont);
/* current sizes: dims = (num_instances, max_num_proofs, num_witness_secs, max_num_inputs); num_proofs / num_inputs
 * (optional) receive one entry per instance; spg_pqx_download: every allocated entry in spg_pqx_new's layout (folds
 * rewrite the low halves in place and the allocation never shrinks, as the reference's nested Vecs) */
int spg_pqx_shape(const spg_pqx* h, size_t* dims, size_t* num_proofs, size_t* num_inputs);
int spg_pqx_download(spg_ctx* ctx, const spg_pqx* h, uint64_t* z_mont);
/* R1CSInstance::multiply_vec_block (src/r1csinstance.rs:363-436; multiply_vec_disjoint_rounds per (p, q),
 * src/sparse_mlpoly.rs:454-472) on an instance from spg_r1cs_inst_new: z_mat (p, q, w, x) -- instance p's
 * num_proofs[p] x num_witness_secs x num_inputs[p] scalars, instances one after another; column c of a matrix reads
 * z[p][q][c / max_num_inputs][c % max_num_inputs], zero past num_inputs[p] -- into three new DensePolynomialPqx tables
 * Az, Bz, Cz in new_rev order (num_proofs, max_num_proofs; num_cons, max_num_cons of the instance; one w section).
 * num_proofs[p] and the instance's num_cons are powers of two; 1..8 witness sections. */
/* One x or q round of the R1CS proof's phase-1 sumcheck (prove_cubic_with_additive_term_disjoint_rounds,
 * src/sumcheck.rs:1173-1245, comb A (B C - D)): out3 = (eval_point_0, eval_point_2, eval_point_3) over the eq
 * factors Ap, Aq, Ax in their current lengths (instance_len = |Ap|; an x round (mode 4) has cons_len = |Ax| / 2, a q
 * round (mode 2, once |Ax| = 1) proof_len = |Aq| / 2) and the tables B, C, D (one shape, one witness section) in
 * their current state. The caller then binds Ax or Aq (spg_buf_bound_top) and B, C, D (spg_pqx_bound) with r_j. */
int spg_phase1_round_evals(spg_ctx* ctx, const spg_buf* Ap, const spg_buf* Aq, const spg_buf* Ax, const spg_pqx* B,
                           const spg_pqx* C, const spg_pqx* D, int mode, uint64_t* out3_mont);
/* One y (mode 4), w (mode 3) or p (mode 1) round of the R1CS proof's phase-2 sumcheck (prove_cubic_disjoint_rounds,
 * src/sumcheck.rs:881-941, comb A B C): out3 = (e0, e2, e3) over eq(r_p) (A; instance_len = |A|, / 2 in a p round),
 * ABC (one instance when single_inst, else one per instance) and Z, both with q bound (one proof row) and in their
 * current state; num_witness_secs is the reference's argument. The caller binds A (p rounds) and ABC, Z with r_j. */
int spg_phase2_round_evals(spg_ctx* ctx, const spg_buf* A, const spg_pqx* ABC, const spg_pqx* Z, int mode,
                           int single_inst, size_t num_witness_secs, uint64_t* out3_mont);
struct spg_r1cs_inst;
int spg_r1cs_multiply_vec_block(spg_ctx* ctx, const struct spg_r1cs_inst* inst, size_t num_instances,
                                const size_t* num_proofs, size_t max_num_proofs, const size_t* num_inputs,
                                size_t max_num_inputs, size_t num_witness_secs, const uint64_t* z_mont, spg_pqx** Az,
                                spg_pqx** Bz, spg_pqx** Cz);

/* ---- generators ------------------------------------------------------------------------------
 * MultiCommitGens::new(n, label) (src/commitments.rs:15-33): n+1 points from SHAKE256(label ||
 * RISTRETTO_BASEPOINT_COMPRESSED) mapped with RistrettoPoint::from_uniform_bytes; G = first n, h = last.
 * The handle keeps the points resident in HBM together with fixed-base window tables. */
int spg_gens_derive(spg_ctx* ctx, const uint8_t* label, size_t label_len, size_t n, spg_gens** out);
/* upload n+1 compressed points (G_0..G_{n-1}, h) instead of deriving them */
int spg_gens_upload(spg_ctx* ctx, const uint8_t* compressed, size_t n, spg_gens** out);
/* (n+1) x 32 bytes: G_0 .. G_{n-1}, h */
int spg_gens_download(spg_ctx* ctx, const spg_gens* g, uint8_t* out);
size_t spg_gens_n(const spg_gens* g);
int spg_gens_free(spg_ctx* ctx, spg_gens* g);

/* ---- multi-scalar multiplication ---------------------------------------------------------------
 * GroupElement::vartime_multiscalar_mul (src/group.rs:98-116) against generators
 * G[gen_offset .. gen_offset + n), plus blind * h when blind_mont != NULL
 * (Commitments::commit for [Scalar], src/commitments.rs:87-92). out: 32-byte compression. */
int spg_msm(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const uint64_t* scalars_mont, size_t n,
            const uint64_t* blind_mont, uint8_t out[32]);
/* Hyrax row commitments, DensePolynomial::commit_inner (src/dense_mlpoly.rs:184-212):
 * for i < L: out[i] = compress( sum_j Z[R*i + j] * G[j] + blinds[i] * h ); blinds may be NULL (zeros,
 * the `random_tape = None` case every SNARK::prove commit uses). Z is L*R scalars, row-major. */
int spg_commit_rows(spg_ctx* ctx, const spg_gens* g, const uint64_t* Z_mont, size_t L, size_t R,
                    const uint64_t* blinds_mont, uint8_t* out);
/* One shard of an MSM split over devices ("split points and scalars into contiguous chunks; each
 * GPU produces a partial sum in extended coordinates"): out_ext = sum_i s_i * G[gen_offset + i] as X, Y, Z, T,
 * each 32 little-endian bytes (a representative < 2^256 of the coordinate mod 2^255 - 19). Not compressed,
 * so the partials of all ranks add exactly. Same group.rs:98-116 semantics as spg_msm without the blind. */
int spg_msm_partial(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const uint64_t* scalars_mont, size_t n,
                    uint8_t out_ext[128]);
/* The same two over scalars already resident in HBM (buf[offset .. offset + n), e.g. a witness uploaded once):
 * no host-to-device copy inside the call. spg_msm_buf has no blind (vartime_multiscalar_mul). */
int spg_msm_partial_buf(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const spg_buf* buf, size_t offset,
                        size_t n, uint8_t out_ext[128]);
int spg_msm_buf(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const spg_buf* buf, size_t offset, size_t n,
                uint8_t out[32]);
/* Host only, needs no device or context: the sum of k partial points (k x 128 bytes, spg_msm_partial layout)
 * encoded as a 32-byte CompressedRistretto (RFC 9496 ENCODE). */
int spg_points_sum_compress(const uint8_t* parts, size_t k, uint8_t out[32]);

/* ---- R1CS data-parallel satisfiability proof --------------------------------------------------
 * Flat C views of the reference's R1CSInstance (src/r1csinstance.rs:19-31) and
 * ProverWitnessSecInfo (src/lib.rs:508-527). Entries are the reference's SparseMatEntry
 * {row: usize, col: usize, val: Scalar} (48 bytes). */
typedef struct {
  uint64_t row, col;
  uint64_t val[4]; /* Montgomery limbs */
} spg_sparse_entry;

typedef struct {
  size_t num_instances;                   /* instances with matrices (1 = shared by every p)    */
  size_t max_num_cons;                    /* power of two                                         */
  size_t num_vars;                        /* power of two: next_pow2(#sections) * max_num_inputs */
  const size_t* num_cons;                 /* [num_instances], powers of two                      */
  const size_t* nnz;                      /* [3*num_instances]: |A_p|, |B_p|, |C_p|               */
  const spg_sparse_entry* const* entries; /* [3*num_instances] -> A_0,B_0,C_0,A_1,...            */
} spg_r1cs_instance;

typedef struct {
  size_t num_instances;       /* 1 (single) or P                                          */
  const size_t* num_proofs;   /* [num_instances]: rows of w_mat[p] (1 = short section)     */
  const size_t* num_inputs;   /* [num_instances]                                          */
  const uint64_t* const* w;   /* [num_instances] -> num_proofs[p]*num_inputs[p] scalars    */
} spg_witness_sec;

/* spg_commit_rows over a device-resident vector: rows are Z[offset + R*i .. offset + R*(i+1)). */
int spg_commit_rows_buf(spg_ctx* ctx, const spg_gens* g, const spg_buf* Z, size_t offset, size_t L, size_t R,
                        const spg_buf* blinds, uint8_t* out);

/* ---- Fiat-Shamir transcript and prover randomness (host objects) -----------------------------
 * ProofTranscript over merlin::Transcript (src/transcript.rs:5-63) and RandomTape
 * (src/random.rs:7-29). RandomTape::new draws its init scalar from OsRng in the reference; here the
 * caller supplies it (the one seam that makes proofs reproducible). Labels are NUL-terminated. */
typedef struct spg_transcript spg_transcript;
typedef struct spg_random_tape spg_random_tape;
int spg_transcript_new(const char* label, spg_transcript** out);
/* A transcript backed by the caller's own Fiat-Shamir state (SNARK::prove's `transcript: &mut Transcript`,
 * src/lib.rs:1022, appended to from :1033 on; ProofTranscript src/transcript.rs:5-63). Every operation of the
 * prover or verifier reduces to merlin's two primitives and is forwarded, in order, to
 *   append(user, label, msg, len)         = Transcript::append_message(label, msg)
 *   challenge(user, label, out, len)      = Transcript::challenge_bytes(label, out[..len])
 * so whatever the caller appended before the call, and whatever it draws after it, continue one transcript.
 * Labels are NUL-terminated; the labels libspg emits itself are string literals of the library (static storage,
 * valid while libspg is loaded: a Rust shim may hand them to merlin as &'static [u8]). A callback returns 0 on
 * success; the first non-zero return is latched: later operations are not forwarded, and the entry point that
 * was running returns SPG_E_CALLBACK. spg_transcript_append_* / challenge_* on such a handle forward too. */
typedef int (*spg_transcript_append_fn)(void* user, const char* label, const uint8_t* msg, size_t len);
typedef int (*spg_transcript_challenge_fn)(void* user, const char* label, uint8_t* out, size_t len);
int spg_transcript_new_callbacks(spg_transcript_append_fn append, spg_transcript_challenge_fn challenge, void* user,
                                 spg_transcript** out);
int spg_transcript_append_message(spg_transcript* t, const char* label, const uint8_t* msg, size_t len);
/* ProofTranscript::append_scalar: label, Scalar::to_bytes (canonical LE) */
int spg_transcript_append_scalar(spg_transcript* t, const char* label, const uint64_t* scalar_mont);
/* ProofTranscript::challenge_scalar: from_bytes_wide of 64 challenge bytes */
int spg_transcript_challenge_scalar(spg_transcript* t, const char* label, uint64_t* out_mont);
int spg_transcript_challenge_bytes(spg_transcript* t, const char* label, uint8_t* out, size_t len);
int spg_transcript_free(spg_transcript* t);
int spg_random_tape_new(const char* name, const uint64_t* init_mont, spg_random_tape** out);
int spg_random_tape_scalar(spg_random_tape* tp, const char* label, uint64_t* out_mont);
int spg_random_tape_free(spg_random_tape* tp);

/* ---- R1CSProof::prove (src/r1csproof.rs:210-685) ----------------------------------------------
 * R1CSGens::new(label, _, num_vars) (src/r1csproof.rs:71-79): gens_pc = PolyCommitmentGens for
 * log2(num_vars) variables; gens_1 = gens_pc.gens_1, gens_4 = MultiCommitGens::new(4, label). All of
 * them are prefixes of the same SHAKE256 stream, held once in HBM. */
typedef struct spg_r1cs_gens spg_r1cs_gens;
typedef struct spg_r1cs_inst spg_r1cs_inst;
typedef struct spg_r1cs_witness spg_r1cs_witness;
int spg_r1cs_gens_new(spg_ctx* ctx, const uint8_t* label, size_t label_len, size_t num_vars, spg_r1cs_gens** out);
/* *count = number of stream points held; out (optional) receives count x 32 bytes */
int spg_r1cs_gens_download(spg_ctx* ctx, const spg_r1cs_gens* g, uint8_t* out, size_t* count);
int spg_r1cs_gens_free(spg_ctx* ctx, spg_r1cs_gens* g);
/* the R1CSInstance, uploaded once (CSR + merged CSC in HBM) */
int spg_r1cs_inst_new(spg_ctx* ctx, const spg_r1cs_instance* inst, spg_r1cs_inst** out);
int spg_r1cs_inst_free(spg_ctx* ctx, spg_r1cs_inst* inst);
/* the witness sections (Vec<&ProverWitnessSecInfo>), uploaded to HBM */
int spg_r1cs_witness_new(spg_ctx* ctx, const spg_witness_sec* secs, size_t nws, spg_r1cs_witness** out);
/* the same for a sharded prover: only instances [p0, p1) of sections with num_instances > 1 are uploaded
 * (w may hold NULL for the others); single sections are uploaded whole */
int spg_r1cs_witness_new_shard(spg_ctx* ctx, const spg_witness_sec* secs, size_t nws, size_t p0, size_t p1,
                               spg_r1cs_witness** out);
int spg_r1cs_witness_free(spg_ctx* ctx, spg_r1cs_witness* w);
/* R1CSProof::prove(num_instances, max_num_proofs, num_proofs, max_num_inputs, num_inputs, witness_secs,
 * inst, gens, transcript, random_tape). Writes bincode(R1CSProof) into proof (proof_cap bytes;
 * *proof_len = size even when it does not fit) and, when challenges_out != NULL, the returned
 * challenges rp | rq_rev | rx | rw||ry (Montgomery limbs) with their lengths in ch_lens[4]. */
int spg_r1cs_prove(spg_ctx* ctx, const spg_r1cs_gens* gens, const spg_r1cs_inst* inst, size_t num_instances,
                   size_t max_num_proofs, const size_t* num_proofs, size_t max_num_inputs, const size_t* num_inputs,
                   const spg_r1cs_witness* witness, spg_transcript* transcript, spg_random_tape* tape,
                   uint8_t* proof, size_t proof_cap, size_t* proof_len, uint64_t* challenges_out, size_t* ch_lens);

/* DensePolynomial::commit without blinds (src/dense_mlpoly.rs:184-256) of n scalars (zero-padded to a power of
 * two 2^k) with gens.gens_pc: L = 2^(k/2) Hyrax row commitments of 2^(k - k/2) scalars into out (32 bytes each,
 * out_cap bytes; *L_out = L). The commitments spg_r1cs_verify takes for every witness section instance. */
int spg_r1cs_gens_commit(spg_ctx* ctx, const spg_r1cs_gens* gens, const uint64_t* Z, size_t n, uint8_t* out,
                         size_t out_cap, size_t* L_out);
/* the verifier's view of one witness section (VerifierWitnessSecInfo, src/lib.rs:606-698) */
typedef struct {
  size_t num_instances;      /* 1 (single) or P                                               */
  const size_t* num_proofs;  /* [num_instances]                                               */
  const size_t* num_inputs;  /* [num_instances]                                               */
  const size_t* comm_len;    /* [num_instances]: Hyrax rows of each instance's commitment       */
  const uint8_t* comms;      /* the row commitments of instance 0, then 1, ... (32 bytes each)   */
} spg_witness_comm;
/* R1CSProof::verify (src/r1csproof.rs:687-954) of bincode(R1CSProof) bytes: evals = the claimed (A, B, C)(rx, ry)
 * bound with eq(rp) (multi_evaluate_bound_rp), num_cons = the instance's max_num_cons. 0 when the proof verifies
 * (and, when challenges_out != NULL, rp | rq_rev | rx | rw||ry with their lengths in ch_lens[4], as
 * spg_r1cs_prove returns them), SPG_E_VERIFY when it does not. challenges_out must hold
 * lg(num_instances) + lg(max_num_proofs) + lg(num_cons) + lg(nws) + lg(max_num_inputs) scalars (4 u64 each, lg
 * rounded up). Shapes are checked before any proof byte is read: every num_proofs[p] a power of two no larger
 * than max_num_proofs, section shapes consistent with the instance (else SPG_E_ARG). */
int spg_r1cs_verify(spg_ctx* ctx, const spg_r1cs_gens* gens, size_t num_instances, size_t max_num_proofs,
                    const size_t* num_proofs, size_t max_num_inputs, const spg_witness_comm* secs, size_t nws,
                    size_t num_cons, const uint64_t* evals, spg_transcript* transcript, const uint8_t* proof,
                    size_t proof_len, uint64_t* challenges_out, size_t* ch_lens);

/* R1CSInstance::multi_evaluate (src/r1csinstance.rs:583-596) via SparseMatPolynomial::evaluate_with_tables
 * (src/sparse_mlpoly.rs:427-450): out[3p + m] = M_p(rx, ry), M in (A, B, C), for every matrix instance p
 * of the uploaded instance; 2^rx_len >= max_num_cons, 2^ry_len >= num_vars. (With one instance this is
 * R1CSInstance::evaluate, :632-641; multi_evaluate_bound_rp folds out[] with eq(rp) on the caller's side.) */
int spg_r1cs_multi_evaluate(spg_ctx* ctx, const spg_r1cs_inst* inst, const uint64_t* rx, size_t rx_len,
                            const uint64_t* ry, size_t ry_len, uint64_t* out);

/* ---- SPARK: sparse matrix polynomial commitments and evaluation proofs ------------------------------
 * The batch is the 3P matrices A_0, B_0, C_0, A_1, ... of an R1CS instance (R1CSInstance::multi_commit,
 * src/r1csinstance.rs:645-700 -> SparseMatPolynomial::multi_commit, src/sparse_mlpoly.rs:566-587).
 * The dense representation (addresses, timestamps, values, comb_ops / comb_mem) stays in HBM. */
typedef struct spg_spark spg_spark;
/* SparseMatPolyCommitmentGens::new(label, nvx, nvy, gens_nnz, gens_batch) (src/sparse_mlpoly.rs:289-317)
 * + multi_commit. Writes bincode(SparseMatPolyCommitment) into comm (*comm_len = its size). */
int spg_spark_commit(spg_ctx* ctx, const spg_r1cs_instance* inst, const uint8_t* label, size_t label_len,
                     size_t gens_nnz, size_t gens_batch, spg_spark** out, uint8_t* comm, size_t comm_cap,
                     size_t* comm_len);
/* SparseMatPolyEvalProof::prove(dense, rx, ry, evals, gens, transcript, random_tape)
 * (src/sparse_mlpoly.rs:1497-1564): evals[3p + m] = M_p(rx, ry) (spg_r1cs_multi_evaluate).
 * Writes bincode(SparseMatPolyEvalProof) into proof (*proof_len = its size even when it does not fit). */
int spg_spark_prove(spg_ctx* ctx, spg_spark* s, const uint64_t* rx, size_t rx_len, const uint64_t* ry,
                    size_t ry_len, const uint64_t* evals, size_t n_evals, spg_transcript* transcript,
                    spg_random_tape* tape, uint8_t* proof, size_t proof_cap, size_t* proof_len);
/* SparseMatPolyEvalProof::verify (src/sparse_mlpoly.rs:1566-1610) of proof bytes against s's commitment: 0 when
 * it verifies, SPG_E_VERIFY when it does not (spg_last_error names the failed check). */
int spg_spark_verify(spg_ctx* ctx, spg_spark* s, const uint64_t* rx, size_t rx_len, const uint64_t* ry,
                     size_t ry_len, const uint64_t* evals, size_t n_evals, spg_transcript* transcript,
                     const uint8_t* proof, size_t proof_len);
int spg_spark_free(spg_ctx* ctx, spg_spark* s);

/* ---- SNARK::prove (src/lib.rs:971-2746) -------------------------------------------------------------
 * Public side: each of the three R1CS instances (block, pairwise check, perm root) with the parameters of
 * the SNARKGens it was encoded with (SNARKGens::new(num_cons, num_vars, num_instances, num_nz_entries),
 * src/lib.rs:164-185; only its gens_r1cs_eval part is used by SNARK::prove). */
typedef struct {
  spg_r1cs_instance inst;  /* unsorted, as generated (src/instance.rs) */
  size_t gens_num_cons, gens_num_vars, gens_num_instances, gens_num_nz_entries;
} spg_snark_instance;

/* The run-time arguments of SNARK::prove in declaration order (src/lib.rs:971-1023). Scalars are Montgomery
 * limbs (4 x u64); witness lists are flattened row-major. */
typedef struct {
  size_t input_block_num, output_block_num;
  const uint8_t* input_liveness; /* [input_len] */
  size_t input_len;
  size_t func_input_width, input_offset, output_offset;
  const uint64_t* input;  /* [input_len][4] */
  const uint64_t* output; /* [4] */
  size_t output_exec_num;
  size_t num_vars, num_ios;
  size_t max_block_num_phy_ops;
  const size_t* block_num_phy_ops; /* [block_num_instances_bound] */
  size_t max_block_num_vir_ops;
  const size_t* block_num_vir_ops; /* [block_num_instances_bound] */
  size_t mem_addr_ts_bits_size, num_inputs_unpadded;
  const size_t* block_num_vars; /* [block_num_instances_bound] */
  size_t block_num_instances_bound, block_max_num_proofs;
  const size_t* block_num_proofs; /* [block_num_instances_bound] */
  size_t consis_num_proofs, total_num_init_phy_mem_accesses, total_num_init_vir_mem_accesses,
      total_num_phy_mem_accesses, total_num_vir_mem_accesses;
  /* [i] -> the witness list of the i-th block in the prover's sort order (block_num_proofs descending, ties in
   * block order; src/lib.rs:1155-1178 pairs block_vars_mat[i] with sorted instance i): block_num_proofs[o_i] rows of
   * block_num_vars[o_i] x 4 limbs, o_i = that block's index; NULL for a block without executions */
  const uint64_t* const* block_vars;
  const uint64_t* exec_inputs;       /* consis_num_proofs x num_ios x 4 */
  const uint64_t* init_phy_mems;     /* total_num_init_phy_mem_accesses x 4 x 4 */
  const uint64_t* init_vir_mems;     /* total_num_init_vir_mem_accesses x 4 x 4 */
  const uint64_t* addr_phy_mems;     /* total_num_phy_mem_accesses x 4 x 4 */
  const uint64_t* addr_vir_mems;     /* total_num_vir_mem_accesses x 8 x 4 */
  const uint64_t* addr_ts_bits;      /* total_num_vir_mem_accesses x mem_addr_ts_bits_size x 4 */
} spg_snark_inputs;

typedef struct spg_snark_comp spg_snark_comp; /* ComputationCommitment + ComputationDecommitment */
typedef struct spg_snark_wit spg_snark_wit;   /* SNARK::prove run-time inputs, resident in HBM */

/* SNARK::multi_encode (multi != 0: matrices grouped by next_power_of_eight(nnz), src/r1csinstance.rs:654-715)
 * or SNARK::encode (one commitment over all 3P matrices, :717-737) of one instance, with
 * SNARKGens::new(gens_num_cons, gens_num_vars, gens_num_instances, gens_num_nz_entries).gens_r1cs_eval
 * (label "gens_r1cs_eval"). The dense representations stay in HBM. */
int spg_snark_encode(spg_ctx* ctx, const spg_snark_instance* inst, int multi, spg_snark_comp** out);
int spg_snark_comp_free(spg_ctx* ctx, spg_snark_comp* comp);
/* Uploads block_vars and exec inputs to HBM (padded to powers of two) and keeps host copies of the parts the
 * witness recurrences read. Block witness lists are given in the sorted order (as in the reference). */
int spg_snark_witness_new(spg_ctx* ctx, const spg_snark_inputs* inputs, spg_snark_wit** out);
int spg_snark_witness_free(spg_ctx* ctx, spg_snark_wit* wit);
/* SNARK::prove (src/lib.rs:971-2746) with vars_gens (spg_r1cs_gens_new(label "gens_r1cs_sat", bound)).
 * Writes bincode(SNARK) into proof (*proof_len = its size even when it does not fit). */
int spg_snark_prove(spg_ctx* ctx, spg_snark_comp* block, spg_snark_comp* pairwise, spg_snark_comp* perm_root,
                    const spg_snark_wit* wit, spg_r1cs_gens* vars_gens, spg_transcript* transcript,
                    spg_random_tape* tape, uint8_t* proof, size_t proof_cap, size_t* proof_len);

/* SNARK::verify (src/lib.rs:2750-3881) on the prover's own argument block: replays the transcript from the public
 * inputs (the spg_snark_inputs sizes, input / output / liveness and the init memory lists; block_vars, exec_inputs
 * and the address lists are not read), the three encoded instances (their SPARK commitments) and the proof bytes,
 * and runs every check of the reference verifier. transcript: the verifier's transcript in the state the prover's
 * was in when SNARK::prove began -- a fresh one with the prover's label, or the caller's own `&mut Transcript` behind
 * spg_transcript_new_callbacks after the same appends. Returns 0 when the proof verifies, SPG_E_VERIFY when it does
 * not (malformed bytes included), another negative code on bad arguments. */
int spg_snark_verify(spg_ctx* ctx, const spg_snark_comp* block, const spg_snark_comp* pairwise,
                     const spg_snark_comp* perm_root, const spg_snark_inputs* inputs, spg_r1cs_gens* vars_gens,
                     spg_transcript* transcript, const uint8_t* proof, size_t proof_len);

/* ---- the verifier's side of the boundary: what SNARK::verify is given (src/lib.rs:2750-2798), no witness data and
 * no sparse matrices. The prover exports its commitments once (preprocessing output, as SNARK::encode returns
 * ComputationCommitment to the caller); the verifier loads them from bytes. */
/* bincode(Vec<ComputationCommitment>) of an encoded instance (as_list != 0: block_comm_list), or of its single
 * ComputationCommitment (pairwise_check_comm, perm_root_comm); *len = the size even when it does not fit */
int spg_snark_comm_bytes(spg_ctx* ctx, const spg_snark_comp* comp, int as_list, uint8_t* out, size_t cap, size_t* len);
/* block_comm_map: list g (lens[g] entries, concatenated in idx) = the matrix indices 3p + m commitment g covers */
int spg_snark_comm_map(spg_ctx* ctx, const spg_snark_comp* comp, size_t* idx, size_t idx_cap, size_t* lens,
                       size_t lens_cap, size_t* n_lists);
/* A verifier-side instance from commitment bytes (replaces the ComputationCommitment + SNARKGens arguments of
 * SNARK::verify, src/lib.rs:2781-2797): bytes = as above; map_idx / map_lens / n_map = block_comm_map for a list
 * (ignored for a single commitment); num_cons = block_num_cons / pairwise_check_num_cons / perm_root_num_cons;
 * gens_* = the SNARKGens::new(num_cons, num_vars, num_instances, num_nz_entries) arguments. Derives the
 * gens_r1cs_eval generators; SPG_E_ARG for bytes that do not decode or do not fit them. Free with
 * spg_snark_comp_free; it serves spg_snark_verify_public only (it cannot prove). */
int spg_snark_comm_load(spg_ctx* ctx, const uint8_t* bytes, size_t len, int as_list, const size_t* map_idx,
                        const size_t* map_lens, size_t n_map, size_t num_cons, size_t gens_num_cons,
                        size_t gens_num_vars, size_t gens_num_instances, size_t gens_num_nz_entries,
                        spg_snark_comp** out);
/* SNARK::verify's public arguments, in its order and meaning (src/lib.rs:2750-2798). Scalars are [u8; 32]
 * canonical little-endian bytes (Scalar::from_bytes; non-canonical bytes are SPG_E_ARG, where the reference's
 * unwrap panics). input_stack / input_mem are the public input stack and memory: the verifier builds and commits
 * their init lists itself (src/lib.rs:3274-3333), and a non-empty list's total_num_init_*_mem_accesses must be its
 * length's next power of two (the reference's assert). */
typedef struct {
  size_t input_block_num, output_block_num;
  const uint8_t* input_liveness; /* [input_len] */
  size_t input_len;
  size_t func_input_width, input_offset, output_offset;
  const uint8_t* input;       /* [input_len][32] */
  const uint8_t* input_stack; /* [input_stack_len][32] */
  size_t input_stack_len;
  const uint8_t* input_mem;   /* [input_mem_len][32] */
  size_t input_mem_len;
  const uint8_t* output;      /* [32] */
  size_t output_exec_num;
  size_t num_vars, num_ios;
  size_t max_block_num_phy_ops;
  const size_t* block_num_phy_ops; /* [block_num_instances_bound] */
  size_t max_block_num_vir_ops;
  const size_t* block_num_vir_ops; /* [block_num_instances_bound] */
  size_t mem_addr_ts_bits_size, num_inputs_unpadded;
  const size_t* block_num_vars; /* [block_num_instances_bound] */
  size_t block_num_instances_bound, block_max_num_proofs;
  const size_t* block_num_proofs; /* [block_num_instances_bound] */
  size_t block_num_cons;
  size_t consis_num_proofs, total_num_init_phy_mem_accesses, total_num_init_vir_mem_accesses,
      total_num_phy_mem_accesses, total_num_vir_mem_accesses;
  size_t pairwise_check_num_cons, perm_root_num_cons;
} spg_snark_public;
/* SNARK::verify from what the reference verifier holds: the loaded commitments, the public arguments, vars_gens and
 * the caller's transcript (any state: a fresh one with the prover's label, or the caller's own behind
 * spg_transcript_new_callbacks). Same return codes as spg_snark_verify. */
int spg_snark_verify_public(spg_ctx* ctx, const spg_snark_comp* block, const spg_snark_comp* pairwise,
                            const spg_snark_comp* perm_root, const spg_snark_public* pub, spg_r1cs_gens* vars_gens,
                            spg_transcript* transcript, const uint8_t* proof, size_t proof_len);

#ifdef __cplusplus
}
#endif
#endif /* SPG_H */
