// spg — prover-side protocol objects and their bincode encoding (serde derive order of the reference):
//   KnowledgeProof / EqualityProof / ProductProof / DotProductProof  src/nizk/mod.rs:16-404
//   DotProductProofLog + BulletReductionProof                          src/nizk/mod.rs:420-523, bullet.rs:32-132
//   PolyEvalProof                                                       src/dense_mlpoly.rs:427-1130
//   ZKSumcheckInstanceProof / SumcheckInstanceProof                     src/sumcheck.rs:28-92
//   R1CSProof                                                           src/r1csproof.rs:24-43
#pragma once
#include <vector>

#include "ctx.hpp"
#include "host.hpp"

namespace spg {

struct KnowledgeProofP {
  Pt alpha;
  Fq z1, z2;
  void ser(Writer& w) const { w.pt(alpha); w.fq(z1); w.fq(z2); }
};
struct EqualityProofP {
  Pt alpha;
  Fq z;
  void ser(Writer& w) const { w.pt(alpha); w.fq(z); }
};
struct ProductProofP {
  Pt alpha, beta, delta;
  Fq z[5];
  void ser(Writer& w) const {
    w.pt(alpha); w.pt(beta); w.pt(delta);
    for (int i = 0; i < 5; i++) w.fq(z[i]);
  }
};
struct DotProductProofP {
  Pt delta, beta;
  FqV z;
  Fq z_delta, z_beta;
  void ser(Writer& w) const { w.pt(delta); w.pt(beta); w.fqs(z); w.fq(z_delta); w.fq(z_beta); }
};
struct DotProductProofLogP {
  std::vector<Pt> L, R;
  Pt delta, beta;
  Fq z1, z2;
  void ser(Writer& w) const { w.pts(L); w.pts(R); w.pt(delta); w.pt(beta); w.fq(z1); w.fq(z2); }
};
struct ZKSumcheckP {
  std::vector<Pt> comm_polys, comm_evals;
  std::vector<DotProductProofP> proofs;
  void ser(Writer& w) const {
    w.pts(comm_polys);
    w.pts(comm_evals);
    w.u64(proofs.size());
    for (auto& p : proofs) p.ser(w);
  }
};
struct SumcheckP {
  std::vector<FqV> polys;  // compressed: coefficients except the linear term
  void ser(Writer& w) const {
    w.u64(polys.size());
    for (auto& p : polys) w.fqs(p);
  }
};
struct R1CSProofP {
  ZKSumcheckP sc1;
  Pt claims_phase2[4];
  KnowledgeProofP pok;
  ProductProofP prod;
  EqualityProofP eq1;
  ZKSumcheckP sc2;
  std::vector<std::vector<Pt>> comm_vars_at_ry_list;
  Pt comm_vars_at_ry;
  std::vector<DotProductProofLogP> evals;
  EqualityProofP eq2;
  void ser(Writer& w) const {
    sc1.ser(w);
    for (int i = 0; i < 4; i++) w.pt(claims_phase2[i]);
    pok.ser(w);
    prod.ser(w);
    eq1.ser(w);
    sc2.ser(w);
    w.u64(comm_vars_at_ry_list.size());
    for (auto& v : comm_vars_at_ry_list) w.pts(v);
    w.pt(comm_vars_at_ry);
    w.u64(evals.size());
    for (auto& e : evals) e.ser(w);
    eq2.ser(w);
  }
};

// A commitment key inside one derived generator stream: G indices + h index (MultiCommitGens view).
struct KeyView {
  std::vector<size_t> G;
  size_t h;
};

// Generators of one label: device handle (all stream points, window tables) + host fixed-base tables.
struct ProverGens {
  spg_gens* dev = nullptr;  // stream points 0 .. count-1
  HostGens host;
  size_t n_pc = 0;          // DotProductProofGens n (gens_pc.gens.gens_n.n)
  KeyView gens_n, gens_1, gens_4;
};

// ---- sigma protocols (host; O(1) points) ----
h::HExt commit_host(ProverGens& g, const KeyView& k, const FqV& x, const Fq& blind);
// one commitment x.commit(blind, k) (or blind * h alone when k is null)
struct CJob {
  const KeyView* k = nullptr;
  size_t h = 0;
  FqV x;
  Fq blind;
  CJob(const KeyView& kv, const FqV& xx, const Fq& b) : k(&kv), h(kv.h), x(xx), blind(b) {}
  CJob(size_t h_index, const Fq& b) : k(nullptr), h(h_index), blind(b) {}
};
struct CommitStats {
  double us = 0;
  size_t calls = 0, points = 0;
};
extern CommitStats g_commit_stats;  // SPG_TRACE >= 2
std::vector<Pt> commit_batch(ProverGens& g, const std::vector<CJob>& jobs);
// pre (optional): the protocol's points computed ahead (sigma1_points), in the order the protocol appends them; the
// protocol still draws its tape scalars itself (the same values), so the tape advances exactly as without them
KnowledgeProofP knowledge_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& x, const Fq& r, Pt* C,
                                const Pt* pre = nullptr);
EqualityProofP equality_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& v1, const Fq& s1,
                              const Fq& v2, const Fq& s2, const Pt* pre = nullptr);
ProductProofP product_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& x, const Fq& rX, const Fq& y,
                            const Fq& rY, const Fq& z, const Fq& rZ, Pt* X, Pt* Y, Pt* Z, const Pt* pre = nullptr);
// The eleven points of R1CSProof::prove's sigma protocols after phase 1 (src/r1csproof.rs:403-456: the knowledge proof
// of Cz, the product proof Az Bz = prod, the equality proof of the two post-phase-1 claims) depend on claims, blinds
// and RandomTape draws alone, never on the transcript: one pool burst computes them all (encodings side by side) from
// a fork of the tape, before the transcript sequence runs. The product proof's delta = b3 X + b5 h is the fixed-base
// commitment (b3 x) G + (b3 rX + b5) h of the same group element (X = x G + rX h), so no variable-base multiple.
struct Sigma1Pre {
  Pt k[2];  // knowledge: C, alpha
  Pt p[6];  // product: X, Y, Z, alpha, beta, delta
  Pt e[3];  // equality: C1, C2, alpha
};
void sigma1_points(ProverGens& g, const KeyView& k, const Tape& tape, const Fq& cz, const Fq& cz_blind, const Fq& az,
                   const Fq& az_blind, const Fq& bz, const Fq& bz_blind, const Fq& prod, const Fq& prod_blind,
                   const Fq& v1, const Fq& s1, const Fq& v2, const Fq& s2, Sigma1Pre* out);
// the prover randomness of one DotProductProof drawn ahead of time (d_vec, r_delta, r_beta from a fork of the
// RandomTape at the same position) with its randomness-only points: delta = d.commit(r_delta, gens_n) and
// r_beta * h of gens_1
struct DotPre {
  FqV d;
  Fq r_delta, r_beta;
  Pt delta;
  h::HExt rbh;
};
DotProductProofP dotproduct_prove(ProverGens& g, const KeyView& k1, const KeyView& kn, Tr& t, Tape& tape, const FqV& x,
                                  const Fq& blind_x, const FqV& a, const Fq& y, const Fq& blind_y, const Pt* Cx_known,
                                  const DotPre* pre = nullptr);
// ---- DotProductProofLog with all MSMs on the GPU over the original generators ----
int dotproduct_log_prove(spg_ctx* ctx, ProverGens& g, Tr& t, Tape& tape, const FqV& x, const Fq& blind_x, const FqV& a,
                         const Fq& y, const Fq& blind_y, DotProductProofLogP* out, Pt* Cy);
// sum_v v * B_v of B bucket sets (bk: B x NB extended points, bucket v at index v - 1), encoded, on host cores
// (plus extra[b] when given)
// carry: every set holds NB + 1 points, the last one added with weight 1 (k_bullet_round_q's top-window carries)
void bucket_finals(const Ext* bk, size_t B, int NB, Pt* out, const h::HExt* extra = nullptr, bool carry = false);
// device MSMs of B x n scalars over explicit generator indices (host buffers), outputs B points
int device_msm_idx(spg_ctx* ctx, ProverGens& g, const std::vector<FqV>& scalars, const std::vector<std::vector<uint32_t>>& idx,
                   std::vector<Pt>* out);

// ---- Hyrax commitments / PolyEvalProof on device polynomials (spark.hip) ----
// PolyCommitmentGens::new(nv, label) as a view of a derived generator stream
ProverGens gens_view(spg_gens* dev, size_t nv);
// DensePolynomial::commit (no blinds) of 2^nv device scalars; rows of 2^(nv - nv/2) <= g.n_pc scalars. With
// sh.n > 1 an SPMD collective: rank r commits its balanced share of the rows, the encodings are allgathered.
int commit_dev(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, size_t nv, std::vector<Pt>* out, const Shard& sh = Shard());
// L rows of R consecutive device scalars -> L row commitments (host)
int commit_rows(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, size_t R, size_t L, Pt* out);
// several row sets at once: the sets that take the latency path's device final (R <= 256, 64 < L <= 65535) are
// launched back to back and encoded by one k_compress_ext launch with one download; the others as commit_rows
struct RowJob {
  const Fq* d_Z;
  size_t R, L;
  Pt* out;
};
int commit_rows_many(spg_ctx* ctx, ProverGens& g, const std::vector<RowJob>& jobs);
// the same in two steps: launch queues the merged sets' points on ctx->stream, finish (same stream) encodes them and
// commits the other sets; the caller may do other host work in between
struct RowsPending {
  Ext* d_ext = nullptr;
  uint8_t* d_out = nullptr;
  size_t tot = 0;
  std::vector<char> hv;  // per merged set: its points are halves (encoded as doubles on the host)
};
int commit_rows_many_launch(spg_ctx* ctx, ProverGens& g, const std::vector<RowJob>& jobs, RowsPending* p);
int commit_rows_many_finish(spg_ctx* ctx, ProverGens& g, const std::vector<RowJob>& jobs, RowsPending& p);
// the same split over the ranks of sh (every rank returns all L commitments)
int commit_rows_sh(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, size_t R, size_t L, Pt* out, const Shard& sh);
// PolyCommitment::append_to_transcript
void append_polycomm(Tr& t, const char* label, const std::vector<Pt>& c);
// PolyEvalProof::prove (no blinds) of a device polynomial of 2^|r| scalars
// (sh.n > 1: the L.Z rows are split over the ranks and the partial vectors summed; the Bullet rounds are replicated)
int poly_eval_prove(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, const FqV& r, const Fq& Zr, Tr& t, Tape& tape,
                    DotProductProofLogP* out, const Shard& sh = Shard());

// ---- SPARK (spark.hip) ----
struct SparsePoly {
  const spg_sparse_entry* e;
  size_t nnz;
};
int spark_commit_polys(spg_ctx* ctx, const std::vector<SparsePoly>& polys, size_t nvx, size_t nvy,
                       const uint8_t* label, size_t label_len, size_t gens_nvx, size_t gens_nvy, size_t gens_nnz,
                       size_t gens_batch, spg_spark** out, const Shard& sh = Shard());
void spark_comm_ser(const spg_spark* S, Writer& w);
// a verifier-side SPARK commitment: the SparseMatPolyCommitment fields (sparse_mlpoly.rs:319-325, read from bytes) with
// the generators SparseMatPolyCommitmentGens::new(label, gens_nvx, gens_nvy, gens_nnz, gens_batch) derives, and no
// dense representation (spg_snark_comm_load); SPG_E_ARG when the fields do not fit those generators
int spark_from_comm(spg_ctx* ctx, size_t B, size_t N, size_t cells, const std::vector<Pt>& comm_ops,
                    const std::vector<Pt>& comm_mem, const uint8_t* label, size_t label_len, size_t gens_nvx,
                    size_t gens_nvy, size_t gens_nnz, size_t gens_batch, spg_spark** out);
void spark_comm_append(const spg_spark* S, Tr& t);
// sh.n > 1: one proof as an SPMD collective over the ranks of sh (every rank holds the whole dense representation
// and returns the same bytes); see spark.hip "sharded proof"
int spark_prove_core(spg_ctx* ctx, spg_spark* S, FqV ex, FqV ey, const FqV& evals, Tr& t, Tape& tape, Writer& w,
                     const Shard& sh = Shard());

// ---- R1CS witness from parts (r1cs.hip) ----
struct WPart {  // one ProverWitnessSecInfo: per instance (num_proofs x num_inputs) scalars at src (host or device)
  std::vector<size_t> num_proofs, num_inputs;
  std::vector<const Fq*> src;
};
int witness_from_parts(spg_ctx* ctx, const std::vector<WPart>& secs, spg_r1cs_witness** inout);

}  // namespace spg

// C-ABI handles of the Fiat-Shamir transcript and the prover random tape
struct spg_transcript {
  spg::Tr t;
  explicit spg_transcript(const char* l) : t(l) {}
};
namespace spg {
// an entry point's return code with a failed transcript callback taking precedence (SPG_E_CALLBACK)
inline int tr_status(spg_ctx* ctx, const Tr& t, int rc) {
  if (t.failed()) return set_err(ctx, SPG_E_CALLBACK, "transcript callback returned " + std::to_string(t.failed()));
  return rc;
}
// for the duration of a sharded prove: every cross-rank exchange carries this transcript's callback failure as the
// rank's status (comm_allgather), so a rank whose caller transcript failed stops every rank in that exchange instead
// of feeding partial sums built from zeroed challenges into it
struct TrFailScope {
  spg_ctx* c;
  TrFailScope(spg_ctx* ctx, const Tr& t) : c(ctx) { c->tr_failed = t.cb ? &t.cb->failed : nullptr; }
  ~TrFailScope() { c->tr_failed = nullptr; }
};
}  // namespace spg
struct spg_random_tape {
  spg::Tape t;
  spg_random_tape(const char* n, const spg::Fq& s) : t(n, s) {}
};
struct spg_r1cs_gens {  // R1CSGens: one derived stream; gens_pc / gens_1 / gens_4 are views of it
  spg::ProverGens g;
};
// SPARK dense representation in HBM (spark.hip) with its commitment and generators (the verifier reads the latter)
struct spg_spark {
  size_t B = 0, N = 0, cells = 0;
  uint32_t* d_addr = nullptr;   // [2][B][N]
  uint32_t* d_rts = nullptr;    // [2][B][N]
  uint32_t* d_audit = nullptr;  // [2][cells]
  spg::Fq* d_val = nullptr;     // [B][N]
  spg::Fq* d_comb_ops = nullptr;
  spg::Fq* d_comb_mem = nullptr;
  size_t comb_ops_len = 0, comb_mem_len = 0;
  spg_gens* dev = nullptr;
  spg::ProverGens g_ops, g_mem, g_der;
  std::vector<spg::Pt> comm_ops, comm_mem;  // SparseMatPolyCommitment
};
namespace spg {
// what SNARK::verify reads of an encoded instance (snark.hip fills it, verify.hip reads it)
struct SnarkCompView {
  size_t num_instances, max_num_cons, num_vars;
  const std::vector<std::vector<size_t>>* label_map;
  const std::vector<spg_spark*>* sparks;
};
int snark_comp_view(const spg_snark_comp* C, SnarkCompView* v);
// a verifier-side encoded instance (spg_snark_comm_load): no sparse matrices, no device instance
spg_snark_comp* snark_comp_from_parts(size_t num_instances, size_t max_num_cons, size_t num_vars,
                                      std::vector<std::vector<size_t>> label_map, std::vector<spg_spark*> sparks);
}  // namespace spg
