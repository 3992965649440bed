// spg — internal interface of the sumcheck / fold kernels (sumcheck.hip).
#pragma once
#include <algorithm>
#include <vector>

#include "ctx.hpp"
#include "pqx.hpp"

namespace spg {

enum { MODE_P = 1, MODE_Q = 2, MODE_W = 3, MODE_X = 4 };  // src/custom_dense_mlpoly.rs:11-14

struct FqArg32 {
  Fq v[32];
  int n;
};

// A small host blob that rides in an eq-table launch's kernel arguments and is written to device memory by it,
// instead of a separate host-to-device copy on the stream (the SPARK layers' descriptors and coefficients).
struct KBlob {
  static constexpr int kWords = 576;  // 2304 B: with FqArg32 the arguments stay well under 4 KB
  uint32_t w[kWords];
  int nwords;
};
// EqPolynomial::evals(r[0..ell]) into out[2^ell] (device); with blob, also blob->w[0..nwords) -> blob_dst
int dev_eq_table(spg_ctx* ctx, const Fq* r, int ell, Fq* out, const KBlob* blob = nullptr, void* blob_dst = nullptr);
// several EqPolynomial::evals tables at once: tables of <= 2^16 entries share launches (up to
// EqTablesArg::kMax per launch), larger ones go through dev_eq_table
struct EqJob {
  const Fq* r;
  int ell;
  Fq* out;
};
struct EqTablesArg {  // kernel argument of k_eq_tables_lds
  static constexpr int kMax = 3;
  FqArg32 r[kMax];
  Fq* out[kMax];
  uint64_t n[kMax];
  uint32_t b0[kMax];  // first block of table k
  int nj;
};
int dev_eq_tables(spg_ctx* ctx, const EqJob* jobs, int nj);
// DensePolynomial::bound_poly_var_top on a device vector of length len
int dev_fold_top(spg_ctx* ctx, Fq* v, size_t len, const Fq& r);

// the previous round's fold, applied by the phase-1 evaluation that follows it (one launch: fused fold + eval)
struct FoldArg {  // kernel argument
  Fq r;
  int fmode;            // MODE_X: the side table is Ax; MODE_Q: Aq
  const Fq* side_in;    // the side eq table before the fold (2 side_half entries)
  Fq* side_out;         // its folded half (the other ping-pong buffer)
  uint32_t side_half;
};
struct FoldPlan {
  FoldArg arg;
  std::vector<uint32_t> stride;  // per instance: element stride to the fold partner (0: scale by 1 - r)
  uint32_t fw = 0;               // mode W: the witness-section count after the fold (a partner exists iff w + fw < anw)
};
// DensePolynomialPqx::bound_poly's size bookkeeping for mode X, Q or W on the host, without a launch; the fold itself
// is then carried by the next phase1_eval / phase2_eval (fold != nullptr)
int pqx_fold_plan(spg_ctx* ctx, PqxDev& T, int mode, FoldPlan* fp);
// phase 2's pending fold of ABC and Z, applied by the next phase2_eval
struct Fold2Arg {  // kernel argument
  Fq r;
  int fmode;     // MODE_X or MODE_W
  uint32_t fw;
  Fq* b_out;     // ABC's folded entries: ABC itself, or its ping-pong buffer when one ABC serves every instance
  int ping;      // b_out is the ping-pong buffer (written by instance 0's points only)
};
struct Fold2 {
  FoldPlan a, z;  // strides of ABC and Z
  Fold2Arg arg;
};

// one phase-1 round: (e0, e2, e3) of eq(p,q,x) * (B*C - D)  (src/sumcheck.rs:1173-1245)
// most workgroups a round evaluation launches (its partials buffer holds 3 scalars per workgroup)
constexpr int kScGridMax = 4096;
int phase1_eval(spg_ctx* ctx, const PqxDev& T, int mode, size_t proof_len, size_t cons_len, size_t instance_len,
                const std::vector<size_t>& sc_np, const std::vector<size_t>& sc_nc, const Fq* Ap, const Fq* Aq,
                const Fq* Ax, Fq* B, Fq* C, Fq* D, Fq* partials, Fq* out3, const FoldPlan* fold = nullptr);
// two phase-1 rounds in one launch (sumcheck.hip, k_phase1_pair): F = A (B C - D) posted on 15 points of round j's and
// round j + 1's 4 x 4 grid -- g 0..3: (t, s) = (g, 0); 4..7: (g - 4, 2); 8..11: (g - 8, 3); 12, 13, 14: (0, 1),
// (2, 1), (3, 1) -- with the pending fold(s) applied on the way (nf 0, 1: fstride per instance, 2: the previous pair's)
// elements (16 lanes each; 16 partials per 256-thread workgroup in `partials`: one Fq per element); the default cap is
// SPG_P1_PAIR_MAX / SPG_P2_PAIR_MAX (8192), this is the largest a caller may ask
constexpr size_t kP1PairMax = 32768;
struct P1Pair {
  int mode = MODE_X;
  std::vector<size_t> rows, cols, step_q, step_x;
  size_t c = 0;
  int nf = 0;
  Fq r1 = fq_zero(), r2 = fq_zero();
  int fmode = MODE_X;
  std::vector<uint32_t> fstride;
  const Fq* side_in = nullptr;
  Fq* side_out = nullptr;
  size_t side_live = 0;
  const Fq *Ap = nullptr, *Aq = nullptr, *Ax = nullptr;
  Fq *B = nullptr, *C = nullptr, *D = nullptr;
};
int phase1_pair(spg_ctx* ctx, const PqxDev& T, const P1Pair& pp, Fq* partials, Fq* out15);
int pair_wait(spg_ctx* ctx, Fq* out15);
int phase1_fold2x(spg_ctx* ctx, const PqxDev& T, const P1Pair& pp);
// two phase-2 y rounds in one launch (k_phase2_pair): eq(p) ABC Z on the 4 x 4 grid of rounds j, j + 1, with ABC
// per instance or one shared ABC (B_out) and every instance's live y size >= 4 in both tables; nf = 2: the previous pair's folds
// (r1, r2) pending in both tables. W: witness-section rows per instance; eq: eq(rp) at the local instances.
struct P2Pair {
  int nf = 0;
  Fq r1 = fq_zero(), r2 = fq_zero();
  size_t W = 0;
  const Fq* eq = nullptr;
  Fq* B_out = nullptr;  // one ABC shared by every instance: the other buffer of its ping-pong pair (null: per instance)
};
int phase2_pair(spg_ctx* ctx, const PqxDev& AB, const PqxDev& Z, const P2Pair& pp, Fq* partials);
// the last pair's two y folds of ABC and Z (sizes: after both folds), before the next single round
int phase2_fold2x(spg_ctx* ctx, const PqxDev& AB, const PqxDev& Z, const P2Pair& pp);
// one phase-2 round: (e0, e2, e3) of eq(p) * ABC * Z  (src/sumcheck.rs:881-941)
int phase2_eval(spg_ctx* ctx, const PqxDev& AB, const PqxDev& Z, int mode, size_t instance_len,
                size_t witness_secs_len, size_t nws_actual, bool single, const std::vector<size_t>& sc_ni,
                const Fq* eq, Fq* partials, Fq* out3, const Fold2* fold = nullptr);
// DensePolynomialPqx::bound_poly on T (and d1, d2 sharing T's shape, may be null)
// side (optional): a dense vector of side_len entries bound by the same r in the same launch
// (DensePolynomial::bound_poly_var_top, as dev_fold_top) - the round's eq factor in phase 1
int pqx_bound(spg_ctx* ctx, PqxDev& T, Fq* d1, Fq* d2, const Fq& r, int mode, Fq* side = nullptr, size_t side_len = 0);
// two single-table folds of different shapes with the same r in one launch
int pqx_bound2(spg_ctx* ctx, PqxDev& TA, PqxDev& TB, const Fq& r, int mode);
// nq q-mode folds (r_0 .. r_{nq-1}) of T in one launch (k_pqx_bound_q); E: eq(r_0 .. r_{nq-1}) on the device
int pqx_bound_q_all(spg_ctx* ctx, PqxDev& T, const Fq* E, size_t nq);
// SumcheckInstanceProof::prove_cubic round on dense A, B, C of length 2*len_half
int cubic_eval(spg_ctx* ctx, const Fq* A, const Fq* B, const Fq* C, size_t len_half, Fq* partials,
               Fq* out3);
// The *_eval calls above return (e0, e2, e3) in out3; with out3 == nullptr they only enqueue the work
// and eval_wait() later blocks for the values (host work of the round runs in between).
int eval_wait(spg_ctx* ctx, Fq* out3);
// waits for the three scalars the last fused eval kernel posts to the host mailbox (no-op if out3 == nullptr)
int eval_reduce_finish(spg_ctx* ctx, Fq* out3);

}  // namespace spg
