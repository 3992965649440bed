// spg — the reference's finer per-operation seams on device-resident vectors (spg_buf): a caller that
// drives its own protocol binds these instead of the whole-proof entries. Each call runs on the context stream and
// returns when its result is ready; the vectors stay in HBM between calls.
//   spg_buf_bound_top      DensePolynomial::bound_poly_var_top   src/dense_mlpoly.rs:267-275
//   spg_buf_bound_bot      DensePolynomial::bound_poly_var_bot   src/dense_mlpoly.rs:350-358
//   spg_buf_evaluate       DensePolynomial::evaluate             src/dense_mlpoly.rs:361-367
//   spg_cubic_round_evals  one round of prove_cubic, comb A B C  src/sumcheck.rs:207-236, src/product_tree.rs:185-189
//   spg_prove_cubic        SumcheckInstanceProof::prove_cubic    src/sumcheck.rs:193-262
//   spg_pqx_*              DensePolynomialPqx new / bound_poly / evaluate   src/custom_dense_mlpoly.rs:45-64, 180-333
#include <hip/hip_runtime.h>
#include <string.h>

#include <vector>

#include "hostpoly.hpp"
#include "proto.hpp"

namespace spg {
namespace {

constexpr size_t kWsSeamPart = 112, kWsSeamTmp = 113;  // (110, 111: the Pqx descriptors, sumcheck.hip)

// bound_poly_var_bot: out[i] = in[2i] + r (in[2i + 1] - in[2i]); out-of-place (in place, a workgroup's outputs would
// overwrite entries another workgroup still reads)
__global__ void k_fold_bot(const Fq* __restrict__ in, Fq* __restrict__ out, size_t n, Fq r) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fq lo = in[2 * i];
  out[i] = fq_add(lo, fq_mul(r, fq_sub(in[2 * i + 1], lo)));
}

// the three tables of a prove_cubic round bound to the same r (bound_poly_var_top of each) in one launch
__global__ void k_fold_top3(Fq* __restrict__ A, Fq* __restrict__ B, Fq* __restrict__ C, size_t n, Fq r) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fq a = A[i], b = B[i], c = C[i];
  A[i] = fq_add(a, fq_mul(r, fq_sub(A[i + n], a)));
  B[i] = fq_add(b, fq_mul(r, fq_sub(B[i + n], b)));
  C[i] = fq_add(c, fq_mul(r, fq_sub(C[i + n], c)));
}

bool pow2(size_t n) { return n && !(n & (n - 1)); }

int d2h(spg_ctx* ctx, void* dst, const void* src, size_t bytes) {
  SPG_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

// (e0, e2, e3) of a prove_cubic round over A, B, C of equal even length
int cubic_round(spg_ctx* ctx, const spg_buf* A, const spg_buf* B, const spg_buf* C, Fq out3[3]) {
  const size_t half = A->n / 2;
  Fq* partials = (Fq*)ws_get(ctx, kWsSeamPart, 3 * kScGridMax * sizeof(Fq) + 64);
  if (!partials) return set_err(ctx, SPG_E_NOMEM, "cubic round partials");
  return cubic_eval(ctx, A->d, B->d, C->d, half, partials, out3);
}

}  // namespace
}  // namespace spg

using spg::Fq;

extern "C" int spg_buf_bound_top(spg_ctx* ctx, spg_buf* b, const uint64_t* r_mont) {
  if (!ctx || !b || !r_mont) return SPG_E_ARG;
  if (b->n < 2 || (b->n & 1)) return spg::set_err(ctx, SPG_E_ARG, "spg_buf_bound_top: length must be even and >= 2");
  int rc = spg::dev_fold_top(ctx, b->d, b->n, spg::ld_fq(r_mont));
  if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = spg::set_err(ctx, SPG_E_HIP, "spg_buf_bound_top");
  if (!rc) b->n /= 2;  // Z.truncate(n): the device allocation keeps its size
  return rc;
}

extern "C" int spg_buf_bound_bot(spg_ctx* ctx, spg_buf* b, const uint64_t* r_mont) {
  if (!ctx || !b || !r_mont) return SPG_E_ARG;
  if (b->n < 2 || (b->n & 1)) return spg::set_err(ctx, SPG_E_ARG, "spg_buf_bound_bot: length must be even and >= 2");
  const size_t n = b->n / 2;
  Fq* tmp = (Fq*)spg::ws_get(ctx, spg::kWsSeamTmp, n * sizeof(Fq) + 64);
  if (!tmp) return spg::set_err(ctx, SPG_E_NOMEM, "spg_buf_bound_bot");
  hipLaunchKernelGGL(spg::k_fold_bot, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, b->d, tmp, n,
                     spg::ld_fq(r_mont));
  SPG_HIP(ctx, hipGetLastError());
  SPG_HIP(ctx, hipMemcpyAsync(b->d, tmp, n * sizeof(Fq), hipMemcpyDeviceToDevice, ctx->stream));
  SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  b->n = n;
  return SPG_OK;
}

// DensePolynomial::evaluate: <Z, chi(r)> with chi = EqPolynomial::evals(r), r[0] the index's most significant bit.
// On the device as ell successive bound_poly_var_top folds of a copy by r[0], r[1], ... : the fold by r_0 leaves
// Z'[i] = (1 - r_0) Z[i] + r_0 Z[i + n/2], so after all ell folds Z''[0] = sum_i chi_i(r) Z[i], the same field value
// as the reference's dot product (exact arithmetic, no rounding to differ).
extern "C" int spg_buf_evaluate(spg_ctx* ctx, const spg_buf* b, const uint64_t* r_mont, size_t ell, uint64_t* out_mont) {
  if (!ctx || !b || !out_mont || (!r_mont && ell)) return SPG_E_ARG;
  if (ell >= 64 || b->n != ((size_t)1 << ell))
    return spg::set_err(ctx, SPG_E_ARG, "spg_buf_evaluate: the vector must hold 2^ell scalars");
  Fq* tmp = (Fq*)spg::ws_get(ctx, spg::kWsSeamTmp, b->n * sizeof(Fq) + 64);
  if (!tmp) return spg::set_err(ctx, SPG_E_NOMEM, "spg_buf_evaluate");
  SPG_HIP(ctx, hipMemcpyAsync(tmp, b->d, b->n * sizeof(Fq), hipMemcpyDeviceToDevice, ctx->stream));
  size_t len = b->n;
  for (size_t j = 0; j < ell; j++, len /= 2) {
    const int rc = spg::dev_fold_top(ctx, tmp, len, spg::ld_fq(r_mont + 4 * j));
    if (rc) return rc;
  }
  Fq v;
  if (int rc = spg::d2h(ctx, &v, tmp, sizeof(Fq))) return rc;
  spg::st_fq(out_mont, v);
  return SPG_OK;
}

extern "C" int spg_cubic_round_evals(spg_ctx* ctx, const spg_buf* A, const spg_buf* B, const spg_buf* C,
                                     uint64_t* out3_mont) {
  if (!ctx || !A || !B || !C || !out3_mont) return SPG_E_ARG;
  if (A->n < 2 || (A->n & 1) || B->n != A->n || C->n != A->n)
    return spg::set_err(ctx, SPG_E_ARG, "spg_cubic_round_evals: A, B, C must have one even length >= 2");
  Fq e[3];
  if (int rc = spg::cubic_round(ctx, A, B, C, e)) return rc;
  for (int k = 0; k < 3; k++) spg::st_fq(out3_mont + 4 * k, e[k]);
  return SPG_OK;
}

// per round: (e0, e2, e3) on the device, UniPoly::from_evals([e0, e - e0, e2, e3]) and its transcript append on the
// host, the challenge, then A, B, C bound in one launch (k_fold_top3) and e = poly(r_j)
extern "C" int spg_prove_cubic(spg_ctx* ctx, const uint64_t* claim_mont, size_t num_rounds, spg_buf* A, spg_buf* B,
                               spg_buf* C, spg_transcript* t, uint64_t* polys_mont, uint64_t* r_mont,
                               uint64_t* claims_mont) {
  if (!ctx || !claim_mont || !A || !B || !C || !t || !claims_mont || (num_rounds && (!polys_mont || !r_mont)))
    return SPG_E_ARG;
  size_t lg = 0;
  while (lg < 63 && ((size_t)1 << lg) < A->n) lg++;
  if (B->n != A->n || C->n != A->n || !spg::pow2(A->n) || num_rounds > lg)
    return spg::set_err(ctx, SPG_E_ARG, "spg_prove_cubic: A, B, C must hold 2^k scalars each, k >= num_rounds");
  Fq e = spg::ld_fq(claim_mont);
  for (size_t j = 0; j < num_rounds; j++) {
    Fq ev[4];
    if (int rc = spg::cubic_round(ctx, A, B, C, ev)) return spg::tr_status(ctx, t->t, rc);
    const Fq evals[4] = {ev[0], spg::fq_sub(e, ev[0]), ev[1], ev[2]};
    const spg::FqV c = spg::uni_from_evals3(evals);
    t->t.msg("poly", "UniPoly_begin");  // UniPoly::append_to_transcript (src/unipoly.rs:112-120)
    for (const Fq& x : c) t->t.scalar("coeff", x);
    t->t.msg("poly", "UniPoly_end");
    const Fq r = t->t.challenge("challenge_nextround");
    const size_t n = A->n / 2;
    hipLaunchKernelGGL(spg::k_fold_top3, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, A->d, B->d,
                       C->d, n, r);
    SPG_HIP(ctx, hipGetLastError());
    A->n = B->n = C->n = n;
    e = spg::uni_eval(c, r);
    // CompressedUniPoly: the coefficients without the linear term (src/unipoly.rs:82-87)
    spg::st_fq(polys_mont + 12 * j, c[0]);
    spg::st_fq(polys_mont + 12 * j + 4, c[2]);
    spg::st_fq(polys_mont + 12 * j + 8, c[3]);
    spg::st_fq(r_mont + 4 * j, r);
  }
  Fq fin[3];
  for (int k = 0; k < 3; k++) {
    const spg_buf* v = k == 0 ? A : k == 1 ? B : C;
    SPG_HIP(ctx, hipMemcpyAsync(&fin[k], v->d, sizeof(Fq), hipMemcpyDeviceToHost, ctx->stream));
  }
  SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (int k = 0; k < 3; k++) spg::st_fq(claims_mont + 4 * k, fin[k]);
  return spg::tr_status(ctx, t->t, SPG_OK);
}

// ---- DensePolynomialPqx (src/custom_dense_mlpoly.rs:22-359) as a handle over the prover's own ragged HBM layout
// (pqx.hpp: instance p owns num_proofs[p] x nws x num_inputs[p] scalars at off[p]; folds rewrite the low halves in
// place and shrink the current sizes, the allocation stays, so index() keeps the reference's bounds semantics)

namespace {
int pqx_bind_one(spg_ctx* ctx, spg::PqxDev& T, const Fq& r, int mode) {
  if (mode < spg::MODE_P || mode > spg::MODE_X) return spg::set_err(ctx, SPG_E_ARG, "DensePolynomialPqx: mode 1..4");
  // bound_poly_p's assert_eq!(max_num_proofs, 1), assert_eq!(max_num_inputs, 1) (custom_dense_mlpoly.rs:206-207)
  if (mode == spg::MODE_P && (T.max_num_proofs != 1 || T.max_num_inputs != 1))
    return spg::set_err(ctx, SPG_E_ARG, "DensePolynomialPqx::bound_poly_p: bind every q and x variable first");
  return spg::pqx_bound(ctx, T, nullptr, nullptr, r, mode);
}
}  // namespace

extern "C" int spg_pqx_new(spg_ctx* ctx, const uint64_t* z_mont, size_t num_instances, const size_t* num_proofs,
                           size_t max_num_proofs, size_t num_witness_secs, const size_t* num_inputs,
                           size_t max_num_inputs, spg_pqx** out) {
  if (!ctx || !out || !num_proofs || !num_inputs || num_instances == 0 || num_witness_secs == 0) return SPG_E_ARG;
  if (!spg::pow2(max_num_proofs) || !spg::pow2(max_num_inputs))
    return spg::set_err(ctx, SPG_E_ARG, "spg_pqx_new: max_num_proofs / max_num_inputs must be powers of two");
  spg_pqx* h = new spg_pqx();
  spg::PqxDev& T = h->T;
  T.zlen = num_instances;
  size_t total = 0;
  for (size_t p = 0; p < num_instances; p++) {
    if (!spg::pow2(num_proofs[p]) || num_proofs[p] > max_num_proofs || !spg::pow2(num_inputs[p]) ||
        num_inputs[p] > max_num_inputs) {
      delete h;
      return spg::set_err(ctx, SPG_E_ARG, "spg_pqx_new: num_proofs[p] / num_inputs[p] must be powers of two <= max");
    }
    T.off.push_back(total);
    T.anp.push_back(num_proofs[p]);
    T.anw.push_back(num_witness_secs);
    T.ani.push_back(num_inputs[p]);
    total += num_proofs[p] * num_witness_secs * num_inputs[p];
  }
  if (total >= ((size_t)1 << 31) || !z_mont) {  // the fold kernels index the domain with 32-bit lanes
    delete h;
    return spg::set_err(ctx, SPG_E_ARG, "spg_pqx_new: at most 2^31 scalars, z required");
  }
  T.total = total;
  T.num_instances = 1;
  while (T.num_instances < num_instances) T.num_instances *= 2;
  T.num_witness_secs = 1;
  while (T.num_witness_secs < num_witness_secs) T.num_witness_secs *= 2;
  T.max_num_proofs = max_num_proofs;
  T.max_num_inputs = max_num_inputs;
  T.num_proofs.assign(num_proofs, num_proofs + num_instances);
  T.num_inputs.assign(num_inputs, num_inputs + num_instances);
  if (hipMalloc(&T.d, total * sizeof(Fq) + 64) != hipSuccess) {
    delete h;
    return spg::set_err(ctx, SPG_E_NOMEM, "spg_pqx_new");
  }
  if (hipMemcpy(T.d, z_mont, total * sizeof(Fq), hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(T.d);
    delete h;
    return spg::set_err(ctx, SPG_E_HIP, "spg_pqx_new: upload");
  }
  *out = h;
  return SPG_OK;
}

extern "C" int spg_pqx_free(spg_ctx* ctx, spg_pqx* h) {
  (void)ctx;
  if (!h) return SPG_OK;
  hipFree(h->T.d);
  delete h;
  return SPG_OK;
}

// the current sizes: dims = (num_instances, max_num_proofs, num_witness_secs, max_num_inputs); num_proofs /
// num_inputs (optional) receive Z.len() entries each
extern "C" int spg_pqx_shape(const spg_pqx* h, size_t* dims, size_t* num_proofs, size_t* num_inputs) {
  if (!h || !dims) return SPG_E_ARG;
  const spg::PqxDev& T = h->T;
  dims[0] = T.num_instances;
  dims[1] = T.max_num_proofs;
  dims[2] = T.num_witness_secs;
  dims[3] = T.max_num_inputs;
  for (size_t p = 0; p < T.zlen; p++) {
    if (num_proofs) num_proofs[p] = T.num_proofs[p];
    if (num_inputs) num_inputs[p] = T.num_inputs[p];
  }
  return SPG_OK;
}

// Z in spg_pqx_new's layout (every allocated entry, folded or not)
extern "C" int spg_pqx_download(spg_ctx* ctx, const spg_pqx* h, uint64_t* z_mont) {
  if (!ctx || !h || !z_mont) return SPG_E_ARG;
  SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  SPG_HIP(ctx, hipMemcpy(z_mont, h->T.d, h->T.total * sizeof(Fq), hipMemcpyDeviceToHost));
  return SPG_OK;
}

// DensePolynomialPqx::bound_poly (custom_dense_mlpoly.rs:180-199): mode 1 p, 2 q, 3 w, 4 x
extern "C" int spg_pqx_bound(spg_ctx* ctx, spg_pqx* h, const uint64_t* r_mont, int mode) {
  if (!ctx || !h || !r_mont) return SPG_E_ARG;
  int rc = pqx_bind_one(ctx, h->T, spg::ld_fq(r_mont), mode);
  if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = spg::set_err(ctx, SPG_E_HIP, "spg_pqx_bound");
  return rc;
}

// DensePolynomialPqx::evaluate (custom_dense_mlpoly.rs:320-333): a clone bound by r_x, r_w, r_q, r_p in that order,
// then index(0, 0, 0, 0); h is left unchanged
extern "C" int spg_pqx_evaluate(spg_ctx* ctx, const spg_pqx* h, const uint64_t* rp, size_t np, const uint64_t* rq,
                                size_t nq, const uint64_t* rw, size_t nw, const uint64_t* rx, size_t nx,
                                uint64_t* out_mont) {
  if (!ctx || !h || !out_mont || (np && !rp) || (nq && !rq) || (nw && !rw) || (nx && !rx)) return SPG_E_ARG;
  spg::PqxDev C = h->T;  // the clone: same descriptors and sizes, its own copy of the entries
  C.d = (Fq*)spg::ws_get(ctx, spg::kWsSeamTmp, C.total * sizeof(Fq) + 64);
  if (!C.d) return spg::set_err(ctx, SPG_E_NOMEM, "spg_pqx_evaluate");
  SPG_HIP(ctx, hipMemcpyAsync(C.d, h->T.d, C.total * sizeof(Fq), hipMemcpyDeviceToDevice, ctx->stream));
  const struct {
    const uint64_t* r;
    size_t n;
    int mode;
  } secs[4] = {{rx, nx, spg::MODE_X}, {rw, nw, spg::MODE_W}, {rq, nq, spg::MODE_Q}, {rp, np, spg::MODE_P}};
  for (const auto& s : secs)
    for (size_t i = 0; i < s.n; i++)
      if (int rc = pqx_bind_one(ctx, C, spg::ld_fq(s.r + 4 * i), s.mode)) return rc;
  // index(0, 0, 0, 0): Z[0][0][0][0] when that entry is allocated (custom_dense_mlpoly.rs:118-128)
  Fq v = spg::fq_zero();
  if (C.zlen && C.anp[0] && C.anw[0] && C.ani[0])
    if (int rc = spg::d2h(ctx, &v, C.d, sizeof(Fq))) return rc;
  spg::st_fq(out_mont, v);
  return SPG_OK;
}

// One round of SumcheckInstanceProof::prove_cubic_with_additive_term_disjoint_rounds (src/sumcheck.rs:1067-1380,
// round loop :1173-1245; comb A (B C - D), src/r1csproof.rs) in an x or q round: (e0, e2, e3) over the eq factors
// Ap, Aq, Ax (dense, their current lengths: the round's instance_len = |Ap|, proof_len = |Aq| (/ 2 in a q round),
// cons_len = |Ax| (/ 2 in an x round)) and B, C, D (Pqx tables of one shape, one witness section) in their current
// state -- the reference's local num_proofs / num_cons are the tables' own sizes, halved at the round start as there.
// The prover's phase-1 evaluation kernels do the work.
extern "C" int spg_phase1_round_evals(spg_ctx* ctx, const spg_buf* Ap, const spg_buf* Aq, const spg_buf* Ax,
                                      const spg_pqx* B, const spg_pqx* C, const spg_pqx* D, int mode,
                                      uint64_t* out3_mont) {
  if (!ctx || !Ap || !Aq || !Ax || !B || !C || !D || !out3_mont) return SPG_E_ARG;
  const spg::PqxDev& T = B->T;
  for (const spg_pqx* o : {C, D})
    if (o->T.zlen != T.zlen || o->T.anp != T.anp || o->T.anw != T.anw || o->T.ani != T.ani ||
        o->T.num_proofs != T.num_proofs || o->T.num_inputs != T.num_inputs)
      return spg::set_err(ctx, SPG_E_ARG, "phase-1 round: B, C, D must share one shape");
  if (T.num_witness_secs != 1)  // sumcheck.rs:1099-1102 assert_eq!(poly_B.num_witness_secs, 1)
    return spg::set_err(ctx, SPG_E_ARG, "phase-1 round: one witness section");
  if (mode != spg::MODE_X && mode != spg::MODE_Q)
    return spg::set_err(ctx, SPG_E_ARG, "phase-1 round: mode 4 (x) or 2 (q); the p rounds run on the host-sized tail");
  if (!spg::pow2(Ap->n) || !spg::pow2(Aq->n) || !spg::pow2(Ax->n) || Ap->n < T.zlen)
    return spg::set_err(ctx, SPG_E_ARG, "phase-1 round: eq tables of power-of-two lengths, |Ap| >= instances");
  if (mode == spg::MODE_X ? Ax->n < 2 : (Ax->n != 1 || Aq->n < 2))
    return spg::set_err(ctx, SPG_E_ARG, "phase-1 round: x rounds first (|Ax| >= 2), q rounds once |Ax| = 1");
  const size_t instance_len = Ap->n, proof_len = mode == spg::MODE_Q ? Aq->n / 2 : Aq->n,
               cons_len = mode == spg::MODE_X ? Ax->n / 2 : 1;
  std::vector<size_t> sc_np = T.num_proofs, sc_nc = T.num_inputs;
  for (size_t p = 0; p < T.zlen; p++) {
    if (mode == spg::MODE_X && sc_nc[p] > 1) sc_nc[p] /= 2;
    if (mode == spg::MODE_Q && sc_np[p] > 1) sc_np[p] /= 2;
    if (proof_len % sc_np[p] || cons_len % sc_nc[p])
      return spg::set_err(ctx, SPG_E_ARG, "phase-1 round: table sizes exceed the eq tables");
  }
  Fq* partials = (Fq*)spg::ws_get(ctx, spg::kWsSeamPart,
                                  std::max(3 * (size_t)spg::kScGridMax, spg::kP1PairMax) * sizeof(Fq) + 64);
  if (!partials) return spg::set_err(ctx, SPG_E_NOMEM, "phase-1 round partials");
  Fq e[3];
  const int rc = spg::phase1_eval(ctx, T, mode, proof_len, cons_len, instance_len, sc_np, sc_nc, Ap->d, Aq->d, Ax->d,
                                  T.d, C->T.d, D->T.d, partials, e);
  if (rc) return rc;
  for (int k = 0; k < 3; k++) spg::st_fq(out3_mont + 4 * k, e[k]);
  return SPG_OK;
}

// One round of the R1CS proof's phase-2 sumcheck (SumcheckInstanceProof::prove_cubic_disjoint_rounds,
// src/sumcheck.rs:788-1065, round loop :881-941; comb A B C): (e0, e2, e3) over eq(r_p) (A, current length:
// instance_len = |A|, / 2 in a p round), ABC (one instance when single_inst, else one per instance) and Z in their
// current state, in a y (mode 4), w (mode 3) or p (mode 1) round; num_witness_secs: the reference's argument (the
// sections that exist); witness_secs_len and the local num_inputs are Z's own sizes, halved at the round start.
extern "C" int spg_phase2_round_evals(spg_ctx* ctx, const spg_buf* A, const spg_pqx* ABC, const spg_pqx* Z, int mode,
                                      int single_inst, size_t num_witness_secs, uint64_t* out3_mont) {
  if (!ctx || !A || !ABC || !Z || !out3_mont || num_witness_secs == 0) return SPG_E_ARG;
  const spg::PqxDev &TA = ABC->T, &TZ = Z->T;
  if (mode != spg::MODE_X && mode != spg::MODE_W && mode != spg::MODE_P)
    return spg::set_err(ctx, SPG_E_ARG, "phase-2 round: mode 4 (y), 3 (w) or 1 (p)");
  if (single_inst ? TA.zlen != 1 : TA.zlen != TZ.zlen)
    return spg::set_err(ctx, SPG_E_ARG, "phase-2 round: ABC holds one instance (single_inst) or one per instance");
  if (!spg::pow2(A->n) || (mode == spg::MODE_P && A->n < 2))  // (the loop runs p < min(instance_len, instances))
    return spg::set_err(ctx, SPG_E_ARG, "phase-2 round: eq(r_p) of power-of-two length (>= 2 in a p round)");
  if ((mode == spg::MODE_X && TZ.max_num_inputs < 2) ||
      (mode == spg::MODE_W && (TZ.max_num_inputs != 1 || TZ.num_witness_secs < 2)) ||
      (mode == spg::MODE_P && (TZ.max_num_inputs != 1 || TZ.num_witness_secs != 1)))
    return spg::set_err(ctx, SPG_E_ARG, "phase-2 round: y rounds, then w rounds, then p rounds");
  for (const spg::PqxDev* T : {&TA, &TZ})
    for (size_t p = 0; p < T->zlen; p++)
      if (T->anp[p] != 1) return spg::set_err(ctx, SPG_E_ARG, "phase-2 round: tables of one proof row (q bound)");
  const size_t instance_len = mode == spg::MODE_P ? A->n / 2 : A->n;
  const size_t ws_len = mode == spg::MODE_W ? TZ.num_witness_secs / 2 : TZ.num_witness_secs;
  std::vector<size_t> sc_ni = TZ.num_inputs;
  for (size_t p = 0; p < sc_ni.size(); p++)
    if (mode == spg::MODE_X && sc_ni[p] > 1) sc_ni[p] /= 2;
  Fq* partials = (Fq*)spg::ws_get(ctx, spg::kWsSeamPart,
                                  std::max(3 * (size_t)spg::kScGridMax, spg::kP1PairMax) * sizeof(Fq) + 64);
  if (!partials) return spg::set_err(ctx, SPG_E_NOMEM, "phase-2 round partials");
  Fq e[3];
  const int rc = spg::phase2_eval(ctx, TA, TZ, mode, instance_len, ws_len, num_witness_secs, single_inst != 0, sc_ni,
                                  A->d, partials, e);
  if (rc) return rc;
  for (int k = 0; k < 3; k++) spg::st_fq(out3_mont + 4 * k, e[k]);
  return SPG_OK;
}
