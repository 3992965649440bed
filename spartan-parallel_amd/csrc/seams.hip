// spg — the reference's finer per-operation seams on device-resident vectors (spg_buf): a caller that
// drives its own protocol binds these instead of the whole-proof entries. Each call runs on the context stream and
// returns when its result is ready; the vectors stay in HBM between calls.
//   spg_buf_bound_top      DensePolynomial::bound_poly_var_top   src/dense_mlpoly.rs:267-275
//   spg_buf_bound_bot      DensePolynomial::bound_poly_var_bot   src/dense_mlpoly.rs:350-358
//   spg_buf_evaluate       DensePolynomial::evaluate             src/dense_mlpoly.rs:361-367
//   spg_cubic_round_evals  one round of prove_cubic, comb A B C  src/sumcheck.rs:207-236, src/product_tree.rs:185-189
//   spg_prove_cubic        SumcheckInstanceProof::prove_cubic    src/sumcheck.rs:193-262
#include <hip/hip_runtime.h>
#include <string.h>

#include <vector>

#include "hostpoly.hpp"
#include "proto.hpp"

namespace spg {
namespace {

constexpr size_t kWsSeamPart = 110, kWsSeamTmp = 111;

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
