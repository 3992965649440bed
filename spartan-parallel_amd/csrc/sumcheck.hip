// spg — sumcheck round evaluation and folding on MI355X.
//
// Replaces the inner loops of
//   ZKSumcheckInstanceProof::prove_cubic_with_additive_term_disjoint_rounds (src/sumcheck.rs:1173-1245)
//   ZKSumcheckInstanceProof::prove_cubic_disjoint_rounds                     (src/sumcheck.rs:881-941)
//   SumcheckInstanceProof::prove_cubic_batched                               (src/sumcheck.rs:300-367)
// and the folds DensePolynomial::bound_poly_var_top (src/dense_mlpoly.rs:267-275) and
// DensePolynomialPqx::bound_poly_{p,q,w,x} (src/custom_dense_mlpoly.rs:205-289).
//
// Every round is one streaming pass over HBM-resident tables: each thread accumulates exact Fq
// partial sums of (e0, e2, e3) over a grid-stride slice, a 256-thread block tree-reduces them in LDS
// and a one-block kernel sums the block partials. Reduction order is irrelevant (exact arithmetic).
#include <string.h>

#include "cube.hpp"
#include "lds.hpp"
#include "qsum.hpp"
#include "sumcheck.hpp"

namespace spg {

__device__ __forceinline__ int find_inst(const PqxArgs& a, uint32_t t) {
  int p = 0;
  for (int k = 1; k < a.P; k++)
    if (pinst(a, k).dom_off <= t) p = k;
  return p;
}

// block-wide sums of three Fq values over a 256-thread block, valid in every thread: butterflies across each wave
// (six shuffle steps), then the four wave sums through 384 bytes of LDS, added by every thread in one order. (A
// 256-entry LDS tree here held 24.6 KB of LDS per workgroup, which capped k_phase1_eval at 6 workgroups per CU.)
__device__ __forceinline__ void block_sum3(Fq& v0, Fq& v1, Fq& v2) {
  __shared__ uint32_t sh[4][3][8];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    v0 = fq_add(v0, fq_shfl_xor(v0, m));
    v1 = fq_add(v1, fq_shfl_xor(v1, m));
    v2 = fq_add(v2, fq_shfl_xor(v2, m));
  }
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < 8; j++) {
      sh[w][0][j] = v0.l[j];
      sh[w][1][j] = v1.l[j];
      sh[w][2][j] = v2.l[j];
    }
  __syncthreads();
  Fq s[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
#pragma unroll
    for (int j = 0; j < 8; j++) s[k].l[j] = sh[0][k][j];
    for (int v = 1; v < 4; v++) {
      Fq o;
#pragma unroll
      for (int j = 0; j < 8; j++) o.l[j] = sh[v][k][j];
      s[k] = fq_add(s[k], o);
    }
  }
  v0 = s[0];
  v1 = s[1];
  v2 = s[2];
  __syncthreads();
}

// Grid-wide (e0, e2, e3): every block publishes its partial sums; the last block to finish (ticket on
// `counter`) adds all partials and posts them to the host mailbox (mbox_post), then re-arms the counter. One launch per round.
// Cross-XCD hand-off: plain stores + agent-scope release before the ticket, agent-scope acquire in
// the reducer before plain loads (MI355X L2s are per-XCD and not coherent).
__device__ __forceinline__ void grid_reduce3(Fq v0, Fq v1, Fq v2, Fq* __restrict__ partials,
                                             unsigned* __restrict__ counter, uint32_t* __restrict__ mb, uint32_t seq) {
  __shared__ bool last;
  block_sum3(v0, v1, v2);
  const int t = threadIdx.x;
  if (gridDim.x == 1) {  // a one-block round posts directly: no partials, ticket or second reduction
    if (t == 0) {
      mbox_post3(mb, seq, v0, v1, v2);
    }
    return;
  }
  if (t == 0) {
    partials[3 * blockIdx.x] = v0;
    partials[3 * blockIdx.x + 1] = v1;
    partials[3 * blockIdx.x + 2] = v2;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  Fq a = fq_zero(), b = fq_zero(), c = fq_zero();
  for (unsigned i = t; i < gridDim.x; i += 256) {
    a = fq_add(a, partials[3 * i]);
    b = fq_add(b, partials[3 * i + 1]);
    c = fq_add(c, partials[3 * i + 2]);
  }
  block_sum3(a, b, c);
  if (t == 0) {
    mbox_post3(mb, seq, a, b, c);
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// EqPolynomial::evals (src/dense_mlpoly.rs:76-92): out[b] = prod_j (bit_{ell-1-j}(b) ? r_j : 1 - r_j)
template <bool BLOB>
__global__ void k_eq_table(FqArg32 r, Fq* __restrict__ out, size_t n, KBlob blob, uint32_t* __restrict__ blob_dst) {
  size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (BLOB && blockIdx.x == 0)
    for (int i = threadIdx.x; i < blob.nwords; i += blockDim.x) blob_dst[i] = blob.w[i];
  if (b >= n) return;
  // factors in groups of four: each group's product is independent of the running product, so the
  // dependent chain is ell/4 + 2 multiplications instead of ell
  auto factor = [&](int j) {
    const bool bit = (b >> (r.n - 1 - j)) & 1;
    return bit ? r.v[j] : fq_sub(fq_one(), r.v[j]);
  };
  Fq acc = fq_one();
  bool first = true;
  int j = 0;
  for (; j + 4 <= r.n; j += 4) {
    const Fq p = fq_mul(fq_mul(factor(j), factor(j + 1)), fq_mul(factor(j + 2), factor(j + 3)));
    acc = first ? p : fq_mul(acc, p);
    first = false;
  }
  for (; j < r.n; j++) {
    const Fq f = factor(j);
    acc = first ? f : fq_mul(acc, f);
    first = false;
  }
  out[b] = acc;
}

// product of the eq factors of bits k0 .. k0+nb-1 of an index whose bits there are v (bit k <-> r[ell-1-k]),
// in groups of four (dependent chain nb/4 + 2 multiplications)
__device__ __forceinline__ Fq eq_bits(const Fq* rv, int ell, int k0, int nb, uint32_t v) {
  auto factor = [&](int i) {
    const Fq& rj = rv[ell - 1 - (k0 + i)];
    return ((v >> i) & 1) ? rj : fq_sub(fq_one(), rj);
  };
  Fq acc = fq_one();
  bool first = true;
  int i = 0;
  for (; i + 4 <= nb; i += 4) {
    const Fq p = fq_mul(fq_mul(factor(i), factor(i + 1)), fq_mul(factor(i + 2), factor(i + 3)));
    acc = first ? p : fq_mul(acc, p);
    first = false;
  }
  for (; i < nb; i++) {
    const Fq f = factor(i);
    acc = first ? f : fq_mul(acc, f);
    first = false;
  }
  return acc;
}

// Same table from LDS sub-tables: a block owns 2^lb consecutive entries (lb = min(ell, 8)); the low bits
// split into two groups of <= 4 whose 16-entry factor tables and the block's high-bit product are built
// by lanes of three different waves at once, then every entry is two multiplications. A lane's chain is
// ~5 products instead of ell - 1 (+ ell/4 grouping): the launch is latency-bound at these sizes.
// the table's entries [bid * 256, bid * 256 + 256) of one block
__device__ __forceinline__ void eq_lds_block(const FqArg32& r, Fq* __restrict__ out, size_t n, uint32_t bid) {
  __shared__ Fq s_lo[16], s_mid[16], s_hi;
  __shared__ Fq s_r[32];
  const int t = threadIdx.x;
  const int ell = r.n;
  // the challenges reach LDS in one parallel round trip (one word per lane) instead of a chain of
  // scalar loads from the argument segment inside every lane's product loop
  if (t < ell * 8) reinterpret_cast<uint32_t*>(s_r)[t] = reinterpret_cast<const uint32_t*>(r.v)[t];
  __syncthreads();
  const int lb = ell < 8 ? ell : 8;
  const int nlo = lb >> 1, nmid = lb - nlo, nhi = ell - lb;
  if (t < (1 << nlo)) s_lo[t] = eq_bits(s_r, ell, 0, nlo, (uint32_t)t);
  else if (t >= 64 && t < 64 + (1 << nmid)) s_mid[t - 64] = eq_bits(s_r, ell, nlo, nmid, (uint32_t)(t - 64));
  else if (t == 128) s_hi = eq_bits(s_r, ell, lb, nhi, bid);
  __syncthreads();
  const size_t b = (size_t)bid * blockDim.x + t;
  if (b >= n) return;
  Fq v = fq_mul(s_mid[t >> nlo], s_lo[t & ((1 << nlo) - 1)]);
  if (nhi) v = fq_mul(v, s_hi);
  out[b] = v;
}

// Same table from LDS sub-tables: a block owns 2^lb consecutive entries (lb = min(ell, 8)); the low bits
// split into two groups of <= 4 whose 16-entry factor tables and the block's high-bit product are built
// by lanes of three different waves at once, then every entry is two multiplications. A lane's chain is
// ~5 products instead of ell - 1 (+ ell/4 grouping): the launch is latency-bound at these sizes.
template <bool BLOB>
__global__ void __launch_bounds__(256) k_eq_table_lds(FqArg32 r, Fq* __restrict__ out, size_t n, KBlob blob,
                                                      uint32_t* __restrict__ blob_dst) {
  if (BLOB && blockIdx.x == 0)
    for (int i = threadIdx.x; i < blob.nwords; i += blockDim.x) blob_dst[i] = blob.w[i];
  eq_lds_block(r, out, n, blockIdx.x);
}

// up to three tables in one launch (their blocks back to back): the tables a prover needs at one point
// (tau_p, tau_q, tau_x; eq(rx), eq(ry); ...) cost one launch on the stream instead of one each
__global__ void __launch_bounds__(256) k_eq_tables_lds(EqTablesArg a) {
  const uint32_t bx = blockIdx.x;
  if (a.nj > 2 && bx >= a.b0[2]) eq_lds_block(a.r[2], a.out[2], a.n[2], bx - a.b0[2]);
  else if (a.nj > 1 && bx >= a.b0[1]) eq_lds_block(a.r[1], a.out[1], a.n[1], bx - a.b0[1]);
  else eq_lds_block(a.r[0], a.out[0], a.n[0], bx);
}

// factored form for large tables: out[b] = hi[b >> lo_bits] * lo[b & (2^lo_bits - 1)]
__global__ void k_eq_combine(const Fq* __restrict__ hi, const Fq* __restrict__ lo, int lo_bits, Fq* __restrict__ out,
                             size_t n) {
  size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  out[b] = fq_mul(hi[b >> lo_bits], lo[b & (((size_t)1 << lo_bits) - 1)]);
}

// bound_poly_var_top on a dense vector of length 2n (in place, first n outputs)
__global__ void k_fold_top(Fq* __restrict__ v, size_t n, Fq r) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fq lo = v[i];
  v[i] = fq_add(lo, fq_mul(r, fq_sub(v[i + n], lo)));
}

// ---------------------------------------------------------------- phase 1 round evaluation
// Fused fold + eval (FOLD): the previous round's bound_poly_var_{x,q} of Az, Bz, Cz and of its eq side table is applied
// by this round's evaluation to exactly the entries it reads. Every live entry of the folded tables is the lo or the hi
// entry of one domain point, so the thread that reads it folds it (T[s] + r (T[s + fstride] - T[s]), or (1 - r) T[s]
// for a dimension already of size 1) and writes it back in place; the partner entries lie outside the new live region
// and nobody writes them. The side table is folded into the other ping-pong buffer (its old entries are read by many
// points), by a grid-stride pass over its new half. One launch per round instead of two.
// the lo and hi entries (hi only when present) and their partners, all loaded before anything is written back (a
// store between them would order the hi loads behind the lo product), folded, then written back in place
__device__ __forceinline__ void fold_pair_rw(Fq* T, size_t lo_i, size_t hi_i, bool has_hi, uint32_t fs, const Fq& r,
                                             const Fq& omr, Fq& lo, Fq& hi) {
  const Fq a = T[lo_i], ap = fs ? T[lo_i + fs] : a;
  Fq b = fq_zero(), bp = fq_zero();
  if (has_hi) {
    b = T[hi_i];
    bp = fs ? T[hi_i + fs] : b;
  }
  lo = fs ? fq_add(a, fq_mul(r, fq_sub(ap, a))) : fq_mul(omr, a);
  hi = has_hi ? (fs ? fq_add(b, fq_mul(r, fq_sub(bp, b))) : fq_mul(omr, b)) : fq_zero();
  T[lo_i] = lo;
  if (has_hi) T[hi_i] = hi;
}
__device__ __forceinline__ Fq fold_side(const FoldArg& F, uint32_t i) {
  const Fq lo = F.side_in[i];
  return fq_add(lo, fq_mul(F.r, fq_sub(F.side_in[i + F.side_half], lo)));
}
// the side table's new half: by the threads the round's points leave idle when there are enough of them (so its
// load-multiply-store chain is not in front of a busy thread's point), else by every thread, grid-stride
__device__ __forceinline__ void fold_side_pass(const FoldArg& F, uint32_t gt, uint32_t gstride, uint32_t busy) {
  if (busy <= gstride && gstride - busy >= F.side_half) {
    if (gt >= busy && gt - busy < F.side_half) F.side_out[gt - busy] = fold_side(F, gt - busy);
    return;
  }
  for (uint32_t i = gt; i < F.side_half; i += gstride) F.side_out[i] = fold_side(F, i);
}

template <bool FOLD>
__global__ void __launch_bounds__(256) k_phase1_eval(PqxArgs a, int mode, uint32_t total, uint32_t proof_len,
                                                     uint32_t cons_len, uint32_t instance_len,
                                                     const Fq* __restrict__ Ap, const Fq* __restrict__ Aq,
                                                     const Fq* __restrict__ Ax, Fq* __restrict__ B, Fq* __restrict__ C,
                                                     Fq* __restrict__ D, Fq* __restrict__ partials,
                                                     unsigned* __restrict__ counter, uint32_t* __restrict__ mb,
                                                     uint32_t seq, FoldArg F) {
  if (FOLD) fold_side_pass(F, blockIdx.x * 256 + threadIdx.x, gridDim.x * 256, total);
  const Fq omr = fq_sub(fq_one(), F.r);
  // the eq entries a point reads (folded on the fly when the pending fold binds that side table); no lambdas over
  // the by-value kernel arguments, which put them on the stack (scratch memory)
  const bool fq_side = FOLD && F.fmode == MODE_Q, fx_side = FOLD && F.fmode == MODE_X;
#define EQ_Q(i) (fq_side ? fold_side(F, (i)) : Aq[(i)])
#define EQ_X(i) (fx_side ? fold_side(F, (i)) : Ax[(i)])
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    int p = find_inst(a, t);
    const PqxInst& d = pinst(a, p);
    uint32_t loc = t - d.dom_off;
    uint32_t q = loc / d.sc_ni, x = loc % d.sc_ni;
    const Fq aq_lo = EQ_Q(q * d.step_q), ax_lo = EQ_X(x * d.step_x);
    Fq apq = fq_mul(Ap[p], aq_lo);
    Fq a_lo = fq_mul(apq, ax_lo);
    Fq a_hi;
    if (mode == MODE_P) a_hi = fq_mul(fq_mul(Ap[p + instance_len], aq_lo), ax_lo);
    else if (mode == MODE_Q) a_hi = fq_mul(fq_mul(Ap[p], EQ_Q(q * d.step_q + proof_len)), ax_lo);
    else a_hi = fq_mul(apq, EQ_X(x * d.step_x + cons_len));
    size_t base = pqx_off(d) + (size_t)q * d.anw * d.ani + x;
    bool zero_hi;
    size_t hi;
    if (mode == MODE_X) {
      zero_hi = d.ni == 1;
      hi = base + d.ni / 2;
    } else if (mode == MODE_Q) {
      zero_hi = d.np == 1;
      hi = base + (size_t)(d.np / 2) * d.anw * d.ani;
    } else {
      int ph = p + a.ninst / 2;
      zero_hi = ph >= a.zlen;
      hi = zero_hi ? 0 : pqx_off(pinst(a, ph)) + (size_t)q * pinst(a, ph).anw * pinst(a, ph).ani + x;
    }
    Fq b_lo, c_lo, d_lo, b_hi = fq_zero(), c_hi = fq_zero(), d_hi = fq_zero();
    if (FOLD) {
      const uint32_t fs = d.fstride;
      fold_pair_rw(B, base, hi, !zero_hi, fs, F.r, omr, b_lo, b_hi);
      fold_pair_rw(C, base, hi, !zero_hi, fs, F.r, omr, c_lo, c_hi);
      fold_pair_rw(D, base, hi, !zero_hi, fs, F.r, omr, d_lo, d_hi);
    } else {
      b_lo = B[base];
      c_lo = C[base];
      d_lo = D[base];
      if (!zero_hi) {
        b_hi = B[hi];
        c_hi = C[hi];
        d_hi = D[hi];
      }
    }
    // comb(A, B, C, D) = A * (B*C - D) at X = 0, 2, 3
    e0 = fq_add(e0, fq_mul(a_lo, fq_sub(fq_mul(b_lo, c_lo), d_lo)));
    Fq a2 = fq_sub(fq_dbl(a_hi), a_lo), b2 = fq_sub(fq_dbl(b_hi), b_lo);
    Fq c2 = fq_sub(fq_dbl(c_hi), c_lo), d2 = fq_sub(fq_dbl(d_hi), d_lo);
    e2 = fq_add(e2, fq_mul(a2, fq_sub(fq_mul(b2, c2), d2)));
    Fq a3 = fq_sub(fq_add(a2, a_hi), a_lo), b3 = fq_sub(fq_add(b2, b_hi), b_lo);
    Fq c3 = fq_sub(fq_add(c2, c_hi), c_lo), d3 = fq_sub(fq_add(d2, d_hi), d_lo);
    e3 = fq_add(e3, fq_mul(a3, fq_sub(fq_mul(b3, c3), d3)));
  }
#undef EQ_Q
#undef EQ_X
  grid_reduce3(e0, e2, e3, partials, counter, mb, seq);
}

// x-mode rounds whose rows (one (p, q) pair: sc_ni consecutive domain points) hold >= 64 J points: a wave takes 64 J
// consecutive points of one row (lane l: points l, l + 64, .., coalesced), and since every point of a row shares the
// eq factor Ap[p] Aq[q] -- e_X = sum_(p,q) Ap Aq sum_x Ax(X) (B C - D)(X) -- a lane sums Ax(X) (B C - D)(X) over its J
// points and multiplies by the row factor once: 6 Fq products per point (+ the folds) instead of 9, the row factor's
// 1 + 3 per J points. The same field sums as k_phase1_eval's, so the same (e0, e2, e3).
template <bool FOLD, int J>
__global__ void __launch_bounds__(256) k_phase1_eval_x(PqxArgs a, uint32_t total, uint32_t cons_len,
                                                       const Fq* __restrict__ Ap, const Fq* __restrict__ Aq,
                                                       const Fq* __restrict__ Ax, Fq* __restrict__ B,
                                                       Fq* __restrict__ C, Fq* __restrict__ D, Fq* __restrict__ partials,
                                                       unsigned* __restrict__ counter, uint32_t* __restrict__ mb,
                                                       uint32_t seq, FoldArg F) {
  const uint32_t nchunk = total / (64u * J);
  if (FOLD) fold_side_pass(F, blockIdx.x * 256 + threadIdx.x, gridDim.x * 256, nchunk * 64u);
  const Fq omr = fq_sub(fq_one(), F.r);
  const bool fx_side = FOLD && F.fmode == MODE_X;
  const uint32_t lane = threadIdx.x & 63;
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunk; c += gridDim.x * 4) {  // uniform per wave
    const uint32_t t0 = c * 64u * J;
    const int p = find_inst(a, t0);
    const PqxInst& d = pinst(a, p);
    const uint32_t loc0 = t0 - d.dom_off, q = loc0 / d.sc_ni, x0 = loc0 % d.sc_ni;
    const Fq apq = fq_mul(Ap[p], Aq[q * d.step_q]);
    const size_t row = pqx_off(d) + (size_t)q * d.anw * d.ani;
    const bool zero_hi = d.ni == 1;
    Fq i0 = fq_zero(), i2 = fq_zero(), i3 = fq_zero();
#pragma unroll 1
    for (int j = 0; j < J; j++) {
      const uint32_t x = x0 + lane + 64u * j, ix = x * d.step_x;
      const Fq ax_lo = fx_side ? fold_side(F, ix) : Ax[ix];
      const Fq ax_hi = fx_side ? fold_side(F, ix + cons_len) : Ax[ix + cons_len];
      const size_t base = row + x, hi = base + d.ni / 2;
      Fq b_lo, c_lo, d_lo, b_hi = fq_zero(), c_hi = fq_zero(), d_hi = fq_zero();
      if (FOLD) {
        const uint32_t fs = d.fstride;
        fold_pair_rw(B, base, hi, !zero_hi, fs, F.r, omr, b_lo, b_hi);
        fold_pair_rw(C, base, hi, !zero_hi, fs, F.r, omr, c_lo, c_hi);
        fold_pair_rw(D, base, hi, !zero_hi, fs, F.r, omr, d_lo, d_hi);
      } else {
        b_lo = B[base];
        c_lo = C[base];
        d_lo = D[base];
        if (!zero_hi) {
          b_hi = B[hi];
          c_hi = C[hi];
          d_hi = D[hi];
        }
      }
      i0 = fq_add(i0, fq_mul(ax_lo, fq_sub(fq_mul(b_lo, c_lo), d_lo)));
      const Fq a2 = fq_sub(fq_dbl(ax_hi), ax_lo), b2 = fq_sub(fq_dbl(b_hi), b_lo);
      const Fq c2 = fq_sub(fq_dbl(c_hi), c_lo), d2 = fq_sub(fq_dbl(d_hi), d_lo);
      i2 = fq_add(i2, fq_mul(a2, fq_sub(fq_mul(b2, c2), d2)));
      const Fq a3 = fq_sub(fq_add(a2, ax_hi), ax_lo), b3 = fq_sub(fq_add(b2, b_hi), b_lo);
      const Fq c3 = fq_sub(fq_add(c2, c_hi), c_lo), d3 = fq_sub(fq_add(d2, d_hi), d_lo);
      i3 = fq_add(i3, fq_mul(a3, fq_sub(fq_mul(b3, c3), d3)));
    }
    e0 = fq_add(e0, fq_mul(apq, i0));
    e2 = fq_add(e2, fq_mul(apq, i2));
    e3 = fq_add(e3, fq_mul(apq, i3));
  }
  grid_reduce3(e0, e2, e3, partials, counter, mb, seq);
}

// ---- quad forms of the round evaluations (small rounds: latency-bound) ------------------------------------------
// A round whose domain leaves the chip mostly idle is bound by the dependent chain of one thread's products (about
// ten Fq products per point in phase 1, each ~0.6 us on one wave). Here a quad (4 lanes) takes each point and its
// lanes compute the point's independent products side by side (operands selected per lane, exchanged by DPP quad
// broadcasts): three levels of products in phase 1, two in phase 2. Lane 0 accumulates e0, lane 1 e2, lane 2 e3.
template <int K>
__device__ __forceinline__ Fq fq_qb(const Fq& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], K * 0x55, 0xf, 0xf, false);
  return r;
}
// word-wise selects: a select of whole structs became a runtime-indexed stack array (scratch memory)
__device__ __forceinline__ Fq fq_pick(int q, const Fq& a0, const Fq& a1, const Fq& a2, const Fq& a3) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = q == 0 ? a0.l[i] : (q == 1 ? a1.l[i] : (q == 2 ? a2.l[i] : a3.l[i]));
  return r;
}

// FOLD: a level 0 first applies the pending fold, lane 0 to B's lo and hi entries, lane 1 to C's, lane 2 to D's and
// lane 3 to the two entries of the folded eq side table the point reads; the values go round the quad by DPP.
template <bool FOLD>
__global__ void __launch_bounds__(256) k_phase1_eval_q(PqxArgs a, int mode, uint32_t total, uint32_t proof_len,
                                                       uint32_t cons_len, uint32_t instance_len,
                                                       const Fq* __restrict__ Ap, const Fq* __restrict__ Aq,
                                                       const Fq* __restrict__ Ax, Fq* __restrict__ B,
                                                       Fq* __restrict__ C, Fq* __restrict__ D,
                                                       Fq* __restrict__ partials, unsigned* __restrict__ counter,
                                                       uint32_t* __restrict__ mb, uint32_t seq, FoldArg F) {
  const int q = threadIdx.x & 3;
  if (FOLD) fold_side_pass(F, blockIdx.x * 256 + threadIdx.x, gridDim.x * 256, total > (1u << 30) ? ~0u : 4 * total);
  const Fq omr = fq_sub(fq_one(), F.r);
  Fq acc = fq_zero();
  for (uint32_t t = blockIdx.x * 64 + (threadIdx.x >> 2); t < total; t += gridDim.x * 64) {  // uniform per quad
    int p = find_inst(a, t);
    const PqxInst& d = pinst(a, p);
    uint32_t loc = t - d.dom_off;
    uint32_t qq = loc / d.sc_ni, x = loc % d.sc_ni;
    size_t base = pqx_off(d) + (size_t)qq * d.anw * d.ani + x;
    bool zero_hi;
    size_t hi;
    if (mode == MODE_X) {
      zero_hi = d.ni == 1;
      hi = base + d.ni / 2;
    } else if (mode == MODE_Q) {
      zero_hi = d.np == 1;
      hi = base + (size_t)(d.np / 2) * d.anw * d.ani;
    } else {
      int ph = p + a.ninst / 2;
      zero_hi = ph >= a.zlen;
      hi = zero_hi ? 0 : pqx_off(pinst(a, ph)) + (size_t)qq * pinst(a, ph).anw * pinst(a, ph).ani + x;
    }
    const uint32_t iq = qq * d.step_q, ix = x * d.step_x;
    Fq b_lo, c_lo, d_lo, b_hi, c_hi, d_hi;
    // the eq entries levels 1 and 2 read, loaded up front (those of a side table the pending fold binds come
    // folded from lane 3 below)
    Fq aq_lo, aq_hi, ax_lo, ax_hi;
    const bool side_q = FOLD && F.fmode == MODE_Q, side_x = FOLD && F.fmode == MODE_X;
    if (!side_q) {
      aq_lo = Aq[iq];
      aq_hi = mode == MODE_Q ? Aq[iq + proof_len] : aq_lo;
    }
    if (!side_x) {
      ax_lo = Ax[ix];
      ax_hi = mode == MODE_X ? Ax[ix + cons_len] : ax_lo;
    }
    const Fq ap_lo = Ap[p], ap_hi = mode == MODE_P ? Ap[p + instance_len] : ap_lo;
    if (FOLD) {
      Fq f_lo, f_hi = fq_zero();
      if (q < 3) {
        Fq* T = q == 0 ? B : (q == 1 ? C : D);
        fold_pair_rw(T, base, hi, !zero_hi, d.fstride, F.r, omr, f_lo, f_hi);
      } else {
        const bool sx = F.fmode == MODE_X;
        f_lo = fold_side(F, sx ? ix : iq);
        if (sx ? mode == MODE_X : mode == MODE_Q) f_hi = fold_side(F, sx ? ix + cons_len : iq + proof_len);
      }
      b_lo = fq_qb<0>(f_lo);
      b_hi = fq_qb<0>(f_hi);
      c_lo = fq_qb<1>(f_lo);
      c_hi = fq_qb<1>(f_hi);
      d_lo = fq_qb<2>(f_lo);
      d_hi = fq_qb<2>(f_hi);
      const Fq s_lo = fq_qb<3>(f_lo), s_hi = fq_qb<3>(f_hi);
      if (side_x) {
        ax_lo = s_lo;
        ax_hi = s_hi;
      } else {
        aq_lo = s_lo;
        aq_hi = s_hi;
      }
    } else {
      b_lo = B[base];
      c_lo = C[base];
      d_lo = D[base];
      b_hi = zero_hi ? fq_zero() : B[hi];
      c_hi = zero_hi ? fq_zero() : C[hi];
      d_hi = zero_hi ? fq_zero() : D[hi];
    }
    const Fq b2 = fq_sub(fq_dbl(b_hi), b_lo), c2 = fq_sub(fq_dbl(c_hi), c_lo), d2 = fq_sub(fq_dbl(d_hi), d_lo);
    const Fq b3 = fq_sub(fq_add(b2, b_hi), b_lo), c3 = fq_sub(fq_add(c2, c_hi), c_lo), d3 = fq_sub(fq_add(d2, d_hi), d_lo);
    // level 1: lane 0 Ap Aq (lo), lane 1 the hi eq prefix (modes P / Q) or b3 c3 (mode X), lane 2 b c, lane 3 b2 c2
    Fq u1, v1;
    if (q == 0) {
      u1 = ap_lo;
      v1 = aq_lo;
    } else if (q == 1) {
      if (mode == MODE_X) {
        u1 = b3;
        v1 = c3;
      } else {
        u1 = ap_hi;
        v1 = mode == MODE_P ? aq_lo : aq_hi;
      }
    } else {
      u1 = q == 2 ? b_lo : b2;
      v1 = q == 2 ? c_lo : c2;
    }
    const Fq r1 = fq_mul(u1, v1);
    const Fq apq = fq_qb<0>(r1), r1_1 = fq_qb<1>(r1), bc_lo = fq_qb<2>(r1), bc2 = fq_qb<3>(r1);
    // level 2: lane 0 a_lo = apq Ax[x], lane 1 a_hi, lane 2 b3 c3 (modes P / Q)
    const Fq u2 = q == 1 && mode != MODE_X ? r1_1 : (q == 2 ? b3 : apq);
    const Fq v2 = q == 2 ? c3 : (q == 1 && mode == MODE_X ? ax_hi : ax_lo);
    const Fq r2 = fq_mul(u2, v2);
    const Fq a_lo = fq_qb<0>(r2), a_hi = fq_qb<1>(r2);
    const Fq bc3 = mode == MODE_X ? r1_1 : fq_qb<2>(r2);
    // level 3: lane 0 e0 = a (b c - d) at X = 0, lane 1 at X = 2, lane 2 at X = 3
    const Fq a2 = fq_sub(fq_dbl(a_hi), a_lo), a3 = fq_sub(fq_add(a2, a_hi), a_lo);
    const Fq u3 = fq_pick(q, a_lo, a2, a3, a_lo);
    const Fq v3 = fq_pick(q, fq_sub(bc_lo, d_lo), fq_sub(bc2, d2), fq_sub(bc3, d3), fq_sub(bc_lo, d_lo));
    acc = fq_add(acc, fq_mul(u3, v3));
  }
  quad_grid_post<256>(acc, partials, counter, mb, seq);
}

// ---------------------------------------------------------------- phase 2 round evaluation
// domain: p < Pd, w < W, y < sc_ni[p] ; B = ABC table (instance pi = single ? 0 : p), C = Z table
__device__ __forceinline__ Fq pqx_get(const PqxArgs& a, const Fq* T, int p, uint32_t w, uint32_t y) {
  if (p >= a.zlen) return fq_zero();
  const PqxInst& d = pinst(a, p);
  if (w >= d.anw || y >= d.ani) return fq_zero();
  return T[pqx_off(d) + (size_t)w * d.ani + y];
}
__device__ __forceinline__ Fq pqx_get_high(const PqxArgs& a, const Fq* T, int p, uint32_t w, uint32_t y, int mode) {
  const PqxInst& d = pinst(a, p);
  if (mode == MODE_X) return d.ni == 1 ? fq_zero() : T[pqx_off(d) + (size_t)w * d.ani + y + d.ni / 2];
  if (mode == MODE_W) {
    uint32_t wh = w + a.nws / 2;
    return wh < d.anw ? T[pqx_off(d) + (size_t)wh * d.ani + y] : fq_zero();
  }
  int ph = p + a.ninst / 2;
  return ph < a.zlen ? T[pqx_off(pinst(a, ph)) + (size_t)w * pinst(a, ph).ani + y] : fq_zero();
}

// Fused fold + eval (FOLD), as in phase 1: the previous round's bound_poly_var_{x,w} of ABC and Z is applied to the
// entries a point reads. Z entries (and ABC entries when every instance has its own) are read by one point each and
// folded in place; one ABC shared by every instance is read by all of them, so it is folded into its ping-pong buffer,
// written by instance 0's points (which read every live ABC entry).
__device__ __forceinline__ long pq_lo(const PqxArgs& a, int p, uint32_t w, uint32_t y) {
  if (p >= a.zlen) return -1;
  const PqxInst& d = pinst(a, p);
  if (w >= d.anw || y >= d.ani) return -1;
  return (long)(pqx_off(d) + (size_t)w * d.ani + y);
}
// the hi entry of modes X and W (pqx_get_high), with its witness-section coordinate
__device__ __forceinline__ long pq_hi(const PqxArgs& a, int p, uint32_t w, uint32_t y, int mode, uint32_t* wc) {
  const PqxInst& d = pinst(a, p);
  if (mode == MODE_X) {
    *wc = w;
    return d.ni == 1 ? -1 : (long)(pqx_off(d) + (size_t)w * d.ani + y + d.ni / 2);
  }
  const uint32_t wh = w + a.nws / 2;
  *wc = wh;
  return wh < d.anw ? (long)(pqx_off(d) + (size_t)wh * d.ani + y) : -1;
}
__device__ __forceinline__ Fq fold2_at(const Fq* T, long s, const PqxInst& d, uint32_t wc, const Fold2Arg& F,
                                       const Fq& omr) {
  const Fq lo = T[s];
  const bool pair = d.fstride && (F.fmode != MODE_W || wc + F.fw < d.anw);
  return pair ? fq_add(lo, fq_mul(F.r, fq_sub(T[s + d.fstride], lo))) : fq_mul(omr, lo);
}
// this point's ABC (tb = 0) or Z (tb = 1) lo and hi entries, folded and written back
__device__ __forceinline__ void fold2_pair(const PqxArgs& a, Fq* T, int p, uint32_t w, uint32_t y, int mode,
                                           const Fold2Arg& F, const Fq& omr, Fq* out, bool write, Fq& lo, Fq& hi) {
  const long sl = pq_lo(a, p, w, y);
  uint32_t wc;
  const long sh = pq_hi(a, p, w, y, mode, &wc);
  lo = fq_zero();
  hi = fq_zero();
  // both folds before either write-back (a store in between would order the hi loads behind the lo product)
  if (sl >= 0) lo = fold2_at(T, sl, pinst(a, p), w, F, omr);
  if (sh >= 0) hi = fold2_at(T, sh, pinst(a, p), wc, F, omr);
  if (write && sl >= 0) out[sl] = lo;
  if (write && sh >= 0) out[sh] = hi;
}

template <bool FOLD>
__global__ void __launch_bounds__(256) k_phase2_eval(PqxArgs ab, PqxArgs zz, int mode, uint32_t total, int W,
                                                     bool single, uint32_t instance_len, const Fq* __restrict__ eq,
                                                     Fq* __restrict__ B, Fq* __restrict__ C,
                                                     Fq* __restrict__ partials, unsigned* __restrict__ counter,
                                                     uint32_t* __restrict__ mb, uint32_t seq, Fold2Arg F) {
  const Fq omr = fq_sub(fq_one(), F.r);
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    int p = find_inst(zz, t);
    uint32_t loc = t - pinst(zz, p).dom_off;
    uint32_t ny = pinst(zz, p).sc_ni;
    uint32_t w = loc / ny, y = loc % ny;
    (void)W;
    int pi = single ? 0 : p;
    Fq a_lo = eq[p];
    Fq a_hi = mode == MODE_P ? eq[p + instance_len] : a_lo;
    Fq b_lo, b_hi, c_lo, c_hi;
    if (FOLD) {
      fold2_pair(ab, B, pi, w, y, mode, F, omr, F.b_out, !F.ping || p == 0, b_lo, b_hi);
      fold2_pair(zz, C, p, w, y, mode, F, omr, C, true, c_lo, c_hi);
    } else {
      b_lo = pqx_get(ab, B, pi, w, y);
      c_lo = pqx_get(zz, C, p, w, y);
      b_hi = pqx_get_high(ab, B, pi, w, y, mode);
      c_hi = pqx_get_high(zz, C, p, w, y, mode);
    }
    e0 = fq_add(e0, fq_mul(fq_mul(a_lo, b_lo), c_lo));
    Fq a2 = fq_sub(fq_dbl(a_hi), a_lo), b2 = fq_sub(fq_dbl(b_hi), b_lo), c2 = fq_sub(fq_dbl(c_hi), c_lo);
    e2 = fq_add(e2, fq_mul(fq_mul(a2, b2), c2));
    Fq a3 = fq_sub(fq_add(a2, a_hi), a_lo), b3 = fq_sub(fq_add(b2, b_hi), b_lo), c3 = fq_sub(fq_add(c2, c_hi), c_lo);
    e3 = fq_add(e3, fq_mul(fq_mul(a3, b3), c3));
  }
  grid_reduce3(e0, e2, e3, partials, counter, mb, seq);
}

// quad form of k_phase2_eval: lane 0 / 1 / 2 forms the point's product at X = 0 / 2 / 3 as (a b) c, two levels (FOLD:
// a level 0 first, lane 0 folding the ABC entries and lane 1 the Z entries, exchanged by DPP)
template <bool FOLD>
__global__ void __launch_bounds__(256) k_phase2_eval_q(PqxArgs ab, PqxArgs zz, int mode, uint32_t total,
                                                       bool single, uint32_t instance_len, const Fq* __restrict__ eq,
                                                       Fq* __restrict__ B, Fq* __restrict__ C,
                                                       Fq* __restrict__ partials, unsigned* __restrict__ counter,
                                                       uint32_t* __restrict__ mb, uint32_t seq, Fold2Arg F) {
  const int q = threadIdx.x & 3;
  const Fq omr = fq_sub(fq_one(), F.r);
  Fq acc = fq_zero();
  for (uint32_t t = blockIdx.x * 64 + (threadIdx.x >> 2); t < total; t += gridDim.x * 64) {  // uniform per quad
    int p = find_inst(zz, t);
    uint32_t loc = t - pinst(zz, p).dom_off;
    uint32_t ny = pinst(zz, p).sc_ni;
    uint32_t w = loc / ny, y = loc % ny;
    int pi = single ? 0 : p;
    const Fq a_lo = eq[p];
    const Fq a_hi = mode == MODE_P ? eq[p + instance_len] : a_lo;
    Fq b_lo, b_hi, c_lo, c_hi;
    if (FOLD) {
      Fq f_lo = fq_zero(), f_hi = fq_zero();
      if (q == 0) fold2_pair(ab, B, pi, w, y, mode, F, omr, F.b_out, !F.ping || p == 0, f_lo, f_hi);
      else if (q == 1) fold2_pair(zz, C, p, w, y, mode, F, omr, C, true, f_lo, f_hi);
      b_lo = fq_qb<0>(f_lo);
      b_hi = fq_qb<0>(f_hi);
      c_lo = fq_qb<1>(f_lo);
      c_hi = fq_qb<1>(f_hi);
    } else {
      b_lo = pqx_get(ab, B, pi, w, y);
      c_lo = pqx_get(zz, C, p, w, y);
      b_hi = pqx_get_high(ab, B, pi, w, y, mode);
      c_hi = pqx_get_high(zz, C, p, w, y, mode);
    }
    const Fq a2 = fq_sub(fq_dbl(a_hi), a_lo), b2 = fq_sub(fq_dbl(b_hi), b_lo), c2 = fq_sub(fq_dbl(c_hi), c_lo);
    const Fq a3 = fq_sub(fq_add(a2, a_hi), a_lo), b3 = fq_sub(fq_add(b2, b_hi), b_lo), c3 = fq_sub(fq_add(c2, c_hi), c_lo);
    const Fq ab_ = fq_mul(fq_pick(q, a_lo, a2, a3, a_lo), fq_pick(q, b_lo, b2, b3, b_lo));
    acc = fq_add(acc, fq_mul(ab_, fq_pick(q, c_lo, c2, c3, c_lo)));
  }
  quad_grid_post<256>(acc, partials, counter, mb, seq);
}

// ---------------------------------------------------------------- Pqx folds (custom_dense_mlpoly.rs:205-289)
// domain per instance: np_cur[p] (rows to fold) x nw_cur x n_cols, flattened with dom_off.
// sc_np = rows, sc_ni = columns written, step_q = nw (sections visited)
// entry t of a Pqx table's fold (bound_poly_var_{p,q,w,x}) for up to three tables of one shape
__device__ __forceinline__ void pqx_fold_at(const PqxArgs& a, int mode, uint32_t t, Fq r, Fq* __restrict__ T0,
                                            Fq* __restrict__ T1, Fq* __restrict__ T2) {
  int p = find_inst(a, t);
  const PqxInst& d = pinst(a, p);
  uint32_t loc = t - d.dom_off;
  uint32_t ncol = d.sc_ni, nw = d.step_q;
  uint32_t x = loc % ncol;
  uint32_t rest = loc / ncol;
  uint32_t w = rest % nw, q = rest / nw;
  size_t base = pqx_off(d) + ((size_t)q * d.anw + w) * d.ani + x;
  size_t hi;
  bool scale = false, zero_hi = false;
  if (mode == MODE_X) {
    if (d.ni == 1) scale = true;
    hi = base + d.ni / 2;
  } else if (mode == MODE_Q) {
    if (d.np == 1) scale = true;
    hi = base + (size_t)(d.np / 2) * d.anw * d.ani;
  } else if (mode == MODE_W) {
    uint32_t wh = w + a.nws;  // a.nws already halved by the host
    zero_hi = wh >= d.anw;
    hi = zero_hi ? 0 : pqx_off(d) + ((size_t)q * d.anw + wh) * d.ani + x;
  } else {
    int ph = p + a.ninst;  // a.ninst already halved by the host
    zero_hi = ph >= a.zlen;
    hi = zero_hi ? 0 : pqx_off(pinst(a, ph)) + ((size_t)q * pinst(a, ph).anw + w) * pinst(a, ph).ani + x;
  }
  Fq* Ts[3] = {T0, T1, T2};
  Fq omr = fq_sub(fq_one(), r);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    Fq* T = Ts[k];
    if (!T) continue;
    Fq lo = T[base];
    if (scale) {
      T[base] = fq_mul(omr, lo);
    } else {
      Fq h = zero_hi ? fq_zero() : T[hi];
      T[base] = fq_add(lo, fq_mul(r, fq_sub(h, lo)));
    }
  }
}


__global__ void k_pqx_fold(PqxArgs a, int mode, uint32_t total, Fq r, Fq* __restrict__ T0, Fq* __restrict__ T1,
                           Fq* __restrict__ T2, Fq* __restrict__ side, uint32_t side_half) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < side_half) {  // the side vector's bound_poly_var_top (k_fold_top)
    const Fq lo = side[t];
    side[t] = fq_add(lo, fq_mul(r, fq_sub(side[t + side_half], lo)));
  }
  if (t < total) pqx_fold_at(a, mode, t, r, T0, T1, T2);
}

// two tables of different shapes bound by the same r in one launch (phase 2: ABC and Z)
__global__ void k_pqx_fold2(PqxArgs a, uint32_t total_a, Fq* __restrict__ A, PqxArgs b, uint32_t total_b,
                            Fq* __restrict__ B, int mode, Fq r) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < total_a) pqx_fold_at(a, mode, t, r, A, nullptr, nullptr);
  else if (t - total_a < total_b) pqx_fold_at(b, mode, t - total_a, r, B, nullptr, nullptr);
}

// Every q-mode fold of DensePolynomialPqx::bound_poly_vars_rq (custom_dense_mlpoly.rs, phase 2's Z prep; round j binds
// the top live row bit of each instance with r_j, or scales a one-row instance by 1 - r_j) in one pass: an instance of
// np = 2^k rows ends as out(w, x) = sum_s W(s) T[s][w][x] with W(s) = prod_{j < k} (bit k-1-j of s ? r_j : 1 - r_j)
// prod_{j >= k} (1 - r_j) = E[s << (nq - k)], E = eq(r_0 .. r_{nq-1}) (most significant index bit <-> r_0). The same field
// element as nq folds (exact arithmetic), one read of the table instead of nq read-write passes. Workgroup: 256 / G
// outputs (consecutive x) x G row groups, G chosen by the host so that few outputs still fill the chip (a 2^20 SNARK's
// block Z has 2048 outputs of 512 rows); the G partial sums of an output meet in an LDS tree and the sum is written to
// row 0 in place (only this workgroup reads that output's rows). Domain: per instance nw x cols outputs rounded up to
// 256 / G.
template <int G>
__global__ void __launch_bounds__(256) k_pqx_bound_q(PqxArgs a, const Fq* __restrict__ E, int nq, Fq* __restrict__ T) {
  constexpr int O = 256 / G;
  __shared__ uint32_t sh[8][256];
  const uint32_t o0 = blockIdx.x * O;
  const int p = find_inst(a, o0);
  const PqxInst& d = pinst(a, p);
  const uint32_t lo = threadIdx.x % O, g = threadIdx.x / O;
  const uint32_t o = o0 - d.dom_off + lo, cols = d.sc_ni, np = d.np;
  const bool live = o < d.step_q * cols;
  const uint32_t w = live ? o / cols : 0, x = live ? o % cols : 0;
  int lgn = 0;
  while ((1u << lgn) < np) lgn++;
  const int se = nq - lgn;
  const size_t base = pqx_off(d) + (size_t)w * d.ani + x, row = (size_t)d.anw * d.ani;
  Fq acc = fq_zero();
  if (live) {
    uint32_t s = g;
    for (; s + 3 * G < np; s += 4 * G) {  // four rows' loads in flight per lane
      const Fq t0 = T[base + s * row], t1 = T[base + (s + G) * row], t2 = T[base + (s + 2 * G) * row],
               t3 = T[base + (s + 3 * G) * row];
      const Fq e0 = E[(size_t)s << se], e1 = E[(size_t)(s + G) << se], e2 = E[(size_t)(s + 2 * G) << se],
               e3 = E[(size_t)(s + 3 * G) << se];
      acc = fq_add(acc, fq_add(fq_add(fq_mul(e0, t0), fq_mul(e1, t1)), fq_add(fq_mul(e2, t2), fq_mul(e3, t3))));
    }
    for (; s < np; s += G) acc = fq_add(acc, fq_mul(E[(size_t)s << se], T[base + s * row]));
  }
#pragma unroll
  for (int c = 0; c < 8; c++) sh[c][threadIdx.x] = acc.l[c];
  __syncthreads();
#pragma unroll
  for (int h = G / 2; h >= 1; h >>= 1) {
    if ((int)g < h) {
      Fq v;
#pragma unroll
      for (int c = 0; c < 8; c++) v.l[c] = sh[c][(g + h) * O + lo];
      acc = fq_add(acc, v);
#pragma unroll
      for (int c = 0; c < 8; c++) sh[c][threadIdx.x] = acc.l[c];
    }
    __syncthreads();
  }
  if (g == 0 && live) T[base] = acc;
}

// ---------------------------------------------------------------- plain cubic (product trees), A*B*C
__global__ void __launch_bounds__(256) k_cubic_eval(const Fq* __restrict__ A, const Fq* __restrict__ B,
                                                    const Fq* __restrict__ C, uint32_t len, Fq* __restrict__ partials,
                                                    unsigned* __restrict__ counter, uint32_t* __restrict__ mb, uint32_t seq) {
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < len; i += gridDim.x * 256) {
    Fq al = A[i], ah = A[i + len], bl = B[i], bh = B[i + len], cl = C[i], ch = C[i + len];
    e0 = fq_add(e0, fq_mul(fq_mul(al, bl), cl));
    Fq a2 = fq_sub(fq_dbl(ah), al), b2 = fq_sub(fq_dbl(bh), bl), c2 = fq_sub(fq_dbl(ch), cl);
    e2 = fq_add(e2, fq_mul(fq_mul(a2, b2), c2));
    Fq a3 = fq_sub(fq_add(a2, ah), al), b3 = fq_sub(fq_add(b2, bh), bl), c3 = fq_sub(fq_add(c2, ch), cl);
    e3 = fq_add(e3, fq_mul(fq_mul(a3, b3), c3));
  }
  grid_reduce3(e0, e2, e3, partials, counter, mb, seq);
}


// ---- phase 1, two rounds per launch (round 6; SPG_P1_PAIR=0 keeps one round per launch) -------------------------------
// The latency-bound rounds of a ZK sumcheck are host round trips (launch, dispatch, mailbox) around a few us of work.
// As the SPARK layer pairs (layer.hpp, k_layer_pair): with every factor of round j's summand F = A (B C - D) multilinear
// in round j's variable t and round j + 1's variable s, round j's evaluation at X is sum F(X, 0) + F(X, 1) and round
// j + 1's at Y is the cubic t -> sum F(t, Y) at t = r_j, so one launch posts F at 15 points of the 4 x 4 grid and the
// host forms round j + 1's (e0, e2, e3) by Lagrange interpolation at r_j -- between the two rounds' commitments and
// sigma proofs, with no device round trip. Pairs run inside one mode (x: bound_poly_x, q: bound_poly_q) where every
// instance's size in that mode is >= 4, so neither round meets the ragged cases (a size-1 dimension's (1 - r) fold,
// a missing hi entry). Element = one point of round j + 1's domain: x mode (p, q, x' < N/4), q mode (p, q' < N/4, x),
// N = the instance's live size in the mode; its 2 x 2 cube is T[k + {0, N/4, N/2, 3N/4} u] (order 00, 01 (s), 10 (t),
// 11; u = 1 in x mode, the row stride anw ani in q mode) and the eq table E of the mode (Ax / Aq) at ie + {0, c/2, c,
// 3c/2} (c: round j's half length), times the other factors Ap[p] Aq[iq] (x mode) or Ap[p] Ax[ix] (q mode).
// Pending folds (nf), applied to what the launch reads, folded entries written back in place:
//   nf = 1, the previous single round's (FoldPlan: per-instance partner stride, 0 = the (1 - r) case; its side table
//     fmode folded on the fly and written to side_out by a grid-stride pass), as k_phase1_eval<true>;
//   nf = 2, the previous pair's (same mode): W = a + r1 (c - a) + r2 (b - a) + r1 r2 (d - c - b + a) over
//     T[k + {0, 1, 2, 3} Q] (Q = the live size N u; r1 the previous pair's round-j challenge), the eq table likewise
//     over its live size.
// A run of pairs ends with k_phase1_fold2x (the last pair's two folds, one launch, no host wait) before the next
// single round. Lanes: 16 per element, as k_layer_pair: g < 12 corner g & 3 of B, C, D (g >> 2); g 12..15 corner
// g - 12 of E times the element's other eq factors; DPP row broadcasts; lane g < 15 forms point g's A (B C - D).
struct P1PairArgs {
  PqxArgs a;           // np / ni: live sizes at round j (N = ni in x mode, np in q mode); sc_np x sc_ni the element grid
  int mode;            // MODE_X or MODE_Q
  uint32_t total;      // elements
  uint32_t c;          // round j's half length of the mode's eq table (its live size is 2 c)
  int nf;              // pending folds: 0, 1 or 2
  Fq r1, r2, r12;      // nf 1: r1 (omr = 1 - r1); nf 2: r1, r2 and their product
  int fmode;           // nf >= 1: the table the pending fold binds (MODE_X: Ax, MODE_Q: Aq)
  const Fq* side_in;   // that table before the pending fold(s)
  Fq* side_out;        // its folded live entries (the other ping-pong buffer)
  uint32_t side_live;  // entries after the pending fold(s) (nf 1: the half; nf 2: a quarter of side_in's live size)
  const Fq* Ap;
  const Fq* Aq;        // the current tables (a pending fold's table is read through side_in)
  const Fq* Ax;
  Fq* B;
  Fq* C;
  Fq* D;
  Fq* partials;        // 16 per workgroup
  unsigned* counter;
  uint32_t* mb;
  uint32_t seq;
};
__device__ __forceinline__ Fq bilerp(const Fq& a, const Fq& b, const Fq& c, const Fq& d, const Fq& r1, const Fq& r2,
                                     const Fq& r12) {
  // a: (0, 0), b: (0, 1) (r2's variable), c: (1, 0) (r1's), d: (1, 1)
  const Fq t1 = fq_mul(r1, fq_sub(c, a)), t2 = fq_mul(r2, fq_sub(b, a)), t3 = fq_mul(r12, fq_add(fq_sub(d, c), fq_sub(a, b)));
  return fq_add(fq_add(a, t1), fq_add(t2, t3));
}
// entry i of the side table as the pending fold(s) leave it
__device__ __forceinline__ Fq p1_side_at(const P1PairArgs& A, uint32_t i) {
  const Fq* s = A.side_in;
  const uint32_t L = A.side_live;
  if (A.nf == 1) {
    const Fq lo = s[i];
    return fq_add(lo, fq_mul(A.r1, fq_sub(s[i + L], lo)));
  }
  return bilerp(s[i], s[i + L], s[i + 2 * L], s[i + 3 * L], A.r1, A.r2, A.r12);
}
template <int BS>
__global__ void __launch_bounds__(BS) k_phase1_pair(P1PairArgs A) {
  __shared__ bool last;
  const int t = threadIdx.x, g = t & 15;
  const uint32_t gt = blockIdx.x * BS + t, gstride = gridDim.x * BS;
  // the pending fold's side table: its folded live entries into side_out (idle lanes first, then grid-stride)
  if (A.nf > 0)
    for (uint32_t i = gt; i < A.side_live; i += gstride) A.side_out[i] = p1_side_at(A, i);
  const uint32_t u = gt >> 4;  // this row's element (rows past the end idle, contribute zero)
  const int pt = g < 4 ? g : (g < 8 ? g - 4 : (g < 12 ? g - 8 : (g == 12 ? 0 : (g == 13 ? 2 : 3))));
  const int ps = g < 4 ? 0 : (g < 8 ? 2 : (g < 12 ? 3 : 1));
  Fq e = fq_zero();
  if (u < A.total) {
    const int p = find_inst(A.a, u);
    const PqxInst& d = pinst(A.a, p);
    const uint32_t loc = u - d.dom_off;
    const uint32_t r = loc / d.sc_ni, col = loc % d.sc_ni;  // x mode: (q, x'); q mode: (q', x)
    const bool xm = A.mode == MODE_X;
    const size_t unit = xm ? 1 : (size_t)d.anw * d.ani;
    const uint32_t N = xm ? d.ni : d.np;
    const size_t base = pqx_off(d) + (size_t)r * d.anw * d.ani + col;
    const int m = g & 3;  // corner: 0 (0, 0), 1 (0, s), 2 (t, 0), 3 (t, s)
    const uint32_t cq = (m & 1 ? N / 4 : 0) + (m & 2 ? N / 2 : 0);
    const bool side_x = A.nf > 0 && A.fmode == MODE_X, side_q = A.nf > 0 && A.fmode == MODE_Q;
    Fq w = fq_zero();
    if (g < 12) {
      Fq* T = g < 4 ? A.B : (g < 8 ? A.C : A.D);
      const size_t k = base + (size_t)cq * unit;
      if (A.nf == 0) {
        w = T[k];
      } else if (A.nf == 1) {
        const uint32_t fs = d.fstride;
        const Fq lo = T[k];
        w = fs ? fq_add(lo, fq_mul(A.r1, fq_sub(T[k + fs], lo))) : fq_mul(fq_sub(fq_one(), A.r1), lo);
        T[k] = w;
      } else {
        const size_t Q = (size_t)N * unit;
        w = bilerp(T[k], T[k + Q], T[k + 2 * Q], T[k + 3 * Q], A.r1, A.r2, A.r12);
        T[k] = w;
      }
    } else {
      // E corner m of the mode's eq table times the element's other eq factors
      const uint32_t cm = (m & 1 ? A.c / 2 : 0) + (m & 2 ? A.c : 0);
      Fq ev, other;
      if (xm) {
        const uint32_t ie = col * d.step_x + cm, iq = r * d.step_q;
        ev = side_x ? p1_side_at(A, ie) : A.Ax[ie];
        other = fq_mul(A.Ap[p], side_q ? p1_side_at(A, iq) : A.Aq[iq]);
      } else {
        const uint32_t ie = r * d.step_q + cm, ix = col * d.step_x;
        ev = side_q ? p1_side_at(A, ie) : A.Aq[ie];
        other = fq_mul(A.Ap[p], side_x ? p1_side_at(A, ix) : A.Ax[ix]);
      }
      w = fq_mul(other, ev);
    }
    const Fq b00 = fq_rowbcast<0>(w), b01 = fq_rowbcast<1>(w), b10 = fq_rowbcast<2>(w), b11 = fq_rowbcast<3>(w);
    const Fq c00 = fq_rowbcast<4>(w), c01 = fq_rowbcast<5>(w), c10 = fq_rowbcast<6>(w), c11 = fq_rowbcast<7>(w);
    const Fq d00 = fq_rowbcast<8>(w), d01 = fq_rowbcast<9>(w), d10 = fq_rowbcast<10>(w), d11 = fq_rowbcast<11>(w);
    const Fq a00 = fq_rowbcast<12>(w), a01 = fq_rowbcast<13>(w), a10 = fq_rowbcast<14>(w), a11 = fq_rowbcast<15>(w);
    const Fq bv = cube_at(b00, b01, b10, b11, pt, ps), cv = cube_at(c00, c01, c10, c11, pt, ps),
             dv = cube_at(d00, d01, d10, d11, pt, ps), av = cube_at(a00, a01, a10, a11, pt, ps);
    e = g < 15 ? fq_mul(av, fq_sub(fq_mul(bv, cv), dv)) : fq_zero();
  }
  row_block_sum<BS>(e);
  if (gridDim.x == 1) {  // lanes 0..14 of wave 0 post the 15 point sums, then lane 0 the sequence number
    if (t < 15) {
      host_put(A.mb + 8 + 8 * t, e);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    __syncthreads();
    if (t == 0) __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  // several workgroups: partials by sc1 stores and a ticket (as k_layer_pair)
  if (t < 16) st_sc1(&A.partials[16 * blockIdx.x + t], e);
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(A.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  Fq sum = fq_zero();
  for (unsigned j = t >> 4; j < gridDim.x; j += BS / 16) sum = fq_add(sum, ld_sc1(&A.partials[16 * j + g]));
  row_block_sum<BS>(sum);
  if (t < 15) {
    host_put(A.mb + 8 + 8 * t, sum);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  __syncthreads();
  if (t == 0) {
    __hip_atomic_store(A.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// the last pair's two folds of B, C, D (every live entry, in place: T[k] from T[k + {0, 1, 2, 3} Q]) and of its eq
// table (side_in -> side_out), before the next single round
__global__ void __launch_bounds__(256) k_phase1_fold2x(P1PairArgs A) {
  const uint32_t gt = blockIdx.x * 256 + threadIdx.x, gstride = gridDim.x * 256;
  for (uint32_t i = gt; i < A.side_live; i += gstride) A.side_out[i] = p1_side_at(A, i);
  for (uint32_t u = gt; u < A.total; u += gstride) {
    const int p = find_inst(A.a, u);
    const PqxInst& d = pinst(A.a, p);
    const uint32_t loc = u - d.dom_off, r = loc / d.sc_ni, col = loc % d.sc_ni;
    const bool xm = A.mode == MODE_X;
    const size_t unit = xm ? 1 : (size_t)d.anw * d.ani;
    const size_t Q = (size_t)(xm ? d.ni : d.np) * unit;
    const size_t k = pqx_off(d) + (size_t)r * d.anw * d.ani + col;
    A.B[k] = bilerp(A.B[k], A.B[k + Q], A.B[k + 2 * Q], A.B[k + 3 * Q], A.r1, A.r2, A.r12);
    A.C[k] = bilerp(A.C[k], A.C[k + Q], A.C[k + 2 * Q], A.C[k + 3 * Q], A.r1, A.r2, A.r12);
    A.D[k] = bilerp(A.D[k], A.D[k + Q], A.D[k + 2 * Q], A.D[k + 3 * Q], A.r1, A.r2, A.r12);
  }
}

// ---- phase 2, two y rounds per launch (round 6; SPG_P2_PAIR=0 keeps one round per launch) ------------------------------
// The phase-1 pair argument on phase 2's y rounds (src/sumcheck.rs:881-941): the summand eq(p) ABC(p, w, y) Z(p, w, y)
// has eq(p) constant over the y rounds and ABC, Z multilinear in round j's and round j + 1's variables, so the launch
// posts F = eq ABC Z on the same 15 points of the 4 x 4 grid and the host interpolates round j + 1 at r_j. Element =
// (instance p, section row w < W, y' < N/4), N = the instance's live y size (the same in ABC and Z); corners at
// y' + {0, N/4, N/2, 3N/4}. ABC is per instance here (a shared ABC is read by every instance and folded by one: those
// proofs keep single rounds). nf = 2: the previous pair's two folds, bilinear over T[k + {0, 1, 2, 3} N], written
// back in place. Lanes as k_phase1_pair with its D factor zero and its A factor the constant eq(p).
struct P2PairArgs {
  PqxArgs ab, zz;  // zz: dom_off (element offset), sc_ni (N/4 elements per row); ni: N
  uint32_t total;
  int nf;
  Fq r1, r2, r12;
  const Fq* eq;
  Fq* B;      // ABC
  Fq* B_out;  // shared ABC (one instance serving all): its folded entries go here, written by instance 0's elements
  int shared;
  Fq* C;      // Z
  Fq* partials;
  unsigned* counter;
  uint32_t* mb;
  uint32_t seq;
};
static_assert(sizeof(P2PairArgs) <= 4096, "phase-2 pair arguments exceed the kernel-argument budget");
template <int BS>
__global__ void __launch_bounds__(BS) k_phase2_pair(P2PairArgs A) {
  __shared__ bool last;
  const int t = threadIdx.x, g = t & 15;
  const uint32_t u = (blockIdx.x * BS + t) >> 4;
  const int pt = g < 4 ? g : (g < 8 ? g - 4 : (g < 12 ? g - 8 : (g == 12 ? 0 : (g == 13 ? 2 : 3))));
  const int ps = g < 4 ? 0 : (g < 8 ? 2 : (g < 12 ? 3 : 1));
  Fq e = fq_zero();
  if (u < A.total) {
    const int p = find_inst(A.zz, u);
    const PqxInst& dz = pinst(A.zz, p);
    const uint32_t loc = u - dz.dom_off, w = loc / dz.sc_ni, y = loc % dz.sc_ni, N = dz.ni;
    const int m = g & 3;  // corner: 0 (0, 0), 1 (0, s), 2 (t, 0), 3 (t, s)
    Fq v = fq_zero();
    if (g < 8) {
      const PqxInst& d = g < 4 ? pinst(A.ab, A.shared ? 0 : p) : dz;
      Fq* T = g < 4 ? A.B : A.C;
      const size_t k = pqx_off(d) + (size_t)w * d.ani + y + (m & 1 ? N / 4 : 0) + (m & 2 ? N / 2 : 0);
      if (A.nf == 0) {
        v = T[k];
      } else {
        v = bilerp(T[k], T[k + N], T[k + 2 * (size_t)N], T[k + 3 * (size_t)N], A.r1, A.r2, A.r12);
        if (g >= 4 || !A.shared) T[k] = v;  // in place: every entry is this element's alone
        else if (p == 0) A.B_out[k] = v;    // the shared ABC is read by every instance: ping-pong
      }
    } else if (g >= 12) {
      v = A.eq[p];
    }
    const Fq b00 = fq_rowbcast<0>(v), b01 = fq_rowbcast<1>(v), b10 = fq_rowbcast<2>(v), b11 = fq_rowbcast<3>(v);
    const Fq c00 = fq_rowbcast<4>(v), c01 = fq_rowbcast<5>(v), c10 = fq_rowbcast<6>(v), c11 = fq_rowbcast<7>(v);
    const Fq a = fq_rowbcast<12>(v);
    const Fq bv = cube_at(b00, b01, b10, b11, pt, ps), cv = cube_at(c00, c01, c10, c11, pt, ps);
    e = g < 15 ? fq_mul(a, fq_mul(bv, cv)) : fq_zero();
  }
  row_block_sum<BS>(e);
  if (gridDim.x == 1) {  // lanes 0..14 of wave 0 post the 15 point sums, then lane 0 the sequence number
    if (t < 15) {
      host_put(A.mb + 8 + 8 * t, e);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    __syncthreads();
    if (t == 0) __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (t < 16) st_sc1(&A.partials[16 * blockIdx.x + t], e);
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(A.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  Fq sum = fq_zero();
  for (unsigned j = t >> 4; j < gridDim.x; j += BS / 16) sum = fq_add(sum, ld_sc1(&A.partials[16 * j + g]));
  row_block_sum<BS>(sum);
  if (t < 15) {
    host_put(A.mb + 8 + 8 * t, sum);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  __syncthreads();
  if (t == 0) {
    __hip_atomic_store(A.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// the last pair's two folds of ABC and Z (every live entry, in place: T[k] from T[k + {0, 1, 2, 3} N], N the live size
// after both folds)
__global__ void __launch_bounds__(256) k_phase2_fold2x(P2PairArgs A) {
  for (uint32_t u = blockIdx.x * 256 + threadIdx.x; u < A.total; u += gridDim.x * 256) {
    const int p = find_inst(A.zz, u);
    const PqxInst& dz = pinst(A.zz, p);
    const PqxInst& da = pinst(A.ab, A.shared ? 0 : p);
    const uint32_t loc = u - dz.dom_off, w = loc / dz.sc_ni, y = loc % dz.sc_ni;
    const size_t N = dz.ni;
    const size_t ka = pqx_off(da) + (size_t)w * da.ani + y, kz = pqx_off(dz) + (size_t)w * dz.ani + y;
    if (!A.shared || p == 0)
      (A.shared ? A.B_out : A.B)[ka] = bilerp(A.B[ka], A.B[ka + N], A.B[ka + 2 * N], A.B[ka + 3 * N], A.r1, A.r2, A.r12);
    A.C[kz] = bilerp(A.C[kz], A.C[kz + N], A.C[kz + 2 * N], A.C[kz + 3 * N], A.r1, A.r2, A.r12);
  }
}

// ---------------------------------------------------------------- host launchers
// round evaluations over at most this many domain points take the quad form (SPG_SC_QUAD_MAX; 0 = never): below it
// the chip is not full and a point's chain of products sets the time
static size_t sc_quad_max() {
  static const size_t m = getenv("SPG_SC_QUAD_MAX") ? (size_t)atol(getenv("SPG_SC_QUAD_MAX")) : ((size_t)1 << 16);
  return m;
}
// workgroups of a round's evaluation: one per 256 threads of work, at most SPG_SC_GRID (default 1024, <= kScGridMax:
// the partials buffer)
static int grid_for(uint32_t total) {
  static const int cap = getenv("SPG_SC_GRID") ? std::max(1, std::min(kScGridMax, atoi(getenv("SPG_SC_GRID")))) : 1024;
  int nb = (int)((total + 255) / 256);
  if (nb > cap) nb = cap;
  return nb < 1 ? 1 : nb;
}

// the round's three scalars arrive in the host mailbox (posted by the last block of the eval kernel);
// out3 == nullptr returns at once (collect them with eval_wait), so host work can overlap the round
int eval_reduce_finish(spg_ctx* ctx, Fq* out3) { return out3 ? eval_wait(ctx, out3) : 0; }
int eval_wait(spg_ctx* ctx, Fq* out3) { return mbox_wait(ctx, ctx->mbox_seq, out3, 3); }

int dev_eq_table(spg_ctx* ctx, const Fq* r, int ell, Fq* out, const KBlob* blob, void* blob_dst) {
  if (ell > 32) return set_err(ctx, SPG_E_ARG, "eq table: too many variables");
  if (blob && (blob->nwords < 0 || blob->nwords > KBlob::kWords || !blob_dst))
    return set_err(ctx, SPG_E_ARG, "eq table: bad blob");
  FqArg32 a;
  a.n = ell;
  for (int i = 0; i < ell; i++) a.v[i] = r[i];
  size_t n = (size_t)1 << ell;
  KScope ks(ctx, "eq_table", 32.0 * n);
  // the first launch carries the blob (an empty one when there is none: the kernel is the <false> form)
  static KBlob none{};
  const KBlob& bl = blob ? *blob : none;
  uint32_t* bd = (uint32_t*)blob_dst;
  // SPG_EQ_LDS=0 restores the one-lane-per-entry kernel (A/B switch)
  static const bool lds_on = !getenv("SPG_EQ_LDS") || atoi(getenv("SPG_EQ_LDS")) != 0;
  auto launch = [&](const FqArg32& ra, Fq* o, size_t cnt, bool with_blob) {
    const dim3 g((unsigned)((cnt + 255) / 256));
    if (lds_on) {
      if (with_blob)
        hipLaunchKernelGGL(k_eq_table_lds<true>, g, dim3(256), 0, ctx->stream, ra, o, cnt, bl, bd);
      else
        hipLaunchKernelGGL(k_eq_table_lds<false>, g, dim3(256), 0, ctx->stream, ra, o, cnt, none, nullptr);
    } else if (with_blob)
      hipLaunchKernelGGL(k_eq_table<true>, g, dim3(256), 0, ctx->stream, ra, o, cnt, bl, bd);
    else
      hipLaunchKernelGGL(k_eq_table<false>, g, dim3(256), 0, ctx->stream, ra, o, cnt, none, nullptr);
  };
  if (ell <= (lds_on ? 16 : 12)) {
    launch(a, out, n, blob != nullptr);
  } else {  // eq(r) = eq(r_hi) (x) eq(r_lo): two small tables, then one multiplication per entry
    const int hb = ell / 2, lb = ell - hb;
    Fq* t = (Fq*)ws_get(ctx, 16, (((size_t)1 << hb) + ((size_t)1 << lb)) * sizeof(Fq) + 64);
    if (!t) return set_err(ctx, SPG_E_NOMEM, "eq table");
    Fq* hi = t;
    Fq* lo = t + ((size_t)1 << hb);
    FqArg32 ah, al;
    ah.n = hb;
    al.n = lb;
    for (int i = 0; i < hb; i++) ah.v[i] = r[i];
    for (int i = 0; i < lb; i++) al.v[i] = r[hb + i];
    launch(ah, hi, (size_t)1 << hb, blob != nullptr);
    launch(al, lo, (size_t)1 << lb, false);
    hipLaunchKernelGGL(k_eq_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, hi, lo, lb, out, n);
  }
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

int dev_eq_tables(spg_ctx* ctx, const EqJob* jobs, int nj) {
  static const bool lds_on = !getenv("SPG_EQ_LDS") || atoi(getenv("SPG_EQ_LDS")) != 0;
  static const bool multi_on = !getenv("SPG_EQ_MULTI") || atoi(getenv("SPG_EQ_MULTI")) != 0;
  EqTablesArg a;
  a.nj = 0;
  uint32_t blocks = 0;
  double bytes = 0;
  auto flush = [&]() -> int {
    if (!a.nj) return 0;
    KScope ks(ctx, "eq_table", bytes);
    hipLaunchKernelGGL(k_eq_tables_lds, dim3(blocks), dim3(256), 0, ctx->stream, a);
    a.nj = 0;
    blocks = 0;
    bytes = 0;
    SPG_HIP(ctx, hipGetLastError());
    return 0;
  };
  for (int k = 0; k < nj; k++) {
    const EqJob& j = jobs[k];
    if (j.ell < 0 || j.ell > 32) return set_err(ctx, SPG_E_ARG, "eq table: too many variables");
    if (!multi_on || !lds_on || j.ell > 16) {  // the one-table path (large tables: factored form)
      int rc = dev_eq_table(ctx, j.r, j.ell, j.out);
      if (rc) return rc;
      continue;
    }
    const size_t n = (size_t)1 << j.ell;
    a.r[a.nj].n = j.ell;
    for (int i = 0; i < j.ell; i++) a.r[a.nj].v[i] = j.r[i];
    a.out[a.nj] = j.out;
    a.n[a.nj] = n;
    a.b0[a.nj] = blocks;
    blocks += (uint32_t)((n + 255) / 256);
    bytes += 32.0 * n;
    if (++a.nj == EqTablesArg::kMax) {
      int rc = flush();
      if (rc) return rc;
    }
  }
  return flush();
}

int dev_fold_top(spg_ctx* ctx, Fq* v, size_t len, const Fq& r) {
  size_t n = len / 2;
  if (n == 0) return 0;
  KScope ks(ctx, "fold_dense", 96.0 * n);
  hipLaunchKernelGGL(k_fold_top, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, v, n, r);
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

// every instance's descriptor (host vector v) and the table-wide fields of a
static void pqx_fill_args(const PqxDev& T, PqxArgs& a, std::vector<PqxInst>& v) {
  a.zlen = (int)T.zlen;
  a.ninst = (int)T.num_instances;
  a.nws = (int)T.num_witness_secs;
  a.ext = nullptr;
  v.assign(T.zlen, PqxInst{});
  for (size_t p = 0; p < T.zlen; p++) {
    PqxInst& d = v[p];
    d.off_lo = (uint32_t)T.off[p];
    d.off_hi = (uint32_t)(T.off[p] >> 32);
    d.anp = (uint32_t)T.anp[p];
    d.anw = (uint32_t)T.anw[p];
    d.ani = (uint32_t)T.ani[p];
    d.np = (uint32_t)T.num_proofs[p];
    d.ni = (uint32_t)T.num_inputs[p];
    d.dom_off = 0;
    d.sc_np = d.sc_ni = d.step_q = d.step_x = 1;
  }
}
// the descriptors into the kernel arguments, or - more than kMaxP instances - into device memory (workspace slot;
// stream-ordered, so the next launch's copy into the same slot lands after this launch has read it)
enum : size_t { kWsPqxA = 110, kWsPqxB = 111 };
static int pqx_pack(spg_ctx* ctx, const std::vector<PqxInst>& v, PqxArgs& a, size_t slot) {
  a.ext = nullptr;
  for (size_t p = 0; p < v.size() && p < (size_t)kMaxP; p++) a.in[p] = v[p];
  if (v.size() <= (size_t)kMaxP) return 0;
  PqxInst* d = (PqxInst*)ws_get(ctx, slot, v.size() * sizeof(PqxInst));
  if (!d) return set_err(ctx, SPG_E_NOMEM, "instance descriptors");
  SPG_HIP(ctx, hipMemcpyAsync(d, v.data(), v.size() * sizeof(PqxInst), hipMemcpyHostToDevice, ctx->stream));
  a.ext = d;
  return 0;
}

int phase1_eval(spg_ctx* ctx, const PqxDev& T, int mode, size_t proof_len, size_t cons_len, size_t instance_len,
                const std::vector<size_t>& sc_np, const std::vector<size_t>& sc_nc, const Fq* Ap, const Fq* Aq,
                const Fq* Ax, Fq* B, Fq* C, Fq* D, Fq* partials, Fq* out3, const FoldPlan* fold) {
  PqxArgs a;
  std::vector<PqxInst> v;
  pqx_fill_args(T, a, v);
  size_t P = std::min(instance_len, sc_np.size());
  if (P > T.zlen) return set_err(ctx, SPG_E_ARG, "phase-1 domain wider than the table");
  a.P = (int)P;
  size_t dom = 0;
  for (size_t p = 0; p < P; p++) {
    PqxInst& d = v[p];
    d.dom_off = (uint32_t)dom;
    d.sc_np = (uint32_t)sc_np[p];
    d.sc_ni = (uint32_t)sc_nc[p];
    d.step_q = (uint32_t)(proof_len / sc_np[p]);
    d.step_x = (uint32_t)(cons_len / sc_nc[p]);
    dom += sc_np[p] * sc_nc[p];
  }
  if (fold) {
    if (mode == MODE_P || fold->stride.size() < P) return set_err(ctx, SPG_E_ARG, "fused fold: bad plan");
    for (size_t p = 0; p < P; p++) v[p].fstride = fold->stride[p];
  }
  if (dom >= 0xffffffffULL) return set_err(ctx, SPG_E_ARG, "phase-1 domain too large");
  if (int rc = pqx_pack(ctx, v, a, kWsPqxA)) return rc;
  const bool quad = dom <= sc_quad_max();
  const int nb = quad ? grid_for((uint32_t)(4 * dom)) : grid_for((uint32_t)dom);
  // x-mode rounds over rows of >= 128 points: the row-factored kernel, J points per lane (SPG_P1_ROWS=0: off)
  static const bool rows_on = !getenv("SPG_P1_ROWS") || atoi(getenv("SPG_P1_ROWS")) != 0;
  int J = 0;
  if (rows_on && !quad && mode == MODE_X && (!fold || fold->arg.fmode == MODE_X)) {
    size_t mn = ~(size_t)0;
    for (size_t p = 0; p < P; p++) mn = std::min(mn, (size_t)v[p].sc_ni);
    J = mn >= 512 ? 8 : (mn >= 256 ? 4 : (mn >= 128 ? 2 : 0));
    // every row a multiple of 64 J points (power-of-two rows), so no wave's chunk straddles two rows
    for (size_t p = 0; p < P && J; p++)
      if (v[p].sc_ni % (64 * (size_t)J)) J = 0;
  }
  if (J) {
    const uint32_t nchunk = (uint32_t)(dom / (64 * (size_t)J));
    const int nbx = std::max(1, std::min(nb, (int)((nchunk + 3) / 4)));
    // Fq products per point: the folds as k_phase1_eval, 6 for A (B C - D) at 3 points, the row factor per J points
    KScope ks(ctx, fold ? "sc_phase1_fold_eval" : "sc_phase1_eval",
              (fold ? 576.0 : 192.0) * dom + (fold ? 96.0 * fold->arg.side_half : 0.0) + 64.0 * (instance_len + proof_len),
              0.0, (double)dom * (6.0 + (fold ? 7.0 : 0.0) + 4.0 / J));
    const FoldArg fa = fold ? fold->arg : FoldArg{};
#define SPG_P1X(FF, JJ)                                                                                              \
  hipLaunchKernelGGL((k_phase1_eval_x<FF, JJ>), dim3(nbx), dim3(256), 0, ctx->stream, a, (uint32_t)dom,              \
                     (uint32_t)cons_len, Ap, Aq, Ax, B, C, D, partials, ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq, fa)
    if (fold) {
      if (J == 8) SPG_P1X(true, 8); else if (J == 4) SPG_P1X(true, 4); else SPG_P1X(true, 2);
    } else {
      if (J == 8) SPG_P1X(false, 8); else if (J == 4) SPG_P1X(false, 4); else SPG_P1X(false, 2);
    }
#undef SPG_P1X
    SPG_HIP(ctx, hipGetLastError());
    return eval_reduce_finish(ctx, out3);
  }
  if (!fold) {
    // B, C, D lo+hi per domain point, plus the three eq factor tables once
    // Fq products per point: the eq factor at lo and hi (x rounds share Ap Aq: 3; else 4), then A (B C - D) at 3 points
    KScope ks(ctx, "sc_phase1_eval", 192.0 * dom + 64.0 * (instance_len + proof_len + cons_len), 0.0,
              (double)dom * ((mode == MODE_X ? 3 : 4) + 6));
    hipLaunchKernelGGL(quad ? k_phase1_eval_q<false> : k_phase1_eval<false>, dim3(nb), dim3(256), 0, ctx->stream, a,
                       mode, (uint32_t)dom, (uint32_t)proof_len, (uint32_t)cons_len, (uint32_t)instance_len, Ap, Aq,
                       Ax, B, C, D, partials, ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq, FoldArg{});
  } else {
    // per point: B, C, D lo + hi and their fold partners read, lo + hi written; the side table's half once
    // Fq products per point: as sc_phase1_eval, plus B, C, D folded at lo and hi (6) and the side table's entries (1)
    KScope ks(ctx, "sc_phase1_fold_eval", 576.0 * dom + 96.0 * fold->arg.side_half + 64.0 * (instance_len + proof_len),
              0.0, (double)dom * ((mode == MODE_X ? 3 : 4) + 6 + 7));
    hipLaunchKernelGGL(quad ? k_phase1_eval_q<true> : k_phase1_eval<true>, dim3(nb), dim3(256), 0, ctx->stream, a,
                       mode, (uint32_t)dom, (uint32_t)proof_len, (uint32_t)cons_len, (uint32_t)instance_len, Ap, Aq,
                       Ax, B, C, D, partials, ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq, fold->arg);
  }
  SPG_HIP(ctx, hipGetLastError());
  return eval_reduce_finish(ctx, out3);
}

// two phase-1 rounds in one launch (k_phase1_pair); the 15 point sums land in out15 (nullptr: collect them with
// pair_wait). rows / cols: the element grid per instance (x mode: live q rows x N/4; q mode: N/4 x live x columns),
// step_q / step_x the eq index steps of round j, c round j's half length of the mode's eq table.
int phase1_pair(spg_ctx* ctx, const PqxDev& T, const P1Pair& pp, Fq* partials, Fq* out15) {
  P1PairArgs A;
  std::vector<PqxInst> v;
  pqx_fill_args(T, A.a, v);
  const size_t P = pp.rows.size();
  if (P > T.zlen || pp.cols.size() != P || pp.step_q.size() != P || pp.step_x.size() != P)
    return set_err(ctx, SPG_E_ARG, "phase-1 pair: bad shape");
  A.a.P = (int)P;
  size_t dom = 0;
  for (size_t p = 0; p < P; p++) {
    PqxInst& d = v[p];
    d.dom_off = (uint32_t)dom;
    d.sc_np = (uint32_t)pp.rows[p];
    d.sc_ni = (uint32_t)pp.cols[p];
    d.step_q = (uint32_t)pp.step_q[p];
    d.step_x = (uint32_t)pp.step_x[p];
    const uint32_t N = pp.mode == MODE_X ? d.ni : d.np;
    if (N < 4 || (N & (N - 1))) return set_err(ctx, SPG_E_ARG, "phase-1 pair: a size below 4");
    if (pp.nf == 1) d.fstride = pp.fstride.at(p);
    dom += pp.rows[p] * pp.cols[p];
  }
  if (dom == 0 || dom > kP1PairMax) return set_err(ctx, SPG_E_ARG, "phase-1 pair: domain size");
  if (int rc = pqx_pack(ctx, v, A.a, kWsPqxA)) return rc;
  A.mode = pp.mode;
  A.total = (uint32_t)dom;
  A.c = (uint32_t)pp.c;
  A.nf = pp.nf;
  A.r1 = pp.r1;
  A.r2 = pp.r2;
  A.r12 = fq_mul(pp.r1, pp.r2);
  A.fmode = pp.fmode;
  A.side_in = pp.side_in;
  A.side_out = pp.side_out;
  A.side_live = pp.nf ? (uint32_t)pp.side_live : 0;
  A.Ap = pp.Ap;
  A.Aq = pp.Aq;
  A.Ax = pp.Ax;
  A.B = pp.B;
  A.C = pp.C;
  A.D = pp.D;
  A.partials = partials;
  A.counter = ctx->d_counter;
  A.mb = ctx->d_mbox;
  A.seq = ++ctx->mbox_seq;
  const unsigned nb = (unsigned)((16 * dom + 255) / 256);
  {
    // per element: 3 tables x 4 corners (x 4 entries read + 1 written with two pending folds) and the eq corners;
    // Fq products: the folds (3 per corner at nf 2, 1 at nf 1), the eq corners (2 each), 15 points x 2
    const double per = 32.0 * (12.0 * (pp.nf == 2 ? 5.0 : (pp.nf == 1 ? 3.0 : 1.0)) + 8.0);
    KScope ks(ctx, "sc_phase1_pair", per * (double)dom + 32.0 * (pp.nf == 2 ? 5.0 : 3.0) * (double)A.side_live, 0.0,
              (double)dom * (30.0 + 8.0 + 12.0 * (pp.nf == 2 ? 3.0 : (pp.nf == 1 ? 1.0 : 0.0))));
    hipLaunchKernelGGL(k_phase1_pair<256>, dim3(nb), dim3(256), 0, ctx->stream, A);
  }
  SPG_HIP(ctx, hipGetLastError());
  return out15 ? mbox_wait(ctx, ctx->mbox_seq, out15, 15) : 0;
}
int pair_wait(spg_ctx* ctx, Fq* out15) { return mbox_wait(ctx, ctx->mbox_seq, out15, 15); }

// the last pair's two folds (k_phase1_fold2x): T's sizes are those after both folds (pqx_fold_plan done twice);
// rows / cols the live entry grid per instance, side: the pair's eq table (side_live entries after the folds)
int phase1_fold2x(spg_ctx* ctx, const PqxDev& T, const P1Pair& pp) {
  P1PairArgs A;
  std::vector<PqxInst> v;
  pqx_fill_args(T, A.a, v);
  const size_t P = pp.rows.size();
  if (P > T.zlen || pp.cols.size() != P) return set_err(ctx, SPG_E_ARG, "phase-1 fold2x: bad shape");
  A.a.P = (int)P;
  size_t dom = 0;
  for (size_t p = 0; p < P; p++) {
    v[p].dom_off = (uint32_t)dom;
    v[p].sc_np = (uint32_t)pp.rows[p];
    v[p].sc_ni = (uint32_t)pp.cols[p];
    dom += pp.rows[p] * pp.cols[p];
  }
  if (dom >= 0xffffffffULL) return set_err(ctx, SPG_E_ARG, "phase-1 fold2x: domain size");
  if (int rc = pqx_pack(ctx, v, A.a, kWsPqxA)) return rc;
  A.mode = pp.mode;
  A.total = (uint32_t)dom;
  A.nf = 2;
  A.r1 = pp.r1;
  A.r2 = pp.r2;
  A.r12 = fq_mul(pp.r1, pp.r2);
  A.side_in = pp.side_in;
  A.side_out = pp.side_out;
  A.side_live = (uint32_t)pp.side_live;
  A.B = pp.B;
  A.C = pp.C;
  A.D = pp.D;
  const size_t n = std::max(dom, pp.side_live);
  {
    KScope ks(ctx, "sc_fold", 32.0 * 5.0 * (3.0 * (double)dom + (double)pp.side_live));
    hipLaunchKernelGGL(k_phase1_fold2x, dim3((unsigned)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 4096))),
                       dim3(256), 0, ctx->stream, A);
  }
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

// the descriptors of a phase-2 pair launch (els: elements per w row, N / 4 for a pair, N for its folds)
static int p2_args(spg_ctx* ctx, const PqxDev& AB, const PqxDev& Z, const P2Pair& pp, bool fold, P2PairArgs& A,
                   size_t* dom_out) {
  std::vector<PqxInst> va, vz;
  pqx_fill_args(AB, A.ab, va);
  pqx_fill_args(Z, A.zz, vz);
  const size_t P = std::min(Z.num_instances, Z.zlen);
  const bool shared = pp.B_out != nullptr;
  if ((shared ? AB.zlen != 1 : AB.zlen != Z.zlen) || P == 0) return set_err(ctx, SPG_E_ARG, "phase-2 pair: ABC shape");
  A.ab.P = shared ? 1 : (int)P;
  A.zz.P = (int)P;
  size_t dom = 0;
  for (size_t p = 0; p < P; p++) {
    const uint32_t N = vz[p].ni;
    const PqxInst& da = va[shared ? 0 : p];
    if (da.ni != N || N < (fold ? 1u : 4u) || (N & (N - 1)) || pp.W > vz[p].anw || pp.W > da.anw)
      return set_err(ctx, SPG_E_ARG, "phase-2 pair: sizes");
    vz[p].dom_off = (uint32_t)dom;
    vz[p].sc_ni = fold ? N : N / 4;
    dom += pp.W * vz[p].sc_ni;
  }
  if (dom == 0 || dom > (fold ? (size_t)0xffffffffULL : (size_t)kP1PairMax))
    return set_err(ctx, SPG_E_ARG, "phase-2 pair: domain size");
  if (int rc = pqx_pack(ctx, va, A.ab, kWsPqxA)) return rc;
  if (int rc = pqx_pack(ctx, vz, A.zz, kWsPqxB)) return rc;
  A.total = (uint32_t)dom;
  A.nf = fold ? 2 : pp.nf;
  A.r1 = pp.r1;
  A.r2 = pp.r2;
  A.r12 = fq_mul(pp.r1, pp.r2);
  A.eq = pp.eq;
  A.B = AB.d;
  A.B_out = pp.B_out;
  A.shared = shared ? 1 : 0;
  A.C = Z.d;
  *dom_out = dom;
  return 0;
}

int phase2_pair(spg_ctx* ctx, const PqxDev& AB, const PqxDev& Z, const P2Pair& pp, Fq* partials) {
  P2PairArgs A;
  size_t dom = 0;
  if (int rc = p2_args(ctx, AB, Z, pp, false, A, &dom)) return rc;
  A.partials = partials;
  A.counter = ctx->d_counter;
  A.mb = ctx->d_mbox;
  A.seq = ++ctx->mbox_seq;
  const unsigned nb = (unsigned)((16 * dom + 255) / 256);
  {
    // per element: 2 tables x 4 corners (4 entries read + 1 written with the pending folds); Fq products: the folds
    // (3 per corner), 15 points x 2
    KScope ks(ctx, "sc_phase2_pair", 32.0 * 8.0 * (pp.nf == 2 ? 5.0 : 1.0) * (double)dom, 0.0,
              (double)dom * (30.0 + 8.0 * (pp.nf == 2 ? 3.0 : 0.0)));
    hipLaunchKernelGGL(k_phase2_pair<256>, dim3(nb), dim3(256), 0, ctx->stream, A);
  }
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

int phase2_fold2x(spg_ctx* ctx, const PqxDev& AB, const PqxDev& Z, const P2Pair& pp) {
  P2PairArgs A;
  size_t dom = 0;
  if (int rc = p2_args(ctx, AB, Z, pp, true, A, &dom)) return rc;
  {
    KScope ks(ctx, "sc_fold", 32.0 * 5.0 * 2.0 * (double)dom);
    hipLaunchKernelGGL(k_phase2_fold2x, dim3((unsigned)std::max<size_t>(1, std::min<size_t>((dom + 255) / 256, 4096))),
                       dim3(256), 0, ctx->stream, A);
  }
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

int phase2_eval(spg_ctx* ctx, const PqxDev& AB, const PqxDev& Z, int mode, size_t instance_len,
                size_t witness_secs_len, size_t nws_actual, bool single, const std::vector<size_t>& sc_ni,
                const Fq* eq, Fq* partials, Fq* out3, const Fold2* fold) {
  PqxArgs ab, zz;
  std::vector<PqxInst> vab, vz;
  pqx_fill_args(AB, ab, vab);
  pqx_fill_args(Z, zz, vz);
  size_t P = std::min(instance_len, sc_ni.size());
  if (P > Z.zlen) return set_err(ctx, SPG_E_ARG, "phase-2 domain wider than the table");
  ab.P = (int)AB.zlen;
  zz.P = (int)P;
  size_t W = std::min(witness_secs_len, nws_actual);
  size_t dom = 0;
  for (size_t p = 0; p < P; p++) {
    vz[p].dom_off = (uint32_t)dom;
    vz[p].sc_ni = (uint32_t)sc_ni[p];
    dom += W * sc_ni[p];
  }
  if (fold) {
    if (mode == MODE_P || fold->a.stride.size() < vab.size() || fold->z.stride.size() < P)
      return set_err(ctx, SPG_E_ARG, "fused fold: bad plan");
    for (size_t p = 0; p < vab.size(); p++) vab[p].fstride = fold->a.stride[p];
    for (size_t p = 0; p < P; p++) vz[p].fstride = fold->z.stride[p];
  }
  if (int rc = pqx_pack(ctx, vab, ab, kWsPqxA)) return rc;
  if (int rc = pqx_pack(ctx, vz, zz, kWsPqxB)) return rc;
  const bool quad = dom <= sc_quad_max();
  const int nb = quad ? grid_for((uint32_t)(4 * dom)) : grid_for((uint32_t)dom);
  const Fold2Arg fa = fold ? fold->arg : Fold2Arg{};
  {
    // ABC and Z lo+hi per domain point; fused: their fold partners read and the folded entries written too
    // Fq products per point: eq ABC Z at 3 points (6), plus ABC and Z folded at lo and hi when fused (4)
    KScope ks(ctx, fold ? "sc_phase2_fold_eval" : "sc_phase2_eval", (fold ? 384.0 : 128.0) * dom, 0.0,
              (double)dom * (fold ? 10 : 6));
    if (quad)
      hipLaunchKernelGGL(fold ? k_phase2_eval_q<true> : k_phase2_eval_q<false>, dim3(nb), dim3(256), 0, ctx->stream,
                         ab, zz, mode, (uint32_t)dom, single, (uint32_t)instance_len, eq, AB.d, Z.d, partials,
                         ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq, fa);
    else
      hipLaunchKernelGGL(fold ? k_phase2_eval<true> : k_phase2_eval<false>, dim3(nb), dim3(256), 0, ctx->stream, ab, zz,
                         mode, (uint32_t)dom, (int)W, single, (uint32_t)instance_len, eq, AB.d, Z.d, partials,
                         ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq, fa);
  }
  SPG_HIP(ctx, hipGetLastError());
  return eval_reduce_finish(ctx, out3);
}

// DensePolynomialPqx::bound_poly(r, mode) applied to up to three tables of identical shape (T[0] owns shape)
// host bookkeeping of one Pqx fold (the reference's field updates) and the kernel arguments; dom = entries
static int pqx_prepare(spg_ctx* ctx, PqxDev& T, int mode, PqxArgs& a, size_t& dom, size_t slot) {
  size_t P = std::min(T.num_instances, T.zlen);
  // host-side size bookkeeping first (mirrors the reference's field updates)
  if (mode == MODE_P) {
    T.num_instances /= 2;
    P = T.num_instances;
  } else if (mode == MODE_Q) {
    T.max_num_proofs /= 2;
  } else if (mode == MODE_W) {
    T.num_witness_secs /= 2;
  } else {
    T.max_num_inputs /= 2;
  }
  std::vector<PqxInst> v;
  pqx_fill_args(T, a, v);  // a.ninst / a.nws are the *new* values
  a.P = (int)P;
  dom = 0;
  std::vector<size_t> np_after(T.num_proofs), ni_after(T.num_inputs);
  for (size_t p = 0; p < P; p++) {
    PqxInst& d = v[p];
    size_t rows, nw, cols;
    if (mode == MODE_P) {
      rows = 1;
      nw = std::min(T.num_witness_secs, T.anw[p]);
      cols = 1;
    } else if (mode == MODE_Q) {
      nw = std::min(T.num_witness_secs, T.anw[p]);
      cols = T.num_inputs[p];
      if (T.num_proofs[p] == 1) rows = 1;
      else { rows = T.num_proofs[p] / 2; np_after[p] = rows; }
    } else if (mode == MODE_W) {
      rows = T.num_proofs[p];
      nw = T.num_witness_secs;
      cols = T.num_inputs[p];
    } else {
      rows = T.num_proofs[p];
      nw = std::min(T.num_witness_secs, T.anw[p]);
      if (T.num_inputs[p] == 1) cols = 1;
      else { cols = T.num_inputs[p] / 2; ni_after[p] = cols; }
    }
    d.dom_off = (uint32_t)dom;
    d.sc_ni = (uint32_t)cols;
    d.step_q = (uint32_t)nw;
    dom += rows * nw * cols;
  }
  T.num_proofs = np_after;
  T.num_inputs = ni_after;
  return pqx_pack(ctx, v, a, slot);
}

int pqx_bound(spg_ctx* ctx, PqxDev& T, Fq* d1, Fq* d2, const Fq& r, int mode, Fq* side, size_t side_len) {
  PqxArgs a;
  size_t dom = 0;
  int rc = pqx_prepare(ctx, T, mode, a, dom, kWsPqxA);
  if (rc) return rc;
  const size_t side_half = side ? side_len / 2 : 0;
  if (dom || side_half) {
    double nt = 1.0 + (d1 ? 1.0 : 0.0) + (d2 ? 1.0 : 0.0);
    KScope ks(ctx, "sc_fold", 96.0 * (nt * dom + side_half));  // read lo+hi, write lo, per table
    const size_t n = std::max(dom, side_half);
    hipLaunchKernelGGL(k_pqx_fold, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, a, mode,
                       (uint32_t)dom, r, T.d, d1, d2, side, (uint32_t)side_half);
    SPG_HIP(ctx, hipGetLastError());
  }
  return 0;
}

int pqx_fold_plan(spg_ctx* ctx, PqxDev& T, int mode, FoldPlan* fp) {
  if (mode != MODE_X && mode != MODE_Q && mode != MODE_W) return set_err(ctx, SPG_E_ARG, "fused fold: mode");
  const size_t P = std::min(T.num_instances, T.zlen);
  fp->stride.assign(T.zlen, 0);
  fp->fw = 0;
  if (mode == MODE_W) {  // partner w + nws / 2, when that section exists (pqx_fold_at)
    const size_t fw = T.num_witness_secs / 2;
    for (size_t p = 0; p < P; p++) {
      const size_t s = fw * T.ani[p];
      if (s >= 0xffffffffULL) return set_err(ctx, SPG_E_ARG, "fused fold: stride");
      fp->stride[p] = (uint32_t)s;
    }
    fp->fw = (uint32_t)fw;
    T.num_witness_secs = fw;
    return 0;
  }
  for (size_t p = 0; p < P; p++) {  // the partner of pqx_fold_at, from the sizes before the fold
    const size_t n = mode == MODE_X ? T.num_inputs[p] : T.num_proofs[p];
    const size_t row = mode == MODE_X ? 1 : T.anw[p] * T.ani[p];
    const size_t s = n == 1 ? 0 : (n / 2) * row;
    if (s >= 0xffffffffULL) return set_err(ctx, SPG_E_ARG, "fused fold: stride");
    fp->stride[p] = (uint32_t)s;
  }
  // the size bookkeeping of pqx_prepare (mirrors the reference's field updates)
  if (mode == MODE_Q) T.max_num_proofs /= 2;
  else T.max_num_inputs /= 2;
  for (size_t p = 0; p < P; p++) {
    size_t& n = mode == MODE_X ? T.num_inputs[p] : T.num_proofs[p];
    if (n != 1) n /= 2;
  }
  return 0;
}

int pqx_bound2(spg_ctx* ctx, PqxDev& TA, PqxDev& TB, const Fq& r, int mode) {
  PqxArgs a, b;
  size_t da = 0, db = 0;
  int rc = pqx_prepare(ctx, TA, mode, a, da, kWsPqxA);
  if (!rc) rc = pqx_prepare(ctx, TB, mode, b, db, kWsPqxB);
  if (rc) return rc;
  if (da + db) {
    KScope ks(ctx, "sc_fold", 96.0 * (double)(da + db));
    hipLaunchKernelGGL(k_pqx_fold2, dim3((unsigned)((da + db + 255) / 256)), dim3(256), 0, ctx->stream, a,
                       (uint32_t)da, TA.d, b, (uint32_t)db, TB.d, mode, r);
    SPG_HIP(ctx, hipGetLastError());
  }
  return 0;
}

int pqx_bound_q_all(spg_ctx* ctx, PqxDev& T, const Fq* E, size_t nq) {
  PqxArgs a;
  std::vector<PqxInst> v;
  pqx_fill_args(T, a, v);  // the sizes before the folds
  const size_t P = std::min(T.num_instances, T.zlen);
  a.P = (int)P;
  // row groups per output: enough lanes for ~2^19 (two per lane slot of the chip), at most 256 and the rows there are
  size_t outs = 0, rows = 1;
  for (size_t p = 0; p < P; p++) {
    outs += std::min(T.num_witness_secs, T.anw[p]) * T.num_inputs[p];
    rows = std::max(rows, T.num_proofs[p]);
  }
  int G = 16;
  while (G < 256 && outs * (size_t)G < ((size_t)1 << 19) && (size_t)G < rows) G *= 2;
  const size_t O = 256 / G;
  size_t dom = 0, reads = 0;
  for (size_t p = 0; p < P; p++) {
    PqxInst& d = v[p];
    const size_t nw = std::min(T.num_witness_secs, T.anw[p]), cols = T.num_inputs[p];
    if (T.num_proofs[p] > ((size_t)1 << nq) || nq > 31) return set_err(ctx, SPG_E_ARG, "q bound: rows exceed 2^nq");
    d.dom_off = (uint32_t)dom;
    d.sc_ni = (uint32_t)cols;
    d.step_q = (uint32_t)nw;
    dom += (nw * cols + O - 1) / O * O;
    reads += T.num_proofs[p] * nw * cols;
  }
  if (dom >= ((size_t)1 << 32)) return set_err(ctx, SPG_E_ARG, "q bound: domain");
  // the bookkeeping of nq pqx_prepare(MODE_Q) calls: every local instance ends with one row
  for (size_t j = 0; j < nq; j++) T.max_num_proofs /= 2;
  for (size_t p = 0; p < P; p++) T.num_proofs[p] = 1;
  int rc = pqx_pack(ctx, v, a, kWsPqxA);
  if (rc) return rc;
  if (dom) {
    KScope ks(ctx, "sc_fold_q_all", 32.0 * (double)(reads + dom));
    const dim3 grid((unsigned)(dom / O));
    if (G == 16) hipLaunchKernelGGL(k_pqx_bound_q<16>, grid, dim3(256), 0, ctx->stream, a, E, (int)nq, T.d);
    else if (G == 32) hipLaunchKernelGGL(k_pqx_bound_q<32>, grid, dim3(256), 0, ctx->stream, a, E, (int)nq, T.d);
    else if (G == 64) hipLaunchKernelGGL(k_pqx_bound_q<64>, grid, dim3(256), 0, ctx->stream, a, E, (int)nq, T.d);
    else if (G == 128) hipLaunchKernelGGL(k_pqx_bound_q<128>, grid, dim3(256), 0, ctx->stream, a, E, (int)nq, T.d);
    else hipLaunchKernelGGL(k_pqx_bound_q<256>, grid, dim3(256), 0, ctx->stream, a, E, (int)nq, T.d);
    SPG_HIP(ctx, hipGetLastError());
  }
  return 0;
}

int cubic_eval(spg_ctx* ctx, const Fq* A, const Fq* B, const Fq* C, size_t len_half, Fq* partials,
               Fq* out3) {
  int nb = grid_for((uint32_t)len_half);
  {
    KScope ks(ctx, "sc_cubic_eval", 192.0 * len_half);
    hipLaunchKernelGGL(k_cubic_eval, dim3(nb), dim3(256), 0, ctx->stream, A, B, C, (uint32_t)len_half, partials,
                       ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq);
  }
  SPG_HIP(ctx, hipGetLastError());
  return eval_reduce_finish(ctx, out3);
}

}  // namespace spg

// EqPolynomial::evals (src/dense_mlpoly.rs:76-92) into a new device vector of 2^ell scalars
extern "C" int spg_eq_evals(spg_ctx* ctx, const uint64_t* r_mont, size_t ell, spg_buf** out) {
  if (!ctx || !out || (!r_mont && ell)) return SPG_E_ARG;
  if (ell > 30) return spg::set_err(ctx, SPG_E_ARG, "spg_eq_evals: at most 30 variables");
  spg_buf* b = new spg_buf();
  b->n = (size_t)1 << ell;
  if (hipMalloc(&b->d, b->n * sizeof(spg::Fq)) != hipSuccess) {
    delete b;
    return spg::set_err(ctx, SPG_E_NOMEM, "spg_eq_evals");
  }
  std::vector<spg::Fq> r(ell);
  if (ell) memcpy(r.data(), r_mont, ell * sizeof(spg::Fq));
  int rc = spg::dev_eq_table(ctx, r.data(), (int)ell, b->d);
  if (!rc) rc = hipStreamSynchronize(ctx->stream) == hipSuccess ? 0 : spg::set_err(ctx, SPG_E_HIP, "spg_eq_evals");
  if (rc) {
    hipFree(b->d);
    delete b;
    return rc;
  }
  *out = b;
  return SPG_OK;
}
