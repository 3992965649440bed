// spg — SPARK layer-sumcheck kernels (ProductCircuitEvalProofBatched rounds, product_tree.rs:271-396);
// spark.hip launches them, scripts/micro/layer_phases.hip times their phases.
#pragma once
#include <hip/hip_runtime.h>

#include "ctx.hpp"
#include "lds.hpp"
#include "qsum.hpp"
#include "cube.hpp"

namespace spg {

struct Triple {
  Fq *A, *B, *C;
};
__device__ __forceinline__ void block_sum3_sp(Fq& v0, Fq& v1, Fq& v2) {
  __shared__ uint32_t sh[3][soa_words<Fq, 256>()];  // component-major: no bank conflicts
  int t = threadIdx.x;
  for (int d = 128; d >= 1; d >>= 1) {
    if (t >= d && t < 2 * d) {
      soa_put<256>(sh[0], t - d, v0);
      soa_put<256>(sh[1], t - d, v1);
      soa_put<256>(sh[2], t - d, v2);
    }
    __syncthreads();
    if (t < d) {
      v0 = fq_add(v0, soa_get<256, Fq>(sh[0], t));
      v1 = fq_add(v1, soa_get<256, Fq>(sh[1], t));
      v2 = fq_add(v2, soa_get<256, Fq>(sh[2], t));
    }
    __syncthreads();
  }
  // broadcast thread 0's sums
  if (t == 0) {
    soa_put<256>(sh[0], 0, v0);
    soa_put<256>(sh[1], 0, v1);
    soa_put<256>(sh[2], 0, v2);
  }
  __syncthreads();
  v0 = soa_get<256, Fq>(sh[0], 0);
  v1 = soa_get<256, Fq>(sh[1], 0);
  v2 = soa_get<256, Fq>(sh[2], 0);
  __syncthreads();
}
// block-wide sums of three Fq values over BS threads; the result is valid in thread 0
template <int BS>
__device__ __forceinline__ void block_sum3_t0(Fq& v0, Fq& v1, Fq& v2) {
  __shared__ uint32_t sh[3][soa_words<Fq, BS / 2>()];
  const int t = threadIdx.x;
  for (int d = BS / 2; d >= 1; d >>= 1) {
    if (t >= d && t < 2 * d) {
      soa_put<BS / 2>(sh[0], t - d, v0);
      soa_put<BS / 2>(sh[1], t - d, v1);
      soa_put<BS / 2>(sh[2], t - d, v2);
    }
    __syncthreads();
    if (t < d) {
      v0 = fq_add(v0, soa_get<BS / 2, Fq>(sh[0], t));
      v1 = fq_add(v1, soa_get<BS / 2, Fq>(sh[1], t));
      v2 = fq_add(v2, soa_get<BS / 2, Fq>(sh[2], t));
    }
    __syncthreads();
  }
}
// ---- fused layer rounds (ProductCircuitEvalProofBatched, product_tree.rs:271-396) -------------------------
// One launch per round: element (c, i) of the nt x len domain first applies the previous round's pending
// bound_poly_var_top to the four entries it reads of each of its triple's vectors (X[k] + r (X[k + 2 len] - X[k])
// at k = i and i + len) and writes those two folded entries back, then evaluates the round. Every folded
// entry is read and written by exactly one element, so any number of workgroups fold in place without a
// grid barrier; only the eq vector C, shared by the product circuits (Triple.C == null), is read by every
// circuit's element i and therefore ping-pongs between two buffers (cin -> cout, written by circuit 0).
// One workgroup posts the round's (e0, e2, e3) directly; more add their partials through a ticket.
__device__ __forceinline__ Fq fold_at(const Fq* __restrict__ p, int k, int fl, const Fq& r) {
  const Fq lo = p[k];
  return fq_add(lo, fq_mul(r, fq_sub(p[k + fl], lo)));
}
template <int BS>
__global__ void __launch_bounds__(BS) k_layer_round(const Triple* __restrict__ tr, const Fq* __restrict__ coeff, int nt,
                                                    int log_len, int do_fold, Fq r, const Fq* __restrict__ cin,
                                                    Fq* __restrict__ cout, Fq* __restrict__ partials,
                                                    unsigned* __restrict__ counter, uint32_t* __restrict__ mb,
                                                    uint32_t seq, unsigned long long* probe, int ends = 0) {
  (void)ends;  // the one-lane form never posts the layer's entries (the host closes the layer with k_layer_close)
  const int t = threadIdx.x, len = 1 << log_len;
  unsigned long long* pr = probe ? probe + 8 * blockIdx.x : nullptr;  // phase timestamps (scripts/micro)
  if (pr && t == 0) pr[0] = wall_clock64();
  const long total = (long)nt << log_len;
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (long u = (long)blockIdx.x * BS + t; u < total; u += (long)gridDim.x * BS) {
    const int c = (int)(u >> log_len), i = (int)(u & (len - 1));
    const Triple x = tr[c];
    const Fq k = coeff[c];
    const Fq* Cp = x.C ? x.C : cin;
    Fq al, ah, bl, bh, cl, ch;
    if (do_fold) {
      const int fl = 2 * len;
      al = fold_at(x.A, i, fl, r);
      ah = fold_at(x.A, i + len, fl, r);
      bl = fold_at(x.B, i, fl, r);
      bh = fold_at(x.B, i + len, fl, r);
      cl = fold_at(Cp, i, fl, r);
      ch = fold_at(Cp, i + len, fl, r);
      x.A[i] = al;
      x.A[i + len] = ah;
      x.B[i] = bl;
      x.B[i + len] = bh;
      Fq* Cw = x.C ? x.C : (c == 0 ? cout : nullptr);
      if (Cw) {
        Cw[i] = cl;
        Cw[i + len] = ch;
      }
    } else {
      al = x.A[i];
      ah = x.A[i + len];
      bl = x.B[i];
      bh = x.B[i + len];
      cl = Cp[i];
      ch = Cp[i + len];
    }
    // the coefficient scales the A factor (k A is linear in X)
    al = fq_mul(k, al);
    ah = fq_mul(k, ah);
    const Fq da = fq_sub(ah, al), db = fq_sub(bh, bl), dc = fq_sub(ch, cl);
    const Fq a2 = fq_add(ah, da), b2 = fq_add(bh, db), c2 = fq_add(ch, dc);
    e0 = fq_add(e0, fq_mul(fq_mul(al, bl), cl));
    e2 = fq_add(e2, fq_mul(fq_mul(a2, b2), c2));
    e3 = fq_add(e3, fq_mul(fq_mul(fq_add(a2, da), fq_add(b2, db)), fq_add(c2, dc)));
  }
  if (pr && t == 0) pr[1] = wall_clock64();
  block_sum3_t0<BS>(e0, e2, e3);
  if (pr && t == 0) pr[2] = wall_clock64();
  if (gridDim.x == 1) {
    if (t == 0) {
      mbox_post3(mb, seq, e0, e2, e3);
      if (pr) pr[3] = wall_clock64();
    }
    return;
  }
  __shared__ bool last;
  if (t == 0) {
    partials[3 * blockIdx.x] = e0;
    partials[3 * blockIdx.x + 1] = e2;
    partials[3 * blockIdx.x + 2] = e3;
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
  Fq a = fq_zero(), b = fq_zero(), cc = fq_zero();
  for (unsigned j = t; j < gridDim.x; j += BS) {
    a = fq_add(a, partials[3 * j]);
    b = fq_add(b, partials[3 * j + 1]);
    cc = fq_add(cc, partials[3 * j + 2]);
  }
  block_sum3_t0<BS>(a, b, cc);
  if (t == 0) {
    mbox_post3(mb, seq, a, b, cc);
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// end of a layer: the last round's fold (length 2 -> 1) of every triple's vectors and the layer's final claims
// A[0], B[0], C[0] per triple, written straight into the mailbox (3 nt scalars, then the sequence number).
// do_fold == 0 posts the entries as they are (a sharded layer whose local vectors already have length 1).
__global__ void __launch_bounds__(256) k_layer_close(const Triple* __restrict__ tr, int nt, int do_fold, Fq r,
                                                     const Fq* __restrict__ cin, uint32_t* __restrict__ mb,
                                                     uint32_t seq) {
  for (int c = threadIdx.x; c < nt; c += 256) {
    const Triple x = tr[c];
    const Fq* Cp = x.C ? x.C : cin;
    const Fq v[3] = {do_fold ? fold_at(x.A, 0, 1, r) : x.A[0], do_fold ? fold_at(x.B, 0, 1, r) : x.B[0],
                     do_fold ? fold_at(Cp, 0, 1, r) : Cp[0]};
    for (int k = 0; k < 3; k++) host_put(mb + 8 + 8 * (3 * c + k), v[k]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- the same round with a quad (4 lanes) per element --------------------------------------------------
// A wave issues one instruction at a time, so an element's ~14 field products cost ~14 product times even when
// independent; spread over a quad they take 5: round 1 folds (lane 0: A lo/hi, 1: B, 2: C), the quad exchanges
// the six values (DPP), then lane p in {0, 1, 2} forms the cubic at X = 0, 2, 3 as ((a_X b_X) c_X) k.
// Lane 3 mirrors lane 0's work (SIMT) and is ignored. The sums meet by cross-quad shuffles inside the wave,
// then across waves in LDS.
template <int K>
__device__ __forceinline__ Fq fq_qbcast(const Fq& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], K * 0x55, 0xf, 0xf, false);
  return r;
}
// the elements u = u0, u0 + ustride, ... of one round (a quad per element): this lane's share of its point's sum
// ends (a layer's last round, one workgroup): lane p < 3 also writes its vector's two entries (lo, hi) to mailbox
// scalars 3 + 6 c + 2 p, + 1, so the host folds the final claims itself once it has drawn the round's challenge
__device__ __forceinline__ Fq layer_round_elems(const Triple* __restrict__ tr, const Fq* __restrict__ coeff, int nt,
                                                int log_len, int do_fold, const Fq& r, const Fq* __restrict__ cin,
                                                Fq* __restrict__ cout, long u0, long ustride,
                                                uint32_t* __restrict__ ends = nullptr) {
  const int q = threadIdx.x & 3, len = 1 << log_len;
  const int pt = q < 3 ? q : 0;  // the evaluation point (and round-1 vector) this lane works on
  const long total = (long)nt << log_len;
  Fq e = fq_zero();
  for (long u = u0; u < total; u += ustride) {
    const int c = (int)(u >> log_len), i = (int)(u & (len - 1));
    const Triple x = tr[c];
    const Fq* Cp = x.C ? x.C : cin;
    const Fq* src = pt == 0 ? x.A : (pt == 1 ? x.B : Cp);
    Fq lo = fq_zero(), hi = fq_zero();
    if (q == 3) {
      // lane 3 holds no vector: nothing is broadcast from it, so it loads nothing (its lanes' product below is unused)
    } else if (do_fold) {
      const int fl = 2 * len;
      lo = fold_at(src, i, fl, r);
      hi = fold_at(src, i + len, fl, r);
      Fq* dst = q == 0 ? x.A : (q == 1 ? x.B : (q == 2 ? (x.C ? x.C : (c == 0 ? cout : nullptr)) : nullptr));
      if (dst) {
        dst[i] = lo;
        dst[i + len] = hi;
      }
    } else {
      lo = src[i];
      hi = src[i + len];
    }
    if (ends && q < 3) {
      uint32_t* d = ends + 8 + 8 * (3 + 6 * c + 2 * q);
      host_put(d, lo);
      host_put(d + 8, hi);
    }
    const Fq al = fq_qbcast<0>(lo), ah = fq_qbcast<0>(hi), bl = fq_qbcast<1>(lo), bh = fq_qbcast<1>(hi);
    const Fq cl = fq_qbcast<2>(lo), ch = fq_qbcast<2>(hi);
    const Fq k = coeff[c];
    // (A B) (C k): two independent products, then one -- a dependent chain of two products instead of three
    e = fq_add(e, fq_mul(fq_mul(line_at(al, ah, pt), line_at(bl, bh, pt)), fq_mul(line_at(cl, ch, pt), k)));
  }
  return e;
}
template <int BS>
__global__ void __launch_bounds__(BS) k_layer_round_q(const Triple* __restrict__ tr, const Fq* __restrict__ coeff,
                                                      int nt, int log_len, int do_fold, Fq r, const Fq* __restrict__ cin,
                                                      Fq* __restrict__ cout, Fq* __restrict__ partials,
                                                      unsigned* __restrict__ counter, uint32_t* __restrict__ mb,
                                                      uint32_t seq, unsigned long long* probe, int ends = 0) {
  __shared__ bool last;
  const int t = threadIdx.x, q = t & 3;
  unsigned long long* pr = probe ? probe + 8 * blockIdx.x : nullptr;
  if (pr && t == 0) pr[0] = wall_clock64();
  // ends: only with one workgroup (the host launches it so), whose barrier below orders every wave's entry stores
  // before the sequence number
  Fq e = layer_round_elems(tr, coeff, nt, log_len, do_fold, r, cin, cout, ((long)blockIdx.x * BS + t) >> 2,
                           (long)gridDim.x * (BS / 4), ends && gridDim.x == 1 ? mb : nullptr);
  if (ends) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (pr && t == 0) pr[1] = wall_clock64();
  quad_block_sum<BS>(e);
  if (pr && t == 0) pr[2] = wall_clock64();
  if (gridDim.x == 1) {  // lanes 0..2 of wave 0 post e0, e2, e3, then lane 0 the sequence number
    if (ends) __syncthreads();
    if (t < 3) {
      host_put(mb + 8 + 8 * t, e);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    if (t == 0) {
      __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (pr) pr[3] = wall_clock64();
    }
    return;
  }
  // cross-workgroup hand-off without L2 write-back (the in-place folds leave many dirty lines, which an agent
  // release would flush): the partials go out as sc1 stores (agent-scope relaxed atomics), the storing wave
  // waits for them, then one lane adds to the ticket; the last workgroup reads them with sc1 loads
  // (MI355X_MICROARCH hand-off table, row 1)
  if (t < 3)
    for (int j = 0; j < 8; j++)
      __hip_atomic_store(&partials[3 * blockIdx.x + t].l[j], e.l[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  // the last workgroup: thread 4 m + p (p < 3) adds point p's partials of blocks m, m + BS / 4, ...
  Fq a = fq_zero();
  if (q < 3)
    for (unsigned j = t >> 2; j < gridDim.x; j += BS / 4) {
      Fq o;
      for (int k = 0; k < 8; k++)
        o.l[k] = __hip_atomic_load(&partials[3 * j + q].l[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a = fq_add(a, o);
    }
  quad_block_sum<BS>(a);
  if (t < 3) {
    host_put(mb + 8 + 8 * t, a);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  if (t == 0) {
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- two rounds per launch (the small, latency-bound rounds) ---------------------------------------------------------
// A small round is a host round trip (launch, dispatch, mailbox) around a few us of work, and a layer's rounds are
// transcript-sequential. Round j + 1's evaluations need round j's challenge r, but only as the argument of a cubic:
// with W the vectors of round j (2 len entries, the pending folds applied) and the 2 x 2 cube of element i < h = len / 2,
//   P(t, s) = p00 + t (p10 - p00) + s (p01 - p00) + t s (p11 - p10 - p01 + p00),  p_ts = W[i + (2 t + s) h]
// (t: round j's variable, offset len; s: round j + 1's, offset h), and F(t, s) = k A(t, s) B(t, s) C(t, s) summed over
// every element, round j's evaluation at X is F(X, 0) + F(X, 1), and round j + 1's at Y is the cubic t -> F(t, Y) taken
// at t = r (the fold by r is P(r, .)). So one launch posts F at 15 points -- t = 0..3 on the lines s = 0, 2, 3, and
// t = 0, 2, 3 on s = 1 -- and the host draws r_j, interpolates round j + 1 at r_j and draws r_j+1 with no device round
// trip between them. The next launch applies both folds at once (nf = 2: W[k] = a + r1 (c - a) + r2 (b - a) +
// r1 r2 (d - c - b + a) over V[k + {0, 2, 4, 6} len], r1 bound first), so a pair costs one launch instead of two.
// Lanes: 16 per element (a DPP row). Stage 1: lane g < 12 computes corner m = g & 3 of vector g >> 2 (A, B, C) and
// writes it back in place (every entry is read and written by its own lane: no grid barrier; the shared eq vector C
// goes cin -> cout, written by circuit 0); lane 12 loads the coefficient k. Stage 2: row broadcasts (DPP row_newbcast)
// give every lane the 12 corners and k. Stage 3: lane g forms its point's three values and k A B C. The row sums
// meet in LDS like the quad sums, and the posted scalars are the 15 point sums in lane order:
//   g 0..3: (t, s) = (g, 0); 4..7: (g - 4, 2); 8..11: (g - 8, 3); 12, 13, 14: (0, 1), (2, 1), (3, 1).
// ends (a layer's last pair, h = 1): lane g < 12 also posts its corner as scalar 15 + 12 c + g, so the host folds the
// final claims itself.
struct PairArgs {
  const Triple* tr;
  const Fq* coeff;
  int nt;
  int log_len;  // round j's half length len = 2^log_len (>= 2: h = len / 2 >= 1)
  int nf;       // pending folds: 0, 1 (r1) or 2 (r1, then r2; r12 = r1 r2)
  Fq r1, r2, r12;
  const Fq* cin;
  Fq* cout;
  Fq* partials;  // 16 per workgroup
  unsigned* counter;
  uint32_t* mb;
  uint32_t seq;
  int ends;
  unsigned long long* probe;  // phase timestamps (scripts/micro), null in the prover
};
template <int BS>
__global__ void __launch_bounds__(BS) k_layer_pair(PairArgs A) {
  __shared__ bool last;
  const int t = threadIdx.x, g = t & 15;
  unsigned long long* pr = A.probe ? A.probe + 8 * blockIdx.x : nullptr;
  if (pr && t == 0) pr[0] = wall_clock64();
  const int len = 1 << A.log_len, h = len >> 1;
  const long total = (long)A.nt << (A.log_len - 1);
  const long u = ((long)blockIdx.x * BS + t) >> 4;  // this row's element (rows past the end idle, contribute zero)
  // this lane's point (t, s)
  const int pt = g < 4 ? g : (g < 8 ? g - 4 : (g < 12 ? g - 8 : (g == 12 ? 0 : (g == 13 ? 2 : 3))));
  const int ps = g < 4 ? 0 : (g < 8 ? 2 : (g < 12 ? 3 : 1));
  Fq e = fq_zero();
  if (u < total) {
    const int c = (int)(u >> (A.log_len - 1)), i = (int)(u & (h - 1));
    const Triple x = A.tr[c];
    // stage 1: corner m of vector v
    Fq w = fq_zero();
    if (g < 12) {
      const int v = g >> 2, m = g & 3, k = i + m * h;
      const Fq* src = v == 0 ? x.A : (v == 1 ? x.B : (x.C ? x.C : A.cin));
      if (A.nf == 0) {
        w = src[k];
      } else if (A.nf == 1) {
        const Fq a = src[k], b = src[k + 2 * len];
        w = fq_add(a, fq_mul(A.r1, fq_sub(b, a)));
      } else {
        const Fq a = src[k], b = src[k + 2 * len], cc = src[k + 4 * len], d = src[k + 6 * len];
        const Fq t1 = fq_mul(A.r1, fq_sub(cc, a)), t2 = fq_mul(A.r2, fq_sub(b, a)),
                 t3 = fq_mul(A.r12, fq_add(fq_sub(d, cc), fq_sub(a, b)));
        w = fq_add(fq_add(a, t1), fq_add(t2, t3));
      }
      if (A.nf > 0) {
        Fq* dst = v == 0 ? x.A : (v == 1 ? x.B : (x.C ? x.C : (c == 0 ? A.cout : nullptr)));
        if (dst) dst[k] = w;
      }
      if (A.ends) {
        uint32_t* d = A.mb + 8 + 8 * (15 + 12 * c + g);
        host_put(d, w);
      }
    } else if (g == 12) {
      w = A.coeff[c];
    }
    if (pr && t == 0) pr[1] = wall_clock64();
    // stage 2: every lane of the row takes the corners and k
    const Fq a00 = fq_rowbcast<0>(w), a01 = fq_rowbcast<1>(w), a10 = fq_rowbcast<2>(w), a11 = fq_rowbcast<3>(w);
    const Fq b00 = fq_rowbcast<4>(w), b01 = fq_rowbcast<5>(w), b10 = fq_rowbcast<6>(w), b11 = fq_rowbcast<7>(w);
    const Fq c00 = fq_rowbcast<8>(w), c01 = fq_rowbcast<9>(w), c10 = fq_rowbcast<10>(w), c11 = fq_rowbcast<11>(w);
    const Fq kk = fq_rowbcast<12>(w);
    // stage 3: this lane's point
    const Fq av = cube_at(a00, a01, a10, a11, pt, ps), bv = cube_at(b00, b01, b10, b11, pt, ps),
             cv = cube_at(c00, c01, c10, c11, pt, ps);
    const Fq ab = fq_mul(av, bv), kc = fq_mul(kk, cv);
    e = fq_mul(ab, kc);
  }
  if (A.ends) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // the corners reach the host before any ticket / post
  if (pr && t == 0) pr[2] = wall_clock64();
  row_block_sum<BS>(e);
  if (pr && t == 0) pr[3] = wall_clock64();
  if (gridDim.x == 1) {  // lanes 0..14 of wave 0 post the 15 point sums, then lane 0 the sequence number
    if (A.ends) __syncthreads();
    if (t < 15) {
      host_put(A.mb + 8 + 8 * t, e);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    __syncthreads();
    if (t == 0) {
      __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (pr) pr[4] = wall_clock64();
    }
    return;
  }
  // several workgroups: partials by sc1 stores and a ticket (as quad_grid_post)
  if (t < 16) st_sc1(&A.partials[16 * blockIdx.x + t], e);
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(A.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  Fq s = fq_zero();
  for (unsigned j = t >> 4; j < gridDim.x; j += BS / 16) s = fq_add(s, ld_sc1(&A.partials[16 * j + g]));
  row_block_sum<BS>(s);
  if (t < 15) {
    host_put(A.mb + 8 + 8 * t, s);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  __syncthreads();
  if (t == 0) {
    __hip_atomic_store(A.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- three rounds per launch ------------------------------------------------------------------------------------------
// The pair argument one level further: with the 2 x 2 x 2 cube of element i < h = len / 4 (t: round j's variable, offset
// len; s: round j + 1's, offset len / 2; u: round j + 2's, offset h), P(t, s, u) trilinear in the eight corners and
// F = k A B C, round j's evaluation at X is the sum of F(X, s, u) over s, u in {0, 1}, round j + 1's at Y the cubic
// t -> F(t, Y, 0) + F(t, Y, 1) taken at t = r_j, and round j + 2's at Z the bicubic (t, s) -> F(t, s, Z) taken at
// (r_j, r_j+1). So one launch posts F on the 4 x 4 x 4 grid (lane g = t + 4 s + 16 u; (1, 1, 1) is not needed) and
// the host draws r_j, r_j+1 and r_j+2 with no device round trip between them. A wave per element:
//   fold: lanes g < 48 compute corner q = g % 24 (vector q >> 3, m = q & 7 = 4 t + 2 s + u) with up to three pending
//     folds (nf; the previous launch's r1, r2, r3 bound in that order, r1 on the top variable) in the multilinear
//     form V_000 + sum_S r_S D_S (D_S: the differences of the 2^nf entries, r_S the products the host forms), half of
//     the products in lane g, half in lane g + 24 (the same instruction stream on selected operands), the halves
//     meeting in LDS; the corner goes back in place like the pair's; lane 48 loads the coefficient
//   points: the grid by tensor extension through LDS, one small-integer lerp per value: u (48 values: 16 per vector),
//     then s (96), then t (192: three per lane), instead of 7 lerps per value
// Sums over the workgroup's waves in LDS, over the workgroups by sc1 partials and a ticket (as the pair).
// ends (a layer's last triple, h = 1): the corner of q is also posted as scalar 64 + 24 c + q.
struct TripleArgs {
  const Triple* tr;
  const Fq* coeff;
  int nt;
  int log_len;  // round j's half length len = 2^log_len (>= 2: h = len / 4 >= 1)
  int nf;       // pending folds 0..3
  Fq r1, r2, r3, r12, r13, r23, r123;
  const Fq* cin;
  Fq* cout;
  Fq* partials;  // 64 per workgroup
  unsigned* counter;
  uint32_t* mb;
  uint32_t seq;
  int ends;
  unsigned long long* probe;
};
__device__ __forceinline__ Fq fq_lerp_small(const Fq& a, const Fq& b, int n) { return fq_add(a, fq_small(fq_sub(b, a), n)); }
__device__ __forceinline__ Fq lds_fq(const uint32_t* p) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = p[i];
  return r;
}
__device__ __forceinline__ void lds_put(uint32_t* p, const Fq& v) {
#pragma unroll
  for (int i = 0; i < 8; i++) p[i] = v.l[i];
}
template <int BS>
__global__ void __launch_bounds__(BS) k_layer_triple(TripleArgs A) {
  constexpr int NW = BS / 64;
  // per wave: corners (24) + coefficient, the folds' second halves (24), the u-extension (48), the s-extension (96)
  __shared__ uint32_t cs[NW][25][8], xs[NW][24][8], us[NW][48][8], ss[NW][96][8];
  __shared__ uint32_t es[NW > 1 ? NW : 1][64][8];
  __shared__ bool last;
  const int t = threadIdx.x, g = t & 63, wv = t >> 6;
  unsigned long long* pr = A.probe ? A.probe + 8 * blockIdx.x : nullptr;
  if (pr && t == 0) pr[0] = wall_clock64();
  const int len = 1 << A.log_len, h = len >> 2;
  const long total = (long)A.nt << (A.log_len - 2);
  const long u = (long)blockIdx.x * NW + wv;  // this wave's element (waves past the end contribute zero)
  const bool live = u < total;
  const int c = live ? (int)(u >> (A.log_len - 2)) : 0, i = (int)(u & (h - 1));
  const int q = g < 24 ? g : g - 24, part = g < 24 ? 0 : 1;  // lanes 0..47: corner q, half `part`
  const int v = q >> 3, m = q & 7, k = i + m * h;
  const int L2 = 2 * len;  // the folded vector's length: the pending folds' innermost stride
  Triple x;
  const Fq* src = nullptr;
  Fq w = fq_zero();
  if (live && g < 48) {
    x = A.tr[c];
    src = v == 0 ? x.A : (v == 1 ? x.B : (x.C ? x.C : A.cin));
    if (A.nf == 0) {
      if (!part) w = src[k];
    } else if (A.nf == 1) {
      if (!part) {
        const Fq a = src[k];
        w = fq_add(a, fq_mul(A.r1, fq_sub(src[k + L2], a)));
      }
    } else if (A.nf == 2) {  // V[2 a + b]: a bound by r1 (offset 2 L2), b by r2
      const Fq v00 = src[k], v01 = src[k + L2], v10 = src[k + 2 * L2], v11 = src[k + 3 * L2];
      const Fq d1 = fq_sub(v10, v00), d2 = fq_sub(v01, v00), d12 = fq_sub(fq_sub(v11, v10), d2);
      const Fq p0 = fq_mul(fq_sel(part, A.r12, A.r1), fq_sel(part, d12, d1));
      const Fq p1 = fq_mul(fq_sel(part, fq_zero(), A.r2), d2);
      w = fq_add(fq_sel(part, fq_zero(), v00), fq_add(p0, p1));
    } else {  // V[4 a + 2 b + c]: a by r1 (offset 4 L2), b by r2, c by r3
      Fq V[8];
#pragma unroll
      for (int j = 0; j < 8; j++) V[j] = src[k + j * L2];
      // the multilinear coefficients D_S (butterflies over the three bits)
#pragma unroll
      for (int bit = 1; bit < 8; bit <<= 1)
#pragma unroll
        for (int j = 0; j < 8; j++)
          if (j & bit) V[j] = fq_sub(V[j], V[j ^ bit]);
      // V[1] = D3, V[2] = D2, V[3] = D23, V[4] = D1, V[5] = D13, V[6] = D12, V[7] = D123
      const Fq p0 = fq_mul(fq_sel(part, A.r13, A.r1), fq_sel(part, V[5], V[4]));
      const Fq p1 = fq_mul(fq_sel(part, A.r23, A.r2), fq_sel(part, V[3], V[2]));
      const Fq p2 = fq_mul(fq_sel(part, A.r123, A.r3), fq_sel(part, V[7], V[1]));
      const Fq p3 = fq_mul(fq_sel(part, fq_zero(), A.r12), V[6]);
      w = fq_add(fq_add(fq_sel(part, fq_zero(), V[0]), p0), fq_add(p1, fq_add(p2, p3)));
    }
  }
  if (A.nf >= 2) {  // the second halves join the first
    if (live && part && g < 48) lds_put(xs[wv][q], w);
    __syncthreads();
    if (live && !part) w = fq_add(w, lds_fq(xs[wv][q]));
  }
  if (live && g < 24) {
    if (A.nf > 0) {
      Fq* dst = v == 0 ? x.A : (v == 1 ? x.B : (x.C ? x.C : (c == 0 ? A.cout : nullptr)));
      if (dst) dst[k] = w;
    }
    if (A.ends) host_put(A.mb + 8 + 8 * (64 + 24 * c + g), w);
    lds_put(cs[wv][g], w);
  } else if (live && g == 48) {
    lds_put(cs[wv][24], A.coeff[c]);
  }
  if (pr && t == 0) pr[1] = wall_clock64();
  __syncthreads();
  // u: value (vector g >> 4, t' = g & 1, s' = (g >> 1) & 1, u = (g >> 2) & 3) from corners 4 t' + 2 s' + {0, 1}
  if (g < 48) {
    const int vv = g >> 4, tt = g & 1, sp = (g >> 1) & 1, uu = (g >> 2) & 3, b = 8 * vv + 4 * tt + 2 * sp;
    lds_put(us[wv][g], fq_lerp_small(lds_fq(cs[wv][b]), lds_fq(cs[wv][b + 1]), uu));
  }
  __syncthreads();
  // s: value (vector idx >> 5, t' = idx & 1, s = (idx >> 1) & 3, u = (idx >> 3) & 3), idx = g and g + 64 (< 96)
#pragma unroll
  for (int rep = 0; rep < 2; rep++) {
    const int idx = g + 64 * rep;
    if (idx < 96) {
      const int vv = idx >> 5, tt = idx & 1, sv = (idx >> 1) & 3, uu = (idx >> 3) & 3;
      const int b = 16 * vv + tt + 4 * uu;  // us index of (vv, tt, s' = 0, uu); s' = 1 is b + 2
      lds_put(ss[wv][idx], fq_lerp_small(lds_fq(us[wv][b]), lds_fq(us[wv][b + 2]), sv));
    }
  }
  __syncthreads();
  if (pr && t == 0) pr[2] = wall_clock64();
  // t: this lane's point (t, s, u) = (g & 3, (g >> 2) & 3, g >> 4) for the three vectors, then k A B C
  Fq e = fq_zero();
  if (live) {
    const int tt = g & 3, b = 2 * ((g >> 2) & 3) + 8 * (g >> 4);  // ss index of (v, t' = 0, s, u), minus 32 v
    const Fq av = fq_lerp_small(lds_fq(ss[wv][b]), lds_fq(ss[wv][b + 1]), tt);
    const Fq bv = fq_lerp_small(lds_fq(ss[wv][32 + b]), lds_fq(ss[wv][33 + b]), tt);
    const Fq cv = fq_lerp_small(lds_fq(ss[wv][64 + b]), lds_fq(ss[wv][65 + b]), tt);
    e = fq_mul(fq_mul(av, bv), fq_mul(lds_fq(cs[wv][24]), cv));
  }
  if (A.ends) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // the corners reach the host before any ticket / post
  if (pr && t == 0) pr[3] = wall_clock64();
  if (NW > 1) {
    lds_put(es[wv][g], e);
    __syncthreads();
    if (wv == 0)
      for (int o = 1; o < NW; o++) e = fq_add(e, lds_fq(es[o][g]));
  }
  if (gridDim.x == 1) {  // wave 0 posts the 64 point sums, then lane 0 the sequence number
    if (t < 64) {
      host_put(A.mb + 8 + 8 * t, e);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    __syncthreads();
    if (t == 0) {
      __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (pr) pr[4] = wall_clock64();
    }
    return;
  }
  if (t < 64) st_sc1(&A.partials[64 * blockIdx.x + t], e);
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(A.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  // the last workgroup: wave w adds the partials of workgroups w, w + NW, ..., four loads in flight at a time
  Fq s0 = fq_zero(), s1 = fq_zero();
  unsigned j = wv;
  for (; j + 3 * NW < gridDim.x; j += 4 * NW) {
    const Fq a0 = ld_sc1(&A.partials[64 * j + g]), a1 = ld_sc1(&A.partials[64 * (j + NW) + g]);
    const Fq a2 = ld_sc1(&A.partials[64 * (j + 2 * NW) + g]), a3 = ld_sc1(&A.partials[64 * (j + 3 * NW) + g]);
    s0 = fq_add(s0, fq_add(a0, a1));
    s1 = fq_add(s1, fq_add(a2, a3));
  }
  for (; j < gridDim.x; j += NW) s0 = fq_add(s0, ld_sc1(&A.partials[64 * j + g]));
  Fq sum = fq_add(s0, s1);
  if (NW > 1) {
    lds_put(es[wv][g], sum);
    __syncthreads();
    if (wv == 0)
      for (int o = 1; o < NW; o++) sum = fq_add(sum, lds_fq(es[o][g]));
  }
  if (t < 64) {
    host_put(A.mb + 8 + 8 * t, sum);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
  __syncthreads();
  if (t == 0) {
    __hip_atomic_store(A.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(A.mb, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- persistent form: the remaining rounds of a layer in one launch ------------------------------------------------
// A launched round costs a host launch (~4 us) and a doorbell-to-first-wave delay (~5 us) on top of its work, and the
// layer rounds are transcript-sequential. Here the workgroups stay resident over the rounds: after posting round k's
// (e0, e2, e3) they wait for the host's answer in the downbox (coherent host memory: the round's challenge, then its
// mailbox sequence number), fold with it and go on. Entries written in one round are read by other workgroups in the
// next, so every access to the vectors inside the launch is an `sc1` access (agent-scope relaxed atomics: L1 bypassed,
// written through) and each workgroup drains its stores before its ticket (MI355X_MICROARCH hand-off table, row 1;
// the host's answer comes only after the last ticket). The layer's last round posts every vector's two entries from
// the workgroup that takes the last ticket, so the host folds the final claims itself. Every wave leaves the loop on
// the last round, on the host's abort word, or after `timeout` ticks without an answer.
__device__ __forceinline__ Fq fold_at_sc1(const Fq* p, int k, int fl, const Fq& r) {
  const Fq lo = ld_sc1(p + k);
  return fq_add(lo, fq_mul(r, fq_sub(ld_sc1(p + k + fl), lo)));
}
// layer_round_elems with sc1 accesses
__device__ __forceinline__ Fq layer_round_elems_sc1(const Triple* __restrict__ tr, const Fq* __restrict__ coeff, int nt,
                                                    int log_len, int do_fold, const Fq& r, const Fq* cin, Fq* cout,
                                                    long u0, long ustride) {
  const int q = threadIdx.x & 3, len = 1 << log_len;
  const int pt = q < 3 ? q : 0;
  const long total = (long)nt << log_len;
  Fq e = fq_zero();
  for (long u = u0; u < total; u += ustride) {
    const int c = (int)(u >> log_len), i = (int)(u & (len - 1));
    const Triple x = tr[c];
    const Fq* Cp = x.C ? x.C : cin;
    const Fq* src = pt == 0 ? x.A : (pt == 1 ? x.B : Cp);
    Fq lo, hi;
    if (do_fold) {
      const int fl = 2 * len;
      lo = fold_at_sc1(src, i, fl, r);
      hi = fold_at_sc1(src, i + len, fl, r);
      Fq* dst = q == 0 ? x.A : (q == 1 ? x.B : (q == 2 ? (x.C ? x.C : (c == 0 ? cout : nullptr)) : nullptr));
      if (dst) {
        st_sc1(dst + i, lo);
        st_sc1(dst + i + len, hi);
      }
    } else {
      lo = ld_sc1(src + i);
      hi = ld_sc1(src + i + len);
    }
    const Fq al = fq_qbcast<0>(lo), ah = fq_qbcast<0>(hi), bl = fq_qbcast<1>(lo), bh = fq_qbcast<1>(hi);
    const Fq cl = fq_qbcast<2>(lo), ch = fq_qbcast<2>(hi);
    const Fq k = coeff[c];
    e = fq_add(e, fq_mul(fq_mul(fq_mul(line_at(al, ah, pt), line_at(bl, bh, pt)), line_at(cl, ch, pt)), k));
  }
  return e;
}
struct PersistArgs {
  const Triple* tr;
  const Fq* coeff;
  int nt;
  int rounds;        // rounds in this launch: round k works on vectors of half length 2^(rounds - 1 - k)
  int do_fold;       // the first round applies the fold pending from the round before the launch
  Fq r;              // ... with this challenge
  Fq* cb[2];         // the shared eq vector's ping-pong pair; cb[cur] holds it
  int cur;
  Fq* partials;
  unsigned* counter;
  uint32_t* mb;
  uint32_t seq0;     // mailbox sequence number of round 0 (round k: seq0 + k)
  uint32_t* down;    // the host's answers
  int ends;          // the last round posts every vector's two entries after the sums (3 + 6 nt scalars)
  unsigned long long timeout;  // wall_clock64 ticks a workgroup waits for an answer before it gives up
  uint32_t* relay;   // non-null: workgroup 0 alone polls the host and copies each answer here (HBM: [0] sequence
                     // number, [8..15] challenge) for the others, instead of every workgroup reading host memory
};
static const uint32_t kDownAbortDev = 0xffffffffu;  // = kDownAbort (ctx.hpp)
template <int BS>
__global__ void __launch_bounds__(BS) k_layer_persist(PersistArgs A) {
  __shared__ bool last;
  __shared__ uint32_t rsh[9];
  const int t = threadIdx.x, q = t & 3;
  int do_fold = A.do_fold, cur = A.cur;
  Fq r = A.r;
  for (int k = 0; k < A.rounds; k++) {
    const int lg = A.rounds - 1 - k;
    const uint32_t seq = A.seq0 + (uint32_t)k;
    Fq* cin = A.cb[cur];
    Fq* cout = A.cb[cur ^ 1];
    Fq e = layer_round_elems_sc1(A.tr, A.coeff, A.nt, lg, do_fold, r, cin, cout, ((long)blockIdx.x * BS + t) >> 2,
                                 (long)gridDim.x * (BS / 4));
    if (do_fold) cur ^= 1;
    quad_block_sum<BS>(e);
    if (t < 3)
      for (int j = 0; j < 8; j++)
        __hip_atomic_store(&A.partials[3 * blockIdx.x + t].l[j], e.l[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its vector and partial stores are out
    __syncthreads();
    if (t == 0)
      last = __hip_atomic_fetch_add(A.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (last) {
      Fq a = fq_zero();
      if (q < 3)
        for (unsigned j = t >> 2; j < gridDim.x; j += BS / 4) {
          Fq o;
          for (int i = 0; i < 8; i++)
            o.l[i] = __hip_atomic_load(&A.partials[3 * j + q].l[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          a = fq_add(a, o);
        }
      quad_block_sum<BS>(a);
      if (lg == 0 && A.ends) {  // every vector's entries 0 and 1 (this round's folded values; C in cb[cur])
        for (int u = t; u < 3 * A.nt; u += BS) {
          const int c = u / 3, p = u % 3;
          const Triple x = A.tr[c];
          const Fq* v = p == 0 ? x.A : (p == 1 ? x.B : (x.C ? x.C : A.cb[cur]));
          const Fq lo = ld_sc1(v), hi = ld_sc1(v + 1);
          uint32_t* d = A.mb + 8 + 8 * (3 + 6 * c + 2 * p);
          host_put(d, lo);
          host_put(d + 8, hi);
        }
      }
      if (t < 3)
        host_put(A.mb + 8 + 8 * t, a);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __syncthreads();
      if (t == 0) {
        __hip_atomic_store(A.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ticket is re-armed before the host can answer
        __hip_atomic_store(A.mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (lg == 0) return;  // the layer's last round: nothing to wait for
    if (t == 0) {  // one lane per workgroup polls the downbox (or, relayed, workgroup 0's copy in HBM)
      const bool host = !A.relay || blockIdx.x == 0;
      uint32_t* src = host ? A.down : A.relay;
      const unsigned long long t0 = wall_clock64();
      uint32_t v;
      uint32_t ok = 1;
      while ((v = host ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                       : __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != seq) {
        if (v == kDownAbortDev || v == (seq | 0x80000000u) || wall_clock64() - t0 > A.timeout) {
          ok = 0;
          break;
        }
        if (host) __builtin_amdgcn_s_sleep(8);
        else __builtin_amdgcn_s_sleep(1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the challenge is read after the matching sequence number
      if (ok)
        for (int i = 0; i < 8; i++)
          rsh[i] = host ? __hip_atomic_load(src + 8 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                        : __hip_atomic_load(src + 8 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      rsh[8] = ok;
      if (A.relay && blockIdx.x == 0) {  // the others' copy: challenge, drained, then the number (or the abort word)
        if (ok)
          for (int i = 0; i < 8; i++) __hip_atomic_store(A.relay + 8 + i, rsh[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // (this round's abort word: a stale value of an earlier launch never equals it)
        __hip_atomic_store(A.relay, ok ? seq : (seq | 0x80000000u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
    if (!rsh[8]) return;
    for (int i = 0; i < 8; i++) r.l[i] = rsh[i];
    do_fold = 1;
    __syncthreads();  // rsh and `last` are rewritten in the next round
  }
}

// ---- big rounds: one thread per index i over every product circuit (throughput form) -----------------------------
// Triples 0 .. np-1 share the eq vector C (cin -> cout); since e_X = sum_i C_i(X) sum_c k_c A_c(X) B_c(X), the
// thread for index i folds C once, then per circuit folds A and B, scales A's two entries by k_c and adds the three
// products A(X) B(X) (X = 0, 2, 3); C(X) multiplies the sums once. Triples np .. nt-1 (dot-product circuits, own C)
// take one thread per (triple, i). About 9 products per circuit and index instead of the quad form's 20 lane
// products, for rounds large enough to fill the chip; the reduction (block sums, ticket, mailbox) is k_layer_round's.
template <int BS>
__global__ void __launch_bounds__(BS) k_layer_round_wide(const Triple* __restrict__ tr, const Fq* __restrict__ coeff,
                                                         int np, int nt, int log_len, int do_fold, Fq r,
                                                         const Fq* __restrict__ cin, Fq* __restrict__ cout,
                                                         Fq* __restrict__ partials, unsigned* __restrict__ counter,
                                                         uint32_t* __restrict__ mb, uint32_t seq) {
  const int t = threadIdx.x, len = 1 << log_len;
  const int ng = (np > 0 ? 1 : 0) + (nt - np);
  const long total = (long)ng << log_len;
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  auto load2 = [&](const Fq* p, Fq* w, int i, Fq& lo, Fq& hi) {
    if (do_fold) {
      lo = fold_at(p, i, 2 * len, r);
      hi = fold_at(p, i + len, 2 * len, r);
      if (w) {
        w[i] = lo;
        w[i + len] = hi;
      }
    } else {
      lo = p[i];
      hi = p[i + len];
    }
  };
  for (long u = (long)blockIdx.x * BS + t; u < total; u += (long)gridDim.x * BS) {
    const int g = (int)(u >> log_len), i = (int)(u & (len - 1));
    if (np > 0 && g == 0) {
      Fq cl, ch;
      load2(cin, cout, i, cl, ch);
      Fq s0 = fq_zero(), s2 = fq_zero(), s3 = fq_zero();
      for (int c = 0; c < np; c++) {
        const Triple x = tr[c];
        const Fq k = coeff[c];
        Fq al, ah, bl, bh;
        load2(x.A, x.A, i, al, ah);
        load2(x.B, x.B, i, bl, bh);
        al = fq_mul(k, al);
        ah = fq_mul(k, ah);
        const Fq da = fq_sub(ah, al), db = fq_sub(bh, bl);
        const Fq a2 = fq_add(ah, da), b2 = fq_add(bh, db);
        s0 = fq_add(s0, fq_mul(al, bl));
        s2 = fq_add(s2, fq_mul(a2, b2));
        s3 = fq_add(s3, fq_mul(fq_add(a2, da), fq_add(b2, db)));
      }
      const Fq dc = fq_sub(ch, cl), c2 = fq_add(ch, dc);
      e0 = fq_add(e0, fq_mul(s0, cl));
      e2 = fq_add(e2, fq_mul(s2, c2));
      e3 = fq_add(e3, fq_mul(s3, fq_add(c2, dc)));
    } else {
      const int c = np + g - (np > 0 ? 1 : 0);
      const Triple x = tr[c];
      const Fq k = coeff[c];
      Fq al, ah, bl, bh, cl, ch;
      load2(x.A, x.A, i, al, ah);
      load2(x.B, x.B, i, bl, bh);
      load2(x.C, x.C, i, cl, ch);
      al = fq_mul(k, al);
      ah = fq_mul(k, ah);
      const Fq da = fq_sub(ah, al), db = fq_sub(bh, bl), dc = fq_sub(ch, cl);
      const Fq a2 = fq_add(ah, da), b2 = fq_add(bh, db), c2 = fq_add(ch, dc);
      e0 = fq_add(e0, fq_mul(fq_mul(al, bl), cl));
      e2 = fq_add(e2, fq_mul(fq_mul(a2, b2), c2));
      e3 = fq_add(e3, fq_mul(fq_mul(fq_add(a2, da), fq_add(b2, db)), fq_add(c2, dc)));
    }
  }
  block_sum3_t0<BS>(e0, e2, e3);
  __shared__ bool last;
  if (t == 0) {
    partials[3 * blockIdx.x] = e0;
    partials[3 * blockIdx.x + 1] = e2;
    partials[3 * blockIdx.x + 2] = e3;
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
  Fq a = fq_zero(), b = fq_zero(), cc = fq_zero();
  for (unsigned j = t; j < gridDim.x; j += BS) {
    a = fq_add(a, partials[3 * j]);
    b = fq_add(b, partials[3 * j + 1]);
    cc = fq_add(cc, partials[3 * j + 2]);
  }
  block_sum3_t0<BS>(a, b, cc);
  if (t == 0) {
    mbox_post3(mb, seq, a, b, cc);
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace spg
