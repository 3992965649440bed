// spg — quad-cooperative point arithmetic (4 lanes per point) for the latency-path MSM kernels (msm.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "curve.hpp"
#include "lds.hpp"

namespace spg {

// ---- quad-cooperative point arithmetic for the latency path --------------------------------------
// The four lanes of a quad hold the same point and split each addition's field products between them:
// product round 1 gives lane r one of A, B, C, D of add-2008-hwcd-3 (for P + Q scaled by a small constant,
// see quad_add), round 2 gives lane r one of X3, Y3, T3, Z3; DPP quad permutations exchange the products.
// The dependent chain of an addition drops from 10 (mixed: 7) field multiplications to 2 plus a small-constant
// product (mixed: 2). The group element, so its encoding, is the one ext_add / ext_madd compute.
template <int K>
__device__ __forceinline__ Fp fp_qbcast(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], K * 0x55, 0xf, 0xf, false);
  return r;
}
__device__ __forceinline__ Fp fp_sel(bool c, const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}
// lane q holds product q of (A, B, C, D); returns the sum point on every lane of the quad
// X3 = E F (lane 0), Y3 = G H (1), T3 = E H (2), Z3 = F G (3), broadcast to the quad
__device__ __forceinline__ Ext quad_out(const Fp& E, const Fp& F, const Fp& G, const Fp& H, int q) {
  const Fp u = fp_sel(q == 0 || q == 2, E, fp_sel(q == 1, G, F));
  const Fp v = fp_sel(q == 0, F, fp_sel(q == 3, G, H));
  const Fp w = fp_mul(u, v);
  Ext r;
  r.X = fp_qbcast<0>(w);
  r.Y = fp_qbcast<1>(w);
  r.T = fp_qbcast<2>(w);
  r.Z = fp_qbcast<3>(w);
  return r;
}
// DPP quad permutation: lane r of each quad reads lane (CTRL >> 2r) & 3 of its quad
template <int CTRL>
__device__ __forceinline__ Fp fp_qperm(const Fp& a) {
  Fp r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], CTRL, 0xf, 0xf, false);
  return r;
}
// second product round of add-2008-hwcd-3: lane r holds p_r in (A, B, C, D) (cneg: the true C is -p_2).
// E = B - A, F = D - C, G = D + C, H = B + A; lane 0 forms X3 = E F, 1 Y3 = G H, 2 T3 = E H, 3 Z3 = F G, so
// every lane needs two of them: u in (E, G, E, F) and v in (F, H, H, G), each one add-or-subtract of two
// gathered products (quad_perm [1,3,1,3] / [0,2,0,2] and [3,1,1,3] / [2,0,0,2]).
__device__ __forceinline__ Ext quad_finish(const Fp& p, int q, bool cneg) {
  const Fp uA = fp_qperm<0xDD>(p), uB = fp_qperm<0x88>(p);
  const Fp vA = fp_qperm<0xD7>(p), vB = fp_qperm<0x82>(p);
  const bool usub = q == 1 ? cneg : (q == 3 ? !cneg : true);
  const bool vsub = q == 0 ? !cneg : (q == 3 ? cneg : false);
  const Fp w = fp_mul(fp_addsub(uA, uB, usub), fp_addsub(vA, vB, vsub));
  Ext r;
  r.X = fp_qbcast<0>(w);
  r.Y = fp_qbcast<1>(w);
  r.T = fp_qbcast<2>(w);
  r.Z = fp_qbcast<3>(w);
  return r;
}
// lane q's first-round operand of P: Y - X, Y + X, T, Z
__device__ __forceinline__ Fp quad_operand(const Ext& P, int q) {
  return q < 2 ? fp_addsub(P.Y, P.X, q == 0) : (q == 2 ? P.T : P.Z);
}
// the Niels coordinate lane q of a quad needs for table entry ent (index | neg << 31): lane 0 the "minus" one
// (neg ? ypx : ymx), lane 1 the "plus" one, lanes 2, 3 t2d; one 32-byte load per lane
// (st: the table's entry stride in 32-byte coordinates, 3 for packed 96-byte entries, 4 for the comb tables padded
// to one 128-byte line per entry)
__device__ __forceinline__ Fp niels_coord(const Niels* __restrict__ tab, uint32_t ent, int q, bool* neg, int st = 3) {
  *neg = ent >> 31;
  const int which = q >= 2 ? 2 : ((q == 0) != *neg ? 1 : 0);  // Niels field order: ypx, ymx, t2d
  return reinterpret_cast<const Fp*>(tab)[(size_t)(ent & 0x7fffffffu) * st + which];
}
// table entry (index | sign << 31) as an extended point, negated when the sign bit is set
__device__ __forceinline__ Ext load_signed(const Niels* __restrict__ tab, uint32_t e) {
  Niels q = tab[e & 0x7fffffffu];
  if (e >> 31) {
    Fp t = q.ypx;
    q.ypx = q.ymx;
    q.ymx = t;
    q.t2d = fp_neg(q.t2d);
  }
  return niels_to_ext(q);
}
// P + (+-Niels); qv is this lane's Niels coordinate: lane 0 the "minus" one (neg ? ypx : ymx), lane 1 the
// "plus" one (neg ? ymx : ypx), lane 2 t2d (lane 3 ignores it); -Q has C negated (cneg)
__device__ __forceinline__ Ext quad_madd(const Ext& P, const Fp& qv, bool neg, int q) {
  const Fp y = q == 3 ? fp_small(2) : qv;
  return quad_finish(fp_mul(quad_operand(P, q), y), q, neg);
}
// P + Q given lane q's first-round operand of Q (quad_operand(Q, q)), scaled as quad_add below
__device__ __forceinline__ Ext quad_add_op(const Ext& P, const Fp& qop, int q) {
  const Fp p = fp_mul(quad_operand(P, q), qop);
  const uint32_t k = q == 2 ? 243330u : (q == 3 ? 243332u : 121666u);
  return quad_finish(fp_mul_k(p, k), q, true);
}
// P + Q with A, B, C, D all scaled by 121666 (so E..H scale alike and the sum is the same projective point,
// its coordinates 121666^2 times ext_add's): C = 2d T1 T2 becomes -243330 T1 T2 since 2d = -2 * 121665 / 121666,
// a small constant like 121666 (A, B) and 243332 (D = 2 Z1 Z2): one full product round fewer than 2d T1 T2.
__device__ __forceinline__ Ext quad_add(const Ext& P, const Ext& Q, int q) {
  const Fp p = fp_mul(quad_operand(P, q), quad_operand(Q, q));
  const uint32_t k = q == 2 ? 243330u : (q == 3 ? 243332u : 121666u);
  return quad_finish(fp_mul_k(p, k), q, true);
}

// 2P (dbl-2008-hwcd as ext_dbl): lane q squares X, Y, Z, X + Y
__device__ __forceinline__ Ext quad_dbl(const Ext& P, int q) {
  const Fp x = fp_sel(q == 0, P.X, fp_sel(q == 1, P.Y, fp_sel(q == 2, P.Z, fp_add(P.X, P.Y))));
  const Fp p = fp_mul(x, x);
  const Fp A = fp_qbcast<0>(p), B = fp_qbcast<1>(p), ZZ = fp_qbcast<2>(p), SS = fp_qbcast<3>(p);
  const Fp C = fp_add(ZZ, ZZ);
  const Fp E = fp_sub(fp_sub(SS, A), B), G = fp_sub(B, A);
  return quad_out(E, fp_sub(G, C), G, fp_neg(fp_add(A, B)), q);
}
// a quad's point into a component-major LDS slot (lane q stores coordinate q: X, Y, Z, T)
template <int SL>
__device__ __forceinline__ void quad_put(uint32_t* sh, int slot, const Ext& P, int q) {
  const Fp c = fp_sel(q == 0, P.X, fp_sel(q == 1, P.Y, fp_sel(q == 2, P.Z, P.T)));
#pragma unroll
  for (int i = 0; i < 8; i++) sh[(q * 8 + i) * SL + slot] = c.l[i];
}

// tree / scan hand-offs through LDS carry first-round operands: the giving quad's lane q stores
// quad_operand(P, q) (component-major slot), the receiving quad's lane q reads only its own 8 words
template <int SL>
__device__ __forceinline__ void quad_put_op(uint32_t* sh, int slot, const Ext& P, int q) {
  const Fp c = quad_operand(P, q);
#pragma unroll
  for (int i = 0; i < 8; i++) sh[(q * 8 + i) * SL + slot] = c.l[i];
}
template <int SL>
__device__ __forceinline__ Fp quad_get_op(const uint32_t* sh, int slot, int q) {
  Fp c;
#pragma unroll
  for (int i = 0; i < 8; i++) c.l[i] = sh[(q * 8 + i) * SL + slot];
  return c;
}

}  // namespace spg
