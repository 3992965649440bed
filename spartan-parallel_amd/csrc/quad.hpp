// spg — quad-cooperative point arithmetic (4 lanes per point) for the latency-path MSM kernels (msm.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "curve.hpp"
#include "lds.hpp"

namespace spg {

// ---- quad-cooperative point arithmetic for the latency path --------------------------------------
// The four lanes of a quad hold the same point and split each addition's field products between them:
// product round 1 gives lane r one of A, B, C', D of add-2008-hwcd-3, round 2 scales C' by 2d (lane 2),
// round 3 gives lane r one of X3, Y3, T3, Z3; DPP quad broadcasts exchange the products. The dependent chain
// of an addition drops from 10 (mixed: 7) field multiplications to 3 (2); every formula and value is the one
// ext_add / ext_madd compute, so the group element (and its encoding) is identical.
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
__device__ __forceinline__ Ext quad_finish(const Fp& p, int q) {
  const Fp A = fp_qbcast<0>(p), B = fp_qbcast<1>(p), C = fp_qbcast<2>(p), D = fp_qbcast<3>(p);
  return quad_out(fp_sub(B, A), fp_sub(D, C), fp_add(D, C), fp_add(B, A), q);
}
// P + (+-Niels); qv is this lane's Niels coordinate: lane 0 the "minus" one (neg ? ypx : ymx), lane 1 the
// "plus" one (neg ? ymx : ypx), lane 2 t2d (lane 3 ignores it)
__device__ __forceinline__ Ext quad_madd(const Ext& P, const Fp& qv, bool neg, int q) {
  const Fp x = fp_sel(q == 0, fp_sub(P.Y, P.X), fp_sel(q == 1, fp_add(P.Y, P.X), fp_sel(q == 2, P.T, P.Z)));
  const Fp y = fp_sel(q == 3, fp_small(2), qv);
  Fp p = fp_mul(x, y);
  p = fp_sel(neg && q == 2, fp_neg(p), p);
  return quad_finish(p, q);
}
__device__ __forceinline__ Ext quad_add(const Ext& P, const Ext& Q, int q) {
  const Fp x = fp_sel(q == 0, fp_sub(P.Y, P.X), fp_sel(q == 1, fp_add(P.Y, P.X), fp_sel(q == 2, P.T, P.Z)));
  const Fp y = fp_sel(q == 0, fp_sub(Q.Y, Q.X), fp_sel(q == 1, fp_add(Q.Y, Q.X), fp_sel(q == 2, Q.T, Q.Z)));
  Fp p = fp_mul(x, y);
  const Fp pd = fp_mul(p, c_d2());  // C = 2d T1 T2 (lane 2)
  p = fp_sel(q == 2, pd, fp_sel(q == 3, fp_add(p, p), p));  // D = 2 Z1 Z2 (lane 3)
  return quad_finish(p, q);
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

}  // namespace spg
