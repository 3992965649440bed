// spg — helpers of the multi-round launches (k_layer_pair / k_layer_triple in layer.hpp, k_phase1_pair in
// sumcheck.hip): DPP row broadcasts, small-integer multiples, the 2 x 2 cube's multilinear extension, row sums.
#pragma once
#include <hip/hip_runtime.h>

#include "ctx.hpp"
#include "qsum.hpp"

namespace spg {

template <int N>
__device__ __forceinline__ Fq fq_rowbcast(const Fq& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], 0x150 + N, 0xf, 0xf, false);
  return r;
}
// word-wise select (no scratch: a select of whole structs put the quad kernels' values in private memory)
__device__ __forceinline__ Fq fq_sel(bool c, const Fq& a, const Fq& b) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}
// n x (n in 0..3, lane-varying)
__device__ __forceinline__ Fq fq_small(const Fq& x, int n) {
  const Fq x2 = fq_add(x, x), x3 = fq_add(x2, x);
  return fq_sel(n == 3, x3, fq_sel(n == 2, x2, fq_sel(n == 1, x, fq_zero())));
}
// P(t, s) from the corners (p00, p01, p10, p11)
__device__ __forceinline__ Fq cube_at(const Fq& p00, const Fq& p01, const Fq& p10, const Fq& p11, int t, int s) {
  const Fq ds = fq_sub(p01, p00), dt = fq_sub(p10, p00), dd = fq_sub(fq_sub(p11, p10), ds);
  const Fq base = fq_add(p00, fq_small(ds, s)), slope = fq_add(dt, fq_small(dd, s));
  return fq_add(base, fq_small(slope, t));
}
// sums of the values of lanes with equal (thread & 15) over a block of BS threads; the sum for g is left in thread g
template <int BS>
__device__ __forceinline__ void row_block_sum(Fq& e) {
  constexpr int NW = BS / 64;
  __shared__ uint32_t wsum[NW > 1 ? NW : 1][16][8];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  e = fq_add(e, fq_shfl_xor(e, 16));
  e = fq_add(e, fq_shfl_xor(e, 32));
  if (NW > 1) {
    if (lane < 16)
      for (int j = 0; j < 8; j++) wsum[w][lane][j] = e.l[j];
    __syncthreads();
    if (w == 0 && lane < 16)
      for (int v = 1; v < NW; v++) {
        Fq o;
        for (int j = 0; j < 8; j++) o.l[j] = wsum[v][lane][j];
        e = fq_add(e, o);
      }
    __syncthreads();
  }
}
}  // namespace spg
