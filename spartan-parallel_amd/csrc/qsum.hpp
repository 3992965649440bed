// spg — block and grid sums of quad-split values: lane q of each quad (4 lanes) holds its share of value q, the
// block's sums meet by cross-quad shuffles inside each wave, then across waves in LDS, and a grid's workgroups hand
// theirs over by sc1 stores and a ticket (the layer rounds of layer.hpp and the quad sumcheck evaluations).
#pragma once
#include <hip/hip_runtime.h>

#include "ctx.hpp"

namespace spg {

__device__ __forceinline__ Fq fq_shfl_xor(const Fq& a, int m) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = (uint32_t)__shfl_xor((int)a.l[i], m);
  return r;
}
// value at X = 0, 2, 3 (p = 0, 1, 2) of the line through (0, lo), (1, hi)
__device__ __forceinline__ Fq line_at(const Fq& lo, const Fq& hi, int p) {
  const Fq d = fq_sub(hi, lo), x2 = fq_add(hi, d);
  return p == 0 ? lo : (p == 1 ? x2 : fq_add(x2, d));
}
// sums of the values of lanes with equal (thread & 3) over a block of BS threads: quads of a wave by
// cross-quad shuffles, then waves through LDS; the sum for q is left in thread q (q < 3)
template <int BS>
__device__ __forceinline__ void quad_block_sum(Fq& e) {
  constexpr int NW = BS / 64;
  __shared__ uint32_t wsum[NW > 1 ? NW : 1][3][8];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int m = 4; m < 64; m <<= 1) e = fq_add(e, fq_shfl_xor(e, m));
  if (NW > 1) {
    if (lane < 3)
      for (int j = 0; j < 8; j++) wsum[w][lane][j] = e.l[j];
    __syncthreads();
    if (w == 0 && lane < 3)
      for (int v = 1; v < NW; v++) {
        Fq o;
        for (int j = 0; j < 8; j++) o.l[j] = wsum[v][lane][j];
        e = fq_add(e, o);
      }
    __syncthreads();
  }
}
// The grid's sums of a quad kernel: value q (< 3) of every lane with (thread & 3) == q over all workgroups, posted
// to the host mailbox as one round's (e0, e2, e3). One workgroup posts directly; more store their partials
// write-through (sc1), drain them, take a ticket, and the last one adds them (sc1 loads) and posts -- no L2
// write-back fence on the way (MI355X_MICROARCH hand-off table, row 1).
template <int BS>
__device__ __forceinline__ void quad_grid_post(Fq e, Fq* __restrict__ partials, unsigned* __restrict__ counter,
                                               uint32_t* __restrict__ mb, uint32_t seq) {
  __shared__ bool last;
  const int t = threadIdx.x, q = t & 3;
  quad_block_sum<BS>(e);
  if (gridDim.x == 1) {  // lanes 0..2 of wave 0 post e0, e2, e3, then lane 0 the sequence number
    if (t < 3) {
      host_put(mb + 8 + 8 * t, e);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    if (t == 0) __hip_atomic_store(mb, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (t < 3) st_sc1(&partials[3 * blockIdx.x + t], e);
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  Fq a = fq_zero();
  if (q < 3)
    for (unsigned j = t >> 2; j < gridDim.x; j += BS / 4) a = fq_add(a, ld_sc1(&partials[3 * j + q]));
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

}  // namespace spg
