// spg — generators and multi-scalar multiplication on MI355X (gfx950).
//
// Replaces GroupElement::vartime_multiscalar_mul (src/group.rs:98-116), Commitments::commit
// (src/commitments.rs:69-92), DensePolynomial::commit_inner (src/dense_mlpoly.rs:184-212) and
// MultiCommitGens::new (src/commitments.rs:15-33).
//
// Design (all commitment bases in Spartan are fixed generator sets, so the MSM is fixed-base):
//   * Every spg_gens keeps, resident in HBM, table[k][i] = 2^k * P_i in affine Niels form for all
//     bit offsets k < 254 (96 B per entry). A c-bit signed-digit window w of a scalar then selects
//     table[w*c][i] directly, so all windows of all scalars of one MSM share ONE bucket set of
//     2^(c-1) buckets and no per-window doublings are needed.
//   * Pipeline per batch of B MSMs (B Hyrax rows, or B = 1):
//       k_count   : Montgomery -> canonical, signed c-bit digits, histogram of (msm, |digit|)
//       scan      : exclusive prefix sums (hipCUB) of counts and of ceil(count / K) work items
//       k_scatter : counting-sort scatter of (table index | sign) into bucket order
//       k_items   : one thread per K-entry slice of a bucket: mixed Niels additions (7M each)
//       k_segments: running sums over 8-bucket segments (sum v * B_v = sum_j T_j + j*m*S_j)
//       k_final   : one block per MSM folds its segments (per-thread groups, LDS suffix scan + tree), encodes
//     Skewed scalar distributions (0/1-heavy witnesses) only lengthen the item list, never a thread.
#include <hipcub/hipcub.hpp>

#include <string.h>

#include <vector>

#include "ctx.hpp"
#include "hcurve.hpp"
#include "host.hpp"
#include "keccak.hpp"
#include "lds.hpp"
#include "bullet.hpp"
#include "quad.hpp"

namespace spg {

static const int kItemK = 16;  // entries summed per work item
static const int kSegM = 8;    // buckets per running-sum segment (k_segments)
static const size_t kSmallMaxB = 4;       // latency path: at most this many MSMs per call ...
static const size_t kSmallMaxN = 16384;   // ... of at most this many points each

// ------------------------------------------------------------------ generators
__global__ void k_map_uniform(const uint8_t* __restrict__ uni, Niels* __restrict__ out, uint8_t* __restrict__ comp,
                              int n1) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n1) return;
  uint8_t b[64];
  for (int k = 0; k < 64; k++) b[k] = uni[64 * (size_t)i + k];
  Ext P = ristretto_from_uniform_bytes(b);
  out[i] = ext_to_niels(P);
  uint8_t c[32];
  ext_compress(P, c);
  for (int k = 0; k < 32; k++) comp[32 * (size_t)i + k] = c[k];
}

__global__ void k_decompress(const uint8_t* __restrict__ comp, Niels* __restrict__ out, int* __restrict__ bad,
                             int n1) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n1) return;
  uint8_t c[32];
  for (int k = 0; k < 32; k++) c[k] = comp[32 * (size_t)i + k];
  Ext P;
  if (!ext_decompress(c, P)) {
    atomicExch(bad, 1);
    P = ext_identity();
  }
  out[i] = ext_to_niels(P);
}

__global__ void k_table(const Niels* __restrict__ base, Niels* __restrict__ tab, int n1) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)n1 * kTableRows) return;
  int k = (int)(t / n1), g = (int)(t % n1);
  Ext P = niels_to_ext(base[g]);
  for (int j = 0; j < k; j++) P = ext_dbl(P);
  tab[t] = ext_to_niels(P);
}

// ------------------------------------------------------------------ MSM kernels
struct MsmArgs {
  const Fq* scalars;  // B x n (Montgomery)
  const Fq* blinds;   // B or null
  int B, n, n1;       // n scalars per MSM, n1 = gens count incl. h
  int gen_offset;     // generator index of scalar 0
  int h_index;        // generator index of h
  const uint32_t* idx;  // optional: explicit generator index per scalar (B x n), overrides gen_offset
  uint32_t* hist;     // B*NB
  const uint32_t* off;
  uint32_t* off_out;  // k_digits_rows: writes the bucket offsets itself
  uint32_t* cursor;
  uint32_t* entries;
};

// canonical limbs of a Montgomery scalar (Scalar::to_bytes / decompress_scalar, src/scalar/mod.rs:32-36)
template <int C>
__device__ __forceinline__ void emit_digits(const Fq& s_mont, int b, uint32_t gidx, int n1, const MsmArgs& a,
                                            bool count) {
  constexpr int W = 253 / C + 1;
  constexpr int NB = 1 << (C - 1);
  constexpr uint32_t MASK = (1u << C) - 1u;
  Fq k = fq_from_mont(s_mont);
  int carry = 0;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const int bit = w * C;
    const int li = bit >> 5, of = bit & 31;
    uint32_t v = k.l[li] >> of;
    if (of + C > 32 && li + 1 < 8) v |= k.l[li + 1] << (32 - of);
    int d = (int)(v & MASK) + carry;
    carry = d > NB ? 1 : 0;
    d -= carry << C;
    if (d != 0) {
      uint32_t mag = (uint32_t)(d < 0 ? -d : d);
      uint32_t key = (uint32_t)b * NB + (mag - 1);
      if (count) {
        atomicAdd(&a.hist[key], 1u);
      } else {
        uint32_t slot = a.off[key] + atomicAdd(&a.cursor[key], 1u);
        uint32_t e = (uint32_t)bit * (uint32_t)n1 + gidx;
        a.entries[slot] = e | (d < 0 ? 0x80000000u : 0u);
      }
    }
  }
}

template <int C>
__global__ void k_digits(MsmArgs a, bool count) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  int per = a.n + (a.blinds ? 1 : 0);
  if (t >= (size_t)a.B * per) return;
  int b = (int)(t / per), i = (int)(t % per);
  Fq s;
  uint32_t gidx;
  if (i < a.n) {
    s = a.scalars[(size_t)b * a.n + i];
    gidx = a.idx ? a.idx[(size_t)b * a.n + i] : (uint32_t)(a.gen_offset + i);
  } else {
    s = a.blinds[b];
    gidx = (uint32_t)a.h_index;
  }
  emit_digits<C>(s, b, gidx, a.n1, a, count);
}

// Row-local counting sort for batches of many MSMs (one workgroup per MSM b): the bucket histogram and the
// cursors live in LDS, so the 24 digit atomics per scalar are LDS atomics instead of L2 atomics on a
// B*NB-key global histogram, and the entries of MSM b land in its own region [b*per*W, (b+1)*per*W) of
// the entries array (off[key] points into it; k_items only reads off[key] and hist[key]). The bucket order
// of entries differs from k_digits', the bucket sums (group elements) do not.
template <int C>
__global__ void __launch_bounds__(256) k_digits_rows(MsmArgs a) {
  constexpr int W = 253 / C + 1;
  constexpr int NB = 1 << (C - 1);
  constexpr uint32_t MASK = (1u << C) - 1u;
  constexpr int PT = (NB + 255) / 256;  // keys per thread in the scan
  __shared__ uint32_t cnt[NB], part[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int per = a.n + (a.blinds ? 1 : 0);
  const uint32_t rowbase = (uint32_t)b * (uint32_t)per * (uint32_t)W;
  for (int k = tid; k < NB; k += 256) cnt[k] = 0;
  __syncthreads();
  for (int pass = 0; pass < 2; pass++) {
    for (int i = tid; i < per; i += 256) {
      Fq sm;
      uint32_t gidx;
      if (i < a.n) {
        sm = a.scalars[(size_t)b * a.n + i];
        gidx = a.idx ? a.idx[(size_t)b * a.n + i] : (uint32_t)(a.gen_offset + i);
      } else {
        sm = a.blinds[b];
        gidx = (uint32_t)a.h_index;
      }
      const Fq k = fq_from_mont(sm);
      int carry = 0;
#pragma unroll
      for (int w = 0; w < W; w++) {
        const int bit = w * C;
        const int li = bit >> 5, of = bit & 31;
        uint32_t v = k.l[li] >> of;
        if (of + C > 32 && li + 1 < 8) v |= k.l[li + 1] << (32 - of);
        int d = (int)(v & MASK) + carry;
        carry = d > NB ? 1 : 0;
        d -= carry << C;
        if (d != 0) {
          const uint32_t mag = (uint32_t)(d < 0 ? -d : d);
          const uint32_t slot = atomicAdd(&cnt[mag - 1], 1u);
          if (pass)
            a.entries[rowbase + slot] = ((uint32_t)bit * (uint32_t)a.n1 + gidx) | (d < 0 ? 0x80000000u : 0u);
        }
      }
    }
    __syncthreads();
    if (pass) break;
    // counts -> global hist; exclusive scan -> off (global) and the LDS cursors
    uint32_t loc[PT], sum = 0;
#pragma unroll
    for (int j = 0; j < PT; j++) {
      const int k = tid * PT + j;
      loc[j] = k < NB ? cnt[k] : 0u;
      sum += loc[j];
    }
    part[tid] = sum;
    __syncthreads();
    for (int st = 1; st < 256; st <<= 1) {  // Hillis-Steele inclusive scan of the 256 partial sums
      const uint32_t x = tid >= st ? part[tid - st] : 0u;
      __syncthreads();
      part[tid] += x;
      __syncthreads();
    }
    uint32_t run = part[tid] - sum;
#pragma unroll
    for (int j = 0; j < PT; j++) {
      const int k = tid * PT + j;
      if (k < NB) {
        a.hist[(size_t)b * NB + k] = loc[j];
        a.off_out[(size_t)b * NB + k] = rowbase + run;
        cnt[k] = run;
      }
      run += loc[j];
    }
    __syncthreads();
  }
}

__global__ void k_item_counts(const uint32_t* __restrict__ hist, uint32_t* __restrict__ items, int nkeys, uint32_t K) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nkeys) return;
  items[i] = i < nkeys ? (hist[i] + K - 1) / K : 0u;
}

__global__ void k_item_keys(const uint32_t* __restrict__ item_off, uint32_t* __restrict__ item_key, int nkeys) {
  int key = blockIdx.x * blockDim.x + threadIdx.x;
  if (key >= nkeys) return;
  for (uint32_t it = item_off[key]; it < item_off[key + 1]; it++) item_key[it] = (uint32_t)key;
}


// one work item: a bucket's entries split into ceil(count / kItemK) items of equal size (+-1), so the lanes of a
// wave carry the same number of additions (fixed 16-entry items left 16 + 8 for a 24-entry bucket: ~75 % of the
// lanes' issue slots busy)
__global__ void __launch_bounds__(256) k_items(const uint32_t* __restrict__ item_key,
                                               const uint32_t* __restrict__ item_off,
                                               const uint32_t* __restrict__ off, const uint32_t* __restrict__ hist,
                                               const uint32_t* __restrict__ entries, const Niels* __restrict__ tab,
                                               Ext* __restrict__ partial, const uint32_t* __restrict__ total_items) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= *total_items) return;
  const uint32_t key = item_key[t];
  const uint32_t i0 = item_off[key], ni = item_off[key + 1] - i0, j = t - i0, h = hist[key];
  const uint32_t start = off[key] + (uint32_t)(((uint64_t)h * j) / ni);
  const uint32_t end = off[key] + (uint32_t)(((uint64_t)h * (j + 1)) / ni);
  Ext P = load_signed(tab, entries[start]);
  for (uint32_t s = start + 1; s < end; s++) {
    uint32_t e = entries[s];
    P = ext_madd(P, tab[e & 0x7fffffffu], (e >> 31) != 0);
  }
  partial[t] = P;
}

// thread per (msm, segment): bucket values v in [lo, hi] (1-based), m = kSegM buckets each
__global__ void __launch_bounds__(64) k_segments(const uint32_t* __restrict__ item_off, const Ext* __restrict__ partial,
                                                 Ext* __restrict__ segT, Ext* __restrict__ segS, int B, int NB,
                                                 int m) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  int S = NB / m;
  if (t >= B * S) return;
  int b = t / S, j = t % S;
  int lo = j * m + 1, hi = j * m + m;
  Ext run = ext_identity(), T = ext_identity();
  bool any = false;
  for (int v = hi; v >= lo; v--) {
    uint32_t key = (uint32_t)b * NB + (v - 1);
    for (uint32_t it = item_off[key]; it < item_off[key + 1]; it++) {
      run = any ? ext_add(run, partial[it]) : partial[it];
      any = true;
    }
    if (any) T = ext_add(T, run);
  }
  segT[t] = T;
  segS[t] = run;
}

// the algorithmic work of a fixed-base MSM pass over `scalars` scalars with c-bit signed windows: one mixed
// addition per nonzero digit, W = 253/c + 1 windows, a digit being zero with probability 2^-c
static inline double madds_model(double scalars, int c) {
  return scalars * (double)(253 / c + 1) * (1.0 - 1.0 / (double)(1 << c));
}

static bool use_quad() {
  static const bool on = !getenv("SPG_SMSM_QUAD") || atoi(getenv("SPG_SMSM_QUAD")) != 0;
  return on;
}

// one 256-thread block per MSM. Segment j (bucket values j*m+1 .. j*m+m) contributes
// T_j + j*m*S_j. Thread t folds the g = S/256 consecutive segments [t*g, t*g+g) into
//   value_t = sum T_j + m * sum_j (j - t*g) S_j      and      V_t = sum S_j,
// leaving sum_t value_t + (g*m) * sum_t t*V_t, done with an LDS suffix scan of V plus a tree sum.
__global__ void __launch_bounds__(256) k_final(const Ext* __restrict__ segT, const Ext* __restrict__ segS,
                                               uint8_t* __restrict__ out, int S, int log2m, Ext* __restrict__ ext_out) {
  __shared__ uint32_t sh[soa_words<Ext, 256>()];
  const int b = blockIdx.x, t = threadIdx.x;
  const int g = S >= 256 ? S / 256 : 1;
  int log2g = 0;
  while ((1 << log2g) < g) log2g++;
  const int lo = t * g, hi = lo + g < S ? lo + g : S;
  const Ext* T = segT + (size_t)b * S;
  const Ext* Sv = segS + (size_t)b * S;
  Ext U = ext_identity(), V = ext_identity(), acc = ext_identity(), tot = ext_identity();
  for (int j = hi - 1; j >= lo; j--) {
    U = ext_add(U, T[j]);
    V = ext_add(V, Sv[j]);
    if (j > lo) {
      acc = ext_add(acc, Sv[j]);
      tot = ext_add(tot, acc);
    }
  }
  for (int k = 0; k < log2m; k++) tot = ext_dbl(tot);
  Ext val = ext_add(U, tot);
  // inclusive suffix scan of V over threads
  Ext suf = V;
  for (int d = 1; d < 256; d <<= 1) {
    soa_put<256>(sh, t, suf);
    __syncthreads();
    if (t + d < 256) suf = ext_add(suf, soa_get<256, Ext>(sh, t + d));
    __syncthreads();
  }
  if (t >= 1) {
    for (int k = 0; k < log2g + log2m; k++) suf = ext_dbl(suf);
    val = ext_add(val, suf);
  }
  for (int d = 128; d >= 1; d >>= 1) {
    soa_put<256>(sh, t, val);
    __syncthreads();
    if (t < d) val = ext_add(val, soa_get<256, Ext>(sh, t + d));
    __syncthreads();
  }
  if (t == 0 && ext_out) ext_out[b] = val;
  if (t == 0 && out) {
    uint8_t c[32];
    ext_compress(val, c);
    for (int k = 0; k < 32; k++) out[32 * (size_t)b + k] = c[k];
  }
}

// k_segments with quads (4 lanes per segment, quad_add): for few MSMs, where the segment sums are a short
// latency-bound phase rather than a throughput-bound one
__global__ void __launch_bounds__(256) k_segments_q(const uint32_t* __restrict__ item_off,
                                                    const Ext* __restrict__ partial, Ext* __restrict__ segT,
                                                    Ext* __restrict__ segS, int B, int NB, int m) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x, q = t & 3, sid = t >> 2;
  const int S = NB / m;
  if (sid >= B * S) return;  // whole quads exit together (4 | blockDim)
  const int b = sid / S, j = sid % S;
  const int lo = j * m + 1, hi = j * m + m;
  Ext run = ext_identity(), T = ext_identity();
  bool any = false;
  for (int v = hi; v >= lo; v--) {
    const uint32_t key = (uint32_t)b * NB + (v - 1);
    for (uint32_t it = item_off[key]; it < item_off[key + 1]; it++) {
      run = any ? quad_add(run, partial[it], q) : partial[it];
      any = true;
    }
    if (any) T = quad_add(T, run, q);
  }
  if (q == 0) {
    segT[sid] = T;
    segS[sid] = run;
  }
}
// Regrouping for few MSMs with many segments: group c of G folds the g consecutive segments
// [c g, c g + g) into T'_c = sum T_j + m sum_j (j - c g) S_j and S'_c = sum S_j (k_final's per-slot fold),
// so the set becomes G segments of m' = m g buckets and k_final_q needs fewer sequential steps per slot.
__global__ void __launch_bounds__(256) k_regroup_q(const Ext* __restrict__ segT, const Ext* __restrict__ segS, int B,
                                                   int S, int log2g, int log2m, Ext* __restrict__ outT,
                                                   Ext* __restrict__ outS) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x, q = t & 3, gid = t >> 2;
  const int g = 1 << log2g, G = S >> log2g;
  if (gid >= B * G) return;
  const int b = gid / G, c = gid % G;
  const Ext* T = segT + (size_t)b * S;
  const Ext* Sv = segS + (size_t)b * S;
  const int lo = c * g, hi = lo + g;
  Ext U = ext_identity(), V = ext_identity(), acc = ext_identity(), tot = ext_identity();
  for (int j = hi - 1; j >= lo; j--) {
    U = quad_add(U, T[j], q);
    V = quad_add(V, Sv[j], q);
    if (j > lo) {
      acc = quad_add(acc, Sv[j], q);
      tot = quad_add(tot, acc, q);
    }
  }
  for (int k = 0; k < log2m; k++) tot = quad_dbl(tot, q);
  const Ext val = quad_add(U, tot, q);
  if (q == 0) {
    outT[gid] = val;
    outS[gid] = V;
  }
}

// k_final with quads: SL slots of 4 lanes (4 SL threads; SL = 128 keeps it under 256 VGPRs), slot plays
// k_final's thread with SL in place of 256, every point operation
// split over the quad (quad_add / quad_dbl)
template <int SL>
__global__ void __launch_bounds__(4 * SL) k_final_q(const Ext* __restrict__ segT, const Ext* __restrict__ segS,
                                                 uint8_t* __restrict__ out, int S, int log2m, Ext* __restrict__ ext_out) {
  __shared__ uint32_t sh[soa_words<Ext, SL>()];
  const int b = blockIdx.x, t = threadIdx.x, q = t & 3, slot = t >> 2;
  const int g = S >= SL ? S / SL : 1;
  int log2g = 0;
  while ((1 << log2g) < g) log2g++;
  const int lo = slot * g, hi = lo + g < S ? lo + g : S;
  const Ext* T = segT + (size_t)b * S;
  const Ext* Sv = segS + (size_t)b * S;
  Ext U = ext_identity(), V = ext_identity(), acc = ext_identity(), tot = ext_identity();
  for (int j = hi - 1; j >= lo; j--) {
    U = quad_add(U, T[j], q);
    V = quad_add(V, Sv[j], q);
    if (j > lo) {
      acc = quad_add(acc, Sv[j], q);
      tot = quad_add(tot, acc, q);
    }
  }
  for (int k = 0; k < log2m; k++) tot = quad_dbl(tot, q);
  Ext val = quad_add(U, tot, q);
  Ext suf = V;
  for (int d = 1; d < SL; d <<= 1) {
    quad_put_op<SL>(sh, slot, suf, q);
    __syncthreads();
    if (slot + d < SL) suf = quad_add_op(suf, quad_get_op<SL>(sh, slot + d, q), q);
    __syncthreads();
  }
  if (slot >= 1) {
    for (int k = 0; k < log2g + log2m; k++) suf = quad_dbl(suf, q);
    val = quad_add(val, suf, q);
  }
  for (int d = SL / 2; d >= 1; d >>= 1) {
    quad_put_op<SL>(sh, slot, val, q);
    __syncthreads();
    if (slot < d) val = quad_add_op(val, quad_get_op<SL>(sh, slot + d, q), q);
    __syncthreads();
  }
  if (t == 0 && ext_out) ext_out[b] = val;
  if (t == 0 && out) {
    uint8_t c[32];
    ext_compress(val, c);
    for (int k = 0; k < 32; k++) out[32 * (size_t)b + k] = c[k];
  }
}

// ------------------------------------------------------------------ latency path for small MSMs
// Bullet rounds and single commitments are MSMs of ~10^3 points whose cost is the depth of the
// dependent group additions, not their count. One block per (msm, bucket value v): every thread
// scans a slice of the scalars, recomputes their signed c-bit digits and mixed-adds the table entry
// of every digit with |d| == v; an LDS tree sums the block. A second kernel forms sum_v v * B_v with
// an LDS suffix scan + tree. Results stay in extended coordinates: the host encodes them (the
// inverse square root of the encoding is ~250 dependent squarings, cheap on a CPU core, slow on one
// GPU lane).
// `blinds` must be a valid pointer even when has_blind == 0: blinds[b] has a wave-uniform address, so
// the compiler issues it as a scalar load inside a divergent branch, and scalar loads are not masked
// by EXEC when the branch is skipped (a null pointer there faults).
template <int C, int BS>
__global__ void __launch_bounds__(BS) k_smsm_bucket(const Fq* __restrict__ scalars, const uint32_t* __restrict__ idx,
                                                     const Fq* __restrict__ blinds, int has_blind, int n, int n1,
                                                     int gen_offset, int h_index, const Niels* __restrict__ tab,
                                                     Ext* __restrict__ buckets) {
  constexpr int W = 253 / C + 1;
  constexpr int NB = 1 << (C - 1);
  constexpr uint32_t MASK = (1u << C) - 1u;
  __shared__ uint32_t sh[soa_words<Ext, BS>()];
  const int v = blockIdx.x + 1, b = blockIdx.y, t = threadIdx.x;
  const int per = n + has_blind;
  Ext acc = ext_identity();
  for (int i = t; i < per; i += BS) {
    Fq s;
    uint32_t gidx;
    if (i < n) {
      s = scalars[(size_t)b * n + i];
      gidx = idx ? idx[(size_t)b * n + i] : (uint32_t)(gen_offset + i);
    } else {
      s = blinds[b];
      gidx = (uint32_t)h_index;
    }
    Fq k = fq_from_mont(s);
    int carry = 0;
    uint64_t hit = 0, neg = 0;  // windows whose digit is +-v (W <= 64)
#pragma unroll
    for (int w = 0; w < W; w++) {
      const int bit = w * C;
      const int li = bit >> 5, of = bit & 31;
      uint32_t x = k.l[li] >> of;
      if (of + C > 32 && li + 1 < 8) x |= k.l[li + 1] << (32 - of);
      int d = (int)(x & MASK) + carry;
      carry = d > NB ? 1 : 0;
      d -= carry << C;
      if (d == v || d == -v) hit |= 1ull << w;
      if (d == -v) neg |= 1ull << w;
    }
    while (hit) {
      const int w = __ffsll((long long)hit) - 1;
      hit &= hit - 1;
#ifdef SPG_CHECKED
      if (w < 0 || w >= W || gidx >= (uint32_t)n1) {
        printf("k_smsm_bucket<%d>: bad index w=%d gidx=%u n1=%d i=%d b=%d v=%d\n", C, w, gidx, n1, i, b, v);
        continue;
      }
#endif
      acc = ext_madd(acc, tab[(size_t)(w * C) * n1 + gidx], (neg >> w) & 1);
    }
  }
  for (int d = BS / 2; d >= 1; d >>= 1) {
    soa_put<BS>(sh, t, acc);
    __syncthreads();
    if (t < d) acc = ext_add(acc, soa_get<BS, Ext>(sh, t + d));
    __syncthreads();
  }
  if (t == 0) buckets[(size_t)b * NB + (v - 1)] = acc;
}

// Latency-path bucket kernel, quad form: one workgroup per (bucket v, MSM b) as k_smsm_bucket, but the
// table entries of bucket v are first collected in LDS (one round of BS scalars at a time) and dealt out
// evenly to the BS/4 quads, which add them with the quad-split arithmetic; the quads' sums then meet in an
// LDS tree (component-major, each lane of a giving quad stores one coordinate).
template <int C, int BS>
__global__ void __launch_bounds__(BS) k_smsm_bucket_q(const Fq* __restrict__ scalars, const uint32_t* __restrict__ idx,
                                                       const Fq* __restrict__ blinds, int has_blind, int n, int n1,
                                                       int gen_offset, int h_index, const Niels* __restrict__ tab,
                                                       Ext* __restrict__ buckets) {
  constexpr int W = 253 / C + 1;
  constexpr int NB = 1 << (C - 1);
  constexpr uint32_t MASK = (1u << C) - 1u;
  constexpr int S = BS / 4;  // quads
  __shared__ uint32_t list[BS * W];  // bucket entries of one round: table index | neg << 31
  __shared__ uint32_t pts[soa_words<Ext, S>()];
  __shared__ uint32_t cnt;
  const int v = blockIdx.x + 1, b = blockIdx.y, t = threadIdx.x, q = t & 3, slot = t >> 2;
  const int per = n + has_blind;
  Ext acc = ext_identity();
  if (t == 0) cnt = 0;
  __syncthreads();
  for (int base = 0; base < per; base += BS) {
    const int i = base + t;
    if (i < per) {
      Fq s;
      uint32_t gidx;
      if (i < n) {
        s = scalars[(size_t)b * n + i];
        gidx = idx ? idx[(size_t)b * n + i] : (uint32_t)(gen_offset + i);
      } else {
        s = blinds[b];
        gidx = (uint32_t)h_index;
      }
      Fq k = fq_from_mont(s);
      int carry = 0;
#pragma unroll
      for (int w = 0; w < W; w++) {
        const int bit = w * C;
        const int li = bit >> 5, of = bit & 31;
        uint32_t x = k.l[li] >> of;
        if (of + C > 32 && li + 1 < 8) x |= k.l[li + 1] << (32 - of);
        int d = (int)(x & MASK) + carry;
        carry = d > NB ? 1 : 0;
        d -= carry << C;
        // the top window holds little more than the final carry (scalars < 2^253), a digit of magnitude 1 for
        // about every second scalar, which would pile onto bucket 1 and set the kernel's critical path: such an
        // entry 2^{(W-1)C} P is taken as 2^s * (2^{(W-1)C - s} P) instead, s = 1 .. C-1 by generator, spreading
        // those entries over buckets 2, 4, .., 2^{C-1} (same point, table row (W-1)C - s)
        int bo = w * C;
        if (w == W - 1 && (d == 1 || d == -1)) {
          const int sh = 1 + (int)(gidx % (uint32_t)(C - 1));
          d <<= sh;
          bo -= sh;
        }
        if (d == v || d == -v) {
          const uint32_t pos = atomicAdd(&cnt, 1u);
          list[pos] = (uint32_t)((size_t)bo * n1 + gidx) | (d < 0 ? 0x80000000u : 0u);
        }
      }
    }
    __syncthreads();
    const uint32_t m = cnt;
    // software-pipelined: the table coordinate of entry e + S is loaded while entry e is added
    uint32_t e = slot;
    Fp qv;
    bool neg = false;
    if (e < m) qv = niels_coord(tab, list[e], q, &neg);
    while (e < m) {
      const uint32_t e2 = e + S;
      Fp qn;
      bool nn = false;
      if (e2 < m) qn = niels_coord(tab, list[e2], q, &nn);
      acc = quad_madd(acc, qv, neg, q);
      qv = qn;
      neg = nn;
      e = e2;
    }
    __syncthreads();
    if (t == 0) cnt = 0;
    __syncthreads();
  }
  for (int d = S / 2; d >= 1; d >>= 1) {
    if (slot >= d && slot < 2 * d) quad_put_op<S>(pts, slot - d, acc, q);
    __syncthreads();
    if (slot < d) acc = quad_add_op(acc, quad_get_op<S>(pts, slot, q), q);
    __syncthreads();
  }
  if (t == 0) buckets[(size_t)b * NB + (v - 1)] = acc;
}

int bullet_round_device(spg_ctx* ctx, const spg_gens* g, const Fq* aa_in, const Fq* cw_in, Fq* aa_out, Fq* cw_out,
                        const uint32_t* gidx, const Fq& u, const Fq& uinv, int k, int n, int nk, Ext* d_buckets,
                        uint32_t* seq_out) {
  SPG_CHECK(ctx, n >= 2 && (n & (n - 1)) == 0 && nk >= 2 && nk <= n && (n % nk) == 0, "bullet round: bad sizes");
  BulletArgs a{aa_in, cw_in, aa_out, cw_out, gidx, u, uinv, k, n, nk, (int)(g->n + 1), g->table, d_buckets,
               ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq, nullptr};
  *seq_out = a.seq;
  constexpr int C = 7, NB = 1 << (C - 1);
  // VALU model: one mixed addition per nonzero signed 7-bit digit of the L and R MSMs' n/2 scalars each
  KScope ks(ctx, "msm_bullet_round", 0.0, madds_model(n, C));
  if (n / 2 <= 64)
    hipLaunchKernelGGL((k_bullet_round_q<C, 64>), dim3(NB + 1, 2), dim3(64), 0, ctx->stream, a);
  else if (n / 2 <= 128)
    hipLaunchKernelGGL((k_bullet_round_q<C, 128>), dim3(NB + 1, 2), dim3(128), 0, ctx->stream, a);
  else
    hipLaunchKernelGGL((k_bullet_round_q<C, 256>), dim3(NB + 1, 2), dim3(256), 0, ctx->stream, a);
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

// the comb form's launch shape by MSM size P = n / 2: G quads per scalar (window groups of ceil(22 / G)), BS threads,
// R points per workgroup (SPG_BCOMB_G / SPG_BCOMB_BS / SPG_BCOMB_R override, for A/B runs)
static void bullet_comb_shape(int P, int* G, int* BS, int* R) {
  static const int eg = getenv("SPG_BCOMB_G") ? atoi(getenv("SPG_BCOMB_G")) : 0;
  static const int ebs = getenv("SPG_BCOMB_BS") ? atoi(getenv("SPG_BCOMB_BS")) : 0;
  static const int er = getenv("SPG_BCOMB_R") ? atoi(getenv("SPG_BCOMB_R")) : 0;
  // same-box A/Bs on the 2^20 SNARK (Bullet device ms per prove; profiles/r04_ab_bullet_shapes.txt): G 4 -> 8 at
  // P = 512: 1.92 -> 1.88; G 8 -> 11 (two dependent quad additions per quad): 1.87 -> 1.81; R 4 -> 8 (one tree level
  // fewer, twice the host-summed parts): 1.89 -> 1.74, R = 16: 1.85
  *G = P >= 2048 ? 4 : 11;
  *BS = P <= 64 ? 64 : (P <= 128 ? 128 : 256);
  // R: round 4 chose 8 on device time alone; on the prover's wall clock the host's part sums weigh more (91 ns per
  // addition on the box, K <= 4 chunks per MSM: scripts/micro/parts_finals_cpu.cpp, profiles/r05_parts_finals.txt),
  // and R = 2 was fastest (2-rep A/B, SNARK median ms: R 8: 16.66 / 17.13, 2: 16.08 / 16.13, 1: 17.56 / 16.71); with the
  // IFMA part sums (hvec.hpp) R = 4 was (ABBA A/B: 15.23 / 15.93 / 16.39 / 15.67 -> 15.13 / 15.04 / 15.84 / 15.02), and
  // later in the round R = 8 (ABBA, 3 blocks: mean 16.03 -> 15.34 ms, device busy 8.65 -> 8.53 ms; R = 16 15.29 against
  // 15.40; profiles/r05_ab_bcomb_r8.txt)
  *R = P >= 2048 ? 1 : 8;  // the SPARK PolyEvalProofs at 2^24 nonzeros (P = 4096): 256 workgroups per MSM
  if (eg == 4 || eg == 8 || eg == 11) *G = eg;
  if (ebs == 64 || ebs == 128 || ebs == 256) *BS = ebs;
  if (er >= 1 && er <= *BS / 4 && (er & (er - 1)) == 0) *R = er;
  // the last rounds (P <= SPG_BCOMB_NOTREE): every quad its own part, no LDS tree (one level is a full quad addition,
  // ~2.1 us on the round's latency path, scripts/micro/bullet_comb_phases) for at most 2 x 16 parts per MSM
  static const int notree = getenv("SPG_BCOMB_NOTREE") ? atoi(getenv("SPG_BCOMB_NOTREE")) : 0;
  if (P <= notree) *R = *BS / 4;
  // at most kBulletPartsMax parts per MSM (the host staging): fewer points per workgroup for the largest proofs
  const int wgs = (P * *G + *BS / 4 - 1) / (*BS / 4);
  while (*R > 1 && wgs * *R > kBulletPartsMax) *R /= 2;
}

int bullet_round_comb(spg_ctx* ctx, const spg_gens* g, const Fq* aa_in, const Fq* cw_in, Fq* aa_out, Fq* cw_out,
                      const uint32_t* gidx, size_t gmax, const Fq& u, const Fq& uinv, int k, int n, int nk,
                      Ext* d_parts, uint32_t* seq_out, int* per_msm) {
  SPG_CHECK(ctx, n >= 2 && (n & (n - 1)) == 0 && nk >= 2 && nk <= n && (n % nk) == 0, "bullet round: bad sizes");
  static const bool on = !getenv("SPG_BULLET_COMB") || atoi(getenv("SPG_BULLET_COMB")) != 0;
  if (!on) return 1;
  spg_gens::Comb cb;
  const int rc = comb_get(ctx, g, gmax, &cb);
  if (rc) return rc == 1 ? 1 : rc;
  if (cb.c != 12 && cb.c != 13) return 1;  // the kernels take 12- or 13-bit windows
  int G, BS, R;
  bullet_comb_shape(n / 2, &G, &BS, &R);
  if (cb.c == 13 && G != 4) G = 10;  // 20 windows: groups of 2 (11 would leave one empty)
  const int S = BS / 4, quads = (n / 2) * G, wgs = (quads + S - 1) / S;
  if (wgs * R > kBulletPartsMax) return 1;
  BulletCombArgs a{aa_in, cw_in, aa_out, cw_out, gidx, u, uinv, k, n, nk, cb.p, (int)cb.slots + 1, R, d_parts,
                   ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq, cb.st};
  *seq_out = a.seq;
  *per_msm = wgs * R;
  // VALU model: one mixed addition per nonzero signed C-bit digit of the n/2 scalars of each of the two MSMs
  // algorithmic bytes: every nonzero digit's 96-byte comb entry, the fold's reads and writes (aa: 2 nk in, nk out;
  // cw: n in, n out; gidx: n)
  const double W = 253 / cb.c + 1, entries = (double)n * W * (1.0 - 1.0 / (double)(1 << cb.c));
  KScope ks(ctx, "msm_bullet_round", 96.0 * entries + 96.0 * nk + 68.0 * n, entries);
  const dim3 grid((unsigned)wgs, 2);
  // SPG_BCOMB_ROLL=1: the rolled-loop form (k_bullet_comb_roll, bullet.hpp: 2,256 instead of 4,033 instructions).
  // Measured slower, so off by default: +0.35 us per dependent pair of quad additions, +0.9 us per three tree levels,
  // event time +0.1..1.2 us per launch (scripts/micro/bullet_comb_phases, profiles/r06_bcomb_roll_phases.txt), bench
  // kernel average 17.2 -> 17.8 us (ABBA x3, profiles/r06_ab_bcomb_roll.txt): the round is bound by its dependent
  // field-product chain, not by fetching its straight-line code
  static const bool roll = getenv("SPG_BCOMB_ROLL") && atoi(getenv("SPG_BCOMB_ROLL")) != 0;
#define SPG_BCOMB(CC, GG, BB)                                                                      \
  do {                                                                                             \
    if (roll)                                                                                      \
      hipLaunchKernelGGL((k_bullet_comb_roll<CC, GG, BB>), grid, dim3(BB), 0, ctx->stream, a);     \
    else                                                                                           \
      hipLaunchKernelGGL((k_bullet_comb<CC, GG, BB>), grid, dim3(BB), 0, ctx->stream, a);          \
  } while (0)
#define SPG_BCOMB_BS(CC, GG) \
  do { if (BS == 64) SPG_BCOMB(CC, GG, 64); else if (BS == 128) SPG_BCOMB(CC, GG, 128); else SPG_BCOMB(CC, GG, 256); } while (0)
  if (cb.c == 13) {
    if (G == 4) SPG_BCOMB_BS(13, 4); else SPG_BCOMB_BS(13, 10);
  } else if (G == 4) {
    SPG_BCOMB_BS(12, 4);
  } else if (G == 8) {
    SPG_BCOMB_BS(12, 8);
  } else {
    SPG_BCOMB_BS(12, 11);
  }
#undef SPG_BCOMB_BS
#undef SPG_BCOMB
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

// DotProductProofLog's delta scalars d cw_j from the device Bullet state: cw (plain integers, bullet.hpp) as the last
// round left it, times the last challenge's fold (u for odd j, u^-1 for even j) and d; cu = (d u) R^2, cinv = (d u^-1) R^2
// (raw limbs), so that one Montgomery product gives the Montgomery scalar d f cw_j R
__global__ void k_bullet_delta_scalars(const Fq* __restrict__ cw, int n, Fq cu, Fq cinv, Fq* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) out[j] = fq_mul((j & 1) ? cu : cinv, cw[j]);
}

int bullet_delta_scalars(spg_ctx* ctx, const Fq* cw, int n, const Fq& d, const Fq& u, const Fq& uinv, Fq* out) {
  const Fq cu = fq_to_mont(fq_mul(d, u)), cinv = fq_to_mont(fq_mul(d, uinv));
  hipLaunchKernelGGL(k_bullet_delta_scalars, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, cw, n, cu,
                     cinv, out);
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

int comb_msm_parts(spg_ctx* ctx, const spg_gens* g, const Fq* d_scalars, const uint32_t* d_idx, size_t gmax, int n,
                   int B, Ext* d_parts, int* per_msm) {
  static const bool on = !getenv("SPG_BULLET_COMB") || atoi(getenv("SPG_BULLET_COMB")) != 0;
  if (!on || n < 1) return 1;
  spg_gens::Comb cb;
  const int rc = comb_get(ctx, g, gmax, &cb);
  if (rc) return rc == 1 ? 1 : rc;
  if (cb.c != 12 && cb.c != 13) return 1;
  int G, BS, R;
  bullet_comb_shape(std::max(2, n), &G, &BS, &R);
  if (cb.c == 13 && G != 4) G = 10;
  const int S = BS / 4, wgs = (n * G + S - 1) / S;
  if (wgs * R > kBulletPartsMax) return 1;
  *per_msm = wgs * R;
  KScope ks(ctx, "msm_comb_parts", 0.0, (double)B * n * (253 / cb.c + 1) * (1.0 - 1.0 / (double)(1 << cb.c)));
  const dim3 grid((unsigned)wgs, (unsigned)B);
  const int NS = (int)cb.slots + 1;
#define SPG_CMP(CC, GG, BB) \
  hipLaunchKernelGGL((k_comb_msm_parts<CC, GG, BB>), grid, dim3(BB), 0, ctx->stream, d_scalars, d_idx, n, cb.p, NS, R, d_parts, \
                     cb.st)
#define SPG_CMP_BS(CC, GG) \
  do { if (BS == 64) SPG_CMP(CC, GG, 64); else if (BS == 128) SPG_CMP(CC, GG, 128); else SPG_CMP(CC, GG, 256); } while (0)
  if (cb.c == 13) {
    if (G == 4) SPG_CMP_BS(13, 4); else SPG_CMP_BS(13, 10);
  } else if (G == 4) {
    SPG_CMP_BS(12, 4);
  } else if (G == 8) {
    SPG_CMP_BS(12, 8);
  } else {
    SPG_CMP_BS(12, 11);
  }
#undef SPG_CMP_BS
#undef SPG_CMP
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

// the latency-path bucket kernel, quad form unless SPG_SMSM_QUAD=0
#define SMSM_LAUNCH(BSZ, ...)                                                                   \
  do {                                                                                          \
    if (use_quad())                                                                             \
      hipLaunchKernelGGL((k_smsm_bucket_q<C, BSZ>), dim3(NB, B), dim3(BSZ), 0, s, __VA_ARGS__); \
    else                                                                                        \
      hipLaunchKernelGGL((k_smsm_bucket<C, BSZ>), dim3(NB, B), dim3(BSZ), 0, s, __VA_ARGS__);   \
  } while (0)

// one block of NB threads per MSM: sum_v v * B_v = sum_t (sum_{u >= t} B_u)
__global__ void __launch_bounds__(256) k_smsm_final(const Ext* __restrict__ buckets, int NB, Ext* __restrict__ out) {
  __shared__ uint32_t sh[soa_words<Ext, 256>()];
  const int b = blockIdx.x, t = threadIdx.x;
  Ext suf = buckets[(size_t)b * NB + t];
  for (int d = 1; d < NB; d <<= 1) {
    soa_put<256>(sh, t, suf);
    __syncthreads();
    if (t + d < NB) suf = ext_add(suf, soa_get<256, Ext>(sh, t + d));
    __syncthreads();
  }
  for (int d = NB / 2; d >= 1; d >>= 1) {
    soa_put<256>(sh, t, suf);
    __syncthreads();
    if (t < d) suf = ext_add(suf, soa_get<256, Ext>(sh, t + d));
    __syncthreads();
  }
  if (t == 0) out[b] = suf;
}

// k_smsm_final with quads: 4 NB threads (NB <= 256), slot = thread / 4 plays bucket slot's thread
__global__ void __launch_bounds__(1024) k_smsm_final_q(const Ext* __restrict__ buckets, int NB, Ext* __restrict__ out) {
  __shared__ uint32_t sh[soa_words<Ext, 256>()];
  const int b = blockIdx.x, t = threadIdx.x, q = t & 3, slot = t >> 2;
  Ext suf = buckets[(size_t)b * NB + slot];
  for (int d = 1; d < NB; d <<= 1) {
    quad_put_op<256>(sh, slot, suf, q);
    __syncthreads();
    if (slot + d < NB) suf = quad_add_op(suf, quad_get_op<256>(sh, slot + d, q), q);
    __syncthreads();
  }
  for (int d = NB / 2; d >= 1; d >>= 1) {
    quad_put_op<256>(sh, slot, suf, q);
    __syncthreads();
    if (slot < d) suf = quad_add_op(suf, quad_get_op<256>(sh, slot + d, q), q);
    __syncthreads();
  }
  if (t == 0) out[b] = suf;
}

static int pick_small_window(size_t per) {
  const char* e = getenv("SPG_SMSM_C");
  if (e) {
    int c = atoi(e);
    if (c >= 4 && c <= 9) return c;
  }
  // measured on MI355X (scripts/perf_small_msm.py): n = 130 -> c = 7, n = 4098 -> c = 8; the compacted
  // Bullet MSMs (n/2 + 2 = 514 scalars) finish on the host, where 64 buckets per MSM are cheaper than 128
  // (scripts/ab_env.sh SPG_SMSM_C "7 0": 39.7 vs 39.9-40.9 ms per SNARK::prove)
  return per <= 1024 ? 7 : 8;
}

template <int C>
static void launch_small(spg_ctx* ctx, const Fq* sc, const uint32_t* idx, const Fq* bl, int n, int n1, int off, int h, const Niels* tab,
                         Ext* bk, Ext* out, int B, hipStream_t s) {
  constexpr int NB = 1 << (C - 1);
  {
    // threads per block = the scalars of one MSM rounded up (a smaller LDS tree and more resident blocks)
    const int per = n + (bl ? 1 : 0);
    KScope ks(ctx, "msm_small_bucket", 0.0, madds_model((double)B * per, C));
    const Fq* blp = bl ? bl : sc;
    if (per <= 64)
      SMSM_LAUNCH(64, sc, idx, blp, bl ? 1 : 0, n, n1, off, h,
                         tab, bk);
    else if (per <= 128)
      SMSM_LAUNCH(128, sc, idx, blp, bl ? 1 : 0, n, n1, off,
                         h, tab, bk);
    else
      SMSM_LAUNCH(256, sc, idx, blp, bl ? 1 : 0, n, n1, off,
                         h, tab, bk);
  }
  KScope ks(ctx, "msm_small_final");
  if (use_quad())
    hipLaunchKernelGGL(k_smsm_final_q, dim3(B), dim3(4 * NB), 0, s, bk, NB, out);
  else
    hipLaunchKernelGGL(k_smsm_final, dim3(B), dim3(NB), 0, s, bk, NB, out);
}

template <int C>
static void launch_buckets(spg_ctx* ctx, const Fq* sc, const uint32_t* idx, const Fq* bl, int n, int n1, int off, int h,
                           const Niels* tab, Ext* bk, int B, hipStream_t s) {
  constexpr int NB = 1 << (C - 1);
  const int per = n + (bl ? 1 : 0);
  KScope ks(ctx, "msm_small_bucket", 0.0, madds_model((double)B * per, C));
  const Fq* blp = bl ? bl : sc;
  if (per <= 64)
    SMSM_LAUNCH(64, sc, idx, blp, bl ? 1 : 0, n, n1, off, h, tab,
                       bk);
  else if (per <= 128)
    SMSM_LAUNCH(128, sc, idx, blp, bl ? 1 : 0, n, n1, off, h,
                       tab, bk);
  else
    SMSM_LAUNCH(256, sc, idx, blp, bl ? 1 : 0, n, n1, off, h,
                       tab, bk);
}

// the bucket stage of the latency path only: d_buckets[b * NB + v - 1] = B_v of MSM b; returns NB. The caller
// forms sum_v v * B_v (2 NB dependent additions: ~100 ns each on a host core with radix-2^51 limbs, ~5 us
// each on one GPU lane).
int msm_small_buckets(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
                      const Fq* d_blinds, const uint32_t* d_idx, long h_index, Ext* d_buckets, int* nb_out) {
  hipStream_t s = ctx->stream;
  const size_t per = n + (d_blinds ? 1 : 0);
  const int c = pick_small_window(per);
  SPG_CHECK(ctx, B <= 65535, "msm batch too large for the latency path");
  const int n1 = (int)(g->n + 1), off = (int)gen_offset, h = h_index < 0 ? (int)g->n : (int)h_index;
  switch (c) {
    case 4: launch_buckets<4>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, d_buckets, (int)B, s); break;
    case 5: launch_buckets<5>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, d_buckets, (int)B, s); break;
    case 6: launch_buckets<6>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, d_buckets, (int)B, s); break;
    case 7: launch_buckets<7>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, d_buckets, (int)B, s); break;
    case 8: launch_buckets<8>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, d_buckets, (int)B, s); break;
    default: launch_buckets<9>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, d_buckets, (int)B, s); break;
  }
  SPG_HIP(ctx, hipGetLastError());
  *nb_out = 1 << (c - 1);
  return 0;
}

int msm_small_device(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
                     const Fq* d_blinds, Ext* d_out, const uint32_t* d_idx, long h_index) {
  hipStream_t s = ctx->stream;
  const size_t per = n + (d_blinds ? 1 : 0);
  const int c = pick_small_window(per);
  const int NB = 1 << (c - 1);
  SPG_CHECK(ctx, B <= 65535, "msm batch too large for the latency path");
  Ext* bk = (Ext*)ws_get(ctx, 13, B * (size_t)NB * sizeof(Ext) + 64);
  if (!bk) return set_err(ctx, SPG_E_NOMEM, "small msm workspace");
  const int n1 = (int)(g->n + 1), off = (int)gen_offset, h = h_index < 0 ? (int)g->n : (int)h_index;
  switch (c) {
    case 4: launch_small<4>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, bk, d_out, (int)B, s); break;
    case 5: launch_small<5>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, bk, d_out, (int)B, s); break;
    case 6: launch_small<6>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, bk, d_out, (int)B, s); break;
    case 7: launch_small<7>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, bk, d_out, (int)B, s); break;
    case 8: launch_small<8>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, bk, d_out, (int)B, s); break;
    default: launch_small<9>(ctx, d_scalars, d_idx, d_blinds, (int)n, n1, off, h, g->table, bk, d_out, (int)B, s); break;
  }
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

// ext_compress of every point (RFC 9496 ENCODE), one lane per point
__global__ void __launch_bounds__(256) k_compress_ext(const Ext* __restrict__ in, size_t n, uint8_t* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) ext_compress(in[i], out + 32 * i);
}

// n extended points -> n x 32 encoded bytes (device), stream-ordered
int compress_ext_device(spg_ctx* ctx, const Ext* d_ext, size_t n, uint8_t* d_out) {
  if (!n) return 0;
  KScope ks(ctx, "msm_compress");
  hipLaunchKernelGGL(k_compress_ext, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, d_ext, n, d_out);
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

// B MSMs of n scalars (rows of a Hyrax commitment) through the latency path, compressed on the device
int msm_small_compressed(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
                         uint8_t* d_out) {
  Ext* d_ext = (Ext*)ws_get(ctx, 15, B * sizeof(Ext) + 64);
  if (!d_ext) return set_err(ctx, SPG_E_NOMEM, "small msm output");
  static const bool trace3 = getenv("SPG_TRACE") && atoi(getenv("SPG_TRACE")) >= 3;
  hipEvent_t e[3];
  if (trace3) {
    for (auto& x : e) hipEventCreate(&x);
    hipEventRecord(e[0], ctx->stream);
  }
  int rc = msm_small_device(ctx, g, gen_offset, d_scalars, n, B, nullptr, d_ext, nullptr, -1);
  if (rc) return rc;
  if (trace3) hipEventRecord(e[1], ctx->stream);
  KScope ks(ctx, "msm_compress");
  hipLaunchKernelGGL(k_compress_ext, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, ctx->stream, d_ext, B, d_out);
  SPG_HIP(ctx, hipGetLastError());
  if (trace3) {
    hipEventRecord(e[2], ctx->stream);
    hipEventSynchronize(e[2]);
    float a = 0, b = 0;
    hipEventElapsedTime(&a, e[0], e[1]);
    hipEventElapsedTime(&b, e[1], e[2]);
    fprintf(stderr, "[spg] small msm B=%zu n=%zu: msm %.0f us compress %.0f us\n", B, n, a * 1e3, b * 1e3);
    for (auto& x : e) hipEventDestroy(x);
  }
  return 0;
}

// ------------------------------------------------------------------ host orchestration
static int pick_window(size_t n_per_msm) {
  int best = 4;
  double best_cost = 1e300;
  for (int c = 4; c <= 16; c++) {
    int W = 253 / c + 1;
    double cost = (double)n_per_msm * W * 7.0 + (double)(1 << c) * 9.0;
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

template <int C>
static void launch_digits(const MsmArgs& a, bool count, hipStream_t s) {
  size_t per = a.n + (a.blinds ? 1 : 0);
  size_t nt = (size_t)a.B * per;
  hipLaunchKernelGGL(k_digits<C>, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, a, count);
}
static void dispatch_digits(int c, const MsmArgs& a, bool count, hipStream_t s) {
  switch (c) {
    case 4: launch_digits<4>(a, count, s); break;
    case 5: launch_digits<5>(a, count, s); break;
    case 6: launch_digits<6>(a, count, s); break;
    case 7: launch_digits<7>(a, count, s); break;
    case 8: launch_digits<8>(a, count, s); break;
    case 9: launch_digits<9>(a, count, s); break;
    case 10: launch_digits<10>(a, count, s); break;
    case 11: launch_digits<11>(a, count, s); break;
    case 12: launch_digits<12>(a, count, s); break;
    case 13: launch_digits<13>(a, count, s); break;
    case 14: launch_digits<14>(a, count, s); break;
    case 15: launch_digits<15>(a, count, s); break;
    default: launch_digits<16>(a, count, s); break;
  }
}

static void dispatch_digits_rows(int c, const MsmArgs& a, hipStream_t s) {
  const dim3 g((unsigned)a.B), t(256);
  switch (c) {
    case 4: hipLaunchKernelGGL(k_digits_rows<4>, g, t, 0, s, a); break;
    case 5: hipLaunchKernelGGL(k_digits_rows<5>, g, t, 0, s, a); break;
    case 6: hipLaunchKernelGGL(k_digits_rows<6>, g, t, 0, s, a); break;
    case 7: hipLaunchKernelGGL(k_digits_rows<7>, g, t, 0, s, a); break;
    case 8: hipLaunchKernelGGL(k_digits_rows<8>, g, t, 0, s, a); break;
    case 9: hipLaunchKernelGGL(k_digits_rows<9>, g, t, 0, s, a); break;
    case 10: hipLaunchKernelGGL(k_digits_rows<10>, g, t, 0, s, a); break;
    case 11: hipLaunchKernelGGL(k_digits_rows<11>, g, t, 0, s, a); break;
    case 12: hipLaunchKernelGGL(k_digits_rows<12>, g, t, 0, s, a); break;
    case 13: hipLaunchKernelGGL(k_digits_rows<13>, g, t, 0, s, a); break;
    case 14: hipLaunchKernelGGL(k_digits_rows<14>, g, t, 0, s, a); break;
    case 15: hipLaunchKernelGGL(k_digits_rows<15>, g, t, 0, s, a); break;
    default: hipLaunchKernelGGL(k_digits_rows<16>, g, t, 0, s, a); break;
  }
}

// B MSMs of n scalars each (device pointers), out_dev: B x 32 bytes (device)
int msm_batch_device(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n, size_t B,
                     const Fq* d_blinds, uint8_t* d_out, const uint32_t* d_idx, long h_index, Ext* d_ext) {
  hipStream_t s = ctx->stream;
  // the comb tables (comb.hip) replace digit sort, buckets and running sums: batches of >= 64 rows over <= 1024 generators, and the large batches of wider rows
  // (up to 2^14 generators: the SPARK derefs / comb_ops commits at 2^24 nonzeros), whose bucket path spends as much
  // time in its digit sort and bucket reduction as in its additions
  const size_t tot = B * (n + (d_blinds ? 1 : 0));
  if (!d_idx && B >= 64 && (n <= 1024 ? tot >= ((size_t)1 << 14) : (n <= 16384 && tot >= ((size_t)1 << 22)))) {
    Ext* ext = d_ext ? d_ext : (Ext*)ws_get(ctx, 17, B * sizeof(Ext) + 64);
    if (!ext) return set_err(ctx, SPG_E_NOMEM, "msm comb points");
    const int hi = !d_blinds ? -1 : (h_index < 0 ? (int)g->n : (int)h_index);
    const int rc = msm_comb(ctx, g, gen_offset, d_scalars, n, B, d_blinds, d_out, hi, ext);
    if (rc != kCombSkip) return rc;
  }
  const int c = pick_window(n + (d_blinds ? 1 : 0));
  const int NB = 1 << (c - 1);
  const int W = 253 / c + 1;
  const size_t nkeys = B * (size_t)NB;
  const size_t per = n + (d_blinds ? 1 : 0);
  const size_t max_entries = B * per * (size_t)W;
  static const int item_k = getenv("SPG_ITEM_K") ? std::max(1, atoi(getenv("SPG_ITEM_K"))) : kItemK;
  static const int seg_m = getenv("SPG_SEG_M") ? std::max(1, atoi(getenv("SPG_SEG_M"))) : kSegM;
  const size_t max_items = max_entries / item_k + nkeys + 1;
  SPG_CHECK(ctx, max_entries < 0x7fffffffULL, "msm batch too large");
  SPG_CHECK(ctx, (size_t)kTableRows * (g->n + 1) < 0x7fffffffULL, "generator table too large");

  uint32_t* hist = (uint32_t*)ws_get(ctx, 1, (nkeys + 1) * 4);
  uint32_t* off = (uint32_t*)ws_get(ctx, 2, (nkeys + 1) * 4);
  uint32_t* cursor = (uint32_t*)ws_get(ctx, 3, (nkeys + 1) * 4);
  uint32_t* items = (uint32_t*)ws_get(ctx, 4, (nkeys + 1) * 4);
  uint32_t* item_off = (uint32_t*)ws_get(ctx, 5, (nkeys + 1) * 4);
  uint32_t* entries = (uint32_t*)ws_get(ctx, 6, max_entries * 4 + 4);
  uint32_t* item_key = (uint32_t*)ws_get(ctx, 7, max_items * 4);
  Ext* partial = (Ext*)ws_get(ctx, 8, max_items * sizeof(Ext));
  const int m = NB < seg_m ? NB : seg_m;  // buckets per segment
  const int S = NB / m;
  int log2m = 0;
  while ((1 << log2m) < m) log2m++;
  Ext* segT = (Ext*)ws_get(ctx, 9, B * (size_t)S * sizeof(Ext));
  Ext* segS = (Ext*)ws_get(ctx, 10, B * (size_t)S * sizeof(Ext));
  if (!hist || !off || !cursor || !items || !item_off || !entries || !item_key || !partial || !segT || !segS)
    return set_err(ctx, SPG_E_NOMEM, "msm workspace allocation failed");

  // many MSMs: one workgroup per MSM sorts its digits in LDS (k_digits_rows; up to 2^15 bucket counters,
  // 128 KiB of the 160 KiB LDS, at c = 16)
  static const int rows_cmax = getenv("SPG_ROWS_CMAX") ? atoi(getenv("SPG_ROWS_CMAX")) : 16;
  const bool rows = B >= 64 && c <= rows_cmax;
  if (rows) {
    SPG_HIP(ctx, hipMemsetAsync(hist + nkeys, 0, 4, s));
  } else {
    SPG_HIP(ctx, hipMemsetAsync(hist, 0, (nkeys + 1) * 4, s));
    SPG_HIP(ctx, hipMemsetAsync(cursor, 0, (nkeys + 1) * 4, s));
  }

  MsmArgs a;
  a.scalars = d_scalars;
  a.blinds = d_blinds;
  a.B = (int)B;
  a.n = (int)n;
  a.n1 = (int)(g->n + 1);
  a.gen_offset = (int)gen_offset;
  a.h_index = h_index < 0 ? (int)g->n : (int)h_index;
  a.idx = d_idx;
  a.hist = hist;
  a.off = off;
  a.off_out = off;
  a.cursor = cursor;
  a.entries = entries;

  size_t tmp_bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, hist, off, (int)(nkeys + 1), s);
  void* tmp = ws_get(ctx, 11, tmp_bytes + 16);
  if (!tmp) return set_err(ctx, SPG_E_NOMEM, "scan workspace");
  if (rows) {
    KScope ks(ctx, "msm_digits_rows");
    dispatch_digits_rows(c, a, s);
  } else {
    KScope ks(ctx, "msm_count");
    dispatch_digits(c, a, true, s);
  }
  SPG_HIP(ctx, hipGetLastError());

  // scans over nkeys+1 entries (hist[nkeys] == 0 so off[nkeys] = total entries)
  if (!rows) SPG_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, hist, off, (int)(nkeys + 1), s));
  hipLaunchKernelGGL(k_item_counts, dim3((unsigned)((nkeys + 1 + 255) / 256)), dim3(256), 0, s, hist, items,
                     (int)nkeys, (uint32_t)item_k);
  SPG_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, items, item_off, (int)(nkeys + 1), s));

  if (!rows) {
    KScope ks(ctx, "msm_scatter");
    dispatch_digits(c, a, false, s);
  }
  hipLaunchKernelGGL(k_item_keys, dim3((unsigned)((nkeys + 255) / 256)), dim3(256), 0, s, item_off, item_key,
                     (int)nkeys);
  // the item count is only known on the device: launch the upper bound, threads past item_off[nkeys] exit
  {
    KScope ks(ctx, "msm_bucket_items", 0.0, madds_model((double)B * per, c));
    hipLaunchKernelGGL(k_items, dim3((unsigned)((max_items + 255) / 256)), dim3(256), 0, s, item_key, item_off,
                       off, hist, entries, g->table, partial, item_off + nkeys);
  }
  {
    KScope ks(ctx, "msm_segments");
    static const size_t seg_quad_max = getenv("SPG_SEG_QUAD_MAX") ? atol(getenv("SPG_SEG_QUAD_MAX")) : 16384;
    if (use_quad() && B * (size_t)S <= seg_quad_max)
      hipLaunchKernelGGL(k_segments_q, dim3((unsigned)((4 * B * S + 255) / 256)), dim3(256), 0, s, item_off, partial,
                         segT, segS, (int)B, NB, m);
    else
      hipLaunchKernelGGL(k_segments, dim3((unsigned)((B * S + 63) / 64)), dim3(64), 0, s, item_off, partial, segT,
                         segS, (int)B, NB, m);
  }
  {
    KScope ks(ctx, "msm_final");
    if (use_quad())
    {
      // encodings one lane per MSM (k_compress_ext) instead of on one lane of each k_final block: the
      // ~250 dependent squarings of an encoding would otherwise serialise behind every block's tree
      Ext* ext = d_ext;
      if (!ext && d_out) ext = (Ext*)ws_get(ctx, 17, B * sizeof(Ext) + 64);
      if (!ext) return set_err(ctx, SPG_E_NOMEM, "msm final points");
      const Ext *fT = segT, *fS = segS;
      int fSn = S, flog2m = log2m;
      if (B <= 16 && S > 1024) {  // few MSMs with many segments: regroup 8 segments per group first
        const int lg = 3, G = S >> lg;
        Ext* rT = (Ext*)ws_get(ctx, 18, 2 * B * (size_t)G * sizeof(Ext) + 64);
        if (!rT) return set_err(ctx, SPG_E_NOMEM, "msm regroup");
        Ext* rS = rT + B * (size_t)G;
        hipLaunchKernelGGL(k_regroup_q, dim3((unsigned)((4 * B * (size_t)G + 255) / 256)), dim3(256), 0, s, segT,
                           segS, (int)B, S, lg, log2m, rT, rS);
        fT = rT;
        fS = rS;
        fSn = G;
        flog2m = log2m + lg;
      }
      // many MSMs fill the chip with blocks: fewer slots per MSM do less redundant scan work (the Hillis-Steele
      // scan costs SL log SL additions), few MSMs need the shortest dependent chain
      static const int sl_env = getenv("SPG_FINAL_SL") ? atoi(getenv("SPG_FINAL_SL")) : 0;
      const int sl = sl_env ? sl_env : (B >= 256 ? 32 : 128);  // B = 1024 rows: 414 -> 155 us (MI355X)
      if (sl == 32)
        hipLaunchKernelGGL(k_final_q<32>, dim3((unsigned)B), dim3(128), 0, s, fT, fS, nullptr, fSn, flog2m, ext);
      else if (sl == 64)
        hipLaunchKernelGGL(k_final_q<64>, dim3((unsigned)B), dim3(256), 0, s, fT, fS, nullptr, fSn, flog2m, ext);
      else
        hipLaunchKernelGGL(k_final_q<128>, dim3((unsigned)B), dim3(512), 0, s, fT, fS, nullptr, fSn, flog2m, ext);
      if (d_out)
        hipLaunchKernelGGL(k_compress_ext, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, ext, B, d_out);
    }
    else
      hipLaunchKernelGGL(k_final, dim3((unsigned)B), dim3(256), 0, s, segT, segS, d_out, S, log2m, d_ext);
  }
  SPG_HIP(ctx, hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ generator handles
// HBM bytes of the 2^k G_i tables of all live generator sets (spg_comb_stats)
std::atomic<size_t> g_gens_table_bytes{0};

static int gens_finish(spg_ctx* ctx, spg_gens* g) {
  hipStream_t s = ctx->stream;
  size_t n1 = g->n + 1;
  size_t tab_entries = n1 * (size_t)kTableRows;
  SPG_HIP(ctx, hipMalloc(&g->table, tab_entries * sizeof(Niels)));
  g_gens_table_bytes += tab_entries * sizeof(Niels);
  hipLaunchKernelGGL(k_table, dim3((unsigned)((tab_entries + 255) / 256)), dim3(256), 0, s, g->niels, g->table,
                     (int)n1);
  SPG_HIP(ctx, hipGetLastError());
  SPG_HIP(ctx, hipStreamSynchronize(s));
  return 0;
}

}  // namespace spg

using namespace spg;

extern "C" int spg_gens_derive(spg_ctx* ctx, const uint8_t* label, size_t label_len, size_t n, spg_gens** out) {
  if (!ctx || !out || (!label && label_len)) return SPG_E_ARG;
  size_t n1 = n + 1;
  if (n1 * (size_t)kTableRows >= 0x7fffffffULL) return set_err(ctx, SPG_E_ARG, "too many generators");
  // SHAKE256(label || basepoint) stream, 64 bytes per point (host; sequential XOF)
  std::vector<uint8_t> uni(64 * n1);
  {
    Shake256 sh;
    sh.update(label, label_len);
    static const uint8_t B[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9,
                                  0x61, 0xc5, 0x00, 0x51, 0x5f, 0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82,
                                  0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};
    sh.update(B, 32);
    sh.read(uni.data(), uni.size());
  }
  spg_gens* g = new spg_gens();
  g->n = n;
  g->compressed = new uint8_t[32 * n1];
  hipStream_t s = ctx->stream;
  uint8_t* d_uni = nullptr;
  uint8_t* d_comp = nullptr;
  if (hipMalloc(&d_uni, uni.size()) != hipSuccess || hipMalloc(&d_comp, 32 * n1) != hipSuccess ||
      hipMalloc(&g->niels, n1 * sizeof(Niels)) != hipSuccess) {
    delete g;
    return set_err(ctx, SPG_E_NOMEM, "gens allocation");
  }
  SPG_HIP(ctx, hipMemcpyAsync(d_uni, uni.data(), uni.size(), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_map_uniform, dim3((unsigned)((n1 + 63) / 64)), dim3(64), 0, s, d_uni, g->niels, d_comp,
                     (int)n1);
  SPG_HIP(ctx, hipGetLastError());
  SPG_HIP(ctx, hipMemcpyAsync(g->compressed, d_comp, 32 * n1, hipMemcpyDeviceToHost, s));
  int rc = gens_finish(ctx, g);
  hipFree(d_uni);
  hipFree(d_comp);
  if (rc) {
    spg_gens_free(ctx, g);
    return rc;
  }
  *out = g;
  return SPG_OK;
}

extern "C" int spg_gens_upload(spg_ctx* ctx, const uint8_t* compressed, size_t n, spg_gens** out) {
  if (!ctx || !out || !compressed) return SPG_E_ARG;
  size_t n1 = n + 1;
  if (n1 * (size_t)kTableRows >= 0x7fffffffULL) return set_err(ctx, SPG_E_ARG, "too many generators");
  spg_gens* g = new spg_gens();
  g->n = n;
  g->compressed = new uint8_t[32 * n1];
  memcpy(g->compressed, compressed, 32 * n1);
  hipStream_t s = ctx->stream;
  uint8_t* d_comp = nullptr;
  int* d_bad = nullptr;
  if (hipMalloc(&d_comp, 32 * n1) != hipSuccess || hipMalloc(&d_bad, sizeof(int)) != hipSuccess ||
      hipMalloc(&g->niels, n1 * sizeof(Niels)) != hipSuccess) {
    delete g;
    return set_err(ctx, SPG_E_NOMEM, "gens allocation");
  }
  SPG_HIP(ctx, hipMemcpyAsync(d_comp, compressed, 32 * n1, hipMemcpyHostToDevice, s));
  SPG_HIP(ctx, hipMemsetAsync(d_bad, 0, sizeof(int), s));
  hipLaunchKernelGGL(k_decompress, dim3((unsigned)((n1 + 63) / 64)), dim3(64), 0, s, d_comp, g->niels, d_bad,
                     (int)n1);
  int bad = 0;
  SPG_HIP(ctx, hipMemcpyAsync(&bad, d_bad, sizeof(int), hipMemcpyDeviceToHost, s));
  SPG_HIP(ctx, hipStreamSynchronize(s));
  hipFree(d_comp);
  hipFree(d_bad);
  if (bad) {
    spg_gens_free(ctx, g);
    return set_err(ctx, SPG_E_POINT, "invalid compressed generator");
  }
  int rc = gens_finish(ctx, g);
  if (rc) {
    spg_gens_free(ctx, g);
    return rc;
  }
  *out = g;
  return SPG_OK;
}

extern "C" int spg_gens_download(spg_ctx* ctx, const spg_gens* g, uint8_t* out) {
  if (!ctx || !g || !out) return SPG_E_ARG;
  memcpy(out, g->compressed, 32 * (g->n + 1));
  return SPG_OK;
}

extern "C" size_t spg_gens_n(const spg_gens* g) { return g ? g->n : 0; }

extern "C" int spg_gens_free(spg_ctx* ctx, spg_gens* g) {
  (void)ctx;
  if (!g) return SPG_OK;
  if (g->niels) hipFree(g->niels);
  if (g->table) {
    hipFree(g->table);
    g_gens_table_bytes -= (g->n + 1) * (size_t)kTableRows * sizeof(Niels);
  }
  comb_free(g);
  delete[] g->compressed;
  delete g;
  return SPG_OK;
}

namespace spg {
// one large MSM (msm_big.hip): sum_i s_i G[gen_offset + i] (+ blind h) of n device scalars into a host point
int msm_single_big(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n,
                   const Fq* d_blind, h::HExt* out);
}  // namespace spg
static bool use_big() {
  static const bool on = !getenv("SPG_MSM_BIG") || atoi(getenv("SPG_MSM_BIG")) != 0;
  return on;
}

static int msm_host(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const uint64_t* scalars, size_t n, size_t B,
                    const uint64_t* blinds, uint8_t* out) {
  if (!ctx || !g || !out || (!scalars && n)) return SPG_E_ARG;
  if (n == 0 && !blinds) {
    // empty MSM: identity, whose encoding is 32 zero bytes
    memset(out, 0, 32 * B);
    return SPG_OK;
  }
  if (gen_offset + n > g->n) return set_err(ctx, SPG_E_ARG, "MSM longer than the generator set");
  hipStream_t s = ctx->stream;
  size_t sb = B * n * sizeof(Fq);
  Fq* d_s = (Fq*)ws_get(ctx, 0, sb + B * sizeof(Fq) + B * 32 + 64);
  if (!d_s) return set_err(ctx, SPG_E_NOMEM, "scalar upload");
  Fq* d_bl = blinds ? d_s + B * n : nullptr;
  uint8_t* d_out = (uint8_t*)(d_s + B * n + B);
  if (n) SPG_HIP(ctx, hipMemcpyAsync(d_s, scalars, sb, hipMemcpyHostToDevice, s));
  if (blinds) SPG_HIP(ctx, hipMemcpyAsync(d_bl, blinds, B * sizeof(Fq), hipMemcpyHostToDevice, s));
  const bool small = B <= kSmallMaxB && n + (blinds ? 1 : 0) <= kSmallMaxN;
  if (!small && B == 1 && n && use_big()) {  // one large MSM (config 2): msm_big.hip, encoded on the host
    h::HExt r;
    timer_start(ctx);
    int rc = msm_single_big(ctx, g, gen_offset, d_s, n, d_bl, &r);
    timer_stop(ctx);
    if (rc) return rc;
    h::hext_compress(r, out);
    float ms = 0.f;
    hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
    ctx->last_us = ms * 1000.0;
    return SPG_OK;
  }
  Ext* d_ext = small ? (Ext*)ws_get(ctx, 14, B * sizeof(Ext) + 64) : nullptr;
  if (small && !d_ext) return set_err(ctx, SPG_E_NOMEM, "msm output");
  timer_start(ctx);
  int rc = small ? msm_small_device(ctx, g, gen_offset, d_s, n, B, d_bl, d_ext, nullptr, -1)
                 : msm_batch_device(ctx, g, gen_offset, d_s, n, B, d_bl, d_out, nullptr, -1);
  if (rc) return rc;
  timer_stop(ctx);
  if (small) {
    std::vector<Ext> r(B);
    SPG_HIP(ctx, hipMemcpyAsync(r.data(), d_ext, B * sizeof(Ext), hipMemcpyDeviceToHost, s));
    SPG_HIP(ctx, hipStreamSynchronize(s));
    for (size_t b = 0; b < B; b++) h::hext_compress(h::hext_from_dev(r[b]), out + 32 * b);
  } else {
    SPG_HIP(ctx, hipMemcpyAsync(out, d_out, 32 * B, hipMemcpyDeviceToHost, s));
    SPG_HIP(ctx, hipStreamSynchronize(s));
  }
  float ms = 0.f;
  hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  ctx->last_us = ms * 1000.0;
  return SPG_OK;
}

extern "C" int spg_msm(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const uint64_t* scalars_mont, size_t n,
                       const uint64_t* blind_mont, uint8_t out[32]) {
  return msm_host(ctx, g, gen_offset, scalars_mont, n, 1, blind_mont, out);
}

// sum_i d_s[i] G[gen_offset + i] of n device scalars, uncompressed: X, Y, Z, T as 32 little-endian bytes each
static int msm_partial_dev(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_s, size_t n,
                           uint8_t out_ext[128]) {
  hipStream_t s = ctx->stream;
  if (n > kSmallMaxN && use_big()) {  // msm_big.hip; the host point's coordinates as canonical bytes
    h::HExt r;
    timer_start(ctx);
    int rc = msm_single_big(ctx, g, gen_offset, d_s, n, nullptr, &r);
    timer_stop(ctx);
    if (rc) return rc;
    h::fe_to_bytes(r.X, out_ext);
    h::fe_to_bytes(r.Y, out_ext + 32);
    h::fe_to_bytes(r.Z, out_ext + 64);
    h::fe_to_bytes(r.T, out_ext + 96);
  } else {
    Ext* d_ext = (Ext*)ws_get(ctx, 19, sizeof(Ext) + 64);
    if (!d_ext) return set_err(ctx, SPG_E_NOMEM, "msm output");
    timer_start(ctx);
    int rc = n <= kSmallMaxN ? msm_small_device(ctx, g, gen_offset, d_s, n, 1, nullptr, d_ext, nullptr, -1)
                             : msm_batch_device(ctx, g, gen_offset, d_s, n, 1, nullptr, nullptr, nullptr, -1, d_ext);
    if (rc) return rc;
    timer_stop(ctx);
    Ext r;
    SPG_HIP(ctx, hipMemcpyAsync(&r, d_ext, sizeof(Ext), hipMemcpyDeviceToHost, s));
    SPG_HIP(ctx, hipStreamSynchronize(s));
    static_assert(sizeof(Ext) == 128, "Ext is X, Y, Z, T of 32 bytes");
    memcpy(out_ext, &r, sizeof(Ext));
  }
  float ms = 0.f;
  hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  ctx->last_us = ms * 1000.0;
  return SPG_OK;
}

// one shard of an MSM that is split over devices: the sum stays uncompressed so that the partials
// of all ranks add exactly; spg_points_sum_compress adds and encodes them on the host
extern "C" int spg_msm_partial(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const uint64_t* scalars_mont,
                               size_t n, uint8_t out_ext[128]) {
  if (!ctx || !g || !out_ext || (!scalars_mont && n)) return SPG_E_ARG;
  if (gen_offset + n > g->n) return set_err(ctx, SPG_E_ARG, "MSM longer than the generator set");
  if (n == 0) {
    const Ext id = ext_identity();
    memcpy(out_ext, &id, sizeof(Ext));
    return SPG_OK;
  }
  Fq* d_s = (Fq*)ws_get(ctx, 0, n * sizeof(Fq) + 64);
  if (!d_s) return set_err(ctx, SPG_E_NOMEM, "scalar upload");
  SPG_HIP(ctx, hipMemcpyAsync(d_s, scalars_mont, n * sizeof(Fq), hipMemcpyHostToDevice, ctx->stream));
  return msm_partial_dev(ctx, g, gen_offset, d_s, n, out_ext);
}

// the same over scalars already resident in HBM: buf[offset .. offset + n)
extern "C" int spg_msm_partial_buf(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const spg_buf* buf,
                                   size_t offset, size_t n, uint8_t out_ext[128]) {
  if (!ctx || !g || !buf || !out_ext) return SPG_E_ARG;
  if (offset > buf->n || n > buf->n - offset) return set_err(ctx, SPG_E_ARG, "msm_partial_buf: range past the buffer");
  if (gen_offset + n > g->n) return set_err(ctx, SPG_E_ARG, "MSM longer than the generator set");
  if (n == 0) {
    const Ext id = ext_identity();
    memcpy(out_ext, &id, sizeof(Ext));
    return SPG_OK;
  }
  return msm_partial_dev(ctx, g, gen_offset, buf->d + offset, n, out_ext);
}

// GroupElement::vartime_multiscalar_mul over resident scalars, compressed
extern "C" int spg_msm_buf(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const spg_buf* buf, size_t offset,
                           size_t n, uint8_t out[32]) {
  uint8_t ext[128];
  const int rc = spg_msm_partial_buf(ctx, g, gen_offset, buf, offset, n, ext);
  if (rc) return rc;
  return spg_points_sum_compress(ext, 1, out);
}

// host only (no device): sum of k partial points (X, Y, Z, T; 32 little-endian bytes each, any representative
// below 2^256 of the coordinate mod 2^255 - 19) and its RFC 9496 encoding
extern "C" int spg_points_sum_compress(const uint8_t* parts, size_t k, uint8_t out[32]) {
  if (!out || (!parts && k)) return SPG_E_ARG;
  h::HExt acc = h::hext_identity();
  for (size_t i = 0; i < k; i++) {
    Ext e;
    memcpy(&e, parts + 128 * i, sizeof(Ext));
    acc = h::hext_add(acc, h::hext_from_dev(e));
  }
  h::hext_compress(acc, out);
  return SPG_OK;
}

extern "C" int spg_commit_rows(spg_ctx* ctx, const spg_gens* g, const uint64_t* Z_mont, size_t L, size_t R,
                               const uint64_t* blinds_mont, uint8_t* out) {
  if (L == 0) return SPG_OK;
  return msm_host(ctx, g, 0, Z_mont, R, L, blinds_mont, out);
}

// B row MSMs of n device scalars (as msm_batch_device, gen_offset 0) with their encodings on the host (out: 32 B each):
// where the comb applies (msm_batch_device's size rule), the rows' halves (scalars and blinds times 2^-1 mod l) come
// back for the host pool's batched encoding of doubles (encode_halved_host) instead of k_compress_ext's lane-per-point
// inverse square roots; else msm_batch_device's device encodings, downloaded. SPG_HALVED_ENC=0: always the latter.
int spg::msm_rows_host_enc(spg_ctx* ctx, const spg_gens* g, const Fq* d_scalars, size_t n, size_t B,
                           const Fq* d_blinds, long h_index, uint8_t* out, bool timed) {
  static const bool halve = !getenv("SPG_HALVED_ENC") || atoi(getenv("SPG_HALVED_ENC")) != 0;
  hipStream_t s = ctx->stream;
  const size_t tot = B * (n + (d_blinds ? 1 : 0));
  const bool comb = B >= 64 && (n <= 1024 ? tot >= ((size_t)1 << 14) : (n <= 16384 && tot >= ((size_t)1 << 22)));
  if (halve && comb && B >= 384) {  // (fewer rows: spark.hip kHalvedMin)
    Ext* ext = (Ext*)ws_get(ctx, 17, B * sizeof(Ext) + 64);
    if (!ext) return set_err(ctx, SPG_E_NOMEM, "msm comb points");
    const int hi = !d_blinds ? -1 : (h_index < 0 ? (int)g->n : (int)h_index);
    const int rc = msm_comb(ctx, g, 0, d_scalars, n, B, d_blinds, nullptr, hi, ext, true);
    if (rc == SPG_OK) {
      if (timed) timer_stop(ctx);
      Ext* h = (Ext*)enc_stage_get(ctx, B * sizeof(Ext));
      if (!h) return set_err(ctx, SPG_E_NOMEM, "encoding staging");
      SPG_HIP(ctx, hipMemcpyAsync(h, ext, B * sizeof(Ext), hipMemcpyDeviceToHost, s));
      SPG_HIP(ctx, hipStreamSynchronize(s));
      encode_halved_host(h, B, reinterpret_cast<Pt*>(out));
      return SPG_OK;
    }
    if (rc != kCombSkip) return rc;
  }
  uint8_t* d_out = (uint8_t*)ws_get(ctx, 12, 32 * B + 64);
  if (!d_out) return set_err(ctx, SPG_E_NOMEM, "commit rows out");
  const int rc = msm_batch_device(ctx, g, 0, d_scalars, n, B, d_blinds, d_out, nullptr, h_index);
  if (rc) return rc;
  if (timed) timer_stop(ctx);
  SPG_HIP(ctx, hipMemcpyAsync(out, d_out, 32 * B, hipMemcpyDeviceToHost, s));
  SPG_HIP(ctx, hipStreamSynchronize(s));
  return SPG_OK;
}

extern "C" int spg_commit_rows_buf(spg_ctx* ctx, const spg_gens* g, const spg_buf* Z, size_t offset, size_t L,
                                   size_t R, const spg_buf* blinds, uint8_t* out) {
  if (!ctx || !g || !Z || !out) return SPG_E_ARG;
  if (offset + L * R > Z->n) return set_err(ctx, SPG_E_ARG, "commit_rows_buf: Z too short");
  if (blinds && blinds->n < L) return set_err(ctx, SPG_E_ARG, "commit_rows_buf: blinds too short");
  if (R > g->n) return set_err(ctx, SPG_E_ARG, "commit_rows_buf: R exceeds generators");
  if (L == 0) return SPG_OK;
  timer_start(ctx);
  // the stop event is recorded after the device work, before the download and the host encodings, so
  // spg_last_kernel_us is device time like every other MSM entry point's
  const int rc = msm_rows_host_enc(ctx, g, Z->d + offset, R, L, blinds ? blinds->d : nullptr, -1, out, true);
  if (rc) return rc;
  SPG_HIP(ctx, hipEventSynchronize(ctx->ev1));
  float ms = 0.f;
  hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  ctx->last_us = ms * 1000.0;
  return SPG_OK;
}
