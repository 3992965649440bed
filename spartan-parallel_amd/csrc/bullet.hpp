// spg — the device Bullet round kernel (one launch per round of BulletReductionProof::prove); msm.hip
// launches it, scripts/micro/bullet_phases.hip times its phases.
#pragma once
#include <hip/hip_runtime.h>

#include "ctx.hpp"
#include "lds.hpp"
#include "quad.hpp"

namespace spg {

// ---- one Bullet round on the device (BulletReductionProof::prove, src/nizk/bullet.rs:32-132) ----------
// Round k of a DotProductProofLog of size n holds a^(k) (nk = n >> k entries, Montgomery) and the generator
// weights cw (n entries, kept as plain integers so that a Montgomery product with them is already the
// canonical scalar). Its L and R are fixed-base MSMs over n/2 ORIGINAL generators each (proto.hip):
//   L: p -> a^(k)[p mod nh] * cw[(p / nh) nk + nh + p mod nh],   R: p -> a^(k)[nh + p mod nh] * cw[(p / nh) nk + p mod nh]
// with nh = nk / 2. For k >= 1 the kernel first applies round k-1's fold with (u, u^-1) from the kernel
// arguments: a^(k)[i] = u a[i] + u^-1 a[i + nk], cw[j] *= (j mod 2nk < nk ? u^-1 : u). Every workgroup
// (bucket v, MSM b) recomputes the scalars of its MSM; the v = 1 workgroups also write the folded state
// (double-buffered: in and out never alias) for the next round. So a round needs no host-computed
// scalars, no host-to-device copy and one launch: the host sends (u, u^-1) and reads back NB bucket sums
// per MSM (coherent mapped memory), whose completion the last workgroup posts to the mailbox.
struct BulletArgs {
  const Fq* aa_in;
  const Fq* cw_in;
  Fq* aa_out;
  Fq* cw_out;
  const uint32_t* gidx;  // generator index of weight j (n entries)
  Fq u, uinv;
  int k, n, nk, n1;
  const Niels* tab;
  Ext* buckets;  // B = 2 bucket sets of NB + 1 (the last: top-window carries; mapped host memory)
  unsigned* counter;
  uint32_t* mb;
  uint32_t seq;
  unsigned long long* probe;  // optional phase timestamps (scripts/micro/bullet_phases.hip), null in the product
};

template <int C, int BS>
__global__ void __launch_bounds__(BS) k_bullet_round_q(BulletArgs a) {
  constexpr int W = 253 / C + 1;
  constexpr int NB = 1 << (C - 1);
  constexpr uint32_t MASK = (1u << C) - 1u;
  constexpr int S = BS / 4;  // quads
  __shared__ uint32_t list[BS * W];
  __shared__ uint32_t pts[soa_words<Ext, S>()];
  __shared__ uint32_t cnt;
  __shared__ bool last;
  // v = 1 .. NB: bucket v; v = NB + 1: the top window's digits of magnitude 1 (the final carries of the signed
  // recoding: about every second scalar, which would nearly double bucket 1's entries and with it the kernel's
  // critical path), summed apart and added with weight 1 on the host
  const int v = blockIdx.x + 1, b = blockIdx.y, t = threadIdx.x, q = t & 3, slot = t >> 2;
  const bool carry_wg = v == NB + 1;
  const int P = a.n / 2, nk = a.nk, nh = nk / 2;
  const bool writer = blockIdx.x == 0;
  Ext acc = ext_identity();
  if (t == 0) cnt = 0;
  unsigned long long* pr = a.probe ? a.probe + 8 * (blockIdx.y * gridDim.x + blockIdx.x) : nullptr;
  if (pr && t == 0) pr[0] = wall_clock64();
  __syncthreads();
  for (int base = 0; base < P; base += BS) {
    const int p = base + t;
    if (p < P) {
      const int blk = p / nh, off = p - blk * nh;
      const int ia = b ? off + nh : off;
      const int j = blk * nk + (b ? 0 : nh) + off;
      Fq av, cv;
      if (a.k == 0) {
        av = a.aa_in[ia];
        cv = fq_zero();
        cv.l[0] = 1u;
      } else {
        av = fq_add(fq_mul(a.aa_in[ia], a.u), fq_mul(a.uinv, a.aa_in[ia + nk]));
        cv = fq_mul(a.cw_in[j], (j & (2 * nk - 1)) < nk ? a.uinv : a.u);
      }
      if (writer) {
        if (blk == 0) a.aa_out[ia] = av;
        a.cw_out[j] = cv;
      }
      const Fq k = fq_mul(av, cv);  // canonical scalar (cw is a plain integer)
      const uint32_t gi = a.gidx[j];
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
        const bool top1 = w == W - 1 && (d == 1 || d == -1);
        if (carry_wg ? top1 : ((d == v || d == -v) && !top1)) {
          const uint32_t pos = atomicAdd(&cnt, 1u);
          list[pos] = (uint32_t)((size_t)(w * C) * a.n1 + gi) | (d < 0 ? 0x80000000u : 0u);
        }
      }
    }
    __syncthreads();
    if (pr && t == 0 && base == 0) pr[1] = wall_clock64();
    const uint32_t m = cnt;
    // software-pipelined: the table coordinate of entry e + S is loaded while entry e is added
    uint32_t e = slot;
    Fp qv;
    bool neg = false;
    if (e < m) qv = niels_coord(a.tab, list[e], q, &neg);
    while (e < m) {
      const uint32_t e2 = e + S;
      Fp qn;
      bool nn = false;
      if (e2 < m) qn = niels_coord(a.tab, list[e2], q, &nn);
      acc = quad_madd(acc, qv, neg, q);
      qv = qn;
      neg = nn;
      e = e2;
    }
    __syncthreads();
    if (t == 0) cnt = 0;
    __syncthreads();
  }
  if (pr && t == 0) pr[2] = wall_clock64();
  for (int d = S / 2; d >= 1; d >>= 1) {
    if (slot >= d && slot < 2 * d) quad_put_op<S>(pts, slot - d, acc, q);
    __syncthreads();
    if (slot < d) acc = quad_add_op(acc, quad_get_op<S>(pts, slot, q), q);
    __syncthreads();
  }
  if (pr && t == 0) pr[3] = wall_clock64();
  if (t == 0) {
    a.buckets[(size_t)b * (NB + 1) + (v - 1)] = acc;
    // the bucket (mapped host memory) and the folded state (HBM) before the ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           gridDim.x * gridDim.y - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      mbox_post(a.mb, a.seq, nullptr, 0);
    }
    if (pr) pr[4] = wall_clock64();
  }
}

// ---- one Bullet round from the comb table (the default device form) -------------------------------------
// The same round as k_bullet_round_q, without buckets. The L and R MSMs are over the ORIGINAL generators G_0..G_{n-1}
// of the proof, whose generator set keeps the comb table of comb.hip: comb[w][s][m - 1] = m 2^(C w) G_s (C = 12, or
// 13 for the 2^14-generator tables). A C-bit signed digit d of scalar p in window w is then one entry
// +-comb[w][gidx_p][|d| - 1] (packed as a 31-bit entry index: < 2^31 for every table comb.hip builds at C >= 12), and
// an MSM is a plain sum of its W P entries (W = 22, or 20 at C = 13) -- no bucket weights, so the host finishes with a plain sum of partial points instead of the
// buckets' running sums, and no workgroup needs more than its own scalars:
//   quad (p, j) of MSM b (G quads per scalar) adds the entries of windows j*WG .. j*WG + WG - 1 of scalar p
//   (WG = ceil(22 / G) dependent quad mixed additions), its Niels coordinates all loaded up front;
//   the workgroup's BS/4 quad sums meet in an LDS quad tree down to R points, written to parts[b][wg][0..R).
// The scalar of quad (p, j): its three operand products of the fold (u a[ia], u^-1 a[ia + nk], cw[j] f) are one
// product on lanes 0..2 of the quad (operands selected per lane), then av = lane0 + lane1, cv = lane2 by DPP and
// k = av cv: two dependent field products instead of four. The j = 0 quads of workgroup column 0 write the folded
// state for the next round (every (ia, jw) pair once), as k_bullet_round_q's v = 1 workgroups do.
struct BulletCombArgs {
  const Fq* aa_in;
  const Fq* cw_in;
  Fq* aa_out;
  Fq* cw_out;
  const uint32_t* gidx;  // generator index of weight j (n entries)
  Fq u, uinv;
  int k, n, nk;
  const Niels* comb;
  int NS;        // comb slots + 1 (the h slot): the stride between windows is NS * 2^(C-1) entries
  int R;         // points each workgroup leaves (a power of two <= BS / 4)
  Ext* parts;    // [2][gridDim.x][R] (mapped host memory)
  unsigned* counter;
  uint32_t* mb;
  uint32_t seq;
  int st;        // comb entry stride (32-byte coordinates)
  unsigned long long* probe = nullptr;  // per-workgroup phase clocks (scripts/micro/bullet_comb_phases.hip), or null
};

__device__ __forceinline__ Fq fq_qbcast_lane(const Fq& a, int lane) {
  Fp x;
#pragma unroll
  for (int i = 0; i < 8; i++) x.l[i] = a.l[i];
  Fp r = lane == 0 ? fp_qbcast<0>(x) : (lane == 1 ? fp_qbcast<1>(x) : fp_qbcast<2>(x));
  Fq o;
#pragma unroll
  for (int i = 0; i < 8; i++) o.l[i] = r.l[i];
  return o;
}

// The comb entries of windows w0 .. w0 + WG - 1 of canonical scalar k on generator slot s (signed C-bit digits):
// ent[x] = entry index of window w0 + x | sign << 31, or ~0 for a zero digit or a window past the last (a short last
// group). Selects, no branches: the recode sits on a Bullet round's latency path (scripts/micro/bullet_comb_phases:
// recode + entry loads 2.5 -> 1.25 us against the shift-register form with its per-window branches).
template <int C, int WG>
__device__ __forceinline__ void comb_window_entries(const Fq& k, int w0, int s, int NS, uint32_t (&ent)[WG]) {
  constexpr int W = 253 / C + 1, NB = 1 << (C - 1);
  constexpr uint32_t MASK = (1u << C) - 1u;
#pragma unroll
  for (int x = 0; x < WG; x++) ent[x] = 0xffffffffu;
  int carry = 0;
  const uint32_t sb = (uint32_t)s * NB - 1u, wst = (uint32_t)NS * NB;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const int bit = w * C;
    const int li = bit >> 5, of = bit & 31;
    uint32_t v = k.l[li] >> of;
    if (of + C > 32 && li + 1 < 8) v |= k.l[li + 1] << (32 - of);
    int d = (int)(v & MASK) + carry;
    carry = d > NB ? 1 : 0;
    d -= carry << C;
    // (w NS + s) NB + |d| - 1, the sign in bit 31; all ones for d = 0
    const uint32_t e = (w * wst + sb + (uint32_t)abs(d)) | ((uint32_t)d & 0x80000000u) | (uint32_t)-(int)(d == 0);
#pragma unroll
    for (int x = 0; x < WG; x++) ent[x] = w == w0 + x ? e : ent[x];
  }
}

template <int C, int G, int BS>
__global__ void __launch_bounds__(BS) k_bullet_comb(BulletCombArgs a) {
  constexpr int W = 253 / C + 1, WG = (W + G - 1) / G, S = BS / 4;
  __shared__ uint32_t pts[soa_words<Ext, S>()];
  __shared__ bool last;
  const int b = blockIdx.y, t = threadIdx.x, q = t & 3, slot = t >> 2;
  const int P = a.n / 2, nk = a.nk, nh = nk / 2;
  const int gq = blockIdx.x * S + slot;  // quad index within MSM b
  const int p = gq / G, jg = gq - p * G, w0 = jg * WG;
  unsigned long long* pr = a.probe ? a.probe + 8 * (blockIdx.y * gridDim.x + blockIdx.x) : nullptr;
  if (pr && t == 0) pr[0] = wall_clock64();
  Ext acc = ext_identity();
  if (p < P) {
    const int blk = p / nh, off = p - blk * nh;
    const int ia = b ? off + nh : off;
    const int j = blk * nk + (b ? 0 : nh) + off;
    Fq av, cv;
    if (a.k == 0) {
      av = a.aa_in[ia];
      cv = fq_zero();
      cv.l[0] = 1u;  // cw = 1: the product below takes av out of Montgomery form
    } else {
      // lanes 0, 1, 2: u a[ia], u^-1 a[ia + nk], cw[j] f; lane 3 repeats lane 0. Every lane loads both operands
      // and selects after: a per-lane choice between the by-value struct's two base pointers otherwise becomes a vector
      // load of the pointer from the kernel arguments that the operand load waits on (one memory latency more on the
      // round's path)
      const Fq xa = a.aa_in[q == 1 ? ia + nk : ia];
      const Fq xc = a.cw_in[j];
      const Fq x = q == 2 ? xc : xa;
      const Fq y = q == 1 ? a.uinv : (q == 2 ? ((j & (2 * nk - 1)) < nk ? a.uinv : a.u) : a.u);
      const Fq r = fq_mul(x, y);
      av = fq_add(fq_qbcast_lane(r, 0), fq_qbcast_lane(r, 1));
      cv = fq_qbcast_lane(r, 2);
    }
    if (jg == 0 && q == 0) {  // the folded state, every (ia, j) once over the two MSMs
      if (blk == 0) a.aa_out[ia] = av;
      a.cw_out[j] = cv;
    }
    const Fq k = fq_mul(av, cv);  // canonical scalar (cw is a plain integer)
    if (pr) { asm volatile("" ::"v"(k.l[0])); if (t == 0) pr[1] = wall_clock64(); }
    const int s = (int)a.gidx[j];
    uint32_t ent[WG];
    comb_window_entries<C, WG>(k, w0, s, a.NS, ent);
    // every entry's coordinate in flight before the first addition
    Fp qv[WG];
    bool ng[WG];
#pragma unroll
    for (int x = 0; x < WG; x++)
      if (ent[x] != 0xffffffffu) qv[x] = niels_coord(a.comb, ent[x], q, &ng[x], a.st);
    if (pr) { asm volatile("" ::"v"(qv[WG - 1].l[0])); if (t == 0) pr[2] = wall_clock64(); }
#pragma unroll
    for (int x = 0; x < WG; x++)
      if (ent[x] != 0xffffffffu) acc = quad_madd(acc, qv[x], ng[x], q);
    if (pr) { asm volatile("" ::"v"(acc.X.l[0])); if (t == 0) pr[3] = wall_clock64(); }
  }
  for (int d = S / 2; d >= a.R; d >>= 1) {
    if (slot >= d && slot < 2 * d) quad_put_op<S>(pts, slot - d, acc, q);
    __syncthreads();
    if (slot < d) acc = quad_add_op(acc, quad_get_op<S>(pts, slot, q), q);
    __syncthreads();
  }
  if (pr) { asm volatile("" ::"v"(acc.X.l[0])); if (t == 0) pr[4] = wall_clock64(); }
  if (slot < a.R && q == 0) a.parts[((size_t)b * gridDim.x + blockIdx.x) * a.R + slot] = acc;
  __syncthreads();
  if (t == 0) {
    // the parts (mapped host memory) and the folded state (HBM) before the ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (pr) pr[5] = wall_clock64();
    last = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           gridDim.x * gridDim.y - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      mbox_post(a.mb, a.seq, nullptr, 0);
    }
    if (pr) pr[6] = wall_clock64();
  }
}

// ---- the same round with rolled loops (round 6; SPG_BCOMB_ROLL=1, measured slower than k_bullet_comb, see msm.hip) ----
// A Bullet round is a latency-bound launch whose code runs once per launch: k_bullet_comb's fully unrolled form is
// 4,033 straight-line instructions (hipcc -S, <13, 10, 64>), ~29 KiB that every launch fetches into cold instruction
// caches (profiles/r05_bcomb_micro_fetch.txt: PMC FETCH_SIZE of back-to-back launches, ~29 KiB per workgroup up to the
// 8 XCDs). Here every field product of a kind has ONE site in the code:
//  * the fold's operand product and k = av cv are two iterations of one Fq-product loop;
//  * the quad's mixed additions (WG of them) and the workgroup's LDS tree levels are iterations of one loop around one
//    quad step: lane q's first-round product quad_operand(acc, q) * y -- y = the entry's Niels coordinate (2 on lane 3)
//    for an addition, the partner quad's first-round operand for a tree level, which also scales by its small
//    constant (quad_add_op) -- then quad_finish. The entries shift down one register slot per addition, so no loop
//    indexes a register array.
// Same group elements, same parts, same bytes (tests/test_gpu_snark.py goldens; test_round_forms keeps the unrolled form).
template <int C, int G, int BS>
__global__ void __launch_bounds__(BS) k_bullet_comb_roll(BulletCombArgs a) {
  constexpr int W = 253 / C + 1, WG = (W + G - 1) / G, S = BS / 4;
  __shared__ uint32_t pts[soa_words<Ext, S>()];
  __shared__ bool last;
  const int b = blockIdx.y, t = threadIdx.x, q = t & 3, slot = t >> 2;
  const int P = a.n / 2, nk = a.nk, nh = nk / 2;
  const int gq = blockIdx.x * S + slot;  // quad index within MSM b
  const int p = gq / G, jg = gq - p * G, w0 = jg * WG;
  unsigned long long* pr = a.probe ? a.probe + 8 * (blockIdx.y * gridDim.x + blockIdx.x) : nullptr;
  if (pr && t == 0) pr[0] = wall_clock64();
  Ext acc = ext_identity();
  uint32_t ent[WG];
  Fp qv[WG];
  bool ng[WG];
#pragma unroll
  for (int x = 0; x < WG; x++) {
    ent[x] = 0xffffffffu;
    ng[x] = false;
  }
  if (p < P) {
    const int blk = p / nh, off = p - blk * nh;
    const int ia = b ? off + nh : off;
    const int j = blk * nk + (b ? 0 : nh) + off;
    Fq av, cv, x, y;
    int it = 0;
    if (a.k == 0) {
      av = a.aa_in[ia];
      cv = fq_zero();
      cv.l[0] = 1u;  // cw = 1: the product below takes av out of Montgomery form
      x = av;
      y = cv;
      it = 1;
    } else {
      // lanes 0, 1, 2: u a[ia], u^-1 a[ia + nk], cw[j] f; lane 3 repeats lane 0 (operands selected after both loads,
      // as in k_bullet_comb)
      const Fq xa = a.aa_in[q == 1 ? ia + nk : ia];
      const Fq xc = a.cw_in[j];
      x = q == 2 ? xc : xa;
      y = q == 1 ? a.uinv : (q == 2 ? ((j & (2 * nk - 1)) < nk ? a.uinv : a.u) : a.u);
    }
    Fq k;
#pragma unroll 1
    for (; it < 2; it++) {  // uniform per launch: iteration 0 the fold (k >= 1 only), iteration 1 k = av cv
      const Fq r = fq_mul(x, y);
      if (it == 0) {
        av = fq_add(fq_qbcast_lane(r, 0), fq_qbcast_lane(r, 1));
        cv = fq_qbcast_lane(r, 2);
        x = av;
        y = cv;
      } else {
        k = r;  // canonical scalar (cw is a plain integer)
      }
    }
    if (jg == 0 && q == 0) {  // the folded state, every (ia, j) once over the two MSMs
      if (blk == 0) a.aa_out[ia] = av;
      a.cw_out[j] = cv;
    }
    if (pr) { asm volatile("" ::"v"(k.l[0])); if (t == 0) pr[1] = wall_clock64(); }
    const int s = (int)a.gidx[j];
    comb_window_entries<C, WG>(k, w0, s, a.NS, ent);
#pragma unroll
    for (int x2 = 0; x2 < WG; x2++)
      if (ent[x2] != 0xffffffffu) qv[x2] = niels_coord(a.comb, ent[x2], q, &ng[x2], a.st);
    if (pr) { asm volatile("" ::"v"(qv[WG - 1].l[0])); if (t == 0) pr[2] = wall_clock64(); }
  }
  // WG mixed additions, then log2(S / R) tree levels (d = S/2, S/4, .., R), through one quad step
  const int levels = __builtin_ctz((unsigned)S) - __builtin_ctz((unsigned)a.R);
#pragma unroll 1
  for (int it = 0; it < WG + levels; it++) {
    const bool tree = it >= WG;  // uniform
    Fp y;
    bool cneg, use;
    if (tree) {
      const int d = (S / 2) >> (it - WG);
      if (slot >= d && slot < 2 * d) quad_put_op<S>(pts, slot - d, acc, q);
      __syncthreads();
      y = quad_get_op<S>(pts, slot, q);  // read by every quad, used by slot < d
      __syncthreads();
      cneg = true;
      use = slot < d;
    } else {
      y = q == 3 ? fp_small(2) : qv[0];
      cneg = ng[0];
      use = ent[0] != 0xffffffffu;
#pragma unroll
      for (int x = 0; x + 1 < WG; x++) {
        ent[x] = ent[x + 1];
        qv[x] = qv[x + 1];
        ng[x] = ng[x + 1];
      }
      ent[WG - 1] = 0xffffffffu;
    }
    Fp prd = fp_mul(quad_operand(acc, q), y);
    if (tree) prd = fp_mul_k(prd, q == 2 ? 243330u : (q == 3 ? 243332u : 121666u));
    const Ext r = quad_finish(prd, q, cneg);
    if (use) acc = r;
    if (pr && it + 1 == WG) { asm volatile("" ::"v"(acc.X.l[0])); if (t == 0) pr[3] = wall_clock64(); }
  }
  if (pr) { asm volatile("" ::"v"(acc.X.l[0])); if (t == 0) pr[4] = wall_clock64(); }
  if (slot < a.R && q == 0) a.parts[((size_t)b * gridDim.x + blockIdx.x) * a.R + slot] = acc;
  __syncthreads();
  if (t == 0) {
    // the parts (mapped host memory) and the folded state (HBM) before the ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (pr) pr[5] = wall_clock64();
    last = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           gridDim.x * gridDim.y - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      mbox_post(a.mb, a.seq, nullptr, 0);
    }
    if (pr) pr[6] = wall_clock64();
  }
}

// B plain MSMs from the comb table, sum_i s_{b,i} G_{idx_{b,i}} (Montgomery scalars), left as partial points: the Cx
// commitment of a device DotProductProofLog (its blind term is added on the host). The same quads, window groups and
// workgroup trees as k_bullet_comb; parts[b][wg][0..R).
template <int C, int G, int BS>
__global__ void __launch_bounds__(BS) k_comb_msm_parts(const Fq* __restrict__ scalars, const uint32_t* __restrict__ idx,
                                                       int n, const Niels* __restrict__ comb, int NS, int R,
                                                       Ext* __restrict__ parts, int st) {
  constexpr int W = 253 / C + 1, WG = (W + G - 1) / G, S = BS / 4;
  __shared__ uint32_t pts[soa_words<Ext, S>()];
  const int b = blockIdx.y, t = threadIdx.x, q = t & 3, slot = t >> 2;
  const int gq = blockIdx.x * S + slot;
  const int p = gq / G, jg = gq - p * G, w0 = jg * WG;
  Ext acc = ext_identity();
  if (p < n) {
    const Fq k = fq_from_mont(scalars[(size_t)b * n + p]);
    const int s = (int)idx[(size_t)b * n + p];
    uint32_t ent[WG];
    comb_window_entries<C, WG>(k, w0, s, NS, ent);
    Fp qv[WG];
    bool ng[WG];
#pragma unroll
    for (int x = 0; x < WG; x++)
      if (ent[x] != 0xffffffffu) qv[x] = niels_coord(comb, ent[x], q, &ng[x], st);
#pragma unroll
    for (int x = 0; x < WG; x++)
      if (ent[x] != 0xffffffffu) acc = quad_madd(acc, qv[x], ng[x], q);
  }
  for (int d = S / 2; d >= R; d >>= 1) {
    if (slot >= d && slot < 2 * d) quad_put_op<S>(pts, slot - d, acc, q);
    __syncthreads();
    if (slot < d) acc = quad_add_op(acc, quad_get_op<S>(pts, slot, q), q);
    __syncthreads();
  }
  if (slot < R && q == 0) parts[((size_t)b * gridDim.x + blockIdx.x) * R + slot] = acc;
}

}  // namespace spg
