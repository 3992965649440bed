// spg — one large MSM (GroupElement::vartime_multiscalar_mul, src/group.rs:98-116; Commitments::commit with a
// blind, src/commitments.rs:87-92) on MI355X: the config-2 shape (2^16 points), spg_msm and the
// spg_msm_partial shards of an MSM split over GPUs.
//
// The batch pipeline of msm.hip sizes its window for many MSMs at once (c = 16 for one 2^16 MSM: 2^15 buckets),
// and for a single MSM its bucket reduction sum_v v B_v -- a chain of dependent group additions -- dominated
// (65 % of 604 us). Here the window is chosen for one MSM (c = 11..12 signed digits, 2^10..2^11 buckets),
// fixed-base over the resident 2^k P_i tables (no doublings), and every phase is either throughput-bound with the
// chip full or a short dependent chain (c = 11 by default: 1024 buckets, 24 windows):
//   k_big_digits   block-local LDS histograms of the signed digits (digits kept in HBM as int16)
//   hipcub scan    over the [bucket][block] histogram matrix: each (bucket, block) pair's entry range
//   k_big_scatter  counting-sort scatter of (table index | sign) into bucket order, LDS cursors; its block 0 also
//                  writes the accumulation's work list: bucket v split into chunks of <= CH entries (skewed scalars
//                  only lengthen the list, never a workgroup)
//   k_big_accum    one workgroup per chunk: each lane adds every 256th entry of the chunk (one-lane mixed
//                  additions), the 256 lane sums meet in LDS (quad.hpp: 4 lanes per point) -> the chunk's sum; the
//                  workgroup finishing the last chunk of a group of 64 buckets then reduces that group: bucket sums
//                  from their chunks, a suffix scan and a tree give W_g = sum_j (j + 1) B_{64 g + j} and
//                  G_g = sum_j B_{64 g + j}
//   host           sum_v v B_v = sum_g W_g + 64 sum_g g G_g over the NB/64 groups (radix-2^51 additions at ~0.1 us
//                  each on a host core, where one dependent GPU addition costs ~2 us), then the encoding.
#include <hipcub/hipcub.hpp>

#include <stdio.h>

#include <vector>

#include "ctx.hpp"
#include "hcurve.hpp"
#include "quad.hpp"

namespace spg {

namespace {

// workspace slots 100..108 (msm.hip 0..18, proto.hip 20..24, r1cs.hip 30.., spark.hip 60.., snark / verify 91..96)
constexpr int kBigBS = 256;      // threads per workgroup (64 quads)
constexpr int kBigQuads = kBigBS / 4;
constexpr int kBigGroup = 64;    // buckets per group reduction (big_group)

struct BigArgs {
  const Fq* scalars;
  const Fq* blind;  // scalar n when per = n + 1; always a valid pointer (a wave-uniform load may be issued as a
                    // scalar load ahead of its branch, which EXEC does not mask)
  int n, per;       // per = n (+1 with a blind)
  int gen_offset, h_index, n1;
  int G, spb;       // digit blocks, scalars per block
  int16_t* digits;  // [W][per]
  uint32_t* bh;     // [NB][G] block histograms (+ a zero at [NB * G])
  uint32_t* off;    // their exclusive scan: the entry range of each (bucket, block); off[NB * G] = total
  uint32_t* entries;
};

struct Chunk {
  uint32_t key, start, len, pad;
};

template <int C>
__global__ void __launch_bounds__(kBigBS) k_big_digits(BigArgs a) {
  constexpr int W = 253 / C + 1;
  constexpr int NB = 1 << (C - 1);
  constexpr uint32_t MASK = (1u << C) - 1u;
  __shared__ uint32_t cnt[NB];
  const int blk = blockIdx.x, t = threadIdx.x;
  for (int k = t; k < NB; k += kBigBS) cnt[k] = 0;
  __syncthreads();
  const int i0 = blk * a.spb, i1 = min(a.per, i0 + a.spb);
  for (int i = i0 + t; i < i1; i += kBigBS) {
    const Fq k = fq_from_mont(i < a.n ? a.scalars[i] : a.blind[0]);  // Scalar::to_bytes (src/scalar/mod.rs:32-36)
    int carry = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const int bit = w * C, li = bit >> 5, of = bit & 31;
      uint32_t v = k.l[li] >> of;
      if (of + C > 32 && li + 1 < 8) v |= k.l[li + 1] << (32 - of);
      int d = (int)(v & MASK) + carry;
      carry = d > NB ? 1 : 0;
      d -= carry << C;
      a.digits[(size_t)w * a.per + i] = (int16_t)d;
      if (d) atomicAdd(&cnt[(d < 0 ? -d : d) - 1], 1u);
    }
  }
  __syncthreads();
  for (int k = t; k < NB; k += kBigBS) a.bh[(size_t)k * a.G + blk] = cnt[k];
  if (blk == 0 && t == 0) a.bh[(size_t)NB * a.G] = 0;
}

// one workgroup of BS threads: bucket v = key + 1 holds entries [bh[key G], bh[(key + 1) G]); it becomes
// ceil(count / ch) chunks; first[key] = its first chunk, first[NB] = the number of chunks
template <int BS>
__device__ __forceinline__ void big_chunks(const uint32_t* __restrict__ bh, int G, int NB, uint32_t ch,
                                           Chunk* __restrict__ chunks, uint32_t* __restrict__ first,
                                           unsigned* __restrict__ gcnt, Ext* __restrict__ out, uint32_t* part) {
  const int t = threadIdx.x;
  const int per_t = (NB + BS - 1) / BS, k0 = t * per_t, k1 = min(NB, k0 + per_t);
  uint32_t mine = 0;
  for (int k = k0; k < k1; k++) {
    const uint32_t c = bh[(size_t)(k + 1) * G] - bh[(size_t)k * G];
    mine += (c + ch - 1) / ch;
  }
  part[t] = mine;
  __syncthreads();
  for (int s = 1; s < BS; s <<= 1) {  // inclusive Hillis-Steele scan of the per-thread chunk counts
    const uint32_t x = t >= s ? part[t - s] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - mine;
  for (int k = k0; k < k1; k++) {
    const uint32_t s = bh[(size_t)k * G], c = bh[(size_t)(k + 1) * G] - s;
    first[k] = run;
    for (uint32_t o = 0; o < c; o += ch) chunks[run++] = Chunk{(uint32_t)k, s + o, min(ch, c - o), 0u};
  }
  if (t == BS - 1) first[NB] = part[BS - 1];
  __syncthreads();
  // the group tickets of k_big_accum, and the sums of groups no chunk will report (no entries at all)
  for (int g = t; g < NB / kBigGroup; g += BS) {
    gcnt[g] = 0u;
    if (first[(g + 1) * kBigGroup] == first[g * kBigGroup]) out[2 * g] = out[2 * g + 1] = ext_identity();
  }
}

// (block 0 also builds the accumulation's chunk list from the scanned histogram: one launch fewer)
template <int C>
__global__ void __launch_bounds__(kBigBS) k_big_scatter(BigArgs a, uint32_t ch, Chunk* __restrict__ chunks,
                                                        uint32_t* __restrict__ first, unsigned* __restrict__ gcnt,
                                                        Ext* __restrict__ out) {
  constexpr int W = 253 / C + 1;
  constexpr int NB = 1 << (C - 1);
  __shared__ uint32_t cur[NB];
  const int blk = blockIdx.x, t = threadIdx.x;
  if (blk == 0) {
    __shared__ uint32_t part[kBigBS];
    big_chunks<kBigBS>(a.off, a.G, NB, ch, chunks, first, gcnt, out, part);
  }
  for (int k = t; k < NB; k += kBigBS) cur[k] = a.off[(size_t)k * a.G + blk];
  __syncthreads();
  const int i0 = blk * a.spb, i1 = min(a.per, i0 + a.spb);
  for (int i = i0 + t; i < i1; i += kBigBS) {
    const uint32_t gidx = i < a.n ? (uint32_t)(a.gen_offset + i) : (uint32_t)a.h_index;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const int d = a.digits[(size_t)w * a.per + i];
      if (d) {
        const uint32_t slot = atomicAdd(&cur[(d < 0 ? -d : d) - 1], 1u);
        a.entries[slot] = ((uint32_t)(w * C) * (uint32_t)a.n1 + gidx) | (d < 0 ? 0x80000000u : 0u);
      }
    }
  }
}

// Group g of 64 buckets (run by the workgroup that finishes the group's last chunk): quad j holds
// B = bucket 64 g + j + 1 (its chunks summed); the suffix scan S_j = sum_{u >= j} B_u and the tree
// sum_j S_j = sum_j (j + 1) B_j; out[2 g] = that weighted sum, out[2 g + 1] = S_0 = the group's plain sum
__device__ __forceinline__ void big_group(int g, const Ext* __restrict__ sums, const uint32_t* __restrict__ first,
                                          Ext* __restrict__ out, uint32_t* pts) {
  const int t = threadIdx.x, q = t & 3, slot = t >> 2;
  const int key = g * kBigGroup + slot;
  Ext B = ext_identity();
  bool any = false;
  for (uint32_t c = first[key]; c < first[key + 1]; c++) {
    B = any ? quad_add(B, sums[c], q) : sums[c];
    any = true;
  }
  Ext suf = B;
  for (int d = 1; d < kBigQuads; d <<= 1) {
    quad_put_op<kBigQuads>(pts, slot, suf, q);
    __syncthreads();
    if (slot + d < kBigQuads) suf = quad_add_op(suf, quad_get_op<kBigQuads>(pts, slot + d, q), q);
    __syncthreads();
  }
  if (slot == 0 && q == 0) out[2 * g + 1] = suf;
  Ext acc = suf;
  for (int d = kBigQuads / 2; d >= 1; d >>= 1) {
    if (slot >= d && slot < 2 * d) quad_put_op<kBigQuads>(pts, slot - d, acc, q);
    __syncthreads();
    if (slot < d) acc = quad_add_op(acc, quad_get_op<kBigQuads>(pts, slot, q), q);
    __syncthreads();
  }
  if (t == 0) out[2 * g] = acc;
}

// one workgroup per chunk; grid = an upper bound of the chunk count. The workgroup that finishes the last chunk
// of a group of 64 buckets (ticket gcnt[g]) goes on to that group's reduction (big_group): no second launch, and
// the groups reduce while other chunks still accumulate.
//   LANE = false: 64 quads (4 lanes per point, quad.hpp) each add ~CH/64 table entries.
//   LANE = true (default, SPG_BIG_ITEMS=0 selects the other): every lane adds every 256th entry of the chunk in
//     one-lane mixed additions (~6 at c = 11 on random scalars: one chunk per bucket; the one-lane form issues
//     ~1.5x fewer instructions per addition than the quad split: 3.0e10 vs 2.0e10 madd/s whole-chip in
//     scripts/micro/ext_throughput), then the 256 lane sums meet in LDS: quad j adds sums 4j .. 4j + 3.
// Either way an LDS quad tree then gives the chunk's sum.
// Cross-XCD hand-off as in grid_reduce3 (sumcheck.hip): plain stores + agent-scope release before the ticket,
// agent-scope acquire in the reducer before plain loads (the per-XCD L2s are not coherent).
template <bool LANE>
__device__ __forceinline__ void big_chunk(uint32_t cid, const Chunk* __restrict__ chunks,
                                          const uint32_t* __restrict__ first, const uint32_t* __restrict__ entries,
                                          const Niels* __restrict__ tab, Ext* __restrict__ sums,
                                          unsigned* __restrict__ gcnt, Ext* __restrict__ out,
                                          unsigned long long* probe, uint32_t* pts, bool& last) {
  const int t = threadIdx.x, q = t & 3, slot = t >> 2;
  if (probe && t == 0) probe[4 * cid] = wall_clock64();
  const Chunk c = chunks[cid];
  Ext acc = ext_identity();
  if (LANE) {
    Ext P = ext_identity();
    if ((uint32_t)t < c.len) {
      P = load_signed(tab, entries[c.start + t]);
      for (uint32_t e = t + kBigBS; e < c.len; e += kBigBS) {
        const uint32_t x = entries[c.start + e];
        P = ext_madd(P, tab[x & 0x7fffffffu], (x >> 31) != 0);
      }
    }
    soa_put<kBigBS>(pts, t, P);
    __syncthreads();
    acc = soa_get<kBigBS, Ext>(pts, 4 * slot);
    for (int k = 1; k < 4; k++) acc = quad_add(acc, soa_get<kBigBS, Ext>(pts, 4 * slot + k), q);
    __syncthreads();
  } else {
    // software-pipelined: the table coordinate of entry e + 64 is loaded while entry e is added
    uint32_t e = slot;
    Fp qv;
    bool neg = false;
    if (e < c.len) qv = niels_coord(tab, entries[c.start + e], q, &neg);
    while (e < c.len) {
      const uint32_t e2 = e + kBigQuads;
      Fp qn;
      bool nn = false;
      if (e2 < c.len) qn = niels_coord(tab, entries[c.start + e2], q, &nn);
      acc = quad_madd(acc, qv, neg, q);
      qv = qn;
      neg = nn;
      e = e2;
    }
  }
  if (probe) {
    __syncthreads();
    if (t == 0) probe[4 * cid + 1] = wall_clock64();
  }
  for (int d = kBigQuads / 2; d >= 1; d >>= 1) {
    if (slot >= d && slot < 2 * d) quad_put_op<kBigQuads>(pts, slot - d, acc, q);
    __syncthreads();
    if (slot < d) acc = quad_add_op(acc, quad_get_op<kBigQuads>(pts, slot, q), q);
    __syncthreads();
  }
  const int g = (int)(c.key / kBigGroup);
  if (t == 0) {
    sums[cid] = acc;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t total = first[(g + 1) * kBigGroup] - first[g * kBigGroup];
    last = __hip_atomic_fetch_add(&gcnt[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (probe) probe[4 * cid + 2] = wall_clock64();
  }
  __syncthreads();
  if (!last) return;
  big_group(g, sums, first, out, pts);
  if (probe && t == 0) probe[4 * cid + 3] = wall_clock64();
}

// grid: the LANE form launches one workgroup per bucket (random scalars: one chunk per bucket) and loops over any
// further chunks (skewed scalars), so no surplus workgroups are dispatched; the quad form one per chunk bound
template <bool LANE>
__global__ void __launch_bounds__(kBigBS, 4) k_big_accum(const Chunk* __restrict__ chunks,
                                                         const uint32_t* __restrict__ first,
                                                         const uint32_t* __restrict__ entries,
                                                         const Niels* __restrict__ tab, Ext* __restrict__ sums,
                                                         unsigned* __restrict__ gcnt, Ext* __restrict__ out, int NB,
                                                         unsigned long long* probe) {
  // LANE: the lane sums (SoA over 256), then the quad tree's operands; else the quad tree's operands only
  __shared__ uint32_t pts[LANE ? soa_words<Ext, kBigBS>() : soa_words<Ext, kBigQuads>()];
  __shared__ bool last;
  const uint32_t n = first[NB];
  for (uint32_t cid = blockIdx.x; cid < n; cid += gridDim.x) {  // uniform per workgroup
    big_chunk<LANE>(cid, chunks, first, entries, tab, sums, gcnt, out, probe, pts, last);
    __syncthreads();  // pts / last are reused by the next chunk
  }
}

int big_window() {
  // c = 11 (1024 buckets, 24 windows): measured best for 2^16 points against 12 and 13 (session r03d); a
  // smaller bucket set shortens the group reductions at the end more than its extra windows cost
  static const int c = getenv("SPG_BIG_C") ? atoi(getenv("SPG_BIG_C")) : 11;
  return c < 8 ? 8 : (c > 14 ? 14 : c);
}

template <int C>
int launch_big(spg_ctx* ctx, const spg_gens* g, BigArgs a, Ext* host_groups_dev, int* ngroups) {
  constexpr int W = 253 / C + 1;
  constexpr int NB = 1 << (C - 1);
  hipStream_t s = ctx->stream;
  const size_t E = (size_t)a.per * W;
  static const bool lane = !getenv("SPG_BIG_ITEMS") || atoi(getenv("SPG_BIG_ITEMS")) != 0;
  // chunk size: the mean bucket load rounded up to whole passes of the 64 quads (random scalars: about one chunk per
  // bucket), at least 2 entries per quad; the lane form takes up to 8 entries per lane (a bucket with more -- skewed
  // scalars -- splits into several chunks)
  const uint32_t ch = lane ? 8 * kBigBS
                           : (uint32_t)std::max<size_t>(2 * kBigQuads,
                                                        ((E / NB + kBigQuads - 1) / kBigQuads + 1) * kBigQuads);
  const size_t max_chunks = E / ch + NB + 1;
  a.digits = (int16_t*)ws_get(ctx, 100, E * sizeof(int16_t) + 64);
  a.bh = (uint32_t*)ws_get(ctx, 101, ((size_t)NB * a.G + 1) * 4 + 64);
  a.off = (uint32_t*)ws_get(ctx, 102, ((size_t)NB * a.G + 1) * 4 + 64);
  a.entries = (uint32_t*)ws_get(ctx, 103, E * 4 + 64);
  Chunk* chunks = (Chunk*)ws_get(ctx, 104, max_chunks * sizeof(Chunk));
  uint32_t* first = (uint32_t*)ws_get(ctx, 105, (NB + 1) * 4 + 64);
  unsigned* gcnt = (unsigned*)ws_get(ctx, 108, (NB / kBigGroup) * 4 + 64);
  Ext* sums = (Ext*)ws_get(ctx, 106, max_chunks * sizeof(Ext));
  if (!a.digits || !a.bh || !a.off || !a.entries || !chunks || !first || !gcnt || !sums) return set_err(ctx, SPG_E_NOMEM, "msm workspace");
  const int nkeys = NB * a.G + 1;
  size_t tmp_bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, a.bh, a.off, nkeys, s);
  void* tmp = ws_get(ctx, 107, tmp_bytes + 16);
  if (!tmp) return set_err(ctx, SPG_E_NOMEM, "msm scan workspace");
  {
    KScope ks(ctx, "msm_big_sort");
    hipLaunchKernelGGL(k_big_digits<C>, dim3(a.G), dim3(kBigBS), 0, s, a);
    SPG_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, a.bh, a.off, nkeys, s));
    hipLaunchKernelGGL(k_big_scatter<C>, dim3(a.G), dim3(kBigBS), 0, s, a, ch, chunks, first, gcnt, host_groups_dev);
  }
  // SPG_BIG_PROBE=1: per-workgroup phase timestamps of the accumulation (+ group reductions), on stderr
  static const bool probe_on = getenv("SPG_BIG_PROBE") != nullptr;
  unsigned long long* pa = nullptr;
  if (probe_on) {
    SPG_HIP(ctx, hipMalloc(&pa, 4 * max_chunks * 8));
    SPG_HIP(ctx, hipMemsetAsync(pa, 0, 4 * max_chunks * 8, s));
  }
  {
    KScope ks(ctx, "msm_big_accum", 0.0, (double)a.per * W * (1.0 - 1.0 / (double)(1 << C)));
    if (lane)
      hipLaunchKernelGGL(k_big_accum<true>, dim3((unsigned)std::min<size_t>(max_chunks, NB)), dim3(kBigBS), 0, s,
                         chunks, first, a.entries, g->table, sums, gcnt, host_groups_dev, NB, pa);
    else
      hipLaunchKernelGGL(k_big_accum<false>, dim3((unsigned)max_chunks), dim3(kBigBS), 0, s, chunks, first,
                         a.entries, g->table, sums, gcnt, host_groups_dev, NB, pa);
  }
  SPG_HIP(ctx, hipGetLastError());
  if (probe_on) {
    std::vector<unsigned long long> A(4 * max_chunks);
    SPG_HIP(ctx, (hipMemcpyAsync)(A.data(), pa, A.size() * 8, hipMemcpyDeviceToHost, s));
    SPG_HIP(ctx, hipStreamSynchronize(s));
    unsigned long long a0 = ~0ull, a1 = 0, g1 = 0, s1 = 0, mx = 0;
    double madd = 0, tree = 0, grp = 0;
    size_t cnt = 0, ng = 0;
    for (size_t i = 0; i < max_chunks; i++) {
      if (!A[4 * i]) continue;
      a0 = std::min(a0, A[4 * i]);
      s1 = std::max(s1, A[4 * i]);
      a1 = std::max(a1, A[4 * i + 2]);
      mx = std::max(mx, A[4 * i + 1] - A[4 * i]);
      madd += (double)(A[4 * i + 1] - A[4 * i]);
      tree += (double)(A[4 * i + 2] - A[4 * i + 1]);
      cnt++;
      if (A[4 * i + 3]) {
        g1 = std::max(g1, A[4 * i + 3]);
        grp += (double)(A[4 * i + 3] - A[4 * i + 2]);
        ng++;
      }
    }
    double xs[8] = {0}, xm[8] = {0};
    size_t xn[8] = {0};
    for (size_t i = 0; i < max_chunks; i++) {  // by workgroup index mod 8 (the XCD of a round-robin dispatch)
      if (!A[4 * i]) continue;
      const double d = (double)(A[4 * i + 1] - A[4 * i]) / 100.0;
      xs[i % 8] += d;
      xm[i % 8] = std::max(xm[i % 8], d);
      xn[i % 8]++;
    }
    for (int x = 0; x < 8; x++)
      if (xn[x]) fprintf(stderr, "[spg]   blockIdx %% 8 = %d: adds mean %.1f max %.1f us\n", x, xs[x] / xn[x], xm[x]);
    fprintf(stderr, "[spg] big accum: %zu chunks, span %.1f us (groups done at %.1f us, last chunk start at %.1f us); "
            "per chunk: adds %.1f us (max %.1f), tree %.1f us; per group reduction %.1f us (%zu)\n", cnt,
            (a1 - a0) / 100.0, (g1 - a0) / 100.0, (s1 - a0) / 100.0, madd / cnt / 100.0, mx / 100.0, tree / cnt / 100.0,
            ng ? grp / ng / 100.0 : 0.0, ng);
    hipFree(pa);
  }
  *ngroups = NB / kBigGroup;
  return 0;
}

}  // namespace

// comb.hip: the same sum from g's comb table (h = generator g->n), summed on the host; 1 when the comb does not apply
int msm_single_comb(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n,
                    const Fq* d_blind, h::HExt* out);

// sum_i s_i G[gen_offset + i] (+ blind h) of n device scalars, into *out (host point)
int msm_single_big(spg_ctx* ctx, const spg_gens* g, size_t gen_offset, const Fq* d_scalars, size_t n,
                   const Fq* d_blind, h::HExt* out) {
  // Large MSMs over a generator set that can keep a comb table (comb.hip; <= 2^16 generators, 47 GB at c = 9, 62 GB
  // with 128-byte entries) take it -- no digit sort, no bucket reduction (SPG_BIG_COMB=0: the buckets below). Round 4
  // measured the comb level with the buckets (0.210-0.213 against 0.204-0.209 ms, profiles/r04_ab_combwgs_bigcomb.txt);
  // with the entries padded to one line and the parts summed on the host's IFMA lanes it is ahead: 0.171-0.179 ms with
  // 4 window groups per scalar, 0.146 ms with 2 (SPG_BIG_COMB_G), against 0.204-0.206 ms (profiles/r05_ab_big_comb.txt)
  static const bool comb_on = !getenv("SPG_BIG_COMB") || atoi(getenv("SPG_BIG_COMB")) != 0;
  if (comb_on && !ctx->comb_off && n >= ((size_t)1 << 14)) {
    const int rc = msm_single_comb(ctx, g, gen_offset, d_scalars, n, d_blind, out);
    if (rc != 1) return rc;
  }
  const int c = big_window();
  const int per = (int)n + (d_blind ? 1 : 0);
  SPG_CHECK(ctx, n >= 1 && (size_t)per * (253 / c + 1) < 0x7fffffffULL, "msm too large");
  SPG_CHECK(ctx, (size_t)kTableRows * (g->n + 1) < 0x7fffffffULL, "generator table too large");
  BigArgs a{};
  a.scalars = d_scalars;
  a.blind = d_blind ? d_blind : d_scalars;
  a.n = (int)n;
  a.per = per;
  a.gen_offset = (int)gen_offset;
  a.h_index = (int)g->n;
  a.n1 = (int)(g->n + 1);
  // digit blocks: SPG_BIG_SPT scalars per thread (default 1), at most 512 blocks (the histogram matrix is NB x G)
  static const int spt = getenv("SPG_BIG_SPT") ? std::max(1, atoi(getenv("SPG_BIG_SPT"))) : 1;
  a.G = std::max(1, std::min(512, (per + spt * kBigBS - 1) / (spt * kBigBS)));
  a.spb = (per + a.G - 1) / a.G;
  int ng = 0, rc = 0;
  Ext* res = (Ext*)ctx->d_res;  // the coherent result page: 2 NB / 64 points (<= 256 at c = 14)
  static_assert(kResScalars * sizeof(Fq) >= 2 * (1 << 13) / kBigGroup * sizeof(Ext), "result page too small");
  switch (c) {
    case 8: rc = launch_big<8>(ctx, g, a, res, &ng); break;
    case 9: rc = launch_big<9>(ctx, g, a, res, &ng); break;
    case 10: rc = launch_big<10>(ctx, g, a, res, &ng); break;
    case 11: rc = launch_big<11>(ctx, g, a, res, &ng); break;
    case 12: rc = launch_big<12>(ctx, g, a, res, &ng); break;
    case 13: rc = launch_big<13>(ctx, g, a, res, &ng); break;
    default: rc = launch_big<14>(ctx, g, a, res, &ng); break;
  }
  if (rc) return rc;
  SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // sum_v v B_v = sum_g W_g + 64 sum_g g G_g, with sum_g g G_g = sum_{g >= 1} sum_{h >= g} G_h
  const Ext* r = (const Ext*)ctx->res;
  h::HExt wsum = h::hext_from_dev(r[0]), S = h::hext_identity(), T = h::hext_identity();
  for (int gi = ng - 1; gi >= 1; gi--) {
    wsum = h::hext_add(wsum, h::hext_from_dev(r[2 * gi]));
    S = h::hext_add(S, h::hext_from_dev(r[2 * gi + 1]));
    T = h::hext_add(T, S);
  }
  for (int k = 0; k < 6; k++) T = h::hext_dbl(T);  // x 64 = kBigGroup
  static_assert(kBigGroup == 64, "six doublings");
  *out = h::hext_add(wsum, T);
  return 0;
}

}  // namespace spg
