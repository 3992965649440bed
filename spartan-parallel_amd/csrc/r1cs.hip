// spg — R1CSProof::prove (src/r1csproof.rs:210-685) with every O(N) table resident in HBM.
//
// Device work (HIP, this file + sumcheck.hip + msm.hip):
//   z_mat assembly into the (p, q_rev, w, x_rev) Z layout        r1csproof.rs:278-293, custom_dense_mlpoly.rs:67-111
//   multiply_vec_block (CSR SpMV for A, B, C at once)             r1csinstance.rs:363-436, sparse_mlpoly.rs:454-472
//   phase-1 / phase-2 round evaluation and folds                  sumcheck.rs:1067-1380, :788-1065
//   compute_eval_table_sparse_disjoint_rounds (CSC, eq-weighted)  r1csinstance.rs:484-534, sparse_mlpoly.rs:524-541
//   bound_poly_vars_rq on Z                                       custom_dense_mlpoly.rs:300-304
//   DensePolynomial::bound / evaluate of the witness sections     dense_mlpoly.rs:258-265, :361-367
//   Bulletproof L/R/delta MSMs                                    proto.hip
// Host work: the Fiat-Shamir transcript, the round polynomials (4 scalars), the sigma protocols over
// <= 5 fixed generators, and the bincode writer. Per sumcheck round exactly three scalars come back.
#include <chrono>
#include <stdio.h>
#include <stdlib.h>

#include "comm.hpp"
#include "hostpoly.hpp"
#include "proto.hpp"
#include "lds.hpp"
#include "sumcheck.hpp"


// R1CSInstance resident in HBM: per matrix instance p, CSR of A_p, B_p, C_p (SpMV) and one merged CSC
// (rows tagged 0/1/2) for the transposed eq-weighted product.
struct spg_r1cs_inst {
  size_t num_instances = 0, max_num_cons = 0, num_vars = 0;
  std::vector<size_t> num_cons;
  std::vector<uint64_t> rp_off, cp_off;  // [3p+m] offsets into rowptr ; [p] offsets into colptr
  std::vector<size_t> nnz;               // [3p+m]
  uint32_t* d_rowptr = nullptr;          // absolute entry indices
  uint32_t* d_col = nullptr;
  spg::Fq* d_val = nullptr;
  uint32_t* d_colptr = nullptr;
  uint32_t* d_crow = nullptr;            // row * 4 + tag
  spg::Fq* d_cval = nullptr;
};

// ProverWitnessSecInfo list resident in HBM: w_mat[p] flattened (q-major), sections concatenated.
static const uint64_t kNotResident = ~0ULL;  // instance held by another rank
struct spg_r1cs_witness {
  size_t nws = 0;
  std::vector<std::vector<size_t>> num_proofs, num_inputs;  // [w][p]
  std::vector<std::vector<uint64_t>> off;                   // [w][p] element offset into d_w
  // [w][p] device address of the instance's w_mat: d_w + off, or a caller's resident device buffer used in place
  // (witness_from_parts); nullptr: held by another rank
  std::vector<std::vector<const spg::Fq*>> ptr;
  spg::Fq* d_w = nullptr;
  size_t total = 0;
};

namespace spg {

// ------------------------------------------------------------------------------------ kernels
__device__ __forceinline__ uint32_t brev(uint32_t v, uint32_t lg) { return lg ? (__brev(v) >> (32 - lg)) : 0u; }

template <class D>
__device__ __forceinline__ int find_desc(const D* d, int P, uint64_t t) {
  int lo = 0, hi = P - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (d[mid].dom_off <= t) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

struct ZDesc {
  uint64_t dom_off, z_off;
  uint32_t lg_q, ni, lg_ni, pad;
};
struct SecDesc {
  const Fq* w;  // the instance's w_mat (spg_r1cs_witness::ptr)
  uint32_t np, ni;
};

// Z[p][q_rev][w][x_rev] = w_mat_w[pw][qw][x]  (zero beyond the section's width)
__global__ void k_z_fill(const ZDesc* __restrict__ zd, int P, const SecDesc* __restrict__ sd, int nws,
                         Fq* __restrict__ Z, uint64_t total) {
  uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  int p = find_desc(zd, P, t);
  const ZDesc d = zd[p];
  uint64_t loc = t - d.dom_off;
  uint32_t i = (uint32_t)(loc % d.ni);
  uint64_t rest = loc / d.ni;
  uint32_t w = (uint32_t)(rest % nws), q = (uint32_t)(rest / nws);
  const SecDesc s = sd[(size_t)w * P + p];
  Fq v = fq_zero();
  if (i < s.ni) v = s.w[(size_t)(s.np == 1 ? 0 : q) * s.ni + i];
  Z[d.z_off + ((size_t)brev(q, d.lg_q) * nws + w) * d.ni + brev(i, d.lg_ni)] = v;
}

// The same fill when every instance has ni >= 256: one workgroup per 16 x 16 tile of a (q, w) row, i = a 2^(lg-4) +
// m 16 + b (a, b < 16; m the tile). brev(i) = brev4(b) 2^(lg-4) + brev(m) 16 + brev4(a), so the tile's reads (b
// contiguous for each a) and its writes (a contiguous for each b) are both 16 runs of 512 bytes; the tile turns
// through LDS. The one-element form's stores land one 32-byte sector per line at bit-reversed positions.
__global__ void __launch_bounds__(256) k_z_fill_tiled(const ZDesc* __restrict__ zd, int P,
                                                      const SecDesc* __restrict__ sd, int nws, Fq* __restrict__ Z) {
  __shared__ uint32_t sh[8][16 * 17];  // component-major, row pitch 17: conflict-free both ways
  const uint64_t t0 = (uint64_t)blockIdx.x * 256;
  const int p = find_desc(zd, P, t0);
  const ZDesc d = zd[p];
  const uint64_t loc0 = t0 - d.dom_off;
  const uint64_t rest = loc0 / d.ni;
  const uint32_t m = (uint32_t)(loc0 % d.ni) >> 8;
  const uint32_t w = (uint32_t)(rest % nws), q = (uint32_t)(rest / nws);
  const SecDesc s = sd[(size_t)w * P + p];
  const uint32_t k = threadIdx.x, sh_hi = d.lg_ni - 4;
  {
    const uint32_t a = k >> 4, b = k & 15;
    const uint32_t i = (a << sh_hi) + (m << 4) + b;
    Fq v = fq_zero();
    if (i < s.ni) v = s.w[(size_t)(s.np == 1 ? 0 : q) * s.ni + i];
#pragma unroll
    for (int c = 0; c < 8; c++) sh[c][a * 17 + b] = v.l[c];
  }
  __syncthreads();
  const uint32_t a = k & 15, b = k >> 4;
  Fq v;
#pragma unroll
  for (int c = 0; c < 8; c++) v.l[c] = sh[c][a * 17 + b];
  const uint32_t ri = (brev(b, 4) << sh_hi) + (brev(m, d.lg_ni - 8) << 4) + brev(a, 4);
  Z[d.z_off + ((size_t)brev(q, d.lg_q) * nws + w) * d.ni + ri] = v;
}

struct SpDesc {
  uint64_t dom_off, out_off;
  uint32_t pi, lg_q, nrows, lg_rows, ni, lg_ni;
};
struct MatDesc {
  uint64_t rp[3];
  uint64_t cp;
};

// Az/Bz/Cz[p][q_rev][x_rev] = sum_e val_e * z[p][q][col_e / Y][col_e % Y], z gathered from the witness sections
// themselves (the mapping k_z_fill applies), so the Z table's fill is off this kernel's path.
// TILED (every instance has >= 256 rows): as k_z_fill_tiled, a workgroup takes a 16 x 16 tile of one q row, lanes read
// 16 consecutive CSR rows each (row = a 2^(lg-4) + m 16 + b) and the three outputs turn through LDS so that the stores
// are 16 runs of 512 bytes at the bit-reversed positions, instead of one 32-byte sector per line per lane. (Mapping the
// lanes to consecutive output positions instead, row = brev(position), made the CSR reads scatter: 289 -> 341 us on
// config 4.) SPG_SPMV_TILED=0: lanes by row, stores scattered.
template <bool TILED>
__global__ void __launch_bounds__(256) k_spmv(const SpDesc* __restrict__ sd, int P, const MatDesc* __restrict__ md,
                                              const uint32_t* __restrict__ rowptr, const uint32_t* __restrict__ col,
                                              const Fq* __restrict__ val, const SecDesc* __restrict__ sec, int nws,
                                              uint32_t Y,
                                              Fq* __restrict__ Az, Fq* __restrict__ Bz, Fq* __restrict__ Cz,
                                              uint64_t total) {
  // the section descriptors of the block's first instance (nws <= 8) sit in LDS: a nonzero's gather then waits on
  // an LDS read instead of a dependent global load; lanes of a later instance in the same block read them globally
  __shared__ SecDesc s_sec[8];
  const uint64_t t0 = (uint64_t)blockIdx.x * 256;
  const int pb = find_desc(sd, P, t0);
  if ((int)threadIdx.x < nws) s_sec[threadIdx.x] = sec[(size_t)threadIdx.x * P + pb];
  __syncthreads();
  uint64_t t = t0 + threadIdx.x;
  if (!TILED && t >= total) return;  // (tiled: total is whole tiles, every lane is live up to the LDS turn)
  const int p = TILED ? pb : find_desc(sd, P, t);
  const SpDesc d = sd[p];
  const uint64_t loc = t - d.dom_off;
  const uint32_t q = (uint32_t)(loc / d.nrows), k = threadIdx.x, mt = (uint32_t)(loc % d.nrows) >> 8;
  const uint32_t row = TILED ? ((k >> 4) << (d.lg_rows - 4)) + (mt << 4) + (k & 15) : (uint32_t)(loc % d.nrows);
  Fq sums[3];
#pragma unroll
  for (int m = 0; m < 3; m++) {
    const uint32_t* rp = rowptr + md[d.pi].rp[m];
    uint32_t e0 = rp[row], e1 = rp[row + 1];
    Fq s = fq_zero();
    for (uint32_t e = e0; e < e1; e++) {
      uint32_t c = col[e];
      uint32_t w = c / Y, i = c % Y;
      if (w < (uint32_t)nws && i < d.ni) {
        const Fq* xw;
        uint32_t xnp, xni;
        if (p == pb) {
          xw = s_sec[w].w;
          xnp = s_sec[w].np;
          xni = s_sec[w].ni;
        } else {
          const SecDesc& x = sec[(size_t)w * P + p];
          xw = x.w;
          xnp = x.np;
          xni = x.ni;
        }
        if (i < xni) s = fq_add(s, fq_mul(val[e], xw[(size_t)(xnp == 1 ? 0 : q) * xni + i]));
      }
    }
    sums[m] = s;
  }
  Fq* outs[3] = {Az, Bz, Cz};
  const size_t rowbase = d.out_off + (size_t)brev(q, d.lg_q) * d.nrows;
  if (!TILED) {
#pragma unroll
    for (int m = 0; m < 3; m++) outs[m][rowbase + brev(row, d.lg_rows)] = sums[m];
    return;
  }
  __shared__ uint32_t sh[3][8][16 * 17];  // component-major, row pitch 17: conflict-free both ways
#pragma unroll
  for (int m = 0; m < 3; m++)
#pragma unroll
    for (int c = 0; c < 8; c++) sh[m][c][(k >> 4) * 17 + (k & 15)] = sums[m].l[c];
  __syncthreads();
  const uint32_t a = k & 15, b = k >> 4;
  const uint32_t ri = (brev(b, 4) << (d.lg_rows - 4)) + (brev(mt, d.lg_rows - 8) << 4) + brev(a, 4);
#pragma unroll
  for (int m = 0; m < 3; m++) {
    Fq v;
#pragma unroll
    for (int c = 0; c < 8; c++) v.l[c] = sh[m][c][a * 17 + b];
    outs[m][rowbase + ri] = v;
  }
}

struct AbcDesc {
  uint64_t dom_off, out_off;
  uint32_t pi, ni, lg_ni, pad;
};

// ABC[p][w][x_rev] = sum_{M in A,B,C} r_M * sum_{e in M_p, col_e = w*Y + x} eq_rx[row_e] * val_e
__global__ void __launch_bounds__(256) k_abc(const AbcDesc* __restrict__ ad, int Pm, const MatDesc* __restrict__ md,
                                             const uint32_t* __restrict__ colptr, const uint32_t* __restrict__ crow,
                                             const Fq* __restrict__ cval, const Fq* __restrict__ eq, uint32_t Y,
                                             Fq rA, Fq rB, Fq rC, Fq* __restrict__ ABC, uint64_t total) {
  uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  int p = find_desc(ad, Pm, t);
  const AbcDesc d = ad[p];
  uint64_t loc = t - d.dom_off;
  uint32_t i = (uint32_t)(loc % d.ni), w = (uint32_t)(loc / d.ni);
  const uint32_t* cp = colptr + md[d.pi].cp;
  uint32_t c = w * Y + i;
  Fq acc[3] = {fq_zero(), fq_zero(), fq_zero()};
  for (uint32_t e = cp[c]; e < cp[c + 1]; e++) {
    uint32_t rt = crow[e];
    Fq v = fq_mul(cval[e], eq[rt >> 2]);
    uint32_t tag = rt & 3;
    if (tag == 0) acc[0] = fq_add(acc[0], v);
    else if (tag == 1) acc[1] = fq_add(acc[1], v);
    else acc[2] = fq_add(acc[2], v);
  }
  Fq r = fq_add(fq_add(fq_mul(rA, acc[0]), fq_mul(rB, acc[1])), fq_mul(rC, acc[2]));
  ABC[d.out_off + (size_t)w * d.ni + brev(i, d.lg_ni)] = r;
}

// DensePolynomial::bound: out[i] = sum_j L[j] * Z[j * Rs + i], split over gridDim.y chunks of j
__global__ void __launch_bounds__(256) k_bound_part(const Fq* __restrict__ Z, const Fq* __restrict__ L, uint32_t Ls,
                                                    uint32_t Rs, uint32_t chunk, Fq* __restrict__ part) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Rs) return;
  uint32_t j0 = blockIdx.y * chunk, j1 = min(Ls, j0 + chunk);
  Fq acc = fq_zero();
  for (uint32_t j = j0; j < j1; j++) acc = fq_add(acc, fq_mul(L[j], Z[(size_t)j * Rs + i]));
  part[(size_t)blockIdx.y * Rs + i] = acc;
}
__global__ void k_sum_cols(const Fq* __restrict__ part, uint32_t S, uint32_t Rs, Fq* __restrict__ out) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Rs) return;
  Fq acc = fq_zero();
  for (uint32_t y = 0; y < S; y++) acc = fq_add(acc, part[(size_t)y * Rs + i]);
  out[i] = acc;
}

// every witness polynomial's L.Z bound of one proof in two launches (instead of two per polynomial): job k's
// partial rows are blocks [b0, b0 + nbx * S) of the first launch, its column sums blocks
// [c0, c0 + ceil(Rs / kSumCols)) of the second
struct BoundDesc {
  const Fq* Z;
  uint32_t offL, Ls, Rs, chunk, S, offP, o, b0, c0;
};
constexpr int kBoundMax = 32;
struct BoundJobs {
  BoundDesc d[kBoundMax];
  int n;
};
__device__ __forceinline__ int bound_job(const BoundJobs& j, uint32_t b, bool cols) {
  int k = 0;
  while (k + 1 < j.n && (cols ? j.d[k + 1].c0 : j.d[k + 1].b0) <= b) k++;
  return k;
}
__global__ void __launch_bounds__(256) k_bound_part_multi(BoundJobs jobs, const Fq* __restrict__ L, Fq* __restrict__ part) {
  const int k = bound_job(jobs, blockIdx.x, false);
  const BoundDesc& d = jobs.d[k];
  const uint32_t nbx = (d.Rs + 255) / 256, rel = blockIdx.x - d.b0, y = rel / nbx;
  const uint32_t i = (rel % nbx) * 256 + threadIdx.x;
  if (i >= d.Rs) return;
  const uint32_t j0 = y * d.chunk, j1 = min(d.Ls, j0 + d.chunk);
  Fq acc = fq_zero();
  for (uint32_t j = j0; j < j1; j++) acc = fq_add(acc, fq_mul(L[d.offL + j], d.Z[(size_t)j * d.Rs + i]));
  part[d.offP + (size_t)y * d.Rs + i] = acc;
}
// a block owns kSumCols columns of one job and 256 / kSumCols lanes per column split its S partials, then an LDS
// tree (one lane per column made S dependent additions)
constexpr int kSumCols = 16;
__global__ void __launch_bounds__(256) k_sum_cols_multi(BoundJobs jobs, const Fq* __restrict__ part, Fq* __restrict__ out) {
  __shared__ Fq sm[256];
  constexpr int YL = 256 / kSumCols;
  const int k = bound_job(jobs, blockIdx.x, true);
  const BoundDesc& d = jobs.d[k];
  const int t = threadIdx.x, y0 = t / kSumCols;
  const uint32_t i = (blockIdx.x - d.c0) * kSumCols + t % kSumCols;
  Fq acc = fq_zero();
  if (i < d.Rs)
    for (uint32_t y = y0; y < d.S; y += YL) acc = fq_add(acc, part[d.offP + (size_t)y * d.Rs + i]);
  sm[t] = acc;
  __syncthreads();
#pragma unroll
  for (int h = YL / 2; h >= 1; h >>= 1) {
    if (y0 < h) sm[t] = fq_add(sm[t], sm[t + kSumCols * h]);
    __syncthreads();
  }
  if (y0 == 0 && i < d.Rs) out[d.o + i] = sm[t];
}

// SparseMatPolynomial::evaluate_with_tables (src/sparse_mlpoly.rs:427-436) for every matrix of the
// instance at once: segment s = 3p + m (A, B, C of matrix instance p); one thread per CSR row computes
// eq_rx[row] * sum_e val_e * eq_ry[col_e]; blocks publish partial sums, k_sum_segments adds them.
__device__ __forceinline__ Fq block_sum1(Fq v) {
  __shared__ uint32_t sh[soa_words<Fq, 256>()];  // component-major: no bank conflicts
  int t = threadIdx.x;
  for (int d = 128; d >= 1; d >>= 1) {
    if (t >= d && t < 2 * d) soa_put<256>(sh, t - d, v);
    __syncthreads();
    if (t < d) v = fq_add(v, soa_get<256, Fq>(sh, t));
    __syncthreads();
  }
  if (t == 0) soa_put<256>(sh, 0, v);
  __syncthreads();
  Fq r = soa_get<256, Fq>(sh, 0);
  __syncthreads();
  return r;
}
__global__ void __launch_bounds__(256) k_sparse_eval(const MatDesc* __restrict__ md, const uint32_t* __restrict__ rows,
                                                     const uint32_t* __restrict__ rowptr, const uint32_t* __restrict__ col,
                                                     const Fq* __restrict__ val, const Fq* __restrict__ eq_rx,
                                                     const Fq* __restrict__ eq_ry, Fq* __restrict__ partials) {
  // rows[2p], rows[2p + 1]: the row range [r0, r1) of instance p evaluated here (a rank's share when sharded)
  const int seg = blockIdx.y, p = seg / 3, m = seg % 3;
  const uint32_t row = rows[2 * p] + blockIdx.x * 256 + threadIdx.x;
  Fq acc = fq_zero();
  if (row < rows[2 * p + 1]) {
    const uint32_t* rp = rowptr + md[p].rp[m];
    Fq sr = fq_zero();
    for (uint32_t e = rp[row]; e < rp[row + 1]; e++) sr = fq_add(sr, fq_mul(val[e], eq_ry[col[e]]));
    acc = fq_mul(eq_rx[row], sr);
  }
  acc = block_sum1(acc);
  if (threadIdx.x == 0) partials[(size_t)seg * gridDim.x + blockIdx.x] = acc;
}
__global__ void __launch_bounds__(256) k_sum_segments(const Fq* __restrict__ partials, int nblk, Fq* __restrict__ out) {
  Fq acc = fq_zero();
  for (int i = threadIdx.x; i < nblk; i += 256) acc = fq_add(acc, partials[(size_t)blockIdx.x * nblk + i]);
  acc = block_sum1(acc);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// ------------------------------------------------------------------------------------ host helpers
// (eq tables, UniPoly::from_evals, short MLE evaluations: hostmath.hpp)

// ZK sumcheck round bookkeeping shared by phase 1 and phase 2 (sumcheck.rs:1247-1370).
// The RandomTape is a transcript that only ever absorbs labels, so the values a round draws do not depend on
// the proof: init() draws blinds_poly / blinds_evals as the reference does, then reads every round's
// DotProductProof randomness (d_vec, r_delta, r_beta) from a copy of the tape at that position and computes,
// in one host burst, the points that depend on randomness alone (blind * h terms, delta). The rounds then
// commit only their data-dependent terms, and the tape continues from the copy's final state after the last
// round (no other draw happens between the rounds), so proofs are byte-identical.
struct ZKRounds {
  FqV blinds_poly, blinds_evals;
  Fq claim, blind_claim;
  Pt comm_claim;
  ZKSumcheckP out;
  FqV poly;
  Pt comm_poly;
  std::vector<DotPre> pre;
  std::vector<h::HExt> hp, he;  // blinds_poly[j] * h (gens_4), blinds_evals[j] * h (gens_1)
  Tape tape_end{"", fq_zero()};
  bool ahead = false;
  void init(ProverGens& g, Tape& tape, size_t rounds, const Fq& c, const Fq& b) {
    blinds_poly = tape.vec("blinds_poly", rounds);
    blinds_evals = tape.vec("blinds_evals", rounds);
    claim = c;
    blind_claim = b;
    static const bool on = !getenv("SPG_TAPE_AHEAD") || atoi(getenv("SPG_TAPE_AHEAD")) != 0;
    ahead = on && rounds > 0 && g.gens_4.G.size() == 4;
    if (!ahead) {
      comm_claim = commit_batch(g, {CJob(g.gens_1, {c}, b)})[0];
      return;
    }
    tape_end = tape;
    pre.resize(rounds);
    for (size_t j = 0; j < rounds; j++) {
      pre[j].d = tape_end.vec("d_vec", 4);
      pre[j].r_delta = tape_end.scalar("r_delta");
      pre[j].r_beta = tape_end.scalar("r_beta");
    }
    hp.resize(rounds);
    he.resize(rounds);
    // jobs: comm_claim, then per round blinds_poly h4, blinds_evals h1, r_beta h1, delta (d G4 + r_delta h4)
    std::vector<std::pair<std::vector<size_t>, FqV>> jobs;
    jobs.push_back({{g.gens_1.G[0], g.gens_1.h}, {c, b}});
    for (size_t j = 0; j < rounds; j++) {
      jobs.push_back({{g.gens_4.h}, {blinds_poly[j]}});
      jobs.push_back({{g.gens_1.h}, {blinds_evals[j]}});
      jobs.push_back({{g.gens_1.h}, {pre[j].r_beta}});
      std::vector<size_t> idx(g.gens_4.G.begin(), g.gens_4.G.end());
      idx.push_back(g.gens_4.h);
      FqV sc = pre[j].d;
      sc.push_back(pre[j].r_delta);
      jobs.push_back({idx, sc});
    }
    g.host.run(jobs, nullptr, [&](size_t k, const h::HExt& sum) {
      if (k == 0) {
        comm_claim = compress(sum);
        return;
      }
      const size_t j = (k - 1) / 4;
      switch ((k - 1) % 4) {
        case 0: hp[j] = sum; break;
        case 1: he[j] = sum; break;
        case 2: pre[j].rbh = sum; break;
        default: pre[j].delta = compress(sum);
      }
    });
  }
  // commit the round polynomial and draw r_j
  Fq begin(ProverGens& g, Tr& t, size_t j, const Fq e[3]) {
    Fq ev[4] = {e[0], fq_sub(claim, e[0]), e[1], e[2]};
    poly = uni_from_evals3(ev);
    if (ahead)
      comm_poly = g.host.commit_many_plus({{g.gens_4.G, poly}}, &hp[j])[0];
    else
      comm_poly = commit_batch(g, {CJob(g.gens_4, poly, blinds_poly[j])})[0];
    t.point("comm_poly", comm_poly);
    out.comm_polys.push_back(comm_poly);
    return t.challenge("challenge_nextround");
  }
  void finish(ProverGens& g, Tr& t, Tape& tape, size_t j, const Fq& r_j) {
    Fq eval = uni_eval(poly, r_j);
    Pt comm_eval = ahead ? g.host.commit_many_plus({{{g.gens_1.G[0]}, {eval}}}, &he[j])[0]
                         : commit_batch(g, {CJob(g.gens_1, {eval}, blinds_evals[j])})[0];
    t.point("comm_claim_per_round", comm_claim);
    t.point("comm_eval", comm_eval);
    FqV w = t.challenges("combine_two_claims_to_one", 2);
    Fq target = fq_add(fq_mul(w[0], claim), fq_mul(w[1], eval));
    Fq blind_sc = j == 0 ? blind_claim : blinds_evals[j - 1];
    Fq blind = fq_add(fq_mul(w[0], blind_sc), fq_mul(w[1], blinds_evals[j]));
    size_t n = poly.size();
    FqV a(n);
    Fq pw = fq_one();
    for (size_t k = 0; k < n; k++) {
      Fq a_sc = k == 0 ? fq_dbl(fq_one()) : fq_one();
      a[k] = fq_add(fq_mul(w[0], a_sc), fq_mul(w[1], pw));
      pw = fq_mul(pw, r_j);
    }
    out.proofs.push_back(dotproduct_prove(g, g.gens_1, g.gens_4, t, tape, poly, blinds_poly[j], a, target, blind,
                                          &comm_poly, ahead ? &pre[j] : nullptr));
    if (ahead && j + 1 == pre.size()) tape = tape_end;  // past every round's draws
    claim = eval;
    comm_claim = comm_eval;
    out.comm_evals.push_back(comm_eval);
  }
};

// host wall-clock breakdown of one prove (printed to stderr when SPG_TRACE is set)

// device eq table of a host vector (uploads through the kernel argument)

// workspace slots used here (msm.hip uses 0..12, proto.hip 20..22)
enum {
  WS_AZ = 30, WS_BZ, WS_CZ, WS_Z, WS_ABC, WS_TP, WS_TQ, WS_TX, WS_EQRX, WS_EQP, WS_PART, WS_OUT3, WS_DESC,
  WS_L, WS_BPART, WS_BOUT, WS_EV_RX, WS_EV_RY, WS_EV_PART, WS_EV_OUT, WS_EV_DESC, WS_C1, WS_C2, WS_TQ2, WS_TX2, WS_ABC2,
  WS_EQQ  // (56; spark.hip starts at 60)
};
// phase-1 rounds in modes x and q fold inside the next round's evaluation (sumcheck.hip, FOLD kernels); SPG_SC_FUSE=0
// restores the separate fold launch
// the cubic Lagrange basis on the nodes 0..3 at r (a pair's round j + 1 from its grid at t = r_j)
static void lagrange4(const Fq& r, Fq L[4]) {
  static const Fq inv2 = fq_inv(fq_from_u64(2)), inv6 = fq_inv(fq_from_u64(6));
  const Fq a0 = r, a1 = fq_sub(r, fq_one()), a2 = fq_sub(a1, fq_one()), a3 = fq_sub(a2, fq_one());
  const Fq a01 = fq_mul(a0, a1), a23 = fq_mul(a2, a3);
  L[0] = fq_neg(fq_mul(fq_mul(a1, a23), inv6));
  L[1] = fq_mul(fq_mul(a0, a23), inv2);
  L[2] = fq_neg(fq_mul(fq_mul(a01, a3), inv2));
  L[3] = fq_mul(fq_mul(a01, a2), inv6);
}
// a pair's posted grid (k_phase1_pair / k_phase2_pair) -> round j's (e0, e2, e3) and, once r_j is drawn, round j + 1's
static void pair_round_j(const Fq ev[15], Fq ej[3]) {
  ej[0] = fq_add(ev[0], ev[12]);
  ej[1] = fq_add(ev[2], ev[13]);
  ej[2] = fq_add(ev[3], ev[14]);
}
static void pair_round_j1(const Fq ev[15], const Fq& r_j, Fq ej1[3]) {
  Fq L[4];
  lagrange4(r_j, L);
  for (int y = 0; y < 3; y++) {
    Fq acc = fq_zero();
    for (int k = 0; k < 4; k++) acc = fq_add(acc, fq_mul(L[k], ev[4 * y + k]));
    ej1[y] = acc;
  }
}
static bool sc_fuse_on() {
  static const bool on = !getenv("SPG_SC_FUSE") || atoi(getenv("SPG_SC_FUSE")) != 0;
  return on;
}

struct Prover {
  spg_ctx* ctx;
  ProverGens& g;
  const spg_r1cs_inst& inst;
  const spg_r1cs_witness& wit;
  size_t P, max_np, Y, nws;
  std::vector<size_t> num_proofs, num_inputs;
  Tr& t;
  Tape& tape;
  R1CSProofP pf;
  std::vector<FqV> challenges;
  // device descriptor staging (kept alive until the stream is synchronised)
  std::vector<uint8_t> desc_host;

  Prover(spg_ctx* c, ProverGens& gg, const spg_r1cs_inst& in, const spg_r1cs_witness& w, Tr& tt, Tape& tp)
      : ctx(c), g(gg), inst(in), wit(w), t(tt), tape(tp) {}

  // descriptors are staged in desc_host (256-byte aligned, at most 1 MB per proof) and go up to the device in one
  // copy per flush_desc(); a staged descriptor's device address is valid for kernels launched after that flush
  size_t desc_cur = 0, desc_done = 0;
  uint8_t* desc_dev = nullptr;
  template <class D>
  int stage_desc(const std::vector<D>& v, D** dptr) {
    if (!desc_dev && !(desc_dev = (uint8_t*)ws_get(ctx, WS_DESC, 1 << 20)))
      return set_err(ctx, SPG_E_NOMEM, "descriptor buffer");
    const size_t bytes = v.size() * sizeof(D), off = (desc_cur + 255) & ~(size_t)255;
    if (off + bytes > (1 << 20)) return set_err(ctx, SPG_E_ARG, "too many descriptors");
    if (desc_host.size() < off + bytes) desc_host.resize(off + bytes);
    memcpy(desc_host.data() + off, v.data(), bytes);
    *dptr = (D*)(desc_dev + off);
    desc_cur = off + bytes;
    return 0;
  }
  int flush_desc() {
    if (desc_cur > desc_done)
      SPG_HIP(ctx, hipMemcpyAsync(desc_dev + desc_done, desc_host.data() + desc_done, desc_cur - desc_done,
                                  hipMemcpyHostToDevice, ctx->stream));
    desc_done = desc_cur;
    return 0;
  }

  // instance shard of this rank (R1CSProof sharded by instance p over nranks processes): balanced split,
  // the first P % nranks ranks hold one instance more, so every rank holds one when nranks <= P
  size_t rank = 0, nranks = 1, p0 = 0, p1 = 0;
  static size_t shard_begin(size_t P, size_t nranks, size_t r) {
    return r * (P / nranks) + std::min(r, P % nranks);
  }
  size_t owner_of(size_t p) const {
    size_t r = 0;
    while (r + 1 < nranks && shard_begin(P, nranks, r + 1) <= p) r++;
    return r;
  }
  int allgather(const void* send, size_t bytes, std::vector<uint8_t>& recv);
  int sum_ranks(Fq e[3]);
  // the exchanges of a sharded prove, in order (payload bytes per rank): their sequence depends only on public
  // sizes, so a rank that fails locally between two of them takes part in the next one with its failure as status
  // (run()) and every rank returns from that same exchange -- none is left blocked in a later one
  std::vector<size_t> xplan;
  size_t xdone = 0;
  bool xshared = false;  // an exchange already returned a failure to every rank
  void plan_exchanges(size_t np, size_t nq, size_t nx, size_t nw, size_t ny);
  int exchange(const void* send, size_t bytes, std::vector<uint8_t>& recv);
  int gather_first(const std::vector<const PqxDev*>& tabs, std::vector<std::vector<Fq>>& full);

  int run();
  int run_inner(Laps& lp);
};

int Prover::run() {
  Laps lp;
  int rc0 = run_inner(lp);
  lp.print();
  if (rc0 && nranks > 1 && !xshared && xdone < xplan.size()) {
    // this rank failed alone: the next exchange of the plan carries the failure to every rank
    std::vector<uint8_t> none(xplan[xdone], 0), r;
    xdone++;
    comm_allgather(ctx, Shard{(int)rank, (int)nranks}, rc0, none.data(), none.size(), r);
  }
  return rc0;
}

// ---- cross-rank exchange (identity when nranks == 1): comm.hpp through api.hip's comm_allgather, so every exchange
// carries this rank's status and a failure on one rank fails all of them
int Prover::exchange(const void* send, size_t bytes, std::vector<uint8_t>& recv) {
  const Shard sh{(int)rank, (int)nranks};
  if (nranks > 1 && (xdone >= xplan.size() || xplan[xdone] != bytes)) {
    // the plan is a restatement of run_inner's control flow; a mismatch is a library bug
    const int rc = set_err(ctx, SPG_E_ARG, "sharded R1CSProof: exchange " + std::to_string(xdone) + " of " +
                                               std::to_string(bytes) + " bytes is not in the exchange plan");
    xshared = true;
    std::vector<uint8_t> r;
    comm_allgather(ctx, sh, rc, send, bytes, r);
    return rc;
  }
  xdone++;
  const int rc = comm_allgather(ctx, sh, 0, send, bytes, recv);
  if (rc) xshared = true;
  return rc;
}
int Prover::allgather(const void* send, size_t bytes, std::vector<uint8_t>& recv) { return exchange(send, bytes, recv); }
// (e0, e2, e3) summed over the ranks' instance shards
int Prover::sum_ranks(Fq e[3]) {
  if (nranks == 1) return 0;
  std::vector<uint8_t> r;
  const int rc = exchange(e, 3 * sizeof(Fq), r);
  if (rc) return rc;
  sum_over_ranks(r.data(), (int)nranks, 3, e);
  return 0;
}
// Witness-section polynomials' L.Z widths: Rs = 2^(nv - nv/2) of each (section, instance) polynomial (the bound
// rows that the LZ allgather carries)
static size_t lz_width(size_t np, size_t ni) {
  const size_t nv = lg2(np) + lg2(ni);
  return (size_t)1 << (nv - nv / 2);
}
void Prover::plan_exchanges(size_t np, size_t nq, size_t nx, size_t nw, size_t ny) {
  xplan.clear();
  xdone = 0;
  xshared = false;
  if (nranks == 1) return;
  const size_t PL = (P + nranks - 1) / nranks, sum = 3 * sizeof(Fq);
  // phase 1: one sum per x / q round, the gather of Az, Bz, Cz before the instance rounds
  const size_t r1 = nx + nq + np;
  if (r1 && nx + nq == 0) xplan.push_back(PL * 3 * sizeof(Fq));
  for (size_t j = 0; j < r1; j++) {
    if (j < nx + nq) xplan.push_back(sum);
    if (j + 1 == nx + nq && np > 0) xplan.push_back(PL * 3 * sizeof(Fq));
  }
  // phase 2: one sum per y / w round, the gather of Z (and ABC unless shared) before the instance rounds
  const size_t k2 = inst.num_instances == 1 ? 1 : 2, r2 = ny + nw + np;
  if (r2 && ny + nw == 0) xplan.push_back(PL * k2 * sizeof(Fq));
  for (size_t j = 0; j < r2; j++) {
    if (j < ny + nw) xplan.push_back(sum);
    if (j + 1 == ny + nw && np > 0) xplan.push_back(PL * k2 * sizeof(Fq));
  }
  // the L.Z bounds of every witness polynomial
  size_t lz_total = 0;
  for (size_t i = 0; i < nws; i++)
    for (size_t p = 0; p < wit.num_proofs[i].size(); p++) lz_total += lz_width(wit.num_proofs[i][p], wit.num_inputs[i][p]);
  xplan.push_back(lz_total * sizeof(Fq));
}
// per local instance p, the element (p, 0, 0, 0) of each table -> the same for all P instances, on the host
int Prover::gather_first(const std::vector<const PqxDev*>& tabs, std::vector<std::vector<Fq>>& full) {
  const size_t k = tabs.size(), PL = (P + nranks - 1) / nranks;  // the largest shard; slots per rank
  std::vector<Fq> mine(PL * k, fq_zero());
  {  // one gather per kSegMax elements
    std::vector<FqSeg> segs;
    std::vector<Fq*> dst;
    std::vector<Fq> got;
    auto flush = [&]() -> int {
      got.resize(segs.size());
      int rc = d2h_multi(ctx, segs.data(), (int)segs.size(), got.data());
      for (size_t j = 0; j < segs.size(); j++) *dst[j] = got[j];
      segs.clear();
      dst.clear();
      return rc;
    };
    for (size_t i = 0; i < k; i++) {
      const PqxDev& T = *tabs[i];
      for (size_t p = 0; p < T.zlen; p++) {
        segs.push_back({T.d + T.off[p], 1});
        dst.push_back(&mine[i * PL + p]);
        if (segs.size() == (size_t)kSegMax)
          if (int rc = flush()) return rc;
      }
    }
    if (!segs.empty())
      if (int rc = flush()) return rc;
  }
  std::vector<uint8_t> r;
  int rc = allgather(mine.data(), mine.size() * sizeof(Fq), r);
  if (rc) return rc;
  const Fq* v = (const Fq*)r.data();
  full.assign(k, std::vector<Fq>(P, fq_zero()));
  for (size_t q = 0; q < nranks; q++)
    for (size_t i = 0; i < k; i++)
      for (size_t b = shard_begin(P, nranks, q), p = 0; b + p < shard_begin(P, nranks, q + 1); p++)
        full[i][b + p] = v[q * PL * k + i * PL + p];
  return 0;
}
// a table of n instances holding one element each (what remains of a Pqx table when only the instance
// variables are left unbound); its index / index_high behave exactly like the full table's at (p,0,0,0)
static PqxDev compact_table(Fq* d, size_t n, size_t P) {
  PqxDev T;
  T.d = d;
  T.zlen = n;
  T.total = n;
  for (size_t p = 0; p < n; p++) T.off.push_back(p);
  T.anp.assign(n, 1);
  T.anw.assign(n, 1);
  T.ani.assign(n, 1);
  T.num_instances = npow2(n);
  T.max_num_proofs = 1;
  T.num_witness_secs = 1;
  T.max_num_inputs = 1;
  T.num_proofs.assign(P, 1);
  T.num_inputs.assign(P, 1);
  return T;
}

int Prover::run_inner(Laps& lp) {
  hipStream_t s = ctx->stream;
  t.protocol("R1CS proof");
  size_t num_cons = inst.max_num_cons;
  std::vector<size_t> block_num_cons(P);
  for (size_t p = 0; p < P; p++) block_num_cons[p] = inst.num_cons[inst.num_instances == 1 ? 0 : p];
  size_t np = lg2(npow2(P)), nq = lg2(max_np), nx = lg2(num_cons), nw = lg2(nws), ny = lg2(Y);
  plan_exchanges(np, nq, nx, nw, ny);
  // this rank's instances [p0, p1): everything O(N) lives only here; nranks == 1 -> all of them
  const size_t PLn = p1 - p0;
  std::vector<size_t> l_proofs(num_proofs.begin() + p0, num_proofs.begin() + p1);
  std::vector<size_t> l_inputs(num_inputs.begin() + p0, num_inputs.begin() + p1);
  std::vector<size_t> l_cons(block_num_cons.begin() + p0, block_num_cons.begin() + p1);

  // ---- Z table (p, q_rev, w, x_rev)
  PqxDev Zp;
  Zp.zlen = PLn;
  Zp.off.resize(PLn);
  Zp.anp = l_proofs;
  Zp.anw.assign(PLn, nws);
  Zp.ani = l_inputs;
  size_t ztot = 0;
  static const bool z_tiles_on = !getenv("SPG_Z_TILED") || atoi(getenv("SPG_Z_TILED")) != 0;
  bool z_tiled = z_tiles_on;  // k_z_fill_tiled: every instance's row is whole 256-element tiles
  for (size_t p = 0; p < PLn; p++) {
    Zp.off[p] = ztot;
    ztot += l_proofs[p] * nws * l_inputs[p];
    if (l_inputs[p] < 256) z_tiled = false;
  }
  Zp.total = ztot;
  Zp.num_instances = npow2(P);
  Zp.max_num_proofs = max_np;
  Zp.num_witness_secs = npow2(nws);
  Zp.max_num_inputs = Y;
  Zp.num_proofs = l_proofs;
  Zp.num_inputs = l_inputs;
  Zp.d = (Fq*)ws_get(ctx, WS_Z, ztot * sizeof(Fq) + 64);
  if (!Zp.d) return set_err(ctx, SPG_E_NOMEM, "Z table");
  // ---- Az, Bz, Cz = multiply_vec_block (p, q_rev, 0, x_rev) for the local instances
  PqxDev Az;
  Az.zlen = PLn;
  Az.off.resize(PLn);
  Az.anp = l_proofs;
  Az.anw.assign(PLn, 1);
  Az.ani = l_cons;
  size_t atot = 0;
  for (size_t p = 0; p < PLn; p++) {
    Az.off[p] = atot;
    atot += l_proofs[p] * l_cons[p];
  }
  Az.total = atot;
  Az.num_instances = npow2(P);
  Az.max_num_proofs = max_np;
  Az.num_witness_secs = 1;
  Az.max_num_inputs = num_cons;
  Az.num_proofs = l_proofs;
  Az.num_inputs = l_cons;
  Az.d = (Fq*)ws_get(ctx, WS_AZ, atot * sizeof(Fq) + 64);
  Fq* Bz = (Fq*)ws_get(ctx, WS_BZ, atot * sizeof(Fq) + 64);
  Fq* Cz = (Fq*)ws_get(ctx, WS_CZ, atot * sizeof(Fq) + 64);
  if (!Az.d || !Bz || !Cz) return set_err(ctx, SPG_E_NOMEM, "Az/Bz/Cz");
  static const bool z_side = !getenv("SPG_Z_SIDE") || atoi(getenv("SPG_Z_SIDE")) != 0;
  // whatever way this returns, `stream` is ordered after the fill before anything later reuses the Z slot
  struct SideJoin {
    spg_ctx* c;
    bool armed = false;
    int join() {
      if (!armed) return 0;
      armed = false;
      return hipStreamWaitEvent(c->stream, c->ev_side, 0) == hipSuccess ? 0 : set_err(c, SPG_E_HIP, "z_fill join");
    }
    ~SideJoin() { join(); }
  } z_join{ctx};
  // every descriptor of the setup kernels (Z fill, Az/Bz/Cz) goes up in one host-to-device copy
  SecDesc* dsec = nullptr;
  ZDesc* dz = nullptr;
  MatDesc* dmd = nullptr;
  SpDesc* dsd = nullptr;
  double visits = 0;
  int rc = 0;
  {
    std::vector<ZDesc> zd(PLn);
    std::vector<SecDesc> sd(nws * PLn);
    for (size_t p = 0; p < PLn; p++) {
      zd[p].dom_off = Zp.off[p];
      zd[p].z_off = Zp.off[p];
      zd[p].lg_q = (uint32_t)lg2(l_proofs[p]);
      zd[p].ni = (uint32_t)l_inputs[p];
      zd[p].lg_ni = (uint32_t)lg2(l_inputs[p]);
      for (size_t w = 0; w < nws; w++) {
        size_t pw = wit.num_proofs[w].size() == 1 ? 0 : p0 + p;
        if (!wit.ptr[w][pw]) return set_err(ctx, SPG_E_ARG, "witness shard does not hold instance");
        sd[w * PLn + p].w = wit.ptr[w][pw];
        sd[w * PLn + p].np = (uint32_t)wit.num_proofs[w][pw];
        sd[w * PLn + p].ni = (uint32_t)wit.num_inputs[w][pw];
      }
    }
    std::vector<MatDesc> md(inst.num_instances);
    for (size_t p = 0; p < inst.num_instances; p++) {
      for (int m = 0; m < 3; m++) md[p].rp[m] = inst.rp_off[3 * p + m];
      md[p].cp = inst.cp_off[p];
    }
    std::vector<SpDesc> spd(PLn);
    for (size_t p = 0; p < PLn; p++) {
      size_t pi = inst.num_instances == 1 ? 0 : p0 + p;
      spd[p].dom_off = Az.off[p];
      spd[p].out_off = Az.off[p];
      spd[p].pi = (uint32_t)pi;
      spd[p].lg_q = (uint32_t)lg2(l_proofs[p]);
      spd[p].nrows = (uint32_t)l_cons[p];
      spd[p].lg_rows = (uint32_t)lg2(l_cons[p]);
      spd[p].ni = (uint32_t)l_inputs[p];
      spd[p].lg_ni = (uint32_t)lg2(l_inputs[p]);
      visits += (double)l_proofs[p] * (inst.nnz[3 * pi] + inst.nnz[3 * pi + 1] + inst.nnz[3 * pi + 2]);
    }
    rc = stage_desc(zd, &dz);
    if (!rc) rc = stage_desc(sd, &dsec);
    if (!rc) rc = stage_desc(md, &dmd);
    if (!rc) rc = stage_desc(spd, &dsd);
    if (!rc) rc = flush_desc();
    if (rc) return rc;
  }
  // ---- tau tables (identical on every rank)
  FqV tau_p = t.challenges("challenge_tau_p", np);
  FqV tau_q = t.challenges("challenge_tau_q", nq);
  FqV tau_x = t.challenges("challenge_tau_x", nx);
  if (getenv("SPG_DEBUG_TR")) fprintf(stderr, "[prove] r1cs P=%zu np=%zu nq=%zu nx=%zu tau_x0 %08x\n", (size_t)P, (size_t)np, (size_t)nq, (size_t)nx, tau_x[0].l[0]);
  Fq* Ap = (Fq*)ws_get(ctx, WS_TP, (sizeof(Fq) << np) + 64);
  Fq* Aq = (Fq*)ws_get(ctx, WS_TQ, (sizeof(Fq) << nq) + 64);
  Fq* Ax = (Fq*)ws_get(ctx, WS_TX, (sizeof(Fq) << nx) + 64);
  if (!Ap || !Aq || !Ax) return set_err(ctx, SPG_E_NOMEM, "eq tables");
  rc = eq_tables(ctx, {{tau_p, Ap}, {tau_q, Aq}, {tau_x, Ax}});
  if (rc) return rc;

  {  // ---- Az, Bz, Cz: outputs, CSR row pointers, and per visited entry its column, value and z gather
    KScope ks(ctx, "spmv_block", 96.0 * atot + 12.0 * atot + 68.0 * visits);
    static const bool tiles_on = !getenv("SPG_SPMV_TILED") || atoi(getenv("SPG_SPMV_TILED")) != 0;
    bool tiled = tiles_on;  // every instance's q rows are whole 256-row tiles
    for (size_t p = 0; p < PLn; p++)
      if (l_cons[p] < 256) tiled = false;
    if (tiled)
      hipLaunchKernelGGL(k_spmv<true>, dim3(blocks_for(atot)), dim3(256), 0, s, dsd, (int)PLn, dmd, inst.d_rowptr,
                         inst.d_col, inst.d_val, dsec, (int)nws, (uint32_t)Y, Az.d, Bz, Cz, (uint64_t)atot);
    else
      hipLaunchKernelGGL(k_spmv<false>, dim3(blocks_for(atot)), dim3(256), 0, s, dsd, (int)PLn, dmd, inst.d_rowptr,
                         inst.d_col, inst.d_val, dsec, (int)nws, (uint32_t)Y, Az.d, Bz, Cz, (uint64_t)atot);
    SPG_HIP(ctx, hipGetLastError());
  }
  // k_spmv gathers from the witness itself, so the Z fill only has to land before phase 2. On the second stream it
  // is queued once phase 1's round SPG_Z_AFTER (default 4) has been evaluated, and runs beside the later, smaller
  // rounds: overlapping k_spmv or the first, HBM-bound rounds, the kernels slow each other (rocprof and same-box
  // A/Bs: DESIGN §4, round 4). SPG_Z_SIDE=0 fills it in order here.
  bool z_queued = false;
  static const size_t z_after = getenv("SPG_Z_AFTER") ? (size_t)atol(getenv("SPG_Z_AFTER")) : 4;
  auto queue_z_fill = [&]() -> int {
    if (z_queued) return 0;
    z_queued = true;
    const hipStream_t main_stream = ctx->stream;
    if (z_side) {
      SPG_HIP(ctx, hipEventRecord(ctx->ev_pre, main_stream));
      SPG_HIP(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_pre, 0));
      ctx->stream = ctx->stream2;
    }
    {
      KScope ks(ctx, "z_fill", 64.0 * ztot);
      if (z_tiled)  // (ztot is a multiple of 256 then, and so is every instance's offset)
        hipLaunchKernelGGL(k_z_fill_tiled, dim3((uint32_t)(ztot / 256)), dim3(256), 0, ctx->stream, dz, (int)PLn, dsec,
                           (int)nws, Zp.d);
      else
        hipLaunchKernelGGL(k_z_fill, dim3(blocks_for(ztot)), dim3(256), 0, ctx->stream, dz, (int)PLn, dsec, (int)nws,
                           Zp.d, (uint64_t)ztot);
    }
    ctx->stream = main_stream;
    SPG_HIP(ctx, hipGetLastError());
    if (z_side) {
      SPG_HIP(ctx, hipEventRecord(ctx->ev_side, ctx->stream2));
      z_join.armed = true;
    }
    return 0;
  };
  if (!z_side && (rc = queue_z_fill())) return rc;

  lp.lap("setup");
  // (round evaluations: 3 per workgroup; pair launches: one per element)
  Fq* partials = (Fq*)ws_get(ctx, WS_PART, std::max(3 * (size_t)kScGridMax, kP1PairMax) * sizeof(Fq) + 64);
  if (!partials) return set_err(ctx, SPG_E_NOMEM, "partials");

  // ---- phase 1 (sumcheck.rs:1067-1380)
  FqV rx_all;
  Fq blind_post1;
  Fq claims1[4];
  {
    size_t rounds = nx + nq + np;
    ZKRounds zk;
    size_t cons_len = (size_t)1 << nx, proof_len = (size_t)1 << nq, instance_len = (size_t)1 << np;
    size_t lenP = instance_len, lenQ = proof_len, lenX = cons_len;
    std::vector<size_t> sc_np = l_proofs, sc_nc = l_cons;  // local; P rounds use all-ones of length P
    PqxDev Ac;  // compact Az for the instance rounds; Bc/Cc share its shape
    Fq *Bc = nullptr, *Cc = nullptr;
    PqxDev* T = &Az;
    Fq *TB = Bz, *TC = Cz;
    const Fq* Ap_l = Ap + p0;  // eq(tau_p) indexed by the global instance in the x / q rounds
    // round j's evaluation is enqueued right after round j-1's folds, so it runs on the device while the
    // host finishes round j-1's proof (comm_eval, DotProductProof); eval_wait then collects (e0, e2, e3)
    auto mode_of = [&](size_t j) { return j < nx ? MODE_X : (j < nx + nq ? MODE_Q : MODE_P); };
    // round j's sizes: the half lengths of the reference's loop and the per-instance domain sizes of the round
    auto advance = [&](size_t j) -> int {
      const int mode = mode_of(j);
      if (cons_len > 1) cons_len /= 2;
      else if (proof_len > 1) proof_len /= 2;
      else instance_len /= 2;
      if (mode != MODE_P)
        for (size_t p = 0; p < sc_np.size(); p++) {  // instance_len >= P here: every instance takes part
          if (mode == MODE_X && sc_nc[p] > 1) sc_nc[p] /= 2;
          if (mode == MODE_Q && sc_np[p] > 1) sc_np[p] /= 2;
        }
      return mode;
    };
    auto launch_eval = [&](size_t j, const FoldPlan* fold) -> int {
      const int mode = advance(j);
      if (mode == MODE_P) {
        std::vector<size_t> ones(P, 1);
        return phase1_eval(ctx, *T, mode, proof_len, cons_len, instance_len, ones, ones, Ap, Aq, Ax, T->d, TB, TC,
                           partials, nullptr);
      }
      return phase1_eval(ctx, *T, mode, proof_len, cons_len, instance_len, sc_np, sc_nc, Ap_l, Aq, Ax, T->d, TB,
                         TC, partials, nullptr, fold);
    };
    // the other halves of the Aq / Ax ping-pong pairs (a fused fold writes the folded side table there)
    Fq* Aq2 = nullptr;
    Fq* Ax2 = nullptr;
    if (sc_fuse_on()) {
      Aq2 = (Fq*)ws_get(ctx, WS_TQ2, (sizeof(Fq) << nq) + 64);
      Ax2 = (Fq*)ws_get(ctx, WS_TX2, (sizeof(Fq) << nx) + 64);
      if (!Aq2 || !Ax2) return set_err(ctx, SPG_E_NOMEM, "eq tables");
    }
    // before the first instance round: collect every instance's remaining (Az, Bz, Cz) value
    auto to_compact = [&]() -> int {
      std::vector<std::vector<Fq>> full;
      PqxDev Bt = Az, Ct = Az;
      Bt.d = Bz;
      Ct.d = Cz;
      int r2 = gather_first({&Az, &Bt, &Ct}, full);
      if (r2) return r2;
      Fq* buf = (Fq*)ws_get(ctx, WS_C1, 3 * P * sizeof(Fq) + 64);
      if (!buf) return set_err(ctx, SPG_E_NOMEM, "compact tables");
      for (int i = 0; i < 3; i++)
        SPG_HIP(ctx, hipMemcpyAsync(buf + i * P, full[i].data(), P * sizeof(Fq), hipMemcpyHostToDevice, s));
      SPG_HIP(ctx, hipStreamSynchronize(s));
      Ac = compact_table(buf, P, P);
      Bc = buf + P;
      Cc = buf + 2 * P;
      T = &Ac;
      TB = Bc;
      TC = Cc;
      return 0;
    };
    // ---- two rounds per launch (sumcheck.hip k_phase1_pair; SPG_P1_PAIR=0: one per launch). A pair takes rounds j,
    // j + 1 of one mode (x or q) when every instance's size in that mode is >= 4 and round j + 1's domain holds at most
    // SPG_P1_PAIR_MAX (default 8192) points: the latency-bound rounds. Unsharded proofs only (a sharded round sums 3
    // scalars over the ranks, a pair would sum 15).
    static const bool pair_on = !getenv("SPG_P1_PAIR") || atoi(getenv("SPG_P1_PAIR")) != 0;
    static const size_t pair_max = std::min<size_t>(
        kP1PairMax, getenv("SPG_P1_PAIR_MAX") ? (size_t)atol(getenv("SPG_P1_PAIR_MAX")) : (size_t)8192);
    auto pair_ok = [&](size_t j) -> bool {
      if (!pair_on || !Aq2 || nranks != 1 || j + 1 >= rounds || T != &Az) return false;
      const int m = mode_of(j);
      if (m == MODE_P || mode_of(j + 1) != m) return false;
      size_t dom = 0;
      for (size_t p = 0; p < sc_np.size(); p++) {
        const size_t N = m == MODE_X ? T->num_inputs[p] : T->num_proofs[p];
        const size_t Nl = m == MODE_X ? sc_nc[p] : sc_np[p];  // the round's local size before its halving
        if (N < 4 || N != Nl) return false;
        dom += m == MODE_X ? sc_np[p] * (N / 4) : (N / 4) * sc_nc[p];
      }
      return dom > 0 && dom <= pair_max;
    };
    // rounds j, j + 1 in one launch; nf = 1: round j - 1's pending fold (fp), 2: the previous pair's (r1, r2)
    auto launch_pair = [&](size_t j, int nf, const FoldPlan* fp, const Fq& r1, const Fq& r2) -> int {
      const int m = advance(j);
      P1Pair pp;
      pp.mode = m;
      pp.c = m == MODE_X ? cons_len : proof_len;  // round j's half length of the mode's eq table
      for (size_t p = 0; p < sc_np.size(); p++) {
        const size_t N = m == MODE_X ? T->num_inputs[p] : T->num_proofs[p];
        if (m == MODE_X) {
          pp.rows.push_back(sc_np[p]);
          pp.cols.push_back(N / 4);
          pp.step_x.push_back(pp.c / (N / 2));
          pp.step_q.push_back(proof_len / sc_np[p]);
        } else {
          pp.rows.push_back(N / 4);
          pp.cols.push_back(sc_nc[p]);
          pp.step_q.push_back(pp.c / (N / 2));
          pp.step_x.push_back(cons_len / sc_nc[p]);
        }
      }
      advance(j + 1);
      pp.nf = nf;
      pp.r1 = r1;
      pp.r2 = r2;
      Fq*& E = m == MODE_X ? Ax : Aq;
      Fq*& Ealt = m == MODE_X ? Ax2 : Aq2;
      size_t& lenE = m == MODE_X ? lenX : lenQ;
      if (nf == 1) {
        pp.fstride = fp->stride;
        pp.fmode = fp->arg.fmode;
        pp.side_in = fp->arg.side_in;
        pp.side_out = fp->arg.side_out;
        pp.side_live = fp->arg.side_half;
      } else if (nf == 2) {  // the previous pair's folds of this mode's eq table: E (live lenE) -> Ealt (lenE / 4)
        pp.fmode = m;
        pp.side_in = E;
        pp.side_out = Ealt;
        pp.side_live = lenE / 4;
        std::swap(E, Ealt);
        lenE /= 4;
      }
      pp.Ap = Ap_l;
      pp.Aq = Aq;
      pp.Ax = Ax;
      pp.B = T->d;
      pp.C = TB;
      pp.D = TC;
      int r = phase1_pair(ctx, *T, pp, partials, nullptr);
      if (r) return r;
      // the size bookkeeping of both rounds' folds (the folds themselves ride in the next launch)
      FoldPlan tmp;
      if ((r = pqx_fold_plan(ctx, *T, m, &tmp)) || (r = pqx_fold_plan(ctx, *T, m, &tmp))) return r;
      return 0;
    };
    // a pair's pending folds (r1, r2) on their own launch, before a single round or the instance rounds
    auto fold2x = [&](int m, const Fq& r1, const Fq& r2) -> int {
      P1Pair pp;
      pp.mode = m;
      for (size_t p = 0; p < sc_np.size(); p++) {
        pp.rows.push_back(T->num_proofs[p]);
        pp.cols.push_back(T->num_inputs[p]);
      }
      Fq*& E = m == MODE_X ? Ax : Aq;
      Fq*& Ealt = m == MODE_X ? Ax2 : Aq2;
      size_t& lenE = m == MODE_X ? lenX : lenQ;
      pp.r1 = r1;
      pp.r2 = r2;
      pp.side_in = E;
      pp.side_out = Ealt;
      pp.side_live = lenE / 4;
      pp.B = T->d;
      pp.C = TB;
      pp.D = TC;
      std::swap(E, Ealt);
      lenE /= 4;
      return phase1_fold2x(ctx, *T, pp);
    };
    if (rounds && nx + nq == 0) rc = to_compact();
    bool cur_pair = false;  // the launch in flight evaluates rounds j, j + 1
    if (!rc && rounds) {
      cur_pair = pair_ok(0);
      rc = cur_pair ? launch_pair(0, 0, nullptr, fq_zero(), fq_zero()) : launch_eval(0, nullptr);
    }
    if (rc) return rc;
    zk.init(g, tape, rounds, fq_zero(), fq_zero());  // host precomputation while round 0 evaluates
    for (size_t j = 0; j < rounds;) {
      if (cur_pair) {
        const int mode = mode_of(j);
        Fq ev[15];
        rc = pair_wait(ctx, ev);
        if (!rc && (j == z_after || j + 1 == z_after)) rc = queue_z_fill();
        if (!rc && (j == 1 || j + 1 == 1) && failpoint(ctx, "r1cs_round")) rc = set_err(ctx, SPG_E_HIP, "failpoint r1cs_round");
        if (rc) return rc;
        lp.lap("p1_eval");
        // round j: F(X, 0) + F(X, 1) at X = 0, 2, 3
        Fq ej[3], ej1[3];
        pair_round_j(ev, ej);
        const Fq r_j = zk.begin(g, t, j, ej);
        zk.finish(g, t, tape, j, r_j);
        rx_all.push_back(r_j);
        // round j + 1: the cubics t -> F(t, Y) (Y = 0, 2, 3) at t = r_j
        pair_round_j1(ev, r_j, ej1);
        const Fq r_j1 = zk.begin(g, t, j + 1, ej1);
        lp.lap("p1_host");
        // the next launch: another pair of this mode (the two folds ride in it), else the folds on their own launch
        // and a single round (or the compaction before the instance rounds)
        if (j + 2 < rounds && mode_of(j + 2) == mode && pair_ok(j + 2)) {
          rc = launch_pair(j + 2, 2, nullptr, r_j, r_j1);
          cur_pair = true;
        } else {
          rc = fold2x(mode, r_j, r_j1);
          if (!rc && j + 2 == nx + nq && np > 0) rc = to_compact();
          if (!rc && j + 2 < rounds) {
            cur_pair = pair_ok(j + 2);
            rc = cur_pair ? launch_pair(j + 2, 0, nullptr, fq_zero(), fq_zero()) : launch_eval(j + 2, nullptr);
          }
        }
        if (rc) return rc;
        lp.lap("p1_fold");
        zk.finish(g, t, tape, j + 1, r_j1);
        lp.lap("p1_host");
        rx_all.push_back(r_j1);
        j += 2;
        continue;
      }
      int mode = mode_of(j);
      Fq e[3];
      rc = eval_wait(ctx, e);
      if (!rc && j == z_after) rc = queue_z_fill();  // round j is done and round j + 1 not yet queued
      if (!rc && j == 1 && failpoint(ctx, "r1cs_round")) rc = set_err(ctx, SPG_E_HIP, "failpoint r1cs_round");
      if (!rc && mode != MODE_P) rc = sum_ranks(e);
      if (rc) return rc;
      lp.lap("p1_eval");
      Fq r_j = zk.begin(g, t, j, e);
      lp.lap("p1_host");
      // the round's eq factor is bound in the same launch as Az, Bz, Cz: by the next round's evaluation (fused) when
      // one follows in mode x or q on the same tables, else by a fold launch of its own
      Fq* side = mode == MODE_P ? Ap : (mode == MODE_Q ? Aq : Ax);
      size_t& side_len = mode == MODE_P ? lenP : (mode == MODE_Q ? lenQ : lenX);
      const bool compact_next = j + 1 == nx + nq && np > 0;
      const int next_mode = mode_of(j + 1);
      cur_pair = false;
      if (Aq2 && mode != MODE_P && j + 1 < rounds && !compact_next && next_mode != MODE_P) {
        FoldPlan fp;
        rc = pqx_fold_plan(ctx, *T, mode, &fp);
        Fq*& cur = mode == MODE_Q ? Aq : Ax;
        Fq*& alt = mode == MODE_Q ? Aq2 : Ax2;
        fp.arg.r = r_j;
        fp.arg.fmode = mode;
        fp.arg.side_in = cur;
        fp.arg.side_out = alt;
        fp.arg.side_half = (uint32_t)(side_len / 2);
        std::swap(cur, alt);
        side_len /= 2;
        if (!rc) {
          cur_pair = pair_ok(j + 1);
          rc = cur_pair ? launch_pair(j + 1, 1, &fp, r_j, fq_zero()) : launch_eval(j + 1, &fp);
        }
      } else {
        rc = pqx_bound(ctx, *T, TB, TC, r_j, mode, side, side_len);
        side_len /= 2;
        if (!rc && compact_next) rc = to_compact();
        if (!rc && j + 1 < rounds) {
          cur_pair = pair_ok(j + 1);
          rc = cur_pair ? launch_pair(j + 1, 0, nullptr, fq_zero(), fq_zero()) : launch_eval(j + 1, nullptr);
        }
      }
      if (rc) return rc;
      lp.lap("p1_fold");
      zk.finish(g, t, tape, j, r_j);
      lp.lap("p1_host");
      rx_all.push_back(r_j);
      j++;
    }
    Fq a[6];  // eq factors, then Az, Bz, Cz (a single instance: it sits on this (only) rank's local tables)
    rc = np == 0 ? d2h_multi(ctx, {{Ap, 1}, {Aq, 1}, {Ax, 1}, {Az.d, 1}, {Bz, 1}, {Cz, 1}}, a)
                 : d2h_multi(ctx, {{Ap, 1}, {Aq, 1}, {Ax, 1}, {T->d, 1}, {TB, 1}, {TC, 1}}, a);
    if (rc) return rc;
    claims1[1] = a[3];
    claims1[2] = a[4];
    claims1[3] = a[5];
    claims1[0] = fq_mul(fq_mul(a[0], a[1]), a[2]);
    blind_post1 = zk.blinds_evals[rounds - 1];
    pf.sc1 = std::move(zk.out);
  }
  lp.lap("p1_claims");
  FqV rx_rev(rx_all.begin(), rx_all.begin() + nx), rq_rev(rx_all.begin() + nx, rx_all.begin() + nx + nq),
      rp(rx_all.begin() + nx + nq, rx_all.end());
  FqV rx(rx_rev.rbegin(), rx_rev.rend()), rq(rq_rev.rbegin(), rq_rev.rend());
  // eq(rx) of phase 2 depends on phase 1's challenges alone: on the device while the host runs the sigma protocols
  Fq* eq_rx = (Fq*)ws_get(ctx, WS_EQRX, (sizeof(Fq) << nx) + 64);
  if (!eq_rx) return set_err(ctx, SPG_E_NOMEM, "eq(rx)");
  rc = eq_table(ctx, rx, eq_rx);
  if (rc) return rc;
  Fq tau_claim = claims1[0], Az_claim = claims1[1], Bz_claim = claims1[2], Cz_claim = claims1[3];
  Fq Az_blind = tape.scalar("Az_blind"), Bz_blind = tape.scalar("Bz_blind"), Cz_blind = tape.scalar("Cz_blind"),
     prod_blind = tape.scalar("prod_Az_Bz_blind");
  Pt comm_Cz, comm_Az, comm_Bz, comm_prod;
  Fq prod = fq_mul(Az_claim, Bz_claim);
  Fq blind_expected1 = fq_mul(tau_claim, fq_sub(prod_blind, Cz_blind));
  Fq claim_post1 = fq_mul(fq_sub(prod, Cz_claim), tau_claim);
  // every point of the three sigma protocols in one host burst ahead of the transcript sequence (SPG_SIGMA_AHEAD=0:
  // each protocol commits on its own)
  static const bool sigma_ahead = !getenv("SPG_SIGMA_AHEAD") || atoi(getenv("SPG_SIGMA_AHEAD")) != 0;
  Sigma1Pre sp;
  if (sigma_ahead)
    sigma1_points(g, g.gens_1, tape, Cz_claim, Cz_blind, Az_claim, Az_blind, Bz_claim, Bz_blind, prod, prod_blind,
                  claim_post1, blind_expected1, claim_post1, blind_post1, &sp);
  pf.pok = knowledge_prove(g, g.gens_1, t, tape, Cz_claim, Cz_blind, &comm_Cz, sigma_ahead ? sp.k : nullptr);
  pf.prod = product_prove(g, g.gens_1, t, tape, Az_claim, Az_blind, Bz_claim, Bz_blind, prod, prod_blind, &comm_Az,
                          &comm_Bz, &comm_prod, sigma_ahead ? sp.p : nullptr);
  t.point("comm_Az_claim", comm_Az);
  t.point("comm_Bz_claim", comm_Bz);
  t.point("comm_Cz_claim", comm_Cz);
  t.point("comm_prod_Az_Bz_claims", comm_prod);
  pf.eq1 = equality_prove(g, g.gens_1, t, tape, claim_post1, blind_expected1, claim_post1, blind_post1,
                          sigma_ahead ? sp.e : nullptr);
  lp.lap("sigma1");
  // ---- phase 2 inputs
  Fq r_A = t.challenge("challenge_Az"), r_B = t.challenge("challenge_Bz"), r_C = t.challenge("challenge_Cz");
  Fq claim2 = fq_add(fq_add(fq_mul(r_A, Az_claim), fq_mul(r_B, Bz_claim)), fq_mul(r_C, Cz_claim));
  Fq blind2 = fq_add(fq_add(fq_mul(r_A, Az_blind), fq_mul(r_B, Bz_blind)), fq_mul(r_C, Cz_blind));
  const bool single = inst.num_instances == 1;
  // ABC: the shared matrix once (every rank), or this rank's instances
  const size_t Ab0 = single ? 0 : p0, Abn = single ? 1 : PLn;
  PqxDev ABC;
  ABC.zlen = Abn;
  ABC.off.resize(Abn);
  ABC.anp.assign(Abn, 1);
  ABC.anw.assign(Abn, nws);
  ABC.ani.assign(num_inputs.begin() + Ab0, num_inputs.begin() + Ab0 + Abn);
  size_t btot = 0;
  for (size_t p = 0; p < Abn; p++) {
    ABC.off[p] = btot;
    btot += nws * num_inputs[Ab0 + p];
  }
  ABC.total = btot;
  ABC.num_instances = npow2(inst.num_instances);
  ABC.max_num_proofs = 1;
  ABC.num_witness_secs = npow2(nws);
  ABC.max_num_inputs = Y;
  ABC.num_proofs.assign(P, 1);
  ABC.num_inputs.assign(num_inputs.begin() + Ab0, num_inputs.end());
  ABC.d = (Fq*)ws_get(ctx, WS_ABC, btot * sizeof(Fq) + 64);
  if (!ABC.d) return set_err(ctx, SPG_E_NOMEM, "ABC");
  {
    std::vector<AbcDesc> ad(Abn);
    double visits = 0;
    for (size_t p = 0; p < Abn; p++) {
      ad[p].dom_off = ABC.off[p];
      ad[p].out_off = ABC.off[p];
      ad[p].pi = (uint32_t)(Ab0 + p);
      ad[p].ni = (uint32_t)num_inputs[Ab0 + p];
      ad[p].lg_ni = (uint32_t)lg2(num_inputs[Ab0 + p]);
      size_t pi = Ab0 + p;
      visits += inst.nnz[3 * pi] + inst.nnz[3 * pi + 1] + inst.nnz[3 * pi + 2];
    }
    AbcDesc* dad;
    rc = stage_desc(ad, &dad);
    if (!rc) rc = flush_desc();
    if (rc) return rc;
    KScope ks(ctx, "eval_table_abc", 32.0 * btot + 4.0 * btot + 68.0 * visits);
    hipLaunchKernelGGL(k_abc, dim3(blocks_for(btot)), dim3(256), 0, s, dad, (int)Abn, dmd, inst.d_colptr, inst.d_crow,
                       inst.d_cval, eq_rx, (uint32_t)Y, r_A, r_B, r_C, ABC.d, (uint64_t)btot);
    SPG_HIP(ctx, hipGetLastError());
  }
  rc = queue_z_fill();  // (phase 1 had no rounds)
  if (!rc) rc = z_join.join();  // the Z table's first use
  if (rc) return rc;
  // Z.bound_poly_vars_rq(rq_rev): every q fold in one pass over Z against eq(rq_rev) (k_pqx_bound_q; SPG_Q_BOUND_ALL=0:
  // one fold launch per challenge, each a read-write pass over the live rows)
  static const bool q_all = !getenv("SPG_Q_BOUND_ALL") || atoi(getenv("SPG_Q_BOUND_ALL")) != 0;
  if (q_all && rq_rev.size() >= 2) {
    Fq* eq_q = (Fq*)ws_get(ctx, WS_EQQ, (sizeof(Fq) << rq_rev.size()) + 64);
    if (!eq_q) return set_err(ctx, SPG_E_NOMEM, "eq(rq)");
    rc = eq_table(ctx, rq_rev, eq_q);
    if (!rc) rc = pqx_bound_q_all(ctx, Zp, eq_q, rq_rev.size());
    if (rc) return rc;
  } else {
    for (size_t k = 0; k < rq_rev.size(); k++) {
      rc = pqx_bound(ctx, Zp, nullptr, nullptr, rq_rev[k], MODE_Q);
      if (rc) return rc;
    }
  }
  Fq* eq_p = (Fq*)ws_get(ctx, WS_EQP, (sizeof(Fq) << np) + 64);
  if (!eq_p) return set_err(ctx, SPG_E_NOMEM, "eq(rp)");
  rc = eq_table(ctx, rp, eq_p);
  if (rc) return rc;

  lp.lap("p2_prep");
  // ---- phase 2 (sumcheck.rs:788-1065)
  FqV ry_all;
  Fq claims2[3], blind_post2;
  {
    size_t rounds = ny + nw + np;
    ZKRounds zk;
    size_t inputs_len = (size_t)1 << ny, ws_len = (size_t)1 << nw, instance_len = (size_t)1 << np;
    size_t lenP = instance_len;
    std::vector<size_t> sc_ni = l_inputs;
    PqxDev Zc, ABCc;
    PqxDev *TZ = &Zp, *TA = &ABC;
    const Fq* eq_l = eq_p + p0;
    auto launch_eval = [&](size_t j, const Fold2* fold) -> int {
      int mode = j < ny ? MODE_X : (j < ny + nw ? MODE_W : MODE_P);
      if (inputs_len > 1) inputs_len /= 2;
      else if (ws_len > 1) ws_len /= 2;
      else instance_len /= 2;
      if (mode == MODE_P) {
        std::vector<size_t> ones(P, 1);
        return phase2_eval(ctx, *TA, *TZ, mode, instance_len, ws_len, nws, single, ones, eq_p, partials,
                           nullptr);
      }
      for (size_t p = 0; p < sc_ni.size(); p++)
        if (mode == MODE_X && sc_ni[p] > 1) sc_ni[p] /= 2;
      return phase2_eval(ctx, *TA, *TZ, mode, instance_len, ws_len, nws, single, sc_ni, eq_l, partials,
                         nullptr, fold);
    };
    // one ABC serving every instance is folded into this buffer by a fused round (then the two swap). The fused fold
    // writes it from the points of local instance 0 (global p0): only when that instance spans ABC's whole width
    // (num_inputs[0]) -- a sharded rank whose first instance is narrower takes the separate fold
    const bool fuse2 = sc_fuse_on() && (!single || num_inputs[p0] == num_inputs[0]);
    Fq* ABC2 = nullptr;
    if (fuse2 && single) {
      ABC2 = (Fq*)ws_get(ctx, WS_ABC2, btot * sizeof(Fq) + 64);
      if (!ABC2) return set_err(ctx, SPG_E_NOMEM, "ABC");
    }
    auto to_compact = [&]() -> int {
      std::vector<std::vector<Fq>> full;
      int r2 = single ? gather_first({&Zp}, full) : gather_first({&Zp, &ABC}, full);
      if (r2) return r2;
      Fq* buf = (Fq*)ws_get(ctx, WS_C2, 2 * P * sizeof(Fq) + 64);
      if (!buf) return set_err(ctx, SPG_E_NOMEM, "compact tables");
      SPG_HIP(ctx, hipMemcpyAsync(buf, full[0].data(), P * sizeof(Fq), hipMemcpyHostToDevice, s));
      if (single) {  // the shared ABC keeps its single (0,0,0,0) element
        SPG_HIP(ctx, hipMemcpyAsync(buf + P, ABC.d, sizeof(Fq), hipMemcpyDeviceToDevice, s));
      } else {
        SPG_HIP(ctx, hipMemcpyAsync(buf + P, full[1].data(), P * sizeof(Fq), hipMemcpyHostToDevice, s));
      }
      SPG_HIP(ctx, hipStreamSynchronize(s));
      Zc = compact_table(buf, P, P);
      ABCc = compact_table(buf + P, single ? 1 : P, P);
      TZ = &Zc;
      TA = &ABCc;
      return 0;
    };
    // ---- two y rounds per launch (sumcheck.hip k_phase2_pair; SPG_P2_PAIR=0: one per launch): rounds j, j + 1 both y
    // rounds, ABC per instance, every instance's live y size >= 4 (the same in ABC and Z), at most SPG_P2_PAIR_MAX
    // (default 8192) elements, unsharded. A run of pairs starts with no fold pending (a single round's fold before it is
    // launched on its own) and ends with k_phase2_fold2x.
    static const bool p2_pair_on = !getenv("SPG_P2_PAIR") || atoi(getenv("SPG_P2_PAIR")) != 0;
    static const size_t p2_pair_max = std::min<size_t>(
        kP1PairMax, getenv("SPG_P2_PAIR_MAX") ? (size_t)atol(getenv("SPG_P2_PAIR_MAX")) : (size_t)8192);
    const size_t W2 = std::min(ws_len, nws);
    // (fold_pending: round j - 1's fold is not yet in the tables' sizes; the caller launches it first)
    auto p2_pair_ok = [&](size_t j, bool fold_pending) -> bool {
      // (one ABC shared by every instance folds through its ping-pong buffer, as the fused single rounds do)
      if (!p2_pair_on || (single && !ABC2) || nranks != 1 || j + 1 >= ny || TA != &ABC || TZ != &Zp ||
          ABC.zlen != (single ? 1 : Zp.zlen))
        return false;
      auto live = [&](size_t n) { return fold_pending && n > 1 ? n / 2 : n; };
      size_t dom = 0;
      for (size_t p = 0; p < sc_ni.size(); p++) {
        const size_t N = live(Zp.num_inputs[p]);
        if (N < 4 || live(ABC.num_inputs[single ? 0 : p]) != N || sc_ni[p] != N) return false;
        dom += W2 * (N / 4);
      }
      return dom > 0 && dom <= p2_pair_max;
    };
    // rounds j, j + 1 in one launch; nf = 2: the previous pair's folds (r1, r2) ride in it
    auto launch_p2pair = [&](int nf, const Fq& r1, const Fq& r2) -> int {
      for (int k = 0; k < 2; k++) {  // launch_eval's size bookkeeping for both y rounds
        if (inputs_len > 1) inputs_len /= 2;
        for (size_t p = 0; p < sc_ni.size(); p++)
          if (sc_ni[p] > 1) sc_ni[p] /= 2;
      }
      P2Pair pp;
      pp.nf = nf;
      pp.r1 = r1;
      pp.r2 = r2;
      pp.W = W2;
      pp.eq = eq_l;
      pp.B_out = single ? ABC2 : nullptr;
      int r = phase2_pair(ctx, ABC, Zp, pp, partials);
      if (r) return r;
      if (single && nf == 2) std::swap(ABC.d, ABC2);  // the folded shared ABC is in the other buffer now
      FoldPlan tmp;  // the table bookkeeping of both rounds' folds (the folds ride in the next launch)
      for (int k = 0; k < 2 && !r; k++) {
        r = pqx_fold_plan(ctx, ABC, MODE_X, &tmp);
        if (!r) r = pqx_fold_plan(ctx, Zp, MODE_X, &tmp);
      }
      return r;
    };
    auto p2_fold2x = [&](const Fq& r1, const Fq& r2) -> int {
      P2Pair pp;
      pp.nf = 2;
      pp.r1 = r1;
      pp.r2 = r2;
      pp.W = W2;
      pp.B_out = single ? ABC2 : nullptr;
      const int r = phase2_fold2x(ctx, ABC, Zp, pp);
      if (!r && single) std::swap(ABC.d, ABC2);
      return r;
    };
    bool cur_pair = false;  // the launch in flight evaluates rounds j, j + 1
    if (rounds && ny + nw == 0) rc = to_compact();
    if (!rc && rounds) {
      cur_pair = p2_pair_ok(0, false);
      rc = cur_pair ? launch_p2pair(0, fq_zero(), fq_zero()) : launch_eval(0, nullptr);
    }
    if (rc) return rc;
    zk.init(g, tape, rounds, claim2, blind2);  // host precomputation while round 0 evaluates
    for (size_t j = 0; j < rounds;) {
      if (cur_pair) {
        Fq ev[15], ej[3], ej1[3];
        rc = pair_wait(ctx, ev);
        if (rc) return rc;
        lp.lap("p2_eval");
        pair_round_j(ev, ej);
        const Fq r_j = zk.begin(g, t, j, ej);
        zk.finish(g, t, tape, j, r_j);
        ry_all.push_back(r_j);
        pair_round_j1(ev, r_j, ej1);
        const Fq r_j1 = zk.begin(g, t, j + 1, ej1);
        lp.lap("p2_host");
        if (j + 2 < ny && p2_pair_ok(j + 2, false)) {
          rc = launch_p2pair(2, r_j, r_j1);
        } else {
          cur_pair = false;
          rc = p2_fold2x(r_j, r_j1);
          if (!rc && j + 2 == ny + nw && np > 0) rc = to_compact();
          if (!rc && j + 2 < rounds) rc = launch_eval(j + 2, nullptr);
        }
        if (rc) return rc;
        lp.lap("p2_fold");
        zk.finish(g, t, tape, j + 1, r_j1);
        lp.lap("p2_host");
        ry_all.push_back(r_j1);
        j += 2;
        continue;
      }
      int mode = j < ny ? MODE_X : (j < ny + nw ? MODE_W : MODE_P);
      Fq e[3];
      rc = eval_wait(ctx, e);
      if (!rc && mode != MODE_P) rc = sum_ranks(e);
      if (rc) return rc;
      lp.lap("p2_eval");
      Fq r_j = zk.begin(g, t, j, e);
      lp.lap("p2_host");
      const bool compact_next = j + 1 == ny + nw && np > 0;
      const int next_mode = j + 1 < ny ? MODE_X : (j + 1 < ny + nw ? MODE_W : MODE_P);
      if (mode == MODE_X && p2_pair_ok(j + 1, true)) {
        // a run of pairs starts here: this round's fold on its own launch, then the pair (no fold pending in it)
        rc = pqx_bound2(ctx, *TA, *TZ, r_j, mode);
        if (!rc) rc = launch_p2pair(0, fq_zero(), fq_zero());
        cur_pair = true;
      } else if (fuse2 && mode != MODE_P && j + 1 < rounds && !compact_next && next_mode != MODE_P) {
        // the fold rides in the next round's evaluation (k_phase2_eval<true>)
        Fold2 f;
        rc = pqx_fold_plan(ctx, *TA, mode, &f.a);
        if (!rc) rc = pqx_fold_plan(ctx, *TZ, mode, &f.z);
        f.arg.r = r_j;
        f.arg.fmode = mode;
        f.arg.fw = f.z.fw;
        f.arg.ping = single ? 1 : 0;
        f.arg.b_out = single ? ABC2 : TA->d;
        if (!rc) rc = launch_eval(j + 1, &f);
        if (!rc && single) std::swap(TA->d, ABC2);
      } else {
        if (mode == MODE_P) { rc = dev_fold_top(ctx, eq_p, lenP, r_j); lenP /= 2; }
        if (!rc && (mode != MODE_P || !single)) rc = pqx_bound2(ctx, *TA, *TZ, r_j, mode);
        else if (!rc) rc = pqx_bound(ctx, *TZ, nullptr, nullptr, r_j, mode);
        if (!rc && compact_next) rc = to_compact();
        if (!rc && j + 1 < rounds) rc = launch_eval(j + 1, nullptr);
      }
      if (rc) return rc;
      lp.lap("p2_fold");
      zk.finish(g, t, tape, j, r_j);
      lp.lap("p2_host");
      ry_all.push_back(r_j);
      j++;
    }
    rc = d2h_multi(ctx, {{eq_p, 1}, {TA->d, 1}, {TZ->d, 1}}, claims2);
    if (rc) return rc;
    blind_post2 = zk.blinds_evals[rounds - 1];
    pf.sc2 = std::move(zk.out);
  }
  FqV ry_rev(ry_all.begin(), ry_all.begin() + ny), rw(ry_all.begin() + ny, ry_all.begin() + ny + nw),
      rp2(ry_all.begin() + ny + nw, ry_all.end());
  FqV ry(ry_rev.rbegin(), ry_rev.rend());

  // ---- witness-section evaluations and their batched opening (r1csproof.rs:518-639)
  FqV ry_factors(ny + 1, fq_one());
  for (size_t i = 0; i < ny; i++) ry_factors[i + 1] = fq_mul(ry_factors[i], fq_sub(fq_one(), ry[i]));
  struct PolyRef {
    size_t w, p, np, ni, Rs;
    bool mine;
    FqV LZ, R;
    Fq ev;
  };
  std::vector<PolyRef> polys;
  size_t lz_total = 0;
  for (size_t i = 0; i < nws; i++) {
    for (size_t p = 0; p < wit.num_proofs[i].size(); p++) {
      PolyRef pr;
      pr.w = i;
      pr.p = p;
      pr.np = wit.num_proofs[i][p];
      pr.ni = wit.num_inputs[i][p];
      size_t lnp = lg2(pr.np), lni = lg2(pr.ni);
      size_t nv = lnp + (pr.ni >= Y ? lni : lni);
      pr.Rs = (size_t)1 << (nv - nv / 2);
      pr.mine = wit.num_proofs[i].size() == 1 ? rank == 0 : (p >= p0 && p < p1);
      lz_total += pr.Rs;
      polys.push_back(std::move(pr));
    }
  }
  // LZ = bound(L) of each owned polynomial on this rank's device, then shared with every rank. Every
  // polynomial's eq(rl), partial column sums and LZ are queued back to back into disjoint workspace ranges and
  // the LZ of all of them come back in one download (one host wait instead of one per polynomial).
  std::vector<Fq> lz_mine(lz_total, fq_zero());
  {
    struct BoundJob {
      FqV rl;
      size_t Ls, Rs, S, chunk, offL, offP, o;
    };
    std::vector<BoundJob> jobs;
    size_t o = 0, totL = 0, totP = 0;
    bool all_mine = true;
    std::vector<FqV> rr_of(polys.size());  // each polynomial's right point; R = eq(rr) once per distinct point, below
    size_t pk = 0;
    for (auto& pr : polys) {
      size_t lnp = lg2(pr.np), lni = lg2(pr.ni);
      FqV r(rq.begin() + (nq - lnp), rq.end());
      if (pr.ni >= Y) {
        r.insert(r.end(), lni - ny, fq_zero());
        r.insert(r.end(), ry.begin(), ry.end());
      } else {
        r.insert(r.end(), ry.begin() + (ny - lni), ry.end());
      }
      size_t nv = r.size(), ln = nv / 2;
      FqV rl(r.begin(), r.begin() + ln), rr(r.begin() + ln, r.end());
      size_t Ls = (size_t)1 << ln, Rs = (size_t)1 << (nv - ln);
      rr_of[pk++] = std::move(rr);
      if (pr.mine) {
        size_t S = std::min<size_t>(Ls, 32);  // 32 partial rows: short column sums
        const size_t chunk = (Ls + S - 1) / S;
        S = (Ls + chunk - 1) / chunk;
        jobs.push_back({std::move(rl), Ls, Rs, S, chunk, totL, totP, o});
        totL += Ls;
        totP += S * Rs;
      } else {
        all_mine = false;
      }
      o += Rs;
    }
    // the host eq tables of the distinct right points (instances of one shape share theirs), on the pool, while the
    // device computes the LZ (queued first; d2h_fq below waits for them)
    auto right_tables = [&]() {
      std::vector<size_t> uniq, at(polys.size());
      for (size_t k = 0; k < polys.size(); k++) {
        size_t u = 0;
        while (u < uniq.size() && !(rr_of[uniq[u]].size() == rr_of[k].size() &&
                                    memcmp(rr_of[uniq[u]].data(), rr_of[k].data(), rr_of[k].size() * sizeof(Fq)) == 0))
          u++;
        if (u == uniq.size()) uniq.push_back(k);
        at[k] = u;
      }
      std::vector<FqV> tabs(uniq.size());
      pool().parallel_for((int)uniq.size(), [&](int u) { tabs[u] = eq_evals_host(rr_of[uniq[u]]); });
      for (size_t k = 0; k < polys.size(); k++) polys[k].R = tabs[at[k]];
    };
    if (jobs.empty()) right_tables();
    if (!jobs.empty()) {
      Fq* dL = (Fq*)ws_get(ctx, WS_L, totL * sizeof(Fq) + 64);
      Fq* dpart = (Fq*)ws_get(ctx, WS_BPART, totP * sizeof(Fq) + 64);
      Fq* dout = (Fq*)ws_get(ctx, WS_BOUT, lz_total * sizeof(Fq) + 64);
      if (!dL || !dpart || !dout) return set_err(ctx, SPG_E_NOMEM, "bound");
      if (!all_mine) SPG_HIP(ctx, hipMemsetAsync(dout, 0, lz_total * sizeof(Fq), s));  // other ranks' ranges
      // one eq table per distinct rl (polynomials of one shape share it)
      std::vector<size_t> eq_at(jobs.size());
      std::vector<EqJob> eqs;
      for (size_t k = 0; k < jobs.size(); k++) {
        size_t same = k;
        for (size_t m = 0; m < k; m++)
          if (jobs[m].rl.size() == jobs[k].rl.size() &&
              memcmp(jobs[m].rl.data(), jobs[k].rl.data(), jobs[k].rl.size() * sizeof(Fq)) == 0) {
            same = m;
            break;
          }
        eq_at[k] = same == k ? jobs[k].offL : eq_at[same];
        if (same == k) eqs.push_back({jobs[k].rl.data(), (int)jobs[k].rl.size(), dL + jobs[k].offL});
      }
      rc = dev_eq_tables(ctx, eqs.data(), (int)eqs.size());
      if (rc) return rc;
      std::vector<const PolyRef*> mine;
      for (auto& pr : polys)
        if (pr.mine) mine.push_back(&pr);
      double bytes = 0;
      for (const BoundJob& j : jobs) bytes += 32.0 * j.Ls * j.Rs + 32.0 * j.Ls + 64.0 * j.S * j.Rs;
      KScope ks(ctx, "poly_bound", bytes);
      for (size_t k0 = 0; k0 < jobs.size(); k0 += kBoundMax) {  // two launches per kBoundMax polynomials
        BoundJobs bj;
        bj.n = (int)std::min<size_t>(kBoundMax, jobs.size() - k0);
        uint32_t nb = 0, nc = 0;
        for (int q = 0; q < bj.n; q++) {
          const BoundJob& j = jobs[k0 + q];
          const PolyRef& pr = *mine[k0 + q];
          const uint32_t nbx = (uint32_t)((j.Rs + 255) / 256);
          bj.d[q] = {wit.ptr[pr.w][pr.p], (uint32_t)eq_at[k0 + q], (uint32_t)j.Ls, (uint32_t)j.Rs,
                     (uint32_t)j.chunk, (uint32_t)j.S, (uint32_t)j.offP, (uint32_t)j.o, nb, nc};
          nb += nbx * (uint32_t)j.S;
          nc += (uint32_t)((j.Rs + kSumCols - 1) / kSumCols);
        }
        hipLaunchKernelGGL(k_bound_part_multi, dim3(nb), dim3(256), 0, s, bj, dL, dpart);
        hipLaunchKernelGGL(k_sum_cols_multi, dim3(nc), dim3(256), 0, s, bj, dpart, dout);
      }
      SPG_HIP(ctx, hipGetLastError());
      right_tables();
      rc = d2h_fq(ctx, dout, lz_mine.data(), lz_total);
      if (rc) return rc;
    }
  }
  {
    std::vector<uint8_t> r;
    rc = allgather(lz_mine.data(), lz_total * sizeof(Fq), r);
    if (rc) return rc;
    const Fq* v = (const Fq*)r.data();
    size_t o = 0;
    for (auto& pr : polys) {
      size_t owner = 0;
      if (wit.num_proofs[pr.w].size() != 1) owner = owner_of(pr.p);
      pr.LZ.assign(v + owner * lz_total + o, v + owner * lz_total + o + pr.Rs);
      o += pr.Rs;
    }
  }
  std::vector<FqV> eval_list(nws);
  pf.comm_vars_at_ry_list.assign(nws, {});
  {
    size_t k = 0;
    std::vector<CJob> cj;  // every evaluation's commitment in one host burst
    // <LZ, R> of every polynomial, one pool task each
    pool().parallel_for((int)polys.size(), [&](int q) {
      PolyRef& pr = polys[q];
      Fq ev = fq_zero();
      for (size_t m = 0; m < pr.Rs; m++) ev = fq_add(ev, fq_mul(pr.LZ[m], pr.R[m]));
      pr.ev = ev;
    });
    for (size_t i = 0; i < nws; i++) {
      eval_list.push_back({});
      for (size_t p = 0; p < wit.num_proofs[i].size(); p++, k++) {
        PolyRef& pr = polys[k];
        const Fq ev = pr.ev;
        size_t lni = lg2(pr.ni);
        eval_list[i].push_back(pr.ni >= Y ? ev : fq_mul(ev, ry_factors[ny - lni]));
        cj.push_back(CJob(g.gens_1, {ev}, fq_zero()));
      }
    }
    const std::vector<Pt> cv = commit_batch(g, cj);
    k = 0;
    for (size_t i = 0; i < nws; i++) {
      pf.comm_vars_at_ry_list.push_back({});
      for (size_t p = 0; p < wit.num_proofs[i].size(); p++) pf.comm_vars_at_ry_list[i].push_back(cv[k++]);
    }
  }
  lp.lap("polyeval_bound");
  // PolyEvalProof::prove_batched_instances_disjoint_rounds (dense_mlpoly.rs:861-960)
  {
    t.protocol("polynomial evaluation proof");
    std::vector<std::pair<size_t, size_t>> keys;
    std::vector<FqV> LZ_list, R_list;
    FqV Zc;
    Fq c_base = t.challenge("challenge_c");
    Fq c = fq_one();
    // the coefficients in the reference's order (c advances once per polynomial joining an earlier shape), then every
    // LZ_list[idx] += c LZ over the pool (axpy_pool; config 4 adds 7 x 1024 products here, ~170 us on one thread)
    std::vector<int> into(polys.size(), -1);
    std::vector<Fq> coef(polys.size());
    for (size_t q = 0; q < polys.size(); q++) {
      const PolyRef& pr = polys[q];
      std::pair<size_t, size_t> key = {pr.np, pr.ni};
      size_t idx = keys.size();
      for (size_t k = 0; k < keys.size(); k++)
        if (keys[k] == key) { idx = k; break; }
      if (idx < keys.size()) {
        c = fq_mul(c, c_base);
        into[q] = (int)idx;
        coef[q] = c;
        Zc[idx] = fq_add(Zc[idx], fq_mul(c, pr.ev));
      } else {
        keys.push_back(key);
        Zc.push_back(pr.ev);
        LZ_list.push_back(pr.LZ);
        R_list.push_back(pr.R);
      }
    }
    std::vector<Axpy> ax;  // (LZ_list no longer grows: its element addresses are stable)
    for (size_t q = 0; q < polys.size(); q++)
      if (into[q] >= 0) ax.push_back({&LZ_list[into[q]], coef[q], &polys[q].LZ});
    axpy_pool(ax);
    for (size_t k = 0; k < LZ_list.size(); k++) {
      DotProductProofLogP dp;
      Pt cy;
      rc = dotproduct_log_prove(ctx, g, t, tape, LZ_list[k], fq_zero(), R_list[k], Zc[k], fq_zero(), &dp, &cy);
      if (rc) return rc;
      pf.evals.push_back(std::move(dp));
    }
  }
  lp.lap("polyeval_dotlog");
  // prefix_list (r1csproof.rs:577-606) and the combined evaluation
  FqV prefix;
  {
    Fq one = fq_one();
    size_t W2 = npow2(nws);
    if (W2 == 1) prefix = {one};
    else if (W2 == 2) prefix = {fq_sub(one, rw[0]), rw[0]};
    else if (W2 == 4)
      prefix = {fq_mul(fq_sub(one, rw[0]), fq_sub(one, rw[1])), fq_mul(fq_sub(one, rw[0]), rw[1]),
                fq_mul(rw[0], fq_sub(one, rw[1])), fq_mul(rw[0], rw[1])};
    else
      for (int i = 0; i < 8; i++) {
        Fq a = (i & 4) ? rw[0] : fq_sub(one, rw[0]);
        Fq b = (i & 2) ? rw[1] : fq_sub(one, rw[1]);
        Fq cc = (i & 1) ? rw[2] : fq_sub(one, rw[2]);
        prefix.push_back(fq_mul(fq_mul(a, b), cc));
      }
  }
  FqV comb_list;
  for (size_t p = 0; p < P; p++) {
    Fq comb = fq_zero();
    for (size_t i = 0; i < nws; i++) {
      size_t pw = wit.num_proofs[i].size() == 1 ? 0 : p;
      comb = fq_add(comb, fq_mul(prefix[i], eval_list[i][pw]));
    }
    for (size_t q = 0; q < nq - lg2(num_proofs[p]); q++) comb = fq_mul(comb, fq_sub(fq_one(), rq[q]));
    comb_list.push_back(comb);
  }
  Fq eval_vars_at_ry = dense_eval_host(comb_list, rp2);
  pf.comm_vars_at_ry = commit_batch(g, {CJob(g.gens_1, {eval_vars_at_ry}, fq_zero())})[0];
  Fq claim_post2 = fq_mul(fq_mul(claims2[0], claims2[1]), claims2[2]);
  pf.eq2 = equality_prove(g, g.gens_1, t, tape, claim_post2, fq_zero(), claim_post2, blind_post2);
  pf.claims_phase2[0] = comm_Az;
  pf.claims_phase2[1] = comm_Bz;
  pf.claims_phase2[2] = comm_Cz;
  pf.claims_phase2[3] = comm_prod;
  FqV rwry(rw);
  rwry.insert(rwry.end(), ry.begin(), ry.end());
  challenges = {rp2, rq_rev, rx, rwry};
  lp.lap("final");
  return 0;
}


}  // namespace spg

using namespace spg;

// ------------------------------------------------------------------------------------ C-ABI
extern "C" int spg_transcript_new(const char* label, spg_transcript** out) {
  if (!label || !out) return SPG_E_ARG;
  *out = new spg_transcript(label);
  return SPG_OK;
}
extern "C" int spg_transcript_new_callbacks(spg_transcript_append_fn append, spg_transcript_challenge_fn challenge,
                                            void* user, spg_transcript** out) {
  if (!append || !challenge || !out) return SPG_E_ARG;
  spg_transcript* t = new spg_transcript("");  // its own merlin state is never used
  t->t.cb = std::make_shared<TrCallbacks>();
  t->t.cb->append = append;
  t->t.cb->challenge = challenge;
  t->t.cb->user = user;
  *out = t;
  return SPG_OK;
}
extern "C" int spg_transcript_append_message(spg_transcript* t, const char* label, const uint8_t* msg, size_t len) {
  if (!t || !label || (!msg && len)) return SPG_E_ARG;
  t->t.message(label, msg, len);
  return t->t.failed() ? SPG_E_CALLBACK : SPG_OK;
}
extern "C" int spg_transcript_append_scalar(spg_transcript* t, const char* label, const uint64_t* scalar_mont) {
  if (!t || !label || !scalar_mont) return SPG_E_ARG;
  t->t.scalar(label, ld_fq(scalar_mont));
  return t->t.failed() ? SPG_E_CALLBACK : SPG_OK;
}
extern "C" int spg_transcript_challenge_scalar(spg_transcript* t, const char* label, uint64_t* out_mont) {
  if (!t || !label || !out_mont) return SPG_E_ARG;
  st_fq(out_mont, t->t.challenge(label));
  return t->t.failed() ? SPG_E_CALLBACK : SPG_OK;
}
extern "C" int spg_transcript_challenge_bytes(spg_transcript* t, const char* label, uint8_t* out, size_t len) {
  if (!t || !label || (!out && len)) return SPG_E_ARG;
  t->t.challenge_bytes(label, out, len);
  return t->t.failed() ? SPG_E_CALLBACK : SPG_OK;
}
extern "C" int spg_transcript_free(spg_transcript* t) {
  delete t;
  return SPG_OK;
}
extern "C" int spg_random_tape_new(const char* name, const uint64_t* init_mont, spg_random_tape** out) {
  if (!name || !init_mont || !out) return SPG_E_ARG;
  *out = new spg_random_tape(name, ld_fq(init_mont));
  return SPG_OK;
}
extern "C" int spg_random_tape_scalar(spg_random_tape* tp, const char* label, uint64_t* out_mont) {
  if (!tp || !label || !out_mont) return SPG_E_ARG;
  st_fq(out_mont, tp->t.scalar(label));
  return SPG_OK;
}
extern "C" int spg_random_tape_free(spg_random_tape* tp) {
  delete tp;
  return SPG_OK;
}

extern "C" int spg_r1cs_gens_new(spg_ctx* ctx, const uint8_t* label, size_t label_len, size_t num_vars,
                                 spg_r1cs_gens** out) {
  if (!ctx || !label || !out || num_vars == 0) return SPG_E_ARG;
  size_t nv = lg2(num_vars);
  size_t n_pc = (size_t)1 << (nv - nv / 2);  // poly_commit_gens_new: 2^right
  spg_r1cs_gens* rg = new spg_r1cs_gens();
  ProverGens& g = rg->g;
  size_t n = std::max<size_t>(n_pc + 1, 4);
  int rc = spg_gens_derive(ctx, label, label_len, n, &g.dev);
  if (rc) {
    delete rg;
    return rc;
  }
  g.host.init(g.dev->compressed, n + 1);
  g.n_pc = n_pc;
  g.gens_n.G.resize(n_pc);
  for (size_t i = 0; i < n_pc; i++) g.gens_n.G[i] = i;
  g.gens_n.h = n_pc + 1;
  g.gens_1.G = {n_pc};
  g.gens_1.h = n_pc + 1;
  g.gens_4.G = {0, 1, 2, 3};
  g.gens_4.h = 4;
  // warm the host fixed-base tables of the sigma-protocol generators
  for (size_t i : {(size_t)0, (size_t)1, (size_t)2, (size_t)3, (size_t)4, n_pc, n_pc + 1}) g.host.get(i);
  *out = rg;
  return SPG_OK;
}
extern "C" int spg_r1cs_gens_free(spg_ctx* ctx, spg_r1cs_gens* g) {
  if (!g) return SPG_OK;
  spg_gens_free(ctx, g->g.dev);
  delete g;
  return SPG_OK;
}
extern "C" int spg_r1cs_gens_download(spg_ctx* ctx, const spg_r1cs_gens* g, uint8_t* out, size_t* count) {
  if (!ctx || !g || !count) return SPG_E_ARG;
  *count = g->g.dev->n + 1;
  if (out) memcpy(out, g->g.dev->compressed, 32 * (g->g.dev->n + 1));
  return SPG_OK;
}

extern "C" int spg_r1cs_inst_new(spg_ctx* ctx, const spg_r1cs_instance* ci, spg_r1cs_inst** out) {
  if (!ctx || !ci || !out || !ci->num_instances || !ci->num_cons || !ci->nnz || !ci->entries) return SPG_E_ARG;
  if (!is_pow2(ci->max_num_cons) || !is_pow2(ci->num_vars))
    return set_err(ctx, SPG_E_ARG, "max_num_cons and num_vars must be powers of two");
  size_t Pm = ci->num_instances;
  std::vector<uint32_t> rowptr, col, colptr, crow;
  std::vector<Fq> val, cval;
  spg_r1cs_inst* I = new spg_r1cs_inst();
  I->num_instances = Pm;
  I->max_num_cons = ci->max_num_cons;
  I->num_vars = ci->num_vars;
  I->num_cons.assign(ci->num_cons, ci->num_cons + Pm);
  for (size_t p = 0; p < Pm; p++) {
    size_t nc = ci->num_cons[p];
    if (!is_pow2(nc) || nc > ci->max_num_cons) {
      delete I;
      return set_err(ctx, SPG_E_ARG, "num_cons must be powers of two <= max_num_cons");
    }
    // CSR per matrix (counting sort by row, stable in entry order)
    for (int m = 0; m < 3; m++) {
      size_t nnz = ci->nnz[3 * p + m];
      I->nnz.push_back(nnz);
      const spg_sparse_entry* E = ci->entries[3 * p + m];
      if (nnz && !E) {
        delete I;
        return SPG_E_ARG;
      }
      std::vector<uint32_t> cnt(nc + 1, 0);
      for (size_t e = 0; e < nnz; e++) {
        if (E[e].row >= nc || E[e].col >= ci->num_vars) {
          delete I;
          return set_err(ctx, SPG_E_ARG, "sparse entry out of range");
        }
        cnt[E[e].row + 1]++;
      }
      for (size_t r = 0; r < nc; r++) cnt[r + 1] += cnt[r];
      I->rp_off.push_back(rowptr.size());
      size_t base = col.size();
      for (size_t r = 0; r <= nc; r++) rowptr.push_back((uint32_t)(base + cnt[r]));
      col.resize(base + nnz);
      val.resize(base + nnz);
      std::vector<uint32_t> fill(cnt.begin(), cnt.end() - 1);
      for (size_t e = 0; e < nnz; e++) {
        size_t d = base + fill[E[e].row]++;
        col[d] = (uint32_t)E[e].col;
        val[d] = ld_fq(E[e].val);
      }
    }
    // merged CSC over A, B, C with tagged rows
    size_t ncol = ci->num_vars;
    std::vector<uint32_t> cnt(ncol + 1, 0);
    for (int m = 0; m < 3; m++)
      for (size_t e = 0; e < ci->nnz[3 * p + m]; e++) cnt[ci->entries[3 * p + m][e].col + 1]++;
    for (size_t c = 0; c < ncol; c++) cnt[c + 1] += cnt[c];
    I->cp_off.push_back(colptr.size());
    size_t base = crow.size();
    for (size_t c = 0; c <= ncol; c++) colptr.push_back((uint32_t)(base + cnt[c]));
    crow.resize(base + cnt[ncol]);
    cval.resize(base + cnt[ncol]);
    std::vector<uint32_t> fill(cnt.begin(), cnt.end() - 1);
    for (int m = 0; m < 3; m++)
      for (size_t e = 0; e < ci->nnz[3 * p + m]; e++) {
        const spg_sparse_entry& en = ci->entries[3 * p + m][e];
        size_t d = base + fill[en.col]++;
        crow[d] = (uint32_t)(en.row * 4 + m);
        cval[d] = ld_fq(en.val);
      }
  }
  if (col.size() >= 0xffffffffULL || crow.size() >= 0xffffffffULL || ci->max_num_cons >= (1ull << 30)) {
    delete I;
    return set_err(ctx, SPG_E_ARG, "instance too large");
  }
  auto up = [&](void** d, const void* h, size_t bytes) -> int {
    if (hipMalloc(d, bytes ? bytes : 16) != hipSuccess) return SPG_E_NOMEM;
    if (bytes && hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice) != hipSuccess) return SPG_E_HIP;
    return 0;
  };
  int rc = up((void**)&I->d_rowptr, rowptr.data(), rowptr.size() * 4);
  if (!rc) rc = up((void**)&I->d_col, col.data(), col.size() * 4);
  if (!rc) rc = up((void**)&I->d_val, val.data(), val.size() * sizeof(Fq));
  if (!rc) rc = up((void**)&I->d_colptr, colptr.data(), colptr.size() * 4);
  if (!rc) rc = up((void**)&I->d_crow, crow.data(), crow.size() * 4);
  if (!rc) rc = up((void**)&I->d_cval, cval.data(), cval.size() * sizeof(Fq));
  if (rc) {
    spg_r1cs_inst_free(ctx, I);
    return set_err(ctx, rc, "instance upload");
  }
  *out = I;
  return SPG_OK;
}
extern "C" int spg_r1cs_inst_free(spg_ctx* ctx, spg_r1cs_inst* I) {
  (void)ctx;
  if (!I) return SPG_OK;
  hipFree(I->d_rowptr);
  hipFree(I->d_col);
  hipFree(I->d_val);
  hipFree(I->d_colptr);
  hipFree(I->d_crow);
  hipFree(I->d_cval);
  delete I;
  return SPG_OK;
}

static int witness_new(spg_ctx* ctx, const spg_witness_sec* secs, size_t nws, size_t p0, size_t p1,
                       spg_r1cs_witness** out) {
  if (!ctx || !secs || !out || nws == 0) return SPG_E_ARG;
  if (nws > 8) return set_err(ctx, SPG_E_ARG, "at most 8 witness sections (prefix_list)");
  spg_r1cs_witness* W = new spg_r1cs_witness();
  W->nws = nws;
  W->num_proofs.resize(nws);
  W->num_inputs.resize(nws);
  W->off.resize(nws);
  size_t total = 0;
  for (size_t w = 0; w < nws; w++) {
    const spg_witness_sec& s = secs[w];
    if (!s.num_instances || !s.num_proofs || !s.num_inputs || !s.w) {
      delete W;
      return SPG_E_ARG;
    }
    for (size_t p = 0; p < s.num_instances; p++) {
      if (!is_pow2(s.num_proofs[p]) || !is_pow2(s.num_inputs[p])) {
        delete W;
        return set_err(ctx, SPG_E_ARG, "witness section sizes must be powers of two");
      }
      W->num_proofs[w].push_back(s.num_proofs[p]);
      W->num_inputs[w].push_back(s.num_inputs[p]);
      bool here = s.num_instances == 1 || (p >= p0 && p < p1);
      if (here && !s.w[p]) {
        delete W;
        return set_err(ctx, SPG_E_ARG, "missing witness data for a resident instance");
      }
      W->off[w].push_back(here ? total : kNotResident);
      if (here) total += s.num_proofs[p] * s.num_inputs[p];
    }
  }
  W->total = total;
  if (!(W->d_w = (Fq*)dev_cache_get(ctx, total * sizeof(Fq) + 64))) {
    delete W;
    return set_err(ctx, SPG_E_NOMEM, "witness upload");
  }
  W->ptr.resize(nws);
  for (size_t w = 0; w < nws; w++)
    for (uint64_t o : W->off[w]) W->ptr[w].push_back(o == kNotResident ? nullptr : W->d_w + o);
  for (size_t w = 0; w < nws; w++)
    for (size_t p = 0; p < secs[w].num_instances; p++) {
      if (W->off[w][p] == kNotResident) continue;
      size_t n = W->num_proofs[w][p] * W->num_inputs[w][p];
      // Scalar([u64; 4]) and Fq(u32[8]) share the little-endian byte image. Streamed through the page-locked ring
      // (h2d_stream: host pool copies, DMA on the upload stream): the call returns once the caller's buffers are read,
      // with the last chunks' DMAs in flight and the context stream ordered after them (round 6; a pageable
      // hipMemcpyAsync ran at ~26 GB/s and was synchronised here)
      if (int rc = h2d_stream(ctx, W->d_w + W->off[w][p], secs[w].w[p], n * sizeof(Fq))) {
        spg_r1cs_witness_free(ctx, W);
        return rc;
      }
    }
  *out = W;
  return SPG_OK;
}
namespace spg {
// witness sections assembled from host or device parts (SNARK::prove's ProverWitnessSecInfo lists); an
// existing *inout whose total size matches is refilled in place
int witness_from_parts(spg_ctx* ctx, const std::vector<WPart>& secs, spg_r1cs_witness** inout) {
  if (secs.empty() || secs.size() > 8) return set_err(ctx, SPG_E_ARG, "1..8 witness sections");
  size_t total = 0;
  for (auto& w : secs) {
    if (w.num_proofs.empty() || w.num_proofs.size() != w.num_inputs.size() || w.src.size() != w.num_proofs.size())
      return set_err(ctx, SPG_E_ARG, "witness part shape");
    for (size_t p = 0; p < w.num_proofs.size(); p++) {
      if (!is_pow2(w.num_proofs[p]) || !is_pow2(w.num_inputs[p]))
        return set_err(ctx, SPG_E_ARG, "witness section sizes must be powers of two");
      total += w.num_proofs[p] * w.num_inputs[p];
    }
  }
  // parts already resident on this device (SNARK::prove's block_vars and exec buffers, alive and unchanged for
  // the whole prove) are read in place; only host parts are copied into d_w
  // (a buffer on another GPU is copied like a host part: k_spmv / k_z_fill would otherwise read it across devices)
  auto on_device = [ctx](const void* q) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, q) != hipSuccess) {
      (void)hipGetLastError();  // an unregistered host pointer: not an error of the prove
      return false;
    }
    return a.type == hipMemoryTypeDevice && a.device == ctx->device;
  };
  static const bool in_place = !getenv("SPG_WIT_IN_PLACE") || atoi(getenv("SPG_WIT_IN_PLACE")) != 0;
  std::vector<std::vector<char>> dev(secs.size());
  size_t host_total = 0;
  for (size_t w = 0; w < secs.size(); w++)
    for (size_t p = 0; p < secs[w].num_proofs.size(); p++) {
      const bool d = in_place && on_device(secs[w].src[p]);
      dev[w].push_back(d);
      if (!d) host_total += secs[w].num_proofs[p] * secs[w].num_inputs[p];
    }
  (void)total;
  spg_r1cs_witness* W = *inout;
  if (W && W->total < host_total) {
    spg_r1cs_witness_free(ctx, W);
    W = nullptr;
  }
  if (!W) {
    W = new spg_r1cs_witness();
    if (hipMalloc(&W->d_w, host_total * sizeof(Fq) + 64) != hipSuccess) {
      delete W;
      *inout = nullptr;
      return set_err(ctx, SPG_E_NOMEM, "witness");
    }
    W->total = host_total;
  }
  *inout = W;
  W->nws = secs.size();
  W->num_proofs.assign(secs.size(), {});
  W->num_inputs.assign(secs.size(), {});
  W->off.assign(secs.size(), {});
  W->ptr.assign(secs.size(), {});
  size_t o = 0;
  for (size_t w = 0; w < secs.size(); w++)
    for (size_t p = 0; p < secs[w].num_proofs.size(); p++) {
      size_t n = secs[w].num_proofs[p] * secs[w].num_inputs[p];
      W->num_proofs[w].push_back(secs[w].num_proofs[p]);
      W->num_inputs[w].push_back(secs[w].num_inputs[p]);
      if (dev[w][p]) {
        W->off[w].push_back(0);
        W->ptr[w].push_back(secs[w].src[p]);
        continue;
      }
      W->off[w].push_back(o);
      W->ptr[w].push_back(W->d_w + o);
      SPG_HIP(ctx, hipMemcpyAsync(W->d_w + o, secs[w].src[p], n * sizeof(Fq), hipMemcpyDefault, ctx->stream));
      o += n;
    }
  return 0;
}
}  // namespace spg

extern "C" int spg_r1cs_witness_new(spg_ctx* ctx, const spg_witness_sec* secs, size_t nws, spg_r1cs_witness** out) {
  return witness_new(ctx, secs, nws, 0, ~(size_t)0, out);
}
extern "C" int spg_r1cs_witness_new_shard(spg_ctx* ctx, const spg_witness_sec* secs, size_t nws, size_t p0,
                                          size_t p1, spg_r1cs_witness** out) {
  return witness_new(ctx, secs, nws, p0, p1, out);
}
extern "C" int spg_r1cs_witness_free(spg_ctx* ctx, spg_r1cs_witness* W) {
  if (!W) return SPG_OK;
  if (ctx) {
    h2d_sync(ctx);  // a streamed upload into it may still be in flight
    dev_cache_put(ctx, W->d_w, W->total * sizeof(Fq) + 64);  // kept for the next witness of this size
  } else {
    hipFree(W->d_w);
  }
  delete W;
  return SPG_OK;
}

// argument check of spg_r1cs_prove; also derives this rank's instance shard [p0, p1)
static int check_prove_args(spg_ctx* ctx, const spg_r1cs_inst* inst, size_t num_instances, size_t max_num_proofs,
                            const size_t* num_proofs, size_t max_num_inputs, const size_t* num_inputs,
                            const spg_r1cs_witness* wit, size_t rank, size_t nranks, size_t* p0, size_t* p1) {
  if (!num_instances || !is_pow2(max_num_proofs) || !is_pow2(max_num_inputs))
    return set_err(ctx, SPG_E_ARG, "bad sizes");
  if (inst->num_instances != 1 && inst->num_instances != num_instances)
    return set_err(ctx, SPG_E_ARG, "instance count mismatch");
  if (wit->nws * max_num_inputs > inst->num_vars) return set_err(ctx, SPG_E_ARG, "witness wider than num_vars");
  for (size_t p = 0; p < num_instances; p++) {
    if (!is_pow2(num_proofs[p]) || num_proofs[p] > max_num_proofs || !is_pow2(num_inputs[p]) ||
        num_inputs[p] > max_num_inputs)
      return set_err(ctx, SPG_E_ARG, "num_proofs / num_inputs must be powers of two within the maxima");
  }
  for (size_t w = 0; w < wit->nws; w++) {
    if (wit->num_proofs[w].size() != 1 && wit->num_proofs[w].size() != num_instances)
      return set_err(ctx, SPG_E_ARG, "witness section instance count mismatch");
    for (size_t p = 0; p < num_instances; p++) {
      size_t pw = wit->num_proofs[w].size() == 1 ? 0 : p;
      if (wit->num_proofs[w][pw] != 1 && wit->num_proofs[w][pw] < num_proofs[p])
        return set_err(ctx, SPG_E_ARG, "witness section has fewer rows than num_proofs");
      if (wit->num_proofs[w][pw] > max_num_proofs) return set_err(ctx, SPG_E_ARG, "witness section too tall");
    }
  }
  if (nranks > num_instances) return set_err(ctx, SPG_E_ARG, "more ranks than instances");
  *p0 = Prover::shard_begin(num_instances, nranks, rank);
  *p1 = Prover::shard_begin(num_instances, nranks, rank + 1);
  for (size_t w = 0; w < wit->nws; w++) {
    if (wit->num_proofs[w].size() == 1) continue;
    for (size_t p = *p0; p < *p1; p++)
      if (wit->off[w][p] == kNotResident) return set_err(ctx, SPG_E_ARG, "witness shard does not hold instance");
  }
  return SPG_OK;
}

static int r1cs_prove_impl(spg_ctx* ctx, const spg_r1cs_gens* gens, const spg_r1cs_inst* inst,
                           size_t num_instances, size_t max_num_proofs, const size_t* num_proofs,
                           size_t max_num_inputs, const size_t* num_inputs, const spg_r1cs_witness* wit,
                           spg_transcript* transcript, spg_random_tape* tape, uint8_t* proof, size_t proof_cap,
                           size_t* proof_len, uint64_t* challenges_out, size_t* ch_lens) {
  Prover pr(ctx, const_cast<spg_r1cs_gens*>(gens)->g, *inst, *wit, transcript->t, tape->t);
  pr.rank = (size_t)ctx->rank;
  pr.nranks = (size_t)ctx->nranks;
  int rc_args = check_prove_args(ctx, inst, num_instances, max_num_proofs, num_proofs, max_num_inputs, num_inputs,
                                 wit, pr.rank, pr.nranks, &pr.p0, &pr.p1);
  if (pr.nranks > 1) {
    // a sharded prove starts with every rank agreeing on the argument check, so a rank-local failure
    // (e.g. a witness shard that does not hold this rank's instances) fails every rank alike instead of
    // leaving the others blocked in the first round's allgather
    int32_t mine = rc_args;
    std::vector<uint8_t> all;
    int rc = comm_allgather(ctx, Shard{(int)pr.rank, (int)pr.nranks}, 0, &mine, sizeof(mine), all);
    if (rc) return rc;
    for (size_t q = 0; q < pr.nranks && !rc_args; q++)
      if (((const int32_t*)all.data())[q]) rc_args = set_err(ctx, SPG_E_ARG, "a peer rank rejected its arguments");
  }
  if (rc_args) return rc_args;
  pr.P = num_instances;
  pr.max_np = max_num_proofs;
  pr.Y = max_num_inputs;
  pr.nws = wit->nws;
  pr.num_proofs.assign(num_proofs, num_proofs + num_instances);
  pr.num_inputs.assign(num_inputs, num_inputs + num_instances);
  timer_start(ctx);
  int rc = pr.run();
  timer_stop(ctx);
  if (rc) return rc;
  Writer wr;
  pr.pf.ser(wr);
  *proof_len = wr.out.size();
  if (challenges_out && ch_lens) {
    size_t k = 0;
    for (int i = 0; i < 4; i++) {
      ch_lens[i] = pr.challenges[i].size();
      for (auto& c : pr.challenges[i]) st_fq(challenges_out + 4 * k++, c);
    }
  }
  if (!proof || wr.out.size() > proof_cap) return set_err(ctx, SPG_E_ARG, "proof buffer too small");
  memcpy(proof, wr.out.data(), wr.out.size());
  return SPG_OK;
}

extern "C" int spg_r1cs_prove(spg_ctx* ctx, const spg_r1cs_gens* gens, const spg_r1cs_inst* inst,
                              size_t num_instances, size_t max_num_proofs, const size_t* num_proofs,
                              size_t max_num_inputs, const size_t* num_inputs, const spg_r1cs_witness* wit,
                              spg_transcript* transcript, spg_random_tape* tape, uint8_t* proof, size_t proof_cap,
                              size_t* proof_len, uint64_t* challenges_out, size_t* ch_lens) {
  if (!ctx || !gens || !inst || !num_proofs || !num_inputs || !wit || !transcript || !tape || !proof_len)
    return SPG_E_ARG;
  HostPin pin;
  TrFailScope tfs(ctx, transcript->t);
  return tr_status(ctx, transcript->t,
                   r1cs_prove_impl(ctx, gens, inst, num_instances, max_num_proofs, num_proofs, max_num_inputs, num_inputs,
                                   wit, transcript, tape, proof, proof_cap, proof_len, challenges_out, ch_lens));
}

// R1CSInstance::multi_evaluate (src/r1csinstance.rs:583-596) / evaluate (:632-641):
// out[3p + m] = M_p(rx, ry) for M in (A, B, C), p < num_instances of the uploaded instance
extern "C" int spg_r1cs_multi_evaluate(spg_ctx* ctx, const spg_r1cs_inst* inst, const uint64_t* rx, size_t rx_len,
                                       const uint64_t* ry, size_t ry_len, uint64_t* out) {
  if (!ctx || !inst || !out || (!rx && rx_len) || (!ry && ry_len)) return SPG_E_ARG;
  if (rx_len > 32 || ry_len > 32 || ((size_t)1 << rx_len) < inst->max_num_cons ||
      ((size_t)1 << ry_len) < inst->num_vars)
    return set_err(ctx, SPG_E_ARG, "multi_evaluate: rx / ry shorter than the matrix dimensions");
  hipStream_t s = ctx->stream;
  const size_t Pm = inst->num_instances;
  // sharded over the ranks of spg_set_comm: every matrix's rows split (balanced), the 3 Pm partial sums added
  const Shard sh = ctx_shard(ctx);
  FqV vx(rx_len), vy(ry_len);
  for (size_t i = 0; i < rx_len; i++) vx[i] = ld_fq(rx + 4 * i);
  for (size_t i = 0; i < ry_len; i++) vy[i] = ld_fq(ry + 4 * i);
  Fq* erx = (Fq*)ws_get(ctx, WS_EV_RX, (sizeof(Fq) << rx_len) + 64);
  Fq* ery = (Fq*)ws_get(ctx, WS_EV_RY, (sizeof(Fq) << ry_len) + 64);
  std::vector<MatDesc> md(Pm);
  std::vector<uint32_t> rr(2 * Pm);
  size_t maxrows = 1;
  double visits = 0, rows = 0;
  for (size_t p = 0; p < Pm; p++) {
    for (int m = 0; m < 3; m++) md[p].rp[m] = inst->rp_off[3 * p + m];
    md[p].cp = inst->cp_off[p];
    rr[2 * p] = (uint32_t)shard_begin(inst->num_cons[p], sh.n, sh.rank);
    rr[2 * p + 1] = (uint32_t)shard_begin(inst->num_cons[p], sh.n, sh.rank + 1);
    maxrows = std::max<size_t>(maxrows, rr[2 * p + 1] - rr[2 * p]);
    const double frac = (double)(rr[2 * p + 1] - rr[2 * p]) / (double)std::max<size_t>(1, inst->num_cons[p]);
    visits += frac * (inst->nnz[3 * p] + inst->nnz[3 * p + 1] + inst->nnz[3 * p + 2]);
    rows += 3.0 * (rr[2 * p + 1] - rr[2 * p]);
  }
  const unsigned nblk = blocks_for(maxrows);
  Fq* part = (Fq*)ws_get(ctx, WS_EV_PART, 3 * Pm * nblk * sizeof(Fq) + 64);
  Fq* dout = (Fq*)ws_get(ctx, WS_EV_OUT, 3 * Pm * sizeof(Fq) + 64);
  uint8_t* ddesc = (uint8_t*)ws_get(ctx, WS_EV_DESC, Pm * (sizeof(MatDesc) + 8) + 64);
  if (!erx || !ery || !part || !dout || !ddesc) {
    int rc = set_err(ctx, SPG_E_NOMEM, "multi_evaluate");
    FqV none(3 * Pm);
    return comm_sum_fq(ctx, sh, rc, none.data(), 3 * Pm);
  }
  MatDesc* dmd = (MatDesc*)ddesc;
  uint32_t* drr = (uint32_t*)(ddesc + Pm * sizeof(MatDesc));
  {  // matrix descriptors and row ranges in one copy
    std::vector<uint8_t> h(Pm * sizeof(MatDesc) + 2 * Pm * 4);
    memcpy(h.data(), md.data(), Pm * sizeof(MatDesc));
    memcpy(h.data() + Pm * sizeof(MatDesc), rr.data(), 2 * Pm * 4);
    SPG_HIP(ctx, hipMemcpyAsync(dmd, h.data(), h.size(), hipMemcpyHostToDevice, s));
  }
  timer_start(ctx);
  int rc = eq_tables(ctx, {{vx, erx}, {vy, ery}});
  if (rc) return rc;
  {
    KScope ks(ctx, "sparse_eval", 68.0 * visits + 40.0 * rows);
    hipLaunchKernelGGL(k_sparse_eval, dim3(nblk, (unsigned)(3 * Pm)), dim3(256), 0, s, dmd, drr, inst->d_rowptr,
                       inst->d_col, inst->d_val, erx, ery, part);
    hipLaunchKernelGGL(k_sum_segments, dim3((unsigned)(3 * Pm)), dim3(256), 0, s, part, (int)nblk, dout);
  }
  SPG_HIP(ctx, hipGetLastError());
  timer_stop(ctx);
  std::vector<Fq> h(3 * Pm);
  SPG_HIP(ctx, hipMemcpyAsync(h.data(), dout, 3 * Pm * sizeof(Fq), hipMemcpyDeviceToHost, s));
  SPG_HIP(ctx, hipStreamSynchronize(s));
  float ms = 0.f;
  hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  ctx->last_us = ms * 1000.0;
  rc = comm_sum_fq(ctx, sh, 0, h.data(), 3 * Pm);
  if (rc) return rc;
  for (size_t i = 0; i < 3 * Pm; i++) st_fq(out + 4 * i, h[i]);
  return SPG_OK;
}

// R1CSInstance::multiply_vec_block (src/r1csinstance.rs:363-436; per (p, q): multiply_vec_disjoint_rounds,
// src/sparse_mlpoly.rs:454-472) as a seam: z_mat (p, q, w, x) -- instance p's num_proofs[p] x num_witness_secs x
// num_inputs[p] scalars, instances one after another, column c of a matrix reading z[p][q][c / max_num_inputs]
// [c % max_num_inputs] (zero past num_inputs[p]) -- into Az, Bz, Cz as new spg_pqx tables in
// DensePolynomialPqx::new_rev order (p, q_rev, x_rev: num_proofs, max_num_proofs, num_cons, max_num_cons; one w
// section). The prover's own k_spmv does the work, over section descriptors pointing into one upload of z.
extern "C" int spg_r1cs_multiply_vec_block(spg_ctx* ctx, const spg_r1cs_inst* inst, size_t num_instances,
                                           const size_t* num_proofs, size_t max_num_proofs, const size_t* num_inputs,
                                           size_t max_num_inputs, size_t num_witness_secs, const uint64_t* z_mont,
                                           spg_pqx** Az, spg_pqx** Bz, spg_pqx** Cz) {
  if (!ctx || !inst || !num_proofs || !num_inputs || !z_mont || !Az || !Bz || !Cz || num_instances == 0)
    return SPG_E_ARG;
  auto pow2 = [](size_t v) { return v && !(v & (v - 1)); };
  // r1csinstance.rs:375-376: one matrix for every instance, or one per instance
  if (!(inst->num_instances == 1 || inst->num_instances == num_instances))
    return set_err(ctx, SPG_E_ARG, "multiply_vec_block: the instance holds 1 or num_instances matrices");
  if (num_witness_secs == 0 || num_witness_secs > 8)  // (k_spmv keeps one block's section descriptors in LDS)
    return set_err(ctx, SPG_E_ARG, "multiply_vec_block: 1..8 witness sections");
  if (!pow2(max_num_proofs) || max_num_inputs == 0 || max_num_inputs > 0xffffffffu)
    return set_err(ctx, SPG_E_ARG, "multiply_vec_block: max_num_proofs a power of two, max_num_inputs > 0");
  const size_t P = num_instances;
  std::vector<size_t> ncons(P);
  size_t zt = 0, total = 0;
  for (size_t p = 0; p < P; p++) {
    const size_t pi = inst->num_instances == 1 ? 0 : p;
    ncons[p] = inst->num_cons[pi];
    if (!pow2(num_proofs[p]) || num_proofs[p] > max_num_proofs || num_inputs[p] > max_num_inputs || !pow2(ncons[p]))
      return set_err(ctx, SPG_E_ARG, "multiply_vec_block: num_proofs[p] (<= max) and num_cons powers of two, "
                                     "num_inputs[p] <= max_num_inputs");
    zt += num_proofs[p] * num_witness_secs * num_inputs[p];
    total += num_proofs[p] * ncons[p];
  }
  if (total >= ((size_t)1 << 31)) return set_err(ctx, SPG_E_ARG, "multiply_vec_block: at most 2^31 outputs");
  // z section-major on the device: section w of instance p as its own (q, x) matrix, as a witness section lies
  std::vector<Fq> zs(zt);
  std::vector<SecDesc> sd(num_witness_secs * P);
  std::vector<size_t> soff(num_witness_secs * P);
  {
    size_t o = 0;
    for (size_t w = 0; w < num_witness_secs; w++)
      for (size_t p = 0; p < P; p++) {
        soff[w * P + p] = o;
        o += num_proofs[p] * num_inputs[p];
      }
    const uint64_t* src = z_mont;
    for (size_t p = 0; p < P; p++)
      for (size_t q = 0; q < num_proofs[p]; q++)
        for (size_t w = 0; w < num_witness_secs; w++)
          for (size_t x = 0; x < num_inputs[p]; x++, src += 4)
            zs[soff[w * P + p] + q * num_inputs[p] + x] = ld_fq(src);
  }
  Fq* d_z = nullptr;
  void* d_desc = nullptr;
  std::vector<SpDesc> spd(P);
  std::vector<MatDesc> md(inst->num_instances);
  for (size_t p = 0; p < inst->num_instances; p++) {
    for (int m = 0; m < 3; m++) md[p].rp[m] = inst->rp_off[3 * p + m];
    md[p].cp = inst->cp_off[p];
  }
  size_t off = 0;
  for (size_t p = 0; p < P; p++) {
    spd[p].dom_off = spd[p].out_off = off;
    spd[p].pi = (uint32_t)(inst->num_instances == 1 ? 0 : p);
    spd[p].lg_q = (uint32_t)lg2(num_proofs[p]);
    spd[p].nrows = (uint32_t)ncons[p];
    spd[p].lg_rows = (uint32_t)lg2(ncons[p]);
    spd[p].ni = (uint32_t)num_inputs[p];
    spd[p].lg_ni = 0;
    off += num_proofs[p] * ncons[p];
  }
  const size_t b_sec = sd.size() * sizeof(SecDesc), b_sp = spd.size() * sizeof(SpDesc),
               b_md = md.size() * sizeof(MatDesc);
  spg_pqx* outs[3] = {new spg_pqx(), new spg_pqx(), new spg_pqx()};
  int rc = 0;
  auto fail = [&](int code, const char* msg) {
    rc = set_err(ctx, code, msg);
  };
  if (hipMalloc(&d_z, zt * sizeof(Fq) + 64) != hipSuccess || hipMalloc(&d_desc, b_sec + b_sp + b_md + 64) != hipSuccess)
    fail(SPG_E_NOMEM, "multiply_vec_block");
  for (int k = 0; k < 3 && !rc; k++) {
    PqxDev& T = outs[k]->T;
    T.zlen = P;
    size_t o = 0;
    for (size_t p = 0; p < P; p++) {
      T.off.push_back(o);
      T.anp.push_back(num_proofs[p]);
      T.anw.push_back(1);
      T.ani.push_back(ncons[p]);
      o += num_proofs[p] * ncons[p];
    }
    T.total = total;
    T.num_instances = 1;
    while (T.num_instances < P) T.num_instances *= 2;
    T.max_num_proofs = max_num_proofs;
    T.num_witness_secs = 1;
    T.max_num_inputs = inst->max_num_cons;
    T.num_proofs.assign(num_proofs, num_proofs + P);
    T.num_inputs = ncons;
    if (hipMalloc(&T.d, total * sizeof(Fq) + 64) != hipSuccess) fail(SPG_E_NOMEM, "multiply_vec_block outputs");
  }
  if (!rc) {
    for (size_t w = 0; w < num_witness_secs; w++)
      for (size_t p = 0; p < P; p++) {
        SecDesc& s = sd[w * P + p];
        s.w = d_z + soff[w * P + p];
        s.np = (uint32_t)num_proofs[p];
        s.ni = (uint32_t)num_inputs[p];
      }
    std::vector<uint8_t> blob(b_sec + b_sp + b_md);
    memcpy(blob.data(), sd.data(), b_sec);
    memcpy(blob.data() + b_sec, spd.data(), b_sp);
    memcpy(blob.data() + b_sec + b_sp, md.data(), b_md);
    uint8_t* dd = (uint8_t*)d_desc;
    if (hipMemcpy(d_z, zs.data(), zt * sizeof(Fq), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dd, blob.data(), blob.size(), hipMemcpyHostToDevice) != hipSuccess)
      fail(SPG_E_HIP, "multiply_vec_block upload");
    if (!rc && total) {
      hipLaunchKernelGGL(k_spmv<false>, dim3(blocks_for(total)), dim3(256), 0, ctx->stream, (const SpDesc*)(dd + b_sec),
                         (int)P, (const MatDesc*)(dd + b_sec + b_sp), inst->d_rowptr, inst->d_col, inst->d_val,
                         (const SecDesc*)dd, (int)num_witness_secs, (uint32_t)max_num_inputs, outs[0]->T.d,
                         outs[1]->T.d, outs[2]->T.d, (uint64_t)total);
      if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess)
        fail(SPG_E_HIP, "multiply_vec_block launch");
    }
  }
  hipFree(d_z);
  hipFree(d_desc);
  if (rc) {
    for (spg_pqx* h : outs) {
      hipFree(h->T.d);
      delete h;
    }
    return rc;
  }
  *Az = outs[0];
  *Bz = outs[1];
  *Cz = outs[2];
  return SPG_OK;
}
