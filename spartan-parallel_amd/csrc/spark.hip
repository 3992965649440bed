// spg — SPARK: commitments to and evaluation proofs of batched sparse matrix polynomials on MI355X.
//
//   SparseMatPolynomial::multi_commit            src/sparse_mlpoly.rs:368-425, 566-587  spg_spark_commit
//   SparseMatPolyEvalProof::prove                src/sparse_mlpoly.rs:1497-1564         spg_spark_prove
//     AddrTimestamps::deref, Derefs::commit      :255-270, :51-67                        k_gather, Hyrax rows
//     Layers::build_hash_layer, ProductCircuit   :612-736, src/product_tree.rs:36-58    k_hash_*, k_tree_level
//     ProductLayerProof::prove                   :1118-1263                              batched_prove
//     ProductCircuitEvalProofBatched::prove      src/product_tree.rs:271-396             k_layer_eval, k_fold_many
//     SumcheckInstanceProof::prove_cubic_batched src/sumcheck.rs:264-434
//     HashLayerProof::prove                      :805-918                                k_seg_dot, PolyEvalProofs
//
// HBM layout (B = 3 x instances matrices, N = next_pow2(max nnz), cells = 2^max(nvx, nvy)):
//   addr / read_ts : u32 [2][B][N] (rows, then cols)    audit : u32 [2][cells]
//   val            : Fq [B][N]
//   comb_ops (Fq)  : [row addr | row read_ts | col addr | col read_ts | val] (each B x N), zero-padded to 2^k
//   comb_mem (Fq)  : [row audit | col audit]
//   product trees  : circuit c at c * 2M; its levels v_0 (the M hashed leaves), v_1, .. v_{L-1} (2 entries)
//                    back to back at offset 2M - 2(M >> k). Layer k of the circuit is (left, right) = the
//                    two halves of v_k, and v_{k+1}[i] = v_k[i] * v_k[i + |v_k|/2].
// All O(N) work stays in HBM; the host runs the transcript and one UniPoly per sumcheck round.
#include <algorithm>
#include <array>

#include <hipcub/hipcub.hpp>

#include "hostpoly.hpp"
#include "proto.hpp"
#include "layer.hpp"
#include "lds.hpp"
#include "sumcheck.hpp"

namespace spg {

// ------------------------------------------------------------------------------------ kernels
__global__ void k_u32_to_fq(const uint32_t* __restrict__ in, Fq* __restrict__ out, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = fq_from_u64(in[i]);
}

// derefs[s][b][i] = mem_s[addr[s][b][i]]  (s = 0: rows with eq(rx), s = 1: cols with eq(ry))
__global__ void k_gather(const uint32_t* __restrict__ addr, const Fq* __restrict__ mem_rx, const Fq* __restrict__ mem_ry,
                         size_t BN, Fq* __restrict__ out) {
  size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= 2 * BN) return;
  out[t] = (t < BN ? mem_rx : mem_ry)[addr[t]];
}

// hash(addr, val, ts) = ts * r_hash^2 + val * r_hash + addr - r_multiset  (sparse_mlpoly.rs:621-626)
__device__ __forceinline__ Fq hash3(const Fq& a, const Fq& v, const Fq& ts, const Fq& rh, const Fq& rh2, const Fq& rms) {
  return fq_sub(fq_add(fq_add(fq_mul(ts, rh2), fq_mul(v, rh)), a), rms);
}
// leaves of the 4B ops circuits (row read b, row write b, col read b, col write b), written into the trees.
// Sharded proofs (W ranks) keep the leaves i = W i' + r of rank r: local leaf i' of m = N / W (W = 1: all)
__global__ void k_hash_ops(const uint32_t* __restrict__ addr, const uint32_t* __restrict__ rts,
                           const Fq* __restrict__ derefs, size_t B, int logN, int logm, uint32_t W, uint32_t r, Fq rh,
                           Fq rh2, Fq rms, Fq* __restrict__ tree) {
  const size_t N = (size_t)1 << logN, m = (size_t)1 << logm;
  size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= 2 * B * m) return;
  size_t sb = t >> logm, il = t & (m - 1);  // sb = side * B + b
  size_t s = sb >= B, b = sb - s * B, g = sb * N + il * W + r;
  Fq a = fq_from_u64(addr[g]), ts = fq_from_u64(rts[g]), v = derefs[g];
  tree[((2 * s) * B + b) * 2 * m + il] = hash3(a, v, ts, rh, rh2, rms);
  tree[((2 * s + 1) * B + b) * 2 * m + il] = hash3(a, v, fq_add(ts, fq_one()), rh, rh2, rms);
}
// leaves of the 4 memory circuits (row init, row audit, col init, col audit); cell i = W i' + r as above
__global__ void k_hash_mem(const uint32_t* __restrict__ audit, const Fq* __restrict__ mem_rx,
                           const Fq* __restrict__ mem_ry, int logC, int logm, uint32_t W, uint32_t r, Fq rh, Fq rh2,
                           Fq rms, Fq* __restrict__ tree) {
  const size_t cells = (size_t)1 << logC, m = (size_t)1 << logm;
  size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= 2 * m) return;
  size_t s = t >> logm, il = t & (m - 1), i = il * W + r;
  Fq a = fq_from_u64(i), v = (s ? mem_ry : mem_rx)[i];
  tree[(2 * s) * 2 * m + il] = hash3(a, v, fq_zero(), rh, rh2, rms);
  tree[(2 * s + 1) * 2 * m + il] = hash3(a, v, fq_from_u64(audit[s * cells + i]), rh, rh2, rms);
}
// AddrTimestamps::new (sparse_mlpoly.rs:219-253) on the device: read_ts[t] = #{t' < t : addr[t'] = addr[t]} and
// audit[a] = #{t : addr[t] = a} over the ops in batch order. counts -> exclusive scan = each address's first
// rank; a stable radix sort of (addr, t) lists every address's ops in order, so sorted position j holds op t with
// read_ts = j - start[addr].
__global__ void k_ts_count(const uint32_t* __restrict__ addr, size_t n, uint32_t* __restrict__ cnt) {
  size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n) atomicAdd(&cnt[addr[t]], 1u);
}
__global__ void k_iota(uint32_t* __restrict__ v, size_t n) {
  size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n) v[t] = (uint32_t)t;
}
__global__ void k_ts_rank(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ ops,
                          const uint32_t* __restrict__ start, size_t n, uint32_t* __restrict__ rts) {
  size_t j = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (j < n) rts[ops[j]] = (uint32_t)j - start[keys[j]];
}

// dst[i] = src[i W + r], i < n (a rank's interleaved share of a vector)
__global__ void k_strided(Fq* __restrict__ dst, const Fq* __restrict__ src, size_t n, uint32_t W, uint32_t r) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[i * W + r];
}
// the dot-product circuits' inputs in one launch: circuit piece j = (2b + h) * 3 + k of length nl is this rank's
// interleaved share (i * W + r) of half h of instance b's row derefs (k = 0), col derefs (k = 1) or values (k = 2)
__global__ void k_dotp_gather(Fq* __restrict__ dst, const Fq* __restrict__ derefs, const Fq* __restrict__ val,
                              size_t BN, size_t N, size_t hN, size_t nl, uint32_t W, uint32_t r) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nl) return;
  const uint32_t j = blockIdx.y, k = j % 3, h = (j / 3) & 1, b = j / 6;
  const Fq* src = (k < 2 ? derefs + k * BN : val) + b * N + h * hN;
  dst[(size_t)j * nl + i] = src[i * W + r];
}
__global__ void k_scale(Fq* __restrict__ v, size_t n, Fq s) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = fq_mul(v[i], s);
}
// v_{k+1}[i] = v_k[i] * v_k[i + half] for every circuit (circuit stride 2M)
__global__ void k_tree_level(Fq* __restrict__ tree, size_t nc, size_t stride, size_t off_k, size_t off_k1, int log_half) {
  const size_t half = (size_t)1 << log_half;
  size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= nc * half) return;
  size_t c = t >> log_half, i = t & (half - 1);
  Fq* v = tree + c * stride;
  v[off_k1 + i] = fq_mul(v[off_k + i], v[off_k + i + half]);
}
// The levels of every circuit's tree from level k0 up, and its top product, in one launch: workgroup c builds circuit c's
// levels (each level's products read the level below, which this workgroup wrote: a barrier between levels) -- the
// small top levels would otherwise be one launch each, ~3 us of work behind a ~4 us launch
__global__ void __launch_bounds__(256) k_tree_top(Fq* __restrict__ tree, size_t stride, int log_m, int k0,
                                                  Fq* __restrict__ tops) {
  Fq* v = tree + blockIdx.x * stride;
  const size_t M = (size_t)1 << log_m;
  for (int k = k0; k + 1 < log_m; k++) {
    const size_t ok = 2 * M - 2 * (M >> k), ok1 = 2 * M - 2 * (M >> (k + 1)), half = M >> (k + 1);
    for (size_t i = threadIdx.x; i < half; i += 256) v[ok1 + i] = fq_mul(v[ok + i], v[ok + i + half]);
    __syncthreads();
  }
  if (threadIdx.x == 0) tops[blockIdx.x] = fq_mul(v[2 * M - 4], v[2 * M - 3]);
}
// ProductCircuit::evaluate of every circuit: product of the top level's two entries
__global__ void k_tops(const Fq* __restrict__ tree, size_t nc, size_t stride, size_t off, Fq* __restrict__ out) {
  size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (c < nc) out[c] = fq_mul(tree[c * stride + off], tree[c * stride + off + 1]);
}

// A whole round of a small layer in one workgroup of 1024 threads (nt * len up to a few thousand): first the previous
// round's bound_poly_var_top of every layer vector (when do_fold; vectors of 2 flen -> flen, one pass,
// __syncthreads), then the round's (e0, e2, e3) with each triple's coefficient applied per element, a block
// reduction and the mailbox post. No grid-wide ticket and one launch instead of fold + eval.
__global__ void __launch_bounds__(1024) k_layer_tiny(const Triple* __restrict__ tr, const Fq* __restrict__ coeff,
                                                     int nt, int log_len, Fq* const* __restrict__ fv, int nv,
                                                     int do_fold, Fq r, uint32_t* __restrict__ mb, uint32_t seq) {
  const int t = threadIdx.x;
  const int len = 1 << log_len;
  if (do_fold) {
    const int flen = 2 * len;  // folded length
    for (int k = t; k < nv * flen; k += 1024) {
      Fq* p = fv[k / flen];
      const int i = k % flen;
      const Fq lo = p[i];
      p[i] = fq_add(lo, fq_mul(r, fq_sub(p[i + flen], lo)));
    }
    __syncthreads();
  }
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (int u = t; u < nt * len; u += 1024) {
    const Triple x = tr[u >> log_len];
    const Fq k = coeff[u >> log_len];
    const int i = u & (len - 1);
    // the coefficient scales the A factor (k A is linear in X), 8 multiplications per element instead of 9
    const Fq al = fq_mul(k, x.A[i]), ah = fq_mul(k, x.A[i + len]);
    const Fq bl = x.B[i], bh = x.B[i + len], cl = x.C[i], ch = x.C[i + len];
    Fq da = fq_sub(ah, al), db = fq_sub(bh, bl), dc = fq_sub(ch, cl);
    Fq a2 = fq_add(ah, da), b2 = fq_add(bh, db), c2 = fq_add(ch, dc);
    e0 = fq_add(e0, fq_mul(fq_mul(al, bl), cl));
    e2 = fq_add(e2, fq_mul(fq_mul(a2, b2), c2));
    e3 = fq_add(e3, fq_mul(fq_mul(fq_add(a2, da), fq_add(b2, db)), fq_add(c2, dc)));
  }
  block_sum3_t0<1024>(e0, e2, e3);
  if (t == 0) {
    mbox_post3(mb, seq, e0, e2, e3);
  }
}
// one batched cubic sumcheck round over nt triples (A_c, B_c, C_c) of length 2 * len:
// sum_c coeff_c * sum_i A*B*C at X = 0, 2, 3 (sumcheck.rs:300-367). blockIdx.y = triple, so the coefficient
// multiplies the block's sums once; the last block to finish (ticket on `counter`) adds every block's
// partials and posts the round's three scalars to the host mailbox (one launch per round).
__global__ void __launch_bounds__(256) k_layer_eval(const Triple* __restrict__ tr, const Fq* __restrict__ coeff,
                                                    size_t len, Fq* __restrict__ partials,
                                                    unsigned* __restrict__ counter, uint32_t* __restrict__ mb,
                                                    uint32_t seq) {
  const Triple x = tr[blockIdx.y];
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < len; i += (size_t)gridDim.x * 256) {
    Fq al = x.A[i], ah = x.A[i + len], bl = x.B[i], bh = x.B[i + len], cl = x.C[i], ch = x.C[i + len];
    Fq da = fq_sub(ah, al), db = fq_sub(bh, bl), dc = fq_sub(ch, cl);
    Fq a2 = fq_add(ah, da), b2 = fq_add(bh, db), c2 = fq_add(ch, dc);
    e0 = fq_add(e0, fq_mul(fq_mul(al, bl), cl));
    e2 = fq_add(e2, fq_mul(fq_mul(a2, b2), c2));
    e3 = fq_add(e3, fq_mul(fq_mul(fq_add(a2, da), fq_add(b2, db)), fq_add(c2, dc)));
  }
  block_sum3_sp(e0, e2, e3);
  __shared__ bool last;
  const unsigned nblocks = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
  if (threadIdx.x == 0) {
    const Fq k = coeff[blockIdx.y];
    partials[3 * bid] = fq_mul(k, e0);
    partials[3 * bid + 1] = fq_mul(k, e2);
    partials[3 * bid + 2] = fq_mul(k, e3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  Fq a = fq_zero(), b = fq_zero(), c = fq_zero();
  for (unsigned i = threadIdx.x; i < nblocks; i += 256) {
    a = fq_add(a, partials[3 * i]);
    b = fq_add(b, partials[3 * i + 1]);
    c = fq_add(c, partials[3 * i + 2]);
  }
  block_sum3_sp(a, b, c);
  if (threadIdx.x == 0) {
    mbox_post3(mb, seq, a, b, c);
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// DensePolynomial::bound_poly_var_top on nv distinct vectors of length 2 * len (in place)
__global__ void k_fold_many(Fq* const* __restrict__ v, size_t nv, int log_len, Fq r) {
  const size_t len = (size_t)1 << log_len;
  size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= nv * len) return;
  Fq* p = v[t >> log_len];
  size_t i = t & (len - 1);
  Fq lo = p[i];
  p[i] = fq_add(lo, fq_mul(r, fq_sub(p[i + len], lo)));
}
// A[0], B[0], C[0] of every triple (the final claims of a layer)
__global__ void k_finals(const Triple* __restrict__ tr, size_t nt, Fq* __restrict__ out) {
  size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= nt) return;
  out[3 * c] = tr[c].A[0];
  out[3 * c + 1] = tr[c].B[0];
  out[3 * c + 2] = tr[c].C[0];
}
// DotProductCircuit::evaluate per triple: sum_i A*B*C over n entries (blockIdx.y = triple)
__global__ void __launch_bounds__(256) k_dot3(const Triple* __restrict__ tr, size_t n, Fq* __restrict__ partials) {
  const Triple x = tr[blockIdx.y];
  Fq acc = fq_zero(), z = fq_zero(), z2 = fq_zero();
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    acc = fq_add(acc, fq_mul(fq_mul(x.A[i], x.B[i]), x.C[i]));
  block_sum3_sp(acc, z, z2);
  if (threadIdx.x == 0) partials[(size_t)blockIdx.y * gridDim.x + blockIdx.x] = acc;
}
// sum_i base[s * seglen + i] * eq[i] for segments s = blockIdx.y (DensePolynomial::evaluate on HBM)
__global__ void __launch_bounds__(256) k_seg_dot(const Fq* __restrict__ base, size_t seglen, const Fq* __restrict__ eq,
                                                 size_t n, Fq* __restrict__ partials) {
  const size_t s = blockIdx.y;
  Fq acc = fq_zero(), z = fq_zero(), z2 = fq_zero();
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    acc = fq_add(acc, fq_mul(base[s * seglen + i], eq[i]));
  block_sum3_sp(acc, z, z2);
  if (threadIdx.x == 0) partials[s * gridDim.x + blockIdx.x] = acc;
}
__global__ void __launch_bounds__(256) k_sum_seg(const Fq* __restrict__ partials, int nb, Fq* __restrict__ out) {
  Fq a = fq_zero(), z = fq_zero(), z2 = fq_zero();
  for (int i = threadIdx.x; i < nb; i += 256) a = fq_add(a, partials[(size_t)blockIdx.x * nb + i]);
  block_sum3_sp(a, z, z2);
  if (threadIdx.x == 0) out[blockIdx.x] = a;
}
// DensePolynomial::bound (dense_mlpoly.rs:258-265): out[i] = sum_j L[j] * Z[j * Rs + i], rows split over y
__global__ void __launch_bounds__(256) k_bound_rows(const Fq* __restrict__ Z, const Fq* __restrict__ L, size_t Ls,
                                                    size_t Rs, size_t chunk, Fq* __restrict__ part) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= Rs) return;
  size_t j0 = blockIdx.y * chunk, j1 = j0 + chunk < Ls ? j0 + chunk : Ls;
  Fq acc = fq_zero();
  for (size_t j = j0; j < j1; j++) acc = fq_add(acc, fq_mul(L[j], Z[j * Rs + i]));
  part[(size_t)blockIdx.y * Rs + i] = acc;
}
// out[i] = sum_y part[y][i]: a block owns 16 columns and 16 lanes per column split the S partials (S reaches
// thousands when Rs is small, and one lane per column made that a chain of S dependent additions), then an LDS tree
constexpr int kBoundSumCols = 16;
__global__ void __launch_bounds__(256) k_bound_sum(const Fq* __restrict__ part, size_t S, size_t Rs,
                                                   Fq* __restrict__ out) {
  __shared__ Fq sm[256];
  const int t = threadIdx.x, c = t % kBoundSumCols, y0 = t / kBoundSumCols;
  const size_t i = (size_t)blockIdx.x * kBoundSumCols + c;
  constexpr int YL = 256 / kBoundSumCols;
  Fq acc = fq_zero();
  if (i < Rs)
    for (size_t y = y0; y < S; y += YL) acc = fq_add(acc, part[y * Rs + i]);
  sm[t] = acc;
  __syncthreads();
#pragma unroll
  for (int h = YL / 2; h >= 1; h >>= 1) {
    if (y0 < h) sm[t] = fq_add(sm[t], sm[t + kBoundSumCols * h]);
    __syncthreads();
  }
  if (y0 == 0 && i < Rs) out[i] = sm[t];
}

}  // namespace spg

using namespace spg;

// ------------------------------------------------------------------------------------ handle

namespace spg {

static unsigned nblk(size_t n) { return (unsigned)((n + 255) / 256); }
// Hyrax rows up to this many scalars go through the latency MSM path (one block per bucket and row)
static const size_t kSmallRowMax = 256;
static const size_t kHostFinalRows = 64;  // latency-path commits of at most this many rows finish on the host
// workspace slots of this file
enum : size_t {
  kWsCommit = 60, kWsL, kWsBoundPart, kWsBound, kWsSegPart, kWsSeg, kWsC, kWsTriples, kWsCoeff, kWsFoldPtr,
  kWsPart, kWs3, kWsMemRx, kWsMemRy, kWsDerefs, kWsTreeOps, kWsTreeMem, kWsDotp, kWsFinals, kWsEqOps, kWsEqMem,
  kWsTops, kWsCommitBk, kWsC2, kWsGather, kWsTopOps, kWsTopMem, kWsStage, kWsTsKeys, kWsTsTemp,  // 60 .. 89
  kWsRelay = 94,
  kWsMultiExt = 120, kWsMultiOut, kWsCommitExt  // (snark.hip uses 91 .. 93 and 95, verify.hip 96, msm_big.hip
                                                // 100 .. 108, sumcheck.hip 110 .. 111)
};

// PolyCommitmentGens::new(nv, label) as a view of one derived generator stream (dense_mlpoly.rs:88-98)
ProverGens gens_view(spg_gens* dev, size_t nv) {
  ProverGens g;
  g.dev = dev;
  g.host.init(dev->compressed, dev->n + 1);
  size_t n = (size_t)1 << (nv - nv / 2);
  g.n_pc = n;
  g.gens_n.G.resize(n);
  for (size_t i = 0; i < n; i++) g.gens_n.G[i] = i;
  g.gens_n.h = n + 1;
  g.gens_1.G = {n};
  g.gens_1.h = n + 1;
  return g;
}

// Encodings of B device points into host Pt's. Up to SPG_HOST_ENC_MAX (384) points the points come down (128 B each)
// and are encoded on the host pool: one encoding is a ~2.4 us inverse square root on a host core, while
// k_compress_ext gives each point one GPU lane whose ~250 dependent squarings take ~130 us whatever the count.
// Larger batches encode on the device (d_out: 32 B per point of device scratch).
// halved: the device points are P / 2 (msm_comb's halve), encoded as the doubles on the host pool in chunks of one
// field inversion each (hext_double_and_compress_batch: ~25 products per point instead of a ~265-step inverse square
// root on a GPU lane or a host core), at any count
static int encode_points(spg_ctx* ctx, const Ext* d_ext, size_t B, Pt* out, uint8_t* d_out, bool halved = false) {
  static const size_t host_max = getenv("SPG_HOST_ENC_MAX") ? (size_t)atol(getenv("SPG_HOST_ENC_MAX")) : 384;
  if (halved) {
    Ext* h = (Ext*)enc_stage_get(ctx, B * sizeof(Ext));
    if (!h) return set_err(ctx, SPG_E_NOMEM, "encoding staging");
    static const bool tr3 = getenv("SPG_TRACE") && atoi(getenv("SPG_TRACE")) >= 3;
    const auto t0 = std::chrono::steady_clock::now();
    SPG_HIP(ctx, hipMemcpyAsync(h, d_ext, B * sizeof(Ext), hipMemcpyDeviceToHost, ctx->stream));
    SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const auto t1 = std::chrono::steady_clock::now();
    encode_halved_host(h, B, out);
    if (tr3)
      fprintf(stderr, "[spg] halved encodings of %zu points: device + download %.0f us, host %.0f us\n", B,
              std::chrono::duration<double, std::micro>(t1 - t0).count(),
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count());
    return 0;
  }
  if (B <= host_max) {
    Ext* h = (Ext*)enc_stage_get(ctx, B * sizeof(Ext));
    if (!h) return set_err(ctx, SPG_E_NOMEM, "encoding staging");
    SPG_HIP(ctx, hipMemcpyAsync(h, d_ext, B * sizeof(Ext), hipMemcpyDeviceToHost, ctx->stream));
    SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const int C = B >= 16 ? (int)std::min<size_t>(B / 2, (size_t)pool().size() + 1) : 1;
    auto enc = [&](int c) {
      for (size_t i = B * c / C; i < B * (c + 1) / C; i++) out[i] = compress(h::hext_from_dev(h[i]));
    };
    if (C == 1)
      enc(0);
    else
      pool().parallel_for(C, enc);
    return 0;
  }
  int rc = compress_ext_device(ctx, d_ext, B, d_out);
  if (rc) return rc;
  SPG_HIP(ctx, hipMemcpyAsync(out, d_out, 32 * B, hipMemcpyDeviceToHost, ctx->stream));
  SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

// L rows of R device scalars on the latency-path generators into device points: the comb tables when they apply
// (>= 64 rows, >= 2^14 scalars in all), else the latency-path bucket kernels
// (*halved: the comb path left P / 2, encode_points' halved form, when `want` -- batches of >= kHalvedMin points: below
// that the host's lone encodings on the pool were as fast in the prover, 142 against 190 us for 128 rows;
// SPG_HALVED_ENC=0 keeps the device / lone encodings everywhere)
static const size_t kHalvedMin = 384;
static int rows_to_points(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, size_t R, size_t L, Ext* d_ext, bool* halved,
                          bool want) {
  static const bool on = !getenv("SPG_HALVED_ENC") || atoi(getenv("SPG_HALVED_ENC")) != 0;
  const bool halve = on && want;
  *halved = false;
  if (L >= 64 && L * R >= ((size_t)1 << 14)) {
    const int rc = msm_comb(ctx, g.dev, 0, d_Z, R, L, nullptr, nullptr, -1, d_ext, halve);
    if (rc != kCombSkip) {
      *halved = halve;
      return rc;
    }
  }
  return msm_small_device(ctx, g.dev, 0, d_Z, R, L, nullptr, d_ext, nullptr, -1);
}

// L Hyrax rows of R consecutive device scalars each -> L compressed row commitments (host). Rows of up to
// kSmallRowMax scalars take the latency MSM path (one block per bucket and row), longer rows the sorted batch
// pipeline in chunks that keep its sort within 32-bit indices.
int commit_rows(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, size_t R, size_t L, Pt* out) {
  if (R > g.n_pc) return set_err(ctx, SPG_E_ARG, "commit: rows wider than the generators");
  const bool small = R <= kSmallRowMax;
  const size_t chunk = small ? std::min<size_t>(L, 65535)
                             : std::max<size_t>(1, std::min<size_t>(L, ((size_t)1 << 24) / R));
  uint8_t* d_out = (uint8_t*)ws_get(ctx, kWsCommit, 32 * chunk + 64);
  if (!d_out) return set_err(ctx, SPG_E_NOMEM, "commit out");
  static const bool trace2 = getenv("SPG_TRACE") && atoi(getenv("SPG_TRACE")) >= 2;
  // SPG_HOST_COMMIT_MAX (default 0: off): row batches of at most this many scalars are committed on the host pool against
  // the generators' fixed-base byte tables (HostGens, built once per generator set): the scalars come down (<= 32 KB)
  // and 32 mixed additions per scalar spread over the pool, instead of a device bucket launch, its host finals and a
  // synchronisation (8 scalars: 35-40 us against 44-49 us; 256: 69 against 79 us; 512 scalars already take longer there,
  // 115 against 86 us, profiles/r05_ab_host_commit.txt). Off: a generator's table is built on its first use (11-24 ms
  // for the 8- and 16-generator rows of config 4's first proof), and config 4 measured 4.03 against 3.86 ms with it
  // (ABBA, profiles/r05_ab_host_commit_c4.txt)
  static const size_t host_commit_max =
      getenv("SPG_HOST_COMMIT_MAX") ? (size_t)atol(getenv("SPG_HOST_COMMIT_MAX")) : 0;
  for (size_t r0 = 0; r0 < L; r0 += chunk) {
    size_t nb = std::min(chunk, L - r0);
    auto t0 = std::chrono::steady_clock::now();
    if (small && nb * R <= host_commit_max) {
      FqV hz(nb * R);
      SPG_HIP(ctx, hipMemcpyAsync(hz.data(), d_Z + r0 * R, nb * R * sizeof(Fq), hipMemcpyDeviceToHost, ctx->stream));
      SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
      std::vector<std::pair<std::vector<size_t>, FqV>> jobs(nb);
      std::vector<size_t> idx(R);
      for (size_t i = 0; i < R; i++) idx[i] = g.gens_n.G[i];
      for (size_t b = 0; b < nb; b++) {
        jobs[b].first = idx;
        jobs[b].second.assign(hz.begin() + b * R, hz.begin() + (b + 1) * R);
      }
      const std::vector<Pt> pts = g.host.commit_many(jobs);
      std::copy(pts.begin(), pts.end(), out + r0);
    } else if (small && nb <= kHostFinalRows) {
      // few rows: the bucket running sums and encodings are cheaper on host cores than the device's
      // one-lane-per-row final + compress (~0.25 ms floor)
      void* d_map = nullptr;
      Ext* mbk = (Ext*)mapped_get(ctx, sizeof(Ext) * nb * 256, &d_map);  // buckets straight into host memory
      Ext* d_bk = mbk ? (Ext*)d_map : (Ext*)ws_get(ctx, kWsCommitBk, sizeof(Ext) * nb * 256 + 64);
      Ext* bk = mbk ? mbk : (Ext*)pinned_get(ctx, sizeof(Ext) * nb * 256);
      if (!d_bk || !bk) return set_err(ctx, SPG_E_NOMEM, "commit buckets");
      int NB = 0;
      int rc = msm_small_buckets(ctx, g.dev, 0, d_Z + r0 * R, R, nb, nullptr, nullptr, -1, d_bk, &NB);
      if (rc) return rc;
      if (!mbk)
        SPG_HIP(ctx, hipMemcpyAsync(bk, d_bk, sizeof(Ext) * nb * NB, hipMemcpyDeviceToHost, ctx->stream));
      SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
      bucket_finals(bk, nb, NB, out + r0);
    } else if (small) {
      Ext* d_ext = (Ext*)ws_get(ctx, kWsCommitExt, sizeof(Ext) * nb + 64);
      if (!d_ext) return set_err(ctx, SPG_E_NOMEM, "commit points");
      bool halved = false;
      int rc = rows_to_points(ctx, g, d_Z + r0 * R, R, nb, d_ext, &halved, nb >= kHalvedMin);
      if (!rc) rc = encode_points(ctx, d_ext, nb, out + r0, d_out, halved);  // synchronous: d_ext, d_out reused next chunk
      if (rc) return rc;
    } else {  // (halved comb points encoded on the host where the comb applies; synchronous)
      const int rc = msm_rows_host_enc(ctx, g.dev, d_Z + r0 * R, R, nb, nullptr, (long)(g.n_pc + 1), (uint8_t*)(out + r0));
      if (rc) return rc;
    }
    if (trace2)
      fprintf(stderr, "[spg] commit rows=%zu R=%zu %s %.0f us\n", nb, R,
              small && nb * R <= host_commit_max ? "host" : (small ? "small" : "batch"),
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  return 0;
}

static bool rows_merged(const RowJob& j) { return j.R <= kSmallRowMax && j.L > kHostFinalRows && j.L <= 65535; }

int commit_rows_many_launch(spg_ctx* ctx, ProverGens& g, const std::vector<RowJob>& jobs, RowsPending* p) {
  p->tot = 0;
  p->hv.clear();
  for (const RowJob& j : jobs) {
    if (j.R > g.n_pc) return set_err(ctx, SPG_E_ARG, "commit: rows wider than the generators");
    if (rows_merged(j)) p->tot += j.L;
  }
  if (!p->tot) return 0;
  p->d_ext = (Ext*)ws_get(ctx, kWsMultiExt, p->tot * sizeof(Ext) + 64);
  p->d_out = (uint8_t*)ws_get(ctx, kWsMultiOut, 32 * p->tot + 64);
  if (!p->d_ext || !p->d_out) return set_err(ctx, SPG_E_NOMEM, "commit rows");
  size_t o = 0;
  for (const RowJob& j : jobs) {
    if (!rows_merged(j)) continue;
    bool h = false;
    const int rc = rows_to_points(ctx, g, j.d_Z, j.R, j.L, p->d_ext + o, &h, p->tot >= kHalvedMin);
    if (rc) return rc;
    p->hv.push_back(h);
    o += j.L;
  }
  return 0;
}

int commit_rows_many_finish(spg_ctx* ctx, ProverGens& g, const std::vector<RowJob>& jobs, RowsPending& p) {
  if (p.tot) {  // the encodings of each run of merged jobs with the same form (halved comb points or not)
    std::vector<Pt> rows(p.tot);
    size_t k = 0, a = 0, o = 0;
    for (const RowJob& j : jobs) {
      if (!rows_merged(j)) continue;
      o += j.L;
      k++;
      if (k == p.hv.size() || p.hv[k] != p.hv[k - 1]) {  // the run [a, o) ends here
        const int rc = encode_points(ctx, p.d_ext + a, o - a, rows.data() + a, p.d_out + 32 * a, p.hv[k - 1] != 0);
        if (rc) return rc;
        a = o;
      }
    }
    o = 0;
    for (const RowJob& j : jobs) {
      if (!rows_merged(j)) continue;
      std::copy(rows.begin() + o, rows.begin() + o + j.L, j.out);
      o += j.L;
    }
  }
  for (const RowJob& j : jobs) {
    if (rows_merged(j)) continue;
    int rc = commit_rows(ctx, g, j.d_Z, j.R, j.L, j.out);
    if (rc) return rc;
  }
  return 0;
}

int commit_rows_many(spg_ctx* ctx, ProverGens& g, const std::vector<RowJob>& jobs) {
  RowsPending p;
  const int rc = commit_rows_many_launch(ctx, g, jobs, &p);
  return rc ? rc : commit_rows_many_finish(ctx, g, jobs, p);
}

// Hyrax rows split over the ranks of sh (SURVEY 8e "Hyrax commits: rows per GPU, allgather of the 32-byte
// rows"): rank r commits rows [b(r), b(r+1)) of the balanced split, then every rank receives all L encodings
int commit_rows_sh(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, size_t R, size_t L, Pt* out, const Shard& sh) {
  if (sh.n == 1) return commit_rows(ctx, g, d_Z, R, L, out);
  const size_t r0 = shard_begin(L, sh.n, sh.rank), r1 = shard_begin(L, sh.n, sh.rank + 1);
  const size_t per = (L + sh.n - 1) / sh.n;  // slots per rank in the gather
  std::vector<Pt> mine(per);
  int rc = r1 > r0 ? commit_rows(ctx, g, d_Z + r0 * R, R, r1 - r0, mine.data()) : 0;
  std::vector<uint8_t> all;
  rc = comm_allgather(ctx, sh, rc, mine.data(), per * sizeof(Pt), all);
  if (rc) return rc;
  for (int q = 0; q < sh.n; q++) {
    const size_t b0 = shard_begin(L, sh.n, q), b1 = shard_begin(L, sh.n, q + 1);
    memcpy(out + b0, all.data() + (size_t)q * per * sizeof(Pt), (b1 - b0) * sizeof(Pt));
  }
  return 0;
}

// DensePolynomial::commit without blinds (dense_mlpoly.rs:184-256) of 2^nv device scalars: L = 2^(nv/2)
// rows of R = 2^(nv - nv/2) scalars against the first R generators
int commit_dev(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, size_t nv, std::vector<Pt>* out, const Shard& sh) {
  size_t L = (size_t)1 << (nv / 2), R = (size_t)1 << (nv - nv / 2);
  out->resize(L);
  return commit_rows_sh(ctx, g, d_Z, R, L, out->data(), sh);
}

void append_polycomm(Tr& t, const char* label, const std::vector<Pt>& c) {
  t.msg(label, "poly_commitment_begin");
  for (auto& p : c) t.point("poly_commitment_share", p);
  t.msg(label, "poly_commitment_end");
}

// PolyEvalProof::prove without blinds (dense_mlpoly.rs:437-490) of a device polynomial of 2^|r| scalars.
// Sharded (sh.n > 1): rank r binds its balanced share of the Ls rows, the partial L.Z vectors are summed over the
// ranks, and every rank runs the same (replicated) Bullet rounds.
int poly_eval_prove(spg_ctx* ctx, ProverGens& g, const Fq* d_Z, const FqV& r, const Fq& Zr, Tr& t, Tape& tape,
                    DotProductProofLogP* out, const Shard& sh) {
  t.protocol("polynomial evaluation proof");
  size_t nv = r.size(), ln = nv / 2;
  FqV rl(r.begin(), r.begin() + ln), rr(r.begin() + ln, r.end());
  size_t Ls = (size_t)1 << ln, Rs = (size_t)1 << (nv - ln);
  if (Rs > g.n_pc) return set_err(ctx, SPG_E_ARG, "poly eval: polynomial wider than the generators");
  FqV R = eq_evals_host(rr);
  const size_t j0 = shard_begin(Ls, sh.n, sh.rank), j1 = shard_begin(Ls, sh.n, sh.rank + 1), Lm = j1 - j0;
  FqV LZ(Rs, fq_zero());
  int rc = 0;
  if (Lm) {
    size_t S = std::min<size_t>(Lm, std::max<size_t>(1, 8192 / nblk(Rs)));  // row splits to fill the chip
    size_t chunk = (Lm + S - 1) / S;
    S = (Lm + chunk - 1) / chunk;
    Fq* dL = (Fq*)ws_get(ctx, kWsL, Ls * sizeof(Fq) + 64);
    Fq* dpart = (Fq*)ws_get(ctx, kWsBoundPart, S * Rs * sizeof(Fq) + 64);
    Fq* dout = (Fq*)ws_get(ctx, kWsBound, Rs * sizeof(Fq) + 64);
    if (!dL || !dpart || !dout) rc = set_err(ctx, SPG_E_NOMEM, "poly_eval_prove");
    if (!rc) rc = eq_table(ctx, rl, dL);
    if (!rc) {
      KScope ks(ctx, "spark_bound", 32.0 * (double)Lm * Rs + 64.0 * S * Rs);
      hipLaunchKernelGGL(k_bound_rows, dim3(nblk(Rs), (unsigned)S), dim3(256), 0, ctx->stream, d_Z + j0 * Rs, dL + j0,
                         Lm, Rs, chunk, dpart);
      hipLaunchKernelGGL(k_bound_sum, dim3((unsigned)((Rs + kBoundSumCols - 1) / kBoundSumCols)), dim3(256), 0,
                         ctx->stream, dpart, S, Rs, dout);
      if (hipGetLastError() != hipSuccess) rc = set_err(ctx, SPG_E_HIP, "poly_eval_prove launch");
    }
    if (!rc) rc = d2h_fq(ctx, dout, LZ.data(), Rs);
  }
  rc = comm_sum_fq(ctx, sh, rc, LZ.data(), Rs);
  if (rc) return rc;
  Pt cy;
  return dotproduct_log_prove(ctx, g, t, tape, LZ, fq_zero(), R, Zr, fq_zero(), out, &cy);
}

// out[s] = sum_i base[s * seglen + i] * eq[i], i < n, s < nseg; sharded: rank r sums its balanced share of i.
// Several such dot sets queued back to back into disjoint workspace ranges: one download (and, sharded, one
// summing allgather) for all of them instead of one per set.
struct SegDotJob {
  const Fq* base;
  size_t seglen, nseg;
  const Fq* d_eq;
  size_t n;
  FqV* out;
};
static int seg_dots_multi(spg_ctx* ctx, const std::vector<SegDotJob>& jobs, const Shard& sh = Shard()) {
  std::vector<unsigned> nbs(jobs.size(), 0);
  size_t tot_part = 0, tot_res = 0;
  bool all_local = true;
  for (size_t k = 0; k < jobs.size(); k++) {
    const SegDotJob& j = jobs[k];
    const size_t nm = shard_begin(j.n, sh.n, sh.rank + 1) - shard_begin(j.n, sh.n, sh.rank);
    if (nm) nbs[k] = (unsigned)std::min<size_t>(nblk(nm), std::max<size_t>(1, 2048 / j.nseg));
    else all_local = false;
    tot_part += j.nseg * nbs[k];
    tot_res += j.nseg;
  }
  FqV all(tot_res, fq_zero());
  int rc = 0;
  if (tot_part) {
    Fq* part = (Fq*)ws_get(ctx, kWsSegPart, tot_part * sizeof(Fq) + 64);
    Fq* dres = (Fq*)ws_get(ctx, kWsSeg, tot_res * sizeof(Fq) + 64);
    if (!part || !dres) rc = set_err(ctx, SPG_E_NOMEM, "seg_dots");
    if (!rc && !all_local && hipMemsetAsync(dres, 0, tot_res * sizeof(Fq), ctx->stream) != hipSuccess)
      rc = set_err(ctx, SPG_E_HIP, "seg_dots memset");
    size_t po = 0, ro = 0;
    for (size_t k = 0; !rc && k < jobs.size(); k++) {
      const SegDotJob& j = jobs[k];
      if (nbs[k]) {
        const size_t i0 = shard_begin(j.n, sh.n, sh.rank), nm = shard_begin(j.n, sh.n, sh.rank + 1) - i0;
        KScope ks(ctx, "spark_evaluate", 32.0 * nm * j.nseg + 32.0 * nm);
        hipLaunchKernelGGL(k_seg_dot, dim3(nbs[k], (unsigned)j.nseg), dim3(256), 0, ctx->stream, j.base + i0, j.seglen,
                           j.d_eq + i0, nm, part + po);
        hipLaunchKernelGGL(k_sum_seg, dim3((unsigned)j.nseg), dim3(256), 0, ctx->stream, part + po, (int)nbs[k],
                           dres + ro);
        if (hipGetLastError() != hipSuccess) rc = set_err(ctx, SPG_E_HIP, "seg_dots launch");
      }
      po += j.nseg * nbs[k];
      ro += j.nseg;
    }
    if (!rc) rc = d2h_fq(ctx, dres, all.data(), tot_res);
  }
  rc = comm_sum_fq(ctx, sh, rc, all.data(), tot_res);
  if (rc) return rc;
  size_t ro = 0;
  for (const SegDotJob& j : jobs) {
    j.out->assign(all.begin() + ro, all.begin() + ro + j.nseg);
    ro += j.nseg;
  }
  return 0;
}

// UniPoly::append_to_transcript (unipoly.rs:112-120)
static void append_unipoly(Tr& t, const FqV& c) {
  t.msg("poly", "UniPoly_begin");
  for (auto& x : c) t.scalar("coeff", x);
  t.msg("poly", "UniPoly_end");
}

struct LayerProofP {
  std::vector<FqV> polys;  // CompressedUniPoly per round
  FqV left, right;
};
struct BatchedProofP {  // ProductCircuitEvalProofBatched
  std::vector<LayerProofP> layers;
  FqV dotp[3];
  void ser(Writer& w) const {
    w.u64(layers.size());
    for (auto& l : layers) {
      w.u64(l.polys.size());
      for (auto& p : l.polys) w.fqs(p);
      w.fqs(l.left);
      w.fqs(l.right);
    }
    for (int i = 0; i < 3; i++) w.fqs(dotp[i]);
  }
};

// workgroups and block size of a fused layer round over W = nt * len elements: one workgroup up to kOneWgMax
// elements (no ticket), else about kEltPerThread elements per thread over 256-thread workgroups
static void layer_grid(size_t W, unsigned* K, int* BS) {
  static const size_t one_wg = getenv("SPG_LAYER_ONEWG") ? (size_t)atoi(getenv("SPG_LAYER_ONEWG")) : 512;
  static const size_t ept = getenv("SPG_LAYER_EPT") ? (size_t)std::max(1, atoi(getenv("SPG_LAYER_EPT"))) : 2;
  if (W <= 64) {
    *K = 1;
    *BS = 64;
  } else if (W <= one_wg) {
    *K = 1;
    *BS = 256;
  } else {
    *BS = 256;
    *K = (unsigned)std::min<size_t>((W + 256 * ept - 1) / (256 * ept), 2048);
  }
}

// A set of nc product circuits (M leaves each), possibly sharded over the W ranks of a proof (see "sharded
// proof" at spark_prove_core): rank r holds leaves i = W i' + r as a local tree of m = M / W leaves (levels of
// >= 2 entries at loc + c 2m, the usual back-to-back layout), and every rank holds the global levels of <= W
// entries as a replicated "top" tree (circuit c at top + c 2W, W entries first). W == 1: loc is the whole tree.
struct TreeSh {
  Fq* loc = nullptr;
  size_t m = 0;
  Fq* top = nullptr;
  int W = 1, r = 0;
};

// ProductCircuitEvalProofBatched::prove with fused layer rounds (k_layer_round / k_layer_close above); same
// transcript and proof as batched_prove below.
// A layer whose vectors are sharded (global half length >= W) runs its first lg(half / W) rounds on the local
// shares (pairs (i, i + len) stay on one rank while W | len; the round's (e0, e2, e3) are summed over the ranks),
// then gathers the W remaining entries of every vector (k_layer_close without the fold when no round ran) and
// runs the last lg W rounds replicated, exactly like an unsharded layer of that length.
static int batched_prove_fused(spg_ctx* ctx, const TreeSh& ts, size_t nc, size_t M, FqV claims,
                               const std::vector<Triple>& dotp, const FqV& dotp_claims, Tr& t, BatchedProofP* out,
                               FqV* rand_out, const Shard& sh) {
  hipStream_t s = ctx->stream;
  const size_t L = lg2(M), W = (size_t)ts.W, lgW = lg2(W), m = ts.m, lgm = lg2(m);
  auto off = [](size_t MM, size_t k) { return 2 * MM - 2 * (MM >> k); };
  const size_t nt_max = nc + dotp.size();
  if (3 * nt_max + 1 > kMboxScalars) return set_err(ctx, SPG_E_ARG, "batched_prove: too many circuits for the mailbox");
  const size_t half_max = std::max<size_t>(M / 2 / W, 1);  // the longest eq vector held here
  Fq* cbuf[2] = {(Fq*)ws_get(ctx, kWsC, std::max(half_max, W) * sizeof(Fq) + 64),
                 (Fq*)ws_get(ctx, kWsC2, std::max(half_max, W) * sizeof(Fq) + 64)};
  // triples, then their coefficients, in one buffer (one upload per layer)
  const size_t tr_bytes = (nt_max * sizeof(Triple) + 63) & ~(size_t)63;
  uint8_t* ddesc = (uint8_t*)ws_get(ctx, kWsTriples, tr_bytes + nt_max * sizeof(Fq) + 64);
  Fq* part = (Fq*)ws_get(ctx, kWsPart, 3 * 2048 * sizeof(Fq) + 64);  // K <= 2048 workgroups per round
  Fq* gbuf = W > 1 ? (Fq*)ws_get(ctx, kWsGather, 3 * nt_max * W * sizeof(Fq) + 64) : nullptr;
  if (!cbuf[0] || !cbuf[1] || !ddesc || !part || (W > 1 && !gbuf)) return set_err(ctx, SPG_E_NOMEM, "batched_prove");
  const Triple* dtr = (const Triple*)ddesc;
  const Fq* dcoef = (const Fq*)(ddesc + tr_bytes);
  FqV rand;
  Laps lp;
  lp.title = "ProductCircuitEvalProofBatched::prove";
  // W > 1: a failure on this rank alone (allocation, HIP, mailbox) is not returned at once -- the peers would wait
  // in the next exchange. The rank stops working (`fail`, skip mode) but keeps the exchange sequence, whose
  // shape depends only on public sizes, until its status reaches every rank: in the next sharded round's
  // exchange, or in the status exchange that ends the function. A failure learned in an exchange is known to
  // every rank (`shared`) and returns at once.
  int fail = 0;
  bool shared = false;
  for (size_t layer = L; layer-- > 0;) {
    const size_t half = M >> (layer + 1);  // |left| = |right| = |C| (global)
    // where this layer's vectors live: local shares (sharded), the replicated top tree, or the whole tree
    const bool sharded = W > 1 && layer < lgm;
    const size_t hl = sharded ? half / W : half;  // entries of each vector held here
    int rc = fail;
    if (!rc && sharded && failpoint(ctx, "spark_layer")) rc = set_err(ctx, SPG_E_HIP, "failpoint spark_layer");
    int cur = 0;  // the buffer holding the shared eq vector C
    const bool with_dotp = layer == 0 && !dotp.empty();
    std::vector<Triple> tr;
    for (size_t c = 0; c < nc; c++) {
      Fq* v = sharded || W == 1 ? ts.loc + c * 2 * m + off(m, layer) : ts.top + c * 2 * W + off(W, layer - lgm);
      tr.push_back({v, v + hl, nullptr});  // C: the shared eq vector
    }
    if (with_dotp) {
      claims.insert(claims.end(), dotp_claims.begin(), dotp_claims.end());
      for (auto& d : dotp) tr.push_back(d);
    }
    FqV coeffs = t.challenges("rand_coeffs_next_layer", claims.size());
    Fq e = fq_zero();
    for (size_t i = 0; i < claims.size(); i++) e = fq_add(e, fq_mul(claims[i], coeffs[i]));
    // the layer's descriptors and coefficients ride in the eq-table launch's arguments when they fit (no copy
    // command on the stream), through page-locked staging otherwise
    KBlob blob;  // 2.3 KB on the stack (contexts on other threads prove concurrently)
    const size_t blob_bytes = tr_bytes + coeffs.size() * sizeof(Fq);
    const bool in_args = blob_bytes <= sizeof(blob.w) && !getenv("SPG_LAYER_DESC_COPY");
    if (in_args) {
      memset(blob.w, 0, tr_bytes);
      memcpy(blob.w, tr.data(), tr.size() * sizeof(Triple));
      memcpy((uint8_t*)blob.w + tr_bytes, coeffs.data(), coeffs.size() * sizeof(Fq));
      blob.nwords = (int)(blob_bytes / 4);
    } else if (!rc) {  // free again here (the previous layer ended with a mailbox wait after its last launch)
      uint8_t* st = (uint8_t*)pinned_get(ctx, blob_bytes + 64);
      if (!st) {
        rc = set_err(ctx, SPG_E_NOMEM, "layer staging");
      } else {
        memcpy(st, tr.data(), tr.size() * sizeof(Triple));
        memcpy(st + tr_bytes, coeffs.data(), coeffs.size() * sizeof(Fq));
        if (hipMemcpyAsync(ddesc, st, blob_bytes, hipMemcpyHostToDevice, s) != hipSuccess)
          rc = set_err(ctx, SPG_E_HIP, "layer descriptors upload");
      }
    }
    const KBlob* bp = in_args ? &blob : nullptr;
    if (rc) {
      // skip mode: no device work this layer
    } else if (sharded) {  // local eq share: eq(rand)[W i' + r] = eq(rand_hi)[i'] * eq(rand_lo)[r]
      const size_t nh = rand.size() - lgW;
      rc = dev_eq_table(ctx, rand.data(), (int)nh, cbuf[0], bp, ddesc);
      Fq sc = fq_one();
      for (size_t k = 0; k < lgW; k++)
        sc = fq_mul(sc, ((ts.r >> (lgW - 1 - k)) & 1) ? rand[nh + k] : fq_sub(fq_one(), rand[nh + k]));
      if (!rc) hipLaunchKernelGGL(k_scale, dim3(nblk(hl)), dim3(256), 0, s, cbuf[0], hl, sc);
    } else {
      rc = dev_eq_table(ctx, rand.data(), (int)rand.size(), cbuf[0], bp, ddesc);
    }
    if (rc && W == 1) return rc;
    lp.lap("layer_setup");
    LayerProofP lpf;
    FqV r_prod;
    bool pending = false;  // a bound_poly_var_top with r_pend not yet applied
    Fq r_pend = fq_zero();
    // after a paired launch (k_layer_pair): a second pending fold, with r_pend2 (bound after r_pend); only a paired
    // launch applies two, and once a layer's rounds pair up they pair up to the layer's end
    bool pend2 = false;
    Fq r_pend2 = fq_zero();
    // after a tripled launch (k_layer_triple): a third, r_pend3; only a triple follows it
    bool pend3 = false;
    Fq r_pend3 = fq_zero();
    // A[0], B[0], C[0] of every triple (after the pending fold, if any), by mailbox
    auto close = [&](FqV& fin) -> int {
      if (pend2 || pend3) return set_err(ctx, SPG_E_ARG, "layer close after a paired round");  // (the last pair posts its ends)
      fin.resize(3 * tr.size());
      KScope ks(ctx, "spark_layer_close");
      const uint32_t seq = ++ctx->mbox_seq;
      hipLaunchKernelGGL(k_layer_close, dim3(1), dim3(256), 0, s, dtr, (int)tr.size(), pending ? 1 : 0, r_pend,
                         cbuf[cur], ctx->d_mbox, seq);
      SPG_HIP(ctx, hipGetLastError());
      pending = false;
      return mbox_wait(ctx, seq, fin.data(), (int)fin.size());
    };
    // the host half of a round: UniPoly from (e0, e2, e3), transcript, r_j
    auto host_round = [&](const Fq ev[3]) -> Fq {
      Fq evals[4] = {ev[0], fq_sub(e, ev[0]), ev[1], ev[2]};
      FqV poly = uni_from_evals3(evals);
      append_unipoly(t, poly);
      Fq r_j = t.challenge("challenge_nextround");
      r_prod.push_back(r_j);
      e = uni_eval(poly, r_j);
      lpf.polys.push_back({poly[0], poly[2], poly[3]});
      return r_j;
    };
    // the remaining log_len rounds of the layer in one persistent launch (layer.hpp, k_layer_persist): the host
    // answers each posted round through the downbox instead of launching the next one
    auto run_persist = [&](size_t log_len, bool close_after, FqV* fin) -> int {
      const int R = (int)log_len;
      const size_t nt = tr.size();
      static const size_t max_wgs = getenv("SPG_PERSIST_WGS") ? (size_t)atol(getenv("SPG_PERSIST_WGS")) : 64;
      const unsigned K = (unsigned)std::max<size_t>(1, std::min<size_t>(((nt << (R - 1)) * 4 + 255) / 256, max_wgs));
      const bool ends = close_after && 3 + 6 * nt <= kMboxScalars;
      PersistArgs A;
      A.tr = dtr;
      A.coeff = dcoef;
      A.nt = (int)nt;
      A.rounds = R;
      A.do_fold = pending ? 1 : 0;
      A.r = r_pend;
      A.cb[0] = cbuf[0];
      A.cb[1] = cbuf[1];
      A.cur = cur;
      A.partials = part;
      A.counter = ctx->d_counter;
      A.mb = ctx->d_mbox;
      A.seq0 = ctx->mbox_seq + 1;
      A.down = ctx->d_down;
      A.ends = ends ? 1 : 0;
      A.timeout = 2000000000ULL;  // 20 s of the 100 MHz wall clock
      static const bool relay_on = !getenv("SPG_PERSIST_RELAY") || atoi(getenv("SPG_PERSIST_RELAY")) != 0;
      A.relay = nullptr;
      if (relay_on && K > 1) {
        A.relay = (uint32_t*)ws_get(ctx, kWsRelay, 64);
        if (!A.relay) return set_err(ctx, SPG_E_NOMEM, "layer relay");
      }
      ctx->mbox_seq += (uint32_t)R;
      ctx->down[0] = 0;  // clear a previous launch's abort word
      {
        KScope ks(ctx, "spark_layer_persist");
        hipLaunchKernelGGL(k_layer_persist<256>, dim3(K), dim3(256), 0, s, A);
      }
      const hipError_t le = hipGetLastError();
      if (le != hipSuccess) return set_err(ctx, SPG_E_HIP, std::string("layer rounds: ") + hipGetErrorString(le));
      for (int k = 0; k < R; k++) {
        const bool last_round = k == R - 1;
        FqV ev(last_round && ends ? 3 + 6 * nt : 3);
        const int rc2 = mbox_wait(ctx, A.seq0 + (uint32_t)k, ev.data(), (int)ev.size());
        if (rc2) {
          if (!last_round) {
            down_post(ctx, kDownAbort, fq_zero());  // every workgroup leaves its wait
            // ... and has left before the next launch clears the abort word: the stream drains here
            (void)hipStreamSynchronize(s);
            (void)hipGetLastError();
          }
          return rc2;
        }
        lp.lap("round_eval_wait");
        if (pending) cur ^= 1;
        r_pend = host_round(ev.data());
        pending = true;
        lp.lap("round_host");
        if (!last_round) {
          down_post(ctx, A.seq0 + (uint32_t)k, r_pend);
        } else if (ends) {  // bound_poly_var_top of the length-2 vectors, on the host
          fin->resize(3 * nt);
          for (size_t c = 0; c < 3 * nt; c++) {
            const Fq lo = ev[3 + 2 * c], hi = ev[4 + 2 * c];
            (*fin)[c] = fq_add(lo, fq_mul(r_pend, fq_sub(hi, lo)));
          }
          pending = false;
          return 0;
        }
      }
      return close_after ? close(*fin) : 0;
    };
    // rounds while the vectors (2 len entries here) have len >= 1; `local` rounds sum over the ranks; with
    // close_after the layer's (or the shard's) final entries follow in `fin`
    static const bool ends_on = !getenv("SPG_LAYER_ENDS") || atoi(getenv("SPG_LAYER_ENDS")) != 0;
    // off by default: same-box A/B (profiles/r04_ab_persist_fuse_bcomb.txt) measured 21.5 ms per prove with the
    // resident launches against 18.9 ms without
    static const bool persist_on = getenv("SPG_LAYER_PERSIST") && atoi(getenv("SPG_LAYER_PERSIST")) != 0;
    auto run_rounds = [&](size_t log_len, bool local, bool close_after, FqV* fin, int status) -> int {
      if (status) {  // skip mode: the first local round's exchange carries the failure to every rank
        if (!local || log_len == 0) return status;
        Fq none[3] = {fq_zero(), fq_zero(), fq_zero()};
        shared = true;
        return comm_sum_fq(ctx, sh, status, none, 3);
      }
      static const bool quad = !getenv("SPG_LAYER_QUAD") || atoi(getenv("SPG_LAYER_QUAD")) != 0;
      static const size_t wide_min = getenv("SPG_WIDE_MIN") ? (size_t)atol(getenv("SPG_WIDE_MIN")) : ((size_t)1 << 19);
      static const size_t persist_max = getenv("SPG_PERSIST_MAX") ? (size_t)atol(getenv("SPG_PERSIST_MAX")) : 4096;
      static const bool pair_on = !getenv("SPG_LAYER_PAIR") || atoi(getenv("SPG_LAYER_PAIR")) != 0;
      static const size_t pair_max = getenv("SPG_PAIR_MAX") ? (size_t)atol(getenv("SPG_PAIR_MAX")) : 4096;
      static const bool triple_on = !getenv("SPG_LAYER_TRIPLE") || atoi(getenv("SPG_LAYER_TRIPLE")) != 0;
      // elements (a wave each, four per workgroup) of a tripled launch: 64 partials per workgroup in `part`
      static const size_t triple_max =
          std::min<size_t>(getenv("SPG_TRIPLE_MAX") ? (size_t)atol(getenv("SPG_TRIPLE_MAX")) : 384, 384);
      // relative wall of a launched single / paired / tripled round trip, for the launch plan below
      static const std::vector<int> step_cost = [] {
        std::vector<int> c = {18, 25, 30};
        if (const char* e = getenv("SPG_STEP_COSTS")) sscanf(e, "%d,%d,%d", &c[0], &c[1], &c[2]);
        return c;
      }();
      const size_t ngroups = (nc ? 1 : 0) + (tr.size() - nc);  // product circuits share one thread per index
      const size_t nt_all = tr.size();
      const bool multi = quad && !local && close_after && !(persist_on && ctx->nranks == 1);
      // two rounds in one launch (k_layer_pair): small rounds of an unsharded layer, every element's 16 lanes within
      // pair_max elements, the last pair's corners within the mailbox; three (k_layer_triple): a wave per element
      // within triple_max elements, the last triple's corners within the mailbox
      // a paired launch of E elements stores 16 partials per workgroup of BSp / 16 elements into `part` (3 x 2048
      // scalars): 16 E / BSp * 16 <= 6144, so E <= 6144 with 256-thread workgroups and E <= 1536 with 64-thread ones
      // (SPG_PAIR_BS = 64)
      static const int pair_bs = getenv("SPG_PAIR_BS") ? atoi(getenv("SPG_PAIR_BS")) : 0;  // 64: more workgroups
      const size_t pair_part_cap = pair_bs == 64 ? 1536 : 6144;
      auto pair_ok = [&](size_t k) {
        return pair_on && multi && k >= 2 && (nt_all << (k - 2)) <= std::min<size_t>(pair_max, pair_part_cap) &&
               15 + 12 * nt_all <= kMboxScalars && ngroups * ((size_t)1 << (k - 1)) < wide_min;
      };
      auto triple_ok = [&](size_t k) {
        return triple_on && multi && k >= 3 && (nt_all << (k - 3)) <= triple_max && 64 + 24 * nt_all <= kMboxScalars &&
               ngroups * ((size_t)1 << (k - 1)) < wide_min;
      };
      // the launch plan: single rounds first, then pairs, then triples (a pair leaves two pending folds, which only
      // a pair or a triple applies; a triple three, which only a triple applies), the cheapest by step_cost.
      // Returns the rounds of the first launch from k rounds left in state mode (0: free, 1: after a pair, 2: after a
      // triple), 0 when none finishes the layer.
      auto plan = [&](size_t k, int mode) -> int {
        const int inf = 1 << 28;
        std::vector<std::array<int, 3>> best(k + 1), first(k + 1);
        for (size_t j = 0; j <= k; j++)
          for (int md = 0; md < 3; md++) {
            int b = j == 0 ? 0 : inf, f = 0;
            if (j >= 1 && md == 0 && best[j - 1][0] < inf && step_cost[0] + best[j - 1][0] < b)
              b = step_cost[0] + best[j - 1][0], f = 1;
            if (md <= 1 && pair_ok(j) && best[j - 2][1] < inf && step_cost[1] + best[j - 2][1] < b)
              b = step_cost[1] + best[j - 2][1], f = 2;
            if (triple_ok(j) && best[j - 3][2] < inf && step_cost[2] + best[j - 3][2] < b)
              b = step_cost[2] + best[j - 3][2], f = 3;
            best[j][md] = b;
            first[j][md] = f;
          }
        return first[k][mode];
      };
      auto lagrange4 = [](const Fq& r, Fq L[4]) {  // the cubic Lagrange basis on 0..3 at r
        static const Fq inv2 = fq_inv(fq_from_u64(2)), inv6 = fq_inv(fq_from_u64(6));
        const Fq a0 = r, a1 = fq_sub(r, fq_one()), a2 = fq_sub(a1, fq_one()), a3 = fq_sub(a2, fq_one());
        const Fq a01 = fq_mul(a0, a1), a23 = fq_mul(a2, a3);
        L[0] = fq_neg(fq_mul(fq_mul(a1, a23), inv6));
        L[1] = fq_mul(fq_mul(a0, a23), inv2);
        L[2] = fq_neg(fq_mul(fq_mul(a01, a3), inv2));
        L[3] = fq_mul(fq_mul(a01, a2), inv6);
      };
      while (log_len > 0) {
        const int step = plan(log_len, pend3 ? 2 : (pend2 ? 1 : 0));
        if (step == 0) return set_err(ctx, SPG_E_ARG, "layer rounds: no launch plan");
        if (step == 3) {
          const int lgj = (int)log_len - 1;  // round j's half length 2^lgj; h = 2^(lgj - 2) elements per vector
          log_len -= 3;
          const size_t nt = tr.size(), h = (size_t)1 << (lgj - 2), E = nt * h;
          const int BSt = E <= 1 ? 64 : 256;
          const unsigned Kt = (unsigned)((E + BSt / 64 - 1) / (BSt / 64));
          const bool ends = log_len == 0;  // the layer's last triple posts every vector's 2 x 2 x 2 corners
          const int nf = pend3 ? 3 : (pend2 ? 2 : (pending ? 1 : 0));
          TripleArgs P;
          P.tr = dtr;
          P.coeff = dcoef;
          P.nt = (int)nt;
          P.log_len = lgj;
          P.nf = nf;
          P.r1 = r_pend;
          P.r2 = r_pend2;
          P.r3 = r_pend3;
          P.r12 = fq_mul(r_pend, r_pend2);
          P.r13 = fq_mul(r_pend, r_pend3);
          P.r23 = fq_mul(r_pend2, r_pend3);
          P.r123 = fq_mul(P.r12, r_pend3);
          P.cin = cbuf[cur];
          P.cout = cbuf[cur ^ 1];
          P.partials = part;
          P.counter = ctx->d_counter;
          P.mb = ctx->d_mbox;
          P.seq = ++ctx->mbox_seq;
          P.ends = ends ? 1 : 0;
          P.probe = nullptr;
          {
            // algorithmic bytes: per distinct vector and element, 8 corners from 8 2^nf entries, written back when folded
            const double per = 32.0 * (8.0 * (double)(1 << nf) + (nf ? 8.0 : 0.0));
            // Fq products per element: the 24 corners folded (2^nf - 1 each), 64 points x 3
            KScope ks(ctx, "spark_layer_triple", per * (double)h * (double)(2 * nt + ngroups), 0.0,
                      (double)nt * (double)h * (192.0 + 24.0 * (double)((1 << nf) - 1)));
            if (BSt == 64)
              hipLaunchKernelGGL(k_layer_triple<64>, dim3(Kt), dim3(64), 0, s, P);
            else
              hipLaunchKernelGGL(k_layer_triple<256>, dim3(Kt), dim3(256), 0, s, P);
          }
          if (nf) cur ^= 1;
          FqV ev(64 + (ends ? 24 * nt : 0));  // F(t, s, u) = ev[t + 4 s + 16 u], then the corners
          const hipError_t le = hipGetLastError();
          lp.lap(ends ? "triple_launch_end" : "triple_launch");
          const int rc2 = le != hipSuccess ? set_err(ctx, SPG_E_HIP, std::string("layer triple: ") + hipGetErrorString(le))
                                           : mbox_wait(ctx, P.seq, ev.data(), (int)ev.size());
          if (rc2) return rc2;
          lp.lap(ends ? "triple_wait_end" : "triple_wait");
          // round j: F(X, s, u) over s, u in {0, 1} at X = 0, 2, 3
          Fq ej[3];
          for (int xi = 0; xi < 3; xi++) {
            const int X = xi == 0 ? 0 : xi + 1;
            ej[xi] = fq_add(fq_add(ev[X], ev[X + 4]), fq_add(ev[X + 16], ev[X + 20]));
          }
          const Fq rj = host_round(ej);
          Fq L[4], M[4];
          lagrange4(rj, L);
          // round j + 1: t -> F(t, Y, 0) + F(t, Y, 1) at t = r_j, Y = 0, 2, 3
          Fq ej1[3];
          for (int yi = 0; yi < 3; yi++) {
            const int Y = yi == 0 ? 0 : yi + 1;
            Fq acc = fq_zero();
            for (int a = 0; a < 4; a++) acc = fq_add(acc, fq_mul(L[a], fq_add(ev[a + 4 * Y], ev[a + 4 * Y + 16])));
            ej1[yi] = acc;
          }
          const Fq rj1 = host_round(ej1);
          lagrange4(rj1, M);
          // round j + 2: (t, s) -> F(t, s, Z) at (r_j, r_j+1), Z = 0, 2, 3
          Fq ej2[3];
          for (int zi = 0; zi < 3; zi++) {
            const int Z = zi == 0 ? 0 : zi + 1;
            Fq acc = fq_zero();
            for (int b = 0; b < 4; b++) {
              Fq row = fq_zero();
              for (int a = 0; a < 4; a++) row = fq_add(row, fq_mul(L[a], ev[a + 4 * b + 16 * Z]));
              acc = fq_add(acc, fq_mul(M[b], row));
            }
            ej2[zi] = acc;
          }
          const Fq rj2 = host_round(ej2);
          lp.lap("triple_host");
          if (ends) {  // the 2 x 2 x 2 cube of every vector folded at (r_j, r_j+1, r_j+2): the layer's final claims
            fin->resize(3 * nt);
            auto fold3 = [&](size_t c0, size_t c1) {
              for (size_t c = c0; c < c1; c++) {
                const Fq* w = &ev[64 + 8 * c];  // corner m = 4 t + 2 s + u of vector c % 3 of triple c / 3
                Fq q[4];
                for (int j = 0; j < 4; j++) q[j] = fq_add(w[j], fq_mul(rj, fq_sub(w[j + 4], w[j])));
                const Fq y0 = fq_add(q[0], fq_mul(rj1, fq_sub(q[2], q[0]))),
                         y1 = fq_add(q[1], fq_mul(rj1, fq_sub(q[3], q[1])));
                (*fin)[c] = fq_add(y0, fq_mul(rj2, fq_sub(y1, y0)));
              }
            };
            // 7 products per vector: 500 for 24 circuits, ~8 us on one core; spread over the pool from 48 vectors
            const size_t nv = 3 * nt;
            const int K = nv >= 48 ? (int)std::min<size_t>(nv / 16, (size_t)pool().size() + 1) : 1;
            if (K == 1)
              fold3(0, nv);
            else
              pool().parallel_for(K, [&](int k) { fold3(nv * k / K, nv * (k + 1) / K); });
            pending = pend2 = pend3 = false;
            lp.lap("triple_fin");
            return 0;
          }
          pending = pend2 = pend3 = true;
          r_pend = rj;
          r_pend2 = rj1;
          r_pend3 = rj2;
          continue;
        }
        if (step == 2) {
          if (pend3) return set_err(ctx, SPG_E_ARG, "paired layer round after a tripled one");
          const int lgj = (int)log_len - 1;  // round j's half length 2^lgj; round j + 1's 2^(lgj - 1)
          log_len -= 2;
          const size_t nt = tr.size(), h = (size_t)1 << (lgj - 1), lanes = 16 * nt * h;
          const int BSp = lanes <= 64 || pair_bs == 64 ? 64 : 256;
          const unsigned Kp = (unsigned)((lanes + BSp - 1) / BSp);
          const bool ends = log_len == 0;  // the layer's last pair posts every vector's 2 x 2 corners
          const int nf = pend2 ? 2 : (pending ? 1 : 0);
          PairArgs P;
          P.tr = dtr;
          P.coeff = dcoef;
          P.nt = (int)nt;
          P.log_len = lgj;
          P.nf = nf;
          P.r1 = r_pend;
          P.r2 = r_pend2;
          P.r12 = fq_mul(r_pend, r_pend2);
          P.cin = cbuf[cur];
          P.cout = cbuf[cur ^ 1];
          P.partials = part;
          P.counter = ctx->d_counter;
          P.mb = ctx->d_mbox;
          P.seq = ++ctx->mbox_seq;
          P.ends = ends ? 1 : 0;
          P.probe = nullptr;
          {
            // algorithmic bytes: per distinct vector and element, 4 corners from 4 2^nf entries, written back when folded
            const double per = 32.0 * (4.0 * (double)(1 << nf) + (nf ? 4.0 : 0.0));
            // Fq products per element: the corners folded (12 x 3 with two pending folds, 12 with one), 15 points x 3
            KScope ks(ctx, "spark_layer_pair", per * (double)h * (double)(2 * nt + ngroups), 0.0,
                      (double)nt * (double)h * (45.0 + (nf == 2 ? 36.0 : nf == 1 ? 12.0 : 0.0)));
            if (BSp == 64)
              hipLaunchKernelGGL(k_layer_pair<64>, dim3(Kp), dim3(64), 0, s, P);
            else
              hipLaunchKernelGGL(k_layer_pair<256>, dim3(Kp), dim3(256), 0, s, P);
          }
          if (nf) cur ^= 1;
          FqV ev(15 + (ends ? 12 * nt : 0));
          const hipError_t le = hipGetLastError();
          lp.lap(ends ? "pair_launch_end" : "pair_launch");
          const int rc2 = le != hipSuccess ? set_err(ctx, SPG_E_HIP, std::string("layer pair: ") + hipGetErrorString(le))
                                           : mbox_wait(ctx, P.seq, ev.data(), (int)ev.size());
          if (rc2) return rc2;
          lp.lap(ends ? "pair_wait_end" : "pair_wait");
          // round j: F(X, 0) + F(X, 1) at X = 0, 2, 3
          const Fq ej[3] = {fq_add(ev[0], ev[12]), fq_add(ev[2], ev[13]), fq_add(ev[3], ev[14])};
          const Fq rj = host_round(ej);
          // round j + 1: the cubics t -> F(t, Y) through t = 0..3 (lines Y = 0, 2, 3) at t = r_j
          Fq L[4];
          lagrange4(rj, L);
          Fq ej1[3];
          for (int y = 0; y < 3; y++) {
            Fq acc = fq_zero();
            for (int k = 0; k < 4; k++) acc = fq_add(acc, fq_mul(L[k], ev[4 * y + k]));
            ej1[y] = acc;
          }
          const Fq rj1 = host_round(ej1);
          lp.lap("pair_host");
          if (ends) {  // the 2 x 2 cube of every vector folded at (r_j, r_j+1): the layer's final claims
            fin->resize(3 * nt);
            for (size_t c = 0; c < 3 * nt; c++) {
              const Fq* w = &ev[15 + 4 * c];  // p00, p01, p10, p11 of vector c % 3 of triple c / 3
              const Fq q0 = fq_add(w[0], fq_mul(rj, fq_sub(w[2], w[0]))), q1 = fq_add(w[1], fq_mul(rj, fq_sub(w[3], w[1])));
              (*fin)[c] = fq_add(q0, fq_mul(rj1, fq_sub(q1, q0)));
            }
            pending = pend2 = false;
            lp.lap("pair_fin");
            return 0;
          }
          pending = pend2 = true;
          r_pend = rj;
          r_pend2 = rj1;
          continue;
        }
        if (pend2 || pend3) return set_err(ctx, SPG_E_ARG, "single layer round after a paired one");
        // every remaining round is a quad round of at most persist_max elements: one persistent launch for them all
        // (one process per GPU only: processes sharing a GPU time-slice its queues, and a resident loop could then
        // wait out its timeout while descheduled)
        if (persist_on && quad && !local && ctx->nranks == 1 && (tr.size() << (log_len - 1)) <= persist_max &&
            ngroups * ((size_t)1 << (log_len - 1)) < wide_min)
          return run_persist(log_len, close_after, fin);
        log_len--;
        const size_t len = (size_t)1 << log_len;
        unsigned K;
        int BS;
        // algorithmic HBM bytes of the round: per distinct vector (A, B of every triple; the shared C once; each
        // dot-product circuit's own C) and index, 2 entries read, or with the pending fold 4 read + 2 written
        const double layer_bytes = (pending ? 192.0 : 64.0) * (double)len * (double)(2 * tr.size() + ngroups);
        if (ngroups * len >= wide_min) {  // throughput form for rounds that fill the chip
          K = (unsigned)std::min<size_t>((ngroups * len + 255) / 256, 2048);
          // Fq products per index: per product circuit k A B at 3 points from the folded A, B (3 + 2 + 4 folds), the
          // shared C folded once (2) and multiplied in (3); a dot-product circuit 14 (its own C folded too)
          const double fqm_w = (double)len * ((pending ? 2.0 : 0.0) + 3.0 + (double)nc * (pending ? 9.0 : 5.0) +
                                              (double)(tr.size() - nc) * (pending ? 14.0 : 8.0));
          KScope ks(ctx, "spark_layer_round", layer_bytes, 0.0, fqm_w);
          hipLaunchKernelGGL(k_layer_round_wide<256>, dim3(K), dim3(256), 0, s, dtr, dcoef, (int)nc, (int)tr.size(),
                             (int)log_len, pending ? 1 : 0, r_pend, cbuf[cur], cbuf[cur ^ 1], part, ctx->d_counter,
                             ctx->d_mbox, ++ctx->mbox_seq);
        } else if (quad) {  // a quad per element, about one element per quad
          const size_t Wd = tr.size() * len;
          BS = Wd <= 16 ? 64 : 256;
          K = (unsigned)std::min<size_t>((Wd * 4 + BS - 1) / BS, 2048);
        } else {
          layer_grid(tr.size() * len, &K, &BS);
        }
        // the layer's last round in one workgroup also posts every vector's two entries: the host then folds the
        // final claims with the round's challenge, and no close launch (another round trip) follows
        const bool ends = close_after && log_len == 0 && quad && K == 1 && 3 + 6 * tr.size() <= kMboxScalars &&
                          ngroups * len < wide_min && ends_on;
        if (ngroups * len < wide_min) {
          // Fq products per element: lanes 0..2 fold their vector's two entries (6) and form k A B C at their point (9)
          KScope ks(ctx, "spark_layer_round", layer_bytes, 0.0, (double)tr.size() * (double)len * (pending ? 15.0 : 9.0));
          const int nt = (int)tr.size(), lg = (int)log_len, df = pending ? 1 : 0;
          const uint32_t seq = ++ctx->mbox_seq;
          if (quad && BS == 64)
            hipLaunchKernelGGL(k_layer_round_q<64>, dim3(K), dim3(64), 0, s, dtr, dcoef, nt, lg, df, r_pend, cbuf[cur],
                               cbuf[cur ^ 1], part, ctx->d_counter, ctx->d_mbox, seq, nullptr, ends ? 1 : 0);
          else if (quad)
            hipLaunchKernelGGL(k_layer_round_q<256>, dim3(K), dim3(256), 0, s, dtr, dcoef, nt, lg, df, r_pend,
                               cbuf[cur], cbuf[cur ^ 1], part, ctx->d_counter, ctx->d_mbox, seq, nullptr, ends ? 1 : 0);
          else if (BS == 64)
            hipLaunchKernelGGL(k_layer_round<64>, dim3(K), dim3(64), 0, s, dtr, dcoef, nt, lg, df, r_pend, cbuf[cur],
                               cbuf[cur ^ 1], part, ctx->d_counter, ctx->d_mbox, seq, nullptr);
          else
            hipLaunchKernelGGL(k_layer_round<256>, dim3(K), dim3(256), 0, s, dtr, dcoef, nt, lg, df, r_pend, cbuf[cur],
                               cbuf[cur ^ 1], part, ctx->d_counter, ctx->d_mbox, seq, nullptr);
        }
        if (pending) cur ^= 1;
        FqV ev(ends ? 3 + 6 * tr.size() : 3);
        const hipError_t le = hipGetLastError();
        int rc2 = le != hipSuccess ? set_err(ctx, SPG_E_HIP, std::string("layer round: ") + hipGetErrorString(le))
                                   : mbox_wait(ctx, ctx->mbox_seq, ev.data(), (int)ev.size());
        if (local) {
          rc2 = comm_sum_fq(ctx, sh, rc2, ev.data(), 3);
          if (rc2) shared = true;
        }
        if (rc2) return rc2;
        lp.lap("round_eval_wait");
        r_pend = host_round(ev.data());
        pending = true;
        lp.lap("round_host");
        if (ends) {  // bound_poly_var_top of the length-2 vectors, on the host
          fin->resize(3 * tr.size());
          for (size_t c = 0; c < 3 * tr.size(); c++) {
            const Fq lo = ev[3 + 2 * c], hi = ev[4 + 2 * c];
            (*fin)[c] = fq_add(lo, fq_mul(r_pend, fq_sub(hi, lo)));
          }
          pending = false;
          return 0;
        }
      }
      return close_after ? close(*fin) : 0;
    };
    FqV fin;
    if (sharded) {
      // gather: every vector has one entry per rank left; rank q's entry is global index q
      FqV mine;
      rc = run_rounds(lg2(hl), true, true, &mine, rc);
      if (rc && shared) return rc;
      mine.resize(3 * tr.size(), fq_zero());
      std::vector<uint8_t> all;
      rc = comm_allgather(ctx, sh, rc, mine.data(), 3 * tr.size() * sizeof(Fq), all);
      if (rc) return rc;  // known to every rank
      const Fq* g = (const Fq*)all.data();
      const size_t nt = tr.size();
      uint8_t* st = (uint8_t*)pinned_get(ctx, 3 * nt * W * sizeof(Fq) + tr_bytes + 64);
      if (!st) {
        rc = set_err(ctx, SPG_E_NOMEM, "gather staging");
      } else {
        Fq* hv = (Fq*)(st + tr_bytes);
        for (size_t c = 0; c < nt; c++)
          for (size_t k = 0; k < 3; k++)
            for (size_t q = 0; q < W; q++) hv[(3 * c + k) * W + q] = g[q * 3 * nt + 3 * c + k];
        for (size_t c = 0; c < nt; c++) {
          const bool own_c = tr[c].C != nullptr;
          tr[c] = {gbuf + 3 * c * W, gbuf + (3 * c + 1) * W, own_c ? gbuf + (3 * c + 2) * W : nullptr};
        }
        memcpy(st, tr.data(), nt * sizeof(Triple));
        if (hipMemcpyAsync(ddesc, st, nt * sizeof(Triple), hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(gbuf, hv, 3 * nt * W * sizeof(Fq), hipMemcpyHostToDevice, s) != hipSuccess ||
            // the product circuits' shared eq vector (every product triple gathered the same entries)
            (nc && hipMemcpyAsync(cbuf[cur], gbuf + 2 * W, W * sizeof(Fq), hipMemcpyDeviceToDevice, s) != hipSuccess))
          rc = set_err(ctx, SPG_E_HIP, "gathered entries upload");
      }
      rc = run_rounds(lgW, false, true, &fin, rc);
    } else {
      rc = run_rounds(lg2(hl), false, true, &fin, rc);
    }
    if (rc && (W == 1 || shared)) return rc;
    if (rc) {  // this rank alone: skip mode until an exchange carries it
      fail = rc;
      continue;
    }
    for (size_t c = 0; c < nc; c++) {
      lpf.left.push_back(fin[3 * c]);
      lpf.right.push_back(fin[3 * c + 1]);
    }
    for (size_t c = 0; c < nc; c++) {
      t.scalar("claim_prod_left", lpf.left[c]);
      t.scalar("claim_prod_right", lpf.right[c]);
    }
    if (with_dotp) {
      for (size_t k = 0; k < dotp.size(); k++)
        for (int i = 0; i < 3; i++) out->dotp[i].push_back(fin[3 * (nc + k) + i]);
      for (size_t k = 0; k < dotp.size(); k++) {
        t.scalar("claim_dotp_left", out->dotp[0][k]);
        t.scalar("claim_dotp_right", out->dotp[1][k]);
        t.scalar("claim_dotp_weight", out->dotp[2][k]);
      }
    }
    Fq r_layer = t.challenge("challenge_r_layer");
    claims.assign(nc, fq_zero());
    for (size_t c = 0; c < nc; c++) claims[c] = fq_add(lpf.left[c], fq_mul(r_layer, fq_sub(lpf.right[c], lpf.left[c])));
    rand.assign(1, r_layer);
    rand.insert(rand.end(), r_prod.begin(), r_prod.end());
    out->layers.push_back(std::move(lpf));
    lp.lap("layer_finals");
  }
  if (W > 1) {  // every rank's status, so a failure still pending here fails every rank alike
    std::vector<uint8_t> none;
    const int rc = comm_allgather(ctx, sh, fail, nullptr, 0, none);
    if (rc) return rc;
  }
  lp.print();
  *rand_out = rand;
  return 0;
}

// ProductCircuitEvalProofBatched::prove (product_tree.rs:271-396) over the nc product circuits of `tree`
// (M leaves each, claims = their ProductCircuit::evaluate) and, at layer 0, the dot-product circuits
// `dotp` (three device vectors of M/2 entries each, folded in place) with claims `dotp_claims`.
static int batched_prove(spg_ctx* ctx, const TreeSh& ts, size_t nc, size_t M, FqV claims,
                         const std::vector<Triple>& dotp, const FqV& dotp_claims, Tr& t, BatchedProofP* out,
                         FqV* rand_out, const Shard& sh) {
  static const bool fused = !getenv("SPG_LAYER_FUSED") || atoi(getenv("SPG_LAYER_FUSED")) != 0;
  if (fused || ts.W > 1) return batched_prove_fused(ctx, ts, nc, M, claims, dotp, dotp_claims, t, out, rand_out, sh);
  Fq* tree = ts.loc;
  hipStream_t s = ctx->stream;
  const size_t L = lg2(M), stride = 2 * M;
  auto off = [&](size_t k) { return 2 * M - 2 * (M >> k); };
  const size_t nt_max = nc + dotp.size();
  Fq* dC = (Fq*)ws_get(ctx, kWsC, (M / 2) * sizeof(Fq) + 64);
  Triple* dtr = (Triple*)ws_get(ctx, kWsTriples, nt_max * sizeof(Triple) + 64);
  Fq* dcoef = (Fq*)ws_get(ctx, kWsCoeff, nt_max * sizeof(Fq) + 64);
  Fq** dptr = (Fq**)ws_get(ctx, kWsFoldPtr, (2 * nc + 1 + 3 * dotp.size()) * sizeof(Fq*) + 64);
  Fq* part = (Fq*)ws_get(ctx, kWsPart, 3 * std::max<size_t>(2048, nt_max) * sizeof(Fq) + 64);
  Fq* dfin = (Fq*)ws_get(ctx, kWsFinals, 3 * nt_max * sizeof(Fq) + 64);
  if (!dC || !dtr || !dcoef || !dptr || !part || !dfin) return set_err(ctx, SPG_E_NOMEM, "batched_prove");
  FqV rand;
  Laps lp;
  lp.title = "ProductCircuitEvalProofBatched::prove";
  for (size_t layer = L; layer-- > 0;) {
    const size_t half = M >> (layer + 1);  // |left| = |right| = |C|
    const size_t rounds = lg2(half);
    int rc = eq_table(ctx, rand, dC);
    if (rc) return rc;
    const bool with_dotp = layer == 0 && !dotp.empty();
    std::vector<Triple> tr;
    std::vector<Fq*> fold;
    for (size_t c = 0; c < nc; c++) {
      Fq* v = tree + c * stride + off(layer);
      tr.push_back({v, v + half, dC});
      fold.push_back(v);
      fold.push_back(v + half);
    }
    fold.push_back(dC);
    if (with_dotp) {
      claims.insert(claims.end(), dotp_claims.begin(), dotp_claims.end());
      for (auto& d : dotp) {
        tr.push_back(d);
        fold.push_back(d.A);
        fold.push_back(d.B);
        fold.push_back(d.C);
      }
    }
    FqV coeffs = t.challenges("rand_coeffs_next_layer", claims.size());
    Fq e = fq_zero();
    for (size_t i = 0; i < claims.size(); i++) e = fq_add(e, fq_mul(claims[i], coeffs[i]));
    {  // descriptors up through page-locked staging (a pageable source blocks the host for a staging blit);
       // the staging is free again here: the previous layer ended with a synchronising download
      const size_t b1 = tr.size() * sizeof(Triple), b2 = coeffs.size() * sizeof(Fq), b3 = fold.size() * sizeof(Fq*);
      uint8_t* st = (uint8_t*)pinned_get(ctx, b1 + b2 + b3 + 64);
      if (!st) return set_err(ctx, SPG_E_NOMEM, "layer staging");
      memcpy(st, tr.data(), b1);
      memcpy(st + b1, coeffs.data(), b2);
      memcpy(st + b1 + b2, fold.data(), b3);
      SPG_HIP(ctx, hipMemcpyAsync(dtr, st, b1, hipMemcpyHostToDevice, s));
      SPG_HIP(ctx, hipMemcpyAsync(dcoef, st + b1, b2, hipMemcpyHostToDevice, s));
      SPG_HIP(ctx, hipMemcpyAsync(dptr, st + b1 + b2, b3, hipMemcpyHostToDevice, s));
    }
    lp.lap("layer_setup");
    LayerProofP lpf;
    FqV r_prod;
    size_t log_len = rounds;
    bool pending = false;  // a bound_poly_var_top with r_pend not yet launched
    Fq r_pend = fq_zero();
    static const bool tiny_ok = !getenv("SPG_SPARK_TINY") || atoi(getenv("SPG_SPARK_TINY")) != 0;
    static const size_t tiny_max = getenv("SPG_SPARK_TINY_MAX") ? (size_t)atoi(getenv("SPG_SPARK_TINY_MAX")) : 2048;
    for (size_t j = 0; j < rounds; j++) {
      log_len--;
      const size_t len = (size_t)1 << log_len;
      const unsigned nbx = (unsigned)std::min<size_t>(nblk(len), std::max<size_t>(1, 2048 / tr.size()));
      const bool tiny = tiny_ok && tr.size() * len <= tiny_max;
      if (pending && !tiny) {
        KScope ks(ctx, "spark_fold", 96.0 * fold.size() * (2 * len));
        hipLaunchKernelGGL(k_fold_many, dim3(nblk(fold.size() * 2 * len)), dim3(256), 0, s, dptr, fold.size(),
                           (int)log_len + 1, r_pend);
        pending = false;
      }
      if (tiny) {  // the pending fold and this round's evaluations in one workgroup
        KScope ks(ctx, "spark_layer_tiny", 192.0 * tr.size() * len + (pending ? 192.0 * fold.size() * len : 0.0));
        hipLaunchKernelGGL(k_layer_tiny, dim3(1), dim3(1024), 0, s, dtr, dcoef, (int)tr.size(), (int)log_len, dptr,
                           (int)fold.size(), pending ? 1 : 0, r_pend, ctx->d_mbox, ++ctx->mbox_seq);
        pending = false;
      } else {
        KScope ks(ctx, "spark_layer_eval", 192.0 * tr.size() * len);
        hipLaunchKernelGGL(k_layer_eval, dim3(nbx, (unsigned)tr.size()), dim3(256), 0, s, dtr, dcoef, len, part,
                           ctx->d_counter, ctx->d_mbox, ++ctx->mbox_seq);
      }
      Fq ev[3];
      rc = eval_reduce_finish(ctx, ev);
      if (rc) return rc;
      lp.lap("round_eval_wait");
      Fq evals[4] = {ev[0], fq_sub(e, ev[0]), ev[1], ev[2]};
      FqV poly = uni_from_evals3(evals);
      append_unipoly(t, poly);
      Fq r_j = t.challenge("challenge_nextround");
      r_prod.push_back(r_j);
      lp.lap("round_host");
      pending = true;  // bound_poly_var_top with r_j: launched with (or before) the next round's evaluation
      r_pend = r_j;
      SPG_HIP(ctx, hipGetLastError());
      e = uni_eval(poly, r_j);
      lpf.polys.push_back({poly[0], poly[2], poly[3]});
      lp.lap("round_fold_launch");
    }
    if (pending) {  // the last round's fold
      KScope ks(ctx, "spark_fold", 96.0 * fold.size());
      hipLaunchKernelGGL(k_fold_many, dim3(nblk(fold.size())), dim3(256), 0, s, dptr, fold.size(), 0, r_pend);
      pending = false;
    }
    // final claims: A[0], B[0] (and C[0] for the dot-product circuits)
    hipLaunchKernelGGL(k_finals, dim3(nblk(tr.size())), dim3(256), 0, s, dtr, tr.size(), dfin);
    FqV fin(3 * tr.size());
    rc = d2h_fq(ctx, dfin, fin.data(), fin.size());
    if (rc) return rc;
    for (size_t c = 0; c < nc; c++) {
      lpf.left.push_back(fin[3 * c]);
      lpf.right.push_back(fin[3 * c + 1]);
    }
    for (size_t c = 0; c < nc; c++) {
      t.scalar("claim_prod_left", lpf.left[c]);
      t.scalar("claim_prod_right", lpf.right[c]);
    }
    if (with_dotp) {
      for (size_t k = 0; k < dotp.size(); k++)
        for (int i = 0; i < 3; i++) out->dotp[i].push_back(fin[3 * (nc + k) + i]);
      for (size_t k = 0; k < dotp.size(); k++) {
        t.scalar("claim_dotp_left", out->dotp[0][k]);
        t.scalar("claim_dotp_right", out->dotp[1][k]);
        t.scalar("claim_dotp_weight", out->dotp[2][k]);
      }
    }
    Fq r_layer = t.challenge("challenge_r_layer");
    claims.assign(nc, fq_zero());
    for (size_t c = 0; c < nc; c++) claims[c] = fq_add(lpf.left[c], fq_mul(r_layer, fq_sub(lpf.right[c], lpf.left[c])));
    rand.assign(1, r_layer);
    rand.insert(rand.end(), r_prod.begin(), r_prod.end());
    out->layers.push_back(std::move(lpf));
    lp.lap("layer_finals");
  }
  lp.print();
  *rand_out = rand;
  return 0;
}

// n-to-1 reduction of claimed evaluations (sparse_mlpoly.rs:92-112, 868-883)
static void combine_evals(const FqV& evals, const FqV& r, const char* label, Tr& t, FqV* r_joint, Fq* eval) {
  FqV ch = t.challenges(label, lg2(evals.size()));
  FqV v = evals;
  for (size_t i = ch.size(); i-- > 0;) {  // bound_poly_var_bot with challenge i
    size_t n = v.size() / 2;
    for (size_t k = 0; k < n; k++) v[k] = fq_add(v[2 * k], fq_mul(ch[i], fq_sub(v[2 * k + 1], v[2 * k])));
    v.resize(n);
  }
  *eval = v[0];
  *r_joint = ch;
  r_joint->insert(r_joint->end(), r.begin(), r.end());
}

}  // namespace spg

// ------------------------------------------------------------------------------------ C-ABI
extern "C" int spg_spark_free(spg_ctx* ctx, spg_spark* S) {
  if (!S) return SPG_OK;
  hipFree(S->d_addr);
  hipFree(S->d_rts);
  hipFree(S->d_audit);
  hipFree(S->d_val);
  hipFree(S->d_comb_ops);
  hipFree(S->d_comb_mem);
  spg_gens_free(ctx, S->dev);
  delete S;
  return SPG_OK;
}

namespace spg {

// SparseMatPolynomial::multi_commit (sparse_mlpoly.rs:566-587) over `polys` (num_vars_x / num_vars_y of the
// matrices) with SparseMatPolyCommitmentGens::new(label, gens_nvx, gens_nvy, gens_nnz, gens_batch)
int spark_commit_polys(spg_ctx* ctx, const std::vector<SparsePoly>& polys, size_t nvx, size_t nvy,
                       const uint8_t* label, size_t label_len, size_t gens_nvx, size_t gens_nvy, size_t gens_nnz,
                       size_t gens_batch, spg_spark** out, const Shard& sh) {
  if (!ctx || polys.empty() || !label || !out) return SPG_E_ARG;
  hipStream_t s = ctx->stream;
  const size_t B = polys.size();
  size_t N = 2;
  for (auto& p : polys) N = std::max(N, npow2(p.nnz));
  const size_t cells = (size_t)1 << std::max<size_t>(std::max(nvx, nvy), 1);
  if (2 * B * N >= 0xffffffffULL || cells > 0xffffffffULL) return set_err(ctx, SPG_E_ARG, "SPARK batch too large");
  // SparseMatPolyCommitmentGens::new (sparse_mlpoly.rs:289-317)
  const size_t nv_ops = lg2(npow2(gens_nnz)) + lg2(npow2(gens_batch * 5));
  const size_t nv_mem = std::max(gens_nvx, gens_nvy) + 1;
  const size_t nv_der = lg2(npow2(gens_nnz)) + lg2(npow2(gens_batch * 2));
  const size_t ops_len = npow2(5 * B * N);
  if (lg2(ops_len) > nv_ops || lg2(npow2(2 * B * N)) > nv_der || std::max(nvx, nvy) + 1 > nv_mem)
    return set_err(ctx, SPG_E_ARG, "SPARK generators (gens_nnz, gens_batch) too small for the batch");
  // the dense representation's addresses (multi_sparse_to_dense_rep, sparse_mlpoly.rs:368-425); padding ops read
  // address 0
  std::vector<uint32_t> addr(2 * B * N, 0);
  std::vector<Fq> val(B * N, fq_zero());
  for (size_t k = 0; k < B; k++) {
    const spg_sparse_entry* E = polys[k].e;
    if (polys[k].nnz && !E) return SPG_E_ARG;
    for (size_t i = 0; i < polys[k].nnz; i++) {
      if (E[i].row >= ((uint64_t)1 << nvx) || E[i].col >= ((uint64_t)1 << nvy))
        return set_err(ctx, SPG_E_ARG, "sparse entry outside the matrix");
      addr[k * N + i] = (uint32_t)E[i].row;
      addr[B * N + k * N + i] = (uint32_t)E[i].col;
      memcpy(val[k * N + i].l, E[i].val, 32);
    }
  }
  spg_spark* S = new spg_spark();
  S->B = B;
  S->N = N;
  S->cells = cells;
  S->comb_ops_len = ops_len;
  S->comb_mem_len = 2 * cells;
  auto up = [&](void** d, const void* h, size_t bytes) -> bool {
    return hipMalloc(d, bytes + 64) == hipSuccess && hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up((void**)&S->d_addr, addr.data(), addr.size() * 4) || hipMalloc(&S->d_rts, addr.size() * 4 + 64) != hipSuccess ||
      hipMalloc(&S->d_audit, 2 * cells * 4 + 64) != hipSuccess ||
      !up((void**)&S->d_val, val.data(), val.size() * sizeof(Fq)) ||
      hipMalloc(&S->d_comb_ops, S->comb_ops_len * sizeof(Fq)) != hipSuccess ||
      hipMalloc(&S->d_comb_mem, S->comb_mem_len * sizeof(Fq)) != hipSuccess) {
    spg_spark_free(ctx, S);
    return set_err(ctx, SPG_E_NOMEM, "spark upload");
  }
  {  // AddrTimestamps::new (sparse_mlpoly.rs:219-253) for the row and the column side, on the device
    const size_t BN = B * N;
    int bits = 1;
    while (((size_t)1 << bits) < cells) bits++;
    uint32_t* tmpk = (uint32_t*)ws_get(ctx, kWsTsKeys, 3 * BN * 4 + 4 * (cells + 1) + 64);
    size_t sort_bytes = 0, scan_bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)BN, 0, bits, s);
    hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)cells, s);
    void* tmps = ws_get(ctx, kWsTsTemp, std::max(sort_bytes, scan_bytes) + 64);
    if (!tmpk || !tmps) {
      spg_spark_free(ctx, S);
      return set_err(ctx, SPG_E_NOMEM, "timestamps workspace");
    }
    uint32_t *keys = tmpk, *ops_in = tmpk + BN, *ops = tmpk + 2 * BN, *start = tmpk + 3 * BN;
    int rc2 = 0;
    for (size_t side = 0; side < 2 && !rc2; side++) {
      const uint32_t* ad = S->d_addr + side * BN;
      uint32_t* au = S->d_audit + side * cells;
      if (hipMemsetAsync(au, 0, cells * 4, s) != hipSuccess) rc2 = SPG_E_HIP;
      hipLaunchKernelGGL(k_ts_count, dim3(nblk(BN)), dim3(256), 0, s, ad, BN, au);
      if (hipcub::DeviceScan::ExclusiveSum(tmps, scan_bytes, au, start, (int)cells, s) != hipSuccess) rc2 = SPG_E_HIP;
      hipLaunchKernelGGL(k_iota, dim3(nblk(BN)), dim3(256), 0, s, ops_in, BN);
      if (hipcub::DeviceRadixSort::SortPairs(tmps, sort_bytes, ad, keys, ops_in, ops, (int)BN, 0, bits, s) != hipSuccess)
        rc2 = SPG_E_HIP;
      hipLaunchKernelGGL(k_ts_rank, dim3(nblk(BN)), dim3(256), 0, s, keys, ops, start, BN, S->d_rts + side * BN);
    }
    if (rc2 || hipGetLastError() != hipSuccess) {
      spg_spark_free(ctx, S);
      return set_err(ctx, SPG_E_HIP, "spark timestamps");
    }
  }
  // comb_ops = merge(row addr, row read_ts, col addr, col read_ts, val); comb_mem = row audit ++ col audit
  const size_t BN = B * N;
  int rc = 0;
  if (hipMemsetAsync(S->d_comb_ops, 0, S->comb_ops_len * sizeof(Fq), s) != hipSuccess) rc = SPG_E_HIP;
  hipLaunchKernelGGL(k_u32_to_fq, dim3(nblk(BN)), dim3(256), 0, s, S->d_addr, S->d_comb_ops, BN);
  hipLaunchKernelGGL(k_u32_to_fq, dim3(nblk(BN)), dim3(256), 0, s, S->d_rts, S->d_comb_ops + BN, BN);
  hipLaunchKernelGGL(k_u32_to_fq, dim3(nblk(BN)), dim3(256), 0, s, S->d_addr + BN, S->d_comb_ops + 2 * BN, BN);
  hipLaunchKernelGGL(k_u32_to_fq, dim3(nblk(BN)), dim3(256), 0, s, S->d_rts + BN, S->d_comb_ops + 3 * BN, BN);
  if (hipMemcpyAsync(S->d_comb_ops + 4 * BN, S->d_val, BN * sizeof(Fq), hipMemcpyDeviceToDevice, s) != hipSuccess)
    rc = SPG_E_HIP;
  hipLaunchKernelGGL(k_u32_to_fq, dim3(nblk(2 * cells)), dim3(256), 0, s, S->d_audit, S->d_comb_mem, 2 * cells);
  if (rc || hipGetLastError() != hipSuccess) {
    spg_spark_free(ctx, S);
    return set_err(ctx, SPG_E_HIP, "spark dense representation");
  }
  // the three PolyCommitmentGens share one label: prefixes of one derived stream
  size_t nmax = 0;
  for (size_t nv : {nv_ops, nv_mem, nv_der}) nmax = std::max(nmax, (size_t)1 << (nv - nv / 2));
  rc = spg_gens_derive(ctx, label, label_len, nmax + 1, &S->dev);
  if (rc) {
    spg_spark_free(ctx, S);
    return rc;
  }
  S->g_ops = gens_view(S->dev, nv_ops);
  S->g_mem = gens_view(S->dev, nv_mem);
  S->g_der = gens_view(S->dev, nv_der);
  std::vector<Pt> comm_ops, comm_mem;
  rc = commit_dev(ctx, S->g_ops, S->d_comb_ops, lg2(S->comb_ops_len), &comm_ops, sh);
  if (!rc) rc = commit_dev(ctx, S->g_mem, S->d_comb_mem, lg2(S->comb_mem_len), &comm_mem, sh);
  if (rc) {
    spg_spark_free(ctx, S);
    return rc;
  }
  S->comm_ops = comm_ops;
  S->comm_mem = comm_mem;
  *out = S;
  return SPG_OK;
}

int spark_from_comm(spg_ctx* ctx, size_t B, size_t N, size_t cells, const std::vector<Pt>& comm_ops,
                    const std::vector<Pt>& comm_mem, const uint8_t* label, size_t label_len, size_t gens_nvx,
                    size_t gens_nvy, size_t gens_nnz, size_t gens_batch, spg_spark** out) {
  const size_t nv_ops = lg2(npow2(gens_nnz)) + lg2(npow2(gens_batch * 5));
  const size_t nv_mem = std::max(gens_nvx, gens_nvy) + 1;
  const size_t nv_der = lg2(npow2(gens_nnz)) + lg2(npow2(gens_batch * 2));
  // the shapes multi_commit gives: N a power of two >= 2, cells a power of two, and one Hyrax row commitment per row
  // of comb_ops (npow2(5 B N) entries) and comb_mem (2 cells entries)
  if (!B || N < 2 || !is_pow2(N) || !cells || !is_pow2(cells) || B > (1u << 20) || N > (1ull << 32) ||
      cells > (1ull << 32) || lg2(npow2(5 * B * N)) > nv_ops || lg2(npow2(2 * B * N)) > nv_der || lg2(2 * cells) > nv_mem)
    return set_err(ctx, SPG_E_ARG, "SPARK commitment sizes do not fit the generators");
  const size_t ops_nv = lg2(npow2(5 * B * N)), mem_nv = lg2(2 * cells);
  if (comm_ops.size() != ((size_t)1 << (ops_nv / 2)) || comm_mem.size() != ((size_t)1 << (mem_nv / 2)))
    return set_err(ctx, SPG_E_ARG, "SPARK commitment row counts do not match its sizes");
  spg_spark* S = new spg_spark();
  S->B = B;
  S->N = N;
  S->cells = cells;
  S->comb_ops_len = npow2(5 * B * N);
  S->comb_mem_len = 2 * cells;
  size_t nmax = 0;
  for (size_t nv : {nv_ops, nv_mem, nv_der}) nmax = std::max(nmax, (size_t)1 << (nv - nv / 2));
  const int rc = spg_gens_derive(ctx, label, label_len, nmax + 1, &S->dev);
  if (rc) {
    delete S;
    return rc;
  }
  S->g_ops = gens_view(S->dev, nv_ops);
  S->g_mem = gens_view(S->dev, nv_mem);
  S->g_der = gens_view(S->dev, nv_der);
  S->comm_ops = comm_ops;
  S->comm_mem = comm_mem;
  *out = S;
  return SPG_OK;
}

// bincode(SparseMatPolyCommitment) (sparse_mlpoly.rs:319-325)
void spark_comm_ser(const spg_spark* S, Writer& w) {
  w.u64(S->B);
  w.u64(S->N);
  w.u64(S->cells);
  w.pts(S->comm_ops);
  w.pts(S->comm_mem);
}
// SparseMatPolyCommitment::append_to_transcript (sparse_mlpoly.rs:327-339)
void spark_comm_append(const spg_spark* S, Tr& t) {
  t.u64("batch_size", S->B);
  t.u64("num_ops", S->N);
  t.u64("num_mem_cells", S->cells);
  append_polycomm(t, "comm_comb_ops", S->comm_ops);
  append_polycomm(t, "comm_comb_mem", S->comm_mem);
}

}  // namespace spg

extern "C" int spg_spark_commit(spg_ctx* ctx, const spg_r1cs_instance* ci, const uint8_t* label, size_t label_len,
                                size_t gens_nnz, size_t gens_batch, spg_spark** out, uint8_t* comm, size_t comm_cap,
                                size_t* comm_len) {
  if (!ctx || !ci || !label || !out || !comm_len || !ci->num_instances || !ci->nnz || !ci->entries) return SPG_E_ARG;
  if (!is_pow2(ci->max_num_cons) || !is_pow2(ci->num_vars)) return set_err(ctx, SPG_E_ARG, "sizes must be powers of 2");
  std::vector<SparsePoly> polys;
  for (size_t k = 0; k < 3 * ci->num_instances; k++) polys.push_back({ci->entries[k], ci->nnz[k]});
  const size_t nvx = lg2(ci->max_num_cons), nvy = lg2(ci->num_vars);
  spg_spark* S = nullptr;
  int rc = spark_commit_polys(ctx, polys, nvx, nvy, label, label_len, nvx, nvy, gens_nnz, gens_batch, &S,
                              ctx_shard(ctx));
  if (rc) return rc;
  Writer w;
  spark_comm_ser(S, w);
  *comm_len = w.out.size();
  *out = S;
  if (!comm || w.out.size() > comm_cap) return set_err(ctx, SPG_E_ARG, "commitment buffer too small");
  memcpy(comm, w.out.data(), w.out.size());
  return SPG_OK;
}

namespace spg {

// SparseMatPolyEvalProof::prove (sparse_mlpoly.rs:1497-1564); appends bincode(proof) to w.
//
// Sharded proof (sh.n = W > 1 processes, one GPU each; SURVEY 8e "SPARK product trees: shard by the low index
// bits"): every rank holds the whole dense representation and runs the same transcript. The O(N) work splits:
//   derefs commitment  Hyrax rows split over the ranks, 32-byte rows allgathered (commit_rows_sh)
//   hash layer, trees  rank r hashes leaves i = W i' + r of each circuit of >= 2W leaves and builds its local
//                      product tree; ProductCircuit::compute_layer pairs i with i + len/2, which keeps the low
//                      lg W bits, so every level stays local down to one entry per rank; those W entries are
//                      allgathered and the top lg W levels built on every rank (TreeSh)
//   layer sumchecks    batched_prove_fused: local rounds with (e0, e2, e3) summed over the ranks, then a gather
//   hash-layer evals   contiguous shares of each dot product, summed (seg_dots)
//   PolyEvalProofs     L.Z rows split, partial vectors summed; Bullet replicated (poly_eval_prove)
// A circuit set of fewer than 2W leaves (or W not a power of two) stays whole on every rank. Every collective
// carries the rank's status.
int spark_prove_core(spg_ctx* ctx, spg_spark* S, FqV ex, FqV ey, const FqV& evals, Tr& t, Tape& tape, Writer& w,
                     const Shard& sh) {
  if (evals.size() != S->B) return set_err(ctx, SPG_E_ARG, "one evaluation per batched matrix");
  Laps lp;
  lp.title = "SparseMatPolyEvalProof::prove";
  hipStream_t s = ctx->stream;
  const size_t B = S->B, N = S->N, BN = B * N, cells = S->cells, hN = N / 2;
  if (ex.size() < ey.size()) ex.insert(ex.begin(), ey.size() - ex.size(), fq_zero());
  if (ey.size() < ex.size()) ey.insert(ey.begin(), ex.size() - ey.size(), fq_zero());
  if (ex.size() > 40 || ((size_t)1 << ex.size()) != cells)
    return set_err(ctx, SPG_E_ARG, "rx / ry do not match the memory size");
  // interleaved shards of the two circuit sets (W = 1: whole)
  const size_t Wr = (size_t)sh.n;
  TreeSh tso, tsm;
  const bool pow2 = Wr > 1 && (Wr & (Wr - 1)) == 0;  // interleaving needs W | M (other world sizes: whole trees)
  tso.W = (pow2 && N >= 2 * Wr) ? (int)Wr : 1;
  tsm.W = (pow2 && cells >= 2 * Wr) ? (int)Wr : 1;
  tso.r = tso.W > 1 ? sh.rank : 0;
  tsm.r = tsm.W > 1 ? sh.rank : 0;
  tso.m = N / tso.W;
  tsm.m = cells / tsm.W;
  const size_t mo = tso.m, mm = tsm.m, hNl = hN / tso.W;
  t.protocol("Sparse polynomial evaluation proof");
  timer_start(ctx);
  const size_t der_len = npow2(2 * BN);
  Fq* mem_rx = (Fq*)ws_get(ctx, kWsMemRx, cells * sizeof(Fq) + 64);
  Fq* mem_ry = (Fq*)ws_get(ctx, kWsMemRy, cells * sizeof(Fq) + 64);
  Fq* derefs = (Fq*)ws_get(ctx, kWsDerefs, der_len * sizeof(Fq) + 64);
  tso.loc = (Fq*)ws_get(ctx, kWsTreeOps, 4 * B * 2 * mo * sizeof(Fq) + 64);
  tsm.loc = (Fq*)ws_get(ctx, kWsTreeMem, 4 * 2 * mm * sizeof(Fq) + 64);
  tso.top = tso.W > 1 ? (Fq*)ws_get(ctx, kWsTopOps, 4 * B * 2 * Wr * sizeof(Fq) + 64) : nullptr;
  tsm.top = tsm.W > 1 ? (Fq*)ws_get(ctx, kWsTopMem, 4 * 2 * Wr * sizeof(Fq) + 64) : nullptr;
  Fq* dotbuf = (Fq*)ws_get(ctx, kWsDotp, 2 * B * 3 * hNl * sizeof(Fq) + 64);
  Fq* dtops = (Fq*)ws_get(ctx, kWsTops, 4 * (B + 1) * sizeof(Fq) + 64);
  Fq* eq_ops = (Fq*)ws_get(ctx, kWsEqOps, N * sizeof(Fq) + 64);
  Fq* eq_mem = (Fq*)ws_get(ctx, kWsEqMem, cells * sizeof(Fq) + 64);
  int rc = 0;
  if (!mem_rx || !mem_ry || !derefs || !tso.loc || !tsm.loc || (tso.W > 1 && !tso.top) || (tsm.W > 1 && !tsm.top) ||
      !dotbuf || !dtops || !eq_ops || !eq_mem)
    rc = set_err(ctx, SPG_E_NOMEM, "spark workspace");
  if (sh.n > 1) {  // every rank enters the proof's collectives only if every rank has its workspace
    std::vector<uint8_t> none;
    rc = comm_allgather(ctx, sh, rc, nullptr, 0, none);
  }
  if (rc) return rc;
  rc = eq_tables(ctx, {{ex, mem_rx}, {ey, mem_ry}});
  if (rc) return rc;
  // Derefs (sparse_mlpoly.rs:51-67): comb = row derefs ++ col derefs, zero-padded
  if (der_len > 2 * BN) SPG_HIP(ctx, hipMemsetAsync(derefs + 2 * BN, 0, (der_len - 2 * BN) * sizeof(Fq), s));
  {
    KScope ks(ctx, "spark_deref", (4.0 + 32.0 + 32.0) * 2 * BN);
    hipLaunchKernelGGL(k_gather, dim3(nblk(2 * BN)), dim3(256), 0, s, S->d_addr, mem_rx, mem_ry, BN, derefs);
  }
  SPG_HIP(ctx, hipGetLastError());
  lp.lap("setup+deref");
  std::vector<Pt> comm_derefs;
  rc = commit_dev(ctx, S->g_der, derefs, lg2(der_len), &comm_derefs, sh);
  lp.lap("derefs_commit");
  if (rc) return rc;
  t.msg("derefs_commitment", "begin_derefs_commitment");
  append_polycomm(t, "comm_poly_row_col_ops_val", comm_derefs);
  t.msg("derefs_commitment", "end_derefs_commitment");
  FqV rmc = t.challenges("challenge_r_hash", 2);
  const Fq rh = rmc[0], rh2 = fq_mul(rmc[0], rmc[0]), rms = rmc[1];
  // hash layer leaves straight into the (local) trees, then the product trees (Layers::new)
  {
    KScope ks(ctx, "spark_hash_layer", (8.0 + 32.0 + 64.0) * 2 * B * mo + (4.0 + 32.0 + 64.0) * 2 * mm);
    hipLaunchKernelGGL(k_hash_ops, dim3(nblk(2 * B * mo)), dim3(256), 0, s, S->d_addr, S->d_rts, derefs, B, (int)lg2(N),
                       (int)lg2(mo), (uint32_t)tso.W, (uint32_t)tso.r, rh, rh2, rms, tso.loc);
    hipLaunchKernelGGL(k_hash_mem, dim3(nblk(2 * mm)), dim3(256), 0, s, S->d_audit, mem_rx, mem_ry, (int)lg2(cells),
                       (int)lg2(mm), (uint32_t)tsm.W, (uint32_t)tsm.r, rh, rh2, rms, tsm.loc);
  }
  for (int which = 0; which < 2; which++) {  // ProductCircuit::new (product_tree.rs:36-58), local trees
    Fq* tree = which ? tsm.loc : tso.loc;
    const size_t M = which ? mm : mo, nc = which ? 4 : 4 * B;
    KScope ks(ctx, "spark_product_tree", 96.0 * nc * M / 2);
    // levels of more than kTopHalf products per circuit: one grid-wide launch each; the rest and the tops: k_tree_top
    static const size_t kTopHalf = getenv("SPG_TREE_TOP") ? (size_t)atol(getenv("SPG_TREE_TOP")) : 1024;
    size_t k = 0;
    for (; k + 1 < lg2(M) && (M >> (k + 1)) > kTopHalf; k++) {
      size_t ok = 2 * M - 2 * (M >> k), ok1 = 2 * M - 2 * (M >> (k + 1));
      hipLaunchKernelGGL(k_tree_level, dim3(nblk(nc * (M >> (k + 1)))), dim3(256), 0, s, tree, nc, 2 * M, ok, ok1,
                         (int)lg2(M >> (k + 1)));
    }
    if (kTopHalf) {
      hipLaunchKernelGGL(k_tree_top, dim3((unsigned)nc), dim3(256), 0, s, tree, 2 * M, (int)lg2(M), (int)k,
                         dtops + (which ? 4 * B : 0));
    } else {
      for (; k + 1 < lg2(M); k++) {
        size_t ok = 2 * M - 2 * (M >> k), ok1 = 2 * M - 2 * (M >> (k + 1));
        hipLaunchKernelGGL(k_tree_level, dim3(nblk(nc * (M >> (k + 1)))), dim3(256), 0, s, tree, nc, 2 * M, ok, ok1,
                           (int)lg2(M >> (k + 1)));
      }
      const size_t top = 2 * M - 4;  // v_{L-1}
      hipLaunchKernelGGL(k_tops, dim3(nblk(nc)), dim3(256), 0, s, tree, nc, 2 * M, top, dtops + (which ? 4 * B : 0));
    }
  }
  SPG_HIP(ctx, hipGetLastError());
  FqV tops(4 * B + 4);
  rc = d2h_fq(ctx, dtops, tops.data(), tops.size());
  if (tso.W > 1 || tsm.W > 1) {
    // sharded sets: the product of a local tree is the rank's entry of the global level with W entries; gather
    // them, build the top lg W levels (ProductCircuit::compute_layer) on every rank, and the circuits' claims
    std::vector<uint8_t> all;
    rc = comm_allgather(ctx, sh, rc, tops.data(), tops.size() * sizeof(Fq), all);
    if (rc) return rc;
    const Fq* g = (const Fq*)all.data();
    for (int which = 0; which < 2; which++) {
      const TreeSh& ts = which ? tsm : tso;
      if (ts.W == 1) continue;
      const size_t nc = which ? 4 : 4 * B, base = which ? 4 * B : 0;
      std::vector<Fq> ht(nc * 2 * Wr, fq_zero());
      for (size_t c = 0; c < nc; c++) {
        Fq* v = ht.data() + c * 2 * Wr;
        for (size_t q = 0; q < Wr; q++) v[q] = g[q * tops.size() + base + c];
        size_t o = 0;
        for (size_t len = Wr; len > 2; len /= 2) {
          for (size_t i = 0; i < len / 2; i++) v[o + len + i] = fq_mul(v[o + i], v[o + i + len / 2]);
          o += len;
        }
        tops[base + c] = fq_mul(v[o], v[o + 1]);
      }
      SPG_HIP(ctx, hipMemcpyAsync(ts.top, ht.data(), ht.size() * sizeof(Fq), hipMemcpyHostToDevice, s));
    }
    SPG_HIP(ctx, hipStreamSynchronize(s));  // ht is a host temporary
  }
  lp.lap("hash+trees");
  if (rc) return rc;
  // ---- PolyEvalNetworkProof -> ProductLayerProof (sparse_mlpoly.rs:1368-1402, 1118-1263)
  t.protocol("Sparse polynomial evaluation proof");
  t.protocol("Sparse polynomial product layer proof");
  const Fq row_init = tops[4 * B], row_audit = tops[4 * B + 1], col_init = tops[4 * B + 2], col_audit = tops[4 * B + 3];
  FqV row_read(tops.begin(), tops.begin() + B), row_write(tops.begin() + B, tops.begin() + 2 * B),
      col_read(tops.begin() + 2 * B, tops.begin() + 3 * B), col_write(tops.begin() + 3 * B, tops.begin() + 4 * B);
  t.scalar("claim_row_eval_init", row_init);
  t.scalars("claim_row_eval_read", row_read);
  t.scalars("claim_row_eval_write", row_write);
  t.scalar("claim_row_eval_audit", row_audit);
  t.scalar("claim_col_eval_init", col_init);
  t.scalars("claim_col_eval_read", col_read);
  t.scalars("claim_col_eval_write", col_write);
  t.scalar("claim_col_eval_audit", col_audit);
  // dot-product circuits (row derefs, col derefs, val) split into halves, interleaved (left_b, right_b);
  // copies (this rank's interleaved shares when the ops set is sharded), since the layer-0 sumcheck folds them
  // while the hash layer evaluates the originals
  std::vector<Triple> dotp;
  for (size_t j = 0; j < 2 * B; j++) {
    Fq* base = dotbuf + j * 3 * hNl;
    dotp.push_back({base, base + hNl, base + 2 * hNl});
  }
  hipLaunchKernelGGL(k_dotp_gather, dim3(nblk(hNl), (unsigned)(6 * B)), dim3(256), 0, s, dotbuf, derefs, S->d_val,
                     BN, N, hN, hNl, (uint32_t)tso.W, (uint32_t)tso.r);
  SPG_HIP(ctx, hipGetLastError());
  FqV dotp_claims(2 * B);
  {
    Triple* dtr = (Triple*)ws_get(ctx, kWsTriples, 6 * B * sizeof(Triple) + 64);
    unsigned nb = (unsigned)std::min<size_t>(nblk(hNl), std::max<size_t>(1, 2048 / (2 * B)));
    Fq* part = (Fq*)ws_get(ctx, kWsSegPart, 2 * B * nb * sizeof(Fq) + 64);
    Fq* dres = (Fq*)ws_get(ctx, kWsSeg, 2 * B * sizeof(Fq) + 64);
    if (!dtr || !part || !dres) rc = set_err(ctx, SPG_E_NOMEM, "dotp eval");
    if (!rc) {
      SPG_HIP(ctx, hipMemcpyAsync(dtr, dotp.data(), dotp.size() * sizeof(Triple), hipMemcpyHostToDevice, s));
      KScope ks(ctx, "spark_dotp_eval", 96.0 * 2 * B * hNl);
      hipLaunchKernelGGL(k_dot3, dim3(nb, (unsigned)(2 * B)), dim3(256), 0, s, dtr, hNl, part);
      hipLaunchKernelGGL(k_sum_seg, dim3((unsigned)(2 * B)), dim3(256), 0, s, part, (int)nb, dres);
      SPG_HIP(ctx, hipGetLastError());
      rc = d2h_fq(ctx, dres, dotp_claims.data(), 2 * B);
    }
    if (tso.W > 1) rc = comm_sum_fq(ctx, sh, rc, dotp_claims.data(), 2 * B);
    if (rc) return rc;
  }
  FqV dl(B), dr(B);
  for (size_t b = 0; b < B; b++) {
    dl[b] = dotp_claims[2 * b];
    dr[b] = dotp_claims[2 * b + 1];
    t.scalar("claim_eval_dotp_left", dl[b]);
    t.scalar("claim_eval_dotp_right", dr[b]);
  }
  lp.lap("dotp_claims");
  BatchedProofP proof_ops, proof_mem;
  FqV rand_ops, rand_mem;
  rc = batched_prove(ctx, tso, 4 * B, N, FqV(tops.begin(), tops.begin() + 4 * B), dotp, dotp_claims, t, &proof_ops,
                     &rand_ops, sh);
  if (!rc)
    rc = batched_prove(ctx, tsm, 4, cells, FqV(tops.begin() + 4 * B, tops.end()), {}, {}, t, &proof_mem, &rand_mem, sh);
  if (rc) return rc;
  lp.lap("layer_sumchecks");
  // ---- HashLayerProof (sparse_mlpoly.rs:805-918)
  t.protocol("Sparse polynomial hash layer proof");
  rc = eq_tables(ctx, {{rand_ops, eq_ops}, {rand_mem, eq_mem}});
  if (rc) return rc;
  FqV ev_der, ev_ops, ev_mem;
  rc = seg_dots_multi(ctx, {{derefs, N, 2 * B, eq_ops, N, &ev_der}, {S->d_comb_ops, N, 5 * B, eq_ops, N, &ev_ops},
                            {S->d_comb_mem, cells, 2, eq_mem, cells, &ev_mem}}, sh);
  if (rc) return rc;
  lp.lap("hash_evals");
  DotProductProofLogP pf_der, pf_ops, pf_mem;
  {  // DerefsEvalProof::prove (sparse_mlpoly.rs:80-146)
    t.protocol("Derefs evaluation proof");
    FqV ev = ev_der;
    ev.resize(npow2(ev.size()), fq_zero());
    t.scalars("evals_ops_val", ev);
    FqV rj;
    Fq ej;
    combine_evals(ev, rand_ops, "challenge_combine_n_to_one", t, &rj, &ej);
    t.scalar("joint_claim_eval", ej);
    rc = poly_eval_prove(ctx, S->g_der, derefs, rj, ej, t, tape, &pf_der, sh);
    if (rc) return rc;
  }
  {
    FqV ev = ev_ops;
    ev.resize(npow2(ev.size()), fq_zero());
    t.scalars("claim_evals_ops", ev);
    FqV rj;
    Fq ej;
    combine_evals(ev, rand_ops, "challenge_combine_n_to_one", t, &rj, &ej);
    t.scalar("joint_claim_eval_ops", ej);
    rc = poly_eval_prove(ctx, S->g_ops, S->d_comb_ops, rj, ej, t, tape, &pf_ops, sh);
    if (rc) return rc;
  }
  {
    t.scalars("claim_evals_mem", ev_mem);
    FqV rj;
    Fq ej;
    combine_evals(ev_mem, rand_mem, "challenge_combine_two_to_one", t, &rj, &ej);
    t.scalar("joint_claim_eval_mem", ej);
    rc = poly_eval_prove(ctx, S->g_mem, S->d_comb_mem, rj, ej, t, tape, &pf_mem, sh);
    if (rc) return rc;
  }
  lp.lap("poly_eval_proofs");
  lp.print();
  timer_stop(ctx);
  // ---- bincode(SparseMatPolyEvalProof)
  w.pts(comm_derefs);
  w.fq(row_init);  // ProductLayerProof
  w.fqs(row_read);
  w.fqs(row_write);
  w.fq(row_audit);
  w.fq(col_init);
  w.fqs(col_read);
  w.fqs(col_write);
  w.fq(col_audit);
  w.fqs(dl);
  w.fqs(dr);
  proof_mem.ser(w);
  proof_ops.ser(w);
  auto seg = [&](size_t k) { return FqV(ev_ops.begin() + k * B, ev_ops.begin() + (k + 1) * B); };
  w.fqs(seg(0));  // HashLayerProof: row addr, row read_ts, row audit, col ..., val, derefs, proofs
  w.fqs(seg(1));
  w.fq(ev_mem[0]);
  w.fqs(seg(2));
  w.fqs(seg(3));
  w.fq(ev_mem[1]);
  w.fqs(seg(4));
  w.fqs(FqV(ev_der.begin(), ev_der.begin() + B));
  w.fqs(FqV(ev_der.begin() + B, ev_der.end()));
  pf_ops.ser(w);
  pf_mem.ser(w);
  pf_der.ser(w);
  float ms = 0.f;
  hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  ctx->last_us = ms * 1000.0;
  return SPG_OK;
}

}  // namespace spg

static int spg_spark_prove_impl(spg_ctx* ctx, spg_spark* S, const uint64_t* rx, size_t rx_len, const uint64_t* ry,
                               size_t ry_len, const uint64_t* evals_in, size_t n_evals, spg_transcript* transcript,
                               spg_random_tape* tape_h, uint8_t* proof, size_t proof_cap, size_t* proof_len) {
  if (!ctx || !S || !transcript || !tape_h || !proof_len || (!rx && rx_len) || (!ry && ry_len) || !evals_in)
    return SPG_E_ARG;
  FqV ex, ey, evals(n_evals);
  for (size_t i = 0; i < rx_len; i++) ex.push_back(ld_fq(rx + 4 * i));
  for (size_t i = 0; i < ry_len; i++) ey.push_back(ld_fq(ry + 4 * i));
  for (size_t i = 0; i < n_evals; i++) evals[i] = ld_fq(evals_in + 4 * i);
  Writer w;
  int rc = spark_prove_core(ctx, S, ex, ey, evals, transcript->t, tape_h->t, w, ctx_shard(ctx));
  if (rc) return rc;
  *proof_len = w.out.size();
  if (!proof || w.out.size() > proof_cap) return set_err(ctx, SPG_E_ARG, "proof buffer too small");
  memcpy(proof, w.out.data(), w.out.size());
  return SPG_OK;
}

extern "C" int spg_spark_prove(spg_ctx* ctx, spg_spark* S, const uint64_t* rx, size_t rx_len, const uint64_t* ry,
                               size_t ry_len, const uint64_t* evals_in, size_t n_evals, spg_transcript* transcript,
                               spg_random_tape* tape_h, uint8_t* proof, size_t proof_cap, size_t* proof_len) {
  if (!ctx || !transcript) return SPG_E_ARG;
  spg::HostPin pin;
  spg::TrFailScope tfs(ctx, transcript->t);
  return spg::tr_status(ctx, transcript->t, spg_spark_prove_impl(ctx, S, rx, rx_len, ry, ry_len, evals_in, n_evals, transcript, tape_h, proof, proof_cap, proof_len));
}
