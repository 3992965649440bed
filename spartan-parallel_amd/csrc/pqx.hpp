// spg — device-resident ragged (p, q_rev, w, x_rev) tables: the HBM layout behind the reference's
// DensePolynomialPqx (src/custom_dense_mlpoly.rs:22-359).
//
// Layout: one flat Fq array; instance p owns alloc_np[p] x alloc_nw[p] x alloc_ni[p] elements at
// off[p], row-major in (q, w, x). The *allocation* never shrinks (as the reference's Vec<Vec<..>>),
// folding only rewrites the low halves and shrinks the *current* sizes np/ni/nws, so index()/
// index_high() keep the reference's bounds semantics exactly (custom_dense_mlpoly.rs:118-173).
#pragma once
#include <vector>

#include "field.hpp"

namespace spg {

static const int kMaxP = 32;  // instances whose descriptors ride in the kernel arguments (two PqxArgs stay under
                              // the 4 KiB kernarg budget); more go to device memory (PqxArgs::ext)

// per-instance view passed by value to kernels
struct PqxInst {
  uint32_t off_lo, off_hi;   // element offset (64-bit split)
  uint32_t anp, anw, ani;    // allocation sizes
  uint32_t np, ni;           // current sizes (Pqx.num_proofs[p], Pqx.num_inputs[p])
  uint32_t dom_off;          // offset of this instance in a kernel's flattened domain
  uint32_t sc_np, sc_ni;     // sumcheck-local sizes for the round (already halved)
  uint32_t step_q, step_x;   // proof_len / sc_np, cons_len / sc_ni (phase 1)
  uint32_t fstride;          // fused fold + eval: element stride to the pending fold's partner (0: scale by 1 - r)
};

struct PqxArgs {
  int P;          // instances in the kernel domain
  int zlen;       // Z.len()
  int ninst;      // Pqx.num_instances (current, power of two)
  int nws;        // Pqx.num_witness_secs (current, power of two)
  const PqxInst* ext;  // more than kMaxP instances: every descriptor in device memory (else null, `in` holds them)
  PqxInst in[kMaxP];
};
// descriptor of instance p (kernel argument or device copy)
__host__ __device__ inline const PqxInst& pinst(const PqxArgs& a, int p) { return a.ext ? a.ext[p] : a.in[p]; }

__host__ __device__ inline size_t pqx_off(const PqxInst& d) { return ((size_t)d.off_hi << 32) | d.off_lo; }

struct PqxDev {
  Fq* d = nullptr;
  size_t total = 0;
  size_t zlen = 0;
  std::vector<size_t> off, anp, anw, ani;
  // current Pqx fields
  size_t num_instances = 0, max_num_proofs = 0, num_witness_secs = 0, max_num_inputs = 0;
  std::vector<size_t> num_proofs, num_inputs;

  size_t at(size_t p, size_t q, size_t w, size_t x) const { return off[p] + (q * anw[p] + w) * ani[p] + x; }
};

}  // namespace spg

// the C-ABI handle of a resident DensePolynomialPqx (seams.hip; spg_r1cs_multiply_vec_block in r1cs.hip makes them too)
struct spg_pqx {
  spg::PqxDev T;
};
