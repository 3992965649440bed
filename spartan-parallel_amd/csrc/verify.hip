// spg — SNARK::verify (src/lib.rs:2750-3881) over the proof bytes spg_snark_prove writes: the transcript is
// replayed from the public inputs, the instance commitments and the proof, and every check of the reference's
// verifier runs. Group work: the sigma-protocol checks on host cores (fixed-base tables of the few gens_1 / gens_4
// points, hcurve.hpp), variable-base MSMs over proof points (Hyrax row commitments, Bullet L/R) by a host
// Pippenger on the pool, and the Bullet generator folds sum_i s_i G_i as fixed-base MSMs on the GPU against the
// resident generator tables (device_msm_idx).
//
//   KnowledgeProof / EqualityProof / ProductProof / DotProductProof::verify   src/nizk/mod.rs:50-404
//   BulletReductionProof::verify, DotProductProofLog::verify                  src/nizk/bullet.rs:138-232, mod.rs:525-570
//   ZKSumcheckInstanceProof::verify, SumcheckInstanceProof::verify            src/sumcheck.rs:37-189
//   PolyEvalProof::verify*                                                    src/dense_mlpoly.rs:492-1205
//   R1CSProof::verify                                                         src/r1csproof.rs:687-954
//   ProductCircuitEvalProofBatched::verify                                    src/product_tree.rs:398-487
//   SparseMatPolyEvalProof::verify (+ product / hash layer)                   src/sparse_mlpoly.rs:920-1610
//   SNARK::verify                                                             src/lib.rs:2750-3881
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "hostpoly.hpp"
#include "proto.hpp"

using namespace spg;
using h::HExt;


namespace {

// ---------------------------------------------------------------- proof bytes
struct Rd {
  const uint8_t* p;
  size_t n, o = 0;
  bool bad = false;
  Rd(const uint8_t* b, size_t len) : p(b), n(len) {}
  bool take(size_t k) {
    if (bad || o + k > n) {
      bad = true;
      return false;
    }
    return true;
  }
  uint64_t u64() {
    if (!take(8)) return 0;
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)p[o + i] << (8 * i);
    o += 8;
    return v;
  }
  size_t len(size_t elem) {  // a Vec length, bounded by the bytes left
    uint64_t v = u64();
    if (bad || (elem && v > (n - o) / elem)) {
      bad = true;
      return 0;
    }
    return (size_t)v;
  }
  Fq fq() {  // Scalar: four u64 Montgomery limbs; limbs >= q are rejected as malformed
    Fq a = fq_zero();
    if (!take(32)) return a;
    for (int i = 0; i < 8; i++)
      a.l[i] = (uint32_t)p[o + 4 * i] | ((uint32_t)p[o + 4 * i + 1] << 8) | ((uint32_t)p[o + 4 * i + 2] << 16) |
               ((uint32_t)p[o + 4 * i + 3] << 24);
    o += 32;
    const uint32_t Q[8] = {SPG_Q0, SPG_Q1, SPG_Q2, SPG_Q3, 0u, 0u, 0u, SPG_Q7};
    uint32_t b = 0;
    for (int i = 0; i < 8; i++) subb(a.l[i], Q[i], b, b);
    if (!b) bad = true;  // a >= q
    return a;
  }
  Pt pt() {
    Pt c;
    memset(c.b, 0, 32);
    if (!take(32)) return c;
    memcpy(c.b, p + o, 32);
    o += 32;
    return c;
  }
  FqV fqs() {
    size_t k = len(32);
    FqV v(k);
    for (auto& a : v) a = fq();
    return v;
  }
  std::vector<Pt> pts() {
    size_t k = len(32);
    std::vector<Pt> v(k);
    for (auto& a : v) a = pt();
    return v;
  }
};

void rd(Rd& r, KnowledgeProofP& p) { p.alpha = r.pt(); p.z1 = r.fq(); p.z2 = r.fq(); }
void rd(Rd& r, EqualityProofP& p) { p.alpha = r.pt(); p.z = r.fq(); }
void rd(Rd& r, ProductProofP& p) {
  p.alpha = r.pt(); p.beta = r.pt(); p.delta = r.pt();
  for (int i = 0; i < 5; i++) p.z[i] = r.fq();
}
void rd(Rd& r, DotProductProofP& p) { p.delta = r.pt(); p.beta = r.pt(); p.z = r.fqs(); p.z_delta = r.fq(); p.z_beta = r.fq(); }
void rd(Rd& r, DotProductProofLogP& p) { p.L = r.pts(); p.R = r.pts(); p.delta = r.pt(); p.beta = r.pt(); p.z1 = r.fq(); p.z2 = r.fq(); }
void rd(Rd& r, ZKSumcheckP& p) {
  p.comm_polys = r.pts();
  p.comm_evals = r.pts();
  p.proofs.resize(r.len(96));
  for (auto& d : p.proofs) rd(r, d);
}
void rd(Rd& r, R1CSProofP& p) {
  rd(r, p.sc1);
  for (int i = 0; i < 4; i++) p.claims_phase2[i] = r.pt();
  rd(r, p.pok);
  rd(r, p.prod);
  rd(r, p.eq1);
  rd(r, p.sc2);
  p.comm_vars_at_ry_list.resize(r.len(8));
  for (auto& v : p.comm_vars_at_ry_list) v = r.pts();
  p.comm_vars_at_ry = r.pt();
  p.evals.resize(r.len(16));
  for (auto& e : p.evals) rd(r, e);
  rd(r, p.eq2);
}
void rd(Rd& r, std::vector<DotProductProofLogP>& v) {
  v.resize(r.len(16));
  for (auto& e : v) rd(r, e);
}

struct LayerV {
  std::vector<FqV> polys;
  FqV left, right;
};
struct BatchedV {  // ProductCircuitEvalProofBatched (src/product_tree.rs:262-269)
  std::vector<LayerV> layers;
  FqV dotp[3];
};
void rd(Rd& r, BatchedV& b) {
  b.layers.resize(r.len(24));
  for (auto& l : b.layers) {
    l.polys.resize(r.len(8));
    for (auto& p : l.polys) p = r.fqs();
    l.left = r.fqs();
    l.right = r.fqs();
  }
  for (int i = 0; i < 3; i++) b.dotp[i] = r.fqs();
}
struct SparkV {  // SparseMatPolyEvalProof (src/sparse_mlpoly.rs:1469-1475), fields in bincode order
  std::vector<Pt> comm_derefs;
  Fq row_init, row_audit, col_init, col_audit;
  FqV row_read, row_write, col_read, col_write, dotp_left, dotp_right;
  BatchedV proof_mem, proof_ops;
  FqV eval_row_addr, eval_row_read_ts, eval_col_addr, eval_col_read_ts, eval_val, eval_row_ops_val, eval_col_ops_val;
  Fq eval_row_audit_ts, eval_col_audit_ts;
  DotProductProofLogP pe_ops, pe_mem, pe_derefs;
};
void rd(Rd& r, SparkV& s) {
  s.comm_derefs = r.pts();
  s.row_init = r.fq(); s.row_read = r.fqs(); s.row_write = r.fqs(); s.row_audit = r.fq();
  s.col_init = r.fq(); s.col_read = r.fqs(); s.col_write = r.fqs(); s.col_audit = r.fq();
  s.dotp_left = r.fqs();
  s.dotp_right = r.fqs();
  rd(r, s.proof_mem);
  rd(r, s.proof_ops);
  s.eval_row_addr = r.fqs(); s.eval_row_read_ts = r.fqs(); s.eval_row_audit_ts = r.fq();
  s.eval_col_addr = r.fqs(); s.eval_col_read_ts = r.fqs(); s.eval_col_audit_ts = r.fq();
  s.eval_val = r.fqs();
  s.eval_row_ops_val = r.fqs();
  s.eval_col_ops_val = r.fqs();
  rd(r, s.pe_ops);
  rd(r, s.pe_mem);
  rd(r, s.pe_derefs);
}
typedef std::vector<Pt> PolyComm;
struct SnarkV {  // SNARK (src/lib.rs:701-756)
  std::vector<PolyComm> block_comm_vars_list, exec_comm_inputs;
  PolyComm addr_comm_phy_mems, addr_comm_phy_mems_shifted, addr_comm_vir_mems, addr_comm_vir_mems_shifted,
      addr_comm_ts_bits, perm_exec_comm_w2_list, perm_exec_comm_w3_list, perm_exec_comm_w3_shifted;
  std::vector<PolyComm> block_comm_w2_list, block_comm_w3_list, block_comm_w3_list_shifted;
  PolyComm mem_comm[4][3];  // init_phy, init_vir, phy_addr, vir_addr x (w2, w3, w3_shifted)
  R1CSProofP block_sat;
  Fq block_bound[3];
  FqV block_evals;
  std::vector<SparkV> block_eval_proofs;
  R1CSProofP pairwise_sat;
  Fq pairwise_bound[3];
  FqV pairwise_evals;
  SparkV pairwise_eval_proof;
  R1CSProofP perm_root_sat;
  Fq perm_root_evals[3];
  SparkV perm_root_eval_proof;
  FqV perm_poly_poly_list;
  std::vector<DotProductProofLogP> perm_prod_proofs;
  DotProductProofLogP shift_proof;
  std::vector<Pt> shift_orig_evals, shift_shifted_evals;
  std::vector<std::vector<Pt>> shift_openings;
  std::vector<DotProductProofLogP> io_proofs;
};
bool rd_snark(Rd& r, SnarkV& s) {
  auto comms = [&](std::vector<PolyComm>& v) {
    v.resize(r.len(8));
    for (auto& c : v) c = r.pts();
  };
  comms(s.block_comm_vars_list);
  comms(s.exec_comm_inputs);
  for (PolyComm* c : {&s.addr_comm_phy_mems, &s.addr_comm_phy_mems_shifted, &s.addr_comm_vir_mems,
                      &s.addr_comm_vir_mems_shifted, &s.addr_comm_ts_bits, &s.perm_exec_comm_w2_list,
                      &s.perm_exec_comm_w3_list, &s.perm_exec_comm_w3_shifted})
    *c = r.pts();
  comms(s.block_comm_w2_list);
  comms(s.block_comm_w3_list);
  comms(s.block_comm_w3_list_shifted);
  for (int m = 0; m < 4; m++)
    for (int k = 0; k < 3; k++) s.mem_comm[m][k] = r.pts();
  rd(r, s.block_sat);
  for (int i = 0; i < 3; i++) s.block_bound[i] = r.fq();
  s.block_evals = r.fqs();
  s.block_eval_proofs.resize(r.len(64));
  for (auto& p : s.block_eval_proofs) rd(r, p);
  rd(r, s.pairwise_sat);
  for (int i = 0; i < 3; i++) s.pairwise_bound[i] = r.fq();
  s.pairwise_evals = r.fqs();
  rd(r, s.pairwise_eval_proof);
  rd(r, s.perm_root_sat);
  for (int i = 0; i < 3; i++) s.perm_root_evals[i] = r.fq();
  rd(r, s.perm_root_eval_proof);
  s.perm_poly_poly_list = r.fqs();
  rd(r, s.perm_prod_proofs);
  rd(r, s.shift_proof);
  s.shift_orig_evals = r.pts();
  s.shift_shifted_evals = r.pts();
  s.shift_openings.resize(r.len(8));
  for (auto& o : s.shift_openings) o = r.pts();
  rd(r, s.io_proofs);
  return !r.bad && r.o == r.n;
}

// ---------------------------------------------------------------- group helpers
// a failed decompression makes the whole proof invalid (ProofVerifyError::DecompressionError)
struct Fail {
  const char* what;
};
HExt dec(const Pt& p) {
  HExt P;
  if (!h::hext_decompress(p.b, P)) throw Fail{"point decompression"};
  return P;
}
HExt mulP(const HExt& P, const Fq& k) { return var_mul(P, k); }
HExt addP(const HExt& a, const HExt& b) { return h::hext_add(a, b); }
HExt negP(const HExt& a) { return HExt{h::fe_neg(a.X), a.Y, a.Z, h::fe_neg(a.T)}; }
HExt subP(const HExt& a, const HExt& b) { return addP(a, negP(b)); }
// ristretto255 equality (RFC 9496 4.3.3): X1 Y2 == Y1 X2 or Y1 Y2 == X1 X2
bool eqP(const HExt& a, const HExt& b) {
  return h::fe_eq(h::fe_mul(a.X, b.Y), h::fe_mul(a.Y, b.X)) || h::fe_eq(h::fe_mul(a.Y, b.Y), h::fe_mul(a.X, b.X));
}
bool eqP(const HExt& a, const Pt& b) { return eqP(a, dec(b)); }

// sum_i s_i P_i over arbitrary points: unsigned c-bit windows, one pool task per window (Pippenger)
HExt msm_var(const FqV& s, const std::vector<HExt>& P) {
  const size_t n = std::min(s.size(), P.size());
  if (n <= 2) {
    HExt acc = h::hext_identity();
    for (size_t i = 0; i < n; i++) acc = addP(acc, mulP(P[i], s[i]));
    return acc;
  }
  const int c = n < 16 ? 4 : (n < 128 ? 6 : 8), W = (256 + c - 1) / c, NB = (1 << c) - 1;
  std::vector<uint8_t> bytes(32 * n);
  for (size_t i = 0; i < n; i++) fq_le_bytes(s[i], bytes.data() + 32 * i);
  auto digit = [&](size_t i, int w) {
    const int bit = w * c;
    unsigned v = 0;
    for (int k = 0; k < c && bit + k < 256; k++) v |= ((bytes[32 * i + (bit + k) / 8] >> ((bit + k) % 8)) & 1u) << k;
    return v;
  };
  std::vector<HExt> win(W);
  pool().parallel_for(W, [&](int w) {
    std::vector<HExt> bk(NB, h::hext_identity());
    std::vector<uint8_t> used(NB, 0);
    for (size_t i = 0; i < n; i++) {
      const unsigned d = digit(i, w);
      if (!d) continue;
      bk[d - 1] = used[d - 1] ? addP(bk[d - 1], P[i]) : P[i];
      used[d - 1] = 1;
    }
    HExt run = h::hext_identity(), acc = h::hext_identity();
    for (int v = NB; v >= 1; v--) {
      if (used[v - 1]) run = addP(run, bk[v - 1]);
      acc = addP(acc, run);
    }
    win[w] = acc;
  });
  HExt acc = win[W - 1];
  for (int w = W - 2; w >= 0; w--) {
    for (int k = 0; k < c; k++) acc = h::hext_dbl(acc);
    acc = addP(acc, win[w]);
  }
  return acc;
}
std::vector<HExt> decs(const std::vector<Pt>& v) {
  std::vector<HExt> out(v.size());
  for (size_t i = 0; i < v.size(); i++) out[i] = dec(v[i]);
  return out;
}

// ---------------------------------------------------------------- verifier context
struct V {
  spg_ctx* ctx;
  Tr& t;
  const char* failed = nullptr;
  V(spg_ctx* c, Tr& tt) : ctx(c), t(tt) {}
  bool fail(const char* what) {
    if (!failed) failed = what;
    return false;
  }
  // x.commit(blind, key) for keys of a few generators (host fixed-base tables)
  HExt commit(ProverGens& g, const KeyView& k, const FqV& x, const Fq& blind) {
    std::vector<size_t> idx(k.G.begin(), k.G.begin() + std::min(x.size(), k.G.size()));
    FqV s(x.begin(), x.begin() + idx.size());
    idx.push_back(k.h);
    s.push_back(blind);
    return g.host.msm(idx, s);
  }
  HExt commit1(ProverGens& g, const KeyView& k, const Fq& x, const Fq& blind) { return commit(g, k, {x}, blind); }
  // sum_i s_i G_i over the first n generators of key k, on the GPU (resident fixed-base tables)
  HExt gens_msm(ProverGens& g, const KeyView& k, const FqV& s) {
    std::vector<uint32_t> idx(s.size());
    for (size_t i = 0; i < s.size(); i++) idx[i] = (uint32_t)k.G[i];
    std::vector<Pt> out;
    if (device_msm_idx(ctx, g, {s}, {idx}, &out)) throw Fail{"device MSM"};
    return dec(out[0]);
  }

  // ---- sigma protocols (src/nizk/mod.rs)
  bool knowledge(ProverGens& g, const KeyView& k, const KnowledgeProofP& p, const Pt& C) {
    t.protocol("knowledge proof");
    t.point("C", C);
    t.point("alpha", p.alpha);
    const Fq c = t.challenge("c");
    return eqP(commit1(g, k, p.z1, p.z2), addP(mulP(dec(C), c), dec(p.alpha))) || fail("KnowledgeProof");
  }
  bool equality(ProverGens& g, const KeyView& k, const EqualityProofP& p, const Pt& C1, const Pt& C2) {
    t.protocol("equality proof");
    t.point("C1", C1);
    t.point("C2", C2);
    t.point("alpha", p.alpha);
    const Fq c = t.challenge("c");
    const HExt C = subP(dec(C1), dec(C2));
    return eqP(g.host.msm({k.h}, {p.z}), addP(mulP(C, c), dec(p.alpha))) || fail("EqualityProof");
  }
  bool product(ProverGens& g, const KeyView& k, const ProductProofP& p, const Pt& X, const Pt& Y, const Pt& Z) {
    t.protocol("product proof");
    t.point("X", X);
    t.point("Y", Y);
    t.point("Z", Z);
    t.point("alpha", p.alpha);
    t.point("beta", p.beta);
    t.point("delta", p.delta);
    const Fq c = t.challenge("c");
    const HExt Xp = dec(X);
    auto check = [&](const Pt& P, const HExt& Q, const HExt& rhs) { return eqP(addP(dec(P), mulP(Q, c)), rhs); };
    const bool ok = check(p.alpha, Xp, commit1(g, k, p.z[0], p.z[1])) && check(p.beta, dec(Y), commit1(g, k, p.z[2], p.z[3])) &&
                    check(p.delta, dec(Z), addP(mulP(Xp, p.z[2]), g.host.msm({k.h}, {p.z[4]})));
    return ok || fail("ProductProof");
  }
  bool dot(ProverGens& g, const KeyView& k1, const KeyView& kn, const DotProductProofP& p, const FqV& a, const Pt& Cx,
           const Pt& Cy) {
    t.protocol("dot product proof");
    t.point("Cx", Cx);
    t.point("Cy", Cy);
    t.scalars("a", a);
    t.point("delta", p.delta);
    t.point("beta", p.beta);
    const Fq c = t.challenge("c");
    if (p.z.size() != a.size() || a.size() > kn.G.size()) return fail("DotProductProof size");
    Fq dz = fq_zero();
    for (size_t i = 0; i < a.size(); i++) dz = fq_add(dz, fq_mul(p.z[i], a[i]));
    const bool ok = eqP(addP(mulP(dec(Cx), c), dec(p.delta)), commit(g, kn, p.z, p.z_delta)) &&
                    eqP(addP(mulP(dec(Cy), c), dec(p.beta)), commit1(g, k1, dz, p.z_beta));
    return ok || fail("DotProductProof");
  }
  // BulletReductionProof::verify + DotProductProofLog::verify (bullet.rs:138-232, nizk/mod.rs:525-570)
  bool dotlog(ProverGens& g, size_t n, const DotProductProofLogP& p, const FqV& a, const HExt& Cx, const HExt& Cy,
              const Pt& Cx_c, const Pt& Cy_c) {
    t.protocol("dot product proof (log)");
    t.point("Cx", Cx_c);
    t.point("Cy", Cy_c);
    t.scalars("a", a);
    const Fq r = t.challenge("r");
    const HExt Gamma = addP(Cx, mulP(Cy, r));
    const size_t lg_n = p.L.size();
    if (lg_n >= 32 || p.R.size() != lg_n || n != ((size_t)1 << lg_n) || a.size() != n || n > g.gens_n.G.size())
      return fail("Bullet sizes");
    FqV ch(lg_n), chinv(lg_n);
    for (size_t i = 0; i < lg_n; i++) {
      t.point("L", p.L[i]);
      t.point("R", p.R[i]);
      ch[i] = t.challenge("u");
    }
    Fq allinv = fq_one();
    for (size_t i = 0; i < lg_n; i++) {
      chinv[i] = fq_inv(ch[i]);
      allinv = fq_mul(allinv, chinv[i]);
    }
    FqV s(n);
    s[0] = allinv;
    for (size_t i = 1; i < n; i++) {
      size_t lg_i = 0;
      while (((size_t)2 << lg_i) <= i) lg_i++;
      const size_t k = (size_t)1 << lg_i;
      s[i] = fq_mul(s[i - k], fq_sqr(ch[(lg_n - 1) - lg_i]));
    }
    const HExt g_hat = gens_msm(g, g.gens_n, s);
    Fq a_hat = fq_zero();
    for (size_t i = 0; i < n; i++) a_hat = fq_add(a_hat, fq_mul(a[i], s[i]));
    FqV sc;
    std::vector<HExt> P;
    for (size_t i = 0; i < lg_n; i++) {
      sc.push_back(fq_sqr(ch[i]));
      P.push_back(dec(p.L[i]));
    }
    for (size_t i = 0; i < lg_n; i++) {
      sc.push_back(fq_sqr(chinv[i]));
      P.push_back(dec(p.R[i]));
    }
    const HExt Gamma_hat = addP(msm_var(sc, P), Gamma);
    t.point("delta", p.delta);
    t.point("beta", p.beta);
    const Fq c = t.challenge("c");
    const HExt G1r = mulP(g.host.point(g.gens_1.G[0]), r);  // gens_1 scaled by r
    const HExt lhs = addP(mulP(addP(mulP(Gamma_hat, c), dec(p.beta)), a_hat), dec(p.delta));
    const HExt rhs = addP(mulP(addP(g_hat, mulP(G1r, a_hat)), p.z1), g.host.msm({g.gens_1.h}, {p.z2}));
    return eqP(lhs, rhs) || fail("DotProductProofLog");
  }
  bool dotlog(ProverGens& g, size_t n, const DotProductProofLogP& p, const FqV& a, const HExt& Cx, const HExt& Cy) {
    return dotlog(g, n, p, a, Cx, Cy, compress(Cx), compress(Cy));
  }

  // ---- sumchecks (src/sumcheck.rs)
  bool zk_sumcheck(ProverGens& g, const ZKSumcheckP& p, const Pt& comm_claim, size_t rounds, Pt* final_comm, FqV* r) {
    if (p.comm_polys.size() != rounds || p.comm_evals.size() != rounds || p.proofs.size() != rounds)
      return fail("ZK sumcheck rounds");
    for (size_t i = 0; i < rounds; i++) {
      t.point("comm_poly", p.comm_polys[i]);
      const Fq r_i = t.challenge("challenge_nextround");
      const Pt& ccpr = i == 0 ? comm_claim : p.comm_evals[i - 1];
      t.point("comm_claim_per_round", ccpr);
      t.point("comm_eval", p.comm_evals[i]);
      const FqV w = t.challenges("combine_two_claims_to_one", 2);
      const Pt target = compress(addP(mulP(dec(ccpr), w[0]), mulP(dec(p.comm_evals[i]), w[1])));
      FqV a(4);
      Fq pw = fq_one();
      for (size_t j = 0; j < 4; j++) {
        const Fq a_sc = j == 0 ? fq_dbl(fq_one()) : fq_one();
        a[j] = fq_add(fq_mul(w[0], a_sc), fq_mul(w[1], pw));
        pw = fq_mul(pw, r_i);
      }
      if (!dot(g, g.gens_1, g.gens_4, p.proofs[i], a, p.comm_polys[i], target)) return false;
      r->push_back(r_i);
    }
    *final_comm = p.comm_evals.back();
    return true;
  }
  // SumcheckInstanceProof::verify, cubic rounds (compressed polys hold c0, c2, c3)
  bool sumcheck(const std::vector<FqV>& polys, Fq claim, size_t rounds, Fq* e_out, FqV* r) {
    if (polys.size() != rounds) return fail("sumcheck rounds");
    Fq e = claim;
    for (size_t i = 0; i < rounds; i++) {
      const FqV& cp = polys[i];
      if (cp.size() != 3) return fail("sumcheck degree");
      // c1 = e - 2 c0 - c2 - c3 (UniPoly::decompress), so p(0) + p(1) == e holds by construction
      const Fq c1 = fq_sub(fq_sub(fq_sub(e, fq_dbl(cp[0])), cp[1]), cp[2]);
      const FqV c = {cp[0], c1, cp[1], cp[2]};
      t.msg("poly", "UniPoly_begin");  // UniPoly::append_to_transcript of the decompressed polynomial
      for (auto& x : c) t.scalar("coeff", x);
      t.msg("poly", "UniPoly_end");
      const Fq ri = t.challenge("challenge_nextround");
      r->push_back(ri);
      e = uni_eval(c, ri);
    }
    *e_out = e;
    return true;
  }

  // ---- PolyEvalProof (src/dense_mlpoly.rs)
  static void factored(const FqV& r, FqV* L, FqV* R) {
    const size_t ln = r.size() / 2;
    *L = eq_evals_host(FqV(r.begin(), r.begin() + ln));
    *R = eq_evals_host(FqV(r.begin() + ln, r.end()));
  }
  static bool same(const FqV& a, const FqV& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); i++)
      if (!fq_eq(a[i], b[i])) return false;
    return true;
  }
  bool pe_verify(ProverGens& g, const DotProductProofLogP& p, const FqV& r, const HExt& C_Zr, const PolyComm& comm) {
    t.protocol("polynomial evaluation proof");
    FqV L, R;
    factored(r, &L, &R);
    if (comm.size() != L.size()) return fail("PolyEvalProof commitment size");
    return dotlog(g, R.size(), p, R, msm_var(L, decs(comm)), C_Zr);
  }
  bool pe_verify_plain(ProverGens& g, const DotProductProofLogP& p, const FqV& r, const Fq& Zr, const PolyComm& comm) {
    return pe_verify(g, p, r, commit1(g, g.gens_1, Zr, fq_zero()), comm);
  }
  static FqV fit(const FqV& r, size_t nv) {  // pad with zeros at the front, or keep the last nv
    if (nv >= r.size()) {
      FqV v(nv - r.size(), fq_zero());
      v.insert(v.end(), r.begin(), r.end());
      return v;
    }
    return FqV(r.end() - nv, r.end());
  }
  bool pe_batched_disjoint(ProverGens& g, const std::vector<DotProductProofLogP>& proofs,
                           const std::vector<size_t>& np_list, const std::vector<size_t>& ni_list, const FqV& rq,
                           const FqV& ry, const std::vector<HExt>& Zr_list, const std::vector<const PolyComm*>& comms) {
    t.protocol("polynomial evaluation proof");
    std::vector<std::pair<size_t, size_t>> keys;
    std::vector<HExt> LZ_list, Zc;
    std::vector<FqV> L_list, R_list;
    const Fq c_base = t.challenge("challenge_c");
    Fq c = fq_one();
    for (size_t i = 0; i < comms.size(); i++) {
      const std::pair<size_t, size_t> key = {np_list[i], ni_list[i]};
      size_t idx = keys.size();
      for (size_t k = 0; k < keys.size(); k++)
        if (keys[k] == key) idx = k;
      if (idx < keys.size()) {
        c = fq_mul(c, c_base);
        if (comms[i]->size() != L_list[idx].size()) return fail("PolyEvalProof commitment size");
        LZ_list[idx] = addP(LZ_list[idx], mulP(msm_var(L_list[idx], decs(*comms[i])), c));
        Zc[idx] = addP(Zc[idx], mulP(Zr_list[i], c));
      } else {
        keys.push_back(key);
        Zc.push_back(Zr_list[i]);
        const size_t nvq = lg2(key.first), nvy = lg2(key.second);
        if (nvq > rq.size()) return fail("PolyEvalProof sizes");
        FqV r(rq.end() - nvq, rq.end());
        const FqV rys = fit(ry, nvy);
        r.insert(r.end(), rys.begin(), rys.end());
        FqV L, R;
        factored(r, &L, &R);
        if (comms[i]->size() != L.size()) return fail("PolyEvalProof commitment size");
        LZ_list.push_back(msm_var(L, decs(*comms[i])));
        L_list.push_back(L);
        R_list.push_back(R);
      }
    }
    if (LZ_list.size() != proofs.size()) return fail("PolyEvalProof count");
    for (size_t i = 0; i < LZ_list.size(); i++)
      if (!dotlog(g, R_list[i].size(), proofs[i], R_list[i], LZ_list[i], Zc[i])) return false;
    return true;
  }
  bool pe_plain_batched_points(ProverGens& g, const std::vector<DotProductProofLogP>& proofs,
                               const std::vector<FqV>& r_list, const FqV& Zr_list, const PolyComm& comm) {
    t.protocol("polynomial evaluation proof");
    const size_t ln = r_list[0].size() / 2;
    std::vector<FqV> keys, L_list, R_list;
    FqV Zc;
    const Fq c_base = t.challenge("challenge_c");
    Fq c = fq_one();
    for (size_t i = 0; i < r_list.size(); i++) {
      FqV Li, Ri;
      factored(r_list[i], &Li, &Ri);
      const FqV key(r_list[i].begin(), r_list[i].begin() + ln);
      size_t idx = keys.size();
      for (size_t k = 0; k < keys.size(); k++)
        if (same(keys[k], key)) {
          idx = k;
          break;
        }
      if (idx < keys.size()) {
        c = fq_mul(c, c_base);
        for (size_t j = 0; j < Ri.size(); j++) R_list[idx][j] = fq_add(R_list[idx][j], fq_mul(c, Ri[j]));
        Zc[idx] = fq_add(Zc[idx], fq_mul(c, Zr_list[i]));
      } else {
        keys.push_back(key);
        L_list.push_back(Li);
        R_list.push_back(Ri);
        Zc.push_back(Zr_list[i]);
      }
    }
    if (L_list.size() != proofs.size()) return fail("PolyEvalProof count");
    const std::vector<HExt> C = decs(comm);
    for (size_t i = 0; i < L_list.size(); i++) {
      if (C.size() != L_list[i].size()) return fail("PolyEvalProof commitment size");
      if (!dotlog(g, R_list[i].size(), proofs[i], R_list[i], msm_var(L_list[i], C),
                  commit1(g, g.gens_1, Zc[i], fq_zero())))
        return false;
    }
    return true;
  }
  bool pe_plain_batched_instances(ProverGens& g, const std::vector<DotProductProofLogP>& proofs,
                                  const std::vector<FqV>& r_list, const FqV& Zr_list,
                                  const std::vector<const PolyComm*>& comms, const std::vector<size_t>& nv_list) {
    t.protocol("polynomial evaluation proof");
    if (comms.size() != r_list.size()) return fail("PolyEvalProof count");
    std::vector<std::pair<size_t, FqV>> keys;
    std::vector<HExt> LZ_list;
    FqV Zc;
    std::vector<FqV> R_list;
    const Fq c_base = t.challenge("challenge_c");
    Fq c = fq_one();
    for (size_t i = 0; i < comms.size(); i++) {
      FqV L, R;
      factored(fit(r_list[i], nv_list[i]), &L, &R);
      if (comms[i]->size() != L.size()) return fail("PolyEvalProof commitment size");
      const HExt LZ = msm_var(L, decs(*comms[i]));
      size_t idx = keys.size();
      for (size_t k = 0; k < keys.size(); k++)
        if (keys[k].first == nv_list[i] && same(keys[k].second, R)) {
          idx = k;
          break;
        }
      if (idx < keys.size()) {
        c = fq_mul(c, c_base);
        LZ_list[idx] = addP(LZ_list[idx], mulP(LZ, c));
        Zc[idx] = fq_add(Zc[idx], fq_mul(c, Zr_list[i]));
      } else {
        keys.push_back({nv_list[i], R});
        Zc.push_back(Zr_list[i]);
        LZ_list.push_back(LZ);
        R_list.push_back(R);
      }
    }
    if (LZ_list.size() != proofs.size()) return fail("PolyEvalProof count");
    for (size_t i = 0; i < LZ_list.size(); i++)
      if (!dotlog(g, R_list[i].size(), proofs[i], R_list[i], LZ_list[i], commit1(g, g.gens_1, Zc[i], fq_zero())))
        return false;
    return true;
  }
  bool pe_uni_batched(ProverGens& g, const DotProductProofLogP& p, const Fq& r, const std::vector<HExt>& C_Zr,
                      const std::vector<const PolyComm*>& comms, const std::vector<size_t>& sizes) {
    t.protocol("polynomial evaluation proof");
    size_t max_size = 0;
    for (auto s : sizes) max_size = std::max(max_size, s);
    const size_t nvm = lg2(npow2(max_size)), rn = nvm - nvm / 2;
    FqV R;
    Fq rb = fq_one();
    for (size_t i = 0; i < ((size_t)1 << rn); i++) {
      R.push_back(rb);
      rb = fq_mul(rb, r);
    }
    std::vector<std::pair<size_t, FqV>> Lmap;
    const Fq c_base = t.challenge("challenge_c");
    Fq c = fq_one();
    HExt LZc = h::hext_identity(), Zrc = h::hext_identity();
    for (size_t i = 0; i < comms.size(); i++) {
      const size_t nv = lg2(npow2(sizes[i]));
      const FqV* L = nullptr;
      for (auto& kv : Lmap)
        if (kv.first == nv) L = &kv.second;
      if (!L) {
        const size_t l2 = nv / 2, r2 = nv - nv / 2;
        Fq r_base = fq_one();
        for (size_t k = 0; k < ((size_t)1 << r2); k++) r_base = fq_mul(r_base, r);
        FqV Lv;
        Fq lb = fq_one();
        for (size_t k = 0; k < ((size_t)1 << l2); k++) {
          Lv.push_back(lb);
          lb = fq_mul(lb, r_base);
        }
        Lmap.push_back({nv, Lv});
        L = &Lmap.back().second;
      }
      if (comms[i]->size() != L->size()) return fail("PolyEvalProof commitment size");
      LZc = addP(LZc, mulP(msm_var(*L, decs(*comms[i])), c));
      Zrc = addP(Zrc, mulP(C_Zr[i], c));
      c = fq_mul(c, c_base);
    }
    return dotlog(g, R.size(), p, R, LZc, Zrc);
  }
};


// VerifierWitnessSecInfo (src/lib.rs:606-698): per instance num_inputs, num_proofs and the Hyrax commitment
struct VSec {
  std::vector<size_t> num_inputs, num_proofs;
  std::vector<PolyComm> comm_w;
  // instances of the components interleaved by decreasing num_proofs (ties: the earlier component)
  static VSec merge(const std::vector<const VSec*>& comps, std::vector<size_t>* inst_map) {
    std::vector<size_t> ptr(comps.size(), 0);
    size_t total = 0;
    for (auto c : comps) total += c->num_inputs.size();
    VSec s;
    inst_map->clear();
    while (inst_map->size() < total) {
      size_t best = 0, nc = 0;
      for (size_t i = 0; i < comps.size(); i++)
        if (ptr[i] < comps[i]->num_proofs.size() && comps[i]->num_proofs[ptr[i]] > best) {
          best = comps[i]->num_proofs[ptr[i]];
          nc = i;
        }
      if (best == 0) throw Fail{"witness section sizes"};
      inst_map->push_back(nc);
      s.num_inputs.push_back(comps[nc]->num_inputs[ptr[nc]]);
      s.num_proofs.push_back(comps[nc]->num_proofs[ptr[nc]]);
      s.comm_w.push_back(comps[nc]->comm_w[ptr[nc]]);
      ptr[nc]++;
    }
    return s;
  }
  static VSec concat(const std::vector<const VSec*>& comps) {
    VSec s;
    for (auto c : comps) {
      s.num_inputs.insert(s.num_inputs.end(), c->num_inputs.begin(), c->num_inputs.end());
      s.num_proofs.insert(s.num_proofs.end(), c->num_proofs.begin(), c->num_proofs.end());
      s.comm_w.insert(s.comm_w.end(), c->comm_w.begin(), c->comm_w.end());
    }
    return s;
  }
};
VSec vsec(std::vector<size_t> ni, std::vector<size_t> np, std::vector<PolyComm> c) {
  VSec v;
  v.num_inputs = ni;
  v.num_proofs = np;
  v.comm_w = c;
  return v;
}

Fq eq_eval(const FqV& a, const FqV& b) {  // EqPolynomial::evaluate
  Fq e = fq_one();
  for (size_t i = 0; i < a.size(); i++)
    e = fq_mul(e, fq_add(fq_mul(a[i], b[i]), fq_mul(fq_sub(fq_one(), a[i]), fq_sub(fq_one(), b[i]))));
  return e;
}
FqV prefix_list(size_t nws, const FqV& rw) {  // r1csproof.rs:880-905
  const Fq one = fq_one();
  FqV v;
  const size_t k = npow2(nws), nb = lg2(k);
  for (size_t i = 0; i < k; i++) {
    Fq f = one;
    for (size_t b = 0; b < nb; b++) f = fq_mul(f, ((i >> (nb - 1 - b)) & 1) ? rw[b] : fq_sub(one, rw[b]));
    v.push_back(f);
  }
  return v;
}

struct SnarkVerifier : V {
  using V::V;

  // R1CSProof::verify (src/r1csproof.rs:687-954); ch = [rp, rq_rev, rx, rw || ry]
  bool r1cs(ProverGens& g, const R1CSProofP& pf, size_t n, size_t max_np, const std::vector<size_t>& num_proofs,
            size_t max_ni, const std::vector<const VSec*>& ws, size_t num_cons, const Fq ev[3], std::vector<FqV>* ch) {
    t.protocol("R1CS proof");
    const size_t nws = ws.size();
    const size_t np = lg2(npow2(n)), nq = lg2(max_np), nx = lg2(num_cons), nw = lg2(nws), ny = lg2(max_ni);
    const FqV tau_p = t.challenges("challenge_tau_p", np), tau_q = t.challenges("challenge_tau_q", nq),
              tau_x = t.challenges("challenge_tau_x", nx);
    if (getenv("SPG_DEBUG_TR")) fprintf(stderr, "[verify] r1cs n=%zu np=%zu nq=%zu nx=%zu tau_x0 %08x\n", n, np, nq, nx, tau_x[0].l[0]);
    const Pt claim1 = compress(commit1(g, g.gens_1, fq_zero(), fq_zero()));
    Pt post1;
    FqV rx_all;
    if (!zk_sumcheck(g, pf.sc1, claim1, nx + nq + np, &post1, &rx_all)) return false;
    const Pt &cA = pf.claims_phase2[0], &cB = pf.claims_phase2[1], &cC = pf.claims_phase2[2], &cP = pf.claims_phase2[3];
    if (!knowledge(g, g.gens_1, pf.pok, cC)) return false;
    if (!product(g, g.gens_1, pf.prod, cA, cB, cP)) return false;
    t.point("comm_Az_claim", cA);
    t.point("comm_Bz_claim", cB);
    t.point("comm_Cz_claim", cC);
    t.point("comm_prod_Az_Bz_claims", cP);
    const FqV rx_rev(rx_all.begin(), rx_all.begin() + nx), rq_rev(rx_all.begin() + nx, rx_all.begin() + nx + nq),
        rp1(rx_all.begin() + nx + nq, rx_all.end());
    const FqV rq(rq_rev.rbegin(), rq_rev.rend());
    const Fq tb = fq_mul(fq_mul(eq_eval(rp1, tau_p), eq_eval(rq_rev, tau_q)), eq_eval(rx_rev, tau_x));
    const Pt expected1 = compress(mulP(subP(dec(cP), dec(cC)), tb));
    if (!equality(g, g.gens_1, pf.eq1, expected1, post1)) return false;
    const Fq r_A = t.challenge("challenge_Az"), r_B = t.challenge("challenge_Bz"), r_C = t.challenge("challenge_Cz");
    const Pt claim2 = compress(addP(addP(mulP(dec(cA), r_A), mulP(dec(cB), r_B)), mulP(dec(cC), r_C)));
    Pt post2;
    FqV ry_all;
    if (!zk_sumcheck(g, pf.sc2, claim2, ny + nw + np, &post2, &ry_all)) return false;
    const FqV ry_rev(ry_all.begin(), ry_all.begin() + ny), rw(ry_all.begin() + ny, ry_all.begin() + ny + nw),
        rp(ry_all.begin() + ny + nw, ry_all.end());
    const FqV ry(ry_rev.rbegin(), ry_rev.rend());
    const Fq p_rp = eq_eval(rp, rp1);
    FqV ry_factors(ny + 1, fq_one());
    for (size_t i = 0; i < ny; i++) ry_factors[i + 1] = fq_mul(ry_factors[i], fq_sub(fq_one(), ry[i]));
    // comm_vars_at_ry_list: nws sections, then (as the prover writes them) nws empty lists (r1csproof.rs:541-542)
    if (pf.comm_vars_at_ry_list.size() < nws) return fail("comm_vars_at_ry_list");
    std::vector<const PolyComm*> comm_list;
    std::vector<size_t> np_list, ni_list;
    std::vector<HExt> comm_Zr;
    for (size_t i = 0; i < nws; i++) {
      if (pf.comm_vars_at_ry_list[i].size() != ws[i]->num_proofs.size()) return fail("comm_vars_at_ry_list");
      for (size_t p = 0; p < ws[i]->num_proofs.size(); p++) {
        comm_list.push_back(&ws[i]->comm_w[p]);
        np_list.push_back(ws[i]->num_proofs[p]);
        ni_list.push_back(ws[i]->num_inputs[p]);
        comm_Zr.push_back(dec(pf.comm_vars_at_ry_list[i][p]));
      }
    }
    if (!pe_batched_disjoint(g, pf.evals, np_list, ni_list, rq, ry, comm_Zr, comm_list)) return false;
    const FqV prefix = prefix_list(nws, rw);
    std::vector<HExt> expected_list;
    for (size_t p = 0; p < n; p++) {
      HExt comb = h::hext_identity();
      for (size_t i = 0; i < nws; i++) {
        const size_t pw = ws[i]->num_proofs.size() == 1 ? 0 : p;
        if (pw >= ws[i]->num_proofs.size()) return fail("witness section instances");
        const HExt c = dec(pf.comm_vars_at_ry_list[i][pw]);
        const size_t lni = lg2(ws[i]->num_inputs[pw]);
        const Fq f = ws[i]->num_inputs[pw] >= max_ni ? fq_one() : ry_factors[ny - lni];
        comb = addP(comb, mulP(c, fq_mul(prefix[i], f)));
      }
      Fq m = fq_one();
      for (size_t q = 0; q < nq - lg2(num_proofs[p]); q++) m = fq_mul(m, fq_sub(fq_one(), rq[q]));
      expected_list.push_back(mulP(comb, m));
    }
    FqV EQ = eq_evals_host(rp);
    EQ.resize(n);
    if (!eqP(msm_var(EQ, expected_list), pf.comm_vars_at_ry)) return fail("comm_vars_at_ry");
    const Fq k = fq_mul(fq_add(fq_add(fq_mul(r_A, ev[0]), fq_mul(r_B, ev[1])), fq_mul(r_C, ev[2])), p_rp);
    const Pt expected2 = compress(mulP(dec(pf.comm_vars_at_ry), k));
    if (!equality(g, g.gens_1, pf.eq2, expected2, post2)) return false;
    const FqV rx(rx_rev.rbegin(), rx_rev.rend());
    FqV rwry(rw);
    rwry.insert(rwry.end(), ry.begin(), ry.end());
    *ch = {rp, rq_rev, rx, rwry};
    return true;
  }

  // ProductCircuitEvalProofBatched::verify (src/product_tree.rs:398-487)
  bool batched(const BatchedV& pf, const FqV& claims_prod, const FqV& claims_dotp_in, size_t len, FqV* claims_out,
               FqV* dotp_out, FqV* rand_out) {
    const size_t num_layers = lg2(len);
    if (pf.layers.size() != num_layers) return fail("product layers");
    FqV rand, claims = claims_prod, dotp_v;
    for (size_t i = 0; i < num_layers; i++) {
      const bool last = i == num_layers - 1;
      if (last) claims.insert(claims.end(), claims_dotp_in.begin(), claims_dotp_in.end());
      const FqV coeffs = t.challenges("rand_coeffs_next_layer", claims.size());
      Fq claim = fq_zero();
      for (size_t k = 0; k < claims.size(); k++) claim = fq_add(claim, fq_mul(claims[k], coeffs[k]));
      Fq claim_last;
      FqV rand_prod;
      if (!sumcheck(pf.layers[i].polys, claim, i, &claim_last, &rand_prod)) return false;
      const FqV &L = pf.layers[i].left, &R = pf.layers[i].right;
      if (L.size() != claims_prod.size() || R.size() != claims_prod.size()) return fail("product layer claims");
      for (size_t k = 0; k < L.size(); k++) {
        t.scalar("claim_prod_left", L[k]);
        t.scalar("claim_prod_right", R[k]);
      }
      const Fq eq = eq_eval(rand, rand_prod);
      Fq expected = fq_zero();
      for (size_t k = 0; k < L.size(); k++) expected = fq_add(expected, fq_mul(coeffs[k], fq_mul(fq_mul(L[k], R[k]), eq)));
      if (last) {
        const size_t np = claims_prod.size(), nd = pf.dotp[0].size();
        if (pf.dotp[1].size() != nd || pf.dotp[2].size() != nd || np + nd != coeffs.size())
          return fail("dot-product circuit claims");
        for (size_t k = 0; k < nd; k++) {
          t.scalar("claim_dotp_left", pf.dotp[0][k]);
          t.scalar("claim_dotp_right", pf.dotp[1][k]);
          t.scalar("claim_dotp_weight", pf.dotp[2][k]);
          expected = fq_add(expected, fq_mul(coeffs[np + k], fq_mul(fq_mul(pf.dotp[0][k], pf.dotp[1][k]), pf.dotp[2][k])));
        }
      }
      if (!fq_eq(expected, claim_last)) return fail("product layer sumcheck");
      const Fq r_layer = t.challenge("challenge_r_layer");
      claims.clear();
      for (size_t k = 0; k < L.size(); k++) claims.push_back(fq_add(L[k], fq_mul(r_layer, fq_sub(R[k], L[k]))));
      if (last)
        for (size_t k = 0; k < claims_dotp_in.size() / 2; k++)
          for (int c = 0; c < 3; c++)
            dotp_v.push_back(fq_add(pf.dotp[c][2 * k], fq_mul(r_layer, fq_sub(pf.dotp[c][2 * k + 1], pf.dotp[c][2 * k]))));
      FqV ext = {r_layer};
      ext.insert(ext.end(), rand_prod.begin(), rand_prod.end());
      rand = ext;
    }
    *claims_out = claims;
    *dotp_out = dotp_v;
    *rand_out = rand;
    return true;
  }

  // combine_n_to_one / two_to_one (sparse_mlpoly.rs:970-1000): bind the low challenges of the claimed evaluations
  void combine(const FqV& evals, const FqV& r, const char* label, FqV* r_joint, Fq* eval) {
    const FqV ch = t.challenges(label, lg2(evals.size()));
    FqV v = evals;
    for (size_t i = ch.size(); i-- > 0;) {
      const size_t n = v.size() / 2;
      for (size_t k = 0; k < n; k++) v[k] = fq_add(v[2 * k], fq_mul(ch[i], fq_sub(v[2 * k + 1], v[2 * k])));
      v.resize(n);
    }
    *eval = v[0];
    *r_joint = ch;
    r_joint->insert(r_joint->end(), r.begin(), r.end());
  }

  // SparseMatPolyEvalProof::verify (src/sparse_mlpoly.rs:1566-1610 with the product and hash layers)
  bool spark(spg_spark* S, const SparkV& pf, const FqV& rx, const FqV& ry, const FqV& evals) {
    t.protocol("Sparse polynomial evaluation proof");
    FqV ex = rx, ey = ry;
    if (ex.size() < ey.size()) ex.insert(ex.begin(), ey.size() - ex.size(), fq_zero());
    if (ey.size() < ex.size()) ey.insert(ey.begin(), ex.size() - ey.size(), fq_zero());
    if (((size_t)1 << ex.size()) != S->cells) return fail("SPARK memory size");
    t.msg("derefs_commitment", "begin_derefs_commitment");
    append_polycomm(t, "comm_poly_row_col_ops_val", pf.comm_derefs);
    t.msg("derefs_commitment", "end_derefs_commitment");
    const FqV rmc = t.challenges("challenge_r_hash", 2);
    const Fq r_hash = rmc[0], r_ms = rmc[1];
    t.protocol("Sparse polynomial evaluation proof");
    const size_t B = evals.size(), num_ops = npow2(S->N), num_cells = S->cells;
    t.protocol("Sparse polynomial product layer proof");
    if (pf.row_read.size() != B || pf.row_write.size() != B || pf.col_read.size() != B || pf.col_write.size() != B)
      return fail("SPARK claim counts");
    auto prod = [](const FqV& v) {
      Fq p = fq_one();
      for (auto& x : v) p = fq_mul(p, x);
      return p;
    };
    if (!fq_eq(fq_mul(pf.row_init, prod(pf.row_write)), fq_mul(prod(pf.row_read), pf.row_audit)))
      return fail("SPARK row multiset");
    t.scalar("claim_row_eval_init", pf.row_init);
    t.scalars("claim_row_eval_read", pf.row_read);
    t.scalars("claim_row_eval_write", pf.row_write);
    t.scalar("claim_row_eval_audit", pf.row_audit);
    if (!fq_eq(fq_mul(pf.col_init, prod(pf.col_write)), fq_mul(prod(pf.col_read), pf.col_audit)))
      return fail("SPARK col multiset");
    t.scalar("claim_col_eval_init", pf.col_init);
    t.scalars("claim_col_eval_read", pf.col_read);
    t.scalars("claim_col_eval_write", pf.col_write);
    t.scalar("claim_col_eval_audit", pf.col_audit);
    if (pf.dotp_left.size() != B || pf.dotp_right.size() != B) return fail("SPARK dot-product claims");
    FqV claims_dotp_circuit;
    for (size_t i = 0; i < B; i++) {
      if (!fq_eq(fq_add(pf.dotp_left[i], pf.dotp_right[i]), evals[i])) return fail("SPARK evaluation claim");
      t.scalar("claim_eval_dotp_left", pf.dotp_left[i]);
      t.scalar("claim_eval_dotp_right", pf.dotp_right[i]);
      claims_dotp_circuit.push_back(pf.dotp_left[i]);
      claims_dotp_circuit.push_back(pf.dotp_right[i]);
    }
    FqV claims_prod;
    for (const FqV* v : {&pf.row_read, &pf.row_write, &pf.col_read, &pf.col_write})
      claims_prod.insert(claims_prod.end(), v->begin(), v->end());
    FqV claims_ops, claims_dotp, rand_ops, claims_mem, claims_mem_dotp, rand_mem;
    if (!batched(pf.proof_ops, claims_prod, claims_dotp_circuit, num_ops, &claims_ops, &claims_dotp, &rand_ops))
      return false;
    if (!batched(pf.proof_mem, {pf.row_init, pf.row_audit, pf.col_init, pf.col_audit}, {}, num_cells, &claims_mem,
                 &claims_mem_dotp, &rand_mem))
      return false;
    t.protocol("Sparse polynomial hash layer proof");
    {
      t.protocol("Derefs evaluation proof");
      FqV ev = pf.eval_row_ops_val;
      ev.insert(ev.end(), pf.eval_col_ops_val.begin(), pf.eval_col_ops_val.end());
      ev.resize(npow2(std::max<size_t>(ev.size(), 1)), fq_zero());
      t.scalars("evals_ops_val", ev);
      FqV rj;
      Fq ej;
      combine(ev, rand_ops, "challenge_combine_n_to_one", &rj, &ej);
      t.scalar("joint_claim_eval", ej);
      if (!pe_verify_plain(S->g_der, pf.pe_derefs, rj, ej, pf.comm_derefs)) return false;
    }
    if (claims_dotp.size() != 3 * pf.eval_row_ops_val.size() || pf.eval_col_ops_val.size() != pf.eval_row_ops_val.size() ||
        pf.eval_val.size() != pf.eval_row_ops_val.size())
      return fail("SPARK derefs claims");
    for (size_t i = 0; i < claims_dotp.size() / 3; i++)
      if (!fq_eq(claims_dotp[3 * i], pf.eval_row_ops_val[i]) || !fq_eq(claims_dotp[3 * i + 1], pf.eval_col_ops_val[i]) ||
          !fq_eq(claims_dotp[3 * i + 2], pf.eval_val[i]))
        return fail("SPARK dot-product circuit claims");
    {
      FqV ev;
      for (const FqV* v : {&pf.eval_row_addr, &pf.eval_row_read_ts, &pf.eval_col_addr, &pf.eval_col_read_ts, &pf.eval_val})
        ev.insert(ev.end(), v->begin(), v->end());
      ev.resize(npow2(std::max<size_t>(ev.size(), 1)), fq_zero());
      t.scalars("claim_evals_ops", ev);
      FqV rj;
      Fq ej;
      combine(ev, rand_ops, "challenge_combine_n_to_one", &rj, &ej);
      t.scalar("joint_claim_eval_ops", ej);
      if (!pe_verify_plain(S->g_ops, pf.pe_ops, rj, ej, S->comm_ops)) return false;
    }
    {
      const FqV ev = {pf.eval_row_audit_ts, pf.eval_col_audit_ts};
      t.scalars("claim_evals_mem", ev);
      FqV rj;
      Fq ej;
      combine(ev, rand_mem, "challenge_combine_two_to_one", &rj, &ej);
      t.scalar("joint_claim_eval_mem", ej);
      if (!pe_verify_plain(S->g_mem, pf.pe_mem, rj, ej, S->comm_mem)) return false;
    }
    // hash-layer checks (sparse_mlpoly.rs:920-969)
    const Fq r2 = fq_mul(r_hash, r_hash);
    auto hash = [&](const Fq& addr, const Fq& val, const Fq& ts) {
      return fq_sub(fq_add(fq_add(fq_mul(ts, r2), fq_mul(val, r_hash)), addr), r_ms);
    };
    Fq init_addr = fq_zero();  // IdentityPolynomial::evaluate: sum_i 2^(n-1-i) r_i
    for (size_t i = 0; i < rand_mem.size(); i++) init_addr = fq_add(fq_dbl(init_addr), rand_mem[i]);
    auto check = [&](const FqV& r, const Fq& cinit, const FqV& cread, const FqV& cwrite, const Fq& caudit,
                     const FqV& ops_val, const FqV& addr, const FqV& rts, const Fq& ats) -> bool {
      if (addr.size() != B || rts.size() != B || ops_val.size() != B) return false;
      const Fq init_val = eq_eval(r, rand_mem);
      if (!fq_eq(hash(init_addr, init_val, fq_zero()), cinit)) return false;
      for (size_t i = 0; i < B; i++) {
        if (!fq_eq(hash(addr[i], ops_val[i], rts[i]), cread[i])) return false;
        if (!fq_eq(hash(addr[i], ops_val[i], fq_add(rts[i], fq_one())), cwrite[i])) return false;
      }
      return fq_eq(hash(init_addr, init_val, ats), caudit);
    };
    if (claims_ops.size() != 4 * B || claims_mem.size() != 4 || rand_mem.size() != ex.size())
      return fail("SPARK layer claims");
    const FqV cr_row(claims_ops.begin(), claims_ops.begin() + B), cw_row(claims_ops.begin() + B, claims_ops.begin() + 2 * B),
        cr_col(claims_ops.begin() + 2 * B, claims_ops.begin() + 3 * B), cw_col(claims_ops.begin() + 3 * B, claims_ops.end());
    if (!check(ex, claims_mem[0], cr_row, cw_row, claims_mem[1], pf.eval_row_ops_val, pf.eval_row_addr,
               pf.eval_row_read_ts, pf.eval_row_audit_ts))
      return fail("SPARK row hash layer");
    if (!check(ey, claims_mem[2], cr_col, cw_col, claims_mem[3], pf.eval_col_ops_val, pf.eval_col_addr,
               pf.eval_col_read_ts, pf.eval_col_audit_ts))
      return fail("SPARK col hash layer");
    return true;
  }
};


// DensePolynomial::commit (no blinds) of a host vector, through the device Hyrax path
PolyComm commit_vec(spg_ctx* ctx, ProverGens& g, FqV Z) {
  Z.resize(npow2(std::max<size_t>(Z.size(), 1)), fq_zero());
  Fq* d = (Fq*)ws_get(ctx, 96, Z.size() * sizeof(Fq) + 64);
  if (!d) throw Fail{"workspace"};
  if (hipMemcpy(d, Z.data(), Z.size() * sizeof(Fq), hipMemcpyHostToDevice) != hipSuccess) throw Fail{"upload"};
  std::vector<Pt> out;
  if (commit_dev(ctx, g, d, lg2(Z.size()), &out)) throw Fail{"commit"};
  return out;
}

const size_t INIT_PHY_MEM_WIDTH = 4, INIT_VIR_MEM_WIDTH = 4, PHY_MEM_WIDTH = 4, VIR_MEM_WIDTH = 8;

// the public values SNARK::verify converts from bytes (src/lib.rs:2836-2850): input, output, and the input stack /
// input memory whose init lists the verifier commits itself (:3274-3333); n = the list's length (unpadded)
struct SnarkPub {
  FqV input;
  Fq output;
  FqV stack, mem;
};

// SNARK::verify (src/lib.rs:2750-3881)
bool snark_verify(SnarkVerifier& v, const SnarkV& pf, const spg_snark_inputs& in, const SnarkPub& pub,
                  const SnarkCompView& block, const SnarkCompView& pairwise, const SnarkCompView& perm_root,
                  ProverGens& gpc) {
  Tr& t = v.t;
  const size_t niu = in.num_inputs_unpadded, num_ios = in.num_ios, Bb = in.block_num_instances_bound;
  std::vector<size_t> bnv_all(in.block_num_vars, in.block_num_vars + Bb), bnp_all(in.block_num_proofs, in.block_num_proofs + Bb);
  std::vector<size_t> phy(in.block_num_phy_ops, in.block_num_phy_ops + Bb), vir(in.block_num_vir_ops, in.block_num_vir_ops + Bb);
  t.protocol("Spartan SNARK proof");
  auto app = [&](const char* l, size_t x) { t.scalar(l, fq_from_u64(x)); };
  app("func_input_width", in.func_input_width);
  app("input_offset", in.input_offset);
  app("output_offset", in.output_offset);
  app("output_exec_num", in.output_exec_num);
  app("num_ios", num_ios);
  for (auto n : bnv_all) app("block_num_vars", n);
  app("mem_addr_ts_bits_size", in.mem_addr_ts_bits_size);
  app("num_inputs_unpadded", niu);
  app("block_num_instances_bound", Bb);
  app("block_max_num_proofs", in.block_max_num_proofs);
  for (auto p : phy) app("block_num_phy_ops", p);
  for (auto x : vir) app("block_num_vir_ops", x);
  app("total_num_init_phy_mem_accesses", in.total_num_init_phy_mem_accesses);
  app("total_num_init_vir_mem_accesses", in.total_num_init_vir_mem_accesses);
  app("total_num_phy_mem_accesses", in.total_num_phy_mem_accesses);
  app("total_num_vir_mem_accesses", in.total_num_vir_mem_accesses);
  app("block_max_num_proofs", in.block_max_num_proofs);
  for (auto n : bnp_all) app("block_num_proofs", n);
  for (auto& b : *block.label_map)
    for (auto l : b) app("block_comm_map", l);
  auto comm_append = [&](const SnarkCompView& c, size_t gi) {  // R1CSCommitment::append_to_transcript
    t.u64("num_cons", c.num_instances * c.max_num_cons);
    t.u64("num_vars", c.num_vars);
    spark_comm_append((*c.sparks)[gi], t);
  };
  for (size_t gi = 0; gi < block.sparks->size(); gi++) comm_append(block, gi);
  comm_append(pairwise, 0);
  comm_append(perm_root, 0);
  const FqV& input = pub.input;
  const Fq output = pub.output;
  app("input_block_num", in.input_block_num);
  app("output_block_num", in.output_block_num);
  t.scalars("input_list", input);
  t.scalar("output_list", output);
  // sort and padding, sizes only (lib.rs:2922-3009)
  size_t P = 0;
  for (auto n : bnp_all)
    if (n > 0) P++;
  std::vector<size_t> order(Bb);
  for (size_t i = 0; i < Bb; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return bnp_all[a] > bnp_all[b]; });
  order.resize(P);
  std::vector<size_t> bnp, bnv;
  for (size_t i : order) {
    bnp.push_back(npow2(bnp_all[i]));
    bnv.push_back(bnv_all[i]);
  }
  const size_t bmax = npow2(in.block_max_num_proofs), consis = npow2(in.consis_num_proofs);
  auto pad0 = [](size_t x) { return x == 0 ? (size_t)0 : npow2(x); };
  const size_t t_iphy = pad0(in.total_num_init_phy_mem_accesses), t_ivir = pad0(in.total_num_init_vir_mem_accesses),
               t_phy = pad0(in.total_num_phy_mem_accesses), t_vir = pad0(in.total_num_vir_mem_accesses);
  std::vector<std::pair<size_t, size_t>> ps = {{consis, 0}, {t_phy, 1}, {t_vir, 2}};
  std::stable_sort(ps.begin(), ps.end(), [](const std::pair<size_t, size_t>& a, const std::pair<size_t, size_t>& b) {
    return a.first > b.first;
  });
  std::vector<size_t> pw_index;
  for (size_t i = 0; i < 1 + (t_phy > 0 ? 1 : 0) + (t_vir > 0 ? 1 : 0); i++) pw_index.push_back(ps[i].second);
  // commitments in the prover's order
  const Fq tau = t.challenge("challenge_tau"), r = t.challenge("challenge_r");
  if (getenv("SPG_DEBUG_TR")) fprintf(stderr, "[verify] tau %08x r %08x\n", tau.l[0], r.l[0]);
  FqV perm_w0 = {tau};
  {
    Fq rt = r;
    for (size_t i = 1; i < 2 * niu; i++) {
      perm_w0.push_back(rt);
      rt = fq_mul(rt, r);
    }
    perm_w0.resize(num_ios, fq_zero());
  }
  const PolyComm c_w0 = commit_vec(v.ctx, gpc, perm_w0);
  append_polycomm(t, "poly_commitment", c_w0);
  append_polycomm(t, "poly_commitment", pf.perm_exec_comm_w2_list);
  append_polycomm(t, "poly_commitment", pf.perm_exec_comm_w3_list);
  append_polycomm(t, "poly_commitment", pf.perm_exec_comm_w3_shifted);
  if (pf.block_comm_w2_list.size() != P || pf.block_comm_w3_list.size() != P || pf.block_comm_w3_list_shifted.size() != P ||
      pf.block_comm_vars_list.size() != P || pf.exec_comm_inputs.size() != 1)
    return v.fail("witness commitment counts");
  for (auto& c : pf.block_comm_w2_list) append_polycomm(t, "poly_commitment", c);
  for (size_t p = 0; p < P; p++) {
    append_polycomm(t, "poly_commitment", pf.block_comm_w3_list[p]);
    append_polycomm(t, "poly_commitment", pf.block_comm_w3_list_shifted[p]);
  }
  // memory (w2, w3, w3_shifted) triples (lib.rs:3100-3240)
  VSec ms[4][3];
  const size_t totals[4] = {t_iphy, t_ivir, t_phy, t_vir}, widths[4] = {INIT_PHY_MEM_WIDTH, INIT_VIR_MEM_WIDTH, PHY_MEM_WIDTH, VIR_MEM_WIDTH};
  for (int m = 0; m < 4; m++) {
    if (totals[m] == 0) continue;
    for (int k = 0; k < 3; k++) append_polycomm(t, "poly_commitment", pf.mem_comm[m][k]);
    ms[m][0] = vsec({widths[m]}, {totals[m]}, {pf.mem_comm[m][0]});
    ms[m][1] = vsec({8}, {totals[m]}, {pf.mem_comm[m][1]});
    ms[m][2] = vsec({8}, {totals[m]}, {pf.mem_comm[m][2]});
  }
  for (auto& c : pf.block_comm_vars_list) append_polycomm(t, "poly_commitment", c);
  append_polycomm(t, "poly_commitment", pf.exec_comm_inputs[0]);
  // the verifier commits the init lists itself from the public input stack / memory (lib.rs:3274-3333): rows
  // (1, 0, i, value_i) for the list, zero rows up to the padded total
  auto init_vsec = [&](size_t total, const FqV& vals, size_t width) {
    VSec s;
    if (vals.empty()) return s;
    FqV flat(total * width, fq_zero());
    for (size_t i = 0; i < vals.size(); i++) {
      flat[i * width] = fq_one();
      flat[i * width + 2] = fq_from_u64(i);
      flat[i * width + 3] = vals[i];
    }
    const PolyComm c = commit_vec(v.ctx, gpc, flat);
    append_polycomm(t, "poly_commitment", c);
    return vsec({width}, {total}, {c});
  };
  if (pub.stack.size() > t_iphy || pub.mem.size() > t_ivir) return v.fail("init memory lists longer than their totals");
  const VSec init_phy_v = init_vsec(t_iphy, pub.stack, INIT_PHY_MEM_WIDTH);
  const VSec init_vir_v = init_vsec(t_ivir, pub.mem, INIT_VIR_MEM_WIDTH);
  VSec addr_phy_v, addr_phy_sv, addr_vir_v, addr_vir_sv, ts_bits_v;
  if (t_phy > 0) {
    append_polycomm(t, "poly_commitment", pf.addr_comm_phy_mems);
    append_polycomm(t, "poly_commitment", pf.addr_comm_phy_mems_shifted);
    addr_phy_v = vsec({PHY_MEM_WIDTH}, {t_phy}, {pf.addr_comm_phy_mems});
    addr_phy_sv = vsec({PHY_MEM_WIDTH}, {t_phy}, {pf.addr_comm_phy_mems_shifted});
  }
  if (t_vir > 0) {
    append_polycomm(t, "poly_commitment", pf.addr_comm_vir_mems);
    append_polycomm(t, "poly_commitment", pf.addr_comm_vir_mems_shifted);
    append_polycomm(t, "poly_commitment", pf.addr_comm_ts_bits);
    addr_vir_v = vsec({VIR_MEM_WIDTH}, {t_vir}, {pf.addr_comm_vir_mems});
    addr_vir_sv = vsec({VIR_MEM_WIDTH}, {t_vir}, {pf.addr_comm_vir_mems_shifted});
    ts_bits_v = vsec({in.mem_addr_ts_bits_size}, {t_vir}, {pf.addr_comm_ts_bits});
  }
  // BLOCK_CORRECTNESS_EXTRACT
  std::vector<size_t> w2sz;
  for (size_t p = 0; p < P; p++) w2sz.push_back(npow2(2 * niu + 2 * phy[order[p]] + 4 * vir[order[p]]));
  const VSec bv = vsec(bnv, bnp, pf.block_comm_vars_list), w0 = vsec({num_ios}, {1}, {c_w0}),
             bw2 = vsec(w2sz, bnp, pf.block_comm_w2_list), bw3 = vsec(std::vector<size_t>(P, 8), bnp, pf.block_comm_w3_list),
             bw3s = vsec(std::vector<size_t>(P, 8), bnp, pf.block_comm_w3_list_shifted);
  std::vector<FqV> ch;
  if (!v.r1cs(gpc, pf.block_sat, P, bmax, bnp, in.num_vars, {&bv, &w0, &bw2, &bw3, &bw3s}, block.max_num_cons,
              pf.block_bound, &ch))
    return false;
  auto bound_rp = [&](const FqV& list, const FqV& rp, const Fq bound[3], const std::vector<size_t>& index) {
    FqV a, b, c;
    for (size_t i : index) {
      if (3 * i + 2 >= list.size()) return false;
      a.push_back(list[3 * i]);
      b.push_back(list[3 * i + 1]);
      c.push_back(list[3 * i + 2]);
    }
    return fq_eq(dense_eval_host(a, rp), bound[0]) && fq_eq(dense_eval_host(b, rp), bound[1]) &&
           fq_eq(dense_eval_host(c, rp), bound[2]);
  };
  {
    const FqV &rp = ch[0], &rx = ch[2], &ry = ch[3];
    if (pf.block_evals.size() != 3 * block.num_instances) return v.fail("block evaluation count");
    if (!bound_rp(pf.block_evals, rp, pf.block_bound, order)) return v.fail("block rp-bound evaluations");
    for (auto& e : pf.block_evals) t.scalar("ABCr_claim", e);
    t.challenge("challenge_c0");
    t.challenge("challenge_c1");
    t.challenge("challenge_c2");
    if (pf.block_eval_proofs.size() != block.sparks->size()) return v.fail("block SPARK proof count");
    for (size_t i = 0; i < block.sparks->size(); i++) {
      FqV ev;
      for (auto l : (*block.label_map)[i]) ev.push_back(pf.block_evals[l]);
      if (!v.spark((*block.sparks)[i], pf.block_eval_proofs[i], rx, ry, ev)) return false;
    }
  }
  // PAIRWISE_CHECK (lib.rs:3474-3568)
  const VSec pe3 = vsec({8}, {consis}, {pf.perm_exec_comm_w3_list}), pe3s = vsec({8}, {consis}, {pf.perm_exec_comm_w3_shifted});
  const size_t pw_nv = std::max<size_t>(8, in.mem_addr_ts_bits_size);
  std::vector<size_t> pw_map, pw_map2;
  const VSec pw = VSec::merge({&pe3, &addr_phy_v, &addr_vir_v}, &pw_map);
  const VSec pws = VSec::merge({&pe3s, &addr_phy_sv, &addr_vir_sv}, &pw_map2);
  VSec pwb;
  {
    std::vector<const VSec*> comps(pw_map.size(), &w0);
    for (size_t i = 0; i < pw_map.size(); i++)
      if (pw_map[i] == 2) comps[i] = &ts_bits_v;
    pwb = VSec::concat(comps);
  }
  const size_t pairwise_size = std::max({consis, t_phy, t_vir});
  if (!v.r1cs(gpc, pf.pairwise_sat, pw.num_proofs.size(), pairwise_size, pw.num_proofs, pw_nv, {&pw, &pws, &pwb},
              pairwise.max_num_cons, pf.pairwise_bound, &ch))
    return false;
  {
    const FqV &rp = ch[0], &rx = ch[2], &ry = ch[3];
    if (pf.pairwise_evals.size() != 3 * pairwise.num_instances) return v.fail("pairwise evaluation count");
    if (!bound_rp(pf.pairwise_evals, rp, pf.pairwise_bound, pw_index)) return v.fail("pairwise rp-bound evaluations");
    for (auto& e : pf.pairwise_evals) t.scalar("ABCr_claim", e);
    t.challenge("challenge_c0");
    t.challenge("challenge_c1");
    t.challenge("challenge_c2");
    if (!v.spark((*pairwise.sparks)[0], pf.pairwise_eval_proof, rx, ry, pf.pairwise_evals)) return false;
  }
  // PERM_EXEC_ROOT, MEM_ADDR_ROOT (lib.rs:3569-3650)
  const VSec ex1 = vsec({num_ios}, {consis}, {pf.exec_comm_inputs[0]}), pw2 = vsec({num_ios}, {consis}, {pf.perm_exec_comm_w2_list});
  std::vector<size_t> mm;
  const VSec r1 = VSec::merge({&ex1, &init_phy_v, &init_vir_v, &addr_phy_v, &addr_vir_v}, &mm);
  const VSec r2 = VSec::merge({&pw2, &ms[0][0], &ms[1][0], &ms[2][0], &ms[3][0]}, &mm);
  const VSec r3 = VSec::merge({&pe3, &ms[0][1], &ms[1][1], &ms[2][1], &ms[3][1]}, &mm);
  const VSec r3s = VSec::merge({&pe3s, &ms[0][2], &ms[1][2], &ms[2][2], &ms[3][2]}, &mm);
  const size_t perm_size = std::max({consis, t_iphy, t_ivir, t_phy, t_vir});
  if (!v.r1cs(gpc, pf.perm_root_sat, r1.num_proofs.size(), perm_size, r1.num_proofs, num_ios, {&w0, &r1, &r2, &r3, &r3s},
              perm_root.max_num_cons, pf.perm_root_evals, &ch))
    return false;
  {
    const FqV &rx = ch[2], &ry = ch[3];
    t.scalar("Ar_claim", pf.perm_root_evals[0]);
    t.scalar("Br_claim", pf.perm_root_evals[1]);
    t.scalar("Cr_claim", pf.perm_root_evals[2]);
    const FqV e(pf.perm_root_evals, pf.perm_root_evals + 3);
    if (!v.spark((*perm_root.sparks)[0], pf.perm_root_eval_proof, rx, ry, e)) return false;
  }
  // PERM_PRODUCT openings and identities (lib.rs:3652-3772)
  {
    std::vector<const VSec*> comps = {&pe3, &ms[0][1], &ms[1][1], &ms[2][1], &ms[3][1], &bw3};
    if (in.max_block_num_phy_ops > 0) comps.push_back(&bw3);
    if (in.max_block_num_vir_ops > 0) comps.push_back(&bw3);
    std::vector<size_t> im;
    const VSec m = VSec::merge(comps, &im);
    if (pf.perm_poly_poly_list.size() != m.num_proofs.size()) return v.fail("perm product count");
    const size_t pm_bl_id = 6, vm_bl_id = in.max_block_num_phy_ops > 0 ? 7 : 6;
    std::vector<FqV> r_list;
    std::vector<size_t> nv_list;
    std::vector<const PolyComm*> cl;
    for (size_t i = 0; i < im.size(); i++) {
      if (im[i] == vm_bl_id) r_list.push_back({fq_one(), fq_one(), fq_zero()});
      else if (im[i] == pm_bl_id) r_list.push_back({fq_one(), fq_zero(), fq_zero()});
      else r_list.push_back({fq_one(), fq_zero()});
      nv_list.push_back(lg2(m.num_proofs[i] * 8));
      cl.push_back(&m.comm_w[i]);
    }
    if (!v.pe_plain_batched_instances(gpc, pf.perm_prod_proofs, r_list, pf.perm_poly_poly_list, cl, nv_list))
      return false;
    Fq pe = fq_one(), pb = fq_one(), pmb = fq_one(), pma = fq_one(), vmb = fq_one(), vma = fq_one();
    for (size_t i = 0; i < im.size(); i++) {
      const Fq& x = pf.perm_poly_poly_list[i];
      switch (im[i]) {
        case 0: pe = fq_mul(pe, x); break;
        case 1: pmb = fq_mul(pmb, x); break;
        case 2: vmb = fq_mul(vmb, x); break;
        case 3: pma = fq_mul(pma, x); break;
        case 4: vma = fq_mul(vma, x); break;
        case 5: pb = fq_mul(pb, x); break;
        case 6:
          if (in.max_block_num_phy_ops > 0) pmb = fq_mul(pmb, x);
          else vmb = fq_mul(vmb, x);
          break;
        case 7: vmb = fq_mul(vmb, x); break;
      }
    }
    if (!fq_eq(pe, pb)) return v.fail("execution / block permutation products");
    if (!fq_eq(pmb, pma)) return v.fail("physical memory permutation products");
    if (!fq_eq(vmb, vma)) return v.fail("virtual memory permutation products");
  }
  // SHIFT_PROOFS (lib.rs:3772-3853 -> ShiftProofs::verify :449-506)
  {
    std::vector<const PolyComm*> orig = {&pf.perm_exec_comm_w3_list}, shifted = {&pf.perm_exec_comm_w3_shifted};
    std::vector<size_t> sizes = {8 * consis}, hl = {6};
    for (size_t p = 0; p < P; p++) {
      orig.push_back(&pf.block_comm_w3_list[p]);
      shifted.push_back(&pf.block_comm_w3_list_shifted[p]);
      sizes.push_back(8 * bnp[p]);
      hl.push_back(8);
    }
    auto add = [&](const PolyComm& o, const PolyComm& sh, size_t size, size_t hh) {
      orig.push_back(&o);
      shifted.push_back(&sh);
      sizes.push_back(size);
      hl.push_back(hh);
    };
    if (t_iphy > 0) add(pf.mem_comm[0][1], pf.mem_comm[0][2], 8 * t_iphy, 6);
    if (t_ivir > 0) add(pf.mem_comm[1][1], pf.mem_comm[1][2], 8 * t_ivir, 6);
    if (t_phy > 0) {
      add(pf.addr_comm_phy_mems, pf.addr_comm_phy_mems_shifted, 4 * t_phy, 4);
      add(pf.mem_comm[2][1], pf.mem_comm[2][2], 8 * t_phy, 6);
    }
    if (t_vir > 0) {
      add(pf.addr_comm_vir_mems, pf.addr_comm_vir_mems_shifted, 8 * t_vir, 6);
      add(pf.mem_comm[3][1], pf.mem_comm[3][2], 8 * t_vir, 6);
    }
    if (pf.shift_openings.size() != orig.size() || pf.shift_orig_evals.size() != orig.size() ||
        pf.shift_shifted_evals.size() != orig.size())
      return v.fail("shift proof counts");
    for (size_t p = 0; p < hl.size(); p++) {
      if (pf.shift_openings[p].size() < hl[p]) return v.fail("shift proof header");
      for (size_t i = 0; i < hl[p]; i++) t.point("shift_header_entry", pf.shift_openings[p][i]);
    }
    const Fq c = t.challenge("challenge_c");
    std::vector<HExt> evals = decs(pf.shift_orig_evals);
    const std::vector<HExt> se = decs(pf.shift_shifted_evals);
    evals.insert(evals.end(), se.begin(), se.end());
    std::vector<const PolyComm*> comms(orig);
    comms.insert(comms.end(), shifted.begin(), shifted.end());
    std::vector<size_t> sz2(sizes);
    sz2.insert(sz2.end(), sizes.begin(), sizes.end());
    if (!v.pe_uni_batched(gpc, pf.shift_proof, c, evals, comms, sz2)) return false;
  }
  // IO_PROOFS (lib.rs:3855-3873 -> IOProofs::verify :283-359)
  {
    const size_t r_len = lg2(consis * num_ios);
    std::vector<uint8_t> live_flags(in.input_liveness, in.input_liveness + in.input_len);
    std::vector<size_t> idx;
    for (size_t i = 0; i + 2 < live_flags.size(); i++) idx.push_back(2 + in.input_offset + i);
    if (live_flags.size() > 1 && live_flags[1]) idx.insert(idx.begin(), 5);
    if (!live_flags.empty() && live_flags[0]) idx.insert(idx.begin(), 6);
    FqV live;
    for (size_t i = 0; i < live_flags.size() && i < input.size(); i++)
      if (live_flags[i]) live.push_back(input[i]);
    idx.resize(live.size());
    const size_t oe = in.output_exec_num * num_ios;
    std::vector<size_t> pts = {0, oe, 2, oe + 2 + (niu - 1), oe + 2 + (niu - 1) + in.output_offset - 1};
    pts.insert(pts.end(), idx.begin(), idx.end());
    std::vector<FqV> r_list;
    for (size_t p : pts) {
      FqV bits(r_len);
      for (size_t i = 0; i < r_len; i++) bits[i] = ((p >> (r_len - 1 - i)) & 1) ? fq_one() : fq_zero();
      r_list.push_back(bits);
    }
    FqV Zr = {fq_one(), fq_one(), fq_from_u64(in.input_block_num), fq_from_u64(in.output_block_num), output};
    Zr.insert(Zr.end(), live.begin(), live.end());
    if (!v.pe_plain_batched_points(gpc, pf.io_proofs, r_list, Zr, pf.exec_comm_inputs[0])) return false;
  }
  return true;
}

}  // namespace

// ------------------------------------------------------------------------------------ C-ABI
static int spg_snark_verify_impl(spg_ctx* ctx, const spg_snark_comp* block, const spg_snark_comp* pairwise,
                                const spg_snark_comp* perm_root, const spg_snark_inputs* inputs,
                                spg_r1cs_gens* vars_gens, spg_transcript* transcript, const uint8_t* proof,
                                size_t proof_len) {
  if (!ctx || !block || !pairwise || !perm_root || !inputs || !vars_gens || !transcript || (!proof && proof_len))
    return SPG_E_ARG;
  const spg_snark_inputs& in = *inputs;
  if (!in.block_num_instances_bound || !in.num_inputs_unpadded || !in.num_ios || !in.block_num_vars ||
      !in.block_num_proofs || !in.block_num_phy_ops || !in.block_num_vir_ops || (in.input_len && !in.input) ||
      !in.output || (in.input_len && !in.input_liveness))
    return set_err(ctx, SPG_E_ARG, "snark verify: public inputs incomplete");
  for (size_t b = 0; b < in.block_num_instances_bound; b++)  // SNARK::verify's assertion, src/lib.rs:2829-2831
    if (in.block_num_proofs[b] > in.block_max_num_proofs)
      return set_err(ctx, SPG_E_ARG, "snark verify: block_num_proofs[b] > block_max_num_proofs");
  SnarkCompView vb, vp, vr;
  if (snark_comp_view(block, &vb) || snark_comp_view(pairwise, &vp) || snark_comp_view(perm_root, &vr))
    return set_err(ctx, SPG_E_ARG, "snark verify: instance commitments incomplete");
  SPG_HIP(ctx, hipSetDevice(ctx->device));
  SnarkV pf;
  Rd r(proof, proof_len);
  if (!rd_snark(r, pf)) return set_err(ctx, SPG_E_VERIFY, "snark verify: malformed proof bytes");
  // the public values of this entry point: Montgomery limbs, and the init lists as full rows (column 3 = the value)
  SnarkPub pub;
  for (size_t i = 0; i < in.input_len; i++) pub.input.push_back(ld_fq(in.input + 4 * i));
  pub.output = ld_fq(in.output);
  if ((in.total_num_init_phy_mem_accesses && !in.init_phy_mems) || (in.total_num_init_vir_mem_accesses && !in.init_vir_mems))
    return set_err(ctx, SPG_E_ARG, "snark verify: init memory lists missing");
  for (size_t i = 0; i < in.total_num_init_phy_mem_accesses; i++)
    pub.stack.push_back(ld_fq(in.init_phy_mems + 4 * (i * INIT_PHY_MEM_WIDTH + 3)));
  for (size_t i = 0; i < in.total_num_init_vir_mem_accesses; i++)
    pub.mem.push_back(ld_fq(in.init_vir_mems + 4 * (i * INIT_VIR_MEM_WIDTH + 3)));
  SnarkVerifier v(ctx, transcript->t);
  bool ok = false;
  try {
    ok = snark_verify(v, pf, in, pub, vb, vp, vr, vars_gens->g);
  } catch (const Fail& f) {
    v.fail(f.what);
  }
  if (!ok) return set_err(ctx, SPG_E_VERIFY, std::string("snark verify: ") + (v.failed ? v.failed : "rejected"));
  return SPG_OK;
}

extern "C" int spg_snark_verify(spg_ctx* ctx, const spg_snark_comp* block, const spg_snark_comp* pairwise,
                                const spg_snark_comp* perm_root, const spg_snark_inputs* inputs,
                                spg_r1cs_gens* vars_gens, spg_transcript* transcript, const uint8_t* proof,
                                size_t proof_len) {
  if (!ctx || !transcript) return SPG_E_ARG;
  spg::HostPin pin;
  return spg::tr_status(ctx, transcript->t, spg_snark_verify_impl(ctx, block, pairwise, perm_root, inputs, vars_gens, transcript, proof, proof_len));
}

/* SparseMatPolyEvalProof::verify (src/sparse_mlpoly.rs:1566-1610) against the commitment held by s */
static int spg_spark_verify_impl(spg_ctx* ctx, spg_spark* S, const uint64_t* rx, size_t rx_len, const uint64_t* ry,
                                size_t ry_len, const uint64_t* evals_in, size_t n_evals, spg_transcript* transcript,
                                const uint8_t* proof, size_t proof_len) {
  if (!ctx || !S || !transcript || (!rx && rx_len) || (!ry && ry_len) || (!evals_in && n_evals) || (!proof && proof_len))
    return SPG_E_ARG;
  if (n_evals != S->B) return set_err(ctx, SPG_E_ARG, "spark verify: one evaluation per matrix");
  FqV ex, ey, evals(n_evals);
  for (size_t i = 0; i < rx_len; i++) ex.push_back(ld_fq(rx + 4 * i));
  for (size_t i = 0; i < ry_len; i++) ey.push_back(ld_fq(ry + 4 * i));
  for (size_t i = 0; i < n_evals; i++) evals[i] = ld_fq(evals_in + 4 * i);
  SPG_HIP(ctx, hipSetDevice(ctx->device));
  SparkV pf;
  Rd r(proof, proof_len);
  rd(r, pf);
  if (r.bad || r.o != r.n) return set_err(ctx, SPG_E_VERIFY, "spark verify: malformed proof bytes");
  SnarkVerifier v(ctx, transcript->t);
  bool ok = false;
  try {
    ok = v.spark(S, pf, ex, ey, evals);
  } catch (const Fail& f) {
    v.fail(f.what);
  }
  if (!ok) return set_err(ctx, SPG_E_VERIFY, std::string("spark verify: ") + (v.failed ? v.failed : "rejected"));
  return SPG_OK;
}

extern "C" int spg_spark_verify(spg_ctx* ctx, spg_spark* S, const uint64_t* rx, size_t rx_len, const uint64_t* ry,
                                size_t ry_len, const uint64_t* evals_in, size_t n_evals, spg_transcript* transcript,
                                const uint8_t* proof, size_t proof_len) {
  if (!ctx || !transcript) return SPG_E_ARG;
  spg::HostPin pin;
  return spg::tr_status(ctx, transcript->t, spg_spark_verify_impl(ctx, S, rx, rx_len, ry, ry_len, evals_in, n_evals, transcript, proof, proof_len));
}

extern "C" int spg_r1cs_gens_commit(spg_ctx* ctx, const spg_r1cs_gens* gens, const uint64_t* Z, size_t n, uint8_t* out,
                                    size_t out_cap, size_t* L_out) {
  if (!ctx || !gens || (!Z && n) || !L_out) return SPG_E_ARG;
  SPG_HIP(ctx, hipSetDevice(ctx->device));
  FqV z(n);
  for (size_t i = 0; i < n; i++) z[i] = ld_fq(Z + 4 * i);
  PolyComm c;
  try {
    c = commit_vec(ctx, const_cast<ProverGens&>(gens->g), z);
  } catch (const Fail& f) {
    return set_err(ctx, SPG_E_HIP, std::string("r1cs gens commit: ") + f.what);
  }
  *L_out = c.size();
  if (!out || 32 * c.size() > out_cap) return set_err(ctx, SPG_E_ARG, "r1cs gens commit: output buffer too small");
  for (size_t i = 0; i < c.size(); i++) memcpy(out + 32 * i, c[i].b, 32);
  return SPG_OK;
}

static int spg_r1cs_verify_impl(spg_ctx* ctx, const spg_r1cs_gens* gens, size_t num_instances, size_t max_num_proofs,
                               const size_t* num_proofs, size_t max_num_inputs, const spg_witness_comm* secs, size_t nws,
                               size_t num_cons, const uint64_t* evals, spg_transcript* transcript, const uint8_t* proof,
                               size_t proof_len, uint64_t* challenges_out, size_t* ch_lens) {
  if (!ctx || !gens || !num_instances || !num_proofs || !secs || !nws || !evals || !transcript || (!proof && proof_len))
    return SPG_E_ARG;
  if (!is_pow2(max_num_proofs) || !is_pow2(max_num_inputs) || !is_pow2(num_cons) || nws > 8)
    return set_err(ctx, SPG_E_ARG, "r1cs verify: sizes");
  // the round counts below take lg2 of these: a count that is not a power of two or exceeds its maximum would
  // index the challenge vectors out of range (R1CSProof::verify asserts the same shapes on the prover's side)
  for (size_t p = 0; p < num_instances; p++)
    if (!is_pow2(num_proofs[p]) || num_proofs[p] > max_num_proofs)
      return set_err(ctx, SPG_E_ARG, "r1cs verify: num_proofs[p] must be a power of two <= max_num_proofs");
  for (size_t i = 0; i < nws; i++) {
    const spg_witness_comm& c = secs[i];
    if (c.num_instances != 1 && c.num_instances != num_instances) return set_err(ctx, SPG_E_ARG, "r1cs verify: section instances");
    for (size_t p = 0; p < c.num_instances && c.num_proofs && c.num_inputs; p++)
      if (!is_pow2(c.num_proofs[p]) || c.num_proofs[p] > max_num_proofs || !is_pow2(c.num_inputs[p]) ||
          c.num_inputs[p] > max_num_inputs)
        return set_err(ctx, SPG_E_ARG, "r1cs verify: section shape (powers of two within the maxima)");
  }
  std::vector<VSec> vs(nws);
  std::vector<const VSec*> ws;
  for (size_t i = 0; i < nws; i++) {
    const spg_witness_comm& c = secs[i];
    if (!c.num_instances || !c.num_proofs || !c.num_inputs || !c.comm_len) return set_err(ctx, SPG_E_ARG, "r1cs verify: section");
    size_t o = 0;
    for (size_t p = 0; p < c.num_instances; p++) {
      vs[i].num_proofs.push_back(c.num_proofs[p]);
      vs[i].num_inputs.push_back(c.num_inputs[p]);
      PolyComm pc(c.comm_len[p]);
      for (size_t k = 0; k < c.comm_len[p]; k++) memcpy(pc[k].b, c.comms + 32 * (o + k), 32);
      o += c.comm_len[p];
      vs[i].comm_w.push_back(pc);
    }
    ws.push_back(&vs[i]);
  }
  const std::vector<size_t> np(num_proofs, num_proofs + num_instances);
  const Fq ev[3] = {ld_fq(evals), ld_fq(evals + 4), ld_fq(evals + 8)};
  SPG_HIP(ctx, hipSetDevice(ctx->device));
  R1CSProofP pf;
  Rd r(proof, proof_len);
  rd(r, pf);
  if (r.bad || r.o != r.n) return set_err(ctx, SPG_E_VERIFY, "r1cs verify: malformed proof bytes");
  SnarkVerifier v(ctx, transcript->t);
  std::vector<FqV> ch;
  bool ok = false;
  try {
    ok = v.r1cs(const_cast<ProverGens&>(gens->g), pf, num_instances, max_num_proofs, np, max_num_inputs, ws, num_cons,
                ev, &ch);
  } catch (const Fail& f) {
    v.fail(f.what);
  }
  if (!ok) return set_err(ctx, SPG_E_VERIFY, std::string("r1cs verify: ") + (v.failed ? v.failed : "rejected"));
  if (challenges_out && ch_lens) {
    size_t o = 0;
    for (int k = 0; k < 4; k++) {
      ch_lens[k] = ch[k].size();
      for (auto& x : ch[k]) st_fq(challenges_out + 4 * o++, x);
    }
  }
  return SPG_OK;
}

extern "C" int spg_r1cs_verify(spg_ctx* ctx, const spg_r1cs_gens* gens, size_t num_instances, size_t max_num_proofs,
                               const size_t* num_proofs, size_t max_num_inputs, const spg_witness_comm* secs, size_t nws,
                               size_t num_cons, const uint64_t* evals, spg_transcript* transcript, const uint8_t* proof,
                               size_t proof_len, uint64_t* challenges_out, size_t* ch_lens) {
  if (!ctx || !transcript) return SPG_E_ARG;
  spg::HostPin pin;
  return spg::tr_status(ctx, transcript->t, spg_r1cs_verify_impl(ctx, gens, num_instances, max_num_proofs, num_proofs, max_num_inputs, secs, nws, num_cons, evals, transcript, proof, proof_len, challenges_out, ch_lens));
}

// ------------------------------------------------------------------------------------ verifier from bytes
// SNARK::verify's commitment arguments (src/lib.rs:2781-2797: block_comm_map + block_comm_list + block_gens,
// pairwise_check_comm + pairwise_check_gens, perm_root_comm + perm_root_gens) as the verifier holds them: the
// bincode bytes of the ComputationCommitment(s) and the SNARKGens::new arguments, no sparse matrices.
extern "C" int spg_snark_comm_load(spg_ctx* ctx, const uint8_t* bytes, size_t len, int as_list, const size_t* map_idx,
                                   const size_t* map_lens, size_t n_map, size_t num_cons, size_t gens_num_cons,
                                   size_t gens_num_vars, size_t gens_num_instances, size_t gens_num_nz_entries,
                                   spg_snark_comp** out) {
  if (!ctx || !bytes || !out || !num_cons || !gens_num_cons || !gens_num_vars || !gens_num_instances ||
      !gens_num_nz_entries)
    return SPG_E_ARG;
  SPG_HIP(ctx, hipSetDevice(ctx->device));
  Rd r(bytes, len);
  const size_t n = as_list ? r.len(56) : 1;
  if (r.bad || n == 0) return set_err(ctx, SPG_E_ARG, "comm load: malformed commitment list");
  // SNARKGens::new -> R1CSCommitmentGens::new("gens_r1cs_eval", num_instances, num_cons, num_vars, num_nz_entries)
  // (src/lib.rs:164-185, src/r1csinstance.rs:39-56), as spg_snark_encode derives it
  const size_t Pg = npow2(gens_num_instances);
  const size_t gens_nvx = lg2(Pg) + lg2(npow2(gens_num_cons)), gens_nvy = lg2(npow2(gens_num_vars));
  const size_t gens_nnz = Pg * gens_num_nz_entries;
  static const char kLabel[] = "gens_r1cs_eval";
  std::vector<spg_spark*> sparks;
  size_t comm_cons = 0, comm_vars = 0;
  auto fail = [&](const char* why) {
    for (auto* S : sparks) spg_spark_free(ctx, S);
    return set_err(ctx, SPG_E_ARG, std::string("comm load: ") + why);
  };
  for (size_t g = 0; g < n; g++) {
    const size_t nc = (size_t)r.u64(), nv = (size_t)r.u64();  // R1CSCommitment { num_cons, num_vars, comm }
    const size_t B = (size_t)r.u64(), N = (size_t)r.u64(), cells = (size_t)r.u64();
    std::vector<Pt> ops = r.pts(), mem = r.pts();
    if (r.bad) return fail("malformed commitment bytes");
    if (g && (nc != comm_cons || nv != comm_vars)) return fail("commitments of one list disagree on num_cons / num_vars");
    comm_cons = nc;
    comm_vars = nv;
    spg_spark* S = nullptr;
    const int rc = spark_from_comm(ctx, B, N, cells, ops, mem, (const uint8_t*)kLabel, sizeof(kLabel) - 1, gens_nvx,
                                   gens_nvy, gens_nnz, 3, &S);
    if (rc) {
      for (auto* S2 : sparks) spg_spark_free(ctx, S2);
      return rc;
    }
    sparks.push_back(S);
  }
  if (r.o != r.n) return fail("trailing bytes");
  if (!is_pow2(num_cons) || comm_cons % num_cons || !is_pow2(comm_vars)) return fail("num_cons does not divide the commitment's");
  const size_t P = comm_cons / num_cons;
  // the matrix map: block_comm_map for a list, every matrix of the instance for a single commitment
  std::vector<std::vector<size_t>> label_map;
  if (as_list) {
    if (!map_idx || !map_lens || n_map != n) return fail("one map list per commitment");
    size_t o = 0;
    std::vector<int> seen(3 * P, 0);
    for (size_t g = 0; g < n; g++) {
      if (map_lens[g] != sparks[g]->B) return fail("map list length differs from the commitment's batch size");
      label_map.push_back(std::vector<size_t>(map_idx + o, map_idx + o + map_lens[g]));
      for (size_t k : label_map.back())
        if (k >= 3 * P || seen[k]++) return fail("map index out of range or repeated");
      o += map_lens[g];
    }
  } else {
    if (sparks[0]->B != 3 * P) return fail("a single commitment covers the 3 matrices of every instance");
    label_map.push_back({});
    for (size_t k = 0; k < 3 * P; k++) label_map[0].push_back(k);
  }
  for (auto* S : sparks)
    if (S->cells != ((size_t)1 << std::max<size_t>(std::max(lg2(num_cons), lg2(comm_vars)), 1)))
      return fail("SPARK memory size differs from num_cons / num_vars");
  *out = snark_comp_from_parts(P, num_cons, comm_vars, std::move(label_map), std::move(sparks));
  return SPG_OK;
}

namespace {
bool scalar_from_bytes(const uint8_t* b, Fq* out) {  // Scalar::from_bytes: canonical little-endian, else None
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int k = 0; k < 8; k++) w[i] |= (uint64_t)b[8 * i + k] << (8 * k);
  }
  Fq a;
  for (int i = 0; i < 8; i++) a.l[i] = (uint32_t)(w[i / 2] >> (32 * (i % 2)));
  const uint32_t Q[8] = {SPG_Q0, SPG_Q1, SPG_Q2, SPG_Q3, 0u, 0u, 0u, SPG_Q7};
  uint32_t br = 0;
  for (int i = 0; i < 8; i++) subb(a.l[i], Q[i], br, br);
  if (!br) return false;  // a >= q
  *out = fq_to_mont(a);
  return true;
}
}  // namespace

static int spg_snark_verify_public_impl(spg_ctx* ctx, const spg_snark_comp* block, const spg_snark_comp* pairwise,
                                        const spg_snark_comp* perm_root, const spg_snark_public* pb,
                                        spg_r1cs_gens* vars_gens, spg_transcript* transcript, const uint8_t* proof,
                                        size_t proof_len) {
  if (!ctx || !block || !pairwise || !perm_root || !pb || !vars_gens || !transcript || (!proof && proof_len))
    return SPG_E_ARG;
  const spg_snark_public& a = *pb;
  if (!a.block_num_instances_bound || !a.num_inputs_unpadded || !a.num_ios || !a.block_num_vars || !a.block_num_proofs ||
      !a.block_num_phy_ops || !a.block_num_vir_ops || (a.input_len && (!a.input || !a.input_liveness)) || !a.output ||
      (a.input_stack_len && !a.input_stack) || (a.input_mem_len && !a.input_mem))
    return set_err(ctx, SPG_E_ARG, "snark verify: public inputs incomplete");
  if (!a.consis_num_proofs) return set_err(ctx, SPG_E_ARG, "snark verify: consis_num_proofs must be positive");
  // the reference's assertions (src/lib.rs:3276-3281, 3305-3310): an init list's total is its padded length
  if (a.input_stack_len ? a.total_num_init_phy_mem_accesses != npow2(a.input_stack_len) : a.total_num_init_phy_mem_accesses)
    return set_err(ctx, SPG_E_ARG, "snark verify: total_num_init_phy_mem_accesses != input_stack.len().next_power_of_two()");
  if (a.input_mem_len ? a.total_num_init_vir_mem_accesses != npow2(a.input_mem_len) : a.total_num_init_vir_mem_accesses)
    return set_err(ctx, SPG_E_ARG, "snark verify: total_num_init_vir_mem_accesses != input_mem.len().next_power_of_two()");

  // Scalar::from_bytes(..).unwrap() on every public scalar (src/lib.rs:2836-2850): non-canonical bytes are rejected
  SnarkPub pub;
  Fq x;
  for (size_t i = 0; i < a.input_len; i++) {
    if (!scalar_from_bytes(a.input + 32 * i, &x)) return set_err(ctx, SPG_E_ARG, "snark verify: input not canonical");
    pub.input.push_back(x);
  }
  for (size_t i = 0; i < a.input_stack_len; i++) {
    if (!scalar_from_bytes(a.input_stack + 32 * i, &x)) return set_err(ctx, SPG_E_ARG, "snark verify: input_stack not canonical");
    pub.stack.push_back(x);
  }
  for (size_t i = 0; i < a.input_mem_len; i++) {
    if (!scalar_from_bytes(a.input_mem + 32 * i, &x)) return set_err(ctx, SPG_E_ARG, "snark verify: input_mem not canonical");
    pub.mem.push_back(x);
  }
  if (!scalar_from_bytes(a.output, &pub.output)) return set_err(ctx, SPG_E_ARG, "snark verify: output not canonical");
  for (size_t b = 0; b < a.block_num_instances_bound; b++)  // src/lib.rs:2829-2831
    if (a.block_num_proofs[b] > a.block_max_num_proofs)
      return set_err(ctx, SPG_E_ARG, "snark verify: block_num_proofs[b] > block_max_num_proofs");
  // the internal argument block (sizes only; the lists are in pub)
  spg_snark_inputs in;
  memset(&in, 0, sizeof in);
  in.input_block_num = a.input_block_num;
  in.output_block_num = a.output_block_num;
  in.input_liveness = a.input_liveness;
  in.input_len = a.input_len;
  in.func_input_width = a.func_input_width;
  in.input_offset = a.input_offset;
  in.output_offset = a.output_offset;
  in.output_exec_num = a.output_exec_num;
  in.num_vars = a.num_vars;
  in.num_ios = a.num_ios;
  in.max_block_num_phy_ops = a.max_block_num_phy_ops;
  in.block_num_phy_ops = a.block_num_phy_ops;
  in.max_block_num_vir_ops = a.max_block_num_vir_ops;
  in.block_num_vir_ops = a.block_num_vir_ops;
  in.mem_addr_ts_bits_size = a.mem_addr_ts_bits_size;
  in.num_inputs_unpadded = a.num_inputs_unpadded;
  in.block_num_vars = a.block_num_vars;
  in.block_num_instances_bound = a.block_num_instances_bound;
  in.block_max_num_proofs = a.block_max_num_proofs;
  in.block_num_proofs = a.block_num_proofs;
  in.consis_num_proofs = a.consis_num_proofs;
  in.total_num_init_phy_mem_accesses = a.total_num_init_phy_mem_accesses;
  in.total_num_init_vir_mem_accesses = a.total_num_init_vir_mem_accesses;
  in.total_num_phy_mem_accesses = a.total_num_phy_mem_accesses;
  in.total_num_vir_mem_accesses = a.total_num_vir_mem_accesses;
  SnarkCompView vb, vp, vr;
  if (snark_comp_view(block, &vb) || snark_comp_view(pairwise, &vp) || snark_comp_view(perm_root, &vr))
    return set_err(ctx, SPG_E_ARG, "snark verify: instance commitments incomplete");
  // the commitments' instance sizes are SNARK::verify's block_num_cons / pairwise_check_num_cons / perm_root_num_cons
  if (vb.max_num_cons != a.block_num_cons || vp.max_num_cons != a.pairwise_check_num_cons ||
      vr.max_num_cons != a.perm_root_num_cons)
    return set_err(ctx, SPG_E_ARG, "snark verify: num_cons arguments differ from the loaded commitments");
  SPG_HIP(ctx, hipSetDevice(ctx->device));
  SnarkV pf;
  Rd r(proof, proof_len);
  if (!rd_snark(r, pf)) return set_err(ctx, SPG_E_VERIFY, "snark verify: malformed proof bytes");
  SnarkVerifier v(ctx, transcript->t);
  bool ok = false;
  try {
    ok = snark_verify(v, pf, in, pub, vb, vp, vr, vars_gens->g);
  } catch (const Fail& f) {
    v.fail(f.what);
  }
  if (!ok) return set_err(ctx, SPG_E_VERIFY, std::string("snark verify: ") + (v.failed ? v.failed : "rejected"));
  return SPG_OK;
}

extern "C" int spg_snark_verify_public(spg_ctx* ctx, const spg_snark_comp* block, const spg_snark_comp* pairwise,
                                       const spg_snark_comp* perm_root, const spg_snark_public* pub,
                                       spg_r1cs_gens* vars_gens, spg_transcript* transcript, const uint8_t* proof,
                                       size_t proof_len) {
  if (!ctx || !transcript) return SPG_E_ARG;
  spg::HostPin pin;
  return spg::tr_status(ctx, transcript->t,
                        spg_snark_verify_public_impl(ctx, block, pairwise, perm_root, pub, vars_gens, transcript, proof,
                                                     proof_len));
}
