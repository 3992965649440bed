// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of the SPARK sparse-polynomial commitment / evaluation argument:
//   src/product_tree.rs:11-108               ProductCircuit, DotProductCircuit
//   src/product_tree.rs:170-487              ProductCircuitEvalProofBatched::{prove, verify}
//   src/sparse_mlpoly.rs:39-209              Derefs, DerefsEvalProof
//   src/sparse_mlpoly.rs:212-271             AddrTimestamps
//   src/sparse_mlpoly.rs:273-339             MultiSparseMatPolynomialAsDense, SparseMatPolyCommitmentGens/Commitment
//   src/sparse_mlpoly.rs:354-426,566-597     sparse_to_dense_vecs, multi_sparse_to_dense_rep, multi_commit, deref
//   src/sparse_mlpoly.rs:599-762             Layers (hash layer + product circuits), PolyEvalNetwork
//   src/sparse_mlpoly.rs:764-1103            HashLayerProof::{prove, verify}
//   src/sparse_mlpoly.rs:1105-1356           ProductLayerProof::{prove, verify}
//   src/sparse_mlpoly.rs:1358-1467           PolyEvalNetworkProof::{prove, verify}
//   src/sparse_mlpoly.rs:1469-1610           SparseMatPolyEvalProof::{prove, verify}
//   src/r1csinstance.rs:645-780              next_power_of_eight, multi_commit, commit, R1CSEvalProof
#pragma once
#include <vector>

#include "r1cs.hpp"

namespace orc {

// ---------------------------------------------------------------- product trees (product_tree.rs)
struct ProductCircuit {
  std::vector<DensePoly> left_vec, right_vec;
  // product_tree.rs:18-58
  static ProductCircuit create(const DensePoly& poly) {
    ProductCircuit c;
    size_t num_layers = log_2(poly.len);
    DensePoly l, r;
    poly.split(poly.len / 2, &l, &r);
    c.left_vec.push_back(l);
    c.right_vec.push_back(r);
    for (size_t i = 0; i + 1 < num_layers; i++) {
      const DensePoly &L = c.left_vec[i], &R = c.right_vec[i];
      size_t len = L.len + R.len;
      FqVec ol, orr;
      for (size_t k = 0; k < len / 4; k++) ol.push_back(fq_mul(L[k], R[k]));
      for (size_t k = len / 4; k < len / 2; k++) orr.push_back(fq_mul(L[k], R[k]));
      c.left_vec.push_back(DensePoly(ol));
      c.right_vec.push_back(DensePoly(orr));
    }
    return c;
  }
  Fq evaluate() const { return fq_mul(left_vec.back()[0], right_vec.back()[0]); }
};

struct DotProductCircuit {
  DensePoly left, right, weight;
  Fq evaluate() const {
    Fq s = fq_zero();
    for (size_t i = 0; i < left.len; i++) s = fq_add(s, fq_mul(fq_mul(left[i], right[i]), weight[i]));
    return s;
  }
  void split(DotProductCircuit* a, DotProductCircuit* b) const {
    size_t idx = left.len / 2;
    left.split(idx, &a->left, &b->left);
    right.split(idx, &a->right, &b->right);
    weight.split(idx, &a->weight, &b->weight);
  }
};

struct LayerProofBatched {
  SumcheckProof proof;
  FqVec claims_prod_left, claims_prod_right;
  void ser(Ser& s) const {
    proof.ser(s);
    s.scs(claims_prod_left);
    s.scs(claims_prod_right);
  }
};

struct ProductCircuitEvalProofBatched {
  std::vector<LayerProofBatched> proof;
  FqVec claims_dotp[3];
  void ser(Ser& s) const {
    s.u64(proof.size());
    for (auto& p : proof) p.ser(s);
    for (int i = 0; i < 3; i++) s.scs(claims_dotp[i]);
  }

  // product_tree.rs:271-396
  static ProductCircuitEvalProofBatched prove(std::vector<ProductCircuit*>& prod, std::vector<DotProductCircuit*>& dotp,
                                              Transcript& t, FqVec* rand_out) {
    ProductCircuitEvalProofBatched out;
    size_t num_layers = prod[0]->left_vec.size();
    FqVec claims;
    for (auto c : prod) claims.push_back(c->evaluate());
    FqVec rand;
    for (size_t layer = num_layers; layer-- > 0;) {
      size_t len = prod[0]->left_vec[layer].len + prod[0]->right_vec[layer].len;
      DensePoly Cpar(eq_evals(rand));
      if (Cpar.len != len / 2) throw std::string("product circuit layer mismatch");
      size_t rounds = log_2(Cpar.len);
      std::vector<DensePoly*> Ap, Bp, As, Bs, Cs;
      for (auto c : prod) {
        Ap.push_back(&c->left_vec[layer]);
        Bp.push_back(&c->right_vec[layer]);
      }
      if (layer == 0 && !dotp.empty()) {
        for (auto d : dotp) claims.push_back(d->evaluate());
        for (auto d : dotp) {
          As.push_back(&d->left);
          Bs.push_back(&d->right);
          Cs.push_back(&d->weight);
        }
      }
      FqVec coeffs = t.challenge_vector("rand_coeffs_next_layer", claims.size());
      Fq claim = fq_zero();
      for (size_t i = 0; i < claims.size(); i++) claim = fq_add(claim, fq_mul(claims[i], coeffs[i]));
      FqVec r_prod;
      SumcheckProof sp = prove_cubic_batched(claim, rounds, Ap, Bp, Cpar, As, Bs, Cs, coeffs, t, &r_prod);
      LayerProofBatched lp;
      lp.proof = sp;
      for (size_t i = 0; i < prod.size(); i++) {
        lp.claims_prod_left.push_back((*Ap[i])[0]);
        lp.claims_prod_right.push_back((*Bp[i])[0]);
      }
      for (size_t i = 0; i < prod.size(); i++) {
        t.append_scalar("claim_prod_left", lp.claims_prod_left[i]);
        t.append_scalar("claim_prod_right", lp.claims_prod_right[i]);
      }
      if (layer == 0 && !dotp.empty()) {
        for (size_t i = 0; i < As.size(); i++) {
          out.claims_dotp[0].push_back((*As[i])[0]);
          out.claims_dotp[1].push_back((*Bs[i])[0]);
          out.claims_dotp[2].push_back((*Cs[i])[0]);
        }
        for (size_t i = 0; i < As.size(); i++) {
          t.append_scalar("claim_dotp_left", out.claims_dotp[0][i]);
          t.append_scalar("claim_dotp_right", out.claims_dotp[1][i]);
          t.append_scalar("claim_dotp_weight", out.claims_dotp[2][i]);
        }
      }
      Fq r_layer = t.challenge_scalar("challenge_r_layer");
      claims.clear();
      for (size_t i = 0; i < prod.size(); i++)
        claims.push_back(fq_add(lp.claims_prod_left[i],
                                fq_mul(r_layer, fq_sub(lp.claims_prod_right[i], lp.claims_prod_left[i]))));
      FqVec ext = {r_layer};
      ext.insert(ext.end(), r_prod.begin(), r_prod.end());
      rand = ext;
      out.proof.push_back(lp);
    }
    *rand_out = rand;
    return out;
  }

  // product_tree.rs:398-487 ; returns false on a failed check
  bool verify(const FqVec& claims_prod_vec, const FqVec& claims_dotp_vec, size_t len, Transcript& t, FqVec* claims_out,
              FqVec* claims_dotp_out, FqVec* rand_out) const {
    size_t num_layers = log_2(len);
    FqVec rand;
    if (proof.size() != num_layers) return false;
    FqVec claims = claims_prod_vec, claims_dotp_v;
    for (size_t i = 0; i < num_layers; i++) {
      if (i == num_layers - 1) claims.insert(claims.end(), claims_dotp_vec.begin(), claims_dotp_vec.end());
      FqVec coeffs = t.challenge_vector("rand_coeffs_next_layer", claims.size());
      Fq claim = fq_zero();
      for (size_t k = 0; k < claims.size(); k++) claim = fq_add(claim, fq_mul(claims[k], coeffs[k]));
      Fq claim_last;
      FqVec rand_prod;
      if (!proof[i].proof.verify(claim, i, 3, t, &claim_last, &rand_prod)) return false;
      const FqVec &L = proof[i].claims_prod_left, &R = proof[i].claims_prod_right;
      if (L.size() != claims_prod_vec.size() || R.size() != claims_prod_vec.size()) return false;
      for (size_t k = 0; k < claims_prod_vec.size(); k++) {
        t.append_scalar("claim_prod_left", L[k]);
        t.append_scalar("claim_prod_right", R[k]);
      }
      if (rand.size() != rand_prod.size()) return false;
      Fq eq = fq_one();
      for (size_t k = 0; k < rand.size(); k++)
        eq = fq_mul(eq, fq_add(fq_mul(rand[k], rand_prod[k]),
                               fq_mul(fq_sub(fq_one(), rand[k]), fq_sub(fq_one(), rand_prod[k]))));
      Fq expected = fq_zero();
      for (size_t k = 0; k < claims_prod_vec.size(); k++)
        expected = fq_add(expected, fq_mul(coeffs[k], fq_mul(fq_mul(L[k], R[k]), eq)));
      if (i == num_layers - 1) {
        size_t np = claims_prod_vec.size();
        for (size_t k = 0; k < claims_dotp[0].size(); k++) {
          t.append_scalar("claim_dotp_left", claims_dotp[0][k]);
          t.append_scalar("claim_dotp_right", claims_dotp[1][k]);
          t.append_scalar("claim_dotp_weight", claims_dotp[2][k]);
          expected = fq_add(expected, fq_mul(coeffs[k + np],
                                             fq_mul(fq_mul(claims_dotp[0][k], claims_dotp[1][k]), claims_dotp[2][k])));
        }
      }
      if (!(expected == claim_last)) return false;
      Fq r_layer = t.challenge_scalar("challenge_r_layer");
      claims.clear();
      for (size_t k = 0; k < L.size(); k++) claims.push_back(fq_add(L[k], fq_mul(r_layer, fq_sub(R[k], L[k]))));
      if (i == num_layers - 1) {
        for (size_t k = 0; k < claims_dotp_vec.size() / 2; k++) {
          for (int c = 0; c < 3; c++)
            claims_dotp_v.push_back(fq_add(claims_dotp[c][2 * k],
                                           fq_mul(r_layer, fq_sub(claims_dotp[c][2 * k + 1], claims_dotp[c][2 * k]))));
        }
      }
      FqVec ext = {r_layer};
      ext.insert(ext.end(), rand_prod.begin(), rand_prod.end());
      rand = ext;
    }
    *claims_out = claims;
    *claims_dotp_out = claims_dotp_v;
    *rand_out = rand;
    return true;
  }
};

// ---------------------------------------------------------------- dense representation (sparse_mlpoly.rs)
struct AddrTimestamps {
  std::vector<std::vector<size_t>> ops_addr_usize;
  std::vector<DensePoly> ops_addr, read_ts;
  DensePoly audit_ts;
  // sparse_mlpoly.rs:219-253
  static AddrTimestamps create(size_t num_cells, size_t num_ops, const std::vector<std::vector<size_t>>& ops_addr) {
    AddrTimestamps a;
    std::vector<size_t> audit(num_cells, 0);
    for (auto& inst : ops_addr) {
      if (inst.size() != num_ops) throw std::string("ops length");
      std::vector<size_t> read(num_ops, 0);
      for (size_t i = 0; i < num_ops; i++) {
        size_t addr = inst[i];
        if (addr >= num_cells) throw std::string("address out of range");
        read[i] = audit[addr];
        audit[addr] = read[i] + 1;
      }
      a.ops_addr.push_back(DensePoly::from_usize(inst));
      a.read_ts.push_back(DensePoly::from_usize(read));
    }
    a.ops_addr_usize = ops_addr;
    a.audit_ts = DensePoly::from_usize(audit);
    return a;
  }
  // sparse_mlpoly.rs:255-270
  std::vector<DensePoly> deref(const FqVec& mem_val) const {
    std::vector<DensePoly> out;
    for (auto& addr : ops_addr_usize) {
      FqVec v(addr.size());
      for (size_t i = 0; i < addr.size(); i++) v[i] = mem_val[addr[i]];
      out.push_back(DensePoly(v));
    }
    return out;
  }
};

struct MultiSparseDense {
  size_t batch_size = 0;
  std::vector<DensePoly> val;
  AddrTimestamps row, col;
  DensePoly comb_ops, comb_mem;
};

// sparse_mlpoly.rs:368-425
static inline MultiSparseDense multi_sparse_to_dense(const std::vector<const SparseMat*>& polys) {
  size_t N = 0;
  for (auto p : polys) N = std::max(N, p->num_nz_entries());
  MultiSparseDense d;
  d.batch_size = polys.size();
  std::vector<std::vector<size_t>> rows, cols;
  for (auto p : polys) {
    std::vector<size_t> r(N, 0), c(N, 0);
    FqVec v(N, fq_zero());
    for (size_t i = 0; i < p->M.size(); i++) {
      r[i] = p->M[i].row;
      c[i] = p->M[i].col;
      v[i] = p->M[i].val;
    }
    rows.push_back(r);
    cols.push_back(c);
    d.val.push_back(DensePoly(v));
  }
  size_t nvx = polys[0]->num_vars_x, nvy = polys[0]->num_vars_y;
  size_t cells = pow2(nvx > nvy ? nvx : nvy);
  d.row = AddrTimestamps::create(cells, N, rows);
  d.col = AddrTimestamps::create(cells, N, cols);
  std::vector<const DensePoly*> all;
  for (auto& p : d.row.ops_addr) all.push_back(&p);
  for (auto& p : d.row.read_ts) all.push_back(&p);
  for (auto& p : d.col.ops_addr) all.push_back(&p);
  for (auto& p : d.col.read_ts) all.push_back(&p);
  for (auto& p : d.val) all.push_back(&p);
  d.comb_ops = DensePoly::merge(all);
  d.comb_mem = d.row.audit_ts;
  d.comb_mem.extend(d.col.audit_ts);
  return d;
}

struct SparkGens {
  DotGens gens_ops, gens_mem, gens_derefs;
  // sparse_mlpoly.rs:289-317
  static SparkGens create(const char* label, size_t nvx, size_t nvy, size_t nnz, size_t batch) {
    SparkGens g;
    size_t nv_ops = log_2(next_pow2(nnz)) + log_2(next_pow2(batch * 5));
    size_t nv_mem = (nvx > nvy ? nvx : nvy) + 1;
    size_t nv_derefs = log_2(next_pow2(nnz)) + log_2(next_pow2(batch * 2));
    g.gens_ops = poly_commit_gens_new(nv_ops, label);
    g.gens_mem = poly_commit_gens_new(nv_mem, label);
    g.gens_derefs = poly_commit_gens_new(nv_derefs, label);
    return g;
  }
};

struct SparkCommitment {
  size_t batch_size = 0, num_ops = 0, num_mem_cells = 0;
  PolyCommitment comm_comb_ops, comm_comb_mem;
  void ser(Ser& s) const {
    s.u64(batch_size);
    s.u64(num_ops);
    s.u64(num_mem_cells);
    s.pts(comm_comb_ops);
    s.pts(comm_comb_mem);
  }
  // sparse_mlpoly.rs:327-339
  void append(Transcript& t) const {
    t.append_u64("batch_size", batch_size);
    t.append_u64("num_ops", num_ops);
    t.append_u64("num_mem_cells", num_mem_cells);
    append_polycomm(t, "comm_comb_ops", comm_comb_ops);
    append_polycomm(t, "comm_comb_mem", comm_comb_mem);
  }
};

// sparse_mlpoly.rs:566-587
static inline SparkCommitment spark_multi_commit(const std::vector<const SparseMat*>& polys, const SparkGens& g,
                                                 MultiSparseDense* dense) {
  *dense = multi_sparse_to_dense(polys);
  SparkCommitment c;
  c.batch_size = polys.size();
  c.num_mem_cells = dense->row.audit_ts.len;
  c.num_ops = dense->row.read_ts[0].len;
  c.comm_comb_ops = poly_commit(dense->comb_ops, g.gens_ops);
  c.comm_comb_mem = poly_commit(dense->comb_mem, g.gens_mem);
  return c;
}

struct Derefs {
  std::vector<DensePoly> row_ops_val, col_ops_val;
  DensePoly comb;
};

// n-to-1 reduction of claimed evaluations (sparse_mlpoly.rs:92-112 and :868-883): returns r_joint, eval
static inline void combine_n_to_one(const FqVec& evals, const FqVec& r, const char* chal_label, Transcript& t,
                                    FqVec* r_joint, Fq* eval) {
  FqVec ch = t.challenge_vector(chal_label, log_2(evals.size()));
  DensePoly pe(evals);
  for (size_t i = ch.size(); i-- > 0;) pe.bound_poly_var_bot(ch[i]);
  *eval = pe[0];
  *r_joint = ch;
  r_joint->insert(r_joint->end(), r.begin(), r.end());
}

struct HashLayerProof {
  FqVec eval_row_addr, eval_row_read_ts, eval_col_addr, eval_col_read_ts, eval_val, eval_row_ops_val,
      eval_col_ops_val;
  Fq eval_row_audit_ts, eval_col_audit_ts;
  PolyEvalProof proof_ops, proof_mem, proof_derefs;
  void ser(Ser& s) const {
    s.scs(eval_row_addr); s.scs(eval_row_read_ts); s.sc(eval_row_audit_ts);
    s.scs(eval_col_addr); s.scs(eval_col_read_ts); s.sc(eval_col_audit_ts);
    s.scs(eval_val);
    s.scs(eval_row_ops_val); s.scs(eval_col_ops_val);
    proof_ops.ser(s);
    proof_mem.ser(s);
    proof_derefs.ser(s);  // DerefsEvalProof { proof_derefs: PolyEvalProof }
  }
};

struct ProductLayerProof {
  Fq row_init, row_audit, col_init, col_audit;
  FqVec row_read, row_write, col_read, col_write, dotp_left, dotp_right;
  ProductCircuitEvalProofBatched proof_mem, proof_ops;
  void ser(Ser& s) const {
    s.sc(row_init); s.scs(row_read); s.scs(row_write); s.sc(row_audit);
    s.sc(col_init); s.scs(col_read); s.scs(col_write); s.sc(col_audit);
    s.scs(dotp_left); s.scs(dotp_right);
    proof_mem.ser(s);
    proof_ops.ser(s);
  }
};

struct SparkEvalProof {  // SparseMatPolyEvalProof
  PolyCommitment comm_derefs;
  ProductLayerProof prod;
  HashLayerProof hash;
  void ser(Ser& s) const {
    s.pts(comm_derefs);
    prod.ser(s);
    hash.ser(s);
  }
};

static inline FqVec prod_all(const FqVec& v) {
  Fq p = fq_one();
  for (auto& x : v) p = fq_mul(p, x);
  return {p};
}

// sparse_mlpoly.rs:612-687 hash layer, then ProductCircuit::new for each hashed polynomial
struct ProdLayer {
  ProductCircuit init, audit;
  std::vector<ProductCircuit> read, write;
};
static inline ProdLayer build_layers(const FqVec& eval_table, const AddrTimestamps& at,
                                     const std::vector<DensePoly>& derefs, const Fq& r_hash, const Fq& r_ms) {
  Fq r2 = fq_mul(r_hash, r_hash);
  auto hash = [&](const Fq& addr, const Fq& val, const Fq& ts) {
    return fq_sub(fq_add(fq_add(fq_mul(ts, r2), fq_mul(val, r_hash)), addr), r_ms);
  };
  size_t cells = eval_table.size();
  FqVec init(cells), audit(cells);
  for (size_t i = 0; i < cells; i++) {
    Fq a = fq_from_u64(i);
    init[i] = hash(a, eval_table[i], fq_zero());
    audit[i] = hash(a, eval_table[i], at.audit_ts[i]);
  }
  ProdLayer L;
  L.init = ProductCircuit::create(DensePoly(init));
  L.audit = ProductCircuit::create(DensePoly(audit));
  for (size_t k = 0; k < at.ops_addr.size(); k++) {
    const DensePoly &ad = at.ops_addr[k], &dv = derefs[k], &ts = at.read_ts[k];
    FqVec rd(ad.len), wr(ad.len);
    for (size_t i = 0; i < ad.len; i++) {
      rd[i] = hash(ad[i], dv[i], ts[i]);
      wr[i] = hash(ad[i], dv[i], fq_add(ts[i], fq_one()));
    }
    L.read.push_back(ProductCircuit::create(DensePoly(rd)));
    L.write.push_back(ProductCircuit::create(DensePoly(wr)));
  }
  return L;
}

// sparse_mlpoly.rs:1479-1495
static inline void spark_equalize(const FqVec& rx, const FqVec& ry, FqVec* ex, FqVec* ey) {
  *ex = rx;
  *ey = ry;
  if (rx.size() < ry.size()) ex->insert(ex->begin(), ry.size() - rx.size(), fq_zero());
  if (ry.size() < rx.size()) ey->insert(ey->begin(), rx.size() - ry.size(), fq_zero());
}

// sparse_mlpoly.rs:1497-1564 (+ PolyEvalNetworkProof :1368-1402, ProductLayerProof :1118-1263,
// HashLayerProof :805-918, DerefsEvalProof :80-146)
static inline SparkEvalProof spark_prove(const MultiSparseDense& dense, const FqVec& rx, const FqVec& ry,
                                         const FqVec& evals, const SparkGens& g, Transcript& t, RandomTape& tape) {
  t.append_protocol_name("Sparse polynomial evaluation proof");
  if (evals.size() != dense.batch_size) throw std::string("evals size");
  FqVec ex, ey;
  spark_equalize(rx, ry, &ex, &ey);
  FqVec mem_rx = eq_evals(ex), mem_ry = eq_evals(ey);
  Derefs d;
  d.row_ops_val = dense.row.deref(mem_rx);
  d.col_ops_val = dense.col.deref(mem_ry);
  {
    std::vector<const DensePoly*> all;
    for (auto& p : d.row_ops_val) all.push_back(&p);
    for (auto& p : d.col_ops_val) all.push_back(&p);
    d.comb = DensePoly::merge(all);
  }
  SparkEvalProof out;
  out.comm_derefs = poly_commit(d.comb, g.gens_derefs);
  t.append_message("derefs_commitment", "begin_derefs_commitment");
  append_polycomm(t, "comm_poly_row_col_ops_val", out.comm_derefs);
  t.append_message("derefs_commitment", "end_derefs_commitment");
  FqVec rmc = t.challenge_vector("challenge_r_hash", 2);
  ProdLayer rowL = build_layers(mem_rx, dense.row, d.row_ops_val, rmc[0], rmc[1]);
  ProdLayer colL = build_layers(mem_ry, dense.col, d.col_ops_val, rmc[0], rmc[1]);

  t.append_protocol_name("Sparse polynomial evaluation proof");  // PolyEvalNetworkProof
  // ---- product layer
  t.append_protocol_name("Sparse polynomial product layer proof");
  ProductLayerProof& P = out.prod;
  P.row_init = rowL.init.evaluate();
  P.row_audit = rowL.audit.evaluate();
  for (auto& c : rowL.read) P.row_read.push_back(c.evaluate());
  for (auto& c : rowL.write) P.row_write.push_back(c.evaluate());
  t.append_scalar("claim_row_eval_init", P.row_init);
  t.append_scalars("claim_row_eval_read", P.row_read);
  t.append_scalars("claim_row_eval_write", P.row_write);
  t.append_scalar("claim_row_eval_audit", P.row_audit);
  P.col_init = colL.init.evaluate();
  P.col_audit = colL.audit.evaluate();
  for (auto& c : colL.read) P.col_read.push_back(c.evaluate());
  for (auto& c : colL.write) P.col_write.push_back(c.evaluate());
  t.append_scalar("claim_col_eval_init", P.col_init);
  t.append_scalars("claim_col_eval_read", P.col_read);
  t.append_scalars("claim_col_eval_write", P.col_write);
  t.append_scalar("claim_col_eval_audit", P.col_audit);
  std::vector<DotProductCircuit> dl(evals.size()), dr(evals.size());
  for (size_t i = 0; i < evals.size(); i++) {
    DotProductCircuit full{d.row_ops_val[i], d.col_ops_val[i], dense.val[i]};
    full.split(&dl[i], &dr[i]);
    Fq el = dl[i].evaluate(), er = dr[i].evaluate();
    t.append_scalar("claim_eval_dotp_left", el);
    t.append_scalar("claim_eval_dotp_right", er);
    P.dotp_left.push_back(el);
    P.dotp_right.push_back(er);
  }
  size_t B = rowL.read.size();
  std::vector<ProductCircuit*> prod;
  std::vector<DotProductCircuit*> dotp;
  for (size_t i = 0; i < B; i++) {
    prod.push_back(&rowL.read[i]);
    dotp.push_back(&dl[i]);
    dotp.push_back(&dr[i]);
  }
  for (size_t i = 0; i < B; i++) prod.push_back(&rowL.write[i]);
  for (size_t i = 0; i < B; i++) prod.push_back(&colL.read[i]);
  for (size_t i = 0; i < B; i++) prod.push_back(&colL.write[i]);
  FqVec rand_ops, rand_mem;
  P.proof_ops = ProductCircuitEvalProofBatched::prove(prod, dotp, t, &rand_ops);
  std::vector<ProductCircuit*> mem = {&rowL.init, &rowL.audit, &colL.init, &colL.audit};
  std::vector<DotProductCircuit*> none;
  P.proof_mem = ProductCircuitEvalProofBatched::prove(mem, none, t, &rand_mem);

  // ---- hash layer
  t.append_protocol_name("Sparse polynomial hash layer proof");
  HashLayerProof& H = out.hash;
  for (auto& p : d.row_ops_val) H.eval_row_ops_val.push_back(p.evaluate(rand_ops));
  for (auto& p : d.col_ops_val) H.eval_col_ops_val.push_back(p.evaluate(rand_ops));
  {  // DerefsEvalProof::prove
    t.append_protocol_name("Derefs evaluation proof");
    FqVec ev = H.eval_row_ops_val;
    ev.insert(ev.end(), H.eval_col_ops_val.begin(), H.eval_col_ops_val.end());
    ev.resize(next_pow2(ev.size()), fq_zero());
    t.append_scalars("evals_ops_val", ev);
    FqVec rj;
    Fq ej;
    combine_n_to_one(ev, rand_ops, "challenge_combine_n_to_one", t, &rj, &ej);
    t.append_scalar("joint_claim_eval", ej);
    CPt cz;
    H.proof_derefs = PolyEvalProof::prove(d.comb, rj, ej, g.gens_derefs, t, tape, &cz);
  }
  for (auto& p : dense.row.ops_addr) H.eval_row_addr.push_back(p.evaluate(rand_ops));
  for (auto& p : dense.row.read_ts) H.eval_row_read_ts.push_back(p.evaluate(rand_ops));
  H.eval_row_audit_ts = dense.row.audit_ts.evaluate(rand_mem);
  for (auto& p : dense.col.ops_addr) H.eval_col_addr.push_back(p.evaluate(rand_ops));
  for (auto& p : dense.col.read_ts) H.eval_col_read_ts.push_back(p.evaluate(rand_ops));
  H.eval_col_audit_ts = dense.col.audit_ts.evaluate(rand_mem);
  for (auto& p : dense.val) H.eval_val.push_back(p.evaluate(rand_ops));
  {
    FqVec ev;
    for (auto* v : {&H.eval_row_addr, &H.eval_row_read_ts, &H.eval_col_addr, &H.eval_col_read_ts, &H.eval_val})
      ev.insert(ev.end(), v->begin(), v->end());
    ev.resize(next_pow2(ev.size()), fq_zero());
    t.append_scalars("claim_evals_ops", ev);
    FqVec rj;
    Fq ej;
    combine_n_to_one(ev, rand_ops, "challenge_combine_n_to_one", t, &rj, &ej);
    t.append_scalar("joint_claim_eval_ops", ej);
    CPt cz;
    H.proof_ops = PolyEvalProof::prove(dense.comb_ops, rj, ej, g.gens_ops, t, tape, &cz);
  }
  {
    FqVec ev = {H.eval_row_audit_ts, H.eval_col_audit_ts};
    t.append_scalars("claim_evals_mem", ev);
    FqVec rj;
    Fq ej;
    combine_n_to_one(ev, rand_mem, "challenge_combine_two_to_one", t, &rj, &ej);
    t.append_scalar("joint_claim_eval_mem", ej);
    CPt cz;
    H.proof_mem = PolyEvalProof::prove(dense.comb_mem, rj, ej, g.gens_mem, t, tape, &cz);
  }
  return out;
}

// sparse_mlpoly.rs:1566-1610 (+ the nested verifiers); false on any failed check
static inline bool spark_verify(const SparkEvalProof& pf, const SparkCommitment& comm, const FqVec& rx,
                                const FqVec& ry, const FqVec& evals, const SparkGens& g, Transcript& t) {
  t.append_protocol_name("Sparse polynomial evaluation proof");
  FqVec ex, ey;
  spark_equalize(rx, ry, &ex, &ey);
  if (pow2(ex.size()) != comm.num_mem_cells) return false;
  t.append_message("derefs_commitment", "begin_derefs_commitment");
  append_polycomm(t, "comm_poly_row_col_ops_val", pf.comm_derefs);
  t.append_message("derefs_commitment", "end_derefs_commitment");
  FqVec rmc = t.challenge_vector("challenge_r_hash", 2);
  const Fq r_hash = rmc[0], r_ms = rmc[1];
  t.append_protocol_name("Sparse polynomial evaluation proof");
  size_t B = evals.size(), num_ops = next_pow2(comm.num_ops), num_cells = pow2(ex.size());
  // ---- product layer
  const ProductLayerProof& P = pf.prod;
  t.append_protocol_name("Sparse polynomial product layer proof");
  if (P.row_read.size() != B || P.row_write.size() != B || P.col_read.size() != B || P.col_write.size() != B)
    return false;
  if (!(fq_mul(P.row_init, prod_all(P.row_write)[0]) == fq_mul(prod_all(P.row_read)[0], P.row_audit))) return false;
  t.append_scalar("claim_row_eval_init", P.row_init);
  t.append_scalars("claim_row_eval_read", P.row_read);
  t.append_scalars("claim_row_eval_write", P.row_write);
  t.append_scalar("claim_row_eval_audit", P.row_audit);
  if (!(fq_mul(P.col_init, prod_all(P.col_write)[0]) == fq_mul(prod_all(P.col_read)[0], P.col_audit))) return false;
  t.append_scalar("claim_col_eval_init", P.col_init);
  t.append_scalars("claim_col_eval_read", P.col_read);
  t.append_scalars("claim_col_eval_write", P.col_write);
  t.append_scalar("claim_col_eval_audit", P.col_audit);
  if (P.dotp_left.size() != B || P.dotp_right.size() != B) return false;
  FqVec claims_dotp_circuit;
  for (size_t i = 0; i < B; i++) {
    if (!(fq_add(P.dotp_left[i], P.dotp_right[i]) == evals[i])) return false;
    t.append_scalar("claim_eval_dotp_left", P.dotp_left[i]);
    t.append_scalar("claim_eval_dotp_right", P.dotp_right[i]);
    claims_dotp_circuit.push_back(P.dotp_left[i]);
    claims_dotp_circuit.push_back(P.dotp_right[i]);
  }
  FqVec claims_prod;
  for (auto* v : {&P.row_read, &P.row_write, &P.col_read, &P.col_write}) claims_prod.insert(claims_prod.end(), v->begin(), v->end());
  FqVec claims_ops, claims_dotp, rand_ops, claims_mem, claims_mem_dotp, rand_mem;
  if (!P.proof_ops.verify(claims_prod, claims_dotp_circuit, num_ops, t, &claims_ops, &claims_dotp, &rand_ops))
    return false;
  if (!P.proof_mem.verify({P.row_init, P.row_audit, P.col_init, P.col_audit}, {}, num_cells, t, &claims_mem,
                          &claims_mem_dotp, &rand_mem))
    return false;
  // ---- hash layer
  const HashLayerProof& H = pf.hash;
  t.append_protocol_name("Sparse polynomial hash layer proof");
  {
    t.append_protocol_name("Derefs evaluation proof");
    FqVec ev = H.eval_row_ops_val;
    ev.insert(ev.end(), H.eval_col_ops_val.begin(), H.eval_col_ops_val.end());
    ev.resize(next_pow2(ev.size()), fq_zero());
    t.append_scalars("evals_ops_val", ev);
    FqVec rj;
    Fq ej;
    combine_n_to_one(ev, rand_ops, "challenge_combine_n_to_one", t, &rj, &ej);
    t.append_scalar("joint_claim_eval", ej);
    if (!H.proof_derefs.verify_plain(g.gens_derefs, t, rj, ej, pf.comm_derefs)) return false;
  }
  if (claims_dotp.size() != 3 * H.eval_row_ops_val.size()) return false;
  for (size_t i = 0; i < claims_dotp.size() / 3; i++) {
    if (!(claims_dotp[3 * i] == H.eval_row_ops_val[i]) || !(claims_dotp[3 * i + 1] == H.eval_col_ops_val[i]) ||
        !(claims_dotp[3 * i + 2] == H.eval_val[i]))
      return false;
  }
  {
    FqVec ev;
    for (auto* v : {&H.eval_row_addr, &H.eval_row_read_ts, &H.eval_col_addr, &H.eval_col_read_ts, &H.eval_val})
      ev.insert(ev.end(), v->begin(), v->end());
    ev.resize(next_pow2(ev.size()), fq_zero());
    t.append_scalars("claim_evals_ops", ev);
    FqVec rj;
    Fq ej;
    combine_n_to_one(ev, rand_ops, "challenge_combine_n_to_one", t, &rj, &ej);
    t.append_scalar("joint_claim_eval_ops", ej);
    if (!H.proof_ops.verify_plain(g.gens_ops, t, rj, ej, comm.comm_comb_ops)) return false;
  }
  {
    FqVec ev = {H.eval_row_audit_ts, H.eval_col_audit_ts};
    t.append_scalars("claim_evals_mem", ev);
    FqVec rj;
    Fq ej;
    combine_n_to_one(ev, rand_mem, "challenge_combine_two_to_one", t, &rj, &ej);
    t.append_scalar("joint_claim_eval_mem", ej);
    if (!H.proof_mem.verify_plain(g.gens_mem, t, rj, ej, comm.comm_comb_mem)) return false;
  }
  // hash checks (sparse_mlpoly.rs:920-969)
  Fq r2 = fq_mul(r_hash, r_hash);
  auto hash = [&](const Fq& addr, const Fq& val, const Fq& ts) {
    return fq_sub(fq_add(fq_add(fq_mul(ts, r2), fq_mul(val, r_hash)), addr), r_ms);
  };
  auto check = [&](const FqVec& r, const Fq& cinit, const FqVec& cread, const FqVec& cwrite, const Fq& caudit,
                   const FqVec& ops_val, const FqVec& addr, const FqVec& rts, const Fq& ats) -> bool {
    Fq init_addr = identity_poly_evaluate(rand_mem);
    Fq init_val = eq_evaluate(r, rand_mem);
    if (!(hash(init_addr, init_val, fq_zero()) == cinit)) return false;
    for (size_t i = 0; i < addr.size(); i++) {
      if (!(hash(addr[i], ops_val[i], rts[i]) == cread[i])) return false;
      if (!(hash(addr[i], ops_val[i], fq_add(rts[i], fq_one())) == cwrite[i])) return false;
    }
    return hash(init_addr, init_val, ats) == caudit;
  };
  FqVec rr(claims_ops.begin(), claims_ops.begin() + B), rw(claims_ops.begin() + B, claims_ops.begin() + 2 * B),
      cr(claims_ops.begin() + 2 * B, claims_ops.begin() + 3 * B), cw(claims_ops.begin() + 3 * B, claims_ops.end());
  if (claims_mem.size() != 4) return false;
  if (!check(ex, claims_mem[0], rr, rw, claims_mem[1], H.eval_row_ops_val, H.eval_row_addr, H.eval_row_read_ts,
             H.eval_row_audit_ts))
    return false;
  return check(ey, claims_mem[2], cr, cw, claims_mem[3], H.eval_col_ops_val, H.eval_col_addr, H.eval_col_read_ts,
               H.eval_col_audit_ts);
}

}  // namespace orc
