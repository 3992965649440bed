// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of
//   src/sparse_mlpoly.rs:19-37,427-541  SparseMatPolynomial {evaluate_with_tables, multi_evaluate,
//                                        multiply_vec_disjoint_rounds, compute_eval_table_sparse_disjoint_rounds}
//   src/r1csinstance.rs:19-31,89-200     R1CSInstance::{new, sort}
//   src/r1csinstance.rs:363-436          multiply_vec_block
//   src/r1csinstance.rs:484-534          compute_eval_table_sparse_disjoint_rounds
//   src/r1csinstance.rs:583-641          multi_evaluate / multi_evaluate_bound_rp / evaluate
//   src/r1csproof.rs:45-80               R1CSSumcheckGens / R1CSGens::new
//   src/r1csproof.rs:210-685             R1CSProof::prove
//   src/r1csproof.rs:687-954             R1CSProof::verify
//   src/lib.rs:508-698                   ProverWitnessSecInfo (new / concat / merge)
#pragma once
#include <vector>

#include "polyeval.hpp"
#include "sumcheck.hpp"

namespace orc {

struct SparseEntry {
  size_t row, col;
  Fq val;
};
struct SparseMat {
  size_t num_vars_x = 0, num_vars_y = 0;
  std::vector<SparseEntry> M;
  size_t num_nz_entries() const { return next_pow2(M.size()); }
  // sparse_mlpoly.rs:427-436
  Fq evaluate_with_tables(const FqVec& erx, const FqVec& ery) const {
    Fq s = fq_zero();
    for (auto& e : M) s = fq_add(s, fq_mul(fq_mul(erx[e.row], ery[e.col]), e.val));
    return s;
  }
  // sparse_mlpoly.rs:454-472 : z[w][i] = col / max_num_cols, col % max_num_cols
  FqVec multiply_vec_disjoint_rounds(size_t num_rows, size_t max_num_cols, const std::vector<FqVec>& z) const {
    FqVec Mz(num_rows, fq_zero());
    for (auto& e : M) Mz[e.row] = fq_add(Mz[e.row], fq_mul(e.val, z[e.col / max_num_cols][e.col % max_num_cols]));
    return Mz;
  }
  // sparse_mlpoly.rs:524-541
  std::vector<FqVec> eval_table_disjoint_rounds(const FqVec& rx, size_t num_segs, size_t max_num_cols,
                                                size_t num_cols) const {
    std::vector<FqVec> out(num_segs, FqVec(num_cols, fq_zero()));
    for (auto& e : M) {
      Fq& d = out[e.col / max_num_cols][e.col % max_num_cols];
      d = fq_add(d, fq_mul(rx[e.row], e.val));
    }
    return out;
  }
};

// sparse_mlpoly.rs:438-450
static inline FqVec sparse_multi_evaluate(const std::vector<const SparseMat*>& polys, const FqVec& rx,
                                          const FqVec& ry) {
  FqVec erx = eq_evals(rx), ery = eq_evals(ry);
  FqVec out;
  for (auto p : polys) out.push_back(p->evaluate_with_tables(erx, ery));
  return out;
}

struct R1CSInstance {
  size_t num_instances = 0, max_num_cons = 0, num_vars = 0;
  std::vector<size_t> num_cons;
  std::vector<SparseMat> A, B, C;

  // r1csinstance.rs:89-182 (per-instance polys; the concatenated mat_* in the reference are unused)
  static R1CSInstance create(size_t num_instances, size_t max_num_cons, const std::vector<size_t>& num_cons,
                             size_t num_vars, const std::vector<std::vector<SparseEntry>>& Al,
                             const std::vector<std::vector<SparseEntry>>& Bl,
                             const std::vector<std::vector<SparseEntry>>& Cl) {
    R1CSInstance r;
    r.num_instances = num_instances;
    r.max_num_cons = max_num_cons;
    r.num_cons = num_cons;
    r.num_vars = num_vars;
    for (size_t i = 0; i < Al.size(); i++) {
      SparseMat a, b, c;
      a.num_vars_x = b.num_vars_x = c.num_vars_x = log_2(max_num_cons);
      a.num_vars_y = b.num_vars_y = c.num_vars_y = log_2(num_vars);
      a.M = Al[i]; b.M = Bl[i]; c.M = Cl[i];
      r.A.push_back(a); r.B.push_back(b); r.C.push_back(c);
    }
    return r;
  }
  // r1csinstance.rs:186-200
  void sort(size_t n, const std::vector<size_t>& index) {
    num_instances = n;
    std::vector<size_t> nc;
    std::vector<SparseMat> a, b, c;
    for (size_t i = 0; i < n; i++) {
      nc.push_back(num_cons[index[i]]);
      a.push_back(A[index[i]]); b.push_back(B[index[i]]); c.push_back(C[index[i]]);
    }
    num_cons = nc; A = a; B = b; C = c;
  }

  // r1csinstance.rs:363-436
  void multiply_vec_block(size_t P, const std::vector<size_t>& num_proofs, size_t max_num_proofs,
                          const std::vector<size_t>& num_inputs, size_t max_num_inputs, size_t max_nc,
                          const std::vector<size_t>& block_num_cons, const Mat4& z_mat, Pqx* Az, Pqx* Bz,
                          Pqx* Cz) const {
    Mat4 az(P), bz(P), cz(P);
    for (size_t p = 0; p < P; p++) {
      size_t pi = num_instances == 1 ? 0 : p;
      for (size_t q = 0; q < num_proofs[p]; q++) {
        const std::vector<FqVec>& z = z_mat[p][q];
        az[p].push_back({A[pi].multiply_vec_disjoint_rounds(block_num_cons[pi], max_num_inputs, z)});
        bz[p].push_back({B[pi].multiply_vec_disjoint_rounds(block_num_cons[pi], max_num_inputs, z)});
        cz[p].push_back({C[pi].multiply_vec_disjoint_rounds(block_num_cons[pi], max_num_inputs, z)});
      }
    }
    (void)num_inputs;
    *Az = Pqx::new_rev(az, num_proofs, max_num_proofs, block_num_cons, max_nc);
    *Bz = Pqx::new_rev(bz, num_proofs, max_num_proofs, block_num_cons, max_nc);
    *Cz = Pqx::new_rev(cz, num_proofs, max_num_proofs, block_num_cons, max_nc);
  }

  // r1csinstance.rs:583-596
  FqVec multi_evaluate(const FqVec& rx, const FqVec& ry) const {
    FqVec out;
    for (size_t i = 0; i < num_instances; i++) {
      FqVec e = sparse_multi_evaluate({&A[i], &B[i], &C[i]}, rx, ry);
      out.insert(out.end(), e.begin(), e.end());
    }
    return out;
  }
  // r1csinstance.rs:598-629
  void multi_evaluate_bound_rp(const FqVec& rp, const FqVec& rx, const FqVec& ry, FqVec* list, Fq out3[3]) const {
    FqVec a, b, c;
    list->clear();
    for (size_t i = 0; i < num_instances; i++) {
      FqVec e = sparse_multi_evaluate({&A[i], &B[i], &C[i]}, rx, ry);
      list->insert(list->end(), e.begin(), e.end());
      a.push_back(e[0]); b.push_back(e[1]); c.push_back(e[2]);
    }
    out3[0] = DensePoly(a).evaluate(rp);
    out3[1] = DensePoly(b).evaluate(rp);
    out3[2] = DensePoly(c).evaluate(rp);
  }
};

// lib.rs:508-604
struct WitnessSec {
  std::vector<size_t> num_inputs;
  std::vector<std::vector<FqVec>> w_mat;  // [p][q][i]
  std::vector<DensePoly> poly_w;
  static WitnessSec create(const std::vector<std::vector<FqVec>>& w_mat, const std::vector<DensePoly>& poly_w) {
    WitnessSec s;
    for (auto& m : w_mat) s.num_inputs.push_back(m[0].size());
    s.w_mat = w_mat;
    s.poly_w = poly_w;
    return s;
  }
  static WitnessSec concat(const std::vector<const WitnessSec*>& comps) {
    WitnessSec s;
    for (auto c : comps) {
      s.num_inputs.insert(s.num_inputs.end(), c->num_inputs.begin(), c->num_inputs.end());
      s.w_mat.insert(s.w_mat.end(), c->w_mat.begin(), c->w_mat.end());
      s.poly_w.insert(s.poly_w.end(), c->poly_w.begin(), c->poly_w.end());
    }
    return s;
  }
  static WitnessSec merge(const std::vector<const WitnessSec*>& comps, std::vector<size_t>* inst_map) {
    std::vector<size_t> ptr(comps.size(), 0);
    size_t total = 0;
    for (auto c : comps) total += c->num_inputs.size();
    WitnessSec s;
    inst_map->clear();
    while (inst_map->size() < total) {
      size_t best = 0, nc = 0;
      for (size_t i = 0; i < comps.size(); i++)
        if (ptr[i] < comps[i]->w_mat.size() && comps[i]->w_mat[ptr[i]].size() > best) {
          best = comps[i]->w_mat[ptr[i]].size();
          nc = i;
        }
      inst_map->push_back(nc);
      s.num_inputs.push_back(comps[nc]->num_inputs[ptr[nc]]);
      s.w_mat.push_back(comps[nc]->w_mat[ptr[nc]]);
      s.poly_w.push_back(comps[nc]->poly_w[ptr[nc]]);
      ptr[nc]++;
    }
    return s;
  }
};

struct R1CSGens {
  Gens gens_1, gens_3, gens_4;
  DotGens gens_pc;
  // r1csproof.rs:71-79
  static R1CSGens create(const char* label, size_t num_vars) {
    R1CSGens g;
    g.gens_pc = poly_commit_gens_new(log_2(num_vars), label);
    g.gens_1 = g.gens_pc.gens_1;
    g.gens_3 = gens_new(3, label);
    g.gens_4 = gens_new(4, label);
    return g;
  }
};

struct R1CSProof {
  ZKSumcheckProof sc1;
  CPt claims_phase2[4];
  KnowledgeProof pok_Cz;
  ProductProof proof_prod;
  EqualityProof eq1;
  ZKSumcheckProof sc2;
  std::vector<std::vector<CPt>> comm_vars_at_ry_list;
  CPt comm_vars_at_ry;
  std::vector<PolyEvalProof> proof_eval_vars_at_ry_list;
  EqualityProof eq2;

  void ser(Ser& s) const {
    sc1.ser(s);
    for (int i = 0; i < 4; i++) s.pt(claims_phase2[i]);
    pok_Cz.ser(s);
    proof_prod.ser(s);
    eq1.ser(s);
    sc2.ser(s);
    s.u64(comm_vars_at_ry_list.size());
    for (auto& v : comm_vars_at_ry_list) s.pts(v);
    s.pt(comm_vars_at_ry);
    ser_proofs(s, proof_eval_vars_at_ry_list);
    eq2.ser(s);
  }

  static FqVec prefix_list(size_t nws, const FqVec& rw) {
    Fq one = fq_one();
    switch (next_pow2(nws)) {
      case 1: return {one};
      case 2: return {fq_sub(one, rw[0]), rw[0]};
      case 4:
        return {fq_mul(fq_sub(one, rw[0]), fq_sub(one, rw[1])), fq_mul(fq_sub(one, rw[0]), rw[1]),
                fq_mul(rw[0], fq_sub(one, rw[1])), fq_mul(rw[0], rw[1])};
      default: {
        FqVec v;
        for (int i = 0; i < 8; i++) {
          Fq a = (i & 4) ? rw[0] : fq_sub(one, rw[0]);
          Fq b = (i & 2) ? rw[1] : fq_sub(one, rw[1]);
          Fq c = (i & 1) ? rw[2] : fq_sub(one, rw[2]);
          v.push_back(fq_mul(fq_mul(a, b), c));
        }
        return v;
      }
    }
  }

  // r1csproof.rs:210-685. Returns challenges [rp, rq_rev, rx, rw || ry].
  static R1CSProof prove(size_t num_instances, size_t max_num_proofs, const std::vector<size_t>& num_proofs,
                         size_t max_num_inputs, const std::vector<size_t>& num_inputs,
                         const std::vector<const WitnessSec*>& ws, const R1CSInstance& inst, const R1CSGens& gens,
                         Transcript& t, RandomTape& tape, std::vector<FqVec>* challenges) {
    t.append_protocol_name("R1CS proof");
    size_t nws = ws.size();
    size_t num_cons = inst.max_num_cons;
    std::vector<size_t> block_num_cons =
        inst.num_instances == 1 ? std::vector<size_t>(num_instances, inst.num_cons[0]) : inst.num_cons;
    // z_mat assembly (r1csproof.rs:278-293)
    Mat4 z_mat(num_instances);
    for (size_t p = 0; p < num_instances; p++) {
      for (size_t q = 0; q < num_proofs[p]; q++) {
        z_mat[p].push_back(std::vector<FqVec>(nws, FqVec(num_inputs[p], fq_zero())));
        for (size_t w = 0; w < nws; w++) {
          const WitnessSec* s = ws[w];
          size_t pw = s->w_mat.size() == 1 ? 0 : p;
          size_t qw = s->w_mat[pw].size() == 1 ? 0 : q;
          for (size_t i = 0; i < std::min(s->num_inputs[pw], num_inputs[p]); i++)
            z_mat[p][q][w][i] = s->w_mat[pw][qw][i];
        }
      }
    }
    size_t np = log_2(next_pow2(num_instances)), nq = log_2(max_num_proofs), nx = log_2(num_cons),
           nw = log_2(nws), ny = log_2(max_num_inputs);
    FqVec tau_p = t.challenge_vector("challenge_tau_p", np);
    FqVec tau_q = t.challenge_vector("challenge_tau_q", nq);
    FqVec tau_x = t.challenge_vector("challenge_tau_x", nx);
    DensePoly poly_tau_p(eq_evals(tau_p)), poly_tau_q(eq_evals(tau_q)), poly_tau_x(eq_evals(tau_x));
    Pqx Az, Bz, Cz;
    inst.multiply_vec_block(num_instances, num_proofs, max_num_proofs, num_inputs, max_num_inputs, num_cons,
                            block_num_cons, z_mat, &Az, &Bz, &Cz);
    R1CSProof pf;
    FqVec rx_all, claims1;
    Fq blind_post1;
    pf.sc1 = prove_phase1(nx + nq + np, nx, nq, np, num_proofs, block_num_cons, poly_tau_p, poly_tau_q, poly_tau_x,
                          Az, Bz, Cz, gens.gens_1, gens.gens_4, t, tape, &rx_all, &claims1, &blind_post1);
    Fq tau_claim = fq_mul(fq_mul(poly_tau_p[0], poly_tau_q[0]), poly_tau_x[0]);
    Fq Az_claim = Az.index(0, 0, 0, 0), Bz_claim = Bz.index(0, 0, 0, 0), Cz_claim = Cz.index(0, 0, 0, 0);
    Fq Az_blind = tape.random_scalar("Az_blind"), Bz_blind = tape.random_scalar("Bz_blind"),
       Cz_blind = tape.random_scalar("Cz_blind"), prod_blind = tape.random_scalar("prod_Az_Bz_blind");
    CPt comm_Cz;
    pf.pok_Cz = KnowledgeProof::prove(gens.gens_1, t, tape, Cz_claim, Cz_blind, &comm_Cz);
    CPt comm_Az, comm_Bz, comm_prod;
    Fq prod = fq_mul(Az_claim, Bz_claim);
    pf.proof_prod = ProductProof::prove(gens.gens_1, t, tape, Az_claim, Az_blind, Bz_claim, Bz_blind, prod, prod_blind,
                                        &comm_Az, &comm_Bz, &comm_prod);
    t.append_point("comm_Az_claim", comm_Az.v);
    t.append_point("comm_Bz_claim", comm_Bz.v);
    t.append_point("comm_Cz_claim", comm_Cz.v);
    t.append_point("comm_prod_Az_Bz_claims", comm_prod.v);
    Fq blind_expected1 = fq_mul(tau_claim, fq_sub(prod_blind, Cz_blind));
    Fq claim_post1 = fq_mul(fq_sub(fq_mul(Az_claim, Bz_claim), Cz_claim), tau_claim);
    CPt c1, c2;
    pf.eq1 = EqualityProof::prove(gens.gens_1, t, tape, claim_post1, blind_expected1, claim_post1, blind_post1, &c1, &c2);
    // split rx_all into rx_rev | rq_rev | rp
    FqVec rx_rev(rx_all.begin(), rx_all.begin() + nx), rq_rev(rx_all.begin() + nx, rx_all.begin() + nx + nq),
        rp(rx_all.begin() + nx + nq, rx_all.end());
    FqVec rx(rx_rev.rbegin(), rx_rev.rend()), rq(rq_rev.rbegin(), rq_rev.rend());

    // PHASE 2
    Fq r_A = t.challenge_scalar("challenge_Az"), r_B = t.challenge_scalar("challenge_Bz"),
       r_C = t.challenge_scalar("challenge_Cz");
    Fq claim2 = fq_add(fq_add(fq_mul(r_A, Az_claim), fq_mul(r_B, Bz_claim)), fq_mul(r_C, Cz_claim));
    Fq blind2 = fq_add(fq_add(fq_mul(r_A, Az_blind), fq_mul(r_B, Bz_blind)), fq_mul(r_C, Cz_blind));
    FqVec evals_rx = eq_evals(rx);
    Mat4 evals_ABC(inst.num_instances);
    for (size_t p = 0; p < inst.num_instances; p++) {
      auto eA = inst.A[p].eval_table_disjoint_rounds(evals_rx, nws, max_num_inputs, num_inputs[p]);
      auto eB = inst.B[p].eval_table_disjoint_rounds(evals_rx, nws, max_num_inputs, num_inputs[p]);
      auto eC = inst.C[p].eval_table_disjoint_rounds(evals_rx, nws, max_num_inputs, num_inputs[p]);
      evals_ABC[p].push_back(std::vector<FqVec>());
      for (size_t w = 0; w < nws; w++) {
        FqVec row;
        for (size_t i = 0; i < num_inputs[p]; i++)
          row.push_back(fq_add(fq_add(fq_mul(r_A, eA[w][i]), fq_mul(r_B, eB[w][i])), fq_mul(r_C, eC[w][i])));
        evals_ABC[p][0].push_back(row);
      }
    }
    Pqx ABC = Pqx::new_rev(evals_ABC, std::vector<size_t>(num_instances, 1), 1, num_inputs, max_num_inputs);
    Pqx Zp = Pqx::new_rev(z_mat, num_proofs, max_num_proofs, num_inputs, max_num_inputs);
    Zp.bound_vars_rq(rq_rev);
    DensePoly eq_p(eq_evals(rp));
    FqVec ry_all, claims2;
    Fq blind_post2;
    pf.sc2 = prove_phase2(claim2, blind2, ny + nw + np, ny, nw, np, inst.num_instances == 1, nws, num_inputs, eq_p, ABC,
                          Zp, gens.gens_1, gens.gens_4, t, tape, &ry_all, &claims2, &blind_post2);
    FqVec ry_rev(ry_all.begin(), ry_all.begin() + ny), rw(ry_all.begin() + ny, ry_all.begin() + ny + nw),
        rp2(ry_all.begin() + ny + nw, ry_all.end());
    FqVec ry(ry_rev.rbegin(), ry_rev.rend());

    // POLY COMMIT (r1csproof.rs:518-639)
    FqVec ry_factors(ny + 1, fq_one());
    for (size_t i = 0; i < ny; i++) ry_factors[i + 1] = fq_mul(ry_factors[i], fq_sub(fq_one(), ry[i]));
    std::vector<const DensePoly*> poly_list;
    std::vector<size_t> nproofs_list, ninputs_list;
    FqVec Zr_list;
    std::vector<FqVec> eval_list(nws);
    pf.comm_vars_at_ry_list.assign(nws, {});
    for (size_t i = 0; i < nws; i++) {
      const WitnessSec* w = ws[i];
      eval_list.push_back({});                 // reference pushes an extra empty Vec per section
      pf.comm_vars_at_ry_list.push_back({});   // (r1csproof.rs:541-542): serialized as-is
      for (size_t p = 0; p < w->w_mat.size(); p++) {
        poly_list.push_back(&w->poly_w[p]);
        nproofs_list.push_back(w->w_mat[p].size());
        ninputs_list.push_back(w->num_inputs[p]);
        FqVec ry_short;
        if (w->num_inputs[p] >= max_num_inputs) {
          ry_short.assign(log_2(w->num_inputs[p]) - log_2(max_num_inputs), fq_zero());
          ry_short.insert(ry_short.end(), ry.begin(), ry.end());
        } else {
          ry_short.assign(ry.begin() + (ny - log_2(w->num_inputs[p])), ry.end());
        }
        FqVec r(rq.begin() + (nq - log_2(nproofs_list.back())), rq.end());
        r.insert(r.end(), ry_short.begin(), ry_short.end());
        Fq ev = poly_list.back()->evaluate(r);
        Zr_list.push_back(ev);
        if (w->num_inputs[p] >= max_num_inputs) eval_list[i].push_back(ev);
        else eval_list[i].push_back(fq_mul(ev, ry_factors[ny - log_2(w->num_inputs[p])]));
        pf.comm_vars_at_ry_list[i].push_back(cpt(commit1(ev, fq_zero(), gens.gens_pc.gens_1)));
      }
    }
    pf.proof_eval_vars_at_ry_list = PolyEvalProof::prove_batched_instances_disjoint_rounds(
        poly_list, nproofs_list, ninputs_list, rq, ry, Zr_list, gens.gens_pc, t, tape);
    FqVec comb_list;
    FqVec prefix = prefix_list(nws, rw);
    for (size_t p = 0; p < num_instances; p++) {
      Fq comb = fq_zero();
      for (size_t i = 0; i < nws; i++) {
        size_t pw = ws[i]->w_mat.size() == 1 ? 0 : p;
        comb = fq_add(comb, fq_mul(prefix[i], eval_list[i][pw]));
      }
      for (size_t q = 0; q < nq - log_2(num_proofs[p]); q++) comb = fq_mul(comb, fq_sub(fq_one(), rq[q]));
      comb_list.push_back(comb);
    }
    Fq eval_vars_at_ry = DensePoly(comb_list).evaluate(rp2);
    pf.comm_vars_at_ry = cpt(commit1(eval_vars_at_ry, fq_zero(), gens.gens_pc.gens_1));
    Fq claim_post2 = fq_mul(fq_mul(claims2[0], claims2[1]), claims2[2]);
    pf.eq2 = EqualityProof::prove(gens.gens_pc.gens_1, t, tape, claim_post2, fq_zero(), claim_post2, blind_post2, &c1,
                                  &c2);
    pf.claims_phase2[0] = comm_Az;
    pf.claims_phase2[1] = comm_Bz;
    pf.claims_phase2[2] = comm_Cz;
    pf.claims_phase2[3] = comm_prod;
    FqVec rwry(rw);
    rwry.insert(rwry.end(), ry.begin(), ry.end());
    *challenges = {rp2, rq_rev, rx, rwry};
    return pf;
  }

  // r1csproof.rs:687-954 ; ws_comm[i][p] = commitment of witness sec i instance p, ws_num_proofs/num_inputs likewise
  bool verify(size_t num_instances, size_t max_num_proofs, const std::vector<size_t>& num_proofs,
              size_t max_num_inputs, const std::vector<std::vector<size_t>>& ws_num_inputs,
              const std::vector<std::vector<size_t>>& ws_num_proofs,
              const std::vector<std::vector<PolyCommitment>>& ws_comm, size_t num_cons, const R1CSGens& gens,
              const Fq evals[3], Transcript& t, std::vector<FqVec>* challenges = nullptr) const {
    t.append_protocol_name("R1CS proof");
    size_t nws = ws_comm.size();
    size_t np = log_2(next_pow2(num_instances)), nq = log_2(max_num_proofs), nx = log_2(num_cons),
           nw = log_2(nws), ny = log_2(max_num_inputs);
    FqVec tau_p = t.challenge_vector("challenge_tau_p", np);
    FqVec tau_q = t.challenge_vector("challenge_tau_q", nq);
    FqVec tau_x = t.challenge_vector("challenge_tau_x", nx);
    CPt claim1 = cpt(commit1(fq_zero(), fq_zero(), gens.gens_1));
    CPt post1;
    FqVec rx_all;
    if (!sc1.verify(claim1, nx + nq + np, 3, gens.gens_1, gens.gens_4, t, &post1, &rx_all)) return false;
    const CPt &cA = claims_phase2[0], &cB = claims_phase2[1], &cC = claims_phase2[2], &cP = claims_phase2[3];
    if (!pok_Cz.verify(gens.gens_1, t, cC)) return false;
    if (!proof_prod.verify(gens.gens_1, t, cA, cB, cP)) return false;
    t.append_point("comm_Az_claim", cA.v);
    t.append_point("comm_Bz_claim", cB.v);
    t.append_point("comm_Cz_claim", cC.v);
    t.append_point("comm_prod_Az_Bz_claims", cP.v);
    FqVec rx_rev(rx_all.begin(), rx_all.begin() + nx), rq_rev(rx_all.begin() + nx, rx_all.begin() + nx + nq),
        rp1(rx_all.begin() + nx + nq, rx_all.end());
    FqVec rq(rq_rev.rbegin(), rq_rev.rend());
    Fq tb = fq_mul(fq_mul(eq_evaluate(rp1, tau_p), eq_evaluate(rq_rev, tau_q)), eq_evaluate(rx_rev, tau_x));
    uint8_t tbb[32];
    fq_to_bytes(tb, tbb);
    CPt expected1 = cpt(ge_scalarmul_bytes(ge_sub(unpack(cP), unpack(cC)), tbb));
    if (!eq1.verify(gens.gens_1, t, expected1, post1)) return false;
    Fq r_A = t.challenge_scalar("challenge_Az"), r_B = t.challenge_scalar("challenge_Bz"),
       r_C = t.challenge_scalar("challenge_Cz");
    FqVec rs = {r_A, r_B, r_C};
    std::vector<Ge> cs = {unpack(cA), unpack(cB), unpack(cC)};
    CPt claim2 = cpt(msm_pts(rs, cs));
    CPt post2;
    FqVec ry_all;
    if (!sc2.verify(claim2, ny + nw + np, 3, gens.gens_1, gens.gens_4, t, &post2, &ry_all)) return false;
    FqVec ry_rev(ry_all.begin(), ry_all.begin() + ny), rw(ry_all.begin() + ny, ry_all.begin() + ny + nw),
        rp(ry_all.begin() + ny + nw, ry_all.end());
    FqVec ry(ry_rev.rbegin(), ry_rev.rend());
    Fq p_rp = eq_evaluate(rp, rp1);
    FqVec ry_factors(ny + 1, fq_one());
    for (size_t i = 0; i < ny; i++) ry_factors[i + 1] = fq_mul(ry_factors[i], fq_sub(fq_one(), ry[i]));
    std::vector<const PolyCommitment*> comm_list;
    std::vector<size_t> nproofs_list, ninputs_list;
    std::vector<Ge> comm_Zr;
    for (size_t i = 0; i < nws; i++)
      for (size_t p = 0; p < ws_num_proofs[i].size(); p++) {
        comm_list.push_back(&ws_comm[i][p]);
        nproofs_list.push_back(ws_num_proofs[i][p]);
        ninputs_list.push_back(ws_num_inputs[i][p]);
        comm_Zr.push_back(unpack(comm_vars_at_ry_list[i][p]));
      }
    if (!PolyEvalProof::verify_batched_instances_disjoint_rounds(proof_eval_vars_at_ry_list, nproofs_list,
                                                                 ninputs_list, gens.gens_pc, t, rq, ry, comm_Zr,
                                                                 comm_list))
      return false;
    FqVec prefix = prefix_list(nws, rw);
    std::vector<Ge> expected_list;
    for (size_t p = 0; p < num_instances; p++) {
      Ge comb = ge_identity();
      for (size_t i = 0; i < nws; i++) {
        size_t pw = ws_num_proofs[i].size() == 1 ? 0 : p;
        Ge c = unpack(comm_vars_at_ry_list[i][pw]);
        Fq f = ws_num_inputs[i][pw] >= max_num_inputs ? fq_one() : ry_factors[ny - log_2(ws_num_inputs[i][pw])];
        uint8_t b[32];
        fq_to_bytes(fq_mul(prefix[i], f), b);
        comb = ge_add(comb, ge_scalarmul_bytes(c, b));
      }
      Fq m = fq_one();
      for (size_t q = 0; q < nq - log_2(num_proofs[p]); q++) m = fq_mul(m, fq_sub(fq_one(), rq[q]));
      uint8_t mb[32];
      fq_to_bytes(m, mb);
      expected_list.push_back(ge_scalarmul_bytes(comb, mb));
    }
    FqVec EQ = eq_evals(rp);
    EQ.resize(num_instances);
    if (!(cpt(msm_pts(EQ, expected_list)) == comm_vars_at_ry)) return false;
    Fq k = fq_mul(fq_add(fq_add(fq_mul(r_A, evals[0]), fq_mul(r_B, evals[1])), fq_mul(r_C, evals[2])), p_rp);
    uint8_t kb[32];
    fq_to_bytes(k, kb);
    CPt expected2 = cpt(ge_scalarmul_bytes(unpack(comm_vars_at_ry), kb));
    bool ok = eq2.verify(gens.gens_1, t, expected2, post2);
    if (challenges) {  // [rp, rq_rev, rx, rw || ry] (r1csproof.rs:953)
      FqVec rx(rx_rev.rbegin(), rx_rev.rend()), rwry(rw);
      rwry.insert(rwry.end(), ry.begin(), ry.end());
      *challenges = {rp, rq_rev, rx, rwry};
    }
    return ok;
  }
};

}  // namespace orc
