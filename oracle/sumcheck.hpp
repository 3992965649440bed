// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of src/sumcheck.rs:
//   SumcheckInstanceProof::{verify :37-71, prove_cubic :193-262, prove_cubic_batched :264-434}
//   ZKSumcheckInstanceProof::{verify :94-189, prove_cubic_disjoint_rounds :788-1065,
//                             prove_cubic_with_additive_term_disjoint_rounds :1067-1380}
// The per-round kernels (eval at 0/2/3 and the fold) are exposed separately as well, so the GPU
// round kernels can be checked round by round.
#pragma once
#include <vector>

#include "nizk.hpp"
#include "poly.hpp"

namespace orc {

struct SumcheckProof {  // SumcheckInstanceProof { compressed_polys: Vec<CompressedUniPoly> }
  std::vector<FqVec> polys;
  void ser(Ser& s) const {
    s.u64(polys.size());
    for (auto& p : polys) s.scs(p);
  }
  // sumcheck.rs:37-71
  bool verify(Fq claim, size_t num_rounds, size_t degree_bound, Transcript& t, Fq* e_out, FqVec* r_out) const {
    Fq e = claim;
    if (polys.size() != num_rounds) return false;
    for (size_t i = 0; i < polys.size(); i++) {
      UniPoly p = UniPoly::decompress(polys[i], e);
      if (p.degree() != degree_bound) return false;
      if (fq_add(p.eval_at_zero(), p.eval_at_one()) != e) return false;
      p.append_to_transcript("poly", t);
      Fq r = t.challenge_scalar("challenge_nextround");
      r_out->push_back(r);
      e = p.evaluate(r);
    }
    *e_out = e;
    return true;
  }
};

struct ZKSumcheckProof {
  std::vector<CPt> comm_polys, comm_evals;
  std::vector<DotProductProof> proofs;
  void ser(Ser& s) const {
    s.pts(comm_polys);
    s.pts(comm_evals);
    s.u64(proofs.size());
    for (auto& p : proofs) p.ser(s);
  }
  // sumcheck.rs:94-189
  bool verify(const CPt& comm_claim, size_t num_rounds, size_t degree_bound, const Gens& g1, const Gens& gn,
              Transcript& t, CPt* final_comm, FqVec* r) const {
    if (comm_polys.size() != num_rounds || comm_evals.size() != num_rounds) return false;
    for (size_t i = 0; i < comm_polys.size(); i++) {
      t.append_point("comm_poly", comm_polys[i].v);
      Fq r_i = t.challenge_scalar("challenge_nextround");
      const CPt& ccpr = i == 0 ? comm_claim : comm_evals[i - 1];
      const CPt& ce = comm_evals[i];
      t.append_point("comm_claim_per_round", ccpr.v);
      t.append_point("comm_eval", ce.v);
      FqVec w = t.challenge_vector("combine_two_claims_to_one", 2);
      std::vector<Ge> P = {unpack(ccpr), unpack(ce)};
      CPt comm_target = cpt(msm_pts(w, P));
      FqVec a_sc(degree_bound + 1, fq_one());
      a_sc[0] = fq_add(a_sc[0], fq_one());
      FqVec a_ev(degree_bound + 1, fq_one());
      for (size_t j = 1; j < a_ev.size(); j++) a_ev[j] = fq_mul(a_ev[j - 1], r_i);
      FqVec a(a_sc.size());
      for (size_t j = 0; j < a.size(); j++) a[j] = fq_add(fq_mul(w[0], a_sc[j]), fq_mul(w[1], a_ev[j]));
      if (!proofs[i].verify(g1, gn, t, a, comm_polys[i], comm_target)) return false;
      r->push_back(r_i);
    }
    *final_comm = comm_evals.back();
    return true;
  }
};

// shared tail of one ZK sumcheck round (sumcheck.rs:1247-1370): commit the cubic, draw r_j, and after the
// caller's fold produce the DotProductProof of <poly, a> = w0*claim + w1*eval.
struct ZKRoundState {
  FqVec blinds_poly, blinds_evals;
  Fq claim, blind_claim;
  CPt comm_claim;
};

static inline UniPoly zk_round_poly(const Fq& e0, const Fq& e2, const Fq& e3, const Fq& claim) {
  FqVec ev = {e0, fq_sub(claim, e0), e2, e3};
  return UniPoly::from_evals(ev);
}

static inline void zk_round_finish(const UniPoly& poly, size_t j, const Fq& r_j, ZKRoundState& st, const Gens& g1,
                                   const Gens& g4, Transcript& t, RandomTape& tape, ZKSumcheckProof& out) {
  Fq eval = poly.evaluate(r_j);
  CPt comm_eval = cpt(commit1(eval, st.blinds_evals[j], g1));
  t.append_point("comm_claim_per_round", st.comm_claim.v);
  t.append_point("comm_eval", comm_eval.v);
  FqVec w = t.challenge_vector("combine_two_claims_to_one", 2);
  Fq target = fq_add(fq_mul(w[0], st.claim), fq_mul(w[1], eval));
  Fq blind_sc = j == 0 ? st.blind_claim : st.blinds_evals[j - 1];
  Fq blind = fq_add(fq_mul(w[0], blind_sc), fq_mul(w[1], st.blinds_evals[j]));
  size_t deg = poly.degree();
  FqVec a_sc(deg + 1, fq_one());
  a_sc[0] = fq_add(a_sc[0], fq_one());
  FqVec a_ev(deg + 1, fq_one());
  for (size_t k = 1; k < a_ev.size(); k++) a_ev[k] = fq_mul(a_ev[k - 1], r_j);
  FqVec a(deg + 1);
  for (size_t k = 0; k <= deg; k++) a[k] = fq_add(fq_mul(w[0], a_sc[k]), fq_mul(w[1], a_ev[k]));
  CPt cx, cy;
  DotProductProof pf =
      DotProductProof::prove(g1, g4, t, tape, poly.coeffs, st.blinds_poly[j], a, target, blind, &cx, &cy);
  out.proofs.push_back(pf);
  st.claim = eval;
  st.comm_claim = comm_eval;
  out.comm_evals.push_back(comm_eval);
}

// ---- phase 1 round evaluation (sumcheck.rs:1173-1245): returns e0, e2, e3 given the sumcheck-local
// num_proofs / num_cons (already halved for this round) and the current lengths.
static inline void phase1_round_evals(int mode, size_t instance_len, size_t proof_len, size_t cons_len,
                                      const std::vector<size_t>& num_proofs, const std::vector<size_t>& num_cons,
                                      const DensePoly& Ap, const DensePoly& Aq, const DensePoly& Ax, const Pqx& B,
                                      const Pqx& C, const Pqx& D, Fq* e0o, Fq* e2o, Fq* e3o) {
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (size_t p = 0; p < std::min(instance_len, num_proofs.size()); p++) {
    for (size_t q = 0; q < num_proofs[p]; q++) {
      size_t step_q = proof_len / num_proofs[p];
      size_t step_x = cons_len / num_cons[p];
      for (size_t x = 0; x < num_cons[p]; x++) {
        Fq a_lo = fq_mul(fq_mul(Ap[p], Aq[q * step_q]), Ax[x * step_x]);
        Fq a_hi;
        if (mode == MODE_P) a_hi = fq_mul(fq_mul(Ap[p + instance_len], Aq[q * step_q]), Ax[x * step_x]);
        else if (mode == MODE_Q) a_hi = fq_mul(fq_mul(Ap[p], Aq[q * step_q + proof_len]), Ax[x * step_x]);
        else a_hi = fq_mul(fq_mul(Ap[p], Aq[q * step_q]), Ax[x * step_x + cons_len]);
        Fq b_lo = B.index(p, q, 0, x), c_lo = C.index(p, q, 0, x), d_lo = D.index(p, q, 0, x);
        Fq b_hi = B.index_high(p, q, 0, x, mode), c_hi = C.index_high(p, q, 0, x, mode), d_hi = D.index_high(p, q, 0, x, mode);
        // comb(A,B,C,D) = A * (B*C - D)
        e0 = fq_add(e0, fq_mul(a_lo, fq_sub(fq_mul(b_lo, c_lo), d_lo)));
        Fq a2 = fq_sub(fq_add(a_hi, a_hi), a_lo), b2 = fq_sub(fq_add(b_hi, b_hi), b_lo);
        Fq c2 = fq_sub(fq_add(c_hi, c_hi), c_lo), d2 = fq_sub(fq_add(d_hi, d_hi), d_lo);
        e2 = fq_add(e2, fq_mul(a2, fq_sub(fq_mul(b2, c2), d2)));
        Fq a3 = fq_sub(fq_add(a2, a_hi), a_lo), b3 = fq_sub(fq_add(b2, b_hi), b_lo);
        Fq c3 = fq_sub(fq_add(c2, c_hi), c_lo), d3 = fq_sub(fq_add(d2, d_hi), d_lo);
        e3 = fq_add(e3, fq_mul(a3, fq_sub(fq_mul(b3, c3), d3)));
      }
    }
  }
  *e0o = e0; *e2o = e2; *e3o = e3;
}

// sumcheck.rs:1067-1380 (R1CS phase 1). Returns proof; r = challenges; claims = [Ap*Aq*Ax, B, C, D]
static inline ZKSumcheckProof prove_phase1(size_t num_rounds, size_t nx, size_t nq, size_t np,
                                           std::vector<size_t> num_proofs, std::vector<size_t> num_cons,
                                           DensePoly& Ap, DensePoly& Aq, DensePoly& Ax, Pqx& B, Pqx& C, Pqx& D,
                                           const Gens& g1, const Gens& g4, Transcript& t, RandomTape& tape,
                                           FqVec* r_out, FqVec* claims, Fq* blind_last) {
  ZKRoundState st;
  st.blinds_poly = tape.random_vector("blinds_poly", num_rounds);
  st.blinds_evals = tape.random_vector("blinds_evals", num_rounds);
  st.claim = fq_zero();
  st.blind_claim = fq_zero();
  st.comm_claim = cpt(commit1(st.claim, st.blind_claim, g1));
  ZKSumcheckProof out;
  size_t cons_len = pow2(nx), proof_len = pow2(nq), instance_len = pow2(np);
  for (size_t j = 0; j < num_rounds; j++) {
    int mode = j < nx ? MODE_X : (j < nx + nq ? MODE_Q : MODE_P);
    if (cons_len > 1) cons_len /= 2;
    else if (proof_len > 1) proof_len /= 2;
    else instance_len /= 2;
    for (size_t p = 0; p < std::min(instance_len, num_proofs.size()); p++) {
      if (mode == MODE_X && num_cons[p] > 1) num_cons[p] /= 2;
      if (mode == MODE_Q && num_proofs[p] > 1) num_proofs[p] /= 2;
    }
    Fq e0, e2, e3;
    phase1_round_evals(mode, instance_len, proof_len, cons_len, num_proofs, num_cons, Ap, Aq, Ax, B, C, D, &e0, &e2,
                       &e3);
    UniPoly poly = zk_round_poly(e0, e2, e3, st.claim);
    CPt comm_poly = cpt(commitv(poly.coeffs, st.blinds_poly[j], g4));
    t.append_point("comm_poly", comm_poly.v);
    out.comm_polys.push_back(comm_poly);
    Fq r_j = t.challenge_scalar("challenge_nextround");
    if (mode == MODE_P) Ap.bound_poly_var_top(r_j);
    else if (mode == MODE_Q) Aq.bound_poly_var_top(r_j);
    else Ax.bound_poly_var_top(r_j);
    B.bound_poly(r_j, mode);
    C.bound_poly(r_j, mode);
    D.bound_poly(r_j, mode);
    zk_round_finish(poly, j, r_j, st, g1, g4, t, tape, out);
    r_out->push_back(r_j);
  }
  *claims = {fq_mul(fq_mul(Ap[0], Aq[0]), Ax[0]), B.index(0, 0, 0, 0), C.index(0, 0, 0, 0), D.index(0, 0, 0, 0)};
  *blind_last = st.blinds_evals[num_rounds - 1];
  return out;
}

// ---- phase 2 round evaluation (sumcheck.rs:881-941)
static inline void phase2_round_evals(int mode, size_t instance_len, size_t witness_secs_len, size_t num_witness_secs,
                                      bool single_inst, const std::vector<size_t>& num_inputs, const DensePoly& A,
                                      const Pqx& B, const Pqx& C, Fq* e0o, Fq* e2o, Fq* e3o) {
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  for (size_t p = 0; p < std::min(instance_len, num_inputs.size()); p++) {
    size_t pi = single_inst ? 0 : p;
    for (size_t w = 0; w < std::min(witness_secs_len, num_witness_secs); w++) {
      for (size_t y = 0; y < num_inputs[p]; y++) {
        Fq a_lo = A[p];
        Fq a_hi = mode == MODE_P ? A[p + instance_len] : A[p];
        Fq b_lo = B.index(pi, 0, w, y), c_lo = C.index(p, 0, w, y);
        Fq b_hi = B.index_high(pi, 0, w, y, mode), c_hi = C.index_high(p, 0, w, y, mode);
        e0 = fq_add(e0, fq_mul(fq_mul(a_lo, b_lo), c_lo));
        Fq a2 = fq_sub(fq_add(a_hi, a_hi), a_lo), b2 = fq_sub(fq_add(b_hi, b_hi), b_lo), c2 = fq_sub(fq_add(c_hi, c_hi), c_lo);
        e2 = fq_add(e2, fq_mul(fq_mul(a2, b2), c2));
        Fq a3 = fq_sub(fq_add(a2, a_hi), a_lo), b3 = fq_sub(fq_add(b2, b_hi), b_lo), c3 = fq_sub(fq_add(c2, c_hi), c_lo);
        e3 = fq_add(e3, fq_mul(fq_mul(a3, b3), c3));
      }
    }
  }
  *e0o = e0; *e2o = e2; *e3o = e3;
}

// sumcheck.rs:788-1065 (R1CS phase 2). claims = [A, B(0,0,0,0), C(0,0,0,0)]
static inline ZKSumcheckProof prove_phase2(const Fq& claim, const Fq& blind_claim, size_t num_rounds, size_t ny,
                                           size_t nw, size_t np, bool single_inst, size_t num_witness_secs,
                                           std::vector<size_t> num_inputs, DensePoly& A, Pqx& B, Pqx& C,
                                           const Gens& g1, const Gens& g4, Transcript& t, RandomTape& tape,
                                           FqVec* r_out, FqVec* claims, Fq* blind_last) {
  ZKRoundState st;
  st.blinds_poly = tape.random_vector("blinds_poly", num_rounds);
  st.blinds_evals = tape.random_vector("blinds_evals", num_rounds);
  st.claim = claim;
  st.blind_claim = blind_claim;
  st.comm_claim = cpt(commit1(st.claim, st.blind_claim, g1));
  ZKSumcheckProof out;
  size_t inputs_len = pow2(ny), witness_secs_len = pow2(nw), instance_len = pow2(np);
  for (size_t j = 0; j < num_rounds; j++) {
    int mode = j < ny ? MODE_X : (j < ny + nw ? MODE_W : MODE_P);
    if (inputs_len > 1) inputs_len /= 2;
    else if (witness_secs_len > 1) witness_secs_len /= 2;
    else instance_len /= 2;
    for (size_t p = 0; p < std::min(instance_len, num_inputs.size()); p++)
      if (mode == MODE_X && num_inputs[p] > 1) num_inputs[p] /= 2;
    Fq e0, e2, e3;
    phase2_round_evals(mode, instance_len, witness_secs_len, num_witness_secs, single_inst, num_inputs, A, B, C, &e0,
                       &e2, &e3);
    UniPoly poly = zk_round_poly(e0, e2, e3, st.claim);
    CPt comm_poly = cpt(commitv(poly.coeffs, st.blinds_poly[j], g4));
    t.append_point("comm_poly", comm_poly.v);
    out.comm_polys.push_back(comm_poly);
    Fq r_j = t.challenge_scalar("challenge_nextround");
    if (mode == MODE_P) A.bound_poly_var_top(r_j);
    if (mode != MODE_P || !single_inst) B.bound_poly(r_j, mode);
    C.bound_poly(r_j, mode);
    zk_round_finish(poly, j, r_j, st, g1, g4, t, tape, out);
    r_out->push_back(r_j);
  }
  *claims = {A[0], B.index(0, 0, 0, 0), C.index(0, 0, 0, 0)};
  *blind_last = st.blinds_evals[num_rounds - 1];
  return out;
}

// ---- plain cubic sumcheck (sumcheck.rs:193-262), comb = A*B*C
static inline void cubic_round_evals(const DensePoly& A, const DensePoly& B, const DensePoly& C, Fq* e0o, Fq* e2o,
                                     Fq* e3o) {
  Fq e0 = fq_zero(), e2 = fq_zero(), e3 = fq_zero();
  size_t len = A.len / 2;
  for (size_t i = 0; i < len; i++) {
    e0 = fq_add(e0, fq_mul(fq_mul(A[i], B[i]), C[i]));
    Fq a2 = fq_sub(fq_add(A[len + i], A[len + i]), A[i]);
    Fq b2 = fq_sub(fq_add(B[len + i], B[len + i]), B[i]);
    Fq c2 = fq_sub(fq_add(C[len + i], C[len + i]), C[i]);
    e2 = fq_add(e2, fq_mul(fq_mul(a2, b2), c2));
    Fq a3 = fq_sub(fq_add(a2, A[len + i]), A[i]);
    Fq b3 = fq_sub(fq_add(b2, B[len + i]), B[i]);
    Fq c3 = fq_sub(fq_add(c2, C[len + i]), C[i]);
    e3 = fq_add(e3, fq_mul(fq_mul(a3, b3), c3));
  }
  *e0o = e0; *e2o = e2; *e3o = e3;
}

// sumcheck.rs:264-434 prove_cubic_batched with comb = A*B*C.
// par: (A_i, B_i) pairs sharing C_par; seq: independent (A, B, C) triples.
static inline SumcheckProof prove_cubic_batched(const Fq& claim, size_t num_rounds, std::vector<DensePoly*>& Apar,
                                                std::vector<DensePoly*>& Bpar, DensePoly& Cpar,
                                                std::vector<DensePoly*>& Aseq, std::vector<DensePoly*>& Bseq,
                                                std::vector<DensePoly*>& Cseq, const FqVec& coeffs, Transcript& t,
                                                FqVec* r_out) {
  SumcheckProof out;
  Fq e = claim;
  for (size_t j = 0; j < num_rounds; j++) {
    std::vector<Fq> E0, E2, E3;
    for (size_t i = 0; i < Apar.size(); i++) {
      Fq a, b, c;
      cubic_round_evals(*Apar[i], *Bpar[i], Cpar, &a, &b, &c);
      E0.push_back(a); E2.push_back(b); E3.push_back(c);
    }
    for (size_t i = 0; i < Aseq.size(); i++) {
      Fq a, b, c;
      cubic_round_evals(*Aseq[i], *Bseq[i], *Cseq[i], &a, &b, &c);
      E0.push_back(a); E2.push_back(b); E3.push_back(c);
    }
    Fq c0 = fq_zero(), c2 = fq_zero(), c3 = fq_zero();
    for (size_t i = 0; i < E0.size(); i++) {
      c0 = fq_add(c0, fq_mul(E0[i], coeffs[i]));
      c2 = fq_add(c2, fq_mul(E2[i], coeffs[i]));
      c3 = fq_add(c3, fq_mul(E3[i], coeffs[i]));
    }
    FqVec ev = {c0, fq_sub(e, c0), c2, c3};
    UniPoly poly = UniPoly::from_evals(ev);
    poly.append_to_transcript("poly", t);
    Fq r_j = t.challenge_scalar("challenge_nextround");
    r_out->push_back(r_j);
    for (size_t i = 0; i < Apar.size(); i++) { Apar[i]->bound_poly_var_top(r_j); Bpar[i]->bound_poly_var_top(r_j); }
    Cpar.bound_poly_var_top(r_j);
    for (size_t i = 0; i < Aseq.size(); i++) {
      Aseq[i]->bound_poly_var_top(r_j); Bseq[i]->bound_poly_var_top(r_j); Cseq[i]->bound_poly_var_top(r_j);
    }
    e = poly.evaluate(r_j);
    out.polys.push_back(poly.compress());
  }
  return out;
}

}  // namespace orc
