// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of PolyEvalProof (src/dense_mlpoly.rs:427-1189) and the Hyrax commit
// (src/dense_mlpoly.rs:184-256). HashMap lookups in the reference only group equal keys in
// first-seen order; a linear search over the insertion-ordered lists reproduces that exactly.
#pragma once
#include <vector>

#include "nizk.hpp"
#include "poly.hpp"

namespace orc {

typedef std::vector<CPt> PolyCommitment;

static inline void ser_polycomm(Ser& s, const PolyCommitment& c) { s.pts(c); }
// dense_mlpoly.rs:415-425
static inline void append_polycomm(Transcript& t, const char* label, const PolyCommitment& c) {
  t.append_message(label, "poly_commitment_begin");
  for (auto& p : c) t.append_point("poly_commitment_share", p.v);
  t.append_message(label, "poly_commitment_end");
}

// DensePolynomial::commit(gens, None) -> Hyrax rows with zero blinds (dense_mlpoly.rs:214-239)
static inline PolyCommitment poly_commit(const DensePoly& poly, const DotGens& g) {
  size_t ln, rn;
  eq_factored_lens(poly.num_vars, &ln, &rn);
  size_t L = pow2(ln), R = pow2(rn);
  PolyCommitment C;
  for (size_t i = 0; i < L; i++) {
    FqVec row(poly.Z.begin() + R * i, poly.Z.begin() + R * (i + 1));
    C.push_back(cpt(commitv(row, fq_zero(), g.gens_n)));
  }
  return C;
}

struct PolyEvalProof {
  DotProductProofLog proof;
  void ser(Ser& s) const { proof.ser(s); }

  // dense_mlpoly.rs:437-490 (blinds = None, blind_Zr = None)
  static PolyEvalProof prove(const DensePoly& poly, const FqVec& r, const Fq& Zr, const DotGens& g, Transcript& t,
                             RandomTape& tape, CPt* C_Zr) {
    t.append_protocol_name("polynomial evaluation proof");
    FqVec L, R;
    eq_factored_evals(r, &L, &R);
    FqVec LZ = poly.bound(L);
    Fq LZ_blind = fq_zero();
    for (size_t i = 0; i < L.size(); i++) LZ_blind = fq_add(LZ_blind, fq_mul(fq_zero(), L[i]));
    CPt cx;
    PolyEvalProof p;
    p.proof = DotProductProofLog::prove(g, t, tape, LZ, LZ_blind, R, Zr, fq_zero(), &cx, C_Zr);
    return p;
  }
  // dense_mlpoly.rs:492-527
  bool verify(const DotGens& g, Transcript& t, const FqVec& r, const CPt& C_Zr, const PolyCommitment& comm) const {
    t.append_protocol_name("polynomial evaluation proof");
    FqVec L, R;
    eq_factored_evals(r, &L, &R);
    std::vector<Ge> C;
    for (auto& c : comm) C.push_back(unpack(c));
    CPt C_LZ = cpt(msm_pts(L, C));
    return proof.verify(R.size(), g, t, R, C_LZ, C_Zr);
  }
  bool verify_plain(const DotGens& g, Transcript& t, const FqVec& r, const Fq& Zr, const PolyCommitment& comm) const {
    CPt C_Zr = cpt(commit1(Zr, fq_zero(), g.gens_1));
    return verify(g, t, r, C_Zr, comm);
  }

  // dense_mlpoly.rs:531-622
  static std::vector<PolyEvalProof> prove_batched_points(const DensePoly& poly, const std::vector<FqVec>& r_list,
                                                         const FqVec& Zr_list, const DotGens& g, Transcript& t,
                                                         RandomTape& tape) {
    t.append_protocol_name("polynomial evaluation proof");
    size_t ln, rn;
    eq_factored_lens(r_list[0].size(), &ln, &rn);
    std::vector<FqVec> keys, L_list, R_list;
    FqVec Zc;
    Fq c_base = t.challenge_scalar("challenge_c");
    Fq c = fq_one();
    for (size_t i = 0; i < r_list.size(); i++) {
      FqVec Li, Ri;
      eq_factored_evals(r_list[i], &Li, &Ri);
      FqVec key(r_list[i].begin(), r_list[i].begin() + ln);
      size_t idx = keys.size();
      for (size_t k = 0; k < keys.size(); k++)
        if (keys[k] == key) { idx = k; break; }
      if (idx < keys.size()) {
        c = fq_mul(c, c_base);
        for (size_t j = 0; j < R_list[idx].size(); j++) R_list[idx][j] = fq_add(R_list[idx][j], fq_mul(c, Ri[j]));
        Zc[idx] = fq_add(Zc[idx], fq_mul(c, Zr_list[i]));
      } else {
        keys.push_back(key);
        L_list.push_back(Li);
        R_list.push_back(Ri);
        Zc.push_back(Zr_list[i]);
      }
    }
    std::vector<PolyEvalProof> out;
    for (size_t i = 0; i < L_list.size(); i++) {
      FqVec LZ = poly.bound(L_list[i]);
      CPt cx, cy;
      PolyEvalProof p;
      p.proof = DotProductProofLog::prove(g, t, tape, LZ, fq_zero(), R_list[i], Zc[i], fq_zero(), &cx, &cy);
      out.push_back(p);
    }
    return out;
  }

  // dense_mlpoly.rs:689-780 (r may be padded with zeros at the front or trimmed from the front)
  static std::vector<PolyEvalProof> prove_batched_instances(const std::vector<const DensePoly*>& polys,
                                                            const std::vector<FqVec>& r_list, const FqVec& Zr_list,
                                                            const DotGens& g, Transcript& t, RandomTape& tape) {
    t.append_protocol_name("polynomial evaluation proof");
    std::vector<std::pair<size_t, FqVec>> keys;
    std::vector<FqVec> LZ_list, L_list, R_list;
    FqVec Zc;
    Fq c_base = t.challenge_scalar("challenge_c");
    Fq c = fq_one();
    for (size_t i = 0; i < polys.size(); i++) {
      const DensePoly& poly = *polys[i];
      size_t nv = poly.num_vars;
      FqVec r = r_list[i];
      if (nv >= r.size()) {
        FqVec pad(nv - r.size(), fq_zero());
        pad.insert(pad.end(), r.begin(), r.end());
        r = pad;
      } else {
        r = FqVec(r.end() - nv, r.end());
      }
      FqVec L, R;
      eq_factored_evals(r, &L, &R);
      size_t idx = keys.size();
      for (size_t k = 0; k < keys.size(); k++)
        if (keys[k].first == nv && keys[k].second == R) { idx = k; break; }
      if (idx < keys.size()) {
        c = fq_mul(c, c_base);
        FqVec LZ = poly.bound(L);
        for (size_t j = 0; j < LZ.size(); j++) LZ_list[idx][j] = fq_add(LZ_list[idx][j], fq_mul(c, LZ[j]));
        Zc[idx] = fq_add(Zc[idx], fq_mul(c, Zr_list[i]));
      } else {
        keys.push_back({nv, R});
        Zc.push_back(Zr_list[i]);
        LZ_list.push_back(poly.bound(L));
        L_list.push_back(L);
        R_list.push_back(R);
      }
    }
    std::vector<PolyEvalProof> out;
    for (size_t i = 0; i < LZ_list.size(); i++) {
      CPt cx, cy;
      PolyEvalProof p;
      p.proof = DotProductProofLog::prove(g, t, tape, LZ_list[i], fq_zero(), R_list[i], Zc[i], fq_zero(), &cx, &cy);
      out.push_back(p);
    }
    return out;
  }

  // dense_mlpoly.rs:861-960
  static std::vector<PolyEvalProof> prove_batched_instances_disjoint_rounds(
      const std::vector<const DensePoly*>& polys, const std::vector<size_t>& num_proofs_list,
      const std::vector<size_t>& num_inputs_list, const FqVec& rq, const FqVec& ry, const FqVec& Zr_list,
      const DotGens& g, Transcript& t, RandomTape& tape) {
    t.append_protocol_name("polynomial evaluation proof");
    std::vector<std::pair<size_t, size_t>> keys;
    std::vector<FqVec> LZ_list, L_list, R_list;
    FqVec Zc;
    Fq c_base = t.challenge_scalar("challenge_c");
    Fq c = fq_one();
    for (size_t i = 0; i < polys.size(); i++) {
      const DensePoly& poly = *polys[i];
      std::pair<size_t, size_t> key = {num_proofs_list[i], num_inputs_list[i]};
      size_t idx = keys.size();
      for (size_t k = 0; k < keys.size(); k++)
        if (keys[k] == key) { idx = k; break; }
      if (idx < keys.size()) {
        c = fq_mul(c, c_base);
        FqVec LZ = poly.bound(L_list[idx]);
        for (size_t j = 0; j < LZ.size(); j++) LZ_list[idx][j] = fq_add(LZ_list[idx][j], fq_mul(c, LZ[j]));
        Zc[idx] = fq_add(Zc[idx], fq_mul(c, Zr_list[i]));
      } else {
        keys.push_back(key);
        Zc.push_back(Zr_list[i]);
        size_t nvq = log_2(key.first), nvy = log_2(key.second);
        FqVec ry_short;
        if (nvy >= ry.size()) {
          ry_short.assign(nvy - ry.size(), fq_zero());
          ry_short.insert(ry_short.end(), ry.begin(), ry.end());
        } else {
          ry_short.assign(ry.end() - nvy, ry.end());
        }
        FqVec r(rq.end() - nvq, rq.end());
        r.insert(r.end(), ry_short.begin(), ry_short.end());
        FqVec L, R;
        eq_factored_evals(r, &L, &R);
        LZ_list.push_back(poly.bound(L));
        L_list.push_back(L);
        R_list.push_back(R);
      }
    }
    std::vector<PolyEvalProof> out;
    for (size_t i = 0; i < LZ_list.size(); i++) {
      CPt cx, cy;
      PolyEvalProof p;
      p.proof = DotProductProofLog::prove(g, t, tape, LZ_list[i], fq_zero(), R_list[i], Zc[i], fq_zero(), &cx, &cy);
      out.push_back(p);
    }
    return out;
  }

  // dense_mlpoly.rs:962-1044 : Zr_list are commitments (points)
  static bool verify_batched_instances_disjoint_rounds(const std::vector<PolyEvalProof>& proofs,
                                                       const std::vector<size_t>& num_proofs_list,
                                                       const std::vector<size_t>& num_inputs_list, const DotGens& g,
                                                       Transcript& t, const FqVec& rq, const FqVec& ry,
                                                       const std::vector<Ge>& Zr_list,
                                                       const std::vector<const PolyCommitment*>& comm_list) {
    t.append_protocol_name("polynomial evaluation proof");
    std::vector<std::pair<size_t, size_t>> keys;
    std::vector<Ge> LZ_list, Zc;
    std::vector<FqVec> L_list, R_list;
    Fq c_base = t.challenge_scalar("challenge_c");
    Fq c = fq_one();
    for (size_t i = 0; i < comm_list.size(); i++) {
      std::vector<Ge> C;
      for (auto& p : *comm_list[i]) C.push_back(unpack(p));
      std::pair<size_t, size_t> key = {num_proofs_list[i], num_inputs_list[i]};
      size_t idx = keys.size();
      for (size_t k = 0; k < keys.size(); k++)
        if (keys[k] == key) { idx = k; break; }
      if (idx < keys.size()) {
        c = fq_mul(c, c_base);
        Ge LZ = msm_pts(L_list[idx], C);
        uint8_t cb[32];
        fq_to_bytes(c, cb);
        LZ_list[idx] = ge_add(LZ_list[idx], ge_scalarmul_bytes(LZ, cb));
        Zc[idx] = ge_add(Zc[idx], ge_scalarmul_bytes(Zr_list[i], cb));
      } else {
        keys.push_back(key);
        Zc.push_back(Zr_list[i]);
        size_t nvq = log_2(key.first), nvy = log_2(key.second);
        FqVec ry_short;
        if (nvy >= ry.size()) {
          ry_short.assign(nvy - ry.size(), fq_zero());
          ry_short.insert(ry_short.end(), ry.begin(), ry.end());
        } else {
          ry_short.assign(ry.end() - nvy, ry.end());
        }
        FqVec r(rq.end() - nvq, rq.end());
        r.insert(r.end(), ry_short.begin(), ry_short.end());
        FqVec L, R;
        eq_factored_evals(r, &L, &R);
        LZ_list.push_back(msm_pts(L, C));
        L_list.push_back(L);
        R_list.push_back(R);
      }
    }
    if (LZ_list.size() != proofs.size()) return false;
    for (size_t i = 0; i < LZ_list.size(); i++)
      if (!proofs[i].proof.verify(R_list[i].size(), g, t, R_list[i], cpt(LZ_list[i]), cpt(Zc[i]))) return false;
    return true;
  }

  // dense_mlpoly.rs:1046-1130
  static PolyEvalProof prove_uni_batched_instances(const std::vector<const DensePoly*>& polys, const Fq& r,
                                                   const FqVec& Zr, const DotGens& g, Transcript& t,
                                                   RandomTape& tape, CPt* C_Zr) {
    t.append_protocol_name("polynomial evaluation proof");
    size_t max_nv = 0;
    for (auto p : polys) max_nv = std::max(max_nv, p->num_vars);
    size_t ln, rn;
    eq_factored_lens(max_nv, &ln, &rn);
    size_t R_size = pow2(rn);
    FqVec R;
    Fq rb = fq_one();
    for (size_t i = 0; i < R_size; i++) { R.push_back(rb); rb = fq_mul(rb, r); }
    std::vector<std::pair<size_t, FqVec>> Lmap;
    Fq c_base = t.challenge_scalar("challenge_c");
    Fq c = fq_one();
    FqVec LZc(R_size, fq_zero());
    Fq Zrc = fq_zero();
    for (size_t i = 0; i < polys.size(); i++) {
      size_t nv = polys[i]->num_vars;
      const FqVec* L = nullptr;
      for (auto& kv : Lmap) if (kv.first == nv) L = &kv.second;
      if (!L) {
        size_t l2, r2;
        eq_factored_lens(nv, &l2, &r2);
        Fq r_base = fq_one();
        for (size_t k = 0; k < pow2(r2); k++) r_base = fq_mul(r_base, r);
        FqVec Lv;
        Fq lb = fq_one();
        for (size_t k = 0; k < pow2(l2); k++) { Lv.push_back(lb); lb = fq_mul(lb, r_base); }
        Lmap.push_back({nv, Lv});
        L = &Lmap.back().second;
      }
      FqVec LZ = polys[i]->bound(*L);
      for (size_t k = 0; k < R_size; k++)
        if (k < LZ.size()) LZc[k] = fq_add(LZc[k], fq_mul(c, LZ[k]));
      Zrc = fq_add(Zrc, fq_mul(c, Zr[i]));
      c = fq_mul(c, c_base);
    }
    CPt cx;
    PolyEvalProof p;
    p.proof = DotProductProofLog::prove(g, t, tape, LZc, fq_zero(), R, Zrc, fq_zero(), &cx, C_Zr);
    return p;
  }
};

// c * P for a scalar c (Montgomery) and a point P
static inline Ge ge_mul_fq(const Ge& P, const Fq& c) {
  uint8_t cb[32];
  fq_to_bytes(c, cb);
  return ge_scalarmul_bytes(P, cb);
}

// PolyEvalProof::verify_plain_batched_points (src/dense_mlpoly.rs:624-680): one proof per distinct L (left half
// of r), the R vectors and claimed values of equal-L points combined with powers of challenge_c
static inline bool verify_plain_batched_points(const std::vector<PolyEvalProof>& proofs, const DotGens& g,
                                               Transcript& t, const std::vector<FqVec>& r_list, const FqVec& Zr_list,
                                               const PolyCommitment& comm) {
  t.append_protocol_name("polynomial evaluation proof");
  size_t ln, rn;
  eq_factored_lens(r_list[0].size(), &ln, &rn);
  std::vector<FqVec> keys, L_list, R_list;
  FqVec Zc;
  Fq c_base = t.challenge_scalar("challenge_c");
  Fq c = fq_one();
  for (size_t i = 0; i < r_list.size(); i++) {
    FqVec Li, Ri;
    eq_factored_evals(r_list[i], &Li, &Ri);
    FqVec key(r_list[i].begin(), r_list[i].begin() + ln);
    size_t idx = keys.size();
    for (size_t k = 0; k < keys.size(); k++)
      if (keys[k] == key) { idx = k; break; }
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
  if (L_list.size() != proofs.size()) return false;
  std::vector<Ge> C;
  for (auto& p : comm) C.push_back(unpack(p));
  for (size_t i = 0; i < L_list.size(); i++) {
    CPt C_Zc = cpt(commit1(Zc[i], fq_zero(), g.gens_1));
    CPt C_LZ = cpt(msm_pts(L_list[i], C));
    if (!proofs[i].proof.verify(R_list[i].size(), g, t, R_list[i], C_LZ, C_Zc)) return false;
  }
  return true;
}

// PolyEvalProof::verify_plain_batched_instances (src/dense_mlpoly.rs:782-858): one proof per (num_vars, R);
// the L.C of equal keys and their claimed values combined with powers of challenge_c
static inline bool verify_plain_batched_instances(const std::vector<PolyEvalProof>& proofs, const DotGens& g,
                                                  Transcript& t, const std::vector<FqVec>& r_list,
                                                  const FqVec& Zr_list, const std::vector<PolyCommitment>& comm_list,
                                                  const std::vector<size_t>& num_vars_list) {
  t.append_protocol_name("polynomial evaluation proof");
  if (comm_list.size() != r_list.size()) return false;
  std::vector<std::pair<size_t, FqVec>> keys;
  std::vector<Ge> LZ_list;
  FqVec Zc;
  std::vector<FqVec> R_list;
  Fq c_base = t.challenge_scalar("challenge_c");
  Fq c = fq_one();
  for (size_t i = 0; i < comm_list.size(); i++) {
    std::vector<Ge> C;
    for (auto& p : comm_list[i]) C.push_back(unpack(p));
    const size_t nv = num_vars_list[i];
    FqVec r;
    if (nv >= r_list[i].size()) {
      r.assign(nv - r_list[i].size(), fq_zero());
      r.insert(r.end(), r_list[i].begin(), r_list[i].end());
    } else {
      r.assign(r_list[i].end() - nv, r_list[i].end());
    }
    FqVec L, R;
    eq_factored_evals(r, &L, &R);
    std::pair<size_t, FqVec> key = {nv, R};
    size_t idx = keys.size();
    for (size_t k = 0; k < keys.size(); k++)
      if (keys[k] == key) { idx = k; break; }
    if (idx < keys.size()) {
      c = fq_mul(c, c_base);
      LZ_list[idx] = ge_add(LZ_list[idx], ge_mul_fq(msm_pts(L, C), c));
      Zc[idx] = fq_add(Zc[idx], fq_mul(c, Zr_list[i]));
    } else {
      keys.push_back(key);
      Zc.push_back(Zr_list[i]);
      LZ_list.push_back(msm_pts(L, C));
      R_list.push_back(R);
    }
  }
  if (LZ_list.size() != proofs.size()) return false;
  for (size_t i = 0; i < LZ_list.size(); i++) {
    CPt C_Zc = cpt(commit1(Zc[i], fq_zero(), g.gens_1));
    if (!proofs[i].proof.verify(R_list[i].size(), g, t, R_list[i], cpt(LZ_list[i]), C_Zc)) return false;
  }
  return true;
}

// PolyEvalProof::verify_uni_batched_instances (src/dense_mlpoly.rs:1132-1205): R = (1, r, r^2, ...), per num_vars
// L = (1, r^k, r^2k, ...) with k = |R_i|; L.C and the claimed-value commitments combined with powers of c
static inline bool verify_uni_batched_instances(const PolyEvalProof& pf, const DotGens& g, Transcript& t, const Fq& r,
                                                const std::vector<Ge>& C_Zr,
                                                const std::vector<const PolyCommitment*>& comm_list,
                                                const std::vector<size_t>& poly_size) {
  t.append_protocol_name("polynomial evaluation proof");
  size_t max_size = 0;
  for (auto s : poly_size) max_size = std::max(max_size, s);
  size_t ln, rn;
  eq_factored_lens(log_2(next_pow2(max_size)), &ln, &rn);
  FqVec R;
  Fq rb = fq_one();
  for (size_t i = 0; i < pow2(rn); i++) {
    R.push_back(rb);
    rb = fq_mul(rb, r);
  }
  std::vector<std::pair<size_t, FqVec>> Lmap;
  Fq c_base = t.challenge_scalar("challenge_c");
  Fq c = fq_one();
  Ge LZc = commit1(fq_zero(), fq_zero(), g.gens_1), Zrc = LZc;
  for (size_t i = 0; i < comm_list.size(); i++) {
    const size_t nv = log_2(next_pow2(poly_size[i]));
    const FqVec* L = nullptr;
    for (auto& kv : Lmap)
      if (kv.first == nv) L = &kv.second;
    if (!L) {
      size_t l2, r2;
      eq_factored_lens(nv, &l2, &r2);
      Fq r_base = fq_one();
      for (size_t k = 0; k < pow2(r2); k++) r_base = fq_mul(r_base, r);
      FqVec Lv;
      Fq lb = fq_one();
      for (size_t k = 0; k < pow2(l2); k++) {
        Lv.push_back(lb);
        lb = fq_mul(lb, r_base);
      }
      Lmap.push_back({nv, Lv});
      L = &Lmap.back().second;
    }
    std::vector<Ge> C;
    for (auto& p : *comm_list[i]) C.push_back(unpack(p));
    LZc = ge_add(LZc, ge_mul_fq(msm_pts(*L, C), c));
    Zrc = ge_add(Zrc, ge_mul_fq(C_Zr[i], c));
    c = fq_mul(c, c_base);
  }
  return pf.proof.verify(R.size(), g, t, R, cpt(LZc), cpt(Zrc));
}

static inline void ser_proofs(Ser& s, const std::vector<PolyEvalProof>& v) {
  s.u64(v.size());
  for (auto& p : v) p.ser(s);
}

}  // namespace orc
