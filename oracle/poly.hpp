// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of the polynomial layer:
//   src/math.rs:14-21                     log_2 (rounds up for non powers of two)
//   src/dense_mlpoly.rs:59-130            EqPolynomial::{evaluate, evals, compute_factored_lens/evals}
//   src/dense_mlpoly.rs:132-148           IdentityPolynomial::evaluate
//   src/dense_mlpoly.rs:150-409           DensePolynomial (new pads to 2^k, split, bound, bound_poly_var_top/bot,
//                                         evaluate, extend, merge, from_usize)
//   src/custom_dense_mlpoly.rs:22-359     DensePolynomialPqx (ragged p, q_rev, w, x_rev tables)
//   src/unipoly.rs:23-120                 UniPoly / CompressedUniPoly
#pragma once
#include <algorithm>
#include <vector>

#include "fq.hpp"
#include "transcript.hpp"

namespace orc {

typedef std::vector<Fq> FqVec;

static inline size_t pow2(size_t k) { return (size_t)1 << k; }
// src/math.rs:14-21
static inline size_t log_2(size_t x) {
  size_t r = 0;
  while (((size_t)1 << r) < x) r++;
  return r;  // exact for powers of two, rounds up otherwise
}
static inline size_t next_pow2(size_t x) {
  size_t r = 1;
  while (r < x) r <<= 1;
  return r;
}

// ---------------------------------------------------------------- EqPolynomial
// dense_mlpoly.rs:68-73
static inline Fq eq_evaluate(const FqVec& r, const FqVec& rx) {
  Fq prod = fq_one();
  for (size_t i = 0; i < rx.size(); i++) {
    Fq t = fq_add(fq_mul(r[i], rx[i]), fq_mul(fq_sub(fq_one(), r[i]), fq_sub(fq_one(), rx[i])));
    prod = fq_mul(prod, t);
  }
  return prod;
}
// dense_mlpoly.rs:76-92
static inline FqVec eq_evals(const FqVec& r) {
  size_t ell = r.size();
  FqVec evals(pow2(ell), fq_one());
  size_t size = 1;
  for (size_t j = 0; j < ell; j++) {
    size *= 2;
    for (size_t i = size - 1;; i -= 2) {
      Fq scalar = evals[i / 2];
      evals[i] = fq_mul(scalar, r[j]);
      evals[i - 1] = fq_sub(scalar, evals[i]);
      if (i < 2) break;
    }
  }
  return evals;
}
// dense_mlpoly.rs:118-130
static inline void eq_factored_lens(size_t ell, size_t* l, size_t* r) { *l = ell / 2; *r = ell - ell / 2; }
static inline void eq_factored_evals(const FqVec& r, FqVec* L, FqVec* R) {
  size_t ell = r.size(), ln, rn;
  eq_factored_lens(ell, &ln, &rn);
  *L = eq_evals(FqVec(r.begin(), r.begin() + ln));
  *R = eq_evals(FqVec(r.begin() + ln, r.end()));
}
// dense_mlpoly.rs:141-147
static inline Fq identity_poly_evaluate(const FqVec& r) {
  size_t len = r.size();
  Fq s = fq_zero();
  for (size_t i = 0; i < len; i++) s = fq_add(s, fq_mul(fq_from_u64((uint64_t)pow2(len - i - 1)), r[i]));
  return s;
}

static inline Fq dot(const FqVec& a, const FqVec& b) {
  Fq s = fq_zero();
  for (size_t i = 0; i < a.size(); i++) s = fq_add(s, fq_mul(a[i], b[i]));
  return s;
}

// ---------------------------------------------------------------- DensePolynomial
struct DensePoly {
  size_t num_vars = 0, len = 0;
  FqVec Z;
  DensePoly() {}
  // dense_mlpoly.rs:151-161
  explicit DensePoly(FqVec z) {
    size_t np2 = next_pow2(z.size() ? z.size() : 1);
    if (z.empty()) np2 = 1;
    z.resize(np2, fq_zero());
    Z = std::move(z);
    len = Z.size();
    num_vars = log_2(len);
  }
  const Fq& operator[](size_t i) const { return Z[i]; }
  // dense_mlpoly.rs:175-181
  void split(size_t idx, DensePoly* a, DensePoly* b) const {
    *a = DensePoly(FqVec(Z.begin(), Z.begin() + idx));
    *b = DensePoly(FqVec(Z.begin() + idx, Z.begin() + 2 * idx));
  }
  // dense_mlpoly.rs:258-265
  FqVec bound(const FqVec& L) const {
    size_t ln, rn;
    eq_factored_lens(num_vars, &ln, &rn);
    size_t Ls = pow2(ln), Rs = pow2(rn);
    FqVec out(Rs);
    for (size_t i = 0; i < Rs; i++) {
      Fq s = fq_zero();
      for (size_t j = 0; j < Ls; j++) s = fq_add(s, fq_mul(L[j], Z[j * Rs + i]));
      out[i] = s;
    }
    return out;
  }
  // dense_mlpoly.rs:267-275
  void bound_poly_var_top(const Fq& r) {
    size_t n = len / 2;
    for (size_t i = 0; i < n; i++) Z[i] = fq_add(Z[i], fq_mul(r, fq_sub(Z[i + n], Z[i])));
    Z.resize(n);
    num_vars -= 1;
    len = n;
  }
  // dense_mlpoly.rs:350-358
  void bound_poly_var_bot(const Fq& r) {
    size_t n = len / 2;
    for (size_t i = 0; i < n; i++) Z[i] = fq_add(Z[2 * i], fq_mul(r, fq_sub(Z[2 * i + 1], Z[2 * i])));
    Z.resize(n);
    num_vars -= 1;
    len = n;
  }
  // dense_mlpoly.rs:361-367
  Fq evaluate(const FqVec& r) const {
    FqVec chis = eq_evals(r);
    return dot(Z, chis);
  }
  // dense_mlpoly.rs:373-383
  void extend(const DensePoly& o) {
    Z.insert(Z.end(), o.Z.begin(), o.Z.end());
    num_vars += 1;
    len *= 2;
  }
  // dense_mlpoly.rs:384-397
  static DensePoly merge(const std::vector<const DensePoly*>& polys) {
    FqVec z;
    for (auto p : polys) z.insert(z.end(), p->Z.begin(), p->Z.end());
    z.resize(next_pow2(z.size()), fq_zero());
    return DensePoly(z);
  }
  static DensePoly from_usize(const std::vector<size_t>& v) {
    FqVec z(v.size());
    for (size_t i = 0; i < v.size(); i++) z[i] = fq_from_u64((uint64_t)v[i]);
    return DensePoly(z);
  }
};

// ---------------------------------------------------------------- DensePolynomialPqx
// custom_dense_mlpoly.rs:36-41
static inline size_t rev_bits(size_t q, size_t max_num_proofs) {
  size_t lg = log_2(max_num_proofs), s = 0;
  for (size_t i = lg; i-- > 0;) s += q / pow2(i) % 2 * (max_num_proofs / pow2(i) / 2);
  return s;
}

typedef std::vector<std::vector<std::vector<FqVec>>> Mat4;  // [p][q][w][x]

enum { MODE_P = 1, MODE_Q = 2, MODE_W = 3, MODE_X = 4 };

struct Pqx {
  size_t num_instances = 0;
  std::vector<size_t> num_proofs;
  size_t max_num_proofs = 0;
  size_t num_witness_secs = 0;
  std::vector<size_t> num_inputs;
  size_t max_num_inputs = 0;
  Mat4 Z;

  // custom_dense_mlpoly.rs:67-111
  static Pqx new_rev(const Mat4& z_mat, const std::vector<size_t>& num_proofs, size_t max_num_proofs,
                     const std::vector<size_t>& num_inputs, size_t max_num_inputs) {
    Pqx P;
    size_t ninst = z_mat.size();
    size_t nws = z_mat[0][0].size();
    P.Z.resize(ninst);
    for (size_t p = 0; p < ninst; p++) {
      P.Z[p].assign(num_proofs[p], std::vector<FqVec>(nws, FqVec(num_inputs[p], fq_zero())));
      size_t step_q = max_num_proofs / num_proofs[p];
      size_t step_x = max_num_inputs / num_inputs[p];
      for (size_t q = 0; q < num_proofs[p]; q++) {
        size_t q_rev = rev_bits(q, max_num_proofs) / step_q;
        for (size_t x = 0; x < num_inputs[p]; x++) {
          size_t x_rev = rev_bits(x, max_num_inputs) / step_x;
          for (size_t w = 0; w < nws; w++) P.Z[p][q_rev][w][x_rev] = z_mat[p][q][w][x];
        }
      }
    }
    P.num_instances = next_pow2(ninst);
    P.num_proofs = num_proofs;
    P.max_num_proofs = max_num_proofs;
    P.num_witness_secs = next_pow2(nws);
    P.num_inputs = num_inputs;
    P.max_num_inputs = max_num_inputs;
    return P;
  }
  size_t len() const { return num_instances * max_num_proofs * max_num_inputs; }
  // custom_dense_mlpoly.rs:118-128
  Fq index(size_t p, size_t q, size_t w, size_t x) const {
    if (p < Z.size() && q < Z[p].size() && w < Z[p][q].size() && x < Z[p][q][w].size()) return Z[p][q][w][x];
    return fq_zero();
  }
  // custom_dense_mlpoly.rs:136-173
  Fq index_high(size_t p, size_t q, size_t w, size_t x, int mode) const {
    switch (mode) {
      case MODE_P: return p + num_instances / 2 < Z.size() ? Z[p + num_instances / 2][q][w][x] : fq_zero();
      case MODE_Q: return num_proofs[p] == 1 ? fq_zero() : Z[p][q + num_proofs[p] / 2][w][x];
      case MODE_W: return w + num_witness_secs / 2 < Z[p][q].size() ? Z[p][q][w + num_witness_secs / 2][x] : fq_zero();
      default: return num_inputs[p] == 1 ? fq_zero() : Z[p][q][w][x + num_inputs[p] / 2];
    }
  }
  void bound_poly(const Fq& r, int mode) {
    switch (mode) {
      case MODE_P: bound_p(r); break;
      case MODE_Q: bound_q(r); break;
      case MODE_W: bound_w(r); break;
      default: bound_x(r); break;
    }
  }
  // custom_dense_mlpoly.rs:205-219
  void bound_p(const Fq& r) {
    num_instances /= 2;
    for (size_t p = 0; p < num_instances; p++) {
      for (size_t w = 0; w < std::min(num_witness_secs, Z[p][0].size()); w++) {
        Fq hi = p + num_instances < Z.size() ? Z[p + num_instances][0][w][0] : fq_zero();
        Z[p][0][w][0] = fq_add(Z[p][0][w][0], fq_mul(r, fq_sub(hi, Z[p][0][w][0])));
      }
    }
  }
  // custom_dense_mlpoly.rs:222-245
  void bound_q(const Fq& r) {
    max_num_proofs /= 2;
    for (size_t p = 0; p < std::min(num_instances, Z.size()); p++) {
      if (num_proofs[p] == 1) {
        for (size_t w = 0; w < std::min(num_witness_secs, Z[p][0].size()); w++)
          for (size_t x = 0; x < num_inputs[p]; x++) Z[p][0][w][x] = fq_mul(fq_sub(fq_one(), r), Z[p][0][w][x]);
      } else {
        num_proofs[p] /= 2;
        for (size_t q = 0; q < num_proofs[p]; q++)
          for (size_t w = 0; w < std::min(num_witness_secs, Z[p][q].size()); w++)
            for (size_t x = 0; x < num_inputs[p]; x++)
              Z[p][q][w][x] = fq_add(Z[p][q][w][x], fq_mul(r, fq_sub(Z[p][q + num_proofs[p]][w][x], Z[p][q][w][x])));
      }
    }
  }
  // custom_dense_mlpoly.rs:248-264
  void bound_w(const Fq& r) {
    num_witness_secs /= 2;
    for (size_t p = 0; p < std::min(num_instances, Z.size()); p++)
      for (size_t q = 0; q < num_proofs[p]; q++)
        for (size_t w = 0; w < num_witness_secs; w++)
          for (size_t x = 0; x < num_inputs[p]; x++) {
            Fq hi = w + num_witness_secs < Z[p][q].size() ? Z[p][q][w + num_witness_secs][x] : fq_zero();
            Z[p][q][w][x] = fq_add(Z[p][q][w][x], fq_mul(r, fq_sub(hi, Z[p][q][w][x])));
          }
  }
  // custom_dense_mlpoly.rs:267-289
  void bound_x(const Fq& r) {
    max_num_inputs /= 2;
    for (size_t p = 0; p < std::min(num_instances, Z.size()); p++) {
      if (num_inputs[p] == 1) {
        for (size_t q = 0; q < num_proofs[p]; q++)
          for (size_t w = 0; w < std::min(num_witness_secs, Z[p][q].size()); w++)
            Z[p][q][w][0] = fq_mul(fq_sub(fq_one(), r), Z[p][q][w][0]);
      } else {
        num_inputs[p] /= 2;
        for (size_t q = 0; q < num_proofs[p]; q++)
          for (size_t w = 0; w < std::min(num_witness_secs, Z[p][q].size()); w++)
            for (size_t x = 0; x < num_inputs[p]; x++)
              Z[p][q][w][x] = fq_add(Z[p][q][w][x], fq_mul(r, fq_sub(Z[p][q][w][x + num_inputs[p]], Z[p][q][w][x])));
      }
    }
  }
  void bound_vars_rq(const FqVec& rq) { for (const Fq& r : rq) bound_q(r); }
};

// ---------------------------------------------------------------- UniPoly (src/unipoly.rs)
struct UniPoly {
  FqVec coeffs;
  // unipoly.rs:23-54
  static UniPoly from_evals(const FqVec& e) {
    UniPoly u;
    Fq two_inv = fq_invert(fq_from_u64(2));
    if (e.size() == 3) {
      Fq c = e[0];
      Fq a = fq_mul(two_inv, fq_add(fq_sub(fq_sub(e[2], e[1]), e[1]), c));
      Fq b = fq_sub(fq_sub(e[1], c), a);
      u.coeffs = {c, b, a};
    } else {
      Fq six_inv = fq_invert(fq_from_u64(6));
      Fq d = e[0];
      Fq a = fq_mul(six_inv, fq_sub(fq_add(fq_add(fq_add(fq_sub(fq_sub(fq_sub(e[3], e[2]), e[2]), e[2]), e[1]), e[1]), e[1]), e[0]));
      Fq b = fq_mul(two_inv,
                    fq_sub(fq_add(fq_add(fq_add(fq_add(fq_sub(fq_sub(fq_sub(fq_sub(fq_sub(fq_add(e[0], e[0]), e[1]), e[1]),
                                                                        e[1]), e[1]), e[1]), e[2]), e[2]), e[2]), e[2]),
                           e[3]));
      Fq c = fq_sub(fq_sub(fq_sub(e[1], d), a), b);
      u.coeffs = {d, c, b, a};
    }
    return u;
  }
  size_t degree() const { return coeffs.size() - 1; }
  // unipoly.rs:72-80
  Fq evaluate(const Fq& r) const {
    Fq ev = coeffs[0], power = r;
    for (size_t i = 1; i < coeffs.size(); i++) {
      ev = fq_add(ev, fq_mul(power, coeffs[i]));
      power = fq_mul(power, r);
    }
    return ev;
  }
  Fq eval_at_zero() const { return coeffs[0]; }
  Fq eval_at_one() const {
    Fq s = fq_zero();
    for (auto& c : coeffs) s = fq_add(s, c);
    return s;
  }
  // unipoly.rs:82-88 (coeffs except linear term)
  FqVec compress() const {
    FqVec v;
    v.push_back(coeffs[0]);
    for (size_t i = 2; i < coeffs.size(); i++) v.push_back(coeffs[i]);
    return v;
  }
  // unipoly.rs:97-111
  static UniPoly decompress(const FqVec& c, const Fq& hint) {
    Fq lin = fq_sub(fq_sub(hint, c[0]), c[0]);
    for (size_t i = 1; i < c.size(); i++) lin = fq_sub(lin, c[i]);
    UniPoly u;
    u.coeffs.push_back(c[0]);
    u.coeffs.push_back(lin);
    for (size_t i = 1; i < c.size(); i++) u.coeffs.push_back(c[i]);
    return u;
  }
  // unipoly.rs:112-120
  void append_to_transcript(const char* label, Transcript& t) const {
    t.append_message(label, "UniPoly_begin");
    for (auto& c : coeffs) t.append_scalar("coeff", c);
    t.append_message(label, "UniPoly_end");
  }
};

}  // namespace orc
