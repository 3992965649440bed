// spg — host-only scalar helpers of the prover drivers (sizes, eq tables, round polynomials). No HIP: shared with
// the CPU test library (hostcheck.cpp), so the CPU suite checks these exact functions against the oracle and the
// reference's own known-answer tests (src/unipoly.rs:127-181, src/dense_mlpoly.rs:1234-1252).
#pragma once
#include <stddef.h>

#include <vector>

#include "host.hpp"

namespace spg {

inline size_t lg2(size_t x) {  // src/math.rs:14-21 (rounds up)
  size_t r = 0;
  while (((size_t)1 << r) < x) r++;
  return r;
}

inline size_t npow2(size_t x) {
  size_t r = 1;
  while (r < x) r <<= 1;
  return r;
}

// EqPolynomial::evals (src/dense_mlpoly.rs:76-92)
inline FqV eq_evals_host(const FqV& r) {
  FqV e((size_t)1 << r.size(), fq_one());
  size_t size = 1;
  for (size_t j = 0; j < r.size(); j++) {
    size *= 2;
    for (size_t i = size - 1;; i -= 2) {
      Fq s = e[i / 2];
      e[i] = fq_mul(s, r[j]);
      e[i - 1] = fq_sub(s, e[i]);
      if (i < 2) break;
    }
  }
  return e;
}

// DensePolynomial::new(z).evaluate(r) (src/dense_mlpoly.rs:361-367) for short host vectors
inline Fq dense_eval_host(FqV z, const FqV& r) {
  z.resize((size_t)1 << r.size(), fq_zero());
  FqV chi = eq_evals_host(r);
  Fq s = fq_zero();
  for (size_t i = 0; i < z.size(); i++) s = fq_add(s, fq_mul(z[i], chi[i]));
  return s;
}

// UniPoly::from_evals for degree 3 (src/unipoly.rs:23-54) and evaluate (:72-80)
inline FqV uni_from_evals3(const Fq e[4]) {
  static const Fq two_inv = fq_inv(fq_from_u64(2)), six_inv = fq_inv(fq_from_u64(6));
  Fq d = e[0];
  Fq three_e1 = fq_add(fq_add(e[1], e[1]), e[1]), three_e2 = fq_add(fq_add(e[2], e[2]), e[2]);
  Fq a = fq_mul(six_inv, fq_sub(fq_add(fq_sub(e[3], three_e2), three_e1), e[0]));
  Fq four_e2 = fq_dbl(fq_dbl(e[2]));
  Fq five_e1 = fq_add(fq_dbl(fq_dbl(e[1])), e[1]);
  Fq b = fq_mul(two_inv, fq_sub(fq_add(fq_sub(fq_dbl(e[0]), five_e1), four_e2), e[3]));
  Fq c = fq_sub(fq_sub(fq_sub(e[1], d), a), b);
  return {d, c, b, a};
}

inline Fq uni_eval(const FqV& c, const Fq& r) {
  Fq ev = c[0], pw = r;
  for (size_t i = 1; i < c.size(); i++) {
    ev = fq_add(ev, fq_mul(pw, c[i]));
    pw = fq_mul(pw, r);
  }
  return ev;
}

inline bool is_pow2(size_t x) { return x && !(x & (x - 1)); }

}  // namespace spg
