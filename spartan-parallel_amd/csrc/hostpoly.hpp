// spg — small host-side helpers shared by the prover drivers (r1cs.hip, spark.hip): sizes, eq tables,
// round polynomials, scalar (de)serialisation at the C-ABI.
#pragma once
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <vector>
#include <string.h>

#include <vector>

#include "ctx.hpp"
#include "host.hpp"
#include "sumcheck.hpp"

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

inline Fq dense_eval_host(FqV z, const FqV& r) {
  z.resize((size_t)1 << r.size(), fq_zero());
  FqV chi = eq_evals_host(r);
  Fq s = fq_zero();
  for (size_t i = 0; i < z.size(); i++) s = fq_add(s, fq_mul(z[i], chi[i]));
  return s;
}

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

// n device scalars to the host (d2h_multi: the result page, or page-locked staging for long ranges)
inline int d2h_fq(spg_ctx* ctx, const Fq* d, Fq* h, size_t n = 1) { return d2h_multi(ctx, {{d, n}}, h); }

inline Fq ld_fq(const uint64_t* v) {
  Fq a;
  for (int i = 0; i < 4; i++) {
    a.l[2 * i] = (uint32_t)v[i];
    a.l[2 * i + 1] = (uint32_t)(v[i] >> 32);
  }
  return a;
}

inline void st_fq(uint64_t* v, const Fq& a) {
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)a.l[2 * i] | ((uint64_t)a.l[2 * i + 1] << 32);
}

inline bool is_pow2(size_t x) { return x && !(x & (x - 1)); }

inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + 255) / 256); }

inline int eq_table(spg_ctx* ctx, const FqV& r, Fq* out) { return dev_eq_table(ctx, r.data(), (int)r.size(), out); }

struct Laps {  // SPG_TRACE=1: wall-time breakdown of a host orchestration
  const char* title = "R1CSProof::prove";
  bool on = getenv("SPG_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  std::vector<std::pair<std::string, double>> acc;
  void lap(const char* name) {
    if (!on) return;
    auto now = std::chrono::steady_clock::now();
    double us = std::chrono::duration<double, std::micro>(now - t).count();
    t = now;
    for (auto& a : acc)
      if (a.first == name) {
        a.second += us;
        return;
      }
    acc.push_back({name, us});
  }
  void print() {
    if (!on) return;
    double tot = 0;
    for (auto& a : acc) tot += a.second;
    fprintf(stderr, "[spg] %s host breakdown (us):", title);
    for (auto& a : acc) fprintf(stderr, " %s=%.0f", a.first.c_str(), a.second);
    fprintf(stderr, " total=%.0f\n", tot);
  }
};

}  // namespace spg
