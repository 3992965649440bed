// spg — small host-side helpers shared by the prover drivers (r1cs.hip, spark.hip): sizes, eq tables,
// round polynomials, scalar (de)serialisation at the C-ABI.
#pragma once
#include <initializer_list>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <vector>
#include <string.h>

#include <vector>

#include "ctx.hpp"
#include "host.hpp"
#include "hostmath.hpp"
#include "sumcheck.hpp"

namespace spg {

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

inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + 255) / 256); }

inline int eq_table(spg_ctx* ctx, const FqV& r, Fq* out) { return dev_eq_table(ctx, r.data(), (int)r.size(), out); }
struct EqOut {
  const FqV& r;
  Fq* out;
};
// the tables one prover step needs together, in as few launches as dev_eq_tables can pack them
inline int eq_tables(spg_ctx* ctx, std::initializer_list<EqOut> l) {
  std::vector<EqJob> j;
  for (const EqOut& e : l) j.push_back({e.r.data(), (int)e.r.size(), e.out});
  return dev_eq_tables(ctx, j.data(), (int)j.size());
}

// dst += c src for every job (over min(|dst|, |src|) entries), on the host pool in index chunks: the random linear
// combinations of PolyEvalProof's batched openings (dense_mlpoly.rs:531-1130, r1csproof.rs's witness opening). Jobs
// into one dst run in job order within a chunk; the sums are exact field sums, so the vectors are the serial loop's.
struct Axpy {
  FqV* dst;
  Fq c;
  const FqV* src;
};
inline void axpy_pool(const std::vector<Axpy>& jobs) {
  size_t work = 0, n = 0;
  for (const Axpy& j : jobs) {
    const size_t m = std::min(j.dst->size(), j.src->size());
    work += m;
    n = std::max(n, m);
  }
  // (1024 products are ~25 us on one core, a burst ~3; SPG_AXPY_POOL=0: always on the calling thread)
  static const bool on = !getenv("SPG_AXPY_POOL") || atoi(getenv("SPG_AXPY_POOL")) != 0;
  const int C = on && work >= 1024 ? 8 : 1;
  pool().parallel_for(C, [&](int ch) {
    const size_t lo = n * ch / C, hi = n * (ch + 1) / C;
    for (const Axpy& j : jobs) {
      FqV& d = *j.dst;
      const FqV& s = *j.src;
      const size_t e = std::min(hi, std::min(d.size(), s.size()));
      for (size_t k = lo; k < e; k++) d[k] = fq_add(d[k], fq_mul(j.c, s[k]));
    }
  });
}

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
    // SPG_TRACE_EVENTS=1: every lap's end on stderr with its CLOCK_MONOTONIC time (the clock of rocprofv3's kernel
    // trace), so scripts/kernel_gaps.py can name the host phase behind each idle gap of the device
    static const bool ev = getenv("SPG_TRACE_EVENTS") != nullptr;
    if (ev)
      fprintf(stderr, "[spgev] %lld %s:%s %.1f\n",
              (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(now.time_since_epoch()).count(), title,
              name, us);
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
