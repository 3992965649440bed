// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of
//   * GroupElement::vartime_multiscalar_mul (src/group.rs:98-116): scalars go through decompress_scalar
//     (src/scalar/mod.rs:32-36, Montgomery -> canonical bytes) and then dalek's variable-time MSM
//     (Straus below ~190 points, Pippenger above with window 6/7/8 -- curve25519-dalek ^4.1.1,
//     backend/serial/scalar_mul/pippenger.rs; restated from its published algorithm).
//   * MultiCommitGens::new (src/commitments.rs:15-33), Commitments::commit (:69-92).
//   * DensePolynomial::commit / commit_inner (src/dense_mlpoly.rs:184-239) Hyrax rows.
#pragma once
#include <vector>
#include "fq.hpp"
#include "ristretto.hpp"
#include "transcript.hpp"

namespace orc {

struct Gens {  // MultiCommitGens
  size_t n;
  std::vector<Ge> G;
  Ge h;
};

// src/commitments.rs:15-33
static inline std::vector<Ge> gens_stream(const uint8_t* label, size_t label_len, size_t count) {
  Shake256 sh;
  sh.absorb(label, label_len);
  sh.absorb(RISTRETTO_BASEPOINT_COMPRESSED, 32);
  std::vector<Ge> out;
  out.reserve(count);
  uint8_t u[64];
  for (size_t i = 0; i < count; i++) {
    sh.squeeze(u, 64);
    out.push_back(ge_from_uniform_bytes(u));
  }
  return out;
}
static inline Gens gens_new(size_t n, const char* label) {
  std::vector<Ge> all = gens_stream((const uint8_t*)label, strlen(label), n + 1);
  Gens g;
  g.n = n;
  g.G.assign(all.begin(), all.begin() + n);
  g.h = all[n];
  return g;
}

// canonical little-endian digits of a Montgomery-form scalar (decompress_scalar)
static inline void scalar_canon(const Fq& s, uint8_t out[32]) { fq_to_bytes(s, out); }

// dalek Straus / double-and-add for tiny inputs; Pippenger for larger (results identical: exact group)
static inline Ge msm_canon(const std::vector<const uint8_t*>& k, const Ge* P, size_t n) {
  if (n == 0) return ge_identity();
  if (n < 190) {
    // Straus with 4-bit signed windows is what dalek runs; a plain interleaved double-and-add gives the same point
    Ge acc = ge_identity();
    for (int i = 255; i >= 0; i--) {
      acc = ge_double(acc);
      for (size_t j = 0; j < n; j++)
        if ((k[j][i >> 3] >> (i & 7)) & 1) acc = ge_add(acc, P[j]);
    }
    return acc;
  }
  int w = n < 500 ? 6 : (n < 800 ? 7 : 8);
  const int radix = 1 << w;
  const int nb = radix / 2;
  const int digits_count = (256 + w - 1) / w + 1;
  // signed radix-2^w recoding (as dalek Scalar::as_radix_2w)
  std::vector<int> digits(n * digits_count);
  for (size_t j = 0; j < n; j++) {
    int carry = 0;
    for (int d = 0; d < digits_count; d++) {
      int bit = d * w;
      uint32_t v = 0;
      for (int b = 0; b < w; b++) {
        int pos = bit + b;
        if (pos < 256 && ((k[j][pos >> 3] >> (pos & 7)) & 1)) v |= (1u << b);
      }
      int dv = (int)v + carry;
      carry = (dv + nb) >> w;  // 1 if dv >= 2^(w-1)
      digits[j * digits_count + d] = dv - (carry << w);
    }
  }
  std::vector<Ge> buckets(nb);
  Ge total = ge_identity();
  for (int d = digits_count - 1; d >= 0; d--) {
    for (int i = 0; i < w; i++) total = ge_double(total);
    for (int b = 0; b < nb; b++) buckets[b] = ge_identity();
    for (size_t j = 0; j < n; j++) {
      int dv = digits[j * digits_count + d];
      if (dv > 0) buckets[dv - 1] = ge_add(buckets[dv - 1], P[j]);
      else if (dv < 0) buckets[-dv - 1] = ge_sub(buckets[-dv - 1], P[j]);
    }
    Ge run = ge_identity(), sum = ge_identity();
    for (int b = nb - 1; b >= 0; b--) { run = ge_add(run, buckets[b]); sum = ge_add(sum, run); }
    total = ge_add(total, sum);
  }
  return total;
}

static inline Ge vartime_msm(const Fq* s, const Ge* P, size_t n) {
  std::vector<uint8_t> canon(32 * n);
  std::vector<const uint8_t*> ptr(n);
  for (size_t i = 0; i < n; i++) { scalar_canon(s[i], &canon[32 * i]); ptr[i] = &canon[32 * i]; }
  return msm_canon(ptr, P, n);
}

// Commitments::commit for [Scalar] (src/commitments.rs:87-92): MSM over the first len gens + blind*h
static inline Ge commit_slice(const Fq* s, size_t len, const Fq& blind, const Gens& g) {
  std::vector<Fq> sc(s, s + len);
  std::vector<Ge> P(g.G.begin(), g.G.begin() + len);
  Ge m = vartime_msm(sc.data(), P.data(), len);
  uint8_t b[32];
  scalar_canon(blind, b);
  return ge_add(m, ge_scalarmul_bytes(g.h, b));
}
// Commitments::commit for Scalar (src/commitments.rs:73-78): 2-point MSM [s, blind] x [G0, h]
static inline Ge commit_scalar(const Fq& s, const Fq& blind, const Gens& g) {
  Fq sc[2] = {s, blind};
  Ge P[2] = {g.G[0], g.h};
  return vartime_msm(sc, P, 2);
}

}  // namespace orc
