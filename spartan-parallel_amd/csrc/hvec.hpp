// spg — eight host point additions at once on AVX-512 IFMA (the prover box's EPYC cores have it): the host sums of
// the sequential protocol parts -- fixed-base commitments of the sigma protocols, the ZK-sumcheck round commitments,
// the small DotProductProofLogs' Bullet rounds on the host pool, the Bullet partial-point sums -- are long runs of
// independent mixed / full additions into one accumulator. Here the run is dealt out to 8 lanes (lane l takes
// entries l, l + 8, ...), each lane an accumulator of its own, and the 8 lane sums meet at the end.
//
// Field elements are hcurve.hpp's radix-2^51 limbs, one lane per element (Fe8 = 5 x 8 u64). vpmadd52{lo,hi}uq
// multiply the low 52 bits of two limbs: every multiply input must be < 2^52, which the operations below keep:
//   products leave limbs <= 2^51 + 18 (two parallel carry passes); sums and differences that feed a product are
//   carried once (inputs < 2^54 -> limbs < 2^51 + 133).
// The limb product a_i b_j (weight 2^(51 (i + j))) comes back as lo + hi 2^52, so hi enters the next limb doubled;
// limbs 5..9 of the product fold back times 19 (2^255 = 19 mod p). Results are the same group elements as
// hcurve.hpp's scalar additions (their encodings are compared in tests/test_product_host.py and every proof byte).
// Compiled with function-level target attributes only: nothing here runs unless ifma_on() found the instructions.
#pragma once
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>

#include "hcurve.hpp"

namespace spg {
namespace h {

// SPG_HOST_IFMA=0: the scalar additions everywhere
inline bool ifma_on() {
  static const bool on = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512ifma") &&
                         __builtin_cpu_supports("avx512dq") &&
                         !(getenv("SPG_HOST_IFMA") && atoi(getenv("SPG_HOST_IFMA")) == 0);
  return on;
}

#define SPG_IFMA __attribute__((target("avx512f,avx512ifma,avx512dq,avx512vl"), always_inline)) inline
#define SPG_IFMA_FN __attribute__((target("avx512f,avx512ifma,avx512dq,avx512vl"), noinline))

namespace v8 {

struct Fe8 {
  __m512i v[5];
};
struct Ext8 {
  Fe8 X, Y, Z, T;
};

SPG_IFMA __m512i m51() { return _mm512_set1_epi64((long long)M51); }
SPG_IFMA __m512i times19(__m512i c) {
  return _mm512_add_epi64(_mm512_add_epi64(_mm512_slli_epi64(c, 4), _mm512_slli_epi64(c, 1)), c);
}
// one parallel carry pass: limbs < 2^62 in; limb i keeps its low 51 bits plus limb i-1's carry (limb 0: 19 x limb
// 4's), so limbs < 2^54 come out < 2^51 + 19 * 7
SPG_IFMA Fe8 carry(const Fe8& a) {
  Fe8 r;
  __m512i c[5];
  const __m512i M = m51();
  for (int i = 0; i < 5; i++) {
    c[i] = _mm512_srli_epi64(a.v[i], 51);
    r.v[i] = _mm512_and_si512(a.v[i], M);
  }
  r.v[0] = _mm512_add_epi64(r.v[0], times19(c[4]));
  for (int i = 1; i < 5; i++) r.v[i] = _mm512_add_epi64(r.v[i], c[i - 1]);
  return r;
}
SPG_IFMA Fe8 add(const Fe8& a, const Fe8& b) {  // carried (feeds a product)
  Fe8 r;
  for (int i = 0; i < 5; i++) r.v[i] = _mm512_add_epi64(a.v[i], b.v[i]);
  return carry(r);
}
SPG_IFMA Fe8 add_nc(const Fe8& a, const Fe8& b) {
  Fe8 r;
  for (int i = 0; i < 5; i++) r.v[i] = _mm512_add_epi64(a.v[i], b.v[i]);
  return r;
}
// a + 4p - b, carried (inputs < 2^53)
SPG_IFMA Fe8 sub(const Fe8& a, const Fe8& b) {
  Fe8 r;
  r.v[0] = _mm512_sub_epi64(_mm512_add_epi64(a.v[0], _mm512_set1_epi64(0x1fffffffffffb4LL)), b.v[0]);
  for (int i = 1; i < 5; i++)
    r.v[i] = _mm512_sub_epi64(_mm512_add_epi64(a.v[i], _mm512_set1_epi64(0x1ffffffffffffcLL)), b.v[i]);
  return carry(r);
}
SPG_IFMA Fe8 mul(const Fe8& a, const Fe8& b) {
  __m512i lo[9], hi[9];
  for (int k = 0; k < 9; k++) lo[k] = hi[k] = _mm512_setzero_si512();
  for (int i = 0; i < 5; i++)
    for (int j = 0; j < 5; j++) {
      lo[i + j] = _mm512_madd52lo_epu64(lo[i + j], a.v[i], b.v[j]);
      hi[i + j] = _mm512_madd52hi_epu64(hi[i + j], a.v[i], b.v[j]);
    }
  // t_k = lo_k + 2 hi_(k-1) < 2^56; t_k + 19 t_(k+5) < 2^61
  __m512i t[10];
  t[0] = lo[0];
  for (int k = 1; k < 9; k++) t[k] = _mm512_add_epi64(lo[k], _mm512_slli_epi64(hi[k - 1], 1));
  t[9] = _mm512_slli_epi64(hi[8], 1);
  Fe8 r;
  for (int k = 0; k < 5; k++) r.v[k] = _mm512_add_epi64(t[k], times19(t[k + 5]));
  return carry(carry(r));
}

// extended += affine Niels (hcurve.hpp hext_madd), lane-wise
SPG_IFMA Ext8 madd(const Ext8& p, const Fe8& ypx, const Fe8& ymx, const Fe8& t2d) {
  const Fe8 A = mul(sub(p.Y, p.X), ymx);
  const Fe8 B = mul(add(p.Y, p.X), ypx);
  const Fe8 C = mul(p.T, t2d);
  const Fe8 D = add_nc(p.Z, p.Z);
  const Fe8 E = sub(B, A), F = sub(D, C), G = add(D, C), H = add(B, A);
  return Ext8{mul(E, F), mul(G, H), mul(F, G), mul(E, H)};
}
// extended + extended (hcurve.hpp hext_add), lane-wise; d2 = 2d in every lane
SPG_IFMA Ext8 addp(const Ext8& p, const Ext8& q, const Fe8& d2) {
  const Fe8 A = mul(sub(p.Y, p.X), sub(q.Y, q.X));
  const Fe8 B = mul(add(p.Y, p.X), add(q.Y, q.X));
  const Fe8 C = mul(mul(p.T, d2), q.T);
  const Fe8 D = mul(add(p.Z, p.Z), q.Z);  // (2 Z carried: a product input)
  const Fe8 E = sub(B, A), F = sub(D, C), G = add(D, C), H = add(B, A);
  return Ext8{mul(E, F), mul(G, H), mul(F, G), mul(E, H)};
}
SPG_IFMA Fe8 splat(const Fe& a) {
  Fe8 r;
  for (int i = 0; i < 5; i++) r.v[i] = _mm512_set1_epi64((long long)a.v[i]);
  return r;
}
SPG_IFMA Ext8 identity8() { return Ext8{splat(fe_zero()), splat(fe_one()), splat(fe_one()), splat(fe_zero())}; }
// lane l of the 8 field elements at src[l] + off (u64 offset): limb i of lane l is ((const uint64_t*)src[l])[off + i]
SPG_IFMA Fe8 gather(const __m512i addr, int off) {
  Fe8 r;
  for (int i = 0; i < 5; i++)
    r.v[i] = _mm512_i64gather_epi64(_mm512_add_epi64(addr, _mm512_set1_epi64(8LL * (off + i))), (const void*)0, 1);
  return r;
}
SPG_IFMA Fe lane(const Fe8& a, int l) {
  alignas(64) uint64_t w[5][8];
  for (int i = 0; i < 5; i++) _mm512_store_si512((void*)w[i], a.v[i]);
  return Fe{{w[0][l], w[1][l], w[2][l], w[3][l], w[4][l]}};
}
// the 8 lane sums, added on this thread (scalar additions: 7 of them)
SPG_IFMA HExt reduce(const Ext8& a) {
  alignas(64) uint64_t w[4][5][8];
  const Fe8* c[4] = {&a.X, &a.Y, &a.Z, &a.T};
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < 5; i++) _mm512_store_si512((void*)w[k][i], c[k]->v[i]);
  HExt s[8];
  for (int l = 0; l < 8; l++) {
    Fe* o[4] = {&s[l].X, &s[l].Y, &s[l].Z, &s[l].T};
    for (int k = 0; k < 4; k++)
      for (int i = 0; i < 5; i++) o[k]->v[i] = w[k][i][l];
  }
  for (int d = 4; d >= 1; d >>= 1)
    for (int l = 0; l < d; l++) s[l] = hext_add(s[l], s[l + d]);
  return s[0];
}

}  // namespace v8

// sum of n affine Niels entries (pointers), from the identity; entries of lanes past the end are the identity's
// Niels form (1, 1, 0), whose mixed addition leaves a point unchanged (projectively)
SPG_IFMA_FN inline HExt niels_sum8(const HNiels* const* ent, size_t n) {
  using namespace v8;
  static const HNiels ident{fe_one(), fe_one(), fe_zero()};
  Ext8 acc = identity8();
  for (size_t b = 0; b < n; b += 8) {
    alignas(64) uint64_t ad[8];
    for (int l = 0; l < 8; l++) ad[l] = (uint64_t)(b + l < n ? ent[b + l] : &ident);
    if (b + 8 < n)  // the next group's lines while this one adds
      for (size_t l = b + 8; l < b + 16 && l < n; l++) {
        __builtin_prefetch(ent[l]);
        __builtin_prefetch((const char*)ent[l] + sizeof(HNiels) - 1);
      }
    const __m512i addr = _mm512_load_si512((const void*)ad);
    acc = madd(acc, gather(addr, 0), gather(addr, 5), gather(addr, 10));
  }
  return reduce(acc);
}

// sum of n extended points (a chunk of device partial points, converted), from the identity
SPG_IFMA_FN inline HExt ext_sum8(const HExt* pts, size_t n) {
  using namespace v8;
  static const HExt ident = hext_identity();
  const Fe8 d2 = splat(K().d2);
  Ext8 acc = identity8();
  for (size_t b = 0; b < n; b += 8) {
    alignas(64) uint64_t ad[8];
    for (int l = 0; l < 8; l++) ad[l] = (uint64_t)(b + l < n ? &pts[b + l] : &ident);
    const __m512i addr = _mm512_load_si512((const void*)ad);
    const Ext8 q{gather(addr, 0), gather(addr, 5), gather(addr, 10), gather(addr, 15)};
    acc = addp(acc, q, d2);
  }
  return reduce(acc);
}

}  // namespace h
}  // namespace spg
