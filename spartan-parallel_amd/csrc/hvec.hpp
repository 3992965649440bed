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

#include <algorithm>
#include <vector>

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

SPG_IFMA Fe8 neg(const Fe8& a) { return sub(splat(fe_zero()), a); }
SPG_IFMA Fe8 select(__mmask8 m, const Fe8& a, const Fe8& b) {  // lane l: m_l ? a : b
  Fe8 r;
  for (int i = 0; i < 5; i++) r.v[i] = _mm512_mask_blend_epi64(m, b.v[i], a.v[i]);
  return r;
}
// fully reduced (canonical) limbs, as hcurve.hpp's fe_canon lane by lane: sequential carries, then p subtracted once
// when the value is >= p
SPG_IFMA Fe8 canon(const Fe8& x) {
  const __m512i M = m51();
  Fe8 a = x;
  for (int pass = 0; pass < 2; pass++) {
    for (int i = 0; i < 4; i++) {
      a.v[i + 1] = _mm512_add_epi64(a.v[i + 1], _mm512_srli_epi64(a.v[i], 51));
      a.v[i] = _mm512_and_si512(a.v[i], M);
    }
    a.v[0] = _mm512_add_epi64(a.v[0], times19(_mm512_srli_epi64(a.v[4], 51)));
    a.v[4] = _mm512_and_si512(a.v[4], M);
    a.v[1] = _mm512_add_epi64(a.v[1], _mm512_srli_epi64(a.v[0], 51));
    a.v[0] = _mm512_and_si512(a.v[0], M);
  }
  __m512i q = _mm512_srli_epi64(_mm512_add_epi64(a.v[0], _mm512_set1_epi64(19)), 51);
  for (int i = 1; i < 5; i++) q = _mm512_srli_epi64(_mm512_add_epi64(a.v[i], q), 51);
  a.v[0] = _mm512_add_epi64(a.v[0], times19(q));
  for (int i = 0; i < 4; i++) {
    a.v[i + 1] = _mm512_add_epi64(a.v[i + 1], _mm512_srli_epi64(a.v[i], 51));
    a.v[i] = _mm512_and_si512(a.v[i], M);
  }
  a.v[4] = _mm512_and_si512(a.v[4], M);
  return a;
}
SPG_IFMA __mmask8 is_negative(const Fe8& a) {
  return _mm512_test_epi64_mask(canon(a).v[0], _mm512_set1_epi64(1));
}
SPG_IFMA __mmask8 is_zero(const Fe8& a) {
  const Fe8 c = canon(a);
  __m512i o = c.v[0];
  for (int i = 1; i < 5; i++) o = _mm512_or_si512(o, c.v[i]);
  return _mm512_cmpeq_epi64_mask(o, _mm512_setzero_si512());
}

}  // namespace v8

// hcurve.hpp's hext_double_and_compress_batch with 8 points per step: lane l of every step takes the points l, l + 8,
// ..., its own chain of prefix products; the 8 lane products are inverted together (scalar Montgomery trick, one
// inversion), then the backward pass and the encodings run 8 points per step. Lanes whose e g f h vanishes take the
// lone encoding of 2 P. Same bytes (tests/test_product_host.py::test_host_double_and_compress_batch).
SPG_IFMA_FN inline void double_and_compress_batch8(const HExt* P, size_t n, uint8_t (*out)[32]) {
  using namespace v8;
  if (!n) return;
  const size_t G = (n + 7) / 8;
  struct St8 {
    Fe8 e, f, g, h, eg, fh, efgh, pre;
    __mmask8 zero;
  };
  // per-thread scratch, 64-byte aligned by hand (a std::vector of a 64-byte-aligned type is not aligned here: its
  // allocation is instantiated outside this target's code)
  thread_local St8* st = nullptr;
  thread_local size_t cap = 0;
  if (G > cap) {
    free(st);
    cap = std::max<size_t>(G, 16);
    st = (St8*)aligned_alloc(64, cap * sizeof(St8));
    if (!st) {
      cap = 0;
      for (size_t i = 0; i < n; i++) hext_compress(hext_dbl(P[i]), out[i]);
      return;
    }
  }
  const Fe8 one = splat(fe_one()), d = splat(K().d), sqrt_m1 = splat(K().sqrt_m1),
            isqrt_amd = splat(K().invsqrt_a_minus_d);
  Fe8 run = one;
  for (size_t k = 0; k < G; k++) {
    alignas(64) uint64_t ad[8];
    for (int l = 0; l < 8; l++) ad[l] = (uint64_t)&P[std::min(8 * k + l, n - 1)];  // the last group repeats a point
    const __m512i addr = _mm512_load_si512((const void*)ad);
    const Fe8 X = gather(addr, 0), Y = gather(addr, 5), Z = gather(addr, 10), T = gather(addr, 15);
    const Fe8 XX = mul(X, X), YY = mul(Y, Y), ZZ = mul(Z, Z), dTT = mul(mul(T, T), d);
    St8& s = st[k];
    s.e = mul(X, add(Y, Y));
    s.f = add(ZZ, dTT);
    s.g = add(YY, XX);
    s.h = sub(ZZ, dTT);
    s.eg = mul(s.e, s.g);
    s.fh = mul(s.f, s.h);
    s.efgh = mul(s.eg, s.fh);
    s.zero = is_zero(s.efgh);
    s.pre = run;
    run = mul(run, select(s.zero, one, s.efgh));
  }
  // the 8 lane products' inverses (Montgomery's trick over the lanes, one inversion)
  Fe lp[8], pre[8], li[8];
  Fe acc = fe_one();
  for (int l = 0; l < 8; l++) {
    lp[l] = lane(run, l);
    pre[l] = acc;
    acc = fe_mul(acc, lp[l]);
  }
  Fe inv = fe_invert(acc);
  for (int l = 7; l >= 0; l--) {
    li[l] = fe_mul(inv, pre[l]);
    inv = fe_mul(inv, lp[l]);
  }
  alignas(64) uint64_t w[5][8];
  for (int i = 0; i < 5; i++)
    for (int l = 0; l < 8; l++) w[i][l] = li[l].v[i];
  Fe8 inv8;
  for (int i = 0; i < 5; i++) inv8.v[i] = _mm512_load_si512((const void*)w[i]);
  for (size_t k = G; k-- > 0;) {
    const St8& s = st[k];
    const Fe8 inv_i = mul(inv8, s.pre);
    inv8 = mul(inv8, select(s.zero, one, s.efgh));
    const Fe8 Zinv = mul(s.eg, inv_i), Tinv = mul(s.fh, inv_i);
    const __mmask8 m1 = is_negative(mul(s.eg, Zinv));
    const Fe8 e = select(m1, s.g, s.e), g = select(m1, neg(s.e), s.g), h = select(m1, mul(s.f, sqrt_m1), s.h),
              magic = select(m1, sqrt_m1, isqrt_amd);
    const __mmask8 m2 = is_negative(mul(mul(h, e), Zinv));
    const Fe8 g2 = select(m2, neg(g), g);
    Fe8 r = mul(sub(h, g2), mul(magic, mul(g2, Tinv)));
    r = select(is_negative(r), neg(r), r);
    const Fe8 c = canon(r);
    alignas(64) uint64_t cw[5][8];
    for (int i = 0; i < 5; i++) _mm512_store_si512((void*)cw[i], c.v[i]);
    for (int l = 0; l < 8 && 8 * k + l < n; l++) {
      uint8_t* o = out[8 * k + l];
      if ((s.zero >> l) & 1) {  // the lone path (identity representatives)
        hext_compress(hext_dbl(P[8 * k + l]), o);
        continue;
      }
      const uint64_t q0 = cw[0][l] | (cw[1][l] << 51), q1 = (cw[1][l] >> 13) | (cw[2][l] << 38),
                     q2 = (cw[2][l] >> 26) | (cw[3][l] << 25), q3 = (cw[3][l] >> 39) | (cw[4][l] << 12);
      const uint64_t q[4] = {q0, q1, q2, q3};
      for (int i = 0; i < 4; i++)
        for (int b = 0; b < 8; b++) o[8 * i + b] = (uint8_t)(q[i] >> (8 * b));
    }
  }
}

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
