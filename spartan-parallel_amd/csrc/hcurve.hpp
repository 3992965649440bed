// spg — host-side ristretto255 arithmetic for the prover's sequential parts (sigma-protocol
// commitments, point encodings between Fiat-Shamir challenges).
//
// The device code (curve.hpp) uses 8 x 32-bit limbs, which suit v_mad_u64_u32; on the host CPU the
// natural form is radix 2^51 with 64x64->128 multiplies, several times faster. Both implement the same
// group law and the same canonical RFC 9496 encoding, so results are bit-identical (tests compare
// them through the hostcheck library and every proof byte).
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

#include "curve.hpp"

namespace spg {
namespace h {

typedef unsigned __int128 u128;
static const uint64_t M51 = (1ULL << 51) - 1;

struct Fe {
  uint64_t v[5];
};

inline Fe fe_zero() { return Fe{{0, 0, 0, 0, 0}}; }
inline Fe fe_one() { return Fe{{1, 0, 0, 0, 0}}; }

inline Fe fe_carry(Fe a) {
  uint64_t c;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= M51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= M51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= M51; a.v[4] += c;
  c = a.v[4] >> 51; a.v[4] &= M51; a.v[0] += c * 19;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  return a;
}
inline Fe fe_add(const Fe& a, const Fe& b) {
  Fe r;
  for (int i = 0; i < 5; i++) r.v[i] = a.v[i] + b.v[i];
  return fe_carry(r);
}
// a + 4p - b (inputs carried: limbs < 2^52)
inline Fe fe_sub(const Fe& a, const Fe& b) {
  Fe r;
  r.v[0] = a.v[0] + 0x1fffffffffffb4ULL - b.v[0];
  for (int i = 1; i < 5; i++) r.v[i] = a.v[i] + 0x1ffffffffffffcULL - b.v[i];
  return fe_carry(r);
}
inline Fe fe_neg(const Fe& a) { return fe_sub(fe_zero(), a); }
// without the carry (the point additions' sums and differences feed a multiply directly, which takes limbs < 2^54:
// 5 products of < 2^54 x 19 * 2^54 stay below 2^128). Inputs: limbs < 2^52 (a multiply's or a carry's output).
inline Fe fe_add_nc(const Fe& a, const Fe& b) {
  Fe r;
  for (int i = 0; i < 5; i++) r.v[i] = a.v[i] + b.v[i];
  return r;
}
inline Fe fe_sub_nc(const Fe& a, const Fe& b) {
  Fe r;
  r.v[0] = a.v[0] + 0x1fffffffffffb4ULL - b.v[0];
  for (int i = 1; i < 5; i++) r.v[i] = a.v[i] + 0x1ffffffffffffcULL - b.v[i];
  return r;
}

// the five column sums of a product (each < 2^115) to limbs < 2^52 (limbs 1 and 4 may exceed 2^51 by < 2^13): two carry
// chains side by side, 0 -> 1 -> 2 -> 3 and 3 -> 4 -> 0, then one step each into limbs 4 and 1 -- four dependent steps
// where a single chain 0 -> 1 -> 2 -> 3 -> 4 -> 0 -> 1 takes six (~10 % off every squaring of an encoding's inverse
// square root in a host micro-benchmark). Column 4 has no 19-folded terms, so its carry times 19 stays below 2^64.
inline Fe fe_carry_wide(u128 t0, u128 t1, u128 t2, u128 t3, u128 t4) {
  Fe r;
  t1 += (uint64_t)(t0 >> 51);
  r.v[0] = (uint64_t)t0 & M51;
  t4 += (uint64_t)(t3 >> 51);
  const uint64_t r3 = (uint64_t)t3 & M51;
  t2 += (uint64_t)(t1 >> 51);
  r.v[1] = (uint64_t)t1 & M51;
  r.v[0] += (uint64_t)(t4 >> 51) * 19;
  r.v[4] = (uint64_t)t4 & M51;
  const uint64_t x3 = r3 + (uint64_t)(t2 >> 51);
  r.v[2] = (uint64_t)t2 & M51;
  r.v[3] = x3 & M51;
  r.v[4] += x3 >> 51;
  r.v[1] += r.v[0] >> 51;
  r.v[0] &= M51;
  return r;
}
inline Fe fe_mul(const Fe& a, const Fe& b) {
  const uint64_t b1 = b.v[1] * 19, b2 = b.v[2] * 19, b3 = b.v[3] * 19, b4 = b.v[4] * 19;
  u128 t0 = (u128)a.v[0] * b.v[0] + (u128)a.v[1] * b4 + (u128)a.v[2] * b3 + (u128)a.v[3] * b2 + (u128)a.v[4] * b1;
  u128 t1 = (u128)a.v[0] * b.v[1] + (u128)a.v[1] * b.v[0] + (u128)a.v[2] * b4 + (u128)a.v[3] * b3 + (u128)a.v[4] * b2;
  u128 t2 = (u128)a.v[0] * b.v[2] + (u128)a.v[1] * b.v[1] + (u128)a.v[2] * b.v[0] + (u128)a.v[3] * b4 +
            (u128)a.v[4] * b3;
  u128 t3 = (u128)a.v[0] * b.v[3] + (u128)a.v[1] * b.v[2] + (u128)a.v[2] * b.v[1] + (u128)a.v[3] * b.v[0] +
            (u128)a.v[4] * b4;
  u128 t4 = (u128)a.v[0] * b.v[4] + (u128)a.v[1] * b.v[3] + (u128)a.v[2] * b.v[2] + (u128)a.v[3] * b.v[1] +
            (u128)a.v[4] * b.v[0];
  return fe_carry_wide(t0, t1, t2, t3, t4);
}
// 15 limb products instead of 25 (the cross terms doubled); the inversion / square-root chains of every
// point encoding are ~250 squarings
inline Fe fe_sqr(const Fe& a) {
  const uint64_t a0_2 = a.v[0] * 2, a1_2 = a.v[1] * 2;
  const uint64_t a3_19 = a.v[3] * 19, a4_19 = a.v[4] * 19;
  u128 t0 = (u128)a.v[0] * a.v[0] + (u128)a1_2 * a4_19 + (u128)(a.v[2] * 2) * a3_19;
  u128 t1 = (u128)a0_2 * a.v[1] + (u128)(a.v[2] * 2) * a4_19 + (u128)a.v[3] * a3_19;
  u128 t2 = (u128)a0_2 * a.v[2] + (u128)a.v[1] * a.v[1] + (u128)(a.v[3] * 2) * a4_19;
  u128 t3 = (u128)a0_2 * a.v[3] + (u128)a1_2 * a.v[2] + (u128)a.v[4] * a4_19;
  u128 t4 = (u128)a0_2 * a.v[4] + (u128)a1_2 * a.v[3] + (u128)a.v[2] * a.v[2];
  return fe_carry_wide(t0, t1, t2, t3, t4);
}
inline Fe fe_sqrn(Fe a, int n) {
  for (int i = 0; i < n; i++) a = fe_sqr(a);
  return a;
}
// canonical value (fully reduced limbs)
inline Fe fe_canon(Fe a) {
  a = fe_carry(fe_carry(a));  // every limb < 2^51
  // a < 2^255 + small; subtract p if a >= p
  uint64_t q = (a.v[0] + 19) >> 51;
  q = (a.v[1] + q) >> 51;
  q = (a.v[2] + q) >> 51;
  q = (a.v[3] + q) >> 51;
  q = (a.v[4] + q) >> 51;
  a.v[0] += 19 * q;
  uint64_t c;
  c = a.v[0] >> 51; a.v[0] &= M51; a.v[1] += c;
  c = a.v[1] >> 51; a.v[1] &= M51; a.v[2] += c;
  c = a.v[2] >> 51; a.v[2] &= M51; a.v[3] += c;
  c = a.v[3] >> 51; a.v[3] &= M51; a.v[4] += c;
  a.v[4] &= M51;
  return a;
}
inline void fe_to_bytes(const Fe& a0, uint8_t out[32]) {
  Fe a = fe_canon(a0);
  uint64_t w[4];
  w[0] = a.v[0] | (a.v[1] << 51);
  w[1] = (a.v[1] >> 13) | (a.v[2] << 38);
  w[2] = (a.v[2] >> 26) | (a.v[3] << 25);
  w[3] = (a.v[3] >> 39) | (a.v[4] << 12);
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(w[i] >> (8 * k));
}
// low 255 bits of a little-endian 32-byte string (top bit ignored)
inline Fe fe_from_bytes(const uint8_t b[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int k = 0; k < 8; k++) w[i] |= (uint64_t)b[8 * i + k] << (8 * k);
  }
  Fe r;
  r.v[0] = w[0] & M51;
  r.v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  r.v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  r.v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  r.v[4] = (w[3] >> 12) & M51;
  return r;
}
// device Fp (8 x u32, loosely reduced in [0, 2^256)) -> Fe
inline Fe fe_from_fp(const Fp& a) {
  uint8_t b[32];
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) b[4 * i + k] = (uint8_t)(a.l[i] >> (8 * k));
  Fe r = fe_from_bytes(b);
  if (b[31] & 0x80) {  // bit 255 set: 2^255 = 19 mod p
    r.v[0] += 19;
    r = fe_carry(r);
  }
  return r;
}
inline bool fe_is_negative(const Fe& a) {
  uint8_t b[32];
  fe_to_bytes(a, b);
  return b[0] & 1;
}
inline bool fe_is_zero(const Fe& a) {
  uint8_t b[32];
  fe_to_bytes(a, b);
  uint8_t o = 0;
  for (int i = 0; i < 32; i++) o |= b[i];
  return o == 0;
}
inline bool fe_eq(const Fe& a, const Fe& b) { return fe_is_zero(fe_sub(a, b)); }
inline Fe fe_abs(const Fe& a) { return fe_is_negative(a) ? fe_neg(a) : a; }

// a^(2^252 - 3)
inline Fe fe_pow22523(const Fe& z) {
  Fe z2 = fe_sqr(z);
  Fe z8 = fe_sqrn(z2, 2);
  Fe z9 = fe_mul(z, z8);
  Fe z11 = fe_mul(z2, z9);
  Fe z22 = fe_sqr(z11);
  Fe z_5_0 = fe_mul(z9, z22);
  Fe z_10_0 = fe_mul(fe_sqrn(z_5_0, 5), z_5_0);
  Fe z_20_0 = fe_mul(fe_sqrn(z_10_0, 10), z_10_0);
  Fe z_40_0 = fe_mul(fe_sqrn(z_20_0, 20), z_20_0);
  Fe z_50_0 = fe_mul(fe_sqrn(z_40_0, 10), z_10_0);
  Fe z_100_0 = fe_mul(fe_sqrn(z_50_0, 50), z_50_0);
  Fe z_200_0 = fe_mul(fe_sqrn(z_100_0, 100), z_100_0);
  Fe z_250_0 = fe_mul(fe_sqrn(z_200_0, 50), z_50_0);
  return fe_mul(fe_sqrn(z_250_0, 2), z);
}
// a^(p-2)
inline Fe fe_invert(const Fe& z) {
  Fe z2 = fe_sqr(z);
  Fe z8 = fe_sqrn(z2, 2);
  Fe z9 = fe_mul(z, z8);
  Fe z11 = fe_mul(z2, z9);
  Fe z22 = fe_sqr(z11);
  Fe z_5_0 = fe_mul(z9, z22);
  Fe z_10_0 = fe_mul(fe_sqrn(z_5_0, 5), z_5_0);
  Fe z_20_0 = fe_mul(fe_sqrn(z_10_0, 10), z_10_0);
  Fe z_40_0 = fe_mul(fe_sqrn(z_20_0, 20), z_20_0);
  Fe z_50_0 = fe_mul(fe_sqrn(z_40_0, 10), z_10_0);
  Fe z_100_0 = fe_mul(fe_sqrn(z_50_0, 50), z_50_0);
  Fe z_200_0 = fe_mul(fe_sqrn(z_100_0, 100), z_100_0);
  Fe z_250_0 = fe_mul(fe_sqrn(z_200_0, 50), z_50_0);
  return fe_mul(fe_sqrn(z_250_0, 5), z11);
}

struct Consts {
  Fe d, d2, sqrt_m1, invsqrt_a_minus_d;
  Consts() {
    d = fe_from_fp(c_d());
    d2 = fe_from_fp(c_d2());
    sqrt_m1 = fe_from_fp(c_sqrt_m1());
    invsqrt_a_minus_d = fe_from_fp(c_invsqrt_a_minus_d());
  }
};
inline const Consts& K() {
  static const Consts k;
  return k;
}

struct HExt {
  Fe X, Y, Z, T;
};
struct HNiels {  // affine: (y+x, y-x, 2d*x*y)
  Fe ypx, ymx, t2d;
};

inline HExt hext_identity() { return HExt{fe_zero(), fe_one(), fe_one(), fe_zero()}; }
inline HExt hext_from_dev(const Ext& p) {
  return HExt{fe_from_fp(p.X), fe_from_fp(p.Y), fe_from_fp(p.Z), fe_from_fp(p.T)};
}
// add-2008-hwcd-3
// (the coordinates of a point here are multiply or carry outputs, limbs < 2^52, so the sums and differences that feed
// the next multiplies skip their carries)
inline HExt hext_add(const HExt& p, const HExt& q) {
  Fe A = fe_mul(fe_sub_nc(p.Y, p.X), fe_sub_nc(q.Y, q.X));
  Fe B = fe_mul(fe_add_nc(p.Y, p.X), fe_add_nc(q.Y, q.X));
  Fe C = fe_mul(fe_mul(p.T, K().d2), q.T);
  Fe D = fe_mul(fe_add_nc(p.Z, p.Z), q.Z);
  Fe E = fe_sub_nc(B, A), F = fe_sub_nc(D, C), G = fe_add_nc(D, C), H = fe_add_nc(B, A);
  return HExt{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
inline HExt hext_madd(const HExt& p, const HNiels& q) {
  Fe A = fe_mul(fe_sub_nc(p.Y, p.X), q.ymx);
  Fe B = fe_mul(fe_add_nc(p.Y, p.X), q.ypx);
  Fe C = fe_mul(p.T, q.t2d);
  Fe D = fe_add_nc(p.Z, p.Z);
  Fe E = fe_sub_nc(B, A), F = fe_sub_nc(D, C), G = fe_add_nc(D, C), H = fe_add_nc(B, A);
  return HExt{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
inline HExt hext_dbl(const HExt& p) {
  Fe A = fe_sqr(p.X), B = fe_sqr(p.Y);
  Fe zz = fe_sqr(p.Z);
  Fe C = fe_add(zz, zz);
  Fe E = fe_sub(fe_sub(fe_sqr(fe_add(p.X, p.Y)), A), B);
  Fe G = fe_sub(B, A);
  Fe F = fe_sub(G, C);
  Fe H = fe_neg(fe_add(A, B));
  return HExt{fe_mul(E, F), fe_mul(G, H), fe_mul(F, G), fe_mul(E, H)};
}
// affine Niels forms of many points with one inversion (Montgomery's trick)
inline void hext_batch_to_niels(const std::vector<HExt>& P, std::vector<HNiels>& out) {
  size_t n = P.size();
  out.resize(n);
  std::vector<Fe> pre(n + 1);
  pre[0] = fe_one();
  for (size_t i = 0; i < n; i++) pre[i + 1] = fe_mul(pre[i], P[i].Z);
  Fe inv = fe_invert(pre[n]);
  for (size_t i = n; i-- > 0;) {
    Fe zi = fe_mul(inv, pre[i]);
    inv = fe_mul(inv, P[i].Z);
    Fe x = fe_mul(P[i].X, zi), y = fe_mul(P[i].Y, zi);
    out[i].ypx = fe_add(y, x);
    out[i].ymx = fe_sub(y, x);
    out[i].t2d = fe_mul(fe_mul(x, y), K().d2);
  }
}

// RFC 9496 SQRT_RATIO_M1
inline bool fe_sqrt_ratio_m1(const Fe& u, const Fe& v, Fe& out) {
  Fe v3 = fe_mul(fe_sqr(v), v);
  Fe v7 = fe_mul(fe_sqr(v3), v);
  Fe r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  Fe check = fe_mul(v, fe_sqr(r));
  Fe nu = fe_neg(u);
  bool correct = fe_eq(check, u);
  bool flipped = fe_eq(check, nu);
  bool flipped_i = fe_eq(check, fe_mul(nu, K().sqrt_m1));
  if (flipped || flipped_i) r = fe_mul(K().sqrt_m1, r);
  out = fe_abs(r);
  return correct || flipped;
}
// RFC 9496 ENCODE
inline void hext_compress(const HExt& P, uint8_t out[32]) {
  Fe u1 = fe_mul(fe_add(P.Z, P.Y), fe_sub(P.Z, P.Y));
  Fe u2 = fe_mul(P.X, P.Y);
  Fe invsqrt;
  fe_sqrt_ratio_m1(fe_one(), fe_mul(u1, fe_sqr(u2)), invsqrt);
  Fe den1 = fe_mul(invsqrt, u1);
  Fe den2 = fe_mul(invsqrt, u2);
  Fe z_inv = fe_mul(fe_mul(den1, den2), P.T);
  bool rotate = fe_is_negative(fe_mul(P.T, z_inv));
  Fe x = P.X, y = P.Y, den_inv = den2;
  if (rotate) {
    x = fe_mul(P.Y, K().sqrt_m1);
    y = fe_mul(P.X, K().sqrt_m1);
    den_inv = fe_mul(den1, K().invsqrt_a_minus_d);
  }
  if (fe_is_negative(fe_mul(x, z_inv))) y = fe_neg(y);
  Fe s = fe_abs(fe_mul(den_inv, fe_sub(P.Z, y)));
  fe_to_bytes(s, out);
}
// RFC 9496 ENCODE of 2 P_i for a batch with ONE field inversion (the batched encoding of curve25519-dalek's
// RistrettoPoint::double_and_compress_batch): with e = 2XY, f = Z^2 + d T^2, g = Y^2 + X^2, h = Z^2 - d T^2 of P, the
// double's encoding needs 1 / (e g f h), inverted for the whole batch by Montgomery's trick, where a lone encoding
// needs an inverse square root (~250 squarings). A caller that wants encode(P) halves P first -- its MSM scalars
// times 2^-1 mod l -- so the host encodes a batch at ~25 products per point instead of ~265. Points whose e g f h
// vanishes (torsion representatives of the identity, whose double encodes to 0) take the lone encoding of 2 P.
inline void hext_double_and_compress_batch(const HExt* P, size_t n, uint8_t (*out)[32]) {
  struct St {
    Fe e, f, g, h, eg, fh, efgh, pre;
    bool zero;
  };
  std::vector<St> st(n);
  Fe run = fe_one();
  for (size_t i = 0; i < n; i++) {
    St& s = st[i];
    const Fe XX = fe_sqr(P[i].X), YY = fe_sqr(P[i].Y), ZZ = fe_sqr(P[i].Z);
    const Fe dTT = fe_mul(fe_sqr(P[i].T), K().d);
    s.e = fe_mul(P[i].X, fe_add(P[i].Y, P[i].Y));
    s.f = fe_add(ZZ, dTT);
    s.g = fe_add(YY, XX);
    s.h = fe_sub(ZZ, dTT);
    s.eg = fe_mul(s.e, s.g);
    s.fh = fe_mul(s.f, s.h);
    s.efgh = fe_mul(s.eg, s.fh);
    s.zero = fe_is_zero(s.efgh);
    s.pre = run;
    if (!s.zero) run = fe_mul(run, s.efgh);
  }
  Fe inv = fe_invert(run);  // 1 / (product of the nonzero e g f h)
  for (size_t i = n; i-- > 0;) {
    const St& s = st[i];
    if (s.zero) {
      hext_compress(hext_dbl(P[i]), out[i]);
      continue;
    }
    const Fe inv_i = fe_mul(inv, s.pre);
    inv = fe_mul(inv, s.efgh);
    const Fe Zinv = fe_mul(s.eg, inv_i), Tinv = fe_mul(s.fh, inv_i);
    Fe magic = K().invsqrt_a_minus_d, e = s.e, g = s.g, h = s.h;
    if (fe_is_negative(fe_mul(s.eg, Zinv))) {
      const Fe minus_e = fe_neg(s.e);
      e = s.g;
      g = minus_e;
      h = fe_mul(s.f, K().sqrt_m1);
      magic = K().sqrt_m1;
    }
    if (fe_is_negative(fe_mul(fe_mul(h, e), Zinv))) g = fe_neg(g);
    Fe r = fe_mul(fe_sub(h, g), fe_mul(magic, fe_mul(g, Tinv)));
    if (fe_is_negative(r)) r = fe_neg(r);
    fe_to_bytes(r, out[i]);
  }
}
// RFC 9496 DECODE
inline bool hext_decompress(const uint8_t in[32], HExt& out) {
  Fe s = fe_from_bytes(in);
  uint8_t chk[32];
  fe_to_bytes(s, chk);
  if (memcmp(chk, in, 32) != 0 || (in[0] & 1)) return false;  // non-canonical or negative
  Fe ss = fe_sqr(s);
  Fe u1 = fe_sub(fe_one(), ss);
  Fe u2 = fe_add(fe_one(), ss);
  Fe u2s = fe_sqr(u2);
  Fe v = fe_sub(fe_neg(fe_mul(K().d, fe_sqr(u1))), u2s);
  Fe invsqrt;
  bool was_square = fe_sqrt_ratio_m1(fe_one(), fe_mul(v, u2s), invsqrt);
  Fe den_x = fe_mul(invsqrt, u2);
  Fe den_y = fe_mul(fe_mul(invsqrt, den_x), v);
  Fe x = fe_abs(fe_mul(fe_add(s, s), den_x));
  Fe y = fe_mul(u1, den_y);
  Fe t = fe_mul(x, y);
  if (!was_square || fe_is_negative(t) || fe_is_zero(y)) return false;
  out = HExt{x, y, fe_one(), t};
  return true;
}
// variable-base scalar multiplication by canonical little-endian bytes
inline HExt hext_scalar_mul(const HExt& P, const uint8_t k[32]) {
  HExt acc = hext_identity();
  bool started = false;
  for (int i = 255; i >= 0; i--) {
    if (started) acc = hext_dbl(acc);
    if ((k[i >> 3] >> (i & 7)) & 1) {
      acc = started ? hext_add(acc, P) : P;
      started = true;
    }
  }
  return acc;
}

}  // namespace h
}  // namespace spg
