// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of the group arithmetic the reference takes from curve25519-dalek ^4.1.1
// (not vendored in /root/reference; call sites: src/group.rs:6-7,14-21,26-46,98-116,
// src/commitments.rs:18,25). The published algorithms restated here:
//   * GF(2^255-19) in radix 2^51 (the "donna-64" representation),
//   * twisted Edwards a=-1 group law in extended coordinates (Hisil-Wong-Carter-Dawson 2008,
//     add-2008-hwcd-3 / dbl-2008-hwcd),
//   * ristretto255 ENCODE / DECODE / MAP / one-way map exactly as RFC 9496 section 4.3,
//   * RistrettoPoint::from_uniform_bytes = MAP(b[0..32]) + MAP(b[32..64]) (RFC 9496 4.3.4).
// Pinned by RFC 9496 constants and cross-checked against libsodium 1.0.18 in tests.
#pragma once
#include <cstdint>
#include <cstring>

namespace orc {

typedef unsigned __int128 u128;

struct Fe { uint64_t l[5]; };
static const uint64_t FE_MASK51 = (1ULL << 51) - 1;

static inline Fe fe_zero() { Fe r = {{0, 0, 0, 0, 0}}; return r; }
static inline Fe fe_one() { Fe r = {{1, 0, 0, 0, 0}}; return r; }
static inline Fe fe_small(uint64_t x) { Fe r = {{x, 0, 0, 0, 0}}; return r; }

static inline Fe fe_carry(Fe a) {
  uint64_t c;
  for (int k = 0; k < 2; k++) {
    c = a.l[0] >> 51; a.l[0] &= FE_MASK51; a.l[1] += c;
    c = a.l[1] >> 51; a.l[1] &= FE_MASK51; a.l[2] += c;
    c = a.l[2] >> 51; a.l[2] &= FE_MASK51; a.l[3] += c;
    c = a.l[3] >> 51; a.l[3] &= FE_MASK51; a.l[4] += c;
    c = a.l[4] >> 51; a.l[4] &= FE_MASK51; a.l[0] += 19 * c;
  }
  return a;
}
static inline Fe fe_add(const Fe& a, const Fe& b) {
  Fe r;
  for (int i = 0; i < 5; i++) r.l[i] = a.l[i] + b.l[i];
  return fe_carry(r);
}
// a - b computed as a + 16p - b (limbs of b are < 2^52 after carry)
static inline Fe fe_sub(const Fe& a, const Fe& b) {
  Fe r;
  r.l[0] = a.l[0] + 0x7FFFFFFFFFFED0ULL - b.l[0];
  for (int i = 1; i < 5; i++) r.l[i] = a.l[i] + 0x7FFFFFFFFFFFF0ULL - b.l[i];
  return fe_carry(r);
}
static inline Fe fe_neg(const Fe& a) { return fe_sub(fe_zero(), a); }
static inline Fe fe_mul(const Fe& a, const Fe& b) {
  const uint64_t* x = a.l;
  const uint64_t* y = b.l;
  uint64_t y1_19 = 19 * y[1], y2_19 = 19 * y[2], y3_19 = 19 * y[3], y4_19 = 19 * y[4];
  u128 c0 = (u128)x[0] * y[0] + (u128)x[1] * y4_19 + (u128)x[2] * y3_19 + (u128)x[3] * y2_19 + (u128)x[4] * y1_19;
  u128 c1 = (u128)x[0] * y[1] + (u128)x[1] * y[0] + (u128)x[2] * y4_19 + (u128)x[3] * y3_19 + (u128)x[4] * y2_19;
  u128 c2 = (u128)x[0] * y[2] + (u128)x[1] * y[1] + (u128)x[2] * y[0] + (u128)x[3] * y4_19 + (u128)x[4] * y3_19;
  u128 c3 = (u128)x[0] * y[3] + (u128)x[1] * y[2] + (u128)x[2] * y[1] + (u128)x[3] * y[0] + (u128)x[4] * y4_19;
  u128 c4 = (u128)x[0] * y[4] + (u128)x[1] * y[3] + (u128)x[2] * y[2] + (u128)x[3] * y[1] + (u128)x[4] * y[0];
  Fe r;
  c1 += (uint64_t)(c0 >> 51); r.l[0] = (uint64_t)c0 & FE_MASK51;
  c2 += (uint64_t)(c1 >> 51); r.l[1] = (uint64_t)c1 & FE_MASK51;
  c3 += (uint64_t)(c2 >> 51); r.l[2] = (uint64_t)c2 & FE_MASK51;
  c4 += (uint64_t)(c3 >> 51); r.l[3] = (uint64_t)c3 & FE_MASK51;
  uint64_t carry = (uint64_t)(c4 >> 51); r.l[4] = (uint64_t)c4 & FE_MASK51;
  r.l[0] += carry * 19;
  return fe_carry(r);
}
static inline Fe fe_sq(const Fe& a) { return fe_mul(a, a); }
static inline Fe fe_pow2k(Fe a, int k) { for (int i = 0; i < k; i++) a = fe_sq(a); return a; }

// canonical little-endian encoding
static inline void fe_to_bytes(const Fe& a0, uint8_t out[32]) {
  Fe a = fe_carry(a0);
  // now each limb < 2^51 (+ tiny); compute a mod p exactly
  uint64_t q = (a.l[0] + 19) >> 51;
  q = (a.l[1] + q) >> 51;
  q = (a.l[2] + q) >> 51;
  q = (a.l[3] + q) >> 51;
  q = (a.l[4] + q) >> 51;
  a.l[0] += 19 * q;
  uint64_t c;
  c = a.l[0] >> 51; a.l[0] &= FE_MASK51; a.l[1] += c;
  c = a.l[1] >> 51; a.l[1] &= FE_MASK51; a.l[2] += c;
  c = a.l[2] >> 51; a.l[2] &= FE_MASK51; a.l[3] += c;
  c = a.l[3] >> 51; a.l[3] &= FE_MASK51; a.l[4] += c;
  a.l[4] &= FE_MASK51;
  uint64_t w[4];
  w[0] = a.l[0] | (a.l[1] << 51);
  w[1] = (a.l[1] >> 13) | (a.l[2] << 38);
  w[2] = (a.l[2] >> 26) | (a.l[3] << 25);
  w[3] = (a.l[3] >> 39) | (a.l[4] << 12);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
// dalek FieldElement::from_bytes: ignores the top bit, accepts non-canonical values (reduces them)
static inline Fe fe_from_bytes(const uint8_t in[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int j = 7; j >= 0; j--) w[i] = (w[i] << 8) | in[8 * i + j];
  }
  Fe r;
  r.l[0] = w[0] & FE_MASK51;
  r.l[1] = ((w[0] >> 51) | (w[1] << 13)) & FE_MASK51;
  r.l[2] = ((w[1] >> 38) | (w[2] << 26)) & FE_MASK51;
  r.l[3] = ((w[2] >> 25) | (w[3] << 39)) & FE_MASK51;
  r.l[4] = (w[3] >> 12) & FE_MASK51;
  return r;
}
static inline bool fe_eq(const Fe& a, const Fe& b) {
  uint8_t x[32], y[32];
  fe_to_bytes(a, x); fe_to_bytes(b, y);
  return memcmp(x, y, 32) == 0;
}
static inline bool fe_is_negative(const Fe& a) { uint8_t x[32]; fe_to_bytes(a, x); return x[0] & 1; }
static inline bool fe_is_zero(const Fe& a) { return fe_eq(a, fe_zero()); }
static inline Fe fe_select(const Fe& a, const Fe& b, bool pick_b) { return pick_b ? b : a; }
static inline Fe fe_abs(const Fe& a) { return fe_is_negative(a) ? fe_neg(a) : a; }

// a^((p-5)/8) = a^(2^252 - 3) via the standard ref10 chain
static inline Fe fe_pow22523(const Fe& z) {
  Fe t0 = fe_sq(z);
  Fe t1 = fe_pow2k(t0, 2);
  t1 = fe_mul(z, t1);
  t0 = fe_mul(t0, t1);
  t0 = fe_sq(t0);
  t0 = fe_mul(t1, t0);
  t1 = fe_pow2k(t0, 5);
  t0 = fe_mul(t1, t0);
  t1 = fe_pow2k(t0, 10);
  t1 = fe_mul(t1, t0);
  Fe t2 = fe_pow2k(t1, 20);
  t1 = fe_mul(t2, t1);
  t1 = fe_pow2k(t1, 10);
  t0 = fe_mul(t1, t0);
  t1 = fe_pow2k(t0, 50);
  t1 = fe_mul(t1, t0);
  t2 = fe_pow2k(t1, 100);
  t1 = fe_mul(t2, t1);
  t1 = fe_pow2k(t1, 50);
  t0 = fe_mul(t1, t0);
  t0 = fe_pow2k(t0, 2);
  return fe_mul(t0, z);
}
static inline Fe fe_invert(const Fe& z) {
  // z^(p-2) = z^(2^255-21) = (z^(2^252-3))^8 * z^3
  Fe t = fe_pow22523(z);
  t = fe_pow2k(t, 3);
  return fe_mul(t, fe_mul(fe_sq(z), z));
}

struct RConsts {
  Fe d, d2, sqrt_m1, sqrt_ad_minus_one, invsqrt_a_minus_d, one_minus_d_sq, d_minus_one_sq;
};

// RFC 9496 4.2 SQRT_RATIO_M1
static inline bool fe_sqrt_ratio_m1(const Fe& u, const Fe& v, const Fe& sqrt_m1, Fe* out) {
  Fe v3 = fe_mul(fe_sq(v), v);
  Fe v7 = fe_mul(fe_sq(v3), v);
  Fe r = fe_mul(fe_mul(u, v3), fe_pow22523(fe_mul(u, v7)));
  Fe check = fe_mul(v, fe_sq(r));
  Fe neg_u = fe_neg(u);
  bool correct = fe_eq(check, u);
  bool flipped = fe_eq(check, neg_u);
  bool flipped_i = fe_eq(check, fe_mul(neg_u, sqrt_m1));
  Fe r_prime = fe_mul(sqrt_m1, r);
  r = fe_select(r, r_prime, flipped || flipped_i);
  *out = fe_abs(r);
  return correct || flipped;
}

// computed once; the function-local static makes the first use thread-safe (bench.py runs one oracle prove per
// host core concurrently for the all-cores CPU baseline)
static inline RConsts rconsts_compute() {
  RConsts c;
  {
    // d = -121665/121666
    c.d = fe_mul(fe_neg(fe_small(121665)), fe_invert(fe_small(121666)));
    c.d2 = fe_add(c.d, c.d);
    // sqrt(-1) = 2^((p-1)/4)
    {
      // (p-1)/4 = 2^253 - 5 ; 2^((p-1)/4) by square-and-multiply over the exponent bits
      Fe base = fe_small(2), acc = fe_one();
      for (int i = 252; i >= 0; i--) {
        acc = fe_sq(acc);
        // 2^253 - 5 = 0b1...1011 : every bit of 0..252 set except bit 2
        if (i != 2) acc = fe_mul(acc, base);
      }
      c.sqrt_m1 = acc;
    }
    // SQRT_AD_MINUS_ONE = sqrt(a*d - 1) with a = -1 ; RFC 9496 fixes the root whose encoding is odd
    // ("negative"), i.e. the negation of the nonnegative root SQRT_RATIO_M1 returns.
    Fe ad_m1 = fe_sub(fe_neg(c.d), fe_one());
    fe_sqrt_ratio_m1(ad_m1, fe_one(), c.sqrt_m1, &c.sqrt_ad_minus_one);
    c.sqrt_ad_minus_one = fe_neg(c.sqrt_ad_minus_one);
    // INVSQRT_A_MINUS_D = 1/sqrt(a - d)
    Fe a_m_d = fe_sub(fe_neg(fe_one()), c.d);
    fe_sqrt_ratio_m1(fe_one(), a_m_d, c.sqrt_m1, &c.invsqrt_a_minus_d);
    c.one_minus_d_sq = fe_sub(fe_one(), fe_sq(c.d));
    Fe dm1 = fe_sub(c.d, fe_one());
    c.d_minus_one_sq = fe_sq(dm1);
  }
  return c;
}
static inline const RConsts& rconsts() {
  static const RConsts c = rconsts_compute();
  return c;
}

// Extended twisted Edwards coordinates (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z, curve -x^2+y^2 = 1+d x^2 y^2
struct Ge { Fe X, Y, Z, T; };

static inline Ge ge_identity() { Ge p; p.X = fe_zero(); p.Y = fe_one(); p.Z = fe_one(); p.T = fe_zero(); return p; }

// add-2008-hwcd-3
static inline Ge ge_add(const Ge& p, const Ge& q) {
  const RConsts& c = rconsts();
  Fe A = fe_mul(fe_sub(p.Y, p.X), fe_sub(q.Y, q.X));
  Fe B = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));
  Fe C = fe_mul(fe_mul(p.T, c.d2), q.T);
  Fe D = fe_mul(fe_add(p.Z, p.Z), q.Z);
  Fe E = fe_sub(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
  Ge r;
  r.X = fe_mul(E, F); r.Y = fe_mul(G, H); r.T = fe_mul(E, H); r.Z = fe_mul(F, G);
  return r;
}
// dbl-2008-hwcd with a = -1
static inline Ge ge_double(const Ge& p) {
  Fe A = fe_sq(p.X), B = fe_sq(p.Y);
  Fe zz = fe_sq(p.Z);
  Fe C = fe_add(zz, zz);
  Fe xy = fe_add(p.X, p.Y);
  Fe E = fe_sub(fe_sub(fe_sq(xy), A), B);
  Fe G = fe_sub(B, A);
  Fe F = fe_sub(G, C);
  Fe H = fe_neg(fe_add(A, B));
  Ge r;
  r.X = fe_mul(E, F); r.Y = fe_mul(G, H); r.T = fe_mul(E, H); r.Z = fe_mul(F, G);
  return r;
}
static inline Ge ge_neg(const Ge& p) { Ge r = p; r.X = fe_neg(p.X); r.T = fe_neg(p.T); return r; }
static inline Ge ge_sub(const Ge& p, const Ge& q) { return ge_add(p, ge_neg(q)); }

// RFC 9496 4.3.2 ENCODE
static inline void ge_compress(const Ge& P, uint8_t out[32]) {
  const RConsts& c = rconsts();
  Fe u1 = fe_mul(fe_add(P.Z, P.Y), fe_sub(P.Z, P.Y));
  Fe u2 = fe_mul(P.X, P.Y);
  Fe invsqrt;
  fe_sqrt_ratio_m1(fe_one(), fe_mul(u1, fe_sq(u2)), c.sqrt_m1, &invsqrt);
  Fe den1 = fe_mul(invsqrt, u1);
  Fe den2 = fe_mul(invsqrt, u2);
  Fe z_inv = fe_mul(fe_mul(den1, den2), P.T);
  Fe ix0 = fe_mul(P.X, c.sqrt_m1);
  Fe iy0 = fe_mul(P.Y, c.sqrt_m1);
  Fe ench = fe_mul(den1, c.invsqrt_a_minus_d);
  bool rotate = fe_is_negative(fe_mul(P.T, z_inv));
  Fe x = fe_select(P.X, iy0, rotate);
  Fe y = fe_select(P.Y, ix0, rotate);
  Fe z = P.Z;
  Fe den_inv = fe_select(den2, ench, rotate);
  if (fe_is_negative(fe_mul(x, z_inv))) y = fe_neg(y);
  Fe s = fe_abs(fe_mul(den_inv, fe_sub(z, y)));
  fe_to_bytes(s, out);
}
// RFC 9496 4.3.1 DECODE; returns false on invalid encoding
static inline bool ge_decompress(const uint8_t in[32], Ge* out) {
  const RConsts& c = rconsts();
  Fe s = fe_from_bytes(in);
  uint8_t chk[32];
  fe_to_bytes(s, chk);
  if (memcmp(chk, in, 32) != 0) return false;  // non-canonical (incl. top bit set)
  if (fe_is_negative(s)) return false;
  Fe ss = fe_sq(s);
  Fe u1 = fe_sub(fe_one(), ss);
  Fe u2 = fe_add(fe_one(), ss);
  Fe u2_sqr = fe_sq(u2);
  Fe v = fe_sub(fe_neg(fe_mul(c.d, fe_sq(u1))), u2_sqr);
  Fe invsqrt;
  bool was_square = fe_sqrt_ratio_m1(fe_one(), fe_mul(v, u2_sqr), c.sqrt_m1, &invsqrt);
  Fe den_x = fe_mul(invsqrt, u2);
  Fe den_y = fe_mul(fe_mul(invsqrt, den_x), v);
  Fe x = fe_abs(fe_mul(fe_add(s, s), den_x));
  Fe y = fe_mul(u1, den_y);
  Fe t = fe_mul(x, y);
  if (!was_square || fe_is_negative(t) || fe_is_zero(y)) return false;
  out->X = x; out->Y = y; out->Z = fe_one(); out->T = t;
  return true;
}
// RFC 9496 4.3.4 MAP
static inline Ge ge_map(const Fe& t) {
  const RConsts& c = rconsts();
  Fe one = fe_one();
  Fe r = fe_mul(c.sqrt_m1, fe_sq(t));
  Fe u = fe_mul(fe_add(r, one), c.one_minus_d_sq);
  Fe v = fe_mul(fe_sub(fe_neg(one), fe_mul(r, c.d)), fe_add(r, c.d));
  Fe s;
  bool was_square = fe_sqrt_ratio_m1(u, v, c.sqrt_m1, &s);
  Fe s_prime = fe_neg(fe_abs(fe_mul(s, t)));
  s = fe_select(s_prime, s, was_square);
  Fe cc = fe_select(r, fe_neg(one), was_square);
  Fe N = fe_sub(fe_mul(fe_mul(cc, fe_sub(r, one)), c.d_minus_one_sq), v);
  Fe w0 = fe_mul(fe_add(s, s), v);
  Fe w1 = fe_mul(N, c.sqrt_ad_minus_one);
  Fe ss = fe_sq(s);
  Fe w2 = fe_sub(one, ss);
  Fe w3 = fe_add(one, ss);
  Ge P;
  P.X = fe_mul(w0, w3); P.Y = fe_mul(w2, w1); P.Z = fe_mul(w1, w3); P.T = fe_mul(w0, w2);
  return P;
}
// RistrettoPoint::from_uniform_bytes (dalek) == RFC 9496 hash-to-group one-way map
static inline Ge ge_from_uniform_bytes(const uint8_t b[64]) {
  Fe t0 = fe_from_bytes(b);
  Fe t1 = fe_from_bytes(b + 32);
  return ge_add(ge_map(t0), ge_map(t1));
}
// ristretto equality (dalek ConstantTimeEq for RistrettoPoint)
static inline bool ge_eq(const Ge& p, const Ge& q) {
  return fe_eq(fe_mul(p.X, q.Y), fe_mul(p.Y, q.X)) || fe_eq(fe_mul(p.Y, q.Y), fe_mul(p.X, q.X));
}
// basepoint = RISTRETTO_BASEPOINT_COMPRESSED (RFC 9496 generator)
static const uint8_t RISTRETTO_BASEPOINT_COMPRESSED[32] = {
    0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9, 0x61, 0xc5, 0x00, 0x51, 0x5f,
    0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82, 0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};

// variable-base scalar multiplication by a canonical little-endian 32-byte scalar (double-and-add)
static inline Ge ge_scalarmul_bytes(const Ge& P, const uint8_t k[32]) {
  Ge acc = ge_identity();
  for (int i = 255; i >= 0; i--) {
    acc = ge_double(acc);
    if ((k[i >> 3] >> (i & 7)) & 1) acc = ge_add(acc, P);
  }
  return acc;
}

}  // namespace orc
