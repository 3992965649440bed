// spg — ristretto255 group arithmetic on Fp (field.hpp), host and device.
// Replaces the curve25519-dalek RistrettoPoint operations the reference calls
// (src/group.rs:6-7,14-46,98-116; src/commitments.rs:25): twisted Edwards a = -1 in extended
// coordinates, the RFC 9496 ristretto255 encode / decode / one-way map, and the mixed "affine Niels"
// form (y+x, y-x, 2d*x*y) that the MSM kernels stream from HBM (96 B per precomputed point).
#pragma once
#include "field.hpp"

namespace spg {

struct Ext {  // (X:Y:Z:T), x = X/Z, y = Y/Z, T = XY/Z
  Fp X, Y, Z, T;
};
struct Niels {  // affine Niels: (y+x, y-x, 2d*x*y)
  Fp ypx, ymx, t2d;
};

// ---- curve constants (canonical little-endian u32 limbs; RFC 9496 section 4.1) ----
SPG_HD Fp c_d() {  // d = -121665/121666
  Fp r;
  const uint32_t v[8] = {0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du,
                         0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu};
  for (int i = 0; i < 8; i++) r.l[i] = v[i];
  return r;
}
SPG_HD Fp c_d2() {  // 2d
  Fp r;
  const uint32_t v[8] = {0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au,
                         0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu};
  for (int i = 0; i < 8; i++) r.l[i] = v[i];
  return r;
}
SPG_HD Fp c_sqrt_m1() {
  Fp r;
  const uint32_t v[8] = {0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u,
                         0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};
  for (int i = 0; i < 8; i++) r.l[i] = v[i];
  return r;
}
SPG_HD Fp c_sqrt_ad_minus_one() {
  Fp r;
  const uint32_t v[8] = {0x497b2e1bu, 0x7e97f6a0u, 0x1b7854bdu, 0xaf9d8e0cu,
                         0x31f5d1fdu, 0x0f3cfcc9u, 0x2b8348acu, 0x376931bfu};
  for (int i = 0; i < 8; i++) r.l[i] = v[i];
  return r;
}
SPG_HD Fp c_invsqrt_a_minus_d() {
  Fp r;
  const uint32_t v[8] = {0x805d40eau, 0x99c8fdaau, 0x5a4172beu, 0x9d2f1617u,
                         0xfe01d840u, 0x16c27b91u, 0xcfaffca2u, 0x786c8905u};
  for (int i = 0; i < 8; i++) r.l[i] = v[i];
  return r;
}
SPG_HD Fp c_one_minus_d_sq() {
  Fp r;
  const uint32_t v[8] = {0x945fc176u, 0xe27c09c1u, 0xcd5e350fu, 0x2c81a138u,
                         0xbe70dfe4u, 0x9994abddu, 0xb2b3e0d7u, 0x029072a8u};
  for (int i = 0; i < 8; i++) r.l[i] = v[i];
  return r;
}
SPG_HD Fp c_d_minus_one_sq() {
  Fp r;
  const uint32_t v[8] = {0x44ed4d20u, 0x31ad5aaau, 0xb01e1999u, 0xd29e4a2cu,
                         0x529b4eebu, 0x4cdcd32fu, 0xf66c2241u, 0x5968b37au};
  for (int i = 0; i < 8; i++) r.l[i] = v[i];
  return r;
}

SPG_HD Ext ext_identity() {
  Ext p;
  p.X = fp_zero(); p.Y = fp_one(); p.Z = fp_one(); p.T = fp_zero();
  return p;
}
// add-2008-hwcd-3 (9M)
SPG_HD Ext ext_add(const Ext& p, const Ext& q) {
  Fp A = fp_mul(fp_sub(p.Y, p.X), fp_sub(q.Y, q.X));
  Fp B = fp_mul(fp_add(p.Y, p.X), fp_add(q.Y, q.X));
  Fp C = fp_mul(fp_mul(p.T, c_d2()), q.T);
  Fp D = fp_mul(fp_add(p.Z, p.Z), q.Z);
  Fp E = fp_sub(B, A), F = fp_sub(D, C), G = fp_add(D, C), H = fp_add(B, A);
  Ext r;
  r.X = fp_mul(E, F); r.Y = fp_mul(G, H); r.T = fp_mul(E, H); r.Z = fp_mul(F, G);
  return r;
}
// mixed addition with an affine Niels point, optionally negated (7M)
SPG_HD Ext ext_madd(const Ext& p, const Niels& q, bool neg) {
  Fp qp = neg ? q.ymx : q.ypx;
  Fp qm = neg ? q.ypx : q.ymx;
  Fp A = fp_mul(fp_sub(p.Y, p.X), qm);
  Fp B = fp_mul(fp_add(p.Y, p.X), qp);
  Fp C = fp_mul(p.T, q.t2d);
  if (neg) C = fp_neg(C);
  Fp D = fp_add(p.Z, p.Z);
  Fp E = fp_sub(B, A), F = fp_sub(D, C), G = fp_add(D, C), H = fp_add(B, A);
  Ext r;
  r.X = fp_mul(E, F); r.Y = fp_mul(G, H); r.T = fp_mul(E, H); r.Z = fp_mul(F, G);
  return r;
}
// dbl-2008-hwcd, a = -1 (4M + 4S)
SPG_HD Ext ext_dbl(const Ext& p) {
  Fp A = fp_sqr(p.X), B = fp_sqr(p.Y);
  Fp zz = fp_sqr(p.Z);
  Fp C = fp_add(zz, zz);
  Fp E = fp_sub(fp_sub(fp_sqr(fp_add(p.X, p.Y)), A), B);
  Fp G = fp_sub(B, A);
  Fp F = fp_sub(G, C);
  Fp H = fp_neg(fp_add(A, B));
  Ext r;
  r.X = fp_mul(E, F); r.Y = fp_mul(G, H); r.T = fp_mul(E, H); r.Z = fp_mul(F, G);
  return r;
}
SPG_HD Ext ext_neg(const Ext& p) {
  Ext r = p;
  r.X = fp_neg(p.X); r.T = fp_neg(p.T);
  return r;
}
SPG_HD Niels ext_to_niels(const Ext& p) {
  Fp zi = fp_inv(p.Z);
  Fp x = fp_mul(p.X, zi), y = fp_mul(p.Y, zi);
  Niels n;
  n.ypx = fp_canon(fp_add(y, x));
  n.ymx = fp_canon(fp_sub(y, x));
  n.t2d = fp_canon(fp_mul(fp_mul(x, y), c_d2()));
  return n;
}
SPG_HD Ext niels_to_ext(const Niels& n) {
  // x = (ypx - ymx)/2, y = (ypx + ymx)/2 ; with Z = 2: X = ypx - ymx, Y = ypx + ymx, T = XY/2
  Ext p;
  p.X = fp_sub(n.ypx, n.ymx);
  p.Y = fp_add(n.ypx, n.ymx);
  p.Z = fp_small(2);
  // T/Z = xy -> T = 2xy = X*Y/2 ; compute via T = X*Y * inv(2)... use Z=4 form instead:
  // scale (X,Y,Z) by 2: X'=2X, Y'=2Y, Z'=4, T'=X*Y  (x = 2X/4 = X/2 ok, T'/Z' = XY/4 = xy)
  p.T = fp_mul(p.X, p.Y);
  p.X = fp_add(p.X, p.X);
  p.Y = fp_add(p.Y, p.Y);
  p.Z = fp_small(4);
  return p;
}

// RFC 9496 4.2 SQRT_RATIO_M1
SPG_HD bool fp_sqrt_ratio_m1(const Fp& u, const Fp& v, Fp& out) {
  Fp v3 = fp_mul(fp_sqr(v), v);
  Fp v7 = fp_mul(fp_sqr(v3), v);
  Fp r = fp_mul(fp_mul(u, v3), fp_pow22523(fp_mul(u, v7)));
  Fp check = fp_mul(v, fp_sqr(r));
  Fp nu = fp_neg(u);
  bool correct = fp_eq(check, u);
  bool flipped = fp_eq(check, nu);
  bool flipped_i = fp_eq(check, fp_mul(nu, c_sqrt_m1()));
  if (flipped || flipped_i) r = fp_mul(c_sqrt_m1(), r);
  out = fp_abs(r);
  return correct || flipped;
}
// RFC 9496 4.3.2 ENCODE
SPG_HD void ext_compress(const Ext& P, uint8_t out[32]) {
  Fp u1 = fp_mul(fp_add(P.Z, P.Y), fp_sub(P.Z, P.Y));
  Fp u2 = fp_mul(P.X, P.Y);
  Fp invsqrt;
  fp_sqrt_ratio_m1(fp_one(), fp_mul(u1, fp_sqr(u2)), invsqrt);
  Fp den1 = fp_mul(invsqrt, u1);
  Fp den2 = fp_mul(invsqrt, u2);
  Fp z_inv = fp_mul(fp_mul(den1, den2), P.T);
  bool rotate = fp_is_negative(fp_mul(P.T, z_inv));
  Fp x = P.X, y = P.Y, den_inv = den2;
  if (rotate) {
    x = fp_mul(P.Y, c_sqrt_m1());
    y = fp_mul(P.X, c_sqrt_m1());
    den_inv = fp_mul(den1, c_invsqrt_a_minus_d());
  }
  if (fp_is_negative(fp_mul(x, z_inv))) y = fp_neg(y);
  Fp s = fp_abs(fp_mul(den_inv, fp_sub(P.Z, y)));
  fp_to_bytes(s, out);
}
// RFC 9496 4.3.1 DECODE (returns false for an invalid encoding)
SPG_HD bool ext_decompress(const uint8_t in[32], Ext& out) {
  Fp s;
  for (int i = 0; i < 8; i++)
    s.l[i] = (uint32_t)in[4 * i] | ((uint32_t)in[4 * i + 1] << 8) | ((uint32_t)in[4 * i + 2] << 16) |
             ((uint32_t)in[4 * i + 3] << 24);
  Fp sc = fp_canon(s);
  bool canonical = true;
  for (int i = 0; i < 8; i++) canonical = canonical && (sc.l[i] == s.l[i]);
  if (!canonical || (s.l[0] & 1u)) return false;
  Fp ss = fp_sqr(s);
  Fp u1 = fp_sub(fp_one(), ss);
  Fp u2 = fp_add(fp_one(), ss);
  Fp u2s = fp_sqr(u2);
  Fp v = fp_sub(fp_neg(fp_mul(c_d(), fp_sqr(u1))), u2s);
  Fp invsqrt;
  bool was_square = fp_sqrt_ratio_m1(fp_one(), fp_mul(v, u2s), invsqrt);
  Fp den_x = fp_mul(invsqrt, u2);
  Fp den_y = fp_mul(fp_mul(invsqrt, den_x), v);
  Fp x = fp_abs(fp_mul(fp_add(s, s), den_x));
  Fp y = fp_mul(u1, den_y);
  Fp t = fp_mul(x, y);
  if (!was_square || fp_is_negative(t) || fp_is_zero(y)) return false;
  out.X = x; out.Y = y; out.Z = fp_one(); out.T = t;
  return true;
}
// RFC 9496 4.3.4 MAP
SPG_HD Ext ristretto_map(const Fp& t) {
  Fp one = fp_one();
  Fp r = fp_mul(c_sqrt_m1(), fp_sqr(t));
  Fp u = fp_mul(fp_add(r, one), c_one_minus_d_sq());
  Fp v = fp_mul(fp_sub(fp_neg(one), fp_mul(r, c_d())), fp_add(r, c_d()));
  Fp s;
  bool was_square = fp_sqrt_ratio_m1(u, v, s);
  Fp c = fp_neg(one);
  if (!was_square) {
    s = fp_neg(fp_abs(fp_mul(s, t)));
    c = r;
  }
  Fp N = fp_sub(fp_mul(fp_mul(c, fp_sub(r, one)), c_d_minus_one_sq()), v);
  Fp w0 = fp_mul(fp_add(s, s), v);
  Fp w1 = fp_mul(N, c_sqrt_ad_minus_one());
  Fp ss = fp_sqr(s);
  Fp w2 = fp_sub(one, ss);
  Fp w3 = fp_add(one, ss);
  Ext P;
  P.X = fp_mul(w0, w3); P.Y = fp_mul(w2, w1); P.Z = fp_mul(w1, w3); P.T = fp_mul(w0, w2);
  return P;
}
// RistrettoPoint::from_uniform_bytes
SPG_HD Ext ristretto_from_uniform_bytes(const uint8_t b[64]) {
  return ext_add(ristretto_map(fp_from_bytes(b)), ristretto_map(fp_from_bytes(b + 32)));
}
// scalar multiplication by canonical integer limbs (8 x u32), variable time
SPG_HD Ext ext_scalar_mul(const Ext& P, const uint32_t k[8]) {
  Ext acc = ext_identity();
  bool started = false;
  for (int i = 255; i >= 0; i--) {
    if (started) acc = ext_dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1u) {
      acc = started ? ext_add(acc, P) : P;
      started = true;
    }
  }
  return acc;
}

}  // namespace spg
