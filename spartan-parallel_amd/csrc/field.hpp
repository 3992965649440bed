// spg — MI355X-native Spartan prover hot path.
// Exact modular arithmetic for the two fields of ristretto255, written for CDNA4's 32-bit VALU
// (v_mad_u64_u32 / v_add_co_ci_u32 chains), usable from host code too (__host__ __device__).
//
//  * Fq : scalar field, q = 2^252 + 27742317777372353535851937790883648493. Montgomery form with
//         R = 2^256 over 8 little-endian u32 limbs. Because R is the same as the reference's
//         (src/scalar/ristretto255.rs:193-199, four u64 limbs), the limb bytes are identical to the
//         reference's in-memory / serde layout and every result is the unique canonical value in [0,q).
//         CIOS Montgomery multiplication; q's limbs 4..6 are zero and limb 7 is 2^28, which the
//         reduction exploits.
//  * Fp : GF(2^255-19) for curve points. Loose representation in [0, 2^256) with 2^256 = 38 (mod p);
//         canonicalised only for encoding and comparisons.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SPG_HD __host__ __device__ __forceinline__
#else
#define SPG_HD inline
#endif

namespace spg {

// ---------------------------------------------------------------- carry helpers
// On the device these lower to single v_add_co_ci / v_sub_co_ci instructions (carry in VCC); the 64-bit
// formulation costs ~4 instructions per limb there.
SPG_HD uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_addc(a, b, cin, &cout);
#else
  uint64_t s = (uint64_t)a + b + cin;
  cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}
SPG_HD uint32_t subb(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_subc(a, b, bin, &bout);
#else
  uint64_t d = (uint64_t)a - b - bin;
  bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
#endif
}
// (hi:lo) = a*b + c + d ; never overflows 64 bits
SPG_HD uint64_t mad(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return (uint64_t)a * b + c + d;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// host form of mac_ov below (same arithmetic; used to test the device algorithms on the CPU)
inline void mac_ov(uint64_t& acc, uint32_t& ov, uint32_t a, uint32_t b) {
  const uint64_t s = acc + (uint64_t)a * b;
  ov += s < acc;
  acc = s;
}
#endif
#if defined(__HIP_DEVICE_COMPILE__)
// acc (64 bits) += a * b with the carry out of bit 64 counted in ov: one v_mad_u64_u32 (64-bit addend,
// carry to an SGPR pair) + one v_addc_co_u32. Product scanning with this keeps a 255-bit product at
// ~2 instructions per limb product instead of ~5 for the row form with 32-bit addends.
__device__ __forceinline__ void mac_ov(uint64_t& acc, uint32_t& ov, uint32_t a, uint32_t b) {
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cy) : "v"(a), "v"(b));
  asm("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(ov), "=s"(cy) : "s"(cy));
}
#endif
// A product-scanning column accumulator whose overflow additions trail their products by two: on gfx950 a VALU
// write of the carry SGPR pair needs two wait states before a VALU reads it as carry-in, so mac_ov's v_addc right
// after its v_mad_u64_u32 costs an s_nop per limb product; here the next two products fill those slots. flush()
// before the column's ov is read. (Host: plain mac_ov.)
struct MacAcc {
  uint64_t acc = 0;
  uint32_t ov = 0;
  uint64_t c0 = 0, c1 = 0;  // carries of the last two products not yet added into ov (device)
  int np = 0;               // how many (a compile-time constant once the column loops unroll)
};
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void mac_addc(uint32_t& ov, uint64_t cy) {
  uint64_t d;
  asm("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(ov), "=s"(d) : "s"(cy));
}
__device__ __forceinline__ void mac(MacAcc& m, uint32_t a, uint32_t b) {
  uint64_t c;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(m.acc), "=s"(c) : "v"(a), "v"(b));
  if (m.np == 2) {
    mac_addc(m.ov, m.c0);
    m.c0 = m.c1;
    m.c1 = c;
  } else if (m.np == 1) {
    m.c1 = c;
    m.np = 2;
  } else {
    m.c0 = c;
    m.np = 1;
  }
}
__device__ __forceinline__ void mac_flush(MacAcc& m) {
  if (m.np >= 1) mac_addc(m.ov, m.c0);
  if (m.np == 2) mac_addc(m.ov, m.c1);
  m.np = 0;
}
#else
inline void mac(MacAcc& m, uint32_t a, uint32_t b) { mac_ov(m.acc, m.ov, a, b); }
inline void mac_flush(MacAcc&) {}
#endif
// column done: its low limb out, the accumulator shifted down with the overflow count on top
SPG_HD uint32_t mac_next(MacAcc& m) {
  mac_flush(m);
  const uint32_t lo = (uint32_t)m.acc;
  m.acc = (m.acc >> 32) | ((uint64_t)m.ov << 32);
  m.ov = 0;
  return lo;
}
// The device's product-scanning forms, compiled for the host too (through the host mac_ov above), so
// tests/test_product_host.py checks them against the oracle without a GPU (fp ops 6 and 7 of hostcheck).
// t[0..16) = a * b (8 x 32-bit limbs each), product scanning
SPG_HD void mul_8x8(const uint32_t* a, const uint32_t* b, uint32_t* t) {
  MacAcc m;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      mac(m, a[i], b[j]);
    }
    t[k] = mac_next(m);
  }
  t[15] = (uint32_t)m.acc;
}
// t[0..16) = a^2: the 28 off-diagonal products once (product scanning), doubled, plus the 8 squares
SPG_HD void sqr_8(const uint32_t* a, uint32_t* t) {
  MacAcc m;
  t[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j <= i || j > 7) continue;
      mac(m, a[i], a[j]);
    }
    t[k] = mac_next(m);
  }
  t[14] = (uint32_t)m.acc;
  t[15] = (uint32_t)(m.acc >> 32);
#pragma unroll
  for (int i = 15; i > 0; i--) t[i] = (t[i] << 1) | (t[i - 1] >> 31);
  t[0] <<= 1;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t v = (uint64_t)a[i] * a[i];
    t[2 * i] = addc(t[2 * i], (uint32_t)v, c, c);
    t[2 * i + 1] = addc(t[2 * i + 1], (uint32_t)(v >> 32), c, c);
  }
}

// ================================================================= Fq (Montgomery, R = 2^256)
struct Fq {
  uint32_t l[8];
};

#define SPG_Q0 0x5cf5d3edu
#define SPG_Q1 0x5812631au
#define SPG_Q2 0xa2f79cd6u
#define SPG_Q3 0x14def9deu
#define SPG_Q7 0x10000000u
#define SPG_QINV 0x12547e1bu  // -q^{-1} mod 2^32

SPG_HD Fq fq_zero() { Fq r; for (int i = 0; i < 8; i++) r.l[i] = 0; return r; }
// R mod q = Montgomery one
SPG_HD Fq fq_one() {
  Fq r;
  r.l[0] = 0x8d98951du; r.l[1] = 0xd6ec3174u; r.l[2] = 0x737dcf70u; r.l[3] = 0xc6ef5bf4u;
  r.l[4] = 0xfffffffeu; r.l[5] = 0xffffffffu; r.l[6] = 0xffffffffu; r.l[7] = 0x0fffffffu;
  return r;
}
SPG_HD Fq fq_r2() {
  Fq r;
  r.l[0] = 0x449c0f01u; r.l[1] = 0xa40611e3u; r.l[2] = 0x68859347u; r.l[3] = 0xd00e1ba7u;
  r.l[4] = 0x17f5be65u; r.l[5] = 0xceec73d2u; r.l[6] = 0x7c309a3du; r.l[7] = 0x0399411bu;
  return r;
}
SPG_HD Fq fq_r3() {
  Fq r;
  r.l[0] = 0x7b83a2dbu; r.l[1] = 0x2a9e4968u; r.l[2] = 0xaef7f3ecu; r.l[3] = 0x278324e6u;
  r.l[4] = 0x04ec5b65u; r.l[5] = 0x8065dc6cu; r.l[6] = 0x3599cec7u; r.l[7] = 0x0e530b77u;
  return r;
}
SPG_HD bool fq_is_zero(const Fq& a) {
  uint32_t o = 0;
  for (int i = 0; i < 8; i++) o |= a.l[i];
  return o == 0;
}
SPG_HD bool fq_eq(const Fq& a, const Fq& b) {
  uint32_t o = 0;
  for (int i = 0; i < 8; i++) o |= a.l[i] ^ b.l[i];
  return o == 0;
}

// t (9 limbs, value < 2q) -> canonical: subtract q if t >= q
SPG_HD Fq fq_cond_sub(const uint32_t t[8], uint32_t t8) {
  const uint32_t Q[8] = {SPG_Q0, SPG_Q1, SPG_Q2, SPG_Q3, 0u, 0u, 0u, SPG_Q7};
  uint32_t d[8], b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = subb(t[i], Q[i], b, b);
  // borrow out of the 9-limb subtraction <=> t < q
  uint32_t b9;
  subb(t8, 0u, b, b9);
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = b9 ? t[i] : d[i];
  return r;
}

SPG_HD Fq fq_add(const Fq& a, const Fq& b) {
  uint32_t t[8], c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = addc(a.l[i], b.l[i], c, c);
  return fq_cond_sub(t, c);
}
SPG_HD Fq fq_sub(const Fq& a, const Fq& b) {
  const uint32_t Q[8] = {SPG_Q0, SPG_Q1, SPG_Q2, SPG_Q3, 0u, 0u, 0u, SPG_Q7};
  uint32_t t[8], bo = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = subb(a.l[i], b.l[i], bo, bo);
  uint32_t mask = 0u - bo, c = 0;
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = addc(t[i], Q[i] & mask, c, c);
  return r;
}
SPG_HD Fq fq_neg(const Fq& a) { return fq_sub(fq_zero(), a); }
SPG_HD Fq fq_dbl(const Fq& a) { return fq_add(a, a); }

// acc += x (x < 2^64) with the carry out of bit 64 counted in ov
SPG_HD void add_ov(uint64_t& acc, uint32_t& ov, uint64_t x) {
  const uint64_t s = acc + x;
  ov += s < acc;
  acc = s;
}
// Montgomery product a*b*2^-256 mod q by product scanning (the device form): column k of a*b and of m*q
// accumulate in one 64-bit register with an overflow counter (mac_ov: 2 instructions per limb product),
// m_k is fixed when column k < 8 completes. q has limbs 4..6 zero and limb 7 = 2^28, so m*q costs 3 limb
// products per column plus one shifted add: 64 + 32 products instead of CIOS's 96 three-instruction mads.
SPG_HD Fq fq_mul_ps(const Fq& a, const Fq& b) {
  const uint32_t Q[4] = {SPG_Q0, SPG_Q1, SPG_Q2, SPG_Q3};
  uint32_t m[8], r[8];
  MacAcc c;
#pragma unroll
  for (int k = 0; k < 16; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j >= 0 && j < 8) mac(c, a.l[i], b.l[j]);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;  // m_i * q_j, j in 1..3 (q_0 is folded in below when m_k is fixed)
      if (i < k && j >= 1 && j <= 3) mac(c, m[i], Q[j]);
    }
    if (k >= 7 && k - 7 < 8) add_ov(c.acc, c.ov, (uint64_t)m[k - 7] << 28);  // m_{k-7} * q_7
    if (k < 8) {
      m[k] = (uint32_t)c.acc * SPG_QINV;
      mac(c, m[k], Q[0]);  // clears the low 32 bits
      mac_next(c);
    } else {
      r[k - 8] = mac_next(c);
    }
  }
  return fq_cond_sub(r, (uint32_t)c.acc);
}

// CIOS Montgomery product a*b*2^-256 mod q over 8 x 32-bit limbs (the device form: v_mad_u64_u32)
SPG_HD Fq fq_mul32(const Fq& a, const Fq& b) {
  uint32_t t[10];
#pragma unroll
  for (int i = 0; i < 10; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t bi = b.l[i];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t v = mad(a.l[j], bi, t[j], c);
      t[j] = (uint32_t)v;
      c = (uint32_t)(v >> 32);
    }
    uint32_t c2;
    t[8] = addc(t[8], c, 0, c2);
    t[9] = c2;
    uint32_t m = t[0] * SPG_QINV;
    uint64_t v = mad(m, SPG_Q0, t[0], 0);
    c = (uint32_t)(v >> 32);
    v = mad(m, SPG_Q1, t[1], c); t[0] = (uint32_t)v; c = (uint32_t)(v >> 32);
    v = mad(m, SPG_Q2, t[2], c); t[1] = (uint32_t)v; c = (uint32_t)(v >> 32);
    v = mad(m, SPG_Q3, t[3], c); t[2] = (uint32_t)v; c = (uint32_t)(v >> 32);
    t[3] = addc(t[4], c, 0, c);
    t[4] = addc(t[5], c, 0, c);
    t[5] = addc(t[6], c, 0, c);
    // limb 7 of q is 2^28: m*q7 = m << 28 spread over two limbs
    uint64_t w = ((uint64_t)m << 28) + t[7] + c;
    t[6] = (uint32_t)w;
    c = (uint32_t)(w >> 32);
    t[7] = addc(t[8], c, 0, c);
    t[8] = t[9] + c;
  }
  return fq_cond_sub(t, t[8]);
}
#if !defined(__HIP_DEVICE_COMPILE__)
// The same Montgomery product on the host CPU over 4 x 64-bit limbs (64x64->128 multiplies), several
// times faster there; the Montgomery representative is unique, so both forms agree bit for bit.
inline Fq fq_mul_host64(const Fq& A, const Fq& B) {
  typedef unsigned __int128 u128;
  static const uint64_t q[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL};
  const uint64_t INV = 0xd2b51da312547e1bULL;  // -q^{-1} mod 2^64
  uint64_t a[4], b[4];
  for (int i = 0; i < 4; i++) {
    a[i] = (uint64_t)A.l[2 * i] | ((uint64_t)A.l[2 * i + 1] << 32);
    b[i] = (uint64_t)B.l[2 * i] | ((uint64_t)B.l[2 * i + 1] << 32);
  }
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
  for (int i = 0; i < 4; i++) {
    u128 c = (u128)a[0] * b[i] + t0;
    t0 = (uint64_t)c;
    c = (c >> 64) + (u128)a[1] * b[i] + t1;
    t1 = (uint64_t)c;
    c = (c >> 64) + (u128)a[2] * b[i] + t2;
    t2 = (uint64_t)c;
    c = (c >> 64) + (u128)a[3] * b[i] + t3;
    t3 = (uint64_t)c;
    c = (c >> 64) + t4;
    t4 = (uint64_t)c;
    uint64_t t5 = (uint64_t)(c >> 64);
    uint64_t m = t0 * INV;
    c = ((u128)m * q[0] + t0) >> 64;
    c += (u128)m * q[1] + t1;
    t0 = (uint64_t)c;
    c = (c >> 64) + t2;  // q[2] == 0
    t1 = (uint64_t)c;
    c = (c >> 64) + (u128)m * q[3] + t3;
    t2 = (uint64_t)c;
    c = (c >> 64) + t4;
    t3 = (uint64_t)c;
    t4 = t5 + (uint64_t)(c >> 64);
  }
  // t < 2q: subtract q once if t >= q
  uint64_t r[4];
  u128 d = (u128)t0 - q[0];
  r[0] = (uint64_t)d;
  uint64_t bw = (uint64_t)(d >> 64) & 1;
  d = (u128)t1 - q[1] - bw;
  r[1] = (uint64_t)d;
  bw = (uint64_t)(d >> 64) & 1;
  d = (u128)t2 - q[2] - bw;
  r[2] = (uint64_t)d;
  bw = (uint64_t)(d >> 64) & 1;
  d = (u128)t3 - q[3] - bw;
  r[3] = (uint64_t)d;
  bw = (uint64_t)(d >> 64) & 1;
  const bool keep = bw && !t4;  // t < q
  const uint64_t o[4] = {keep ? t0 : r[0], keep ? t1 : r[1], keep ? t2 : r[2], keep ? t3 : r[3]};
  Fq out;
  for (int i = 0; i < 4; i++) {
    out.l[2 * i] = (uint32_t)o[i];
    out.l[2 * i + 1] = (uint32_t)(o[i] >> 32);
  }
  return out;
}
#endif

SPG_HD Fq fq_mul(const Fq& a, const Fq& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fq_mul_ps(a, b);
#else
  return fq_mul_host64(a, b);
#endif
}
SPG_HD Fq fq_sqr(const Fq& a) { return fq_mul(a, a); }
// Montgomery -> canonical integer limbs (a * 2^-256 mod q), i.e. Scalar::to_bytes as limbs
SPG_HD Fq fq_from_mont(const Fq& a) {
  Fq one;
  for (int i = 0; i < 8; i++) one.l[i] = 0;
  one.l[0] = 1;
  return fq_mul(a, one);
}
SPG_HD Fq fq_to_mont(const Fq& a) { return fq_mul(a, fq_r2()); }
SPG_HD Fq fq_from_u64(uint64_t x) {
  Fq t = fq_zero();
  t.l[0] = (uint32_t)x;
  t.l[1] = (uint32_t)(x >> 32);
  return fq_to_mont(t);
}
#if !defined(__HIP_DEVICE_COMPILE__)
// Host inverse: Kaliski's almost-Montgomery inverse on 4 x 64-bit limbs, runs of trailing zeros shifted out at
// once (__builtin_ctzll). Invariant q = u s + v r; it ends with r' = am^-1 2^k mod q, n <= k <= 2n, and one
// Montgomery product with the precomputed R^3 2^-k turns that into (a^-1) R for am = a R. Variable time, which is
// fine here: the prover only inverts public Fiat-Shamir challenges (BulletReductionProof's u, src/nizk/bullet.rs:100).
// Same value as Scalar::invert (src/scalar/ristretto255.rs:541-595); 0 maps to 0 like the Fermat chain.
// tests/test_product_host.py::test_fq_ops[invert] checks it against the oracle.
struct FqInvTable {
  Fq c[512];  // c[k] = R^3 2^-k mod q (Montgomery form of R^2 2^-k)
  FqInvTable() {
    typedef unsigned __int128 u128;
    static const uint64_t q[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL};
    // x = R^3 mod q: fq_r2() is R^2 mod q in plain limbs; R^3 = fq_mul(R^2, R^2) (Montgomery: R^4 R^-1)
    const Fq r3 = fq_mul(fq_r2(), fq_r2());
    uint64_t x[4];
    for (int i = 0; i < 4; i++) x[i] = (uint64_t)r3.l[2 * i] | ((uint64_t)r3.l[2 * i + 1] << 32);
    for (int k = 0; k < 512; k++) {
      for (int i = 0; i < 4; i++) {
        c[k].l[2 * i] = (uint32_t)x[i];
        c[k].l[2 * i + 1] = (uint32_t)(x[i] >> 32);
      }
      if (x[0] & 1) {  // x + q (x < q < 2^253: no overflow)
        u128 cy = 0;
        for (int i = 0; i < 4; i++) {
          cy += (u128)x[i] + q[i];
          x[i] = (uint64_t)cy;
          cy >>= 64;
        }
      }
      for (int i = 0; i < 3; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 63);
      x[3] >>= 1;
    }
  }
};
inline Fq fq_inv_host(const Fq& am) {
  typedef unsigned __int128 u128;
  static const uint64_t q[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL};
  static const FqInvTable tab;
  uint64_t u[4] = {q[0], q[1], q[2], q[3]}, v[4], r[4] = {0, 0, 0, 0}, s[4] = {1, 0, 0, 0};
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)am.l[2 * i] | ((uint64_t)am.l[2 * i + 1] << 32);
  if ((v[0] | v[1] | v[2] | v[3]) == 0) return fq_zero();
  auto shr = [](uint64_t* a, int t) {  // 0 < t < 64
    for (int i = 0; i < 3; i++) a[i] = (a[i] >> t) | (a[i + 1] << (64 - t));
    a[3] >>= t;
  };
  auto shl = [](uint64_t* a, int t) {  // 0 < t < 64, no overflow by the invariant (r, s < 2q < 2^254)
    for (int i = 3; i > 0; i--) a[i] = (a[i] << t) | (a[i - 1] >> (64 - t));
    a[0] <<= t;
  };
  auto sub = [](uint64_t* a, const uint64_t* b) {  // a -= b, a >= b
    uint64_t bw = 0;
    for (int i = 0; i < 4; i++) {
      const u128 d = (u128)a[i] - b[i] - bw;
      a[i] = (uint64_t)d;
      bw = (uint64_t)(d >> 64) & 1;
    }
  };
  auto add = [](uint64_t* a, const uint64_t* b) {  // a += b, no overflow
    u128 cy = 0;
    for (int i = 0; i < 4; i++) {
      cy += (u128)a[i] + b[i];
      a[i] = (uint64_t)cy;
      cy >>= 64;
    }
  };
  auto gt = [](const uint64_t* a, const uint64_t* b) {
    for (int i = 3; i >= 0; i--)
      if (a[i] != b[i]) return a[i] > b[i];
    return false;
  };
  auto ctz = [](const uint64_t* a) {  // a != 0
    for (int i = 0; i < 4; i++)
      if (a[i]) return 64 * i + __builtin_ctzll(a[i]);
    return 256;
  };
  int k = 0;
  while (v[0] | v[1] | v[2] | v[3]) {
    if (!(u[0] & 1)) {
      for (int t = ctz(u); t > 0; t -= 63) {
        const int c = t < 63 ? t : 63;
        shr(u, c);
        shl(s, c);
        k += c;
      }
    } else if (!(v[0] & 1)) {
      for (int t = ctz(v); t > 0; t -= 63) {
        const int c = t < 63 ? t : 63;
        shr(v, c);
        shl(r, c);
        k += c;
      }
    } else if (gt(u, v)) {
      sub(u, v);
      shr(u, 1);
      add(r, s);
      shl(s, 1);
      k++;
    } else {
      sub(v, u);
      shr(v, 1);
      add(s, r);
      shl(r, 1);
      k++;
    }
  }
  if (!gt(q, r)) sub(r, q);  // r < q
  uint64_t o[4] = {q[0], q[1], q[2], q[3]};
  sub(o, r);  // am^-1 2^k mod q (r != 0 for am != 0)
  Fq y;
  for (int i = 0; i < 4; i++) {
    y.l[2 * i] = (uint32_t)o[i];
    y.l[2 * i + 1] = (uint32_t)(o[i] >> 32);
  }
  // y = a^-1 R^-1 2^k; fq_mul(y, R^3 2^-k) = a^-1 R
  return fq_mul(y, tab.c[k]);
}
#endif

// x^(q-2) by 4-bit fixed windows over the exponent (device; the host uses fq_inv_host)
SPG_HD Fq fq_inv(const Fq& a) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return fq_inv_host(a);
#endif
  // q - 2 limbs (little-endian u32)
  const uint32_t E[8] = {SPG_Q0 - 2u, SPG_Q1, SPG_Q2, SPG_Q3, 0u, 0u, 0u, SPG_Q7};
  Fq tab[16];
  tab[0] = fq_one();
  tab[1] = a;
  for (int i = 2; i < 16; i++) tab[i] = fq_mul(tab[i - 1], a);
  Fq r = fq_one();
  for (int i = 63; i >= 0; i--) {
    r = fq_sqr(fq_sqr(fq_sqr(fq_sqr(r))));
    uint32_t nib = (E[i >> 3] >> ((i & 7) * 4)) & 15u;
    if (nib) r = fq_mul(r, tab[nib]);
  }
  return r;
}

// ================================================================= Fp = GF(2^255 - 19)
struct Fp {
  uint32_t l[8];
};

SPG_HD Fp fp_zero() { Fp r; for (int i = 0; i < 8; i++) r.l[i] = 0; return r; }
SPG_HD Fp fp_one() { Fp r = fp_zero(); r.l[0] = 1; return r; }
SPG_HD Fp fp_small(uint32_t x) { Fp r = fp_zero(); r.l[0] = x; return r; }

// add c*38 (c small) into t with carry; returns the final carry
SPG_HD uint32_t fp_fold38(uint32_t t[8], uint32_t c) {
  uint64_t v = (uint64_t)c * 38u + t[0];
  t[0] = (uint32_t)v;
  uint32_t cc = (uint32_t)(v >> 32);
#pragma unroll
  for (int i = 1; i < 8; i++) t[i] = addc(t[i], 0, cc, cc);
  return cc;
}
SPG_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = addc(a.l[i], b.l[i], c, c);
  c = fp_fold38(r.l, c);
  r.l[0] += c * 38u;  // a second wrap leaves r < 38: no carry past limb 0
  return r;
}
SPG_HD Fp fp_sub(const Fp& a, const Fp& b) {
  Fp r;
  uint32_t bo = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = subb(a.l[i], b.l[i], bo, bo);
  // wrapped by 2^256 = 38 (mod p): subtract 38 per wrap (at most twice)
  uint32_t s = bo * 38u, b2 = 0;
  r.l[0] = subb(r.l[0], s, 0, b2);
#pragma unroll
  for (int i = 1; i < 8; i++) r.l[i] = subb(r.l[i], 0, b2, b2);
  // a second wrap leaves r >= 2^256 - 38 (limb 0 >= 2^32 - 38): no borrow past limb 0
  r.l[0] -= b2 * 38u;
  return r;
}
SPG_HD Fp fp_neg(const Fp& a) { return fp_sub(fp_zero(), a); }
// a + b (neg false) or a - b (neg true) in one carry pass, for lanes that need different ones: a + (b ^ m) + neg,
// then the wrap folded as in fp_add / fp_sub (the same representative as theirs)
SPG_HD Fp fp_addsub(const Fp& a, const Fp& b, bool neg) {
  const uint32_t m = neg ? 0xffffffffu : 0u;
  Fp r;
  uint32_t c = neg ? 1u : 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = addc(a.l[i], b.l[i] ^ m, c, c);
  // add: carry -> r + 38 ; sub: no carry (a < b, r = a - b + 2^256) -> r - 38, as + (2^256 - 38)
  const bool t = (c != 0) != neg;
  const uint32_t k0 = t ? (neg ? 0u - 38u : 38u) : 0u, kh = (t && neg) ? 0xffffffffu : 0u;
  uint32_t c2 = 0;
  r.l[0] = addc(r.l[0], k0, 0u, c2);
#pragma unroll
  for (int i = 1; i < 8; i++) r.l[i] = addc(r.l[i], kh, c2, c2);
  // a second wrap (add: r < 38 now; sub: r >= 2^256 - 76 now) touches limb 0 alone
  if (t) r.l[0] += neg ? (c2 ? 0u : 0u - 38u) : (c2 ? 38u : 0u);
  return r;
}
// a * k for a small k (< 2^18): 8 limb products and one 38-fold
SPG_HD Fp fp_mul_k(const Fp& a, uint32_t k) {
  Fp r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t v = mad(a.l[i], k, c, 0);
    r.l[i] = (uint32_t)v;
    c = (uint32_t)(v >> 32);
  }
  c = fp_fold38(r.l, c);  // c < 2^18: c * 38 + r[0] carries at most 1
  r.l[0] += c * 38u;      // a second wrap leaves r < 38 * 2^18: no carry past limb 0
  return r;
}

SPG_HD Fp fp_reduce512(uint32_t t[16]) {
  Fp r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t v = mad(t[8 + i], 38u, t[i], c);
    r.l[i] = (uint32_t)v;
    c = (uint32_t)(v >> 32);
  }
  c = fp_fold38(r.l, c);
  r.l[0] += c * 38u;  // c <= 38 above, so a second wrap leaves r < 38 * 38: no carry past limb 0
  return r;
}
// the device forms (product scanning), callable on the host for testing
SPG_HD Fp fp_mul_ps(const Fp& a, const Fp& b) {
  uint32_t t[16];
  mul_8x8(a.l, b.l, t);
  return fp_reduce512(t);
}
SPG_HD Fp fp_sqr_ps(const Fp& a) {
  uint32_t t[16];
  sqr_8(a.l, t);
  return fp_reduce512(t);
}
SPG_HD Fp fp_mul(const Fp& a, const Fp& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fp_mul_ps(a, b);
#else
  uint32_t t[16];
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t v = mad(a.l[j], b.l[i], t[i + j], c);
      t[i + j] = (uint32_t)v;
      c = (uint32_t)(v >> 32);
    }
    t[i + 8] = c;
  }
  return fp_reduce512(t);
#endif
}
SPG_HD Fp fp_sqr(const Fp& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fp_sqr_ps(a);
#else
  // off-diagonal products once, doubled, plus the diagonal
  uint32_t t[16];
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 7; i++) {
    uint32_t c = 0;
#pragma unroll
    for (int j = i + 1; j < 8; j++) {
      uint64_t v = mad(a.l[i], a.l[j], t[i + j], c);
      t[i + j] = (uint32_t)v;
      c = (uint32_t)(v >> 32);
    }
    t[i + 8] = c;
  }
  uint32_t top = 0;
#pragma unroll
  for (int i = 1; i < 16; i++) {
    uint32_t nt = t[i] >> 31;
    t[i] = (t[i] << 1) | top;
    top = nt;
  }
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t v = (uint64_t)a.l[i] * a.l[i];
    t[2 * i] = addc(t[2 * i], (uint32_t)v, c, c);
    t[2 * i + 1] = addc(t[2 * i + 1], (uint32_t)(v >> 32), c, c);
  }
  return fp_reduce512(t);
#endif
}
// canonical representative in [0, p)
SPG_HD Fp fp_canon(const Fp& a) {
  Fp r = a;
  // fold bit 255: v = (v mod 2^255) + 19*(v >> 255)
  uint32_t top = r.l[7] >> 31;
  r.l[7] &= 0x7fffffffu;
  uint32_t c = 0;
  r.l[0] = addc(r.l[0], top * 19u, 0, c);
#pragma unroll
  for (int i = 1; i < 8; i++) r.l[i] = addc(r.l[i], 0, c, c);
  // now r < 2^255 + 19 ; subtract p if r >= p (p = 2^255 - 19)
  const uint32_t P[8] = {0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                         0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};
  uint32_t d[8], b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = subb(r.l[i], P[i], b, b);
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = b ? r.l[i] : d[i];
  return r;
}
SPG_HD bool fp_is_zero(const Fp& a) {
  Fp c = fp_canon(a);
  uint32_t o = 0;
  for (int i = 0; i < 8; i++) o |= c.l[i];
  return o == 0;
}
SPG_HD bool fp_eq(const Fp& a, const Fp& b) { return fp_is_zero(fp_sub(a, b)); }
SPG_HD bool fp_is_negative(const Fp& a) { return fp_canon(a).l[0] & 1u; }
SPG_HD Fp fp_cneg(const Fp& a, bool neg) { return neg ? fp_neg(a) : a; }
SPG_HD Fp fp_abs(const Fp& a) { return fp_cneg(a, fp_is_negative(a)); }
SPG_HD Fp fp_sqrn(Fp a, int n) {
  for (int i = 0; i < n; i++) a = fp_sqr(a);
  return a;
}
// a^(2^252 - 3)
SPG_HD Fp fp_pow22523(const Fp& z) {
  Fp z2 = fp_sqr(z);
  Fp z9 = fp_mul(fp_sqrn(z2, 2), z);
  Fp z11 = fp_mul(z9, z2);
  Fp z2_5_0 = fp_mul(fp_sqr(z11), z9);
  Fp z2_10_0 = fp_mul(fp_sqrn(z2_5_0, 5), z2_5_0);
  Fp z2_20_0 = fp_mul(fp_sqrn(z2_10_0, 10), z2_10_0);
  Fp z2_40_0 = fp_mul(fp_sqrn(z2_20_0, 20), z2_20_0);
  Fp z2_50_0 = fp_mul(fp_sqrn(z2_40_0, 10), z2_10_0);
  Fp z2_100_0 = fp_mul(fp_sqrn(z2_50_0, 50), z2_50_0);
  Fp z2_200_0 = fp_mul(fp_sqrn(z2_100_0, 100), z2_100_0);
  Fp z2_250_0 = fp_mul(fp_sqrn(z2_200_0, 50), z2_50_0);
  return fp_mul(fp_sqrn(z2_250_0, 2), z);
}
SPG_HD Fp fp_inv(const Fp& z) {
  // z^(p-2) = (z^(2^252-3))^8 * z^3
  Fp t = fp_sqrn(fp_pow22523(z), 3);
  return fp_mul(t, fp_mul(fp_sqr(z), z));
}
SPG_HD Fp fp_from_bytes(const uint8_t b[32]) {
  Fp r;
  for (int i = 0; i < 8; i++)
    r.l[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
             ((uint32_t)b[4 * i + 3] << 24);
  r.l[7] &= 0x7fffffffu;  // dalek FieldElement::from_bytes ignores the top bit
  return r;
}
SPG_HD void fp_to_bytes(const Fp& a, uint8_t out[32]) {
  Fp c = fp_canon(a);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)c.l[i];
    out[4 * i + 1] = (uint8_t)(c.l[i] >> 8);
    out[4 * i + 2] = (uint8_t)(c.l[i] >> 16);
    out[4 * i + 3] = (uint8_t)(c.l[i] >> 24);
  }
}

}  // namespace spg
