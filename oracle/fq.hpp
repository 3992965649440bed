// ORACLE — test infrastructure only. Never linked into the product (spartan-parallel_amd/).
// CPU restatement of the scalar field Fq of ristretto255, q = 2^252 + 27742317777372353535851937790883648493,
// Montgomery form with R = 2^256 over four little-endian u64 limbs.
// Follows /root/reference/src/scalar/ristretto255.rs line by line:
//   adc/sbb/mac :19-36, MODULUS :244-249, INV :300, R/R2/R3 :303-324,
//   from_bytes :391-415, to_bytes :419-431, from_bytes_wide/from_u512 :435-466,
//   square :476-504, invert :541-595, batch_invert :597-639, montgomery_reduce :642-686,
//   mul :690-714, sub :718-735, add :738-747, neg :750-763.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace orc {

typedef unsigned __int128 u128;

struct Fq {
  uint64_t v[4];
  bool operator==(const Fq& o) const {
    return v[0] == o.v[0] && v[1] == o.v[1] && v[2] == o.v[2] && v[3] == o.v[3];
  }
  bool operator!=(const Fq& o) const { return !(*this == o); }
  bool is_zero() const { return (v[0] | v[1] | v[2] | v[3]) == 0; }
};

// ristretto255.rs:19-36
static inline uint64_t adc(uint64_t a, uint64_t b, uint64_t carry, uint64_t* c) {
  u128 r = (u128)a + (u128)b + (u128)carry;
  *c = (uint64_t)(r >> 64);
  return (uint64_t)r;
}
static inline uint64_t sbb(uint64_t a, uint64_t b, uint64_t borrow, uint64_t* bo) {
  u128 r = (u128)a - ((u128)b + (u128)(borrow >> 63));
  *bo = (uint64_t)(r >> 64);
  return (uint64_t)r;
}
static inline uint64_t mac(uint64_t a, uint64_t b, uint64_t c, uint64_t carry, uint64_t* co) {
  u128 r = (u128)a + (u128)b * (u128)c + (u128)carry;
  *co = (uint64_t)(r >> 64);
  return (uint64_t)r;
}

static const Fq FQ_MODULUS = {{0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL}};
static const uint64_t FQ_INV = 0xd2b51da312547e1bULL;
static const Fq FQ_R = {{0xd6ec31748d98951dULL, 0xc6ef5bf4737dcf70ULL, 0xfffffffffffffffeULL, 0x0fffffffffffffffULL}};
static const Fq FQ_R2 = {{0xa40611e3449c0f01ULL, 0xd00e1ba768859347ULL, 0xceec73d217f5be65ULL, 0x0399411b7c309a3dULL}};
static const Fq FQ_R3 = {{0x2a9e49687b83a2dbULL, 0x278324e6aef7f3ecULL, 0x8065dc6c04ec5b65ULL, 0x0e530b773599cec7ULL}};

static inline Fq fq_zero() { Fq z = {{0, 0, 0, 0}}; return z; }
static inline Fq fq_one() { return FQ_R; }

// ristretto255.rs:718-735
static inline Fq fq_sub(const Fq& a, const Fq& b) {
  uint64_t bo = 0, c = 0;
  uint64_t d0 = sbb(a.v[0], b.v[0], 0, &bo);
  uint64_t d1 = sbb(a.v[1], b.v[1], bo, &bo);
  uint64_t d2 = sbb(a.v[2], b.v[2], bo, &bo);
  uint64_t d3 = sbb(a.v[3], b.v[3], bo, &bo);
  d0 = adc(d0, FQ_MODULUS.v[0] & bo, 0, &c);
  d1 = adc(d1, FQ_MODULUS.v[1] & bo, c, &c);
  d2 = adc(d2, FQ_MODULUS.v[2] & bo, c, &c);
  d3 = adc(d3, FQ_MODULUS.v[3] & bo, c, &c);
  Fq r = {{d0, d1, d2, d3}};
  return r;
}
// ristretto255.rs:738-747
static inline Fq fq_add(const Fq& a, const Fq& b) {
  uint64_t c = 0;
  uint64_t d0 = adc(a.v[0], b.v[0], 0, &c);
  uint64_t d1 = adc(a.v[1], b.v[1], c, &c);
  uint64_t d2 = adc(a.v[2], b.v[2], c, &c);
  uint64_t d3 = adc(a.v[3], b.v[3], c, &c);
  Fq t = {{d0, d1, d2, d3}};
  return fq_sub(t, FQ_MODULUS);
}
// ristretto255.rs:750-763
static inline Fq fq_neg(const Fq& a) {
  uint64_t bo = 0;
  uint64_t d0 = sbb(FQ_MODULUS.v[0], a.v[0], 0, &bo);
  uint64_t d1 = sbb(FQ_MODULUS.v[1], a.v[1], bo, &bo);
  uint64_t d2 = sbb(FQ_MODULUS.v[2], a.v[2], bo, &bo);
  uint64_t d3 = sbb(FQ_MODULUS.v[3], a.v[3], bo, &bo);
  uint64_t mask = (uint64_t)((a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0) - 1;
  Fq r = {{d0 & mask, d1 & mask, d2 & mask, d3 & mask}};
  return r;
}
// ristretto255.rs:642-686
static inline Fq fq_mont_reduce(uint64_t r0, uint64_t r1, uint64_t r2, uint64_t r3, uint64_t r4,
                                uint64_t r5, uint64_t r6, uint64_t r7) {
  uint64_t carry, carry2;
  uint64_t k = r0 * FQ_INV;
  mac(r0, k, FQ_MODULUS.v[0], 0, &carry);
  r1 = mac(r1, k, FQ_MODULUS.v[1], carry, &carry);
  r2 = mac(r2, k, FQ_MODULUS.v[2], carry, &carry);
  r3 = mac(r3, k, FQ_MODULUS.v[3], carry, &carry);
  r4 = adc(r4, 0, carry, &carry2);

  k = r1 * FQ_INV;
  mac(r1, k, FQ_MODULUS.v[0], 0, &carry);
  r2 = mac(r2, k, FQ_MODULUS.v[1], carry, &carry);
  r3 = mac(r3, k, FQ_MODULUS.v[2], carry, &carry);
  r4 = mac(r4, k, FQ_MODULUS.v[3], carry, &carry);
  r5 = adc(r5, carry2, carry, &carry2);

  k = r2 * FQ_INV;
  mac(r2, k, FQ_MODULUS.v[0], 0, &carry);
  r3 = mac(r3, k, FQ_MODULUS.v[1], carry, &carry);
  r4 = mac(r4, k, FQ_MODULUS.v[2], carry, &carry);
  r5 = mac(r5, k, FQ_MODULUS.v[3], carry, &carry);
  r6 = adc(r6, carry2, carry, &carry2);

  k = r3 * FQ_INV;
  mac(r3, k, FQ_MODULUS.v[0], 0, &carry);
  r4 = mac(r4, k, FQ_MODULUS.v[1], carry, &carry);
  r5 = mac(r5, k, FQ_MODULUS.v[2], carry, &carry);
  r6 = mac(r6, k, FQ_MODULUS.v[3], carry, &carry);
  uint64_t dummy;
  r7 = adc(r7, carry2, carry, &dummy);

  Fq t = {{r4, r5, r6, r7}};
  return fq_sub(t, FQ_MODULUS);
}
// ristretto255.rs:690-714
static inline Fq fq_mul(const Fq& a, const Fq& b) {
  uint64_t c;
  uint64_t r0 = mac(0, a.v[0], b.v[0], 0, &c);
  uint64_t r1 = mac(0, a.v[0], b.v[1], c, &c);
  uint64_t r2 = mac(0, a.v[0], b.v[2], c, &c);
  uint64_t r4, r5, r6, r7;
  uint64_t r3 = mac(0, a.v[0], b.v[3], c, &r4);

  r1 = mac(r1, a.v[1], b.v[0], 0, &c);
  r2 = mac(r2, a.v[1], b.v[1], c, &c);
  r3 = mac(r3, a.v[1], b.v[2], c, &c);
  r4 = mac(r4, a.v[1], b.v[3], c, &r5);

  r2 = mac(r2, a.v[2], b.v[0], 0, &c);
  r3 = mac(r3, a.v[2], b.v[1], c, &c);
  r4 = mac(r4, a.v[2], b.v[2], c, &c);
  r5 = mac(r5, a.v[2], b.v[3], c, &r6);

  r3 = mac(r3, a.v[3], b.v[0], 0, &c);
  r4 = mac(r4, a.v[3], b.v[1], c, &c);
  r5 = mac(r5, a.v[3], b.v[2], c, &c);
  r6 = mac(r6, a.v[3], b.v[3], c, &r7);
  return fq_mont_reduce(r0, r1, r2, r3, r4, r5, r6, r7);
}
// ristretto255.rs:476-504
static inline Fq fq_square(const Fq& a) {
  uint64_t c;
  uint64_t r1 = mac(0, a.v[0], a.v[1], 0, &c);
  uint64_t r2 = mac(0, a.v[0], a.v[2], c, &c);
  uint64_t r4;
  uint64_t r3 = mac(0, a.v[0], a.v[3], c, &r4);
  r3 = mac(r3, a.v[1], a.v[2], 0, &c);
  uint64_t r5;
  r4 = mac(r4, a.v[1], a.v[3], c, &r5);
  uint64_t r6;
  r5 = mac(r5, a.v[2], a.v[3], 0, &r6);
  uint64_t r7 = r6 >> 63;
  r6 = (r6 << 1) | (r5 >> 63);
  r5 = (r5 << 1) | (r4 >> 63);
  r4 = (r4 << 1) | (r3 >> 63);
  r3 = (r3 << 1) | (r2 >> 63);
  r2 = (r2 << 1) | (r1 >> 63);
  r1 = r1 << 1;
  uint64_t r0 = mac(0, a.v[0], a.v[0], 0, &c);
  r1 = adc(0, r1, c, &c);
  r2 = mac(r2, a.v[1], a.v[1], c, &c);
  r3 = adc(0, r3, c, &c);
  r4 = mac(r4, a.v[2], a.v[2], c, &c);
  r5 = adc(0, r5, c, &c);
  r6 = mac(r6, a.v[3], a.v[3], c, &c);
  uint64_t d;
  r7 = adc(0, r7, c, &d);
  return fq_mont_reduce(r0, r1, r2, r3, r4, r5, r6, r7);
}
// ristretto255.rs:211-215  From<u64>
static inline Fq fq_from_u64(uint64_t x) {
  Fq t = {{x, 0, 0, 0}};
  return fq_mul(t, FQ_R2);
}
// ristretto255.rs:468-470  from_raw
static inline Fq fq_from_raw(const uint64_t v[4]) {
  Fq t = {{v[0], v[1], v[2], v[3]}};
  return fq_mul(t, FQ_R2);
}
// ristretto255.rs:419-431
static inline void fq_to_bytes(const Fq& a, uint8_t out[32]) {
  Fq t = fq_mont_reduce(a.v[0], a.v[1], a.v[2], a.v[3], 0, 0, 0, 0);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(t.v[i] >> (8 * j));
}
static inline uint64_t load_le64(const uint8_t* p) {
  uint64_t r = 0;
  for (int j = 7; j >= 0; j--) r = (r << 8) | p[j];
  return r;
}
// ristretto255.rs:391-415; returns canonical flag
static inline bool fq_from_bytes(const uint8_t b[32], Fq* out) {
  Fq t;
  for (int i = 0; i < 4; i++) t.v[i] = load_le64(b + 8 * i);
  uint64_t bo = 0;
  sbb(t.v[0], FQ_MODULUS.v[0], 0, &bo);
  sbb(t.v[1], FQ_MODULUS.v[1], bo, &bo);
  sbb(t.v[2], FQ_MODULUS.v[2], bo, &bo);
  sbb(t.v[3], FQ_MODULUS.v[3], bo, &bo);
  bool is_some = (bo & 1) != 0;
  *out = fq_mul(t, FQ_R2);
  return is_some;
}
// ristretto255.rs:449-466
static inline Fq fq_from_u512(const uint64_t l[8]) {
  Fq d0 = {{l[0], l[1], l[2], l[3]}};
  Fq d1 = {{l[4], l[5], l[6], l[7]}};
  return fq_add(fq_mul(d0, FQ_R2), fq_mul(d1, FQ_R3));
}
// ristretto255.rs:435-446
static inline Fq fq_from_bytes_wide(const uint8_t b[64]) {
  uint64_t l[8];
  for (int i = 0; i < 8; i++) l[i] = load_le64(b + 8 * i);
  return fq_from_u512(l);
}
// ristretto255.rs:541-595 (addition chain from curve25519-dalek)
static inline Fq fq_square_multiply(Fq y, int squarings, const Fq& x) {
  for (int i = 0; i < squarings; i++) y = fq_square(y);
  return fq_mul(y, x);
}
static inline Fq fq_invert(const Fq& a) {
  Fq _1 = a;
  Fq _10 = fq_square(_1);
  Fq _100 = fq_square(_10);
  Fq _11 = fq_mul(_10, _1);
  Fq _101 = fq_mul(_10, _11);
  Fq _111 = fq_mul(_10, _101);
  Fq _1001 = fq_mul(_10, _111);
  Fq _1011 = fq_mul(_10, _1001);
  Fq _1111 = fq_mul(_100, _1011);
  Fq y = fq_mul(_1111, _1);
  y = fq_square_multiply(y, 123 + 3, _101);
  y = fq_square_multiply(y, 2 + 2, _11);
  y = fq_square_multiply(y, 1 + 4, _1111);
  y = fq_square_multiply(y, 1 + 4, _1111);
  y = fq_square_multiply(y, 4, _1001);
  y = fq_square_multiply(y, 2, _11);
  y = fq_square_multiply(y, 1 + 4, _1111);
  y = fq_square_multiply(y, 1 + 3, _101);
  y = fq_square_multiply(y, 3 + 3, _101);
  y = fq_square_multiply(y, 3, _111);
  y = fq_square_multiply(y, 1 + 4, _1111);
  y = fq_square_multiply(y, 2 + 3, _111);
  y = fq_square_multiply(y, 2 + 2, _11);
  y = fq_square_multiply(y, 1 + 4, _1011);
  y = fq_square_multiply(y, 2 + 4, _1011);
  y = fq_square_multiply(y, 6 + 4, _1001);
  y = fq_square_multiply(y, 2 + 2, _11);
  y = fq_square_multiply(y, 3 + 2, _11);
  y = fq_square_multiply(y, 3 + 2, _11);
  y = fq_square_multiply(y, 1 + 4, _1001);
  y = fq_square_multiply(y, 1 + 3, _111);
  y = fq_square_multiply(y, 2 + 4, _1111);
  y = fq_square_multiply(y, 1 + 4, _1011);
  y = fq_square_multiply(y, 3, _101);
  y = fq_square_multiply(y, 2 + 4, _1111);
  y = fq_square_multiply(y, 3, _101);
  y = fq_square_multiply(y, 1 + 2, _11);
  return y;
}
// ristretto255.rs:597-639
static inline Fq fq_batch_invert(std::vector<Fq>& inputs) {
  size_t n = inputs.size();
  std::vector<Fq> scratch(n, fq_one());
  Fq acc = fq_one();
  for (size_t i = 0; i < n; i++) { scratch[i] = acc; acc = fq_mul(acc, inputs[i]); }
  acc = fq_invert(acc);
  Fq ret = acc;
  for (size_t i = n; i-- > 0;) {
    Fq tmp = fq_mul(acc, inputs[i]);
    inputs[i] = fq_mul(acc, scratch[i]);
    acc = tmp;
  }
  return ret;
}
// scalar/mod.rs:10-15  usize::to_scalar (repeated addition; equal to from_u64 for any usize)
static inline Fq fq_from_usize(size_t x) { return fq_from_u64((uint64_t)x); }

}  // namespace orc
