// spg — host build of the product's field / curve / transcript code (the same headers the HIP kernels
// compile), exported for the CPU test suite so the arithmetic can be checked against the oracle
// without a GPU. Not part of the proving path.
#include <string.h>

#include "curve.hpp"
#include "keccak.hpp"

using namespace spg;

static Fq ldq(const uint64_t* p) { Fq a; memcpy(a.l, p, 32); return a; }
static void stq(uint64_t* p, const Fq& a) { memcpy(p, a.l, 32); }

extern "C" {

// op: 0 add, 1 sub, 2 mul, 3 neg, 4 square, 5 invert, 6 from_mont, 7 to_mont
void spgh_fq_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) {
    Fq x = ldq(a + 4 * i), y = b ? ldq(b + 4 * i) : fq_zero(), r;
    switch (op) {
      case 0: r = fq_add(x, y); break;
      case 1: r = fq_sub(x, y); break;
      case 2: r = fq_mul(x, y); break;
      case 3: r = fq_neg(x); break;
      case 4: r = fq_sqr(x); break;
      case 5: r = fq_inv(x); break;
      case 6: r = fq_from_mont(x); break;
      default: r = fq_to_mont(x); break;
    }
    stq(out + 4 * i, r);
  }
}

// op: 0 add, 1 sub, 2 mul, 3 sqr, 4 inv, 5 canon ; inputs/outputs as 8 x u32 (loose allowed)
void spgh_fp_op(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) {
    Fp x, y, r;
    memcpy(x.l, a + 8 * i, 32);
    if (b) memcpy(y.l, b + 8 * i, 32); else y = fp_zero();
    switch (op) {
      case 0: r = fp_add(x, y); break;
      case 1: r = fp_sub(x, y); break;
      case 2: r = fp_mul(x, y); break;
      case 3: r = fp_sqr(x); break;
      case 4: r = fp_inv(x); break;
      default: r = x; break;
    }
    r = fp_canon(r);
    memcpy(out + 8 * i, r.l, 32);
  }
}

void spgh_from_uniform(const uint8_t* b64, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) ext_compress(ristretto_from_uniform_bytes(b64 + 64 * i), out + 32 * i);
}
int spgh_roundtrip(const uint8_t* in, uint8_t* out) {
  Ext p;
  if (!ext_decompress(in, p)) return 0;
  ext_compress(p, out);
  return 1;
}
// op: 0 add, 1 double, 2 madd via niels, 3 madd negated
int spgh_point_op(int op, const uint8_t* a, const uint8_t* b, uint8_t* out) {
  Ext p, q;
  if (!ext_decompress(a, p)) return 0;
  if (op != 1 && !ext_decompress(b, q)) return 0;
  Ext r;
  switch (op) {
    case 0: r = ext_add(p, q); break;
    case 1: r = ext_dbl(p); break;
    case 2: r = ext_madd(p, ext_to_niels(q), false); break;
    default: r = ext_madd(p, ext_to_niels(q), true); break;
  }
  ext_compress(r, out);
  return 1;
}
int spgh_niels_roundtrip(const uint8_t* a, uint8_t* out) {
  Ext p;
  if (!ext_decompress(a, p)) return 0;
  ext_compress(niels_to_ext(ext_to_niels(p)), out);
  return 1;
}
void spgh_shake256(const uint8_t* in, size_t n, uint8_t* out, size_t m) {
  Shake256 s;
  s.update(in, n);
  s.read(out, m);
}
void spgh_merlin_simple(const char* label, const char* l1, const uint8_t* m1, size_t m1n, const char* l2,
                        uint8_t* out, size_t m) {
  Merlin t(label);
  t.message(l1, m1, m1n);
  t.challenge(l2, out, m);
}

}  // extern "C"
