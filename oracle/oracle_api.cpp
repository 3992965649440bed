// ORACLE — test infrastructure only. C entry points over the CPU restatement, loaded by tests/
// (ctypes), __graft_entry__.smoke() and bench.py's cpu_baseline leg. Never linked into the product.
#include <cstdint>
#include <cstring>
#include <vector>
#include "fq.hpp"
#include "msm.hpp"
#include "ristretto.hpp"
#include "transcript.hpp"

using namespace orc;

static inline Fq ld(const uint64_t* p) { Fq a; memcpy(a.v, p, 32); return a; }
static inline void st(uint64_t* p, const Fq& a) { memcpy(p, a.v, 32); }

extern "C" {

// ---- Fq (src/scalar/ristretto255.rs) ----
// op: 0 add, 1 sub, 2 mul, 3 neg(a), 4 square(a), 5 invert(a)
void orc_fq_binop(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) {
    Fq x = ld(a + 4 * i), y = (b ? ld(b + 4 * i) : fq_zero()), r;
    switch (op) {
      case 0: r = fq_add(x, y); break;
      case 1: r = fq_sub(x, y); break;
      case 2: r = fq_mul(x, y); break;
      case 3: r = fq_neg(x); break;
      case 4: r = fq_square(x); break;
      default: r = fq_invert(x); break;
    }
    st(out + 4 * i, r);
  }
}
void orc_fq_to_bytes(const uint64_t* a, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) fq_to_bytes(ld(a + 4 * i), out + 32 * i);
}
int orc_fq_from_bytes(const uint8_t* b, uint64_t* out) {
  Fq r;
  bool ok = fq_from_bytes(b, &r);
  st(out, r);
  return ok ? 1 : 0;
}
void orc_fq_from_bytes_wide(const uint8_t* b, uint64_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) st(out + 4 * i, fq_from_bytes_wide(b + 64 * i));
}
void orc_fq_from_u512(const uint64_t* limbs, uint64_t* out) { st(out, fq_from_u512(limbs)); }
void orc_fq_from_raw(const uint64_t* limbs, uint64_t* out) { st(out, fq_from_raw(limbs)); }
void orc_fq_from_u64(uint64_t x, uint64_t* out) { st(out, fq_from_u64(x)); }
void orc_fq_batch_invert(uint64_t* a, size_t n, uint64_t* allinv) {
  std::vector<Fq> v(n);
  for (size_t i = 0; i < n; i++) v[i] = ld(a + 4 * i);
  Fq r = fq_batch_invert(v);
  for (size_t i = 0; i < n; i++) st(a + 4 * i, v[i]);
  st(allinv, r);
}

// ---- hashing / transcript ----
void orc_keccak_f1600(uint8_t* state200) { keccak_f1600_bytes(state200); }
void orc_shake256(const uint8_t* in, size_t n, uint8_t* out, size_t m) {
  Shake256 s;
  s.absorb(in, n);
  s.squeeze(out, m);
}
// merlin conformance: Transcript::new(label); append_message(l1, m1); challenge_bytes(l2, out, m)
void orc_merlin_simple(const char* label, const char* l1, const uint8_t* m1, size_t m1n, const char* l2,
                       uint8_t* out, size_t m) {
  Transcript t(label);
  t.append_message(l1, m1, m1n);
  t.challenge_bytes(l2, out, m);
}

// ---- ristretto255 ----
int orc_ge_decompress_compress(const uint8_t* in, uint8_t* out) {
  Ge p;
  if (!ge_decompress(in, &p)) return 0;
  ge_compress(p, out);
  return 1;
}
void orc_ge_from_uniform_bytes(const uint8_t* b64, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) ge_compress(ge_from_uniform_bytes(b64 + 64 * i), out + 32 * i);
}
int orc_ge_add(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  Ge p, q;
  if (!ge_decompress(a, &p) || !ge_decompress(b, &q)) return 0;
  ge_compress(ge_add(p, q), out);
  return 1;
}
int orc_ge_double(const uint8_t* a, uint8_t* out) {
  Ge p;
  if (!ge_decompress(a, &p)) return 0;
  ge_compress(ge_double(p), out);
  return 1;
}
// k: canonical little-endian 32 bytes
int orc_ge_scalarmul(const uint8_t* P, const uint8_t* k, uint8_t* out) {
  Ge p;
  if (!ge_decompress(P, &p)) return 0;
  ge_compress(ge_scalarmul_bytes(p, k), out);
  return 1;
}
// RFC 9496 constants as canonical bytes: d, sqrt_m1, sqrt_ad_minus_one, invsqrt_a_minus_d, one_minus_d_sq, d_minus_one_sq
void orc_ristretto_consts(uint8_t* out6x32) {
  const RConsts& c = rconsts();
  fe_to_bytes(c.d, out6x32);
  fe_to_bytes(c.sqrt_m1, out6x32 + 32);
  fe_to_bytes(c.sqrt_ad_minus_one, out6x32 + 64);
  fe_to_bytes(c.invsqrt_a_minus_d, out6x32 + 96);
  fe_to_bytes(c.one_minus_d_sq, out6x32 + 128);
  fe_to_bytes(c.d_minus_one_sq, out6x32 + 160);
}

// ---- generators (src/commitments.rs:15-33) : count = n+1 compressed points ----
void orc_gens_stream(const uint8_t* label, size_t label_len, size_t count, uint8_t* out) {
  std::vector<Ge> g = gens_stream(label, label_len, count);
  for (size_t i = 0; i < count; i++) ge_compress(g[i], out + 32 * i);
}

// ---- MSM (src/group.rs:98-116) over compressed bases; scalars Montgomery ----
int orc_msm(const uint8_t* bases, const uint64_t* scalars, size_t n, uint8_t* out) {
  std::vector<Ge> P(n);
  for (size_t i = 0; i < n; i++)
    if (!ge_decompress(bases + 32 * i, &P[i])) return 0;
  std::vector<Fq> s(n);
  for (size_t i = 0; i < n; i++) s[i] = ld(scalars + 4 * i);
  ge_compress(vartime_msm(s.data(), P.data(), n), out);
  return 1;
}
// Hyrax rows (src/dense_mlpoly.rs:200-212): for i < L: C_i = MSM(Z[R i .. R(i+1)], G[0..R]) + blind_i * h
// bases: (>= R) compressed G followed by h at index nb. blinds may be NULL (zeros).
int orc_commit_rows(const uint8_t* bases, size_t nb, const uint8_t* h, const uint64_t* Z, size_t L, size_t R,
                    const uint64_t* blinds, uint8_t* out) {
  if (R > nb) return 0;
  Gens g;
  g.n = nb;
  g.G.resize(nb);
  for (size_t i = 0; i < nb; i++)
    if (!ge_decompress(bases + 32 * i, &g.G[i])) return 0;
  if (!ge_decompress(h, &g.h)) return 0;
  for (size_t i = 0; i < L; i++) {
    std::vector<Fq> row(R);
    for (size_t j = 0; j < R; j++) row[j] = ld(Z + 4 * (R * i + j));
    Fq bl = blinds ? ld(blinds + 4 * i) : fq_zero();
    ge_compress(commit_slice(row.data(), R, bl, g), out + 32 * i);
  }
  return 1;
}

}  // extern "C"
