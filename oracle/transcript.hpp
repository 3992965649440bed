// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of the third-party hashing the reference depends on (absent from /root/reference):
//   * Keccak-f[1600] (FIPS 202), SHAKE256 XOF as used by sha3 ^0.8.2 in src/commitments.rs:15-33,
//   * merlin ^3.0.0: Strobe128 (STROBE v1.0.2, the minimal subset merlin implements) and Transcript
//     (append_message / challenge_bytes / append_u64), used by src/transcript.rs:1-63, src/random.rs:7-29,
//   * ProofTranscript helpers of src/transcript.rs:19-63 (append_scalar, challenge_scalar = from_bytes_wide(64 B)).
// Keccak is pinned against hashlib.sha3/shake in tests; merlin against its published conformance vector.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>
#include "fq.hpp"

namespace orc {

static inline uint64_t rotl64(uint64_t x, int s) { return s == 0 ? x : (x << s) | (x >> (64 - s)); }

static inline void keccak_f1600(uint64_t st[25]) {
  static const uint64_t RC[24] = {
      0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
      0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
      0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
      0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
      0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
      0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
  static const int ROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  for (int round = 0; round < 24; round++) {
    uint64_t C[5], D[5], B[25];
    for (int x = 0; x < 5; x++) C[x] = st[x] ^ st[x + 5] ^ st[x + 10] ^ st[x + 15] ^ st[x + 20];
    for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; i++) st[i] ^= D[i % 5];
    // rho + pi: B[y, 2x+3y] = rot(A[x,y], r[x,y])
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(st[x + 5 * y], ROT[x + 5 * y]);
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) st[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]);
    st[0] ^= RC[round];
  }
}
static inline void keccak_f1600_bytes(uint8_t s[200]) {
  uint64_t st[25];
  for (int i = 0; i < 25; i++) { st[i] = 0; for (int j = 7; j >= 0; j--) st[i] = (st[i] << 8) | s[8 * i + j]; }
  keccak_f1600(st);
  for (int i = 0; i < 25; i++) for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(st[i] >> (8 * j));
}

// SHAKE256: rate 136, domain suffix 0x1F
struct Shake256 {
  uint8_t s[200];
  size_t pos;
  bool squeezing;
  Shake256() { memset(s, 0, 200); pos = 0; squeezing = false; }
  void absorb(const uint8_t* d, size_t n) {
    for (size_t i = 0; i < n; i++) { s[pos++] ^= d[i]; if (pos == 136) { keccak_f1600_bytes(s); pos = 0; } }
  }
  void squeeze(uint8_t* out, size_t n) {
    if (!squeezing) { s[pos] ^= 0x1F; s[135] ^= 0x80; keccak_f1600_bytes(s); pos = 0; squeezing = true; }
    for (size_t i = 0; i < n; i++) { if (pos == 136) { keccak_f1600_bytes(s); pos = 0; } out[i] = s[pos++]; }
  }
};

// merlin Strobe128
struct Strobe128 {
  static const uint8_t R = 166;
  static const uint8_t FLAG_I = 1, FLAG_A = 2, FLAG_C = 4, FLAG_T = 8, FLAG_M = 16, FLAG_K = 32;
  uint8_t st[200];
  uint8_t pos, pos_begin, cur_flags;
  explicit Strobe128(const uint8_t* label, size_t len) {
    memset(st, 0, 200);
    const uint8_t init[6] = {1, R + 2, 1, 0, 1, 96};
    memcpy(st, init, 6);
    memcpy(st + 6, "STROBEv1.0.2", 12);
    keccak_f1600_bytes(st);
    pos = 0; pos_begin = 0; cur_flags = 0;
    meta_ad(label, len, false);
  }
  void run_f() {
    st[pos] ^= pos_begin;
    st[pos + 1] ^= 0x04;
    st[R + 1] ^= 0x80;
    keccak_f1600_bytes(st);
    pos = 0; pos_begin = 0;
  }
  void absorb(const uint8_t* d, size_t n) {
    for (size_t i = 0; i < n; i++) { st[pos] ^= d[i]; pos++; if (pos == R) run_f(); }
  }
  void overwrite(const uint8_t* d, size_t n) {
    for (size_t i = 0; i < n; i++) { st[pos] = d[i]; pos++; if (pos == R) run_f(); }
  }
  void squeeze(uint8_t* d, size_t n) {
    for (size_t i = 0; i < n; i++) { d[i] = st[pos]; st[pos] = 0; pos++; if (pos == R) run_f(); }
  }
  void begin_op(uint8_t flags, bool more) {
    if (more) return;  // merlin asserts cur_flags == flags
    uint8_t old_begin = pos_begin;
    pos_begin = pos + 1;
    cur_flags = flags;
    uint8_t b[2] = {old_begin, flags};
    absorb(b, 2);
    bool force_f = (flags & (FLAG_C | FLAG_K)) != 0;
    if (force_f && pos != 0) run_f();
  }
  void meta_ad(const uint8_t* d, size_t n, bool more) { begin_op(FLAG_M | FLAG_A, more); absorb(d, n); }
  void ad(const uint8_t* d, size_t n, bool more) { begin_op(FLAG_A, more); absorb(d, n); }
  void prf(uint8_t* d, size_t n, bool more) { begin_op(FLAG_I | FLAG_A | FLAG_C, more); squeeze(d, n); }
  void key(const uint8_t* d, size_t n, bool more) { begin_op(FLAG_A | FLAG_C, more); overwrite(d, n); }
};

struct Transcript {
  Strobe128 strobe;
  explicit Transcript(const char* label) : strobe((const uint8_t*)"Merlin v1.0", 11) {
    append_message("dom-sep", (const uint8_t*)label, strlen(label));
  }
  void append_message(const char* label, const uint8_t* msg, size_t n) {
    uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
    strobe.meta_ad((const uint8_t*)label, strlen(label), false);
    strobe.meta_ad(len, 4, true);
    strobe.ad(msg, n, false);
  }
  void append_message(const char* label, const char* msg) { append_message(label, (const uint8_t*)msg, strlen(msg)); }
  void append_u64(const char* label, uint64_t x) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(x >> (8 * i));
    append_message(label, b, 8);
  }
  void challenge_bytes(const char* label, uint8_t* dest, size_t n) {
    uint8_t len[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
    strobe.meta_ad((const uint8_t*)label, strlen(label), false);
    strobe.meta_ad(len, 4, true);
    strobe.prf(dest, n, false);
  }
  // src/transcript.rs:15-46
  void append_protocol_name(const char* name) { append_message("protocol-name", name); }
  void append_scalar(const char* label, const Fq& s) {
    uint8_t b[32];
    fq_to_bytes(s, b);
    append_message(label, b, 32);
  }
  void append_point(const char* label, const uint8_t p[32]) { append_message(label, p, 32); }
  Fq challenge_scalar(const char* label) {
    uint8_t buf[64];
    challenge_bytes(label, buf, 64);
    return fq_from_bytes_wide(buf);
  }
  std::vector<Fq> challenge_vector(const char* label, size_t len) {
    std::vector<Fq> v;
    for (size_t i = 0; i < len; i++) v.push_back(challenge_scalar(label));
    return v;
  }
  // src/transcript.rs:48-56  [Scalar]::append_to_transcript
  void append_scalars(const char* label, const std::vector<Fq>& v) {
    append_message(label, "begin_append_vector");
    for (const Fq& s : v) append_scalar(label, s);
    append_message(label, "end_append_vector");
  }
};

// src/random.rs:7-29 with the seeding seam: init_randomness is a caller-supplied scalar.
struct RandomTape {
  Transcript tape;
  RandomTape(const char* name, const Fq& init) : tape(name) { tape.append_scalar("init_randomness", init); }
  Fq random_scalar(const char* label) { return tape.challenge_scalar(label); }
  std::vector<Fq> random_vector(const char* label, size_t n) { return tape.challenge_vector(label, n); }
};

}  // namespace orc
