// spg — host-side Keccak-f[1600] sponge, SHAKE256 XOF (sha3 ^0.8.2 as used by
// src/commitments.rs:15-33) and the merlin ^3.0.0 transcript (STROBE-128 subset) behind
// src/transcript.rs / src/random.rs. Fiat-Shamir is inherently sequential and stays on the host.
#pragma once
#include <stdint.h>
#include <string.h>

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "keccak lanes assume a little-endian host");

namespace spg {

// permutations run on this thread (SPG_TRACE=2 prints the count per SNARK::prove)
inline uint64_t& keccak_count() {
  static thread_local uint64_t n = 0;
  return n;
}

struct KeccakState {
  uint64_t a[25];

  static inline uint64_t rol(uint64_t x, unsigned n) { return (x << n) | (x >> ((64 - n) & 63)); }

  // Keccak-f[1600] over lanes a[x + 5 y]; every loop has constant trip count and constant indices, so
  // the compiler keeps the 25 lanes in registers (~4x faster than the table-driven lane cycle)
  void permute() {
    static const uint64_t rc[24] = {
        0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
        0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
        0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
        0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
        0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
        0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
    // rho offset of lane x + 5 y
    static constexpr unsigned rho[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                         25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};
    keccak_count()++;
    uint64_t A[25], B[25], C[5], D[5];
    for (int i = 0; i < 25; i++) A[i] = a[i];
    for (int r = 0; r < 24; r++) {
#pragma GCC unroll 5
      for (int x = 0; x < 5; x++) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
#pragma GCC unroll 5
      for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rol(C[(x + 1) % 5], 1);
      // theta + rho + pi: B[y, 2x + 3y] = rol(A[x, y] ^ D[x], rho[x, y])
#pragma GCC unroll 25
      for (int i = 0; i < 25; i++) {
        const int x = i % 5, y = i / 5;
        B[y + 5 * ((2 * x + 3 * y) % 5)] = rol(A[i] ^ D[x], rho[i]);
      }
      // chi
#pragma GCC unroll 25
      for (int i = 0; i < 25; i++) {
        const int x = i % 5, y5 = i - x;
        A[i] = B[i] ^ (~B[y5 + (x + 1) % 5] & B[y5 + (x + 2) % 5]);
      }
      A[0] ^= rc[r];  // iota
    }
    for (int i = 0; i < 25; i++) a[i] = A[i];
  }
  uint8_t get(unsigned i) const { return (uint8_t)(a[i >> 3] >> (8 * (i & 7))); }
  void put(unsigned i, uint8_t v) {
    a[i >> 3] &= ~(0xffULL << (8 * (i & 7)));
    a[i >> 3] |= (uint64_t)v << (8 * (i & 7));
  }
  // lanes are little-endian byte strings (x86-64 / aarch64 hosts): byte i of the state is byte i of a[]
  void xor_byte(unsigned i, uint8_t v) { reinterpret_cast<uint8_t*>(a)[i] ^= v; }
};

class Shake256 {
 public:
  Shake256() : pos_(0), out_(false) { memset(s_.a, 0, sizeof(s_.a)); }
  void update(const void* data, size_t n) {
    const uint8_t* p = (const uint8_t*)data;
    for (size_t i = 0; i < n; i++) {
      s_.xor_byte(pos_, p[i]);
      if (++pos_ == kRate) { s_.permute(); pos_ = 0; }
    }
  }
  void read(void* dst, size_t n) {
    uint8_t* d = (uint8_t*)dst;
    if (!out_) {
      s_.xor_byte(pos_, 0x1f);
      s_.xor_byte(kRate - 1, 0x80);
      s_.permute();
      pos_ = 0;
      out_ = true;
    }
    for (size_t i = 0; i < n; i++) {
      if (pos_ == kRate) { s_.permute(); pos_ = 0; }
      d[i] = s_.get(pos_++);
    }
  }

 private:
  static const unsigned kRate = 136;
  KeccakState s_;
  unsigned pos_;
  bool out_;
};

// merlin::Transcript over STROBE-128 (rate 166): only the operations merlin uses.
class Merlin {
 public:
  explicit Merlin(const char* label) {
    memset(s_.a, 0, sizeof(s_.a));
    const uint8_t hdr[6] = {1, kR + 2, 1, 0, 1, 96};
    for (unsigned i = 0; i < 6; i++) s_.put(i, hdr[i]);
    const char* ver = "STROBEv1.0.2";
    for (unsigned i = 0; i < 12; i++) s_.put(6 + i, (uint8_t)ver[i]);
    s_.permute();
    pos_ = begin_ = flags_ = 0;
    op(kM | kA);
    absorb("Merlin v1.0", 11);
    message("dom-sep", label, strlen(label));
  }
  void message(const char* label, const void* msg, size_t n) {
    meta_len(label, (uint32_t)n);
    op(kA);
    absorb(msg, n);
  }
  void challenge(const char* label, void* dst, size_t n) {
    meta_len(label, (uint32_t)n);
    op(kI | kA | kC);
    uint8_t* d = (uint8_t*)dst;
    uint8_t* st = reinterpret_cast<uint8_t*>(s_.a);
    while (n) {  // runs of bytes up to the end of the rate: copied out, then zeroed (PRF output, STROBE's "I" flag)
      const size_t c = n < (size_t)(kR - pos_) ? n : (size_t)(kR - pos_);
      memcpy(d, st + pos_, c);
      memset(st + pos_, 0, c);
      pos_ = (uint8_t)(pos_ + c);
      d += c;
      n -= c;
      if (pos_ == kR) run_f();
    }
  }

 private:
  static const uint8_t kR = 166, kI = 1, kA = 2, kC = 4, kM = 16, kK = 32;
  KeccakState s_;
  uint8_t pos_, begin_, flags_;

  void run_f() {
    s_.xor_byte(pos_, begin_);
    s_.xor_byte(pos_ + 1, 0x04);
    s_.xor_byte(kR + 1, 0x80);
    s_.permute();
    pos_ = begin_ = 0;
  }
  void absorb(const void* data, size_t n) {
    const uint8_t* p = (const uint8_t*)data;
    uint8_t* st = reinterpret_cast<uint8_t*>(s_.a);
    while (n) {  // runs of bytes up to the end of the rate
      const size_t c = n < (size_t)(kR - pos_) ? n : (size_t)(kR - pos_);
      for (size_t i = 0; i < c; i++) st[pos_ + i] ^= p[i];
      pos_ = (uint8_t)(pos_ + c);
      p += c;
      n -= c;
      if (pos_ == kR) run_f();
    }
  }
  void op(uint8_t flags) {
    uint8_t b[2] = {begin_, flags};
    begin_ = pos_ + 1;
    flags_ = flags;
    absorb(b, 2);
    if ((flags & (kC | kK)) && pos_ != 0) run_f();
  }
  // meta-AD(label) followed by a continued meta-AD(le32 length)
  void meta_len(const char* label, uint32_t n) {
    op(kM | kA);
    absorb(label, strlen(label));
    uint8_t le[4] = {(uint8_t)n, (uint8_t)(n >> 8), (uint8_t)(n >> 16), (uint8_t)(n >> 24)};
    absorb(le, 4);
  }
};

}  // namespace spg
