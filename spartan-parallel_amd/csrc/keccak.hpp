// spg — host-side Keccak-f[1600] sponge, SHAKE256 XOF (sha3 ^0.8.2 as used by
// src/commitments.rs:15-33) and the merlin ^3.0.0 transcript (STROBE-128 subset) behind
// src/transcript.rs / src/random.rs. Fiat-Shamir is inherently sequential and stays on the host.
#pragma once
#include <stdint.h>
#include <string.h>

namespace spg {

struct KeccakState {
  uint64_t a[25];

  static uint64_t rol(uint64_t x, unsigned n) { return n ? (x << n) | (x >> (64 - n)) : x; }

  void permute() {
    static const uint64_t rc[24] = {
        0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
        0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
        0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
        0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
        0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
        0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
    // pi lane cycle and the rho offsets along it (starting from lane 1)
    static const int piln[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
    static const unsigned rotc[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
    for (int r = 0; r < 24; r++) {
      uint64_t bc[5];
      for (int i = 0; i < 5; i++) bc[i] = a[i] ^ a[i + 5] ^ a[i + 10] ^ a[i + 15] ^ a[i + 20];
      for (int i = 0; i < 5; i++) {
        uint64_t t = bc[(i + 4) % 5] ^ rol(bc[(i + 1) % 5], 1);
        for (int j = 0; j < 25; j += 5) a[j + i] ^= t;
      }
      uint64_t t = a[1];
      for (int i = 0; i < 24; i++) {
        int j = piln[i];
        uint64_t tmp = a[j];
        a[j] = rol(t, rotc[i]);
        t = tmp;
      }
      for (int j = 0; j < 25; j += 5) {
        uint64_t b0 = a[j], b1 = a[j + 1], b2 = a[j + 2], b3 = a[j + 3], b4 = a[j + 4];
        a[j] = b0 ^ (~b1 & b2);
        a[j + 1] = b1 ^ (~b2 & b3);
        a[j + 2] = b2 ^ (~b3 & b4);
        a[j + 3] = b3 ^ (~b4 & b0);
        a[j + 4] = b4 ^ (~b0 & b1);
      }
      a[0] ^= rc[r];
    }
  }
  uint8_t get(unsigned i) const { return (uint8_t)(a[i >> 3] >> (8 * (i & 7))); }
  void put(unsigned i, uint8_t v) {
    a[i >> 3] &= ~(0xffULL << (8 * (i & 7)));
    a[i >> 3] |= (uint64_t)v << (8 * (i & 7));
  }
  void xor_byte(unsigned i, uint8_t v) { a[i >> 3] ^= (uint64_t)v << (8 * (i & 7)); }
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
    for (size_t i = 0; i < n; i++) {
      d[i] = s_.get(pos_);
      s_.put(pos_, 0);
      if (++pos_ == kR) run_f();
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
    for (size_t i = 0; i < n; i++) {
      s_.xor_byte(pos_, p[i]);
      if (++pos_ == kR) run_f();
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
