// spg — host-side pieces of the prover: Fiat-Shamir transcript, bincode writer, and the O(1)-size
// commitments of the sigma protocols (<= 5 fixed generators), which stay on the host because they
// sit between sequential transcript challenges. Every commitment whose size depends on the input goes
// through the GPU MSM (msm.hip).
//
//   ProofTranscript        src/transcript.rs:5-63   (merlin, keccak.hpp)
//   RandomTape (seedable)  src/random.rs:7-29
//   Scalar byte codecs     src/scalar/ristretto255.rs:391-466
#pragma once
#include <string.h>

#include <functional>
#include <atomic>
#include <map>
#include <memory>
#include <vector>

#include "curve.hpp"
#include "hcurve.hpp"
#include "hpool.hpp"
#include "keccak.hpp"

namespace spg {

typedef std::vector<Fq> FqV;

struct Pt {
  uint8_t b[32];
  bool operator==(const Pt& o) const { return memcmp(b, o.b, 32) == 0; }
};

inline void fq_le_bytes(const Fq& a, uint8_t out[32]) {
  Fq c = fq_from_mont(a);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(c.l[i] >> (8 * k));
}
// Scalar::from_bytes_wide: d0 * R2 + d1 * R3 (ristretto255.rs:449-466)
inline Fq fq_from_wide(const uint8_t b[64]) {
  Fq d0, d1;
  for (int i = 0; i < 8; i++) {
    d0.l[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
              ((uint32_t)b[4 * i + 3] << 24);
    d1.l[i] = (uint32_t)b[32 + 4 * i] | ((uint32_t)b[33 + 4 * i] << 8) | ((uint32_t)b[34 + 4 * i] << 16) |
              ((uint32_t)b[35 + 4 * i] << 24);
  }
  return fq_add(fq_mul(d0, fq_r2()), fq_mul(d1, fq_r3()));
}
inline Fq fq_u64(uint64_t x) { return fq_from_u64(x); }

struct Writer {
  std::vector<uint8_t> out;
  void u64(uint64_t x) {
    for (int i = 0; i < 8; i++) out.push_back((uint8_t)(x >> (8 * i)));
  }
  void fq(const Fq& a) {  // serde of Scalar([u64;4]): the Montgomery limbs
    for (int i = 0; i < 8; i++)
      for (int k = 0; k < 4; k++) out.push_back((uint8_t)(a.l[i] >> (8 * k)));
  }
  void pt(const Pt& p) { out.insert(out.end(), p.b, p.b + 32); }
  void fqs(const FqV& v) {
    u64(v.size());
    for (auto& a : v) fq(a);
  }
  void pts(const std::vector<Pt>& v) {
    u64(v.size());
    for (auto& p : v) pt(p);
  }
};

struct Tr {
  Merlin m;
  explicit Tr(const char* label) : m(label) {}
  void msg(const char* label, const char* s) { m.message(label, s, strlen(s)); }
  void protocol(const char* name) { msg("protocol-name", name); }
  void scalar(const char* label, const Fq& a) {
    uint8_t b[32];
    fq_le_bytes(a, b);
    m.message(label, b, 32);
  }
  void point(const char* label, const Pt& p) { m.message(label, p.b, 32); }
  void u64(const char* label, uint64_t x) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(x >> (8 * i));
    m.message(label, b, 8);
  }
  Fq challenge(const char* label) {
    uint8_t b[64];
    m.challenge(label, b, 64);
    return fq_from_wide(b);
  }
  FqV challenges(const char* label, size_t n) {
    FqV v;
    for (size_t i = 0; i < n; i++) v.push_back(challenge(label));
    return v;
  }
  void scalars(const char* label, const FqV& v) {  // [Scalar]::append_to_transcript
    msg(label, "begin_append_vector");
    for (auto& a : v) scalar(label, a);
    msg(label, "end_append_vector");
  }
};

struct Tape {
  Tr t;
  Tape(const char* name, const Fq& init) : t(name) { t.scalar("init_randomness", init); }
  Fq scalar(const char* label) { return t.challenge(label); }
  FqV vec(const char* label, size_t n) { return t.challenges(label, n); }
};

inline Pt compress(const h::HExt& p) {
  Pt c;
  h::hext_compress(p, c.b);
  return c;
}

// Fixed-base host scalar multiplication: tab[w][j] = j * 2^(8w) * P (affine Niels), 32 windows of 8
// bits, so k * P costs at most 32 mixed additions.
struct FixedBase {
  std::vector<h::HNiels> tab;  // 32 * 256 (entry 0 of each window unused)
  void build(const h::HExt& P) {
    std::vector<h::HExt> ext(32 * 256, h::hext_identity());
    h::HExt base = P;
    for (int w = 0; w < 32; w++) {
      ext[w * 256 + 1] = base;
      for (int j = 2; j < 256; j++) ext[w * 256 + j] = h::hext_add(ext[w * 256 + j - 1], base);
      for (int k = 0; k < 8; k++) base = h::hext_dbl(base);
    }
    h::hext_batch_to_niels(ext, tab);
  }
  // acc += k * P   (k Montgomery)
  void mul_add(h::HExt& acc, const Fq& k) const { mul_add_windows(acc, k, 0, 32); }
  // acc += (sum over byte windows w0 <= w < w1 of k_w 2^(8w)) * P: one share of k * P
  void mul_add_windows(h::HExt& acc, const Fq& k, int w0, int w1) const {
    uint8_t b[32];
    fq_le_bytes(k, b);
    for (int w = w0; w < w1; w++)
      if (b[w]) acc = h::hext_madd(acc, tab[w * 256 + b[w]]);
  }
};

// Host view of a generator set for the sigma protocols: fixed-base tables for the few indices used.
struct HostGens {
  std::map<size_t, FixedBase> fb;
  std::vector<uint8_t> comp;  // compressed stream points (index -> 32 bytes); decompressed on first use
  void init(const uint8_t* compressed, size_t count) { comp.assign(compressed, compressed + 32 * count); }
  h::HExt point(size_t idx) const {
    h::HExt P;
    h::hext_decompress(comp.data() + 32 * idx, P);
    return P;
  }
  const FixedBase& get(size_t idx) {
    auto it = fb.find(idx);
    if (it != fb.end()) return it->second;
    FixedBase& f = fb[idx];
    f.build(point(idx));
    return f;
  }
  // sum_i s_i * P_{idx_i}
  h::HExt msm(const std::vector<size_t>& idx, const FqV& s) {
    h::HExt acc = h::hext_identity();
    for (size_t i = 0; i < idx.size(); i++) get(idx[i]).mul_add(acc, s[i]);
    return acc;
  }
  // several independent commitments (index list, scalars) at once on the host pool, encoded. Every
  // scalar multiple is split into kShares window ranges, so even a 2-term commitment keeps several cores
  // busy: the pool's workers spin between the bursts of a sumcheck round, so a burst costs ~1 us to start.
  std::vector<Pt> commit_many(const std::vector<std::pair<std::vector<size_t>, FqV>>& jobs) {
    std::vector<Pt> out(jobs.size());
    run_many(jobs, [&](size_t j, const h::HExt& sum) { out[j] = compress(sum); });
    return out;
  }
  // the same sums left uncompressed (terms a caller adds to a device result before encoding it)
  std::vector<h::HExt> sum_many(const std::vector<std::pair<std::vector<size_t>, FqV>>& jobs) {
    std::vector<h::HExt> out(jobs.size());
    run_many(jobs, [&](size_t j, const h::HExt& sum) { out[j] = sum; });
    return out;
  }

 private:
  // one pool burst over every (job, term, window share); the last share of a job to finish (per-job
  // countdown) adds the job's shares and hands the sum to done(job, sum)
  template <class Done>
  void run_many(const std::vector<std::pair<std::vector<size_t>, FqV>>& jobs, const Done& done) {
    static const int kShares = 4;  // 8 byte-windows (<= 8 mixed additions) per task
    std::vector<std::pair<size_t, size_t>> terms;  // (job, term)
    for (size_t j = 0; j < jobs.size(); j++) {
      for (size_t i = 0; i < jobs[j].first.size(); i++) {
        get(jobs[j].first[i]);  // build tables on this thread (map insertion is not thread-safe)
        terms.push_back({j, i});
      }
    }
    const int ntask = (int)terms.size() * kShares;
    std::vector<h::HExt> part(ntask);
    std::vector<int> first(jobs.size() + 1, 0);
    for (size_t k = 0; k < terms.size(); k++) first[terms[k].first + 1] = (int)(k + 1) * kShares;
    for (size_t j = 1; j <= jobs.size(); j++) first[j] = std::max(first[j], first[j - 1]);
    std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[jobs.size()]);
    for (size_t j = 0; j < jobs.size(); j++) {
      left[j].store(first[j + 1] - first[j]);
      if (first[j + 1] == first[j]) done(j, h::hext_identity());
    }
    pool().parallel_for(ntask, [&](int k) {
      const auto& tm = terms[k / kShares];
      const auto& jb = jobs[tm.first];
      const int w0 = (k % kShares) * (32 / kShares);
      h::HExt acc = h::hext_identity();
      fb.find(jb.first[tm.second])->second.mul_add_windows(acc, jb.second[tm.second], w0, w0 + 32 / kShares);
      part[k] = acc;
      if (left[tm.first].fetch_sub(1, std::memory_order_acq_rel) == 1) {
        h::HExt sum = part[first[tm.first]];
        for (int i = first[tm.first] + 1; i < first[tm.first + 1]; i++) sum = h::hext_add(sum, part[i]);
        done(tm.first, sum);
      }
    });
  }
};

// variable-base scalar multiplication (k Montgomery), used once per ProductProof (gens_X)
inline h::HExt var_mul(const h::HExt& P, const Fq& k) {
  uint8_t b[32];
  fq_le_bytes(k, b);
  return h::hext_scalar_mul(P, b);
}

}  // namespace spg
