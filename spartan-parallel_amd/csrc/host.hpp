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

#include <algorithm>
#include <functional>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/spg.h"
#include "curve.hpp"
#include "hcurve.hpp"
#include "hvec.hpp"
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

// The caller's transcript behind spg_transcript_new_callbacks: every append_message / challenge_bytes of the
// prover is forwarded, so the caller's merlin::Transcript stays the one Fiat-Shamir state (SNARK::prove's
// `transcript: &mut Transcript`, src/lib.rs:1022). The first failing callback is kept in `failed`; later
// operations are skipped (challenges read as zero) and the entry point returns SPG_E_CALLBACK.
struct TrCallbacks {
  spg_transcript_append_fn append = nullptr;
  spg_transcript_challenge_fn challenge = nullptr;
  void* user = nullptr;
  int failed = 0;
};

struct Tr {
  Merlin m;
  std::shared_ptr<TrCallbacks> cb;  // null: the library's own merlin transcript
  explicit Tr(const char* label) : m(label) {}
  // the two merlin operations every ProofTranscript method reduces to (src/transcript.rs:13-46)
  void message(const char* label, const void* data, size_t n) {
    if (!cb) return m.message(label, data, n);
    if (cb->failed) return;
    const int rc = cb->append(cb->user, label, (const uint8_t*)data, n);
    if (rc) cb->failed = rc;
  }
  void challenge_bytes(const char* label, void* dst, size_t n) {
    if (!cb) return m.challenge(label, dst, n);
    if (!cb->failed) {
      const int rc = cb->challenge(cb->user, label, (uint8_t*)dst, n);
      if (rc) cb->failed = rc;
    }
    if (cb->failed) memset(dst, 0, n);
  }
  int failed() const { return cb ? cb->failed : 0; }
  void msg(const char* label, const char* s) { message(label, s, strlen(s)); }
  void protocol(const char* name) { msg("protocol-name", name); }
  void scalar(const char* label, const Fq& a) {
    uint8_t b[32];
    fq_le_bytes(a, b);
    message(label, b, 32);
  }
  void point(const char* label, const Pt& p) { message(label, p.b, 32); }
  void u64(const char* label, uint64_t x) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(x >> (8 * i));
    message(label, b, 8);
  }
  Fq challenge(const char* label) {
    uint8_t b[64];
    challenge_bytes(label, b, 64);
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
// encodings of B device points that are halves (a comb MSM with halved scalars: encode(2 P') = encode(P)), as the
// doubles' batched encodings (hext_double_and_compress_batch), on the pool in chunks of >= 64 points (one inversion each)
inline void encode_halved_host(const Ext* d, size_t B, Pt* out) {
  static_assert(sizeof(Pt) == 32, "Pt is the 32-byte encoding");
  // (batches under 384 points stay on the calling thread: a 128-point batch took 84-99 us through a pool burst inside
  // config 4's R1CSProof, against 34 us single-threaded in scripts/micro/enc_batch.cpp)
  const int C = B < 384 ? 1 : (int)std::max<size_t>(1, std::min<size_t>(B / 64, (size_t)pool().size() + 1));
  auto enc = [&](int c) {
    const size_t lo = B * c / C, hi = B * (c + 1) / C;
    thread_local std::vector<h::HExt> P;
    P.resize(hi - lo);
    for (size_t i = lo; i < hi; i++) P[i - lo] = h::hext_from_dev(d[i]);
    if (h::ifma_on())  // 8 points per step on AVX-512 IFMA (~2.5x the scalar batch)
      h::double_and_compress_batch8(P.data(), hi - lo, reinterpret_cast<uint8_t(*)[32]>(out + lo));
    else
      h::hext_double_and_compress_batch(P.data(), hi - lo, reinterpret_cast<uint8_t(*)[32]>(out + lo));
  };
  if (C == 1)
    enc(0);
  else
    pool().parallel_for(C, enc);
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
  // each HostGens guards its own table map (contexts on several threads may share a generator set; a table, once
  // built, never moves: std::map nodes are stable). Per set, not process-wide: contexts proving with
  // different generator sets no longer wait on each other's table builds (11-24 ms each) and lookups
  std::shared_ptr<std::mutex> mu_ = std::make_shared<std::mutex>();
  std::mutex& table_mu() { return *mu_; }
  const FixedBase& get(size_t idx) {
    std::lock_guard<std::mutex> lk(table_mu());
    return get_locked(idx);
  }
  const FixedBase& get_locked(size_t idx) {
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
  // several independent commitments (index list, scalars) at once on the host pool, encoded
  std::vector<Pt> commit_many(const std::vector<std::pair<std::vector<size_t>, FqV>>& jobs) {
    std::vector<Pt> out(jobs.size());
    run(jobs, nullptr, [&](size_t j, const h::HExt& sum) { out[j] = compress(sum); });
    return out;
  }
  // the same with a precomputed point extra[j] added to commitment j before it is encoded
  std::vector<Pt> commit_many_plus(const std::vector<std::pair<std::vector<size_t>, FqV>>& jobs, const h::HExt* extra) {
    std::vector<Pt> out(jobs.size());
    run(jobs, extra, [&](size_t j, const h::HExt& sum) { out[j] = compress(sum); });
    return out;
  }
  // the same sums left uncompressed (terms a caller adds to a device result before encoding it)
  std::vector<h::HExt> sum_many(const std::vector<std::pair<std::vector<size_t>, FqV>>& jobs) {
    std::vector<h::HExt> out(jobs.size());
    run(jobs, nullptr, [&](size_t j, const h::HExt& sum) { out[j] = sum; });
    return out;
  }

  // One pool burst over every (job, term, byte window) unit: the units are cut into at most one contiguous
  // slice per pool thread (>= 8 windows each); a slice adds its units per job, and the last slice of a job to
  // finish (per-job countdown) adds that job's slice sums (+ extra[j]) and hands them to done(job, sum), which
  // may encode on that thread. A sumcheck round's few commitments thus keep every core busy for ~ (terms x 32
  // / threads) mixed additions instead of queueing whole scalar multiples.
  template <class Done>
  void run(const std::vector<std::pair<std::vector<size_t>, FqV>>& jobs, const h::HExt* extra, const Done& done) {
    const size_t J = jobs.size();
    struct Term {
      const FixedBase* fb;
      uint8_t b[32];
    };
    std::vector<Term> terms;
    std::vector<size_t> tfirst(J + 1, 0);  // terms of job j: [tfirst[j], tfirst[j + 1])
    {
      std::lock_guard<std::mutex> lk(table_mu());  // tables are built on this thread, under the lock
      for (size_t j = 0; j < J; j++) {
        for (size_t i = 0; i < jobs[j].first.size(); i++) {
          Term tm;
          tm.fb = &get_locked(jobs[j].first[i]);
          fq_le_bytes(jobs[j].second[i], tm.b);
          terms.push_back(tm);
        }
        tfirst[j + 1] = terms.size();
      }
    }
    const size_t U = 32 * terms.size();
    const size_t threads = (size_t)pool().size() + 1;
    // >= 64 units per slice: with the IFMA sums a slice's run is cheap, and fewer slices mean less burst hand-off
    // (2-rep A/B, SNARK median ms: 8: 16.91 / 16.80, 32: 16.79 / 16.26, 64: 16.32 / 16.38)
    static const size_t min_slice = getenv("SPG_SLICE_MIN") ? (size_t)atol(getenv("SPG_SLICE_MIN")) : 64;
    // several small jobs (a DotProductProof's Cy and beta: 96 units) get a slice each, so their encodings (~2.4 us
    // inverse square roots) run side by side instead of one after another on the calling thread (SPG_ENC_SPLIT=0: off)
    static const bool enc_split = !getenv("SPG_ENC_SPLIT") || atoi(getenv("SPG_ENC_SPLIT")) != 0;
    size_t S = std::max<size_t>(1, std::min(threads, U / min_slice));
    const bool per_job = enc_split && J > S && J <= threads;
    if (per_job) S = J;  // slice s = job s
    auto slice_lo = [&](size_t s) { return per_job ? 32 * tfirst[s] : U * s / S; };
    // slices touching job j: [sfirst[j], slast[j]]
    std::vector<size_t> sfirst(J), slast(J);
    std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[J]);
    for (size_t j = 0; j < J; j++) {
      if (tfirst[j + 1] == tfirst[j]) {  // no terms: the extra point alone
        done(j, extra ? extra[j] : h::hext_identity());
        left[j].store(0);
        continue;
      }
      const size_t u0 = 32 * tfirst[j], u1 = 32 * tfirst[j + 1] - 1;
      size_t s0 = 0;
      while (s0 + 1 < S && slice_lo(s0 + 1) <= u0) s0++;
      size_t s1 = s0;
      while (s1 + 1 < S && slice_lo(s1 + 1) <= u1) s1++;
      sfirst[j] = s0;
      slast[j] = s1;
      left[j].store((int)(s1 - s0 + 1));
    }
    std::vector<h::HExt> part(S * std::max<size_t>(J, 1));
    // the job of unit u
    std::vector<size_t> tjob(terms.size());
    for (size_t j = 0; j < J; j++)
      for (size_t k = tfirst[j]; k < tfirst[j + 1]; k++) tjob[k] = j;
    // The table entry of a unit depends only on the scalar byte, not on the running sum, so the entry kPf units
    // ahead is prefetched while this one is added: a small DotProductProofLog's rounds read ~1000 random entries of
    // ~1 MB tables per generator, which mostly miss the caches (host-path proofs 1.63 -> 0.98 ms per SNARK::prove in
    // situ, session r03zm; a standalone micro with warm tables showed no gain). SPG_HOST_PREFETCH=0: off.
    static const size_t kPf = getenv("SPG_HOST_PREFETCH") ? (size_t)atol(getenv("SPG_HOST_PREFETCH")) : 3;
    // with AVX-512 IFMA a job's run of at least kVecMin units goes through the 8-lane sums (hvec.hpp): the entries of
    // its nonzero bytes, 8 accumulators, one reduction (SPG_VEC_MIN: the threshold; 0 = never)
    static const size_t kVecMin = getenv("SPG_VEC_MIN") ? (size_t)atol(getenv("SPG_VEC_MIN")) : 16;
    const bool vec = kVecMin && h::ifma_on();
    pool().parallel_for((int)S, [&](int si) {
      const size_t s = (size_t)si, u0 = slice_lo(s), u1 = slice_lo(s + 1);
      size_t u = u0;
      while (u < u1) {
        const size_t j = tjob[u / 32], ue = std::min(u1, 32 * tfirst[j + 1]);
        h::HExt acc = h::hext_identity();
        if (vec && ue - u >= kVecMin) {
          constexpr size_t kCap = 256;
          const h::HNiels* ent[kCap];
          size_t m = 0;
          bool any = false;
          for (; u < ue; u++) {
            const Term& tm = terms[u / 32];
            const int w = (int)(u % 32);
            if (!tm.b[w]) continue;
            ent[m] = &tm.fb->tab[w * 256 + tm.b[w]];
            if (m < 16) __builtin_prefetch(ent[m]);
            if (++m == kCap) {
              const h::HExt part = h::niels_sum8(ent, m);
              acc = any ? h::hext_add(acc, part) : part;
              any = true;
              m = 0;
            }
          }
          if (m) {
            const h::HExt part = h::niels_sum8(ent, m);
            acc = any ? h::hext_add(acc, part) : part;
          }
        }
        for (; u < ue; u++) {
          if (kPf && u + kPf < u1) {
            const Term& tp = terms[(u + kPf) / 32];
            const char* e = (const char*)&tp.fb->tab[((u + kPf) % 32) * 256 + tp.b[(u + kPf) % 32]];
            __builtin_prefetch(e);
            __builtin_prefetch(e + sizeof(h::HNiels) - 1);
          }
          const Term& tm = terms[u / 32];
          const int w = (int)(u % 32);
          if (tm.b[w]) acc = h::hext_madd(acc, tm.fb->tab[w * 256 + tm.b[w]]);
        }
        part[s * J + j] = acc;
        if (left[j].fetch_sub(1, std::memory_order_acq_rel) == 1) {
          h::HExt sum = part[sfirst[j] * J + j];
          for (size_t q = sfirst[j] + 1; q <= slast[j]; q++) sum = h::hext_add(sum, part[q * J + j]);
          if (extra) sum = h::hext_add(sum, extra[j]);
          done(j, sum);
        }
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
