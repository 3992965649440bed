// spg — host build of the product's field / curve / transcript code (the same headers the HIP kernels
// compile), exported for the CPU test suite so the arithmetic can be checked against the oracle
// without a GPU. Not part of the proving path.
#include <string.h>

#include <vector>

#include <atomic>
#include <memory>
#include <random>

#include "comm.hpp"
#include "curve.hpp"
#include "hcurve.hpp"
#include "hvec.hpp"
#include "hostmath.hpp"
#include "hpool.hpp"
#include "keccak.hpp"

using namespace spg;

static Fq ldq(const uint64_t* p) { Fq a; memcpy(a.l, p, 32); return a; }
static void stq(uint64_t* p, const Fq& a) { memcpy(p, a.l, 32); }

extern "C" {

// op: 0 add, 1 sub, 2 mul, 3 neg, 4 square, 5 invert, 6 from_mont, 7 to_mont, 8 mul_ps, 9 mul32
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
      case 8: r = fq_mul_ps(x, y); break;  // the device's product-scanning Montgomery product
      case 9: r = fq_mul32(x, y); break;   // the CIOS form
      default: r = fq_to_mont(x); break;
    }
    stq(out + 4 * i, r);
  }
}

// op: 0 add, 1 sub, 2 mul, 3 sqr, 4 inv, 5 canon, 6 mul (device product scanning), 7 sqr (device),
// 12 mul_k (k = b's low 18 bits); raw (not canonicalised) outputs: 8 addsub(+), 9 addsub(-), 10 add, 11 sub;
// inputs/outputs as 8 x u32 (loose allowed)
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
      case 6: r = fp_mul_ps(x, y); break;
      case 7: r = fp_sqr_ps(x); break;
      case 8: r = fp_addsub(x, y, false); break;
      case 9: r = fp_addsub(x, y, true); break;
      case 10: r = fp_add(x, y); break;
      case 11: r = fp_sub(x, y); break;
      case 12: r = fp_mul_k(x, y.l[0] & 0x3ffffu); break;
      default: r = x; break;
    }
    if (op < 8 || op > 11) r = fp_canon(r);
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

// A caller-owned merlin::Transcript behind spg_transcript_new_callbacks, in native code: what the Rust caller's
// `extern "C"` trampolines over `&mut Transcript` do (src/lib.rs:1022). The two
// callbacks have the spg_transcript_append_fn / spg_transcript_challenge_fn signatures and take the Merlin as `user`,
// so bench.py can time a prove in the drop-in mode with no Python on the transcript path.
void* spgh_merlin_new(const char* label) { return new Merlin(label); }
void spgh_merlin_free(void* t) { delete static_cast<Merlin*>(t); }
int spgh_merlin_append_cb(void* user, const char* label, const uint8_t* msg, size_t len) {
  static_cast<Merlin*>(user)->message(label, msg, len);
  return 0;
}
int spgh_merlin_challenge_cb(void* user, const char* label, uint8_t* out, size_t len) {
  static_cast<Merlin*>(user)->challenge(label, out, len);
  return 0;
}

// Host radix-2^51 curve (hcurve.hpp) against the device-form curve on the same inputs: for n uniform
// 64-byte strings, P_i = from_uniform_bytes; checks compress, decompress->compress, add, dbl, mixed add
// through batch-normalised Niels, and scalar multiplication by the 32-byte scalars k. Returns the
// number of mismatches.
int spgh_hcurve_check(const uint8_t* uni, const uint8_t* k, size_t n) {
  using namespace spg;
  int bad = 0;
  std::vector<Ext> P(n);
  std::vector<h::HExt> H(n);
  for (size_t i = 0; i < n; i++) {
    P[i] = ristretto_from_uniform_bytes(uni + 64 * i);
    H[i] = h::hext_from_dev(P[i]);
  }
  std::vector<h::HNiels> N;
  h::hext_batch_to_niels(H, N);
  for (size_t i = 0; i < n; i++) {
    uint8_t a[32], b[32];
    ext_compress(P[i], a);
    h::hext_compress(H[i], b);
    bad += memcmp(a, b, 32) != 0;
    h::HExt D;
    bad += !h::hext_decompress(a, D);
    h::hext_compress(D, b);
    bad += memcmp(a, b, 32) != 0;
    size_t j = (i + 1) % n;
    ext_compress(ext_add(P[i], P[j]), a);
    h::hext_compress(h::hext_add(H[i], H[j]), b);
    bad += memcmp(a, b, 32) != 0;
    h::hext_compress(h::hext_madd(H[i], N[j]), b);
    bad += memcmp(a, b, 32) != 0;
    ext_compress(ext_dbl(P[i]), a);
    h::hext_compress(h::hext_dbl(H[i]), b);
    bad += memcmp(a, b, 32) != 0;
    uint32_t kk[8];
    for (int w = 0; w < 8; w++)
      kk[w] = (uint32_t)k[32 * i + 4 * w] | ((uint32_t)k[32 * i + 4 * w + 1] << 8) |
              ((uint32_t)k[32 * i + 4 * w + 2] << 16) | ((uint32_t)k[32 * i + 4 * w + 3] << 24);
    ext_compress(ext_scalar_mul(P[i], kk), a);
    h::hext_compress(h::hext_scalar_mul(H[i], k + 32 * i), b);
    bad += memcmp(a, b, 32) != 0;
  }
  uint8_t bad_enc[32];
  memset(bad_enc, 0xff, 32);
  h::HExt X;
  bad += h::hext_decompress(bad_enc, X);  // non-canonical must be rejected
  return bad;
}

// The 8-lane IFMA sums (hvec.hpp) against the scalar additions: for m = 0 .. n entries, the sum of the first m Niels
// forms (mixed additions) and of the first m extended points (full additions), compared by encoding. Returns the
// number of mismatches, or -1 when this CPU has no AVX-512 IFMA (nothing to check).
int spgh_vec_check(const uint8_t* uni, size_t n) {
  using namespace spg;
  if (!h::ifma_on()) return -1;
  int bad = 0;
  std::vector<h::HExt> H(n);
  for (size_t i = 0; i < n; i++) H[i] = h::hext_from_dev(ristretto_from_uniform_bytes(uni + 64 * i));
  std::vector<h::HNiels> N;
  h::hext_batch_to_niels(H, N);
  std::vector<const h::HNiels*> ptr(n);
  for (size_t i = 0; i < n; i++) ptr[i] = &N[i];
  h::HExt s1 = h::hext_identity(), s2 = h::hext_identity();
  for (size_t m = 0; m <= n; m++) {
    if (m) {
      s1 = h::hext_madd(s1, N[m - 1]);
      s2 = h::hext_add(s2, H[m - 1]);
    }
    uint8_t a[32], b[32];
    h::hext_compress(s1, a);
    h::hext_compress(h::niels_sum8(ptr.data(), m), b);
    bad += memcmp(a, b, 32) != 0;
    h::hext_compress(s2, a);
    h::hext_compress(h::ext_sum8(H.data(), m), b);
    bad += memcmp(a, b, 32) != 0;
  }
  return bad;
}

// The batched encoding of doubles (hcurve.hpp, hext_double_and_compress_batch) against the lone encoding of 2 Q, over
// n hash-to-group points, each also moved by the 2- and 4-torsion points, and the identity and the torsion points
// themselves (zero e g f h). Returns the mismatches (0), or -1 for n == 0.
int spgh_dbl_compress_check(const uint8_t* uni, size_t n) {
  using namespace spg;
  if (!n) return -1;
  const h::HExt T2{h::fe_zero(), h::fe_neg(h::fe_one()), h::fe_one(), h::fe_zero()};
  const h::HExt T4{h::K().sqrt_m1, h::fe_zero(), h::fe_one(), h::fe_zero()};
  std::vector<h::HExt> Q;
  for (size_t i = 0; i < n; i++) {
    const h::HExt P = h::hext_from_dev(ristretto_from_uniform_bytes(uni + 64 * i));
    Q.push_back(P);
    Q.push_back(h::hext_add(P, T2));
    Q.push_back(h::hext_add(P, T4));
    if (i == n / 2) {
      Q.push_back(h::hext_identity());
      Q.push_back(T2);
      Q.push_back(T4);
    }
  }
  std::vector<uint8_t> got(32 * Q.size());
  h::hext_double_and_compress_batch(Q.data(), Q.size(), (uint8_t(*)[32])got.data());
  std::vector<uint8_t> got8(32 * Q.size());
  const bool vec = h::ifma_on();
  if (vec) h::double_and_compress_batch8(Q.data(), Q.size(), (uint8_t(*)[32])got8.data());
  int bad = 0;
  for (size_t i = 0; i < Q.size(); i++) {
    uint8_t want[32];
    h::hext_compress(h::hext_dbl(Q[i]), want);
    bad += memcmp(want, got.data() + 32 * i, 32) != 0;
    if (vec) bad += memcmp(want, got8.data() + 32 * i, 32) != 0;
  }
  // every length 1 .. 20 through the 8-lane form (partial groups)
  for (size_t m = 1; vec && m <= 20 && m <= Q.size(); m++) {
    h::double_and_compress_batch8(Q.data(), m, (uint8_t(*)[32])got8.data());
    for (size_t i = 0; i < m; i++) bad += memcmp(got.data() + 32 * i, got8.data() + 32 * i, 32) != 0;
  }
  return bad;
}

// The cross-rank exchange of every sharded call (comm.hpp: api.hip's comm_sum_fq, which Prover::sum_ranks and the
// SPARK / multi_evaluate shards use): gather every rank's status and n partial scalars through the caller's
// allgather and sum them mod q. Returns the transport's error (-1), else the first non-zero status of any rank
// (so a failing rank fails every rank alike), else 0 with out = the sums.
int spgh_comm_sum(spg_allgather_fn fn, void* user, int nranks, int status, const uint64_t* mine, size_t n,
                  uint64_t* out) {
  std::vector<Fq> v(n);
  for (size_t i = 0; i < n; i++) v[i] = ldq(mine + 4 * i);
  std::vector<uint8_t> all;
  int64_t first = 0;
  if (allgather_with_status(fn, user, nranks, status, v.data(), n * sizeof(Fq), all, &first) != 0) return -1;
  if (first) return (int)first;
  sum_over_ranks(all.data(), nranks, n, v.data());
  for (size_t i = 0; i < n; i++) stq(out + 4 * i, v[i]);
  return 0;
}

// the prover's host scalar helpers (hostmath.hpp): UniPoly::from_evals of degree 3 -> coeffs[4] and evaluate(r)
void spgh_uni_from_evals3(const uint64_t* evals, const uint64_t* r, uint64_t* coeffs, uint64_t* at_r) {
  Fq e[4];
  for (int i = 0; i < 4; i++) e[i] = ldq(evals + 4 * i);
  FqV c = uni_from_evals3(e);
  for (int i = 0; i < 4; i++) stq(coeffs + 4 * i, c[i]);
  stq(at_r, uni_eval(c, ldq(r)));
}
// DensePolynomial::evaluate of n host scalars at r (ell scalars) and EqPolynomial::evals(r) (2^ell scalars)
void spgh_dense_eval(const uint64_t* Z, size_t n, const uint64_t* r, size_t ell, uint64_t* out, uint64_t* chis) {
  FqV z(n), rv(ell);
  for (size_t i = 0; i < n; i++) z[i] = ldq(Z + 4 * i);
  for (size_t i = 0; i < ell; i++) rv[i] = ldq(r + 4 * i);
  stq(out, dense_eval_host(z, rv));
  FqV e = eq_evals_host(rv);
  for (size_t i = 0; i < e.size(); i++) stq(chis + 4 * i, e[i]);
}

// The host pool (hpool.hpp) under stress: `bursts` parallel_for calls of random size 1..max_n on a fresh
// pool of `workers` threads whose workers sleep `delay_us` between their generation and function loads
// and whose caller sleeps `delay_us` between publishing a burst's function/count and opening it (the two
// sides of the stale-snapshot race window). Every task bumps its own counter; right after each call
// returns, every counter must be exactly 1 and no task may still be running. Returns the number of
// violations (0 = pass).
long spgh_pool_stress(int workers, int bursts, int max_n, int delay_us, unsigned seed) {
  spg::Pool pool(workers, delay_us, delay_us);
  std::mt19937 rng(seed);
  std::atomic<long> bad{0};
  std::atomic<int> running{0};
  for (int b = 0; b < bursts; b++) {
    const int n = 1 + (int)(rng() % (unsigned)max_n);
    std::unique_ptr<std::atomic<int>[]> cnt(new std::atomic<int>[n]);
    for (int i = 0; i < n; i++) cnt[i].store(0);
    const int tag = b;
    pool.parallel_for(n, [&, tag](int i) {
      running.fetch_add(1);
      if (i < 0 || i >= n || tag != b) bad.fetch_add(1);
      else cnt[i].fetch_add(1);
      if ((i & 7) == 0) std::this_thread::yield();
      running.fetch_sub(1);
    });
    if (running.load() != 0) bad.fetch_add(1);
    for (int i = 0; i < n; i++) bad.fetch_add(cnt[i].load() != 1);
  }
  return bad.load();
}

}  // extern "C"

#ifdef SPGH_MAIN
// TSan driver (make sanitize -> lib/spg_pool_tsan): the pool stress test with its race-window delays, then the
// cross-rank exchange (comm.hpp) over an in-process allgather between threads, one thread per rank.
#include <stdio.h>

#include <condition_variable>
#include <mutex>
#include <thread>

namespace {
struct Barrier {
  std::mutex mu;
  std::condition_variable cv;
  int n, waiting = 0;
  unsigned gen = 0;
  explicit Barrier(int k) : n(k) {}
  void arrive_and_wait() {
    std::unique_lock<std::mutex> lk(mu);
    const unsigned g = gen;
    if (++waiting == n) {
      waiting = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};
struct ThreadComm {  // allgather between `n` threads through one shared buffer and a barrier per phase
  int n;
  std::vector<uint8_t> buf;
  Barrier bar;
  explicit ThreadComm(int nr) : n(nr), bar(nr) {}
};
struct RankUser {
  ThreadComm* c;
  int rank;
};
int thread_allgather(void* user, const void* send, size_t bytes, void* recv) {
  RankUser* u = (RankUser*)user;
  ThreadComm* c = u->c;
  if (u->rank == 0) c->buf.assign(bytes * c->n, 0);
  c->bar.arrive_and_wait();
  memcpy(c->buf.data() + bytes * u->rank, send, bytes);
  c->bar.arrive_and_wait();
  memcpy(recv, c->buf.data(), bytes * c->n);
  c->bar.arrive_and_wait();
  return 0;
}
}  // namespace

int main() {
  long bad = spgh_pool_stress(7, 300, 64, 0, 1) + spgh_pool_stress(7, 100, 16, 20, 2) + spgh_pool_stress(3, 200, 9, 5, 3);
  const int n = 4;
  ThreadComm comm(n);
  std::vector<std::thread> ts;
  std::vector<int> rcs(n), fails(n);
  std::vector<std::vector<uint64_t>> outs(n, std::vector<uint64_t>(12));
  for (int r = 0; r < n; r++)
    ts.emplace_back([&, r] {
      RankUser u{&comm, r};
      std::vector<uint64_t> mine(12);
      for (int i = 0; i < 12; i++) mine[i] = (uint64_t)(r + 1) * (i % 4 == 3 ? 1 : 1000003);
      rcs[r] = spgh_comm_sum(thread_allgather, &u, n, 0, mine.data(), 3, outs[r].data());
      std::vector<uint64_t> junk(12);
      fails[r] = spgh_comm_sum(thread_allgather, &u, n, r == 2 ? -3 : 0, mine.data(), 3, junk.data());
    });
  for (auto& t : ts) t.join();
  for (int r = 0; r < n; r++) {
    bad += rcs[r] != 0 || fails[r] != -3;
    bad += outs[r] != outs[0];
  }
  printf("pool stress + thread exchange: %ld violations\n", bad);
  return bad ? 1 : 0;
}
#endif
