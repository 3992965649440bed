// spg — sigma protocols (host) and DotProductProofLog / Bulletproofs with GPU MSMs.
//
// Bulletproofs rewrite (src/nizk/bullet.rs:32-132): the prover folds G_L[i] = u^-1 G_L[i] + u G_R[i] every
// round. After k rounds G^(k)[i] = sum_{j = i mod n_k} cw[j] * G_j over the ORIGINAL generators, with
// per-generator weights cw that are products of u / u^-1. So every L, R (and the final g_hat) is a
// fixed-base MSM over the generator table already resident in HBM (msm.hip); no curve point is ever
// folded and the group elements produced are identical to the reference's.
#include <atomic>
#include <chrono>
#include <functional>
#include <memory>

#include "hostpoly.hpp"

#include "proto.hpp"

namespace spg {

static Fq dot(const FqV& a, const FqV& b, size_t ao, size_t bo, size_t n) {
  Fq s = fq_zero();
  for (size_t i = 0; i < n; i++) s = fq_add(s, fq_mul(a[ao + i], b[bo + i]));
  return s;
}

h::HExt commit_host(ProverGens& g, const KeyView& k, const FqV& x, const Fq& blind) {
  std::vector<size_t> idx(k.G.begin(), k.G.begin() + x.size());
  idx.push_back(k.h);
  FqV s(x);
  s.push_back(blind);
  return g.host.msm(idx, s);
}

// independent commitments computed together on the host pool (Commitments::commit, src/commitments.rs:69-92)
// SPG_TRACE >= 2: cumulative host time and count of the sigma-protocol commitments (printed by SNARK::prove)
CommitStats g_commit_stats;
std::vector<Pt> commit_batch(ProverGens& g, const std::vector<CJob>& jobs) {
  static const bool tr2 = getenv("SPG_TRACE") && atoi(getenv("SPG_TRACE")) >= 2;
  const auto t0 = tr2 ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  struct Done {
    bool on;
    std::chrono::steady_clock::time_point t0;
    size_t n;
    ~Done() {
      if (!on) return;
      g_commit_stats.us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      g_commit_stats.calls++;
      g_commit_stats.points += n;
    }
  } done{tr2, t0, jobs.size()};
  std::vector<std::pair<std::vector<size_t>, FqV>> j2;
  for (auto& j : jobs) {
    std::vector<size_t> idx;
    FqV s;
    if (j.k) {
      idx.assign(j.k->G.begin(), j.k->G.begin() + j.x.size());
      s = j.x;
    }
    idx.push_back(j.h);
    s.push_back(j.blind);
    j2.push_back({idx, s});
  }
  return g.host.commit_many(j2);
}

// src/nizk/mod.rs:27-53
KnowledgeProofP knowledge_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& x, const Fq& r, Pt* C,
                                const Pt* pre) {
  t.protocol("knowledge proof");
  Fq t1 = tape.scalar("t1"), t2 = tape.scalar("t2");
  std::vector<Pt> c = pre ? std::vector<Pt>(pre, pre + 2) : commit_batch(g, {CJob(k, {x}, r), CJob(k, {t1}, t2)});
  *C = c[0];
  t.point("C", *C);
  KnowledgeProofP p;
  p.alpha = c[1];
  t.point("alpha", p.alpha);
  Fq ch = t.challenge("c");
  p.z1 = fq_add(fq_mul(x, ch), t1);
  p.z2 = fq_add(fq_mul(r, ch), t2);
  return p;
}

// src/nizk/mod.rs:87-115
EqualityProofP equality_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& v1, const Fq& s1,
                              const Fq& v2, const Fq& s2, const Pt* pre) {
  t.protocol("equality proof");
  Fq r = tape.scalar("r");
  std::vector<Pt> c =
      pre ? std::vector<Pt>(pre, pre + 3) : commit_batch(g, {CJob(k, {v1}, s1), CJob(k, {v2}, s2), CJob(k.h, r)});
  t.point("C1", c[0]);
  t.point("C2", c[1]);
  EqualityProofP p;
  p.alpha = c[2];
  t.point("alpha", p.alpha);
  Fq ch = t.challenge("c");
  p.z = fq_add(fq_mul(ch, fq_sub(s1, s2)), r);
  return p;
}

// src/nizk/mod.rs:159-226
ProductProofP product_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& x, const Fq& rX, const Fq& y,
                            const Fq& rY, const Fq& z, const Fq& rZ, Pt* X, Pt* Y, Pt* Z, const Pt* pre) {
  t.protocol("product proof");
  Fq b1 = tape.scalar("b1"), b2 = tape.scalar("b2"), b3 = tape.scalar("b3"), b4 = tape.scalar("b4"),
     b5 = tape.scalar("b5");
  std::vector<Pt> c =
      pre ? std::vector<Pt>(pre, pre + 5)
          : commit_batch(g, {CJob(k, {x}, rX), CJob(k, {y}, rY), CJob(k, {z}, rZ), CJob(k, {b1}, b2), CJob(k, {b3}, b4)});
  *X = c[0];
  *Y = c[1];
  *Z = c[2];
  t.point("X", *X);
  t.point("Y", *Y);
  t.point("Z", *Z);
  ProductProofP p;
  p.alpha = c[3];
  t.point("alpha", p.alpha);
  p.beta = c[4];
  t.point("beta", p.beta);
  if (pre) {
    p.delta = pre[5];  // (b3 x) G + (b3 rX + b5) h = b3 X + b5 h (sigma1_points)
  } else {
    // gens_X = {G: [X.decompress()], h}: X is used through its encoding, as the reference does
    h::HExt Xd;
    h::hext_decompress(X->b, Xd);
    h::HExt dl = h::hext_add(var_mul(Xd, b3), g.host.msm({k.h}, {b5}));
    p.delta = compress(dl);
  }
  t.point("delta", p.delta);
  Fq ch = t.challenge("c");
  p.z[0] = fq_add(b1, fq_mul(ch, x));
  p.z[1] = fq_add(b2, fq_mul(ch, rX));
  p.z[2] = fq_add(b3, fq_mul(ch, y));
  p.z[3] = fq_add(b4, fq_mul(ch, rY));
  p.z[4] = fq_add(b5, fq_mul(ch, fq_sub(rZ, fq_mul(rX, y))));
  return p;
}

void sigma1_points(ProverGens& g, const KeyView& k, const Tape& tape, const Fq& cz, const Fq& cz_blind, const Fq& az,
                   const Fq& az_blind, const Fq& bz, const Fq& bz_blind, const Fq& prod, const Fq& prod_blind,
                   const Fq& v1, const Fq& s1, const Fq& v2, const Fq& s2, Sigma1Pre* out) {
  Tape tp = tape;  // the draws knowledge_prove, product_prove and equality_prove make next, in their order
  const Fq t1 = tp.scalar("t1"), t2 = tp.scalar("t2");
  const Fq b1 = tp.scalar("b1"), b2 = tp.scalar("b2"), b3 = tp.scalar("b3"), b4 = tp.scalar("b4"), b5 = tp.scalar("b5");
  const Fq r = tp.scalar("r");
  std::vector<Pt> c = commit_batch(
      g, {CJob(k, {cz}, cz_blind), CJob(k, {t1}, t2), CJob(k, {az}, az_blind), CJob(k, {bz}, bz_blind),
          CJob(k, {prod}, prod_blind), CJob(k, {b1}, b2), CJob(k, {b3}, b4),
          CJob(k, {fq_mul(b3, az)}, fq_add(fq_mul(b3, az_blind), b5)), CJob(k, {v1}, s1), CJob(k, {v2}, s2),
          CJob(k.h, r)});
  for (int i = 0; i < 2; i++) out->k[i] = c[i];
  for (int i = 0; i < 6; i++) out->p[i] = c[2 + i];
  for (int i = 0; i < 3; i++) out->e[i] = c[8 + i];
}

// src/nizk/mod.rs:306-370 (n = 4 in every sumcheck round). Cx_known: the caller already holds
// x.commit(blind_x, gens_n) (the sumcheck round's comm_poly is exactly that commitment). pre: the randomness
// and its points were drawn / computed ahead (the tape is then not touched here; the caller advances it).
DotProductProofP dotproduct_prove(ProverGens& g, const KeyView& k1, const KeyView& kn, Tr& t, Tape& tape, const FqV& x,
                                  const Fq& blind_x, const FqV& a, const Fq& y, const Fq& blind_y, const Pt* Cx_known,
                                  const DotPre* pre) {
  t.protocol("dot product proof");
  size_t n = x.size();
  DotProductProofP p;
  Pt Cx, Cy;
  FqV d;
  Fq r_delta, r_beta;
  if (pre && Cx_known) {
    d = pre->d;
    r_delta = pre->r_delta;
    r_beta = pre->r_beta;
    Fq ad = dot(a, d, 0, 0, n);
    // Cy = y G_1 + blind_y h; beta = <a, d> G_1 + (r_beta h, precomputed)
    const h::HExt ex[2] = {h::hext_identity(), pre->rbh};
    std::vector<Pt> c = g.host.commit_many_plus({{{k1.G[0], k1.h}, {y, blind_y}}, {{k1.G[0]}, {ad}}}, ex);
    Cx = *Cx_known;
    Cy = c[0];
    p.delta = pre->delta;
    p.beta = c[1];
  } else {
    d = tape.vec("d_vec", n);
    r_delta = tape.scalar("r_delta");
    r_beta = tape.scalar("r_beta");
    Fq ad = dot(a, d, 0, 0, n);
    std::vector<CJob> jobs = {CJob(k1, {y}, blind_y), CJob(kn, d, r_delta), CJob(k1, {ad}, r_beta)};
    if (!Cx_known) jobs.push_back(CJob(kn, x, blind_x));
    std::vector<Pt> c = commit_batch(g, jobs);
    Cx = Cx_known ? *Cx_known : c[3];
    Cy = c[0];
    p.delta = c[1];
    p.beta = c[2];
  }
  t.point("Cx", Cx);
  t.point("Cy", Cy);
  t.scalars("a", a);
  t.point("delta", p.delta);
  t.point("beta", p.beta);
  Fq ch = t.challenge("c");
  p.z.resize(n);
  for (size_t i = 0; i < n; i++) p.z[i] = fq_add(fq_mul(ch, x[i]), d[i]);
  p.z_delta = fq_add(fq_mul(ch, blind_x), r_delta);
  p.z_beta = fq_add(fq_mul(ch, blind_y), r_beta);
  return p;
}

// B fixed-base MSMs of n host scalars each over generator indices already on the device (d_idx: B x n)
// SPG_TRACE >= 2: where a Bullet round's time goes (accumulated over a process, printed per DotProductProofLog)
static Laps g_msm_laps{"DotProductProofLog::prove (cumulative)", getenv("SPG_TRACE") && atoi(getenv("SPG_TRACE")) >= 2};

static h::HExt hext_small_mul(h::HExt P, unsigned k) {
  h::HExt r = h::hext_identity();
  for (; k; k >>= 1) {
    if (k & 1) r = h::hext_add(r, P);
    P = h::hext_dbl(P);
  }
  return r;
}

void bucket_finals(const Ext* bk, size_t B, int NB, Pt* out, const h::HExt* extra, bool carry) {
  // chunk (lo, hi] of a bucket set: run = sum B_v, acc = sum (v - lo) B_v; the set's sum is
  // sum over chunks of acc + lo * run. Chunks spread one MSM's 2 NB dependent additions over the pool;
  // the last chunk of an MSM to finish (countdown) adds the chunks and encodes, all in one burst.
  // chunks per set: one burst wave over the pool (B sets x K chunks ~ threads; at least 2 buckets per chunk)
  static const int kmax = getenv("SPG_FINALS_K") ? std::max(1, atoi(getenv("SPG_FINALS_K"))) : 8;
  const int threads = pool().size() + 1;
  int K = NB >= 64 ? std::max(1, std::min(kmax, threads / (int)std::max<size_t>(B, 1))) : 1;
  while (NB % K) K--;
  const int per = NB / K, stride = NB + (carry ? 1 : 0);
  std::vector<h::HExt> part(B * K);
  std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[B]);
  for (size_t b = 0; b < B; b++) left[b].store(K);
  pool().parallel_for((int)(B * K), [&](int task) {
    const size_t b = task / K;
    const int lo = (task % K) * per;
    for (const uint8_t* q = (const uint8_t*)(bk + b * stride + lo); q < (const uint8_t*)(bk + b * stride + lo + per);
         q += 64)
      __builtin_prefetch(q, 0, 0);  // (as parts_finals)
    h::HExt run = h::hext_identity(), acc = h::hext_identity();
    for (int v = lo + per; v > lo; v--) {
      run = h::hext_add(run, h::hext_from_dev(bk[b * stride + v - 1]));
      acc = h::hext_add(acc, run);
    }
    part[task] = lo ? h::hext_add(acc, hext_small_mul(run, (unsigned)lo)) : acc;
    if (left[b].fetch_sub(1, std::memory_order_acq_rel) == 1) {
      h::HExt s = part[b * K];
      for (int c = 1; c < K; c++) s = h::hext_add(s, part[b * K + c]);
      if (carry) s = h::hext_add(s, h::hext_from_dev(bk[b * stride + NB]));
      if (extra) s = h::hext_add(s, extra[b]);
      out[b] = compress(s);
    }
  });
}

// B MSMs finished from their partial points (the comb form of a Bullet round): MSM b = the sum of bk[b per ..
// b per + per) (+ extra[b]), encoded; chunks of each MSM's parts spread over the pool, the last chunk of an MSM to
// finish adds the chunk sums and encodes
static void parts_finals(const Ext* bk, size_t B, size_t per, Pt* out, const h::HExt* extra) {
  const int threads = pool().size() + 1;
  // chunks of >= 8 parts (>= 48 with the 8-lane IFMA sums, whose lanes want several points each)
  static const bool vec = h::ifma_on() && !(getenv("SPG_VEC_MIN") && atol(getenv("SPG_VEC_MIN")) == 0);
  const size_t cmin = vec ? 48 : 8;
  const int K = (int)std::max<size_t>(1, std::min<size_t>(per / cmin, (size_t)threads / std::max<size_t>(B, 1)));
  std::vector<h::HExt> part(B * K);
  std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[B]);
  for (size_t b = 0; b < B; b++) left[b].store(K);
  pool().parallel_for((int)(B * K), [&](int task) {
    const size_t b = task / K, c = task % K;
    const size_t lo = per * c / K, hi = per * (c + 1) / K;
    // the parts' lines were written by the device (coherent host memory, so not in this core's caches): every line
    // of the chunk requested at once, their misses overlapping, before the dependent additions read them
    for (const uint8_t* q = (const uint8_t*)(bk + b * per + lo); q < (const uint8_t*)(bk + b * per + hi); q += 64)
      __builtin_prefetch(q, 0, 0);
    h::HExt acc;
    if (vec && hi - lo >= 16) {
      thread_local std::vector<h::HExt> hx;
      hx.resize(hi - lo);
      for (size_t i = lo; i < hi; i++) hx[i - lo] = h::hext_from_dev(bk[b * per + i]);
      acc = h::ext_sum8(hx.data(), hi - lo);
    } else {
      acc = h::hext_from_dev(bk[b * per + lo]);
      for (size_t i = lo + 1; i < hi; i++) acc = h::hext_add(acc, h::hext_from_dev(bk[b * per + i]));
    }
    part[task] = acc;
    if (left[b].fetch_sub(1, std::memory_order_acq_rel) == 1) {
      h::HExt sum = part[b * K];
      for (int k = 1; k < K; k++) sum = h::hext_add(sum, part[b * K + k]);
      if (extra) sum = h::hext_add(sum, extra[b]);
      out[b] = compress(sum);
    }
  });
}

// B fixed-base MSMs of n host scalars each over generator indices already on the device (d_idx: B x n)
// h_idx (optional, host, B x n): generator indices uploaded with the scalars in the same copy, d_idx unused
static int device_msm_flat(spg_ctx* ctx, ProverGens& g, const std::vector<Fq>& hs, size_t n, size_t B,
                           const uint32_t* d_idx, std::vector<Pt>* out, const std::vector<uint32_t>* h_idx = nullptr) {
  hipStream_t s = ctx->stream;
  g_msm_laps.lap("bullet_host");
  const size_t sc_bytes = hs.size() * sizeof(Fq), ix_bytes = h_idx ? h_idx->size() * 4 : 0;
  const size_t in_bytes = sc_bytes + ix_bytes, bk_bytes = sizeof(Ext) * B * 256;
  Fq* d_s = (Fq*)ws_get(ctx, 20, in_bytes + 64);
  Ext* d_bk = (Ext*)ws_get(ctx, 23, bk_bytes + 64);
  uint8_t* stage = (uint8_t*)pinned_get(ctx, in_bytes + bk_bytes + 256);
  if (!d_s || !d_bk || !stage) return set_err(ctx, SPG_E_NOMEM, "device_msm");
  // scalars (and indices) up through page-locked staging (a pageable source costs a staging copy + blit per call)
  memcpy(stage, hs.data(), sc_bytes);
  if (h_idx) {
    memcpy(stage + sc_bytes, h_idx->data(), ix_bytes);
    d_idx = (const uint32_t*)((const uint8_t*)d_s + sc_bytes);
  }
  SPG_HIP(ctx, hipMemcpyAsync(d_s, stage, in_bytes, hipMemcpyHostToDevice, s));
  // bucket sums on the device; sum_v v * B_v and the encoding on host cores (a short dependent chain of
  // additions is ~50x faster there than on one GPU lane)
  int NB = 0;
  void* d_map = nullptr;
  Ext* mbk = (Ext*)mapped_get(ctx, bk_bytes, &d_map);  // buckets straight into host memory
  int rc = msm_small_buckets(ctx, g.dev, 0, d_s, n, B, nullptr, d_idx, -1, mbk ? (Ext*)d_map : d_bk, &NB);
  if (rc) return rc;
  Ext* bk = mbk ? mbk : (Ext*)(stage + ((in_bytes + 255) & ~(size_t)255));
  if (!mbk) SPG_HIP(ctx, hipMemcpyAsync(bk, d_bk, sizeof(Ext) * B * NB, hipMemcpyDeviceToHost, s));
  SPG_HIP(ctx, hipStreamSynchronize(s));
  g_msm_laps.lap("msm_device");
  out->resize(B);
  bucket_finals(bk, B, NB, out->data());
  g_msm_laps.lap("msm_host_final");
  return 0;
}

int device_msm_idx(spg_ctx* ctx, ProverGens& g, const std::vector<FqV>& scalars,
                   const std::vector<std::vector<uint32_t>>& idx, std::vector<Pt>* out) {
  size_t B = scalars.size();
  size_t n = 0;
  for (auto& v : scalars) n = std::max(n, v.size());
  std::vector<Fq> hs(B * n, fq_zero());
  std::vector<uint32_t> hi(B * n, 0);
  for (size_t b = 0; b < B; b++) {
    for (size_t i = 0; i < scalars[b].size(); i++) {
      hs[b * n + i] = scalars[b][i];
      hi[b * n + i] = idx[b][i];
    }
  }
  uint32_t* d_i = (uint32_t*)ws_get(ctx, 21, hi.size() * 4 + 64);
  if (!d_i) return set_err(ctx, SPG_E_NOMEM, "device_msm_idx");
  SPG_HIP(ctx, hipMemcpyAsync(d_i, hi.data(), hi.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  return device_msm_flat(ctx, g, hs, n, B, d_i, out);
}

// runs f(lo, hi) over [0, n) in chunks on the host pool
static void par_range(size_t n, const std::function<void(size_t, size_t)>& f) {
  const size_t chunks = n >= 256 ? 8 : 1;
  pool().parallel_for((int)chunks, [&](int c) { f(n * c / chunks, n * (c + 1) / chunks); });
}

// Folds of one Bullet round on host copies (a, b for the next c_L / c_R, cw for the final g_hat) with u and
// u^-1 of the round that took the size from 2 nn to nn (when fold), plus the next round's cross products
// c_L = <a_L, b_R>, c_R = <a_R, b_L> over the halves of nn / 2 entries, in one pool burst.
static void host_fold_dots(FqV& aa, FqV& bb, FqV* cw, size_t n, size_t nn, bool fold, const Fq& u, const Fq& uinv,
                           Fq* cL, Fq* cR) {
  const size_t nh = nn / 2;  // nn: size after the fold (2 nn before it)
  const int C = nh >= 64 ? 8 : 1;
  Fq pl[8], pr[8];
  pool().parallel_for(C, [&](int c) {
    Fq sl = fq_zero(), sr = fq_zero();
    for (size_t i = nh * c / C; i < nh * (c + 1) / C; i++) {
      if (fold) {
        for (size_t i2 : {i, i + nh}) {
          aa[i2] = fq_add(fq_mul(aa[i2], u), fq_mul(uinv, aa[i2 + nn]));
          bb[i2] = fq_add(fq_mul(bb[i2], uinv), fq_mul(u, bb[i2 + nn]));
        }
      }
      sl = fq_add(sl, fq_mul(aa[i], bb[i + nh]));
      sr = fq_add(sr, fq_mul(aa[i + nh], bb[i]));
    }
    if (fold && cw)  // (cw null: delta's scalars come from the device's own cw, DevFinal)
      for (size_t j = n * c / C; j < n * (c + 1) / C; j++) (*cw)[j] = fq_mul((*cw)[j], (j % (2 * nn)) < nn ? uinv : u);
    pl[c] = sl;
    pr[c] = sr;
  });
  *cL = pl[0];
  *cR = pr[0];
  for (int c = 1; c < C; c++) {
    *cL = fq_add(*cL, pl[c]);
    *cR = fq_add(*cR, pr[c]);
  }
}

// Every Bullet round of one DotProductProofLog with the round's fold and MSM scalars computed on the device
// (bullet_round_device): per round the host launches one kernel with (u, u^-1), then - while it runs - folds
// its own copies of a, b, cw and computes c_L, c_R and the G_1 / h terms of L and R, waits for the bucket
// sums (mailbox), finishes L and R on the pool and draws the next challenge. Same transcript, same points.
// Round 0 of bullet_rounds_device launched ahead (with the Cx MSM, before the transcript yields r): its L and R
// MSM scalars are a and the unit weights alone, and the r-dependent G_1 terms are added on the host afterwards.
// x: the n scalars on the device (copied into the round state); *seq: round 0's mailbox number.
// One device Bullet round: the comb form (k_bullet_comb; partial points, *per = parts per MSM) when the generator set
// has a comb table for the proof's generators (gmax = the largest generator index + 1), else the bucket form
// (k_bullet_round_q; *per = 0: 2 x (64 + 1) bucket sums)
static int bullet_round_launch(spg_ctx* ctx, ProverGens& g, const Fq* aa_in, const Fq* cw_in, Fq* aa_out, Fq* cw_out,
                               const uint32_t* d_idx, size_t gmax, const Fq& u, const Fq& uinv, int k, size_t n,
                               size_t nk, Ext* d_bk, uint32_t* seq, int* per) {
  *per = 0;
  int rc = bullet_round_comb(ctx, g.dev, aa_in, cw_in, aa_out, cw_out, d_idx, gmax, u, uinv, k, (int)n, (int)nk, d_bk,
                             seq, per);
  if (rc != 1) return rc;
  *per = 0;
  return bullet_round_device(ctx, g.dev, aa_in, cw_in, aa_out, cw_out, d_idx, u, uinv, k, (int)n, (int)nk, d_bk, seq);
}

static int bullet_round0_launch(spg_ctx* ctx, ProverGens& g, size_t n, const Fq* d_x, const uint32_t* d_idx,
                                size_t gmax, Ext* d_bk, uint32_t* seq, int* per) {
  Fq* st = (Fq*)ws_get(ctx, 24, 4 * n * sizeof(Fq) + 64);  // aa[2], cw[2]
  if (!st) return set_err(ctx, SPG_E_NOMEM, "bullet state");
  // round 0 reads a = x where the Cx MSM's scalars already are, and writes the state round 1 reads (aa[1], cw[1]);
  // no later round reads aa[0] before writing it
  return bullet_round_launch(ctx, g, d_x, st + 2 * n, st + n, st + 3 * n, d_idx, gmax, fq_zero(), fq_zero(), 0, n, n,
                             d_bk, seq, per);
}

// what the device rounds leave for delta's scalars (fin != null: the host keeps no copy of cw; the rounds fold the
// device's)
struct DevFinal {
  const Fq* cw = nullptr;  // the device cw before the last challenge's fold (plain integers)
  Fq u, uinv;              // the last challenge
};

static int bullet_rounds_device(spg_ctx* ctx, ProverGens& g, Tr& t, const FqV& x, const FqV& a, const Fq& r,
                                const FqV& v1, const FqV& v2, const uint32_t* d_idx, size_t gmax, Ext* mbk, Ext* d_bk,
                                FqV* aa, FqV* bb, FqV* cw, Fq* blind_fin, DotProductProofLogP* out, bool pre0 = false,
                                uint32_t seq0 = 0, int per0 = 0, DevFinal* fin = nullptr) {
  const size_t n = x.size();
  const size_t G1 = g.gens_1.G[0], H = g.gens_n.h;
  Fq* st = (Fq*)ws_get(ctx, 24, 4 * n * sizeof(Fq) + 64);  // aa[2], cw[2]
  if (!st) return set_err(ctx, SPG_E_NOMEM, "bullet state");
  Fq* d_aa[2] = {st, st + n};
  Fq* d_cw[2] = {st + 2 * n, st + 3 * n};
  if (!pre0) {
    uint8_t* stage = (uint8_t*)pinned_get(ctx, n * sizeof(Fq));
    if (!stage) return set_err(ctx, SPG_E_NOMEM, "bullet staging");
    memcpy(stage, x.data(), n * sizeof(Fq));
    SPG_HIP(ctx, hipMemcpyAsync(d_aa[0], stage, n * sizeof(Fq), hipMemcpyHostToDevice, ctx->stream));
  }
  Fq u = fq_zero(), uinv = fq_zero();
  size_t nk = n;
  for (int k = 0; nk != 1; k++) {
    uint32_t seq = seq0;
    int per = per0;
    int rc = k == 0 && pre0 ? 0
                            : bullet_round_launch(ctx, g, d_aa[k & 1], d_cw[k & 1], d_aa[(k + 1) & 1], d_cw[(k + 1) & 1],
                                                  d_idx, gmax, u, uinv, k, n, nk, d_bk, &seq, &per);
    if (rc) return rc;
    g_msm_laps.lap("bullet_launch");
    Fq cL, cR;
    host_fold_dots(*aa, *bb, fin ? nullptr : cw, n, nk, k > 0, u, uinv, &cL, &cR);
    const Fq blind_L = v1[k], blind_R = v2[k];
    std::vector<h::HExt> ex = g.host.sum_many({{{G1, H}, {fq_mul(cL, r), blind_L}}, {{G1, H}, {fq_mul(cR, r), blind_R}}});
    g_msm_laps.lap("bullet_host_overlap");
    rc = mbox_wait(ctx, seq, nullptr, 0);
    if (rc) return rc;
    g_msm_laps.lap("msm_device");
    Pt LR[2];
    if (per)
      parts_finals(mbk, 2, (size_t)per, LR, ex.data());
    else
      bucket_finals(mbk, 2, kBulletNB, LR, ex.data(), true);
    g_msm_laps.lap("msm_host_final");
    t.point("L", LR[0]);
    t.point("R", LR[1]);
    u = t.challenge("u");
    uinv = fq_inv(u);
    *blind_fin = fq_add(fq_add(*blind_fin, fq_mul(fq_mul(blind_L, u), u)), fq_mul(fq_mul(blind_R, uinv), uinv));
    out->L.push_back(LR[0]);
    out->R.push_back(LR[1]);
    g_msm_laps.lap("bullet_challenge");
    nk /= 2;
  }
  // the last round's fold of the host copies (a_hat, b_hat and the final generator weights; with fin, delta's scalars
  // come from the device cw instead)
  (*aa)[0] = fq_add(fq_mul((*aa)[0], u), fq_mul(uinv, (*aa)[1]));
  (*bb)[0] = fq_add(fq_mul((*bb)[0], uinv), fq_mul(u, (*bb)[1]));
  if (fin) {
    size_t lg = 0;
    while (((size_t)1 << lg) < n) lg++;
    fin->cw = d_cw[lg & 1];  // round lg - 1 wrote d_cw[lg & 1]
    fin->u = u;
    fin->uinv = uinv;
  } else {
    par_range(n, [&](size_t lo, size_t hi) {
      for (size_t j = lo; j < hi; j++) (*cw)[j] = fq_mul((*cw)[j], (j & 1) ? u : uinv);
    });
  }
  g_msm_laps.lap("bullet_fold");
  return 0;
}

// src/nizk/mod.rs:439-523 + src/nizk/bullet.rs:32-132
int dotproduct_log_prove(spg_ctx* ctx, ProverGens& g, Tr& t, Tape& tape, const FqV& x, const Fq& blind_x, const FqV& a,
                         const Fq& y, const Fq& blind_y, DotProductProofLogP* out, Pt* Cy_out) {
  g_msm_laps.lap("outside_bullet");
  // SPG_TRACE >= 3: this proof's own laps (the difference of the cumulative ones), one line per proof
  static const bool per_proof = getenv("SPG_TRACE") && atoi(getenv("SPG_TRACE")) >= 3;
  const std::vector<std::pair<std::string, double>> laps0 = per_proof ? g_msm_laps.acc : decltype(laps0)();
  t.protocol("dot product proof (log)");
  size_t n = x.size();
  size_t lg = 0;
  while (((size_t)1 << lg) < n) lg++;
  if (n > g.n_pc) return set_err(ctx, SPG_E_ARG, "DotProductProofLog: n exceeds gens");
  Fq d = tape.scalar("d");
  Fq r_delta = tape.scalar("r_delta");
  Fq r_beta = tape.scalar("r_delta");
  FqV v1 = tape.vec("blinds_vec_1", 2 * lg);
  FqV v2 = tape.vec("blinds_vec_2", 2 * lg);
  const KeyView& kn = g.gens_n;
  const uint32_t G1 = (uint32_t)g.gens_1.G[0], H = (uint32_t)kn.h;
  // Small proofs (n <= SPG_BULLET_HOST_MAX, default 32) run every MSM on the host pool against fixed-base
  // tables of their n generators: a round's two MSMs are then 32 n byte-window additions spread over the pool
  // instead of a device round trip. Early in round 6 (comb rounds ~17 us) 16 beat 32; once the host proof had its
  // Cy / beta off the chain, side-by-side encodings and the two-chain Fp carries, 32 beat 16 in 9 of 10 alternations
  // (median -0.5 to -0.9 ms) and tied 64, and 128 lost (profiles/r06_ab_bullet_host_max.txt).
  static const size_t host_max = getenv("SPG_BULLET_HOST_MAX") ? (size_t)atol(getenv("SPG_BULLET_HOST_MAX")) : 32;
  const bool on_host = n <= host_max;
  // generator indices G_0..G_{n-1}, G_1, h for B = 2 MSMs, uploaded once for all rounds
  const size_t n2 = n + 2;
  uint32_t* d_idx = nullptr;
  using HostJob = std::pair<std::vector<size_t>, FqV>;
  static const bool dev_rounds = !getenv("SPG_BULLET_DEV") || atoi(getenv("SPG_BULLET_DEV")) != 0;
  static const bool ahead = !getenv("SPG_BULLET_AHEAD") || atoi(getenv("SPG_BULLET_AHEAD")) != 0;
  const bool dev_path = dev_rounds && !on_host && n >= 2 && (n & (n - 1)) == 0;
  std::vector<uint32_t> idx2;
  if (!on_host) {
    idx2.resize(2 * n2);
    for (size_t b = 0; b < 2; b++) {
      for (size_t j = 0; j < n; j++) idx2[b * n2 + j] = (uint32_t)kn.G[j];
      idx2[b * n2 + n] = G1;
      idx2[b * n2 + n + 1] = H;
    }
    if (!(dev_path && ahead)) {  // (the ahead path uploads them with the Cx scalars)
      d_idx = (uint32_t*)ws_get(ctx, 21, idx2.size() * 4 + 64);
      if (!d_idx) return set_err(ctx, SPG_E_NOMEM, "bullet indices");
      SPG_HIP(ctx, hipMemcpyAsync(d_idx, idx2.data(), idx2.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    }
  }
  // mapped host memory for the bucket sums: [Cx MSM (B = 1, up to 256 buckets)][Bullet rounds: 2 x 65 buckets, or
  // 2 x up to kBulletPartsMax partial points of the comb form]
  const size_t cx_bytes = sizeof(Ext) * std::max<size_t>(256, kBulletPartsMax),
               br_bytes = sizeof(Ext) * 2 * std::max<size_t>(kBulletNB + 1, kBulletPartsMax) + 64;
  size_t gmax = 0;  // the comb form needs the table to cover G_0 .. G_{n-1} of this proof
  for (size_t j = 0; j < n; j++) gmax = std::max(gmax, kn.G[j] + 1);
  void* d_map = nullptr;
  uint8_t* mapped = dev_path ? (uint8_t*)mapped_get(ctx, cx_bytes + br_bytes, &d_map) : nullptr;
  Ext* mbk = mapped ? (Ext*)(mapped + cx_bytes) : nullptr;
  Ext* d_mbk = mapped ? (Ext*)((uint8_t*)d_map + cx_bytes) : nullptr;
  // Cx = x.commit(blind_x, gens_n)
  std::vector<Pt> pts;
  bool pre0 = false;
  uint32_t seq0 = 0;
  int per0 = 0;
  // Cy = y.commit(blind_y, gens_1) depends on no challenge: it is computed beside Cx (in Cx's host burst, or on the
  // pool while the device computes Cx) instead of in a burst of its own after it; the transcript still takes Cx first
  // (SPG_DOTLOG_EARLY=0: Cy and beta in bursts of their own, in transcript order)
  static const bool early = !getenv("SPG_DOTLOG_EARLY") || atoi(getenv("SPG_DOTLOG_EARLY")) != 0;
  Pt Cy;
  bool cy_done = false;
  auto cy_job = [&]() -> HostJob {
    return HostJob{{(size_t)g.gens_1.G[0], (size_t)g.gens_1.h}, {y, blind_y}};
  };
  if (mbk && ahead) {
    // the Cx bucket sums, then Bullet round 0 (which needs no challenge), on the stream before the host waits
    // for Cx: one device round trip fewer per proof
    // one page-locked copy: the Cx scalars (x, 0, blind_x), then the generator indices of every round
    const size_t sb = n2 * sizeof(Fq), ib = idx2.size() * 4;
    Fq* d_s = (Fq*)ws_get(ctx, 20, sb + ib + 64);
    uint8_t* stage = (uint8_t*)pinned_get(ctx, sb + ib + 64);
    if (!d_s || !stage || idx2.empty()) return set_err(ctx, SPG_E_NOMEM, "Cx");
    memcpy(stage, x.data(), n * sizeof(Fq));
    memset(stage + n * sizeof(Fq), 0, sizeof(Fq));
    memcpy(stage + (n + 1) * sizeof(Fq), &blind_x, sizeof(Fq));
    memcpy(stage + sb, idx2.data(), ib);
    SPG_HIP(ctx, hipMemcpyAsync(d_s, stage, sb + ib, hipMemcpyHostToDevice, ctx->stream));
    d_idx = (uint32_t*)((uint8_t*)d_s + sb);
    // Cx from the comb table as partial points (+ blind_x h on the host), or the bucket sums of the latency path
    int NB = 0, cper = 0;
    int rc = comb_msm_parts(ctx, g.dev, d_s, d_idx, gmax, (int)n, 1, (Ext*)d_map, &cper);
    if (rc == 1) {
      cper = 0;
      rc = msm_small_buckets(ctx, g.dev, 0, d_s, n2, 1, nullptr, d_idx, -1, (Ext*)d_map, &NB);
    }
    if (rc) return rc;
    SPG_HIP(ctx, hipEventRecord(ctx->ev_cx, ctx->stream));
    rc = bullet_round0_launch(ctx, g, n, d_s, d_idx, gmax, d_mbk, &seq0, &per0);
    if (rc) return rc;
    pre0 = true;
    h::HExt blind_h;
    if (cper) blind_h = g.host.sum_many({{{(size_t)H}, {blind_x}}})[0];  // while the device works
    if (early) {
      Cy = g.host.commit_many({cy_job()})[0];
      cy_done = true;
    }
    SPG_HIP(ctx, hipEventSynchronize(ctx->ev_cx));
    pts.resize(1);
    if (cper)
      parts_finals((const Ext*)mapped, 1, (size_t)cper, pts.data(), &blind_h);
    else
      bucket_finals((const Ext*)mapped, 1, NB, pts.data());
  } else if (on_host) {
    HostJob j{std::vector<size_t>(kn.G.begin(), kn.G.begin() + n), x};
    j.first.push_back(kn.h);
    j.second.push_back(blind_x);
    pts = early ? g.host.commit_many({j, cy_job()}) : g.host.commit_many({j});
    if (early) {
      Cy = pts[1];
      cy_done = true;
    }
  } else {
    std::vector<Fq> hs(n2, fq_zero());
    std::copy(x.begin(), x.end(), hs.begin());
    hs[n + 1] = blind_x;
    int rc = device_msm_flat(ctx, g, hs, n2, 1, d_idx, &pts);
    if (rc) return rc;
  }
  Pt Cx = pts[0];
  t.point("Cx", Cx);
  g_msm_laps.lap("bp_cx");
  if (!cy_done) Cy = commit_batch(g, {CJob(g.gens_1, {y}, blind_y)})[0];
  g_msm_laps.lap("bp_cy");
  t.point("Cy", Cy);
  t.scalars("a", a);
  g_msm_laps.lap("bp_tr");
  Fq r = t.challenge("r");
  Fq blind_fin = fq_add(blind_x, fq_mul(r, blind_y));
  FqV aa(x), bb(a), cw(n, fq_one());
  // per-round L / R MSM inputs: hn = n/2 + 2 scalars and generator indices each (G_1 and h last)
  const size_t hn = n / 2 + 2;
  std::vector<Fq> hc(2 * hn);
  std::vector<uint32_t> ic(2 * hn);
  FqV fa(n / 2), fb(n / 2);  // fold products that need u only
  for (size_t b = 0; b < 2; b++) {
    ic[b * hn + n / 2] = G1;
    ic[b * hn + n / 2 + 1] = H;
  }
  size_t nk = n, k = 0;
  bool beta_done = false;
  g_msm_laps.lap("bullet_prep");
  // delta's scalars d cw_j on the device from the rounds' own cw (no host fold of cw, no upload; SPG_DELTA_DEV=0: host)
  static const bool delta_dev = !getenv("SPG_DELTA_DEV") || atoi(getenv("SPG_DELTA_DEV")) != 0;
  static const bool delta_comb = !getenv("SPG_DELTA_COMB") || atoi(getenv("SPG_DELTA_COMB")) != 0;
  DevFinal dfin;
  const bool use_dfin = mbk && delta_comb && delta_dev;
  if (mbk) {
    int rc = bullet_rounds_device(ctx, g, t, x, a, r, v1, v2, d_idx, gmax, mbk, d_mbk, &aa, &bb, &cw, &blind_fin, out,
                                  pre0, seq0, per0, use_dfin ? &dfin : nullptr);
    if (rc) return rc;
    nk = 1;
  }
  while (nk != 1) {
    size_t nh = nk / 2;
    Fq cL = dot(aa, bb, 0, nh, nh), cR = dot(aa, bb, nh, 0, nh);
    g_msm_laps.lap("bullet_dot");
    Fq blind_L = v1[k], blind_R = v2[k];
    // L = sum over the n/2 generators j with (j mod nk) >= nh of a[j mod nk - nh] cw_j G_j (+ cL r G_1 +
    // blind_L h), R over the other half; each MSM carries only its own half (hc = n/2 + 2 scalars, explicit
    // generator indices uploaded with them), so the bucket kernel extracts digits of half as many scalars
    par_range(n / 2, [&](size_t lo, size_t hi) {
      for (size_t p = lo; p < hi; p++) {
        const size_t blk = p / nh, off = p % nh, jl = blk * nk + nh + off, jr = blk * nk + off;
        hc[p] = fq_mul(aa[off], cw[jl]);
        ic[p] = (uint32_t)kn.G[jl];
        hc[hn + p] = fq_mul(aa[off + nh], cw[jr]);
        ic[hn + p] = (uint32_t)kn.G[jr];
      }
    });
    hc[n / 2] = fq_mul(cL, r);
    hc[n / 2 + 1] = blind_L;
    hc[hn + n / 2] = fq_mul(cR, r);
    hc[hn + n / 2 + 1] = blind_R;
    g_msm_laps.lap("bullet_scalars");
    if (on_host) {
      std::vector<HostJob> jobs(2);
      for (size_t b = 0; b < 2; b++) {
        jobs[b].first.assign(ic.begin() + b * hn, ic.begin() + (b + 1) * hn);
        jobs[b].second.assign(hc.begin() + b * hn, hc.begin() + (b + 1) * hn);
      }
      // beta = (d r) G_1 + r_beta h needs r alone: it rides in round 0's burst (appended to the transcript at the end)
      const bool with_beta = early && k == 0;
      if (with_beta) jobs.push_back(HostJob{{(size_t)G1, (size_t)H}, {fq_mul(d, r), r_beta}});
      pts = g.host.commit_many(jobs);
      if (with_beta) {
        out->beta = pts[2];
        beta_done = true;
      }
    } else {
      int rc = device_msm_flat(ctx, g, hc, hn, 2, nullptr, &pts, &ic);
      if (rc) return rc;
    }
    t.point("L", pts[0]);
    t.point("R", pts[1]);
    Fq u = t.challenge("u");
    Fq uinv;
    static const bool overlap = !getenv("SPG_BULLET_OVERLAP") || atoi(getenv("SPG_BULLET_OVERLAP")) != 0;
    if (n < 256 || !overlap) {
      uinv = fq_inv(u);
      for (size_t i = 0; i < nh; i++) {
        aa[i] = fq_add(fq_mul(aa[i], u), fq_mul(uinv, aa[i + nh]));
        bb[i] = fq_add(fq_mul(bb[i], uinv), fq_mul(u, bb[i + nh]));
      }
      for (size_t j = 0; j < n; j++) cw[j] = fq_mul(cw[j], (j % nk) < nh ? uinv : u);
    } else {
      // two bursts: the inversion of u (a ~5 us binary GCD) runs as task 0 of the first, beside the
      // products that need u only; the second finishes every fold with u^-1 (same field values)
      const int C = 8;
      pool().parallel_for(C + 1, [&](int task) {
        if (task == 0) {
          uinv = fq_inv(u);
          return;
        }
        const int c = task - 1;
        for (size_t i = nh * c / C; i < nh * (c + 1) / C; i++) {
          fa[i] = fq_mul(aa[i], u);
          fb[i] = fq_mul(u, bb[i + nh]);
        }
        for (size_t j = n * c / C; j < n * (c + 1) / C; j++)
          if ((j % nk) >= nh) cw[j] = fq_mul(cw[j], u);
      });
      pool().parallel_for(C, [&](int c) {
        for (size_t i = nh * c / C; i < nh * (c + 1) / C; i++) {
          aa[i] = fq_add(fa[i], fq_mul(uinv, aa[i + nh]));
          bb[i] = fq_add(fq_mul(bb[i], uinv), fb[i]);
        }
        for (size_t j = n * c / C; j < n * (c + 1) / C; j++)
          if ((j % nk) < nh) cw[j] = fq_mul(cw[j], uinv);
      });
    }
    blind_fin = fq_add(fq_add(blind_fin, fq_mul(fq_mul(blind_L, u), u)), fq_mul(fq_mul(blind_R, uinv), uinv));
    g_msm_laps.lap("bullet_fold");
    out->L.push_back(pts[0]);
    out->R.push_back(pts[1]);
    nk = nh;
    k++;
  }
  // x_hat = folded x (secret), a_hat = folded a (public), as BulletReductionProof::prove returns them
  Fq x_hat = aa[0], a_hat = bb[0];
  Fq y_hat = fq_mul(x_hat, a_hat);
  // delta = d * g_hat + r_delta * h with g_hat = sum_j cw[j] G_j
  if (on_host) {
    HostJob j{std::vector<size_t>(kn.G.begin(), kn.G.begin() + n), FqV(n)};
    for (size_t i = 0; i < n; i++) j.second[i] = fq_mul(d, cw[i]);
    j.first.push_back(kn.h);
    j.second.push_back(r_delta);
    pts = g.host.commit_many({j});
  } else {
    // device rounds: d g_hat from the comb table as partial points (as Cx), r_delta h and beta on the host meanwhile;
    // the bucket form (device_msm_flat) where the comb does not apply
    int cper = 0, rc = 1;
    if (mbk && delta_comb) {  // (the mapped region's Cx part and slot 26 are free again: Cx is done, the rounds are over)
      Fq* d_s = (Fq*)ws_get(ctx, 26, n * sizeof(Fq) + 64);
      if (!d_s) return set_err(ctx, SPG_E_NOMEM, "delta scalars");
      if (use_dfin) {
        rc = bullet_delta_scalars(ctx, dfin.cw, (int)n, d, dfin.u, dfin.uinv, d_s);
        if (rc) return rc;
      } else {
        Fq* stage = (Fq*)pinned_get(ctx, n * sizeof(Fq) + 64);
        if (!stage) return set_err(ctx, SPG_E_NOMEM, "delta scalars");
        par_range(n, [&](size_t lo, size_t hi) {
          for (size_t j = lo; j < hi; j++) stage[j] = fq_mul(d, cw[j]);
        });
        SPG_HIP(ctx, hipMemcpyAsync(d_s, stage, n * sizeof(Fq), hipMemcpyHostToDevice, ctx->stream));
      }
      rc = comb_msm_parts(ctx, g.dev, d_s, d_idx, gmax, (int)n, 1, (Ext*)d_map, &cper);
      if (rc != 0 && rc != 1) return rc;
    }
    if (rc == 1 && use_dfin) {  // the comb does not apply: cw from the device (plain integers), with the last fold
      SPG_HIP(ctx, hipMemcpyAsync(cw.data(), dfin.cw, n * sizeof(Fq), hipMemcpyDeviceToHost, ctx->stream));
      SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
      par_range(n, [&](size_t lo, size_t hi) {
        for (size_t j = lo; j < hi; j++) cw[j] = fq_mul(fq_to_mont(cw[j]), (j & 1) ? dfin.u : dfin.uinv);
      });
    }
    if (rc == 0) {
      SPG_HIP(ctx, hipEventRecord(ctx->ev_cx, ctx->stream));
      const h::HExt rdh = g.host.sum_many({{{(size_t)H}, {r_delta}}})[0];
      out->beta = g.host.commit_many({{{(size_t)G1, (size_t)H}, {fq_mul(d, r), r_beta}}})[0];
      beta_done = true;
      SPG_HIP(ctx, hipEventSynchronize(ctx->ev_cx));
      pts.resize(1);
      parts_finals((const Ext*)mapped, 1, (size_t)cper, pts.data(), &rdh);
    } else {
      std::vector<Fq> s(n2, fq_zero());
      par_range(n, [&](size_t lo, size_t hi) {
        for (size_t j = lo; j < hi; j++) s[j] = fq_mul(d, cw[j]);
      });
      s[n + 1] = r_delta;
      rc = device_msm_flat(ctx, g, s, n2, 1, d_idx, &pts);
      if (rc) return rc;
    }
  }
  out->delta = pts[0];
  t.point("delta", out->delta);
  if (!beta_done)
    out->beta = g.host.commit_many({{{(size_t)G1, (size_t)H}, {fq_mul(d, r), r_beta}}})[0];
  t.point("beta", out->beta);
  Fq c = t.challenge("c");
  out->z1 = fq_add(d, fq_mul(c, y_hat));
  out->z2 = fq_add(fq_mul(a_hat, fq_add(fq_mul(c, blind_fin), r_beta)), r_delta);
  if (Cy_out) *Cy_out = Cy;
  g_msm_laps.lap("bullet_host");
  g_msm_laps.print();
  if (per_proof) {
    fprintf(stderr, "[spg] DotProductProofLog n=%zu %s:", n, on_host ? "host" : (mbk ? "device" : "device-flat"));
    double tot = 0;
    for (auto& a : g_msm_laps.acc) {
      double before = 0;
      for (auto& b : laps0)
        if (b.first == a.first) before = b.second;
      if (a.first != "outside_bullet" && a.second - before > 0.5) {
        fprintf(stderr, " %s=%.0f", a.first.c_str(), a.second - before);
        tot += a.second - before;
      }
    }
    fprintf(stderr, " total=%.0f\n", tot);
  }
  return 0;
}

}  // namespace spg
