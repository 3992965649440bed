// spg — sigma protocols (host) and DotProductProofLog / Bulletproofs with GPU MSMs.
//
// Bulletproofs rewrite (src/nizk/bullet.rs:32-132): the prover folds G_L[i] = u^-1 G_L[i] + u G_R[i] every
// round. After k rounds G^(k)[i] = sum_{j = i mod n_k} cw[j] * G_j over the ORIGINAL generators, with
// per-generator weights cw that are products of u / u^-1. So every L, R (and the final g_hat) is a
// fixed-base MSM over the generator table already resident in HBM (msm.hip); no curve point is ever
// folded and the group elements produced are identical to the reference's.
#include "proto.hpp"

namespace spg {

static Fq dot(const FqV& a, const FqV& b, size_t ao, size_t bo, size_t n) {
  Fq s = fq_zero();
  for (size_t i = 0; i < n; i++) s = fq_add(s, fq_mul(a[ao + i], b[bo + i]));
  return s;
}

Ext commit_host(ProverGens& g, const KeyView& k, const FqV& x, const Fq& blind) {
  std::vector<size_t> idx(k.G.begin(), k.G.begin() + x.size());
  idx.push_back(k.h);
  FqV s(x);
  s.push_back(blind);
  return g.host.msm(idx, s);
}

// src/nizk/mod.rs:27-53
KnowledgeProofP knowledge_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& x, const Fq& r, Pt* C) {
  t.protocol("knowledge proof");
  Fq t1 = tape.scalar("t1"), t2 = tape.scalar("t2");
  *C = compress(commit_host(g, k, {x}, r));
  t.point("C", *C);
  KnowledgeProofP p;
  p.alpha = compress(commit_host(g, k, {t1}, t2));
  t.point("alpha", p.alpha);
  Fq c = t.challenge("c");
  p.z1 = fq_add(fq_mul(x, c), t1);
  p.z2 = fq_add(fq_mul(r, c), t2);
  return p;
}

// src/nizk/mod.rs:87-115
EqualityProofP equality_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& v1, const Fq& s1,
                              const Fq& v2, const Fq& s2) {
  t.protocol("equality proof");
  Fq r = tape.scalar("r");
  Pt C1 = compress(commit_host(g, k, {v1}, s1));
  t.point("C1", C1);
  Pt C2 = compress(commit_host(g, k, {v2}, s2));
  t.point("C2", C2);
  EqualityProofP p;
  p.alpha = compress(g.host.msm({k.h}, {r}));
  t.point("alpha", p.alpha);
  Fq c = t.challenge("c");
  p.z = fq_add(fq_mul(c, fq_sub(s1, s2)), r);
  return p;
}

// src/nizk/mod.rs:159-226
ProductProofP product_prove(ProverGens& g, const KeyView& k, Tr& t, Tape& tape, const Fq& x, const Fq& rX, const Fq& y,
                            const Fq& rY, const Fq& z, const Fq& rZ, Pt* X, Pt* Y, Pt* Z) {
  t.protocol("product proof");
  Fq b1 = tape.scalar("b1"), b2 = tape.scalar("b2"), b3 = tape.scalar("b3"), b4 = tape.scalar("b4"),
     b5 = tape.scalar("b5");
  Ext Xe = commit_host(g, k, {x}, rX);
  *X = compress(Xe);
  t.point("X", *X);
  *Y = compress(commit_host(g, k, {y}, rY));
  t.point("Y", *Y);
  *Z = compress(commit_host(g, k, {z}, rZ));
  t.point("Z", *Z);
  ProductProofP p;
  p.alpha = compress(commit_host(g, k, {b1}, b2));
  t.point("alpha", p.alpha);
  p.beta = compress(commit_host(g, k, {b3}, b4));
  t.point("beta", p.beta);
  // gens_X = {G: [X.decompress()], h}: X is used through its encoding, as the reference does
  Ext Xd;
  ext_decompress(X->b, Xd);
  Ext dl = ext_add(var_mul(Xd, b3), g.host.msm({k.h}, {b5}));
  p.delta = compress(dl);
  t.point("delta", p.delta);
  Fq c = t.challenge("c");
  p.z[0] = fq_add(b1, fq_mul(c, x));
  p.z[1] = fq_add(b2, fq_mul(c, rX));
  p.z[2] = fq_add(b3, fq_mul(c, y));
  p.z[3] = fq_add(b4, fq_mul(c, rY));
  p.z[4] = fq_add(b5, fq_mul(c, fq_sub(rZ, fq_mul(rX, y))));
  return p;
}

// src/nizk/mod.rs:306-370 (n = 4 in every sumcheck round)
DotProductProofP dotproduct_prove(ProverGens& g, const KeyView& k1, const KeyView& kn, Tr& t, Tape& tape, const FqV& x,
                                  const Fq& blind_x, const FqV& a, const Fq& y, const Fq& blind_y) {
  t.protocol("dot product proof");
  size_t n = x.size();
  FqV d = tape.vec("d_vec", n);
  Fq r_delta = tape.scalar("r_delta"), r_beta = tape.scalar("r_beta");
  Pt Cx = compress(commit_host(g, kn, x, blind_x));
  t.point("Cx", Cx);
  Pt Cy = compress(commit_host(g, k1, {y}, blind_y));
  t.point("Cy", Cy);
  t.scalars("a", a);
  DotProductProofP p;
  p.delta = compress(commit_host(g, kn, d, r_delta));
  t.point("delta", p.delta);
  Fq ad = dot(a, d, 0, 0, n);
  p.beta = compress(commit_host(g, k1, {ad}, r_beta));
  t.point("beta", p.beta);
  Fq c = t.challenge("c");
  p.z.resize(n);
  for (size_t i = 0; i < n; i++) p.z[i] = fq_add(fq_mul(c, x[i]), d[i]);
  p.z_delta = fq_add(fq_mul(c, blind_x), r_delta);
  p.z_beta = fq_add(fq_mul(c, blind_y), r_beta);
  return p;
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
  hipStream_t s = ctx->stream;
  Fq* d_s = (Fq*)ws_get(ctx, 20, hs.size() * sizeof(Fq) + 64);
  uint32_t* d_i = (uint32_t*)ws_get(ctx, 21, hi.size() * 4 + 64);
  uint8_t* d_o = (uint8_t*)ws_get(ctx, 22, 32 * B + 64);
  if (!d_s || !d_i || !d_o) return set_err(ctx, SPG_E_NOMEM, "device_msm_idx");
  SPG_HIP(ctx, hipMemcpyAsync(d_s, hs.data(), hs.size() * sizeof(Fq), hipMemcpyHostToDevice, s));
  SPG_HIP(ctx, hipMemcpyAsync(d_i, hi.data(), hi.size() * 4, hipMemcpyHostToDevice, s));
  int rc = msm_batch_device(ctx, g.dev, 0, d_s, n, B, nullptr, d_o, d_i, -1);
  if (rc) return rc;
  out->resize(B);
  SPG_HIP(ctx, hipMemcpyAsync(out->data(), d_o, 32 * B, hipMemcpyDeviceToHost, s));
  SPG_HIP(ctx, hipStreamSynchronize(s));
  return 0;
}

// src/nizk/mod.rs:439-523 + src/nizk/bullet.rs:32-132
int dotproduct_log_prove(spg_ctx* ctx, ProverGens& g, Tr& t, Tape& tape, const FqV& x, const Fq& blind_x, const FqV& a,
                         const Fq& y, const Fq& blind_y, DotProductProofLogP* out, Pt* Cy_out) {
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
  std::vector<uint32_t> idx_full(n + 2);
  for (size_t j = 0; j < n; j++) idx_full[j] = (uint32_t)kn.G[j];
  idx_full[n] = G1;
  idx_full[n + 1] = H;
  // Cx = x.commit(blind_x, gens_n)
  std::vector<Pt> pts;
  {
    FqV s(x);
    s.push_back(fq_zero());
    s.push_back(blind_x);
    int rc = device_msm_idx(ctx, g, {s}, {idx_full}, &pts);
    if (rc) return rc;
  }
  Pt Cx = pts[0];
  t.point("Cx", Cx);
  Pt Cy = compress(commit_host(g, g.gens_1, {y}, blind_y));
  t.point("Cy", Cy);
  t.scalars("a", a);
  Fq r = t.challenge("r");
  Fq blind_fin = fq_add(blind_x, fq_mul(r, blind_y));
  FqV aa(x), bb(a), cw(n, fq_one());
  size_t nk = n, k = 0;
  while (nk != 1) {
    size_t nh = nk / 2;
    Fq cL = dot(aa, bb, 0, nh, nh), cR = dot(aa, bb, nh, 0, nh);
    Fq blind_L = v1[k], blind_R = v2[k];
    FqV sL(n + 2, fq_zero()), sR(n + 2, fq_zero());
    for (size_t j = 0; j < n; j++) {
      size_t m = j % nk;
      if (m >= nh) sL[j] = fq_mul(aa[m - nh], cw[j]);
      else sR[j] = fq_mul(aa[m + nh], cw[j]);
    }
    sL[n] = fq_mul(cL, r);
    sL[n + 1] = blind_L;
    sR[n] = fq_mul(cR, r);
    sR[n + 1] = blind_R;
    int rc = device_msm_idx(ctx, g, {sL, sR}, {idx_full, idx_full}, &pts);
    if (rc) return rc;
    t.point("L", pts[0]);
    t.point("R", pts[1]);
    Fq u = t.challenge("u");
    Fq uinv = fq_inv(u);
    for (size_t i = 0; i < nh; i++) {
      aa[i] = fq_add(fq_mul(aa[i], u), fq_mul(uinv, aa[i + nh]));
      bb[i] = fq_add(fq_mul(bb[i], uinv), fq_mul(u, bb[i + nh]));
    }
    for (size_t j = 0; j < n; j++) cw[j] = fq_mul(cw[j], (j % nk) < nh ? uinv : u);
    blind_fin = fq_add(fq_add(blind_fin, fq_mul(fq_mul(blind_L, u), u)), fq_mul(fq_mul(blind_R, uinv), uinv));
    out->L.push_back(pts[0]);
    out->R.push_back(pts[1]);
    nk = nh;
    k++;
  }
  // x_hat = folded x (secret), a_hat = folded a (public), as BulletReductionProof::prove returns them
  Fq x_hat = aa[0], a_hat = bb[0];
  Fq y_hat = fq_mul(x_hat, a_hat);
  // delta = d * g_hat + r_delta * h with g_hat = sum_j cw[j] G_j
  {
    FqV s(n + 2, fq_zero());
    for (size_t j = 0; j < n; j++) s[j] = fq_mul(d, cw[j]);
    s[n + 1] = r_delta;
    int rc = device_msm_idx(ctx, g, {s}, {idx_full}, &pts);
    if (rc) return rc;
  }
  out->delta = pts[0];
  t.point("delta", out->delta);
  out->beta = compress(g.host.msm({G1, H}, {fq_mul(d, r), r_beta}));
  t.point("beta", out->beta);
  Fq c = t.challenge("c");
  out->z1 = fq_add(d, fq_mul(c, y_hat));
  out->z2 = fq_add(fq_mul(a_hat, fq_add(fq_mul(c, blind_fin), r_beta)), r_delta);
  if (Cy_out) *Cy_out = Cy;
  return 0;
}

}  // namespace spg
