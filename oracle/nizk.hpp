// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of
//   src/nizk/mod.rs:16-75     KnowledgeProof::{prove, verify}
//   src/nizk/mod.rs:78-143    EqualityProof::{prove, verify}
//   src/nizk/mod.rs:146-289   ProductProof::{prove, verify}
//   src/nizk/mod.rs:292-404   DotProductProof::{prove, verify}
//   src/nizk/mod.rs:407-418   DotProductProofGens::new
//   src/nizk/mod.rs:420-576   DotProductProofLog::{prove, verify}
//   src/nizk/bullet.rs:32-243 BulletReductionProof::{prove, verify}, inner_product
//   src/dense_mlpoly.rs:26-37 PolyCommitmentGens::new
// plus the bincode 1.x encoding of these structs (serde derive order; Vec = u64 LE length + items;
// Scalar = its four Montgomery u64 limbs; CompressedRistretto = 32 raw bytes; fixed arrays unprefixed).
#pragma once
#include <cstring>
#include <string>
#include <vector>

#include "msm.hpp"
#include "poly.hpp"

namespace orc {

struct CPt {
  uint8_t v[32];
  bool operator==(const CPt& o) const { return memcmp(v, o.v, 32) == 0; }
};
static inline CPt cpt(const Ge& g) { CPt c; ge_compress(g, c.v); return c; }
static inline Ge unpack(const CPt& c) {
  Ge g;
  if (!ge_decompress(c.v, &g)) throw std::string("DecompressionError");
  return g;
}

// ---- bincode writer ----
struct Ser {
  std::vector<uint8_t> b;
  void u64(uint64_t x) { for (int i = 0; i < 8; i++) b.push_back((uint8_t)(x >> (8 * i))); }
  void sc(const Fq& s) { for (int i = 0; i < 4; i++) u64(s.v[i]); }
  void pt(const CPt& p) { b.insert(b.end(), p.v, p.v + 32); }
  void scs(const FqVec& v) { u64(v.size()); for (auto& s : v) sc(s); }
  void pts(const std::vector<CPt>& v) { u64(v.size()); for (auto& p : v) pt(p); }
};

// ---- commitments (src/commitments.rs:69-92) ----
static inline Ge msm_pts(const FqVec& s, const std::vector<Ge>& P) { return vartime_msm(s.data(), P.data(), s.size()); }
// Scalar::commit : gens.n must be 1
static inline Ge commit1(const Fq& x, const Fq& blind, const Gens& g) { return commit_scalar(x, blind, g); }
// [Scalar]::commit : first len generators + blind*h
static inline Ge commitv(const FqVec& x, const Fq& blind, const Gens& g) {
  FqVec s(x);
  s.push_back(blind);
  std::vector<Ge> P(g.G.begin(), g.G.begin() + x.size());
  P.push_back(g.h);
  return msm_pts(s, P);
}
static inline Gens gens_scale(const Gens& g, const Fq& s) {
  Gens r = g;
  uint8_t k[32];
  fq_to_bytes(s, k);
  for (auto& p : r.G) p = ge_scalarmul_bytes(p, k);
  return r;
}

// DotProductProofGens::new(n, label) = MultiCommitGens::new(n+1, label).split_at(n)
struct DotGens {
  size_t n;
  Gens gens_n, gens_1;
};
static inline DotGens dot_gens_new(size_t n, const char* label) {
  Gens all = gens_new(n + 1, label);
  DotGens d;
  d.n = n;
  d.gens_n.n = n;
  d.gens_n.G.assign(all.G.begin(), all.G.begin() + n);
  d.gens_n.h = all.h;
  d.gens_1.n = 1;
  d.gens_1.G.assign(all.G.begin() + n, all.G.end());
  d.gens_1.h = all.h;
  return d;
}
// PolyCommitmentGens::new(num_vars, label)
static inline DotGens poly_commit_gens_new(size_t num_vars, const char* label) {
  size_t l, r;
  eq_factored_lens(num_vars, &l, &r);
  return dot_gens_new(pow2(r), label);
}

// ---------------------------------------------------------------- KnowledgeProof
struct KnowledgeProof {
  CPt alpha;
  Fq z1, z2;
  void ser(Ser& s) const { s.pt(alpha); s.sc(z1); s.sc(z2); }
  static KnowledgeProof prove(const Gens& g, Transcript& t, RandomTape& tape, const Fq& x, const Fq& r, CPt* C) {
    t.append_protocol_name("knowledge proof");
    Fq t1 = tape.random_scalar("t1"), t2 = tape.random_scalar("t2");
    *C = cpt(commit1(x, r, g));
    t.append_point("C", C->v);
    KnowledgeProof p;
    p.alpha = cpt(commit1(t1, t2, g));
    t.append_point("alpha", p.alpha.v);
    Fq c = t.challenge_scalar("c");
    p.z1 = fq_add(fq_mul(x, c), t1);
    p.z2 = fq_add(fq_mul(r, c), t2);
    return p;
  }
  bool verify(const Gens& g, Transcript& t, const CPt& C) const {
    t.append_protocol_name("knowledge proof");
    t.append_point("C", C.v);
    t.append_point("alpha", alpha.v);
    Fq c = t.challenge_scalar("c");
    uint8_t cb[32];
    fq_to_bytes(c, cb);
    CPt lhs = cpt(commit1(z1, z2, g));
    CPt rhs = cpt(ge_add(ge_scalarmul_bytes(unpack(C), cb), unpack(alpha)));
    return lhs == rhs;
  }
};

// ---------------------------------------------------------------- EqualityProof
struct EqualityProof {
  CPt alpha;
  Fq z;
  void ser(Ser& s) const { s.pt(alpha); s.sc(z); }
  static EqualityProof prove(const Gens& g, Transcript& t, RandomTape& tape, const Fq& v1, const Fq& s1, const Fq& v2,
                             const Fq& s2, CPt* C1, CPt* C2) {
    t.append_protocol_name("equality proof");
    Fq r = tape.random_scalar("r");
    *C1 = cpt(commit1(v1, s1, g));
    t.append_point("C1", C1->v);
    *C2 = cpt(commit1(v2, s2, g));
    t.append_point("C2", C2->v);
    EqualityProof p;
    uint8_t rb[32];
    fq_to_bytes(r, rb);
    p.alpha = cpt(ge_scalarmul_bytes(g.h, rb));
    t.append_point("alpha", p.alpha.v);
    Fq c = t.challenge_scalar("c");
    p.z = fq_add(fq_mul(c, fq_sub(s1, s2)), r);
    return p;
  }
  bool verify(const Gens& g, Transcript& t, const CPt& C1, const CPt& C2) const {
    t.append_protocol_name("equality proof");
    t.append_point("C1", C1.v);
    t.append_point("C2", C2.v);
    t.append_point("alpha", alpha.v);
    Fq c = t.challenge_scalar("c");
    uint8_t cb[32], zb[32];
    fq_to_bytes(c, cb);
    fq_to_bytes(z, zb);
    Ge C = ge_sub(unpack(C1), unpack(C2));
    CPt rhs = cpt(ge_add(ge_scalarmul_bytes(C, cb), unpack(alpha)));
    CPt lhs = cpt(ge_scalarmul_bytes(g.h, zb));
    return lhs == rhs;
  }
};

// ---------------------------------------------------------------- ProductProof
struct ProductProof {
  CPt alpha, beta, delta;
  Fq z[5];
  void ser(Ser& s) const {
    s.pt(alpha); s.pt(beta); s.pt(delta);
    for (int i = 0; i < 5; i++) s.sc(z[i]);
  }
  static ProductProof prove(const Gens& g, Transcript& t, RandomTape& tape, const Fq& x, const Fq& rX, const Fq& y,
                            const Fq& rY, const Fq& zz, const Fq& rZ, CPt* X, CPt* Y, CPt* Z) {
    t.append_protocol_name("product proof");
    Fq b1 = tape.random_scalar("b1"), b2 = tape.random_scalar("b2"), b3 = tape.random_scalar("b3"),
       b4 = tape.random_scalar("b4"), b5 = tape.random_scalar("b5");
    *X = cpt(commit1(x, rX, g)); t.append_point("X", X->v);
    *Y = cpt(commit1(y, rY, g)); t.append_point("Y", Y->v);
    *Z = cpt(commit1(zz, rZ, g)); t.append_point("Z", Z->v);
    ProductProof p;
    p.alpha = cpt(commit1(b1, b2, g)); t.append_point("alpha", p.alpha.v);
    p.beta = cpt(commit1(b3, b4, g)); t.append_point("beta", p.beta.v);
    Gens gX;
    gX.n = 1;
    gX.G = {unpack(*X)};
    gX.h = g.h;
    p.delta = cpt(commit1(b3, b5, gX)); t.append_point("delta", p.delta.v);
    Fq c = t.challenge_scalar("c");
    p.z[0] = fq_add(b1, fq_mul(c, x));
    p.z[1] = fq_add(b2, fq_mul(c, rX));
    p.z[2] = fq_add(b3, fq_mul(c, y));
    p.z[3] = fq_add(b4, fq_mul(c, rY));
    p.z[4] = fq_add(b5, fq_mul(c, fq_sub(rZ, fq_mul(rX, y))));
    return p;
  }
  static bool check_eq(const CPt& P, const CPt& X, const Fq& c, const Gens& g, const Fq& z1, const Fq& z2) {
    uint8_t cb[32];
    fq_to_bytes(c, cb);
    CPt lhs = cpt(ge_add(unpack(P), ge_scalarmul_bytes(unpack(X), cb)));
    return lhs == cpt(commit1(z1, z2, g));
  }
  bool verify(const Gens& g, Transcript& t, const CPt& X, const CPt& Y, const CPt& Z) const {
    t.append_protocol_name("product proof");
    t.append_point("X", X.v); t.append_point("Y", Y.v); t.append_point("Z", Z.v);
    t.append_point("alpha", alpha.v); t.append_point("beta", beta.v); t.append_point("delta", delta.v);
    Fq c = t.challenge_scalar("c");
    Gens gX;
    gX.n = 1;
    gX.G = {unpack(X)};
    gX.h = g.h;
    return check_eq(alpha, X, c, g, z[0], z[1]) && check_eq(beta, Y, c, g, z[2], z[3]) &&
           check_eq(delta, Z, c, gX, z[2], z[4]);
  }
};

// ---------------------------------------------------------------- DotProductProof
struct DotProductProof {
  CPt delta, beta;
  FqVec z;
  Fq z_delta, z_beta;
  void ser(Ser& s) const { s.pt(delta); s.pt(beta); s.scs(z); s.sc(z_delta); s.sc(z_beta); }
  static DotProductProof prove(const Gens& g1, const Gens& gn, Transcript& t, RandomTape& tape, const FqVec& x,
                               const Fq& blind_x, const FqVec& a, const Fq& y, const Fq& blind_y, CPt* Cx, CPt* Cy) {
    t.append_protocol_name("dot product proof");
    size_t n = x.size();
    FqVec d = tape.random_vector("d_vec", n);
    Fq r_delta = tape.random_scalar("r_delta"), r_beta = tape.random_scalar("r_beta");
    *Cx = cpt(commitv(x, blind_x, gn)); t.append_point("Cx", Cx->v);
    *Cy = cpt(commit1(y, blind_y, g1)); t.append_point("Cy", Cy->v);
    t.append_scalars("a", a);
    DotProductProof p;
    p.delta = cpt(commitv(d, r_delta, gn)); t.append_point("delta", p.delta.v);
    Fq ad = dot(a, d);
    p.beta = cpt(commit1(ad, r_beta, g1)); t.append_point("beta", p.beta.v);
    Fq c = t.challenge_scalar("c");
    p.z.resize(n);
    for (size_t i = 0; i < n; i++) p.z[i] = fq_add(fq_mul(c, x[i]), d[i]);
    p.z_delta = fq_add(fq_mul(c, blind_x), r_delta);
    p.z_beta = fq_add(fq_mul(c, blind_y), r_beta);
    return p;
  }
  bool verify(const Gens& g1, const Gens& gn, Transcript& t, const FqVec& a, const CPt& Cx, const CPt& Cy) const {
    t.append_protocol_name("dot product proof");
    t.append_point("Cx", Cx.v); t.append_point("Cy", Cy.v);
    t.append_scalars("a", a);
    t.append_point("delta", delta.v); t.append_point("beta", beta.v);
    Fq c = t.challenge_scalar("c");
    uint8_t cb[32];
    fq_to_bytes(c, cb);
    bool ok = ge_eq(ge_add(ge_scalarmul_bytes(unpack(Cx), cb), unpack(delta)), commitv(z, z_delta, gn));
    Fq dz = dot(z, a);
    ok = ok && ge_eq(ge_add(ge_scalarmul_bytes(unpack(Cy), cb), unpack(beta)), commit1(dz, z_beta, g1));
    return ok;
  }
};

// ---------------------------------------------------------------- BulletReductionProof
struct BulletProof {
  std::vector<CPt> L_vec, R_vec;
  void ser(Ser& s) const { s.pts(L_vec); s.pts(R_vec); }
  static BulletProof prove(Transcript& t, const Ge& Q, std::vector<Ge> G, const Ge& H, FqVec a, FqVec b,
                           const Fq& blind, const std::vector<std::pair<Fq, Fq>>& blinds, Ge* Gamma_hat, Fq* a0,
                           Fq* b0, Ge* g0, Fq* blind_fin_out) {
    size_t n = G.size();
    BulletProof p;
    Fq blind_fin = blind;
    size_t bi = 0;
    while (n != 1) {
      n /= 2;
      FqVec aL(a.begin(), a.begin() + n), aR(a.begin() + n, a.begin() + 2 * n);
      FqVec bL(b.begin(), b.begin() + n), bR(b.begin() + n, b.begin() + 2 * n);
      std::vector<Ge> GL(G.begin(), G.begin() + n), GR(G.begin() + n, G.begin() + 2 * n);
      Fq cL = dot(aL, bR), cR = dot(aR, bL);
      Fq blind_L = blinds[bi].first, blind_R = blinds[bi].second;
      bi++;
      FqVec sL(aL);
      sL.push_back(cL); sL.push_back(blind_L);
      std::vector<Ge> PL(GR);
      PL.push_back(Q); PL.push_back(H);
      FqVec sR(aR);
      sR.push_back(cR); sR.push_back(blind_R);
      std::vector<Ge> PR(GL);
      PR.push_back(Q); PR.push_back(H);
      CPt L = cpt(msm_pts(sL, PL)), R = cpt(msm_pts(sR, PR));
      t.append_point("L", L.v);
      t.append_point("R", R.v);
      Fq u = t.challenge_scalar("u");
      Fq u_inv = fq_invert(u);
      for (size_t i = 0; i < n; i++) {
        aL[i] = fq_add(fq_mul(aL[i], u), fq_mul(u_inv, aR[i]));
        bL[i] = fq_add(fq_mul(bL[i], u_inv), fq_mul(u, bR[i]));
        FqVec s2 = {u_inv, u};
        std::vector<Ge> p2 = {GL[i], GR[i]};
        GL[i] = msm_pts(s2, p2);
      }
      blind_fin = fq_add(fq_add(blind_fin, fq_mul(fq_mul(blind_L, u), u)), fq_mul(fq_mul(blind_R, u_inv), u_inv));
      p.L_vec.push_back(L);
      p.R_vec.push_back(R);
      a = aL; b = bL; G = GL;
    }
    FqVec s3 = {a[0], fq_mul(a[0], b[0]), blind_fin};
    std::vector<Ge> p3 = {G[0], Q, H};
    *Gamma_hat = msm_pts(s3, p3);
    *a0 = a[0];
    *b0 = b[0];
    *g0 = G[0];
    *blind_fin_out = blind_fin;
    return p;
  }
  // bullet.rs:138-232
  bool verify(size_t n, const FqVec& a, Transcript& t, const Ge& Gamma, const std::vector<Ge>& G, Ge* G_hat,
              Ge* Gamma_hat, Fq* a_hat) const {
    size_t lg_n = L_vec.size();
    if (lg_n >= 32 || n != ((size_t)1 << lg_n)) return false;
    FqVec ch;
    for (size_t i = 0; i < lg_n; i++) {
      t.append_point("L", L_vec[i].v);
      t.append_point("R", R_vec[i].v);
      ch.push_back(t.challenge_scalar("u"));
    }
    FqVec chinv = ch;
    Fq allinv = fq_batch_invert(chinv);
    FqVec sq(lg_n), isq(lg_n);
    for (size_t i = 0; i < lg_n; i++) { sq[i] = fq_square(ch[i]); isq[i] = fq_square(chinv[i]); }
    FqVec s;
    s.push_back(allinv);
    for (size_t i = 1; i < n; i++) {
      size_t lg_i = 0;
      while (((size_t)2 << lg_i) <= i) lg_i++;
      size_t k = (size_t)1 << lg_i;
      s.push_back(fq_mul(s[i - k], sq[(lg_n - 1) - lg_i]));
    }
    *G_hat = msm_pts(s, G);
    *a_hat = dot(a, s);
    FqVec sc(sq);
    sc.insert(sc.end(), isq.begin(), isq.end());
    sc.push_back(fq_one());
    std::vector<Ge> P;
    for (auto& l : L_vec) P.push_back(unpack(l));
    for (auto& r : R_vec) P.push_back(unpack(r));
    P.push_back(Gamma);
    *Gamma_hat = msm_pts(sc, P);
    return true;
  }
};

// ---------------------------------------------------------------- DotProductProofLog
struct DotProductProofLog {
  BulletProof bullet;
  CPt delta, beta;
  Fq z1, z2;
  void ser(Ser& s) const { bullet.ser(s); s.pt(delta); s.pt(beta); s.sc(z1); s.sc(z2); }
  static DotProductProofLog prove(const DotGens& g, Transcript& t, RandomTape& tape, const FqVec& x,
                                  const Fq& blind_x, const FqVec& a, const Fq& y, const Fq& blind_y, CPt* Cx, CPt* Cy) {
    t.append_protocol_name("dot product proof (log)");
    size_t n = x.size();
    Fq d = tape.random_scalar("d");
    Fq r_delta = tape.random_scalar("r_delta");
    Fq r_beta = tape.random_scalar("r_delta");
    size_t lg = log_2(n);
    FqVec v1 = tape.random_vector("blinds_vec_1", 2 * lg);
    FqVec v2 = tape.random_vector("blinds_vec_2", 2 * lg);
    std::vector<std::pair<Fq, Fq>> blinds;
    for (size_t i = 0; i < v1.size(); i++) blinds.push_back({v1[i], v2[i]});
    *Cx = cpt(commitv(x, blind_x, g.gens_n)); t.append_point("Cx", Cx->v);
    *Cy = cpt(commit1(y, blind_y, g.gens_1)); t.append_point("Cy", Cy->v);
    t.append_scalars("a", a);
    Fq r = t.challenge_scalar("r");
    Gens g1s = gens_scale(g.gens_1, r);
    Fq blind_Gamma = fq_add(blind_x, fq_mul(r, blind_y));
    Ge Gamma_hat, g_hat;
    Fq x_hat, a_hat, rhat;
    std::vector<Ge> Gn(g.gens_n.G.begin(), g.gens_n.G.begin() + n);
    DotProductProofLog p;
    p.bullet = BulletProof::prove(t, g1s.G[0], Gn, g.gens_n.h, x, a, blind_Gamma, blinds, &Gamma_hat, &x_hat, &a_hat,
                                  &g_hat, &rhat);
    Fq y_hat = fq_mul(x_hat, a_hat);
    Gens ghat;
    ghat.n = 1;
    ghat.G = {g_hat};
    ghat.h = g.gens_1.h;
    p.delta = cpt(commit1(d, r_delta, ghat)); t.append_point("delta", p.delta.v);
    p.beta = cpt(commit1(d, r_beta, g1s)); t.append_point("beta", p.beta.v);
    Fq c = t.challenge_scalar("c");
    p.z1 = fq_add(d, fq_mul(c, y_hat));
    p.z2 = fq_add(fq_mul(a_hat, fq_add(fq_mul(c, rhat), r_beta)), r_delta);
    return p;
  }
  bool verify(size_t n, const DotGens& g, Transcript& t, const FqVec& a, const CPt& Cx, const CPt& Cy) const {
    t.append_protocol_name("dot product proof (log)");
    t.append_point("Cx", Cx.v); t.append_point("Cy", Cy.v);
    t.append_scalars("a", a);
    Fq r = t.challenge_scalar("r");
    Gens g1s = gens_scale(g.gens_1, r);
    uint8_t rb[32];
    fq_to_bytes(r, rb);
    Ge Gamma = ge_add(unpack(Cx), ge_scalarmul_bytes(unpack(Cy), rb));
    Ge g_hat, Gamma_hat;
    Fq a_hat;
    std::vector<Ge> Gn(g.gens_n.G.begin(), g.gens_n.G.begin() + n);
    if (!bullet.verify(n, a, t, Gamma, Gn, &g_hat, &Gamma_hat, &a_hat)) return false;
    t.append_point("delta", delta.v); t.append_point("beta", beta.v);
    Fq c = t.challenge_scalar("c");
    uint8_t cb[32], ab[32], z1b[32], z2b[32];
    fq_to_bytes(c, cb); fq_to_bytes(a_hat, ab); fq_to_bytes(z1, z1b); fq_to_bytes(z2, z2b);
    Ge lhs = ge_add(ge_scalarmul_bytes(ge_add(ge_scalarmul_bytes(Gamma_hat, cb), unpack(beta)), ab), unpack(delta));
    Ge rhs = ge_add(ge_scalarmul_bytes(ge_add(g_hat, ge_scalarmul_bytes(g1s.G[0], ab)), z1b),
                    ge_scalarmul_bytes(g1s.h, z2b));
    return cpt(lhs) == cpt(rhs);
  }
};

}  // namespace orc
