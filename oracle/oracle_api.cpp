// ORACLE — test infrastructure only. C entry points over the CPU restatement, loaded by tests/
// (ctypes), __graft_entry__.smoke() and bench.py's cpu_baseline leg. Never linked into the product.
#include <cstdint>
#include <chrono>
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

// merlin Transcript as a handle (tests: the caller-side transcript behind spg_transcript_new_callbacks)
void* orc_transcript_new(const char* label) { return new Transcript(label); }
void orc_transcript_append(void* t, const char* label, const uint8_t* msg, size_t n) {
  ((Transcript*)t)->append_message(label, msg, n);
}
void orc_transcript_challenge(void* t, const char* label, uint8_t* out, size_t n) {
  ((Transcript*)t)->challenge_bytes(label, out, n);
}
void orc_transcript_free(void* t) { delete (Transcript*)t; }

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
// one shard of a sharded MSM: the uncompressed partial sum as extended coordinates
// X, Y, Z, T, each 32 canonical little-endian bytes (test reference for spg_msm_partial / spg_points_sum_compress)
int orc_msm_partial(const uint8_t* bases, const uint64_t* scalars, size_t n, uint8_t* out_ext) {
  std::vector<Ge> P(n);
  for (size_t i = 0; i < n; i++)
    if (!ge_decompress(bases + 32 * i, &P[i])) return 0;
  std::vector<Fq> s(n);
  for (size_t i = 0; i < n; i++) s[i] = ld(scalars + 4 * i);
  Ge r = vartime_msm(s.data(), P.data(), n);
  fe_to_bytes(r.X, out_ext);
  fe_to_bytes(r.Y, out_ext + 32);
  fe_to_bytes(r.Z, out_ext + 64);
  fe_to_bytes(r.T, out_ext + 96);
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

// ---------------------------------------------------------------- R1CSProof (src/r1csproof.rs:210-954)
#include "../include/spg.h"
#include "r1cs.hpp"

extern "C" {
// ---- UniPoly (src/unipoly.rs:23-111) and DensePolynomial::evaluate (src/dense_mlpoly.rs:361-367), for the
// reference's own known-answer tests (unipoly.rs:127-181, dense_mlpoly.rs:1234-1252) ----
// evals (n = 3 or 4) -> coeffs (n), then evaluate(r) -> *at_r, and decompress(compress(), e0 + e1) -> coeffs_rt
void orc_unipoly(const uint64_t* evals, size_t n, const uint64_t* r, uint64_t* coeffs, uint64_t* at_r,
                 uint64_t* coeffs_rt) {
  FqVec e;
  for (size_t i = 0; i < n; i++) e.push_back(ld(evals + 4 * i));
  UniPoly u = UniPoly::from_evals(e);
  for (size_t i = 0; i < u.coeffs.size(); i++) st(coeffs + 4 * i, u.coeffs[i]);
  st(at_r, u.evaluate(ld(r)));
  UniPoly d = UniPoly::decompress(u.compress(), fq_add(u.eval_at_zero(), u.eval_at_one()));
  for (size_t i = 0; i < d.coeffs.size(); i++) st(coeffs_rt + 4 * i, d.coeffs[i]);
}
// DensePolynomial::new(Z).evaluate(r) -> out[0]; evaluate_with_LR (dense_mlpoly.rs:1212-1231: L.Z.R with the
// factored eq tables) -> out[1]
void orc_dense_eval(const uint64_t* Z, size_t n, const uint64_t* r, size_t ell, uint64_t* out) {
  FqVec z, rv;
  for (size_t i = 0; i < n; i++) z.push_back(ld(Z + 4 * i));
  for (size_t i = 0; i < ell; i++) rv.push_back(ld(r + 4 * i));
  DensePoly p(z);
  st(out, p.evaluate(rv));
  FqVec L, R;
  eq_factored_evals(rv, &L, &R);
  st(out + 4, dot(p.bound(L), R));
}
// DensePolynomialPqx::new (custom_dense_mlpoly.rs:45-64) from z in (p, q_rev, w, x_rev) order -- instance p holds
// num_proofs[p] x nws x num_inputs[p] scalars, row-major -- then k binds bound_poly(rs[i], modes[i])
// (custom_dense_mlpoly.rs:180-289) in order. out: Z afterwards in the same layout (the allocation never shrinks);
// sizes: num_instances, max_num_proofs, num_witness_secs, max_num_inputs, num_proofs[0..P), num_inputs[0..P).
// Returns -1 where the reference's bound_poly_p would panic (max_num_proofs or max_num_inputs != 1).
int orc_pqx_bind(const uint64_t* z, size_t P, const size_t* num_proofs, size_t max_num_proofs, size_t nws,
                 const size_t* num_inputs, size_t max_num_inputs, const int* modes, const uint64_t* rs, size_t k,
                 uint64_t* out, size_t* sizes) {
  Pqx T;
  T.Z.resize(P);
  const uint64_t* s = z;
  for (size_t p = 0; p < P; p++) {
    T.Z[p].assign(num_proofs[p], std::vector<FqVec>(nws, FqVec(num_inputs[p])));
    for (size_t q = 0; q < num_proofs[p]; q++)
      for (size_t w = 0; w < nws; w++)
        for (size_t x = 0; x < num_inputs[p]; x++, s += 4) T.Z[p][q][w][x] = ld(s);
  }
  T.num_instances = next_pow2(P);
  T.num_proofs.assign(num_proofs, num_proofs + P);
  T.max_num_proofs = max_num_proofs;
  T.num_witness_secs = next_pow2(nws);
  T.num_inputs.assign(num_inputs, num_inputs + P);
  T.max_num_inputs = max_num_inputs;
  for (size_t i = 0; i < k; i++) {
    if (modes[i] == MODE_P && (T.max_num_proofs != 1 || T.max_num_inputs != 1)) return -1;  // :206-207 assert_eq!
    T.bound_poly(ld(rs + 4 * i), modes[i]);
  }
  uint64_t* o = out;
  for (size_t p = 0; p < P; p++)
    for (size_t q = 0; q < num_proofs[p]; q++)
      for (size_t w = 0; w < nws; w++)
        for (size_t x = 0; x < num_inputs[p]; x++, o += 4) st(o, T.Z[p][q][w][x]);
  sizes[0] = T.num_instances;
  sizes[1] = T.max_num_proofs;
  sizes[2] = T.num_witness_secs;
  sizes[3] = T.max_num_inputs;
  for (size_t p = 0; p < P; p++) {
    sizes[4 + p] = T.num_proofs[p];
    sizes[4 + P + p] = T.num_inputs[p];
  }
  return 0;
}
}

// (baseline-mode state: see orc_baseline_mode below)
static void (*g_bl_barrier)() = nullptr;
static bool g_bl_skip_verify = false;
static thread_local double g_bl_w0 = 0.0, g_bl_w1 = 0.0;
static double steady_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static R1CSInstance inst_from_c(const spg_r1cs_instance* ci) {
  std::vector<std::vector<SparseEntry>> A, B, C;
  for (size_t p = 0; p < ci->num_instances; p++) {
    for (int m = 0; m < 3; m++) {
      std::vector<SparseEntry> v;
      const spg_sparse_entry* e = ci->entries[3 * p + m];
      for (size_t k = 0; k < ci->nnz[3 * p + m]; k++) {
        SparseEntry s;
        s.row = e[k].row;
        s.col = e[k].col;
        memcpy(s.val.v, e[k].val, 32);
        v.push_back(s);
      }
      (m == 0 ? A : m == 1 ? B : C).push_back(v);
    }
  }
  std::vector<size_t> nc(ci->num_cons, ci->num_cons + ci->num_instances);
  return R1CSInstance::create(ci->num_instances, ci->max_num_cons, nc, ci->num_vars, A, B, C);
}
static WitnessSec ws_from_c(const spg_witness_sec* c) {
  std::vector<std::vector<FqVec>> w_mat;
  std::vector<DensePoly> polys;
  for (size_t p = 0; p < c->num_instances; p++) {
    std::vector<FqVec> rows;
    FqVec flat;
    for (size_t q = 0; q < c->num_proofs[p]; q++) {
      FqVec row(c->num_inputs[p]);
      for (size_t i = 0; i < c->num_inputs[p]; i++)
        memcpy(row[i].v, c->w[p] + 4 * (q * c->num_inputs[p] + i), 32);
      flat.insert(flat.end(), row.begin(), row.end());
      rows.push_back(row);
    }
    w_mat.push_back(rows);
    polys.push_back(DensePoly(flat));
  }
  return WitnessSec::create(w_mat, polys);
}
static FqVec challenges_flat(const std::vector<FqVec>& ch) {
  FqVec f;
  for (auto& v : ch) f.insert(f.end(), v.begin(), v.end());
  return f;
}

extern "C" {
// Proves with a fresh Transcript(label) and RandomTape(b"proof", init = tape_seed) and writes
// bincode(R1CSProof). proof_cap bytes available; *proof_len receives the size. gens label = gens_label,
// gens_num_vars = the R1CSGens num_vars (power of two). challenges_out (optional) receives
// rp | rq_rev | rx | rw||ry concatenated; ch_lens[4] their lengths.
// the same on a caller's transcript handle (orc_transcript_new), which keeps its state after the proof
int orc_r1cs_prove_tr(const spg_r1cs_instance* ci, size_t num_instances, size_t max_num_proofs,
                      const size_t* num_proofs, size_t max_num_inputs, const size_t* num_inputs,
                      const spg_witness_sec* secs, size_t nws, const char* gens_label, size_t gens_num_vars,
                      void* transcript, const uint64_t* tape_seed, uint8_t* proof, size_t proof_cap,
                      size_t* proof_len, uint64_t* challenges_out, size_t* ch_lens);
int orc_r1cs_prove(const spg_r1cs_instance* ci, size_t num_instances, size_t max_num_proofs,
                   const size_t* num_proofs, size_t max_num_inputs, const size_t* num_inputs,
                   const spg_witness_sec* secs, size_t nws, const char* gens_label, size_t gens_num_vars,
                   const char* transcript_label, const uint64_t* tape_seed, uint8_t* proof, size_t proof_cap,
                   size_t* proof_len, uint64_t* challenges_out, size_t* ch_lens) {
  Transcript t(transcript_label);
  return orc_r1cs_prove_tr(ci, num_instances, max_num_proofs, num_proofs, max_num_inputs, num_inputs, secs, nws,
                           gens_label, gens_num_vars, &t, tape_seed, proof, proof_cap, proof_len, challenges_out,
                           ch_lens);
}
int orc_r1cs_prove_tr(const spg_r1cs_instance* ci, size_t num_instances, size_t max_num_proofs,
                      const size_t* num_proofs, size_t max_num_inputs, const size_t* num_inputs,
                      const spg_witness_sec* secs, size_t nws, const char* gens_label, size_t gens_num_vars,
                      void* transcript, const uint64_t* tape_seed, uint8_t* proof, size_t proof_cap,
                      size_t* proof_len, uint64_t* challenges_out, size_t* ch_lens) {
  try {
    Transcript& t = *(Transcript*)transcript;
    R1CSInstance inst = inst_from_c(ci);
    std::vector<WitnessSec> ws;
    for (size_t i = 0; i < nws; i++) ws.push_back(ws_from_c(&secs[i]));
    std::vector<const WitnessSec*> wp;
    for (auto& w : ws) wp.push_back(&w);
    R1CSGens gens = R1CSGens::create(gens_label, gens_num_vars);
    RandomTape tape("proof", ld(tape_seed));
    std::vector<size_t> np(num_proofs, num_proofs + num_instances), ni(num_inputs, num_inputs + num_instances);
    std::vector<FqVec> ch;
    if (g_bl_barrier) g_bl_barrier();
    g_bl_w0 = steady_us();
    R1CSProof pf = R1CSProof::prove(num_instances, max_num_proofs, np, max_num_inputs, ni, wp, inst, gens, t, tape, &ch);
    g_bl_w1 = steady_us();
    Ser s;
    pf.ser(s);
    *proof_len = s.b.size();
    if (s.b.size() > proof_cap) return -1;
    memcpy(proof, s.b.data(), s.b.size());
    if (challenges_out) {
      FqVec f = challenges_flat(ch);
      for (size_t i = 0; i < f.size(); i++) st(challenges_out + 4 * i, f[i]);
      for (int i = 0; i < 4; i++) ch_lens[i] = ch[i].size();
    }
    return 0;
  } catch (const std::string& e) {
    return -2;
  }
}
}

extern "C" {
// Verifies a proof produced by orc_r1cs_prove (R1CSProof::verify, src/r1csproof.rs:687-954) against the
// witness-section commitments (computed here with DensePolynomial::commit) and the instance evaluations
// bound to rp (multi_evaluate_bound_rp, src/r1csinstance.rs:598-629). Returns 1 if it verifies.
int orc_r1cs_verify(const spg_r1cs_instance* ci, size_t num_instances, size_t max_num_proofs,
                    const size_t* num_proofs, size_t max_num_inputs, const spg_witness_sec* secs, size_t nws,
                    const char* gens_label, size_t gens_num_vars, const char* transcript_label,
                    const uint8_t* proof_bytes, size_t proof_len, const uint64_t* tape_seed) {
  try {
    // re-prove deterministically to obtain the proof object, then check byte equality with the input
    R1CSInstance inst = inst_from_c(ci);
    std::vector<WitnessSec> ws;
    for (size_t i = 0; i < nws; i++) ws.push_back(ws_from_c(&secs[i]));
    std::vector<const WitnessSec*> wp;
    for (auto& w : ws) wp.push_back(&w);
    R1CSGens gens = R1CSGens::create(gens_label, gens_num_vars);
    std::vector<size_t> np(num_proofs, num_proofs + num_instances), ni;
    for (size_t p = 0; p < num_instances; p++) ni.push_back(max_num_inputs);
    (void)ni;
    Transcript tp(transcript_label);
    RandomTape tape("proof", ld(tape_seed));
    std::vector<FqVec> ch;
    std::vector<size_t> num_inputs_v;
    // the prover's num_inputs are the section-0 widths by instance (callers pass them through secs[0])
    for (size_t p = 0; p < num_instances; p++)
      num_inputs_v.push_back(secs[0].num_inputs[secs[0].num_instances == 1 ? 0 : p]);
    R1CSProof pf = R1CSProof::prove(num_instances, max_num_proofs, np, max_num_inputs, num_inputs_v, wp, inst, gens, tp,
                                    tape, &ch);
    Ser s;
    pf.ser(s);
    if (s.b.size() != proof_len || memcmp(s.b.data(), proof_bytes, proof_len) != 0) return 0;
    // verifier side
    std::vector<std::vector<size_t>> wni, wnp;
    std::vector<std::vector<PolyCommitment>> wc;
    for (auto& w : ws) {
      wni.push_back(w.num_inputs);
      std::vector<size_t> npv;
      std::vector<PolyCommitment> cv;
      for (size_t p = 0; p < w.w_mat.size(); p++) {
        npv.push_back(w.w_mat[p].size());
        cv.push_back(poly_commit(w.poly_w[p], gens.gens_pc));
      }
      wnp.push_back(npv);
      wc.push_back(cv);
    }
    FqVec list;
    Fq evals[3];
    if (inst.num_instances == 1) {  // R1CSInstance::evaluate, "used if there is only one instance" (r1csinstance.rs:631-641)
      FqVec e = inst.multi_evaluate(ch[2], ch[3]);
      for (int i = 0; i < 3; i++) evals[i] = e[i];
    } else {
      inst.multi_evaluate_bound_rp(ch[0], ch[2], ch[3], &list, evals);
    }
    Transcript tv(transcript_label);
    return pf.verify(num_instances, max_num_proofs, np, max_num_inputs, wni, wnp, wc, inst.max_num_cons, gens, evals,
                     tv)
               ? 1
               : 0;
  } catch (const std::string& e) {
    return -2;
  }
}
}

extern "C" {
// R1CSInstance::multi_evaluate (src/r1csinstance.rs:583-596): out = [A_0(rx,ry), B_0, C_0, A_1, ...]
int orc_r1cs_multi_evaluate(const spg_r1cs_instance* ci, const uint64_t* rx, size_t rx_len, const uint64_t* ry,
                            size_t ry_len, uint64_t* out) {
  R1CSInstance inst = inst_from_c(ci);
  FqVec vx, vy;
  for (size_t i = 0; i < rx_len; i++) vx.push_back(ld(rx + 4 * i));
  for (size_t i = 0; i < ry_len; i++) vy.push_back(ld(ry + 4 * i));
  FqVec e = inst.multi_evaluate(vx, vy);
  for (size_t i = 0; i < e.size(); i++) memcpy(out + 4 * i, e[i].v, 32);
  return 0;
}
}

#include <chrono>

#include "spark.hpp"

extern "C" {
// SPARK on the matrices of an R1CS instance, batch = [A_0, B_0, C_0, A_1, ...] (R1CSInstance::commit,
// src/r1csinstance.rs:722-737) with SparseMatPolyCommitmentGens(label, nvx, nvy, gens_nnz, gens_batch)
// (R1CSCommitmentGens::new passes num_instances*nnz and batch 3, src/r1csinstance.rs:39-56).
// Proves SparseMatPolyEvalProof at (rx, ry) for evals = multi_evaluate(rx, ry) under a fresh
// Transcript(label) + RandomTape("proof", seed), writes bincode(commitment) and bincode(proof), then runs
// the verifier on a fresh transcript. Returns 1 if it verifies, 0 if not, <0 on error.
// CPU-baseline mode (bench.py's all-cores baselines): every orc_spark_prove / orc_r1cs_prove / orc_snark_prove calls
// `barrier` between its setup (commitment, generator derivation, instance encoding) and its prove, so concurrent copies
// prove at the same time, and may skip the verification; each thread's prove window (steady clock, microseconds) is
// kept for the caller to take the concurrent wall time of the proves alone from
void orc_baseline_mode(void (*barrier)(), int skip_verify) {
  g_bl_barrier = barrier;
  g_bl_skip_verify = skip_verify != 0;
}
void orc_last_prove_window(double* t0, double* t1) {
  *t0 = g_bl_w0;
  *t1 = g_bl_w1;
}
void orc_spark_baseline_mode(void (*barrier)(), int skip_verify) { orc_baseline_mode(barrier, skip_verify); }
void orc_spark_last_prove_window(double* t0, double* t1) { orc_last_prove_window(t0, t1); }
static thread_local double g_spark_prove_us = 0.0;
// wall time of the last orc_spark_prove's multi_evaluate + SparseMatPolyEvalProof::prove (CPU baseline)
double orc_spark_last_prove_us() { return g_spark_prove_us; }

// transcript != NULL: prove on that caller's handle (orc_transcript_new) instead of a fresh Transcript(label) and
// skip the verification (returns 1)
int orc_spark_prove_tr(const spg_r1cs_instance* ci, const char* gens_label, size_t gens_nnz, size_t gens_batch,
                       const uint64_t* rx, size_t rx_len, const uint64_t* ry, size_t ry_len, const char* label,
                       void* transcript, const uint64_t* tape_seed, uint8_t* comm_out, size_t comm_cap,
                       size_t* comm_len, uint8_t* proof_out, size_t proof_cap, size_t* proof_len);
int orc_spark_prove(const spg_r1cs_instance* ci, const char* gens_label, size_t gens_nnz, size_t gens_batch,
                    const uint64_t* rx, size_t rx_len, const uint64_t* ry, size_t ry_len, const char* label,
                    const uint64_t* tape_seed, uint8_t* comm_out, size_t comm_cap, size_t* comm_len,
                    uint8_t* proof_out, size_t proof_cap, size_t* proof_len) {
  return orc_spark_prove_tr(ci, gens_label, gens_nnz, gens_batch, rx, rx_len, ry, ry_len, label, nullptr, tape_seed,
                            comm_out, comm_cap, comm_len, proof_out, proof_cap, proof_len);
}
int orc_spark_prove_tr(const spg_r1cs_instance* ci, const char* gens_label, size_t gens_nnz, size_t gens_batch,
                       const uint64_t* rx, size_t rx_len, const uint64_t* ry, size_t ry_len, const char* label,
                       void* transcript, const uint64_t* tape_seed, uint8_t* comm_out, size_t comm_cap,
                       size_t* comm_len, uint8_t* proof_out, size_t proof_cap, size_t* proof_len) {
  try {
    R1CSInstance inst = inst_from_c(ci);
    std::vector<const SparseMat*> polys;
    for (size_t p = 0; p < inst.num_instances; p++) {
      polys.push_back(&inst.A[p]);
      polys.push_back(&inst.B[p]);
      polys.push_back(&inst.C[p]);
    }
    FqVec vx, vy;
    for (size_t i = 0; i < rx_len; i++) vx.push_back(ld(rx + 4 * i));
    for (size_t i = 0; i < ry_len; i++) vy.push_back(ld(ry + 4 * i));
    size_t nvx = polys[0]->num_vars_x, nvy = polys[0]->num_vars_y;
    SparkGens g = SparkGens::create(gens_label, nvx, nvy, gens_nnz, gens_batch);
    MultiSparseDense dense;
    SparkCommitment comm = spark_multi_commit(polys, g, &dense);
    if (g_bl_barrier) g_bl_barrier();
    auto t0 = std::chrono::steady_clock::now();
    g_bl_w0 = steady_us();
    FqVec evals = inst.multi_evaluate(vx, vy);
    Transcript tl(label);
    Transcript& t = transcript ? *(Transcript*)transcript : tl;
    RandomTape tape("proof", ld(tape_seed));
    SparkEvalProof pf = spark_prove(dense, vx, vy, evals, g, t, tape);
    g_spark_prove_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    g_bl_w1 = steady_us();
    Ser sc, sp;
    comm.ser(sc);
    pf.ser(sp);
    *comm_len = sc.b.size();
    *proof_len = sp.b.size();
    if (sc.b.size() > comm_cap || sp.b.size() > proof_cap) return -1;
    memcpy(comm_out, sc.b.data(), sc.b.size());
    memcpy(proof_out, sp.b.data(), sp.b.size());
    if (transcript || g_bl_skip_verify) return 1;
    Transcript tv(label);
    return spark_verify(pf, comm, vx, vy, evals, g, tv) ? 1 : 0;
  } catch (const std::string& e) {
    return -2;
  }
}
}

#include "snark.hpp"

namespace {
using namespace orc;
thread_local double g_snark_verify_us = 0;
thread_local double g_snark_prove_us = 0.0;

SnarkIn snark_in_from_c(const spg_snark_inputs* c) {
  SnarkIn in;
  in.input_block_num = c->input_block_num;
  in.output_block_num = c->output_block_num;
  for (size_t i = 0; i < c->input_len; i++) {
    in.input_liveness.push_back(c->input_liveness[i] != 0);
    in.input.push_back(ld(c->input + 4 * i));
  }
  in.func_input_width = c->func_input_width;
  in.input_offset = c->input_offset;
  in.output_offset = c->output_offset;
  in.output = ld(c->output);
  in.output_exec_num = c->output_exec_num;
  in.num_vars = c->num_vars;
  in.num_ios = c->num_ios;
  in.max_block_num_phy_ops = c->max_block_num_phy_ops;
  in.max_block_num_vir_ops = c->max_block_num_vir_ops;
  const size_t B = c->block_num_instances_bound;
  in.block_num_phy_ops.assign(c->block_num_phy_ops, c->block_num_phy_ops + B);
  in.block_num_vir_ops.assign(c->block_num_vir_ops, c->block_num_vir_ops + B);
  in.mem_addr_ts_bits_size = c->mem_addr_ts_bits_size;
  in.num_inputs_unpadded = c->num_inputs_unpadded;
  in.block_num_vars.assign(c->block_num_vars, c->block_num_vars + B);
  in.block_num_instances_bound = B;
  in.block_max_num_proofs = c->block_max_num_proofs;
  in.block_num_proofs.assign(c->block_num_proofs, c->block_num_proofs + B);
  in.consis_num_proofs = c->consis_num_proofs;
  in.total_num_init_phy_mem_accesses = c->total_num_init_phy_mem_accesses;
  in.total_num_init_vir_mem_accesses = c->total_num_init_vir_mem_accesses;
  in.total_num_phy_mem_accesses = c->total_num_phy_mem_accesses;
  in.total_num_vir_mem_accesses = c->total_num_vir_mem_accesses;
  auto rows = [](const uint64_t* p, size_t n, size_t w) {
    std::vector<FqVec> m(n, FqVec(w));
    for (size_t q = 0; q < n; q++)
      for (size_t i = 0; i < w; i++) m[q][i] = ld(p + 4 * (q * w + i));
    return m;
  };
  // block_vars[i]: the witness list of the i-th instance in the prover's sort order (lib.rs:1155-1178 pairs
  // block_vars_mat[i] with sorted instance i), sized by that instance's num_proofs and num_vars
  std::vector<size_t> order(B);
  for (size_t i = 0; i < B; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [&](size_t x, size_t y) { return c->block_num_proofs[x] > c->block_num_proofs[y]; });
  // (blocks that never execute sort last and have no list: the reference's block_vars_mat holds the executed
  // blocks only, ProverWitnessSecInfo::new reads every list's first row, lib.rs:520-526)
  for (size_t i = 0; i < B; i++) {
    const size_t b = order[i];
    if (c->block_num_proofs[b]) in.block_vars_mat.push_back(rows(c->block_vars[i], c->block_num_proofs[b], c->block_num_vars[b]));
  }
  in.exec_inputs_list = rows(c->exec_inputs, c->consis_num_proofs, c->num_ios);
  if (c->total_num_init_phy_mem_accesses)
    in.init_phy_mems_list = rows(c->init_phy_mems, c->total_num_init_phy_mem_accesses, INIT_PHY_MEM_WIDTH);
  if (c->total_num_init_vir_mem_accesses)
    in.init_vir_mems_list = rows(c->init_vir_mems, c->total_num_init_vir_mem_accesses, INIT_VIR_MEM_WIDTH);
  if (c->total_num_phy_mem_accesses)
    in.addr_phy_mems_list = rows(c->addr_phy_mems, c->total_num_phy_mem_accesses, PHY_MEM_WIDTH);
  if (c->total_num_vir_mem_accesses) {
    in.addr_vir_mems_list = rows(c->addr_vir_mems, c->total_num_vir_mem_accesses, VIR_MEM_WIDTH);
    in.addr_ts_bits_list = rows(c->addr_ts_bits, c->total_num_vir_mem_accesses, c->mem_addr_ts_bits_size);
  }
  return in;
}

SnarkInst snark_inst_from_c(const spg_snark_instance* c, bool multi) {
  SnarkInst s;
  s.inst = inst_from_c(&c->inst);
  s.gens = snark_eval_gens(c->gens_num_cons, c->gens_num_vars, c->gens_num_instances, c->gens_num_nz_entries);
  s.multi = multi;
  s.encode();
  return s;
}
}  // namespace

extern "C" {
// SNARK::multi_encode(block) / encode(pairwise) / encode(perm_root), then SNARK::prove under a fresh
// Transcript(label) + RandomTape("proof", seed) with vars_gens = R1CSGens(gens_label, gens_num_vars); writes
// bincode(SNARK). Returns 0 when the oracle's verifier accepts, >0 = failing verifier stage, <0 on error.
// SNARK::prove alone on a caller's transcript handle (orc_transcript_new, possibly appended to already; it keeps
// its state after the proof, as `transcript: &mut Transcript` does, src/lib.rs:1022). 0 on success.
int orc_snark_prove_tr(const spg_snark_inputs* in_c, const spg_snark_instance* block_c,
                       const spg_snark_instance* pairwise_c, const spg_snark_instance* perm_root_c,
                       const char* gens_label, size_t gens_num_vars, void* transcript, const uint64_t* tape_seed,
                       uint8_t* out, size_t cap, size_t* out_len) {
  try {
    SnarkIn in = snark_in_from_c(in_c);
    SnarkInst block = snark_inst_from_c(block_c, true), pairwise = snark_inst_from_c(pairwise_c, false),
              perm_root = snark_inst_from_c(perm_root_c, false);
    R1CSGens vg = R1CSGens::create(gens_label, gens_num_vars);
    RandomTape tape("proof", ld(tape_seed));
    SNARKProof pf = snark_prove(in, block, pairwise, perm_root, vg, *(Transcript*)transcript, tape);
    Ser s;
    pf.ser(s);
    *out_len = s.b.size();
    if (s.b.size() > cap) return -1;
    memcpy(out, s.b.data(), s.b.size());
    return 0;
  } catch (const std::string& e) {
    return -2;
  }
}
// SNARK::prove on the caller's prover transcript handle, then SNARK::verify of the same proof on the caller's verifier
// transcript handle (each in whatever state the caller left it, as `&mut Transcript`): the oracle's verdict on a
// caller transcript (0 = accepted, >0 = the failing verifier stage, <0 on error)
int orc_snark_prove_verify_tr(const spg_snark_inputs* in_c, const spg_snark_instance* block_c,
                              const spg_snark_instance* pairwise_c, const spg_snark_instance* perm_root_c,
                              const char* gens_label, size_t gens_num_vars, void* prover_tr, void* verifier_tr,
                              const uint64_t* tape_seed, uint8_t* out, size_t cap, size_t* out_len) {
  try {
    SnarkIn in = snark_in_from_c(in_c);
    SnarkInst block = snark_inst_from_c(block_c, true), pairwise = snark_inst_from_c(pairwise_c, false),
              perm_root = snark_inst_from_c(perm_root_c, false);
    R1CSGens vg = R1CSGens::create(gens_label, gens_num_vars);
    RandomTape tape("proof", ld(tape_seed));
    SNARKProof pf = snark_prove(in, block, pairwise, perm_root, vg, *(Transcript*)prover_tr, tape);
    Ser s;
    pf.ser(s);
    *out_len = s.b.size();
    if (s.b.size() > cap) return -1;
    memcpy(out, s.b.data(), s.b.size());
    return snark_verify(pf, in, block, pairwise, perm_root, vg, *(Transcript*)verifier_tr);
  } catch (const std::string& e) {
    return -2;
  }
}
int orc_snark_prove(const spg_snark_inputs* in_c, const spg_snark_instance* block_c,
                    const spg_snark_instance* pairwise_c, const spg_snark_instance* perm_root_c, const char* gens_label,
                    size_t gens_num_vars, const char* label, const uint64_t* tape_seed, uint8_t* out, size_t cap,
                    size_t* out_len) {
  try {
    SnarkIn in = snark_in_from_c(in_c);
    SnarkInst block = snark_inst_from_c(block_c, true), pairwise = snark_inst_from_c(pairwise_c, false),
              perm_root = snark_inst_from_c(perm_root_c, false);
    R1CSGens vg = R1CSGens::create(gens_label, gens_num_vars);
    if (g_bl_barrier) g_bl_barrier();
    g_bl_w0 = steady_us();
    auto t0 = std::chrono::steady_clock::now();
    Transcript t(label);
    RandomTape tape("proof", ld(tape_seed));
    SNARKProof pf = snark_prove(in, block, pairwise, perm_root, vg, t, tape);
    g_snark_prove_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    g_bl_w1 = steady_us();
    Ser s;
    pf.ser(s);
    *out_len = s.b.size();
    if (s.b.size() > cap) return -1;
    memcpy(out, s.b.data(), s.b.size());
    // negative tests (tests/test_oracle_snark.py): ORC_TAMPER corrupts what the verifier sees
    const char* tamper = getenv("ORC_TAMPER");
    if (tamper && std::string(tamper) == "io_proof" && pf.io_proof.proofs.size() > 1)
      std::swap(pf.io_proof.proofs[0], pf.io_proof.proofs[1]);
    if (tamper && std::string(tamper) == "shift_eval" && pf.shift_proof.C_orig_evals.size() > 1)
      std::swap(pf.shift_proof.C_orig_evals[0], pf.shift_proof.C_orig_evals[1]);
    if (tamper && std::string(tamper) == "perm_opening" && !pf.proof_eval_perm_poly_prod_list.empty())
      std::swap(pf.proof_eval_perm_poly_prod_list[0], pf.proof_eval_perm_poly_prod_list.back());
    if (g_bl_skip_verify) return 0;
    Transcript tv(label);
    auto t1 = std::chrono::steady_clock::now();
    const int rc = snark_verify(pf, in, block, pairwise, perm_root, vg, tv);
    g_snark_verify_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
    return rc;
  } catch (const std::string& e) {
    return -2;
  }
}
double orc_snark_last_prove_us() { return g_snark_prove_us; }
// the last snark_prove's phases: up to `max` (name[32], microseconds) pairs, returns their count
int orc_snark_last_phases(char* names, double* us, int max) {
  int k = 0;
  for (auto& l : g_snark_phases.laps) {
    if (k >= max) break;
    snprintf(names + 32 * k, 32, "%s", l.first.c_str());
    us[k++] = l.second;
  }
  return k;
}
double orc_snark_last_verify_us() { return g_snark_verify_us; }
}

extern "C" {
// R1CSInstance::multiply_vec_block (src/r1csinstance.rs:363-436) -> Az, Bz, Cz flattened in DensePolynomialPqx layout
// (instance p: num_proofs[p] x 1 x num_cons[p], q_rev / x_rev order). z: instance p's num_proofs[p] x nws x
// num_inputs[p] scalars; each section row is padded with zeros to max_num_inputs for the reference's z[w][c % max].
int orc_multiply_vec_block(const spg_r1cs_instance* ci, size_t P, const size_t* num_proofs, size_t max_num_proofs,
                           const size_t* num_inputs, size_t max_num_inputs, size_t nws, const uint64_t* z,
                           uint64_t* outA, uint64_t* outB, uint64_t* outC) {
  R1CSInstance inst = inst_from_c(ci);
  Mat4 zm(P);
  const uint64_t* s = z;
  for (size_t p = 0; p < P; p++) {
    zm[p].assign(num_proofs[p], std::vector<FqVec>(nws, FqVec(max_num_inputs, fq_zero())));
    for (size_t q = 0; q < num_proofs[p]; q++)
      for (size_t w = 0; w < nws; w++)
        for (size_t x = 0; x < num_inputs[p]; x++, s += 4) zm[p][q][w][x] = ld(s);
  }
  std::vector<size_t> np(num_proofs, num_proofs + P), ni(num_inputs, num_inputs + P), nc(P);
  for (size_t p = 0; p < P; p++) nc[p] = inst.num_cons[inst.num_instances == 1 ? 0 : p];
  Pqx Az, Bz, Cz;
  inst.multiply_vec_block(P, np, max_num_proofs, ni, max_num_inputs, inst.max_num_cons, nc, zm, &Az, &Bz, &Cz);
  uint64_t* outs[3] = {outA, outB, outC};
  const Pqx* T[3] = {&Az, &Bz, &Cz};
  for (int k = 0; k < 3; k++) {
    uint64_t* o = outs[k];
    for (size_t p = 0; p < P; p++)
      for (size_t q = 0; q < T[k]->Z[p].size(); q++)
        for (const Fq& v : T[k]->Z[p][q][0]) {
          st(o, v);
          o += 4;
        }
  }
  return 0;
}
}
