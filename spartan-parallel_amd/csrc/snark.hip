// spg — SNARK::prove (src/lib.rs:971-2746): the orchestration around the device-resident R1CSProof, SPARK
// and Hyrax kernels.
//
//   SNARK::multi_encode / encode      src/lib.rs:793-829, src/r1csinstance.rs:654-737    spg_snark_encode
//   witness upload (block_vars, exec inputs stay in HBM)                                  spg_snark_witness_new
//   SNARK::prove                      src/lib.rs:971-2746                                 spg_snark_prove
//     instance commitments -> transcript, block / pairwise sort and padding             (host, O(#instances))
//     permutation / memory witnesses w2, w3, w3_shifted    lib.rs:1299-1955, 831-968    (host, O(Q * 8))
//     Hyrax commitments of every witness polynomial        lib.rs:1957-2221             commit_dev (device MSMs)
//     three R1CSProof::prove + multi_evaluate + R1CSEvalProof                             r1cs.hip / spark.hip
//     perm product, shift and IO PolyEvalProofs            lib.rs:2534-2693, 187-446    host bound + device Bullet
// The host side is the transcript, the small witness recurrences and the bincode writer; every O(N) table
// (block_vars, Az/Bz/Cz, SPARK dense representations) lives in HBM.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "hostpoly.hpp"
#include "proto.hpp"

using namespace spg;

namespace {

const size_t INIT_PHY_MEM_WIDTH = 4, INIT_VIR_MEM_WIDTH = 4, PHY_MEM_WIDTH = 4, VIR_MEM_WIDTH = 8, W3_WIDTH = 8;

typedef std::vector<FqV> Rows;  // w_mat of one instance: rows (executions) of scalars

FqV flatten(const Rows& m) {
  FqV v;
  for (auto& r : m) v.insert(v.end(), r.begin(), r.end());
  return v;
}
Rows shift_rows(const Rows& m, size_t width) {
  Rows s(m.begin() + 1, m.end());
  s.push_back(FqV(width, fq_zero()));
  return s;
}
FqV pad_pow2(FqV v) {  // DensePolynomial::new pads to a power of two (dense_mlpoly.rs:152-161)
  v.resize(npow2(std::max<size_t>(v.size(), 1)), fq_zero());
  return v;
}
// DensePolynomial::bound (dense_mlpoly.rs:258-265) of several host (Z, L) pairs in one pool burst: each job's columns are cut into slices of >= ~2048
// products, all slices of all jobs go to the pool together (one wake-up instead of one per polynomial)
std::vector<FqV> host_bounds(const std::vector<std::pair<const FqV*, const FqV*>>& jobs) {
  std::vector<FqV> out(jobs.size());
  struct Slice {
    size_t j, Ls, Rs, i0, i1;
  };
  std::vector<Slice> sl;
  for (size_t j = 0; j < jobs.size(); j++) {
    const size_t nv = lg2(jobs[j].first->size()), Ls = (size_t)1 << (nv / 2), Rs = (size_t)1 << (nv - nv / 2);
    out[j].assign(Rs, fq_zero());
    const size_t C = std::max<size_t>(1, std::min<size_t>({8, Rs, Ls * Rs / 2048}));
    for (size_t c = 0; c < C; c++) sl.push_back({j, Ls, Rs, Rs * c / C, Rs * (c + 1) / C});
  }
  auto run = [&](int k) {
    const Slice& s = sl[k];
    const FqV& Z = *jobs[s.j].first;
    const FqV& L = *jobs[s.j].second;
    FqV& o = out[s.j];
    for (size_t j = 0; j < s.Ls; j++)
      for (size_t i = s.i0; i < s.i1; i++) o[i] = fq_add(o[i], fq_mul(L[j], Z[j * s.Rs + i]));
  };
  if (sl.size() == 1)
    run(0);
  else if (!sl.empty())
    pool().parallel_for((int)sl.size(), run);
  return out;
}
void eq_factored(const FqV& r, FqV* L, FqV* R) {
  const size_t ln = r.size() / 2;
  *L = eq_evals_host(FqV(r.begin(), r.begin() + ln));
  *R = eq_evals_host(FqV(r.begin() + ln, r.end()));
}

}  // namespace

// ------------------------------------------------------------------------------------ handles
// SNARK::encode / multi_encode of one R1CS instance: the host matrices, the SPARK decommitments in HBM, the
// device instance (unsorted, for multi_evaluate) and a cache of the sorted device instance.
struct spg_snark_comp {
  size_t num_instances = 0, max_num_cons = 0, num_vars = 0;
  std::vector<size_t> num_cons, nnz;
  std::vector<std::vector<spg_sparse_entry>> mats;  // [3p + m]
  std::vector<std::vector<size_t>> label_map;
  std::vector<spg_spark*> sparks;
  spg_r1cs_inst* dev = nullptr;
  spg_r1cs_inst* dev_sorted = nullptr;
  std::vector<size_t> sorted_order;
  spg_r1cs_instance view(const std::vector<size_t>& order, std::vector<const spg_sparse_entry*>* ptrs,
                         std::vector<size_t>* nnz_o, std::vector<size_t>* nc_o) const {
    ptrs->clear();
    nnz_o->clear();
    nc_o->clear();
    for (size_t i : order) {
      nc_o->push_back(num_cons[i]);
      for (int m = 0; m < 3; m++) {
        ptrs->push_back(mats[3 * i + m].data());
        nnz_o->push_back(mats[3 * i + m].size());
      }
    }
    spg_r1cs_instance ci;
    ci.num_instances = order.size();
    ci.max_num_cons = max_num_cons;
    ci.num_vars = num_vars;
    ci.num_cons = nc_o->data();
    ci.nnz = nnz_o->data();
    ci.entries = ptrs->data();
    return ci;
  }
};

// the run-time inputs of SNARK::prove, with block_vars and exec_inputs resident in HBM
struct spg_snark_wit {
  spg_snark_inputs a;  // sizes and scalars (pointer fields below are owned copies)
  std::vector<uint8_t> liveness;
  FqV input;
  Fq output;
  std::vector<size_t> phy_ops, vir_ops, nvars, nproofs;
  std::vector<Rows> block_io;  // [b][q] first 2 * num_inputs_unpadded entries of every block_vars row
  std::vector<Fq*> d_block_vars;
  std::vector<size_t> d_block_bytes;  // their allocation sizes (dev_cache_put on free)
  Rows exec, init_phy, init_vir, addr_phy, addr_vir, ts_bits;
  Fq* d_exec = nullptr;
};

// R1CSProof bincode + challenges (rp, rq_rev, rx, rw||ry)
struct SatOut {
  std::vector<uint8_t> bytes;
  FqV ch[4];
};

namespace {

int snark_comp_free(spg_ctx* ctx, spg_snark_comp* C) {
  if (!C) return SPG_OK;
  for (auto* s : C->sparks) spg_spark_free(ctx, s);
  spg_r1cs_inst_free(ctx, C->dev);
  spg_r1cs_inst_free(ctx, C->dev_sorted);
  delete C;
  return SPG_OK;
}

// R1CSProof::prove through the device prover (r1cs.hip)
int sat_prove(spg_ctx* ctx, spg_r1cs_gens* gens, spg_r1cs_inst* inst, size_t P, size_t max_np,
              const std::vector<size_t>& num_proofs, size_t max_ni, const std::vector<size_t>& num_inputs,
              const std::vector<WPart>& secs, spg_r1cs_witness** W, spg_transcript* t, spg_random_tape* tape,
              SatOut* out) {
  Laps lp;
  lp.title = "sat_prove";
  lp.on = lp.on && atoi(getenv("SPG_TRACE")) >= 2;
  int rc = witness_from_parts(ctx, secs, W);
  if (rc) return rc;
  lp.lap("witness_from_parts");
  lp.print();
  // output staging kept across proves: a fresh 4 MB vector is zero-filled on every call, and when glibc serves it from
  // new pages that is ~1000 page faults (~0.8 ms in the SNARK's kernel trace, the device idle meanwhile)
  static thread_local std::vector<uint8_t> buf;
  static thread_local std::vector<uint64_t> ch;
  if (buf.size() < ((size_t)1 << 22)) buf.resize((size_t)1 << 22);
  if (ch.size() < 4 * 4096) ch.resize(4 * 4096);
  size_t len = 0, chl[4] = {0, 0, 0, 0};
  rc = spg_r1cs_prove(ctx, gens, inst, P, max_np, num_proofs.data(), max_ni, num_inputs.data(), *W, t, tape,
                      buf.data(), buf.size(), &len, ch.data(), chl);
  if (rc) return rc;
  out->bytes.assign(buf.begin(), buf.begin() + len);
  size_t o = 0;
  for (int k = 0; k < 4; k++) {
    out->ch[k].clear();
    for (size_t i = 0; i < chl[k]; i++) out->ch[k].push_back(ld_fq(&ch[4 * (o + i)]));
    o += chl[k];
  }
  return 0;
}

// R1CSInstance::multi_evaluate on the unsorted device instance (3 evals per instance)
int multi_eval(spg_ctx* ctx, spg_snark_comp* C, const FqV& rx, const FqV& ry, FqV* out) {
  std::vector<uint64_t> a(4 * rx.size()), b(4 * ry.size()), o(4 * 3 * C->num_instances);
  for (size_t i = 0; i < rx.size(); i++) st_fq(&a[4 * i], rx[i]);
  for (size_t i = 0; i < ry.size(); i++) st_fq(&b[4 * i], ry[i]);
  int rc = spg_r1cs_multi_evaluate(ctx, C->dev, a.data(), rx.size(), b.data(), ry.size(), o.data());
  if (rc) return rc;
  out->clear();
  for (size_t i = 0; i < 3 * C->num_instances; i++) out->push_back(ld_fq(&o[4 * i]));
  return 0;
}
// multi_evaluate_bound_rp (r1csinstance.rs:597-630) from the unsorted list and the sort order
void bound_rp(const FqV& list, const std::vector<size_t>& order, const FqV& rp, Fq out[3]) {
  for (int m = 0; m < 3; m++) {
    FqV v;
    for (size_t i : order) v.push_back(list[3 * i + m]);
    out[m] = dense_eval_host(v, rp);
  }
}

int ensure_sorted(spg_ctx* ctx, spg_snark_comp* C, const std::vector<size_t>& order) {
  if (C->dev_sorted && C->sorted_order == order) return 0;
  spg_r1cs_inst_free(ctx, C->dev_sorted);
  C->dev_sorted = nullptr;
  std::vector<const spg_sparse_entry*> ptrs;
  std::vector<size_t> nnz, nc;
  spg_r1cs_instance ci = C->view(order, &ptrs, &nnz, &nc);
  int rc = spg_r1cs_inst_new(ctx, &ci, &C->dev_sorted);
  if (rc) return rc;
  C->sorted_order = order;
  return 0;
}

// R1CSCommitment::append_to_transcript (r1csinstance.rs:64-70) of group g
void append_r1cs_comm(const spg_snark_comp* C, size_t g, Tr& t) {
  t.u64("num_cons", C->num_instances * C->max_num_cons);
  t.u64("num_vars", C->num_vars);
  spark_comm_append(C->sparks[g], t);
}

// PolyEvalProof::prove_batched_points (dense_mlpoly.rs:531-622) on a host polynomial
int prove_batched_points(spg_ctx* ctx, ProverGens& g, const FqV& Z, const std::vector<FqV>& r_list, const FqV& Zr,
                         Tr& t, Tape& tape, Writer& w) {
  t.protocol("polynomial evaluation proof");
  const size_t ln = r_list[0].size() / 2;
  std::vector<FqV> keys, Ls, Rs;
  FqV Zc;
  Fq c_base = t.challenge("challenge_c"), c = fq_one();
  std::vector<FqV> Rv(r_list.size());
  std::vector<std::pair<size_t, Fq>> acc(r_list.size(), {SIZE_MAX, fq_zero()});  // Rs[idx] += c R_i (axpy_pool)
  for (size_t i = 0; i < r_list.size(); i++) {
    FqV L;
    FqV& R = Rv[i];
    eq_factored(r_list[i], &L, &R);
    FqV key(r_list[i].begin(), r_list[i].begin() + ln);
    size_t idx = keys.size();
    for (size_t k = 0; k < keys.size(); k++)
      if (keys[k].size() == key.size() && std::equal(keys[k].begin(), keys[k].end(), key.begin(),
                                                     [](const Fq& a, const Fq& b) { return memcmp(&a, &b, 32) == 0; })) {
        idx = k;
        break;
      }
    if (idx < keys.size()) {
      c = fq_mul(c, c_base);
      acc[i] = {idx, c};
      Zc[idx] = fq_add(Zc[idx], fq_mul(c, Zr[i]));
    } else {
      keys.push_back(key);
      Ls.push_back(L);
      Rs.push_back(R);
      Zc.push_back(Zr[i]);
    }
  }
  {
    std::vector<Axpy> ax;
    for (size_t i = 0; i < r_list.size(); i++)
      if (acc[i].first != SIZE_MAX) ax.push_back({&Rs[acc[i].first], acc[i].second, &Rv[i]});
    axpy_pool(ax);
  }
  w.u64(Ls.size());
  // every distinct point's L.Z bound up front, in one pool burst
  std::vector<std::pair<const FqV*, const FqV*>> bj;
  for (size_t i = 0; i < Ls.size(); i++) bj.push_back({&Z, &Ls[i]});
  std::vector<FqV> LZs = host_bounds(bj);
  for (size_t i = 0; i < Ls.size(); i++) {
    DotProductProofLogP p;
    Pt cy;
    int rc = dotproduct_log_prove(ctx, g, t, tape, LZs[i], fq_zero(), Rs[i], Zc[i], fq_zero(), &p, &cy);
    if (rc) return rc;
    p.ser(w);
  }
  return 0;
}

// PolyEvalProof::prove_batched_instances (dense_mlpoly.rs:689-780) on host polynomials
int prove_batched_instances(spg_ctx* ctx, ProverGens& g, const std::vector<const FqV*>& polys,
                            const std::vector<FqV>& r_list, const FqV& Zr, Tr& t, Tape& tape, Writer& w) {
  t.protocol("polynomial evaluation proof");
  std::vector<std::pair<size_t, FqV>> keys;
  std::vector<FqV> LZs, Rs;
  FqV Zc;
  Fq c_base = t.challenge("challenge_c"), c = fq_one();
  // every polynomial's eq factors, then all L.Z bounds in one pool burst
  std::vector<FqV> Lv(polys.size()), Rv(polys.size());
  std::vector<std::pair<const FqV*, const FqV*>> bj;
  for (size_t i = 0; i < polys.size(); i++) {
    const size_t nv = lg2(polys[i]->size());
    FqV r = r_list[i];
    if (nv >= r.size())
      r.insert(r.begin(), nv - r.size(), fq_zero());
    else
      r = FqV(r.end() - nv, r.end());
    eq_factored(r, &Lv[i], &Rv[i]);
    bj.push_back({polys[i], &Lv[i]});
  }
  std::vector<FqV> LZall = host_bounds(bj);
  std::vector<std::pair<size_t, Fq>> acc(polys.size(), {SIZE_MAX, fq_zero()});  // LZs[idx] += c LZ_i (axpy_pool)
  for (size_t i = 0; i < polys.size(); i++) {
    const size_t nv = lg2(polys[i]->size());
    const FqV& R = Rv[i];
    size_t idx = keys.size();
    for (size_t k = 0; k < keys.size(); k++)
      if (keys[k].first == nv && keys[k].second.size() == R.size() &&
          memcmp(keys[k].second.data(), R.data(), R.size() * sizeof(Fq)) == 0) {
        idx = k;
        break;
      }
    FqV& LZ = LZall[i];
    if (idx < keys.size()) {
      c = fq_mul(c, c_base);
      acc[i] = {idx, c};
      Zc[idx] = fq_add(Zc[idx], fq_mul(c, Zr[i]));
    } else {
      keys.push_back({nv, R});
      Zc.push_back(Zr[i]);
      LZs.push_back(LZ);
      Rs.push_back(R);
    }
  }
  {
    std::vector<Axpy> ax;
    for (size_t i = 0; i < polys.size(); i++)
      if (acc[i].first != SIZE_MAX) ax.push_back({&LZs[acc[i].first], acc[i].second, &LZall[i]});
    axpy_pool(ax);
  }
  w.u64(LZs.size());
  for (size_t i = 0; i < LZs.size(); i++) {
    DotProductProofLogP p;
    Pt cy;
    int rc = dotproduct_log_prove(ctx, g, t, tape, LZs[i], fq_zero(), Rs[i], Zc[i], fq_zero(), &p, &cy);
    if (rc) return rc;
    p.ser(w);
  }
  return 0;
}

// The L.Z bounds of PolyEvalProof::prove_uni_batched_instances (dense_mlpoly.rs:1046-1130): L = (r^(Rs j))_j for
// each polynomial size 2^nv, all bounds in one pool burst. The shift proof also reads its evaluations from them:
// sum_k LZ[k] r^k = sum_i Z[i] r^i.
std::vector<FqV> uni_bounds(const std::vector<const FqV*>& polys, const Fq& r) {
  std::vector<size_t> nvs;
  std::vector<FqV> Lv;
  std::vector<size_t> li(polys.size());
  for (size_t i = 0; i < polys.size(); i++) {
    const size_t nv = lg2(polys[i]->size());
    size_t k = 0;
    while (k < nvs.size() && nvs[k] != nv) k++;
    if (k == nvs.size()) {
      Fq r_base = fq_one();
      for (size_t e = 0; e < ((size_t)1 << (nv - nv / 2)); e++) r_base = fq_mul(r_base, r);
      FqV L;
      Fq lb = fq_one();
      for (size_t e = 0; e < ((size_t)1 << (nv / 2)); e++) {
        L.push_back(lb);
        lb = fq_mul(lb, r_base);
      }
      nvs.push_back(nv);
      Lv.push_back(L);
    }
    li[i] = k;
  }
  std::vector<std::pair<const FqV*, const FqV*>> bj;
  for (size_t i = 0; i < polys.size(); i++) bj.push_back({polys[i], &Lv[li[i]]});
  return host_bounds(bj);
}

// PolyEvalProof::prove_uni_batched_instances (dense_mlpoly.rs:1046-1130) from the bounds of uni_bounds(polys, r)
int prove_uni_batched(spg_ctx* ctx, ProverGens& g, const std::vector<const FqV*>& polys, const std::vector<FqV>& LZs,
                      const Fq& r, const FqV& Zr, Tr& t, Tape& tape, Writer& w) {
  t.protocol("polynomial evaluation proof");
  size_t max_nv = 0;
  for (auto p : polys) max_nv = std::max(max_nv, lg2(p->size()));
  const size_t R_size = (size_t)1 << (max_nv - max_nv / 2);
  FqV R;
  Fq rb = fq_one();
  for (size_t i = 0; i < R_size; i++) {
    R.push_back(rb);
    rb = fq_mul(rb, r);
  }
  Fq c_base = t.challenge("challenge_c"), c = fq_one();
  FqV LZc(R_size, fq_zero());
  Fq Zrc = fq_zero();
  std::vector<Axpy> ax;
  for (size_t i = 0; i < polys.size(); i++) {
    ax.push_back({&LZc, c, &LZs[i]});
    Zrc = fq_add(Zrc, fq_mul(c, Zr[i]));
    c = fq_mul(c, c_base);
  }
  axpy_pool(ax);
  DotProductProofLogP p;
  Pt cy;
  int rc = dotproduct_log_prove(ctx, g, t, tape, LZc, fq_zero(), R, Zrc, fq_zero(), &p, &cy);
  if (rc) return rc;
  p.ser(w);
  return 0;
}

// one host witness section (ProverWitnessSecInfo): rows per instance and their flattened polynomials
struct HSec {
  std::vector<Rows> w;
  std::vector<FqV> poly;   // flattened, padded (DensePolynomial)
  std::vector<const Fq*> dev;  // device copies when resident (block_vars, exec inputs)
  size_t n() const { return w.size() ? w.size() : dev.size(); }
};

struct SecInfo {  // sizes + data pointers for merges (ProverWitnessSecInfo::merge / concat, lib.rs:546-604)
  std::vector<size_t> num_proofs, num_inputs;
  std::vector<const Fq*> src;  // host or device data of each instance
  std::vector<const FqV*> poly;  // host polynomial (nullptr for device-only data)
};
SecInfo merge(const std::vector<const SecInfo*>& comps, std::vector<size_t>* inst_map) {
  std::vector<size_t> ptr(comps.size(), 0);
  size_t total = 0;
  for (auto c : comps) total += c->num_proofs.size();
  SecInfo s;
  inst_map->clear();
  while (inst_map->size() < total) {
    size_t best = 0, nc = 0;
    for (size_t i = 0; i < comps.size(); i++)
      if (ptr[i] < comps[i]->num_proofs.size() && comps[i]->num_proofs[ptr[i]] > best) {
        best = comps[i]->num_proofs[ptr[i]];
        nc = i;
      }
    inst_map->push_back(nc);
    s.num_proofs.push_back(comps[nc]->num_proofs[ptr[nc]]);
    s.num_inputs.push_back(comps[nc]->num_inputs[ptr[nc]]);
    s.src.push_back(comps[nc]->src[ptr[nc]]);
    s.poly.push_back(comps[nc]->poly[ptr[nc]]);
    ptr[nc]++;
  }
  return s;
}
SecInfo concat(const std::vector<const SecInfo*>& comps) {
  SecInfo s;
  for (auto c : comps) {
    s.num_proofs.insert(s.num_proofs.end(), c->num_proofs.begin(), c->num_proofs.end());
    s.num_inputs.insert(s.num_inputs.end(), c->num_inputs.begin(), c->num_inputs.end());
    s.src.insert(s.src.end(), c->src.begin(), c->src.end());
    s.poly.insert(s.poly.end(), c->poly.begin(), c->poly.end());
  }
  return s;
}
WPart wpart(const SecInfo& s) { return {s.num_proofs, s.num_inputs, s.src}; }
// a host section of one instance per rows block
SecInfo host_sec(const std::vector<Rows>& w, const std::vector<FqV>& poly) {
  SecInfo s;
  for (size_t p = 0; p < w.size(); p++) {
    s.num_proofs.push_back(w[p].size());
    s.num_inputs.push_back(w[p][0].size());
    s.src.push_back(poly[p].data());
    s.poly.push_back(&poly[p]);
  }
  return s;
}

// Hyrax commitment of a host polynomial (uploads into a staging slot, device MSMs)
// Hyrax commitments of the witness polynomials of SNARK::prove, deferred so that all rows of one width go to
// the device in one MSM launch; flush() appends them to the transcript in the order they were added (every
// commitment between challenge_r and the block R1CSProof depends only on the witness and tau, r).
struct CQ {
  struct Item {
    const FqV* host;
    const Fq* dev;
    size_t len;
    std::vector<Pt>* out;
  };
  std::vector<Item> items;
  // Early group: device-resident polynomials (the block witnesses) whose rows are committed by one batch MSM
  // launched before the host builds the permutation witnesses, so the device works while the host does;
  // flush() only downloads those rows. Their commitments depend on the witness alone, never on the
  // transcript, and they are recomputed in every prove.
  std::vector<const Fq*> early_dev;
  size_t early_R = 0, early_L = 0;
  uint8_t* early_out = nullptr;
  const Ext* early_ext = nullptr;  // halved comb points (encoded on the host at flush), else early_out's encodings
  int launch_early(spg_ctx* ctx, ProverGens& g, const std::vector<std::pair<const Fq*, size_t>>& its) {
    size_t R = 0, total = 0;
    for (auto& it : its) {
      const size_t nv = lg2(it.second), r = (size_t)1 << (nv - nv / 2);
      if (R && r != R) return 0;  // one width only; otherwise flush() groups them as usual
      R = r;
      total += it.second;
    }
    // the one-launch batch path of commit_rows only (rows wider than the latency path, one chunk)
    if (its.empty() || R <= 256 || R > g.n_pc || total / R > ((size_t)1 << 24) / R) return 0;
    Fq* d = (Fq*)ws_get(ctx, 92, total * sizeof(Fq) + 64);
    uint8_t* out = (uint8_t*)ws_get(ctx, 93, 32 * (total / R) + 64);
    if (!d || !out) return set_err(ctx, SPG_E_NOMEM, "early commit staging");
    SPG_HIP(ctx, hipEventRecord(ctx->ev_pre, ctx->stream));  // flush()'s side stream starts from here
    size_t o = 0;
    for (auto& it : its) {
      SPG_HIP(ctx, hipMemcpyAsync(d + o, it.first, it.second * sizeof(Fq), hipMemcpyDeviceToDevice, ctx->stream));
      o += it.second;
    }
    // the comb rows with halved scalars: flush() encodes the points' doubles on the host in one batch (~50 us on the
    // pool for 1024 rows) instead of a k_compress_ext launch (~140 us of dependent squarings per lane)
    static const bool halve = !getenv("SPG_HALVED_ENC") || atoi(getenv("SPG_HALVED_ENC")) != 0;
    // slot 95: 94 is spark.hip's kWsRelay (the persistent layer kernel's relay word)
    Ext* ext = halve && total / R >= 384 ? (Ext*)ws_get(ctx, 95, sizeof(Ext) * (total / R) + 64) : nullptr;
    int rc = ext ? msm_comb(ctx, g.dev, 0, d, R, total / R, nullptr, nullptr, -1, ext, true) : kCombSkip;
    if (rc == kCombSkip) {
      ext = nullptr;
      rc = msm_batch_device(ctx, g.dev, 0, d, R, total / R, nullptr, out, nullptr, (long)(g.n_pc + 1));
    }
    if (rc) return rc;
    early_ext = ext;
    for (auto& it : its) early_dev.push_back(it.first);
    early_R = R;
    early_L = total / R;
    early_out = out;
    return 0;
  }
  bool is_early(const Item& it) const {
    return it.dev && std::find(early_dev.begin(), early_dev.end(), it.dev) != early_dev.end();
  }
  void add(const FqV& v, std::vector<Pt>* out) { items.push_back({&v, nullptr, v.size(), out}); }
  void add_dev(const Fq* d, size_t len, std::vector<Pt>* out) { items.push_back({nullptr, d, len, out}); }
  int flush(spg_ctx* ctx, ProverGens& g, Tr& t) {
    std::vector<size_t> widths;
    for (auto& it : items) {
      const size_t nv = lg2(it.len), R = (size_t)1 << (nv - nv / 2);
      it.out->assign((size_t)1 << (nv / 2), Pt());
      if (!is_early(it) && std::find(widths.begin(), widths.end(), R) == widths.end()) widths.push_back(R);
    }
    // While the early MSM runs, the other rows go to the device on the second stream: their uploads and
    // latency-path MSMs then overlap it instead of queueing behind it. Rows of at most kSideMaxR scalars take
    // commit_rows' latency path, whose workspace slots, mapped buckets and staging the batch pipeline of the early
    // MSM never touches; wider rows stay on the main stream.
    static const size_t kSideMaxR = 256;
    static const bool side_on = !getenv("SPG_CQ_SIDE") || atoi(getenv("SPG_CQ_SIDE")) != 0;
    bool side = side_on && early_L > 0;
    for (size_t R : widths) side = side && R <= kSideMaxR;
    Laps lp;
    lp.title = "commit queue flush";
    lp.on = lp.on && getenv("SPG_TRACE") && atoi(getenv("SPG_TRACE")) >= 2;
    const hipStream_t main_stream = ctx->stream;
    if (side) {
      SPG_HIP(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_pre, 0));
      ctx->stream = ctx->stream2;
    }
    int rc = flush_rows_launch(ctx, g, widths);
    ctx->stream = main_stream;
    if (rc) return rc;
    lp.lap(side ? "rows_side_launch" : "rows_launch");
    // the early group's encodings while the other rows' points are computed
    if (early_L) {
      std::vector<Pt> rows(early_L);
      if (early_ext) {
        Ext* h = (Ext*)enc_stage_get(ctx, early_L * sizeof(Ext));
        if (!h) return set_err(ctx, SPG_E_NOMEM, "encoding staging");
        SPG_HIP(ctx, hipMemcpyAsync(h, early_ext, early_L * sizeof(Ext), hipMemcpyDeviceToHost, ctx->stream));
        SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
        encode_halved_host(h, early_L, rows.data());
        early_ext = nullptr;
      } else {
        SPG_HIP(ctx, hipMemcpyAsync(rows.data(), early_out, 32 * early_L, hipMemcpyDeviceToHost, ctx->stream));
        SPG_HIP(ctx, hipStreamSynchronize(ctx->stream));
      }
      size_t o = 0;
      for (const Fq* d : early_dev)  // rows in launch order
        for (auto& it : items)
          if (it.dev == d) {
            std::copy(rows.begin() + o, rows.begin() + o + it.out->size(), it.out->begin());
            o += it.out->size();
          }
      early_dev.clear();
      early_L = 0;
    }
    lp.lap("early_wait");
    if (side) ctx->stream = ctx->stream2;
    rc = flush_rows_finish(ctx, g, widths);
    ctx->stream = main_stream;
    if (rc) return rc;
    lp.lap(side ? "rows_side_finish" : "rows_finish");
    for (auto& it : items) append_polycomm(t, "poly_commitment", *it.out);
    items.clear();
    lp.lap("append");
    lp.print();
    return 0;
  }
  // the rows of every item outside the early group, on ctx->stream: launched (uploads and points), then finished
  // (encodings; the host may encode the early group in between)
  std::vector<std::vector<Pt>> rows;
  std::vector<RowJob> jobs;
  RowsPending pend;
  int flush_rows_finish(spg_ctx* ctx, ProverGens& g, const std::vector<size_t>& widths) {
    int rc = commit_rows_many_finish(ctx, g, jobs, pend);
    if (rc) return rc;
    for (size_t w = 0; w < widths.size(); w++) {
      size_t ro = 0;
      for (auto& it : items) {
        if (is_early(it) || ((size_t)1 << (lg2(it.len) - lg2(it.len) / 2)) != widths[w]) continue;
        std::copy(rows[w].begin() + ro, rows[w].begin() + ro + it.out->size(), it.out->begin());
        ro += it.out->size();
      }
    }
    rows.clear();
    jobs.clear();
    return 0;
  }
  int flush_rows_launch(spg_ctx* ctx, ProverGens& g, const std::vector<size_t>& widths) {
    // one staging range per width, every width's rows committed together (the latency-path widths share one
    // encoding launch and one download)
    size_t total = 0;
    for (auto& it : items)
      if (!is_early(it)) total += it.len;
    Fq* d = (Fq*)ws_get(ctx, 91, total * sizeof(Fq) + 64);
    if (total && !d) return set_err(ctx, SPG_E_NOMEM, "commit staging");
    rows.assign(widths.size(), {});
    jobs.clear();
    size_t o = 0;
    for (size_t w = 0; w < widths.size(); w++) {
      const size_t R = widths[w], o0 = o;
      for (auto& it : items) {
        if (is_early(it) || ((size_t)1 << (lg2(it.len) - lg2(it.len) / 2)) != R) continue;
        if (it.host)
          SPG_HIP(ctx, hipMemcpyAsync(d + o, it.host->data(), it.len * sizeof(Fq), hipMemcpyHostToDevice, ctx->stream));
        else
          SPG_HIP(ctx, hipMemcpyAsync(d + o, it.dev, it.len * sizeof(Fq), hipMemcpyDeviceToDevice, ctx->stream));
        o += it.len;
      }
      rows[w].resize((o - o0) / R);
      jobs.push_back({d + o0, R, (o - o0) / R, rows[w].data()});
    }
    return commit_rows_many_launch(ctx, g, jobs, &pend);
  }
};

}  // namespace

// ------------------------------------------------------------------------------------ C-ABI
extern "C" int spg_snark_encode(spg_ctx* ctx, const spg_snark_instance* si, int multi, spg_snark_comp** out) {
  if (!ctx || !si || !out || !si->inst.num_instances || !si->inst.nnz || !si->inst.entries) return SPG_E_ARG;
  const spg_r1cs_instance& ci = si->inst;
  spg_snark_comp* C = new spg_snark_comp();
  C->num_instances = ci.num_instances;
  C->max_num_cons = ci.max_num_cons;
  C->num_vars = ci.num_vars;
  C->num_cons.assign(ci.num_cons, ci.num_cons + ci.num_instances);
  for (size_t k = 0; k < 3 * ci.num_instances; k++) {
    C->nnz.push_back(ci.nnz[k]);
    C->mats.push_back(std::vector<spg_sparse_entry>(ci.entries[k], ci.entries[k] + ci.nnz[k]));
  }
  int rc = spg_r1cs_inst_new(ctx, &ci, &C->dev);
  if (rc) {
    snark_comp_free(ctx, C);
    return rc;
  }
  // R1CSCommitmentGens::new(label, P_pad, num_cons, num_vars_pad, nnz) (lib.rs:164-185, r1csinstance.rs:39-56)
  const size_t Pg = npow2(si->gens_num_instances);
  const size_t gens_nvx = lg2(Pg) + lg2(si->gens_num_cons), gens_nvy = lg2(npow2(si->gens_num_vars));
  const size_t gens_nnz = Pg * si->gens_num_nz_entries;
  const size_t nvx = lg2(ci.max_num_cons), nvy = lg2(ci.num_vars);
  std::vector<std::vector<SparsePoly>> groups;
  if (multi) {  // R1CSInstance::multi_commit: group by next_power_of_eight(nnz) (r1csinstance.rs:654-715)
    std::vector<size_t> sizes;
    for (size_t k = 0; k < 3 * ci.num_instances; k++) {
      size_t len = 1;
      while (len < npow2(ci.nnz[k])) len *= 8;
      size_t idx = std::find(sizes.begin(), sizes.end(), len) - sizes.begin();
      if (idx == sizes.size()) {
        sizes.push_back(len);
        C->label_map.push_back({});
        groups.push_back({});
      }
      C->label_map[idx].push_back(k);
      groups[idx].push_back({C->mats[k].data(), C->nnz[k]});
    }
  } else {
    groups.push_back({});
    C->label_map.push_back({});
    for (size_t k = 0; k < 3 * ci.num_instances; k++) {
      C->label_map[0].push_back(k);
      groups[0].push_back({C->mats[k].data(), C->nnz[k]});
    }
  }
  static const char kLabel[] = "gens_r1cs_eval";
  for (auto& g : groups) {
    spg_spark* S = nullptr;
    rc = spark_commit_polys(ctx, g, nvx, nvy, (const uint8_t*)kLabel, sizeof(kLabel) - 1, gens_nvx, gens_nvy, gens_nnz, 3,
                            &S);
    if (rc) {
      snark_comp_free(ctx, C);
      return rc;
    }
    C->sparks.push_back(S);
  }
  *out = C;
  return SPG_OK;
}
extern "C" int spg_snark_comp_free(spg_ctx* ctx, spg_snark_comp* C) { return snark_comp_free(ctx, C); }

// bincode(Vec<ComputationCommitment>) (as_list) or bincode(ComputationCommitment) of an encoded instance:
// R1CSCommitment { num_cons: num_instances * max_num_cons, num_vars, comm } (src/r1csinstance.rs:60-64, 700-705)
extern "C" int spg_snark_comm_bytes(spg_ctx* ctx, const spg_snark_comp* C, int as_list, uint8_t* out, size_t cap,
                                    size_t* len) {
  if (!ctx || !C || !len || C->sparks.empty()) return SPG_E_ARG;
  if (!as_list && C->sparks.size() != 1) return set_err(ctx, SPG_E_ARG, "several commitments: ask for the list");
  Writer w;
  if (as_list) w.u64(C->sparks.size());
  for (const spg_spark* S : C->sparks) {
    w.u64(C->num_instances * C->max_num_cons);
    w.u64(C->num_vars);
    spark_comm_ser(S, w);
  }
  *len = w.out.size();
  if (!out || w.out.size() > cap) return set_err(ctx, SPG_E_ARG, "commitment buffer too small");
  memcpy(out, w.out.data(), w.out.size());
  return SPG_OK;
}

// block_comm_map (src/lib.rs:2781): list g holds the matrix indices 3p + m that commitment g covers
extern "C" int spg_snark_comm_map(spg_ctx* ctx, const spg_snark_comp* C, size_t* idx, size_t idx_cap, size_t* lens,
                                  size_t lens_cap, size_t* n_lists) {
  if (!ctx || !C || !n_lists) return SPG_E_ARG;
  *n_lists = C->label_map.size();
  size_t tot = 0;
  for (auto& l : C->label_map) tot += l.size();
  if (!idx || !lens || tot > idx_cap || C->label_map.size() > lens_cap) return set_err(ctx, SPG_E_ARG, "map buffer too small");
  size_t o = 0;
  for (size_t g = 0; g < C->label_map.size(); g++) {
    lens[g] = C->label_map[g].size();
    for (size_t k : C->label_map[g]) idx[o++] = k;
  }
  return SPG_OK;
}

namespace spg {
// what SNARK::verify reads of an encoded instance (verify.hip)
spg_snark_comp* snark_comp_from_parts(size_t num_instances, size_t max_num_cons, size_t num_vars,
                                      std::vector<std::vector<size_t>> label_map, std::vector<spg_spark*> sparks) {
  spg_snark_comp* C = new spg_snark_comp();
  C->num_instances = num_instances;
  C->max_num_cons = max_num_cons;
  C->num_vars = num_vars;
  C->label_map = std::move(label_map);
  C->sparks = std::move(sparks);
  return C;
}
int snark_comp_view(const spg_snark_comp* C, SnarkCompView* v) {
  if (!C || C->sparks.empty() || C->label_map.size() != C->sparks.size()) return SPG_E_ARG;
  v->num_instances = C->num_instances;
  v->max_num_cons = C->max_num_cons;
  v->num_vars = C->num_vars;
  v->label_map = &C->label_map;
  v->sparks = &C->sparks;
  return 0;
}
}  // namespace spg

extern "C" int spg_snark_witness_new(spg_ctx* ctx, const spg_snark_inputs* a, spg_snark_wit** out) {
  if (!ctx || !a || !out || !a->block_num_instances_bound || !a->num_inputs_unpadded || !a->num_ios) return SPG_E_ARG;
  spg_snark_wit* W = new spg_snark_wit();
  W->a = *a;
  const size_t B = a->block_num_instances_bound, io = 2 * a->num_inputs_unpadded;
  W->liveness.assign(a->input_liveness, a->input_liveness + a->input_len);
  for (size_t i = 0; i < a->input_len; i++) W->input.push_back(ld_fq(a->input + 4 * i));
  W->output = ld_fq(a->output);
  W->phy_ops.assign(a->block_num_phy_ops, a->block_num_phy_ops + B);
  W->vir_ops.assign(a->block_num_vir_ops, a->block_num_vir_ops + B);
  W->nvars.assign(a->block_num_vars, a->block_num_vars + B);
  W->nproofs.assign(a->block_num_proofs, a->block_num_proofs + B);
  auto rows = [](const uint64_t* p, size_t n, size_t w, size_t keep) {
    Rows m(n, FqV(keep));
    for (size_t q = 0; q < n; q++)
      for (size_t i = 0; i < keep; i++) m[q][i] = ld_fq(p + 4 * (q * w + i));
    return m;
  };
  auto fail = [&](int rc, const char* msg) {
    h2d_sync(ctx);
    for (size_t i = 0; i < W->d_block_vars.size(); i++) dev_cache_put(ctx, W->d_block_vars[i], W->d_block_bytes[i]);
    hipFree(W->d_exec);
    delete W;
    return set_err(ctx, rc, msg);
  };
  // block_vars[i] is the witness list of the i-th instance in the prover's sort order (num_proofs descending,
  // ties in block order; lib.rs:1155-1178): the reference pairs block_vars_mat[i] with sorted instance i, so list
  // i holds num_proofs[order[i]] rows of num_vars[order[i]] entries
  std::vector<size_t> order(B);
  for (size_t i = 0; i < B; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return W->nproofs[x] > W->nproofs[y]; });
  for (size_t i = 0; i < B; i++) {
    const size_t b = order[i], n = W->nproofs[b], w = W->nvars[b];
    if (n && !a->block_vars[i]) return fail(SPG_E_ARG, "missing block_vars");
    // the io part of every row (and the memory-op part the w2 recurrences read)
    const size_t keep = std::min(w, io + 2 * W->phy_ops[b] + 4 * W->vir_ops[b]);
    W->block_io.push_back(n ? rows(a->block_vars[i], n, w, keep) : Rows());
    // resident copy, padded to next_pow2(num_proofs) rows of zeros (lib.rs:1209-1216)
    Fq* d = nullptr;
    const size_t rows_p = npow2(std::max<size_t>(n, 1));
    if (!(d = (Fq*)dev_cache_get(ctx, rows_p * w * sizeof(Fq) + 64))) return fail(SPG_E_NOMEM, "block_vars");
    W->d_block_vars.push_back(d);
    W->d_block_bytes.push_back(rows_p * w * sizeof(Fq) + 64);
    // the padding rows zeroed on the context stream, the rows themselves streamed (h2d_stream: page-locked ring, host
    // pool copies, DMA on the upload stream; disjoint bytes, and the context stream waits for the DMAs)
    if (rows_p > n && hipMemsetAsync(d + n * w, 0, (rows_p - n) * w * sizeof(Fq), ctx->stream) != hipSuccess)
      return fail(SPG_E_HIP, "block_vars upload");
    if (n) {
      const int rc = h2d_stream(ctx, d, a->block_vars[i], n * w * sizeof(Fq));
      if (rc) return fail(rc, "block_vars upload");
    }
  }
  const size_t ce = npow2(a->consis_num_proofs);
  W->exec = rows(a->exec_inputs, a->consis_num_proofs, a->num_ios, a->num_ios);
  W->exec.resize(ce, FqV(a->num_ios, fq_zero()));
  {
    FqV f = flatten(W->exec);
    if (hipMalloc(&W->d_exec, f.size() * sizeof(Fq) + 64) != hipSuccess) return fail(SPG_E_NOMEM, "exec inputs");
    if (hipMemcpy(W->d_exec, f.data(), f.size() * sizeof(Fq), hipMemcpyHostToDevice) != hipSuccess)
      return fail(SPG_E_HIP, "exec inputs upload");
  }
  if (a->total_num_init_phy_mem_accesses)
    W->init_phy = rows(a->init_phy_mems, a->total_num_init_phy_mem_accesses, INIT_PHY_MEM_WIDTH, INIT_PHY_MEM_WIDTH);
  if (a->total_num_init_vir_mem_accesses)
    W->init_vir = rows(a->init_vir_mems, a->total_num_init_vir_mem_accesses, INIT_VIR_MEM_WIDTH, INIT_VIR_MEM_WIDTH);
  if (a->total_num_phy_mem_accesses)
    W->addr_phy = rows(a->addr_phy_mems, a->total_num_phy_mem_accesses, PHY_MEM_WIDTH, PHY_MEM_WIDTH);
  if (a->total_num_vir_mem_accesses) {
    W->addr_vir = rows(a->addr_vir_mems, a->total_num_vir_mem_accesses, VIR_MEM_WIDTH, VIR_MEM_WIDTH);
    W->ts_bits = rows(a->addr_ts_bits, a->total_num_vir_mem_accesses, a->mem_addr_ts_bits_size, a->mem_addr_ts_bits_size);
  }
  // (no synchronisation: the streamed DMAs complete on their own, ahead of everything later on the context stream)
  *out = W;
  return SPG_OK;
}
extern "C" int spg_snark_witness_free(spg_ctx* ctx, spg_snark_wit* W) {
  if (!W) return SPG_OK;
  if (ctx) {
    h2d_sync(ctx);  // a streamed upload into it may still be in flight
    for (size_t i = 0; i < W->d_block_vars.size(); i++) dev_cache_put(ctx, W->d_block_vars[i], W->d_block_bytes[i]);
  } else {
    for (auto* d : W->d_block_vars) hipFree(d);
  }
  hipFree(W->d_exec);
  delete W;
  return SPG_OK;
}

namespace {

struct MemGen {  // SNARK::mem_gen output (lib.rs:831-968)
  std::vector<Rows> w2, w3, w3s;
  std::vector<FqV> p2, p3, p3s;
  std::vector<Pt> c2, c3, c3s;
  SecInfo s2, s3, s3s;
};
int mem_gen(size_t width, Rows mems, size_t total, const Fq& r, const Fq& tau, bool vir, CQ& q, MemGen* o) {
  if (total == 0) return 0;
  Rows w2(total, FqV(width, fq_zero())), w3(total, FqV(W3_WIDTH, fq_zero()));
  const Fq r2 = fq_mul(r, r), r3 = fq_mul(r2, r);
  for (size_t q = 0; q < total; q++) {
    w2[q][3] = fq_mul(r, mems[q][3]);
    if (vir) {
      w2[q][4] = fq_mul(r2, mems[q][4]);
      w2[q][5] = fq_mul(r3, mems[q][5]);
    }
  }
  for (size_t q = total; q-- > 0;) {
    Fq rest = w2[q][3];
    if (vir) rest = fq_add(fq_add(rest, w2[q][4]), w2[q][5]);
    w3[q][0] = mems[q][0];
    w3[q][1] = fq_mul(mems[q][0], fq_sub(fq_sub(tau, mems[q][2]), rest));
    w3[q][3] = q != total - 1 ? fq_mul(w3[q][1], fq_sub(fq_add(w3[q + 1][2], fq_one()), w3[q + 1][0])) : w3[q][1];
    w3[q][2] = fq_mul(w3[q][0], w3[q][3]);
    w3[q][4] = fq_mul(mems[q][0], fq_add(fq_add(mems[q][0], mems[q][2]), rest));
    w3[q][5] = mems[q][0];
  }
  o->w2 = {w2};
  o->w3 = {w3};
  o->w3s = {shift_rows(w3, W3_WIDTH)};
  o->p2 = {pad_pow2(flatten(o->w2[0]))};
  o->p3 = {pad_pow2(flatten(o->w3[0]))};
  o->p3s = {pad_pow2(flatten(o->w3s[0]))};
  q.add(o->p2[0], &o->c2);
  q.add(o->p3[0], &o->c3);
  q.add(o->p3s[0], &o->c3s);
  o->s2 = host_sec(o->w2, o->p2);
  o->s3 = host_sec(o->w3, o->p3);
  o->s3s = host_sec(o->w3s, o->p3s);
  return 0;
}

}  // namespace

static int spg_snark_prove_impl(spg_ctx* ctx, spg_snark_comp* block, spg_snark_comp* pairwise, spg_snark_comp* perm_root,
                               const spg_snark_wit* W, spg_r1cs_gens* vars_gens, spg_transcript* transcript,
                               spg_random_tape* tape_h, uint8_t* proof, size_t proof_cap, size_t* proof_len) {
  if (!ctx || !block || !pairwise || !perm_root || !W || !vars_gens || !transcript || !tape_h || !proof_len)
    return SPG_E_ARG;
  Tr& t = transcript->t;
  Tape& tape = tape_h->t;
  ProverGens& g = vars_gens->g;
  const spg_snark_inputs& a = W->a;
  const size_t niu = a.num_inputs_unpadded, num_ios = a.num_ios, io_width = 2 * niu;
  const size_t Bb = a.block_num_instances_bound;
  if (2 * niu > num_ios) return set_err(ctx, SPG_E_ARG, "num_ios < 2 * num_inputs_unpadded");
  Laps lp;
  lp.title = "SNARK::prove";
  t.protocol("Spartan SNARK proof");
  const bool dbg0 = getenv("SPG_DEBUG_SNARK") != nullptr;
  auto fp = [&](const char* where) {
    if (!dbg0 || t.cb) return;  // (a fork of a caller-backed transcript cannot be taken)
    Tr c = t;
    Fq x = c.challenge("dbg");
    fprintf(stderr, "fp %s %08x\n", where, x.l[0]);
  };
  // ---- INSTANCE COMMITMENTS (lib.rs:1086-1153)
  auto app = [&](const char* l, size_t v) { t.scalar(l, fq_from_u64(v)); };
  app("func_input_width", a.func_input_width);
  app("input_offset", a.input_offset);
  app("output_offset", a.output_offset);
  app("output_exec_num", a.output_exec_num);
  app("num_ios", num_ios);
  for (size_t b = 0; b < Bb; b++) app("block_num_vars", W->nvars[b]);
  app("mem_addr_ts_bits_size", a.mem_addr_ts_bits_size);
  app("num_inputs_unpadded", niu);
  app("block_num_instances_bound", Bb);
  app("block_max_num_proofs", a.block_max_num_proofs);
  for (size_t b = 0; b < Bb; b++) app("block_num_phy_ops", W->phy_ops[b]);
  for (size_t b = 0; b < Bb; b++) app("block_num_vir_ops", W->vir_ops[b]);
  app("total_num_init_phy_mem_accesses", a.total_num_init_phy_mem_accesses);
  app("total_num_init_vir_mem_accesses", a.total_num_init_vir_mem_accesses);
  app("total_num_phy_mem_accesses", a.total_num_phy_mem_accesses);
  app("total_num_vir_mem_accesses", a.total_num_vir_mem_accesses);
  app("block_max_num_proofs", a.block_max_num_proofs);
  for (size_t b = 0; b < Bb; b++) app("block_num_proofs", W->nproofs[b]);
  fp("params");
  for (auto& lm : block->label_map)
    for (auto l : lm) app("block_comm_map", l);
  fp("map");
  for (size_t gi = 0; gi < block->sparks.size(); gi++) append_r1cs_comm(block, gi, t);
  fp("block");
  append_r1cs_comm(pairwise, 0, t);
  fp("pairwise");
  append_r1cs_comm(perm_root, 0, t);
  fp("perm_root");
  const Fq input_block_num = fq_from_u64(a.input_block_num), output_block_num = fq_from_u64(a.output_block_num);
  t.scalar("input_block_num", input_block_num);
  t.scalar("output_block_num", output_block_num);
  t.scalars("input_list", W->input);
  t.scalar("output_list", W->output);

  // ---- BLOCK SORT + PADDING (lib.rs:1155-1273)
  size_t P = 0;
  for (auto n : W->nproofs)
    if (n > 0) P++;
  std::vector<size_t> order(Bb);
  for (size_t i = 0; i < Bb; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return W->nproofs[x] > W->nproofs[y]; });
  order.resize(P);
  // block_vars_mat[i] pairs with sorted instance i (the reference never permutes the witness list)
  std::vector<size_t> bnp(P), bnv(P), bphy(P), bvir(P);
  for (size_t i = 0; i < P; i++) {
    bnp[i] = W->nproofs[order[i]];
    bnv[i] = W->nvars[order[i]];
    bphy[i] = W->phy_ops[order[i]];
    bvir[i] = W->vir_ops[order[i]];
  }
  const size_t bmax = npow2(a.block_max_num_proofs);
  std::vector<size_t> bnp_pad(P);
  for (size_t i = 0; i < P; i++) bnp_pad[i] = npow2(bnp[i]);
  const size_t consis = npow2(a.consis_num_proofs);
  auto padded = [](size_t n) { return n ? npow2(n) : 0; };
  const size_t t_iphy = padded(a.total_num_init_phy_mem_accesses), t_ivir = padded(a.total_num_init_vir_mem_accesses),
               t_phy = padded(a.total_num_phy_mem_accesses), t_vir = padded(a.total_num_vir_mem_accesses);
  auto pad_rows = [](Rows m, size_t n, size_t w) {
    m.resize(n, FqV(w, fq_zero()));
    return m;
  };
  Rows init_phy = pad_rows(W->init_phy, t_iphy, INIT_PHY_MEM_WIDTH), init_vir = pad_rows(W->init_vir, t_ivir, INIT_VIR_MEM_WIDTH),
       addr_phy = pad_rows(W->addr_phy, t_phy, PHY_MEM_WIDTH), addr_vir = pad_rows(W->addr_vir, t_vir, VIR_MEM_WIDTH),
       ts_bits = pad_rows(W->ts_bits, t_vir, a.mem_addr_ts_bits_size);
  int rc = ensure_sorted(ctx, block, order);
  if (rc) return rc;
  // PAIRWISE SORT (lib.rs:1275-1296)
  std::vector<std::pair<size_t, size_t>> ps = {{consis, 0}, {t_phy, 1}, {t_vir, 2}};
  std::stable_sort(ps.begin(), ps.end(), [](const std::pair<size_t, size_t>& x, const std::pair<size_t, size_t>& y) {
    return x.first > y.first;
  });
  const size_t pw_inst = 1 + (t_phy > 0) + (t_vir > 0);
  std::vector<size_t> pw_order;
  for (size_t i = 0; i < pw_inst; i++) pw_order.push_back(ps[i].second);
  rc = ensure_sorted(ctx, pairwise, pw_order);
  if (rc) return rc;

  lp.lap("inst_commit+sort");
  CQ cq;
  {  // block_vars commitments: on the device now, read back when the queue is flushed
    std::vector<std::pair<const Fq*, size_t>> bv;
    for (size_t p = 0; p < P; p++) bv.push_back({W->d_block_vars[p], bnp_pad[p] * bnv[p]});
    if ((rc = cq.launch_early(ctx, g, bv))) return rc;
  }
  // ---- WITNESS GEN: block (lib.rs:1299-1741)
  const Fq tau = t.challenge("challenge_tau"), r = t.challenge("challenge_r");
  if (getenv("SPG_DEBUG_TR")) fprintf(stderr, "[prove] tau %08x r %08x\n", tau.l[0], r.l[0]);
  const bool dbg = getenv("SPG_DEBUG_SNARK") != nullptr;
  if (dbg) fprintf(stderr, "snark tau %08x %08x r %08x\n", tau.l[0], tau.l[1], r.l[0]);
  FqV perm_w0 = {tau};
  {
    Fq rt = r;
    for (size_t i = 1; i < 2 * niu; i++) {
      perm_w0.push_back(rt);
      rt = fq_mul(rt, r);
    }
    perm_w0.resize(num_ios, fq_zero());
  }
  std::vector<Pt> c_w0;
  cq.add(perm_w0, &c_w0);
  const Rows& exec = W->exec;
  Rows pe_w2(consis), pe_w3(consis);
  // rows are independent except the reverse-q recurrence of w3[3] (and w3[2]): the per-row work runs on the
  // host pool in chunks, the recurrence (2 products per row) afterwards in order
  auto par_rows = [](size_t n, const std::function<void(size_t)>& f) {
    const int C = n >= 64 ? 8 : 1;
    pool().parallel_for(C, [&](int c) {
      for (size_t q = n * c / C; q < n * (c + 1) / C; q++) f(q);
    });
  };
  par_rows(consis, [&](size_t q) {
    FqV v(3, fq_zero());
    for (size_t j = 1; j < 2 * niu - 2; j++) v.push_back(fq_mul(perm_w0[j], exec[q][j + 2]));
    v.resize(num_ios, fq_zero());
    v[0] = exec[q][0];
    v[1] = exec[q][0];
    for (size_t i = 0; i + 1 < niu; i++) {
      const Fq perm = i == 0 ? fq_one() : perm_w0[i];
      v[0] = fq_add(v[0], fq_mul(perm, exec[q][2 + i]));
      v[2] = fq_add(v[2], fq_mul(perm, exec[q][2 + (niu - 1) + i]));
    }
    v[0] = fq_mul(v[0], exec[q][0]);
    v[1] = fq_mul(fq_add(v[1], v[2]), exec[q][0]);
    FqV w(8, fq_zero());
    w[0] = exec[q][0];
    Fq sacc = fq_zero();
    for (size_t k = 3; k < v.size(); k++) sacc = fq_add(sacc, v[k]);
    w[1] = fq_mul(w[0], fq_sub(fq_sub(tau, sacc), exec[q][2]));
    w[4] = v[0];
    w[5] = v[1];
    pe_w2[q] = std::move(v);
    pe_w3[q] = std::move(w);
  });
  for (size_t q = consis; q-- > 0;) {
    FqV& w = pe_w3[q];
    w[3] = q != consis - 1 ? fq_mul(w[1], fq_sub(fq_add(pe_w3[q + 1][2], fq_one()), pe_w3[q + 1][0])) : w[1];
    w[2] = fq_mul(w[0], w[3]);
  }
  std::vector<Rows> pe_w2v = {pe_w2}, pe_w3v = {pe_w3}, pe_w3sv = {shift_rows(pe_w3, 8)};
  std::vector<FqV> pe_p2 = {pad_pow2(flatten(pe_w2))}, pe_p3 = {pad_pow2(flatten(pe_w3))},
                   pe_p3s = {pad_pow2(flatten(pe_w3sv[0]))};
  if (dbg)
    for (size_t q = 0; q < 2; q++)
      for (size_t i = 0; i < num_ios; i++) fprintf(stderr, "pe_w2[%zu][%zu] %08x\n", q, i, pe_w2[q][i].l[0]);
  lp.lap("perm_exec_witness");
  std::vector<Pt> c_pe2, c_pe3, c_pe3s;
  cq.add(pe_p2[0], &c_pe2);
  cq.add(pe_p3[0], &c_pe3);
  cq.add(pe_p3s[0], &c_pe3s);

  lp.lap("perm_exec_commit");
  std::vector<Rows> b_w2(P), b_w3(P), b_w3s(P);
  const Fq r2 = fq_mul(r, r), r3 = fq_mul(r2, r);
  for (size_t p = 0; p < P; p++) {
    const size_t np_ = bphy[p], nv_ = bvir[p], Q = bnp_pad[p];
    const size_t w2_size = npow2(2 * niu + 2 * np_ + 4 * nv_);
    const Rows& bio = W->block_io[p];
    const size_t keep = bio.empty() ? 0 : bio[0].size();
    b_w2[p].assign(Q, FqV());
    b_w3[p].assign(Q, FqV());
    FqV zero_row(keep, fq_zero());
    std::vector<Fq> pxs(Q), vxs(Q);  // the chain ends read by the reverse-q recurrences
    par_rows(Q, [&](size_t q) {  // everything of row q that does not depend on row q + 1
      const FqV& bv = q < bio.size() ? bio[q] : zero_row;
      const Fq V_CNST = bv[0];
      FqV w2(w2_size, fq_zero());
      w2[0] = bv[0];
      w2[1] = bv[0];
      for (size_t i = 1; i < 2 * (niu - 1); i++) w2[2 + i] = fq_add(w2[2 + i], fq_mul(perm_w0[i], bv[i + 2]));
      for (size_t i = 0; i + 1 < niu; i++) {
        const Fq perm = i == 0 ? fq_one() : perm_w0[i];
        w2[0] = fq_add(w2[0], fq_mul(perm, bv[2 + i]));
        w2[2] = fq_add(w2[2], fq_mul(perm, bv[2 + (niu - 1) + i]));
      }
      w2[0] = fq_mul(w2[0], bv[0]);
      w2[1] = fq_mul(fq_add(w2[1], w2[2]), bv[0]);
      FqV w3(8, fq_zero());
      w3[0] = bv[0];
      Fq sacc = fq_zero();
      for (size_t k = 3; k < w2.size(); k++) sacc = fq_add(sacc, w2[k]);
      w3[1] = fq_mul(w3[0], fq_sub(fq_sub(tau, sacc), bv[2]));
      for (size_t i = 0; i < np_; i++) {
        const size_t PMR = 2 * niu + 2 * i, PMC = PMR + 1;
        w2[PMR] = fq_mul(r, bv[io_width + 2 * i + 1]);
        const Fq tt = i == 0 ? V_CNST : w2[PMC - 2];
        w2[PMC] = fq_mul(tt, fq_sub(fq_sub(tau, bv[io_width + 2 * i]), w2[PMR]));
      }
      pxs[q] = np_ == 0 ? V_CNST : w2[2 * niu + 2 * (np_ - 1) + 1];
      for (size_t i = 0; i < nv_; i++) {
        const size_t base = 2 * niu + 2 * np_ + 4 * i, vb = io_width + 2 * np_ + 4 * i;
        w2[base] = fq_mul(r, bv[vb + 1]);
        w2[base + 1] = fq_mul(r2, bv[vb + 2]);
        w2[base + 2] = fq_mul(r3, bv[vb + 3]);
        const Fq tt = i == 0 ? V_CNST : w2[base - 1];
        w2[base + 3] = fq_mul(tt, fq_sub(fq_sub(fq_sub(fq_sub(tau, bv[vb]), w2[base]), w2[base + 1]), w2[base + 2]));
      }
      vxs[q] = nv_ == 0 ? V_CNST : w2[2 * niu + 2 * np_ + 4 * (nv_ - 1) + 3];
      b_w2[p][q] = std::move(w2);
      b_w3[p][q] = std::move(w3);
    });
    for (size_t q = Q; q-- > 0;) {  // the reverse-q recurrences (src/lib.rs:1539-1611)
      FqV& w3 = b_w3[p][q];
      const Fq V_CNST = w3[0];
      const FqV* nx = q != Q - 1 ? &b_w3[p][q + 1] : nullptr;
      w3[3] = nx ? fq_mul(w3[1], fq_sub(fq_add((*nx)[2], fq_one()), (*nx)[0])) : w3[1];
      w3[2] = fq_mul(w3[0], w3[3]);
      w3[5] = nx ? fq_mul(pxs[q], fq_sub(fq_add((*nx)[4], fq_one()), (*nx)[0])) : pxs[q];
      w3[4] = fq_mul(V_CNST, w3[5]);
      w3[7] = nx ? fq_mul(vxs[q], fq_sub(fq_add((*nx)[6], fq_one()), (*nx)[0])) : vxs[q];
      w3[6] = fq_mul(V_CNST, w3[7]);
    }
    b_w3s[p] = shift_rows(b_w3[p], 8);
  }
  lp.lap("block_witness");
  std::vector<FqV> b_p2(P), b_p3(P), b_p3s(P);
  std::vector<std::vector<Pt>> c_b2(P), c_b3(P), c_b3s(P), c_bv(P);
  for (size_t p = 0; p < P; p++) {
    b_p2[p] = pad_pow2(flatten(b_w2[p]));
    cq.add(b_p2[p], &c_b2[p]);
  }
  for (size_t p = 0; p < P; p++) {
    b_p3[p] = pad_pow2(flatten(b_w3[p]));
    b_p3s[p] = pad_pow2(flatten(b_w3s[p]));
    cq.add(b_p3[p], &c_b3[p]);
    cq.add(b_p3s[p], &c_b3s[p]);
  }
  lp.lap("block_w_commit");
  // ---- memory witnesses (lib.rs:1742-1955)
  MemGen m_iphy, m_ivir, m_phy, m_vir;
  mem_gen(INIT_PHY_MEM_WIDTH, init_phy, t_iphy, r, tau, false, cq, &m_iphy);
  mem_gen(INIT_VIR_MEM_WIDTH, init_vir, t_ivir, r, tau, false, cq, &m_ivir);
  mem_gen(PHY_MEM_WIDTH, addr_phy, t_phy, r, tau, false, cq, &m_phy);
  mem_gen(VIR_MEM_WIDTH, addr_vir, t_vir, r, tau, true, cq, &m_vir);
  lp.lap("mem_gen");
  // ---- WITNESS COMMITMENTS (lib.rs:1957-2221): block_vars and exec inputs from HBM
  for (size_t p = 0; p < P; p++) cq.add_dev(W->d_block_vars[p], bnp_pad[p] * bnv[p], &c_bv[p]);
  std::vector<Pt> c_exec;
  cq.add_dev(W->d_exec, consis * num_ios, &c_exec);
  std::vector<FqV> p_iphy, p_ivir, p_aphy, p_aphys, p_avir, p_avirs, p_ts;
  std::vector<Rows> r_aphys, r_avirs;
  std::vector<Pt> c_aphy, c_aphys, c_avir, c_avirs, c_ts, c_iphy_in, c_ivir_in;
  if (t_iphy) {
    p_iphy = {pad_pow2(flatten(init_phy))};
    cq.add(p_iphy[0], &c_iphy_in);
  }
  if (t_ivir) {
    p_ivir = {pad_pow2(flatten(init_vir))};
    cq.add(p_ivir[0], &c_ivir_in);
  }
  if (t_phy) {
    p_aphy = {pad_pow2(flatten(addr_phy))};
    cq.add(p_aphy[0], &c_aphy);
    r_aphys = {shift_rows(addr_phy, PHY_MEM_WIDTH)};
    p_aphys = {pad_pow2(flatten(r_aphys[0]))};
    cq.add(p_aphys[0], &c_aphys);
  }
  if (t_vir) {
    p_avir = {pad_pow2(flatten(addr_vir))};
    cq.add(p_avir[0], &c_avir);
    r_avirs = {shift_rows(addr_vir, VIR_MEM_WIDTH)};
    p_avirs = {pad_pow2(flatten(r_avirs[0]))};
    cq.add(p_avirs[0], &c_avirs);
    p_ts = {pad_pow2(flatten(ts_bits))};
    cq.add(p_ts[0], &c_ts);
  }
  if ((rc = cq.flush(ctx, g, t))) return rc;
  lp.lap("input_commit");
  // witness sections
  std::vector<FqV> w0v = {perm_w0};
  SecInfo s_w0 = host_sec({{perm_w0}}, w0v);
  SecInfo s_bvars;
  for (size_t p = 0; p < P; p++) {
    s_bvars.num_proofs.push_back(bnp_pad[p]);
    s_bvars.num_inputs.push_back(bnv[p]);
    s_bvars.src.push_back(W->d_block_vars[p]);
    s_bvars.poly.push_back(nullptr);
  }
  SecInfo s_bw2 = host_sec(b_w2, b_p2), s_bw3 = host_sec(b_w3, b_p3), s_bw3s = host_sec(b_w3s, b_p3s);
  SecInfo s_pe2 = host_sec(pe_w2v, pe_p2), s_pe3 = host_sec(pe_w3v, pe_p3), s_pe3s = host_sec(pe_w3sv, pe_p3s);
  SecInfo s_exec;
  s_exec.num_proofs = {consis};
  s_exec.num_inputs = {num_ios};
  s_exec.src = {W->d_exec};
  s_exec.poly = {nullptr};
  SecInfo s_none, s_iphy, s_ivir, s_aphy, s_aphys, s_avir, s_avirs, s_ts;
  if (t_iphy) s_iphy = host_sec({init_phy}, p_iphy);
  if (t_ivir) s_ivir = host_sec({init_vir}, p_ivir);
  if (t_phy) {
    s_aphy = host_sec({addr_phy}, p_aphy);
    s_aphys = host_sec(r_aphys, p_aphys);
  }
  if (t_vir) {
    s_avir = host_sec({addr_vir}, p_avir);
    s_avirs = host_sec(r_avirs, p_avirs);
    s_ts = host_sec({ts_bits}, p_ts);
  }
  spg_r1cs_witness* Wt = ctx->wt_cache;  // refilled in place (witness_from_parts) when large enough
  ctx->wt_cache = nullptr;
  struct WGuard {
    spg_ctx* c;
    spg_r1cs_witness** w;
    ~WGuard() {
      if (!c->wt_cache) c->wt_cache = *w;
      else spg_r1cs_witness_free(c, *w);
    }
  } guard{ctx, &Wt};

  Writer w;  // bincode(SNARK) in declaration order (lib.rs:701-756)
  w.u64(P);
  for (auto& c : c_bv) w.pts(c);
  w.u64(1);
  w.pts(c_exec);
  w.pts(c_aphy);
  w.pts(c_aphys);
  w.pts(c_avir);
  w.pts(c_avirs);
  w.pts(c_ts);
  w.pts(c_pe2);
  w.pts(c_pe3);
  w.pts(c_pe3s);
  for (auto* L : {&c_b2, &c_b3, &c_b3s}) {
    w.u64(P);
    for (auto& c : *L) w.pts(c);
  }
  for (auto* M : {&m_iphy, &m_ivir, &m_phy, &m_vir}) {
    w.pts(M->c2);
    w.pts(M->c3);
    w.pts(M->c3s);
  }

  // ---- BLOCK_CORRECTNESS_EXTRACT (lib.rs:2223-2309)
  SatOut so;
  rc = sat_prove(ctx, vars_gens, block->dev_sorted, P, bmax, bnp_pad, a.num_vars, bnv,
                 {wpart(s_bvars), wpart(s_w0), wpart(s_bw2), wpart(s_bw3), wpart(s_bw3s)}, &Wt, transcript, tape_h, &so);
  if (rc) return rc;
  lp.lap("block_sat");
  w.out.insert(w.out.end(), so.bytes.begin(), so.bytes.end());
  {
    FqV list;
    Fq brp[3];
    if ((rc = multi_eval(ctx, block, so.ch[2], so.ch[3], &list))) return rc;
    bound_rp(list, order, so.ch[0], brp);
    for (auto& e : list) t.scalar("ABCr_claim", e);
    t.challenge("challenge_c0");
    t.challenge("challenge_c1");
    t.challenge("challenge_c2");
    for (int k = 0; k < 3; k++) w.fq(brp[k]);
    w.fqs(list);
    w.u64(block->sparks.size());
    for (size_t gi = 0; gi < block->sparks.size(); gi++) {
      FqV ev;
      for (auto l : block->label_map[gi]) ev.push_back(list[l]);
      if ((rc = spark_prove_core(ctx, block->sparks[gi], so.ch[2], so.ch[3], ev, t, tape, w))) return rc;
    }
  }
  lp.lap("block_eval");
  // ---- PAIRWISE_CHECK (lib.rs:2311-2424)
  {
    const size_t pairwise_size = std::max({consis, t_phy, t_vir});
    std::vector<size_t> im, im2;
    SecInfo pw = merge({&s_pe3, &s_aphy, &s_avir}, &im);
    SecInfo pws = merge({&s_pe3s, &s_aphys, &s_avirs}, &im2);
    std::vector<const SecInfo*> comps(im.size(), &s_w0);
    for (size_t i = 0; i < im.size(); i++)
      if (im[i] == 2) comps[i] = &s_ts;
    SecInfo tsb = concat(comps);
    const size_t pw_nv = std::max<size_t>(8, a.mem_addr_ts_bits_size);
    rc = sat_prove(ctx, vars_gens, pairwise->dev_sorted, pw.num_proofs.size(), pairwise_size, pw.num_proofs, pw_nv,
                   std::vector<size_t>(pw.num_proofs.size(), pw_nv), {wpart(pw), wpart(pws), wpart(tsb)}, &Wt,
                   transcript, tape_h, &so);
    if (rc) return rc;
    w.out.insert(w.out.end(), so.bytes.begin(), so.bytes.end());
    FqV list;
    Fq brp[3];
    if ((rc = multi_eval(ctx, pairwise, so.ch[2], so.ch[3], &list))) return rc;
    bound_rp(list, pw_order, so.ch[0], brp);
    for (auto& e : list) t.scalar("ABCr_claim", e);
    t.challenge("challenge_c0");
    t.challenge("challenge_c1");
    t.challenge("challenge_c2");
    for (int k = 0; k < 3; k++) w.fq(brp[k]);
    w.fqs(list);
    if ((rc = spark_prove_core(ctx, pairwise->sparks[0], so.ch[2], so.ch[3], list, t, tape, w))) return rc;
  }
  lp.lap("pairwise");
  // ---- PERM_ROOT (lib.rs:2426-2532)
  {
    const size_t perm_size = std::max({consis, t_iphy, t_ivir, t_phy, t_vir});
    std::vector<size_t> m1, m2, m3, m4;
    SecInfo w1 = merge({&s_exec, &s_iphy, &s_ivir, &s_aphy, &s_avir}, &m1);
    SecInfo w2s = merge({&s_pe2, &m_iphy.s2, &m_ivir.s2, &m_phy.s2, &m_vir.s2}, &m2);
    SecInfo w3s_ = merge({&s_pe3, &m_iphy.s3, &m_ivir.s3, &m_phy.s3, &m_vir.s3}, &m3);
    SecInfo w4 = merge({&s_pe3s, &m_iphy.s3s, &m_ivir.s3s, &m_phy.s3s, &m_vir.s3s}, &m4);
    std::vector<size_t> pr_np = w1.num_proofs;
    rc = sat_prove(ctx, vars_gens, perm_root->dev, pr_np.size(), perm_size, pr_np, num_ios,
                   std::vector<size_t>(pr_np.size(), num_ios), {wpart(s_w0), wpart(w1), wpart(w2s), wpart(w3s_), wpart(w4)},
                   &Wt, transcript, tape_h, &so);
    if (rc) return rc;
    w.out.insert(w.out.end(), so.bytes.begin(), so.bytes.end());
    FqV e;
    if ((rc = multi_eval(ctx, perm_root, so.ch[2], so.ch[3], &e))) return rc;
    t.scalar("Ar_claim", e[0]);
    t.scalar("Br_claim", e[1]);
    t.scalar("Cr_claim", e[2]);
    for (int k = 0; k < 3; k++) w.fq(e[k]);
    if ((rc = spark_prove_core(ctx, perm_root->sparks[0], so.ch[2], so.ch[3], FqV(e.begin(), e.begin() + 3), t, tape,
                               w)))
      return rc;
  }
  lp.lap("perm_root");
  // ---- PERM_PRODUCT_PROOF (lib.rs:2534-2609)
  {
    std::vector<const SecInfo*> comps = {&s_pe3, &m_iphy.s3, &m_ivir.s3, &m_phy.s3, &m_vir.s3, &s_bw3};
    if (a.max_block_num_phy_ops > 0) comps.push_back(&s_bw3);
    if (a.max_block_num_vir_ops > 0) comps.push_back(&s_bw3);
    std::vector<size_t> im;
    SecInfo pw3 = merge(comps, &im);
    const size_t pm_bl_id = 6, vm_bl_id = a.max_block_num_phy_ops > 0 ? 7 : 6;
    FqV prod;
    std::vector<FqV> r_list;
    for (size_t i = 0; i < im.size(); i++) {
      const FqV& p = *pw3.poly[i];
      if (im[i] == vm_bl_id) {
        prod.push_back(p[6]);
        r_list.push_back({fq_one(), fq_one(), fq_zero()});
      } else if (im[i] == pm_bl_id) {
        prod.push_back(p[4]);
        r_list.push_back({fq_one(), fq_zero(), fq_zero()});
      } else {
        prod.push_back(p[2]);
        r_list.push_back({fq_one(), fq_zero()});
      }
    }
    w.fqs(prod);
    if ((rc = prove_batched_instances(ctx, g, pw3.poly, r_list, prod, t, tape, w))) return rc;
  }
  lp.lap("perm_product");
  // ---- SHIFT_PROOFS (lib.rs:2611-2668)
  {
    std::vector<const FqV*> orig = {&pe_p3[0]}, shifted = {&pe_p3s[0]};
    std::vector<size_t> hl = {6};
    for (size_t p = 0; p < P; p++) {
      orig.push_back(&b_p3[p]);
      shifted.push_back(&b_p3s[p]);
      hl.push_back(8);
    }
    if (t_iphy) {
      orig.push_back(&m_iphy.p3[0]);
      shifted.push_back(&m_iphy.p3s[0]);
      hl.push_back(6);
    }
    if (t_ivir) {
      orig.push_back(&m_ivir.p3[0]);
      shifted.push_back(&m_ivir.p3s[0]);
      hl.push_back(6);
    }
    if (t_phy) {
      orig.push_back(&p_aphy[0]);
      shifted.push_back(&p_aphys[0]);
      hl.push_back(4);
      orig.push_back(&m_phy.p3[0]);
      shifted.push_back(&m_phy.p3s[0]);
      hl.push_back(6);
    }
    if (t_vir) {
      orig.push_back(&p_avir[0]);
      shifted.push_back(&p_avirs[0]);
      hl.push_back(6);
      orig.push_back(&m_vir.p3[0]);
      shifted.push_back(&m_vir.p3s[0]);
      hl.push_back(6);
    }
    const size_t n = orig.size();
    std::vector<std::vector<Pt>> openings(n);
    {
      std::vector<CJob> jobs;
      for (size_t p = 0; p < n; p++)
        for (size_t i = 0; i < hl[p]; i++) jobs.push_back(CJob(g.gens_1, {(*orig[p])[i]}, fq_zero()));
      std::vector<Pt> pts = commit_batch(g, jobs);
      size_t k = 0;
      for (size_t p = 0; p < n; p++)
        for (size_t i = 0; i < hl[p]; i++) {
          t.point("shift_header_entry", pts[k]);
          openings[p].push_back(pts[k++]);
        }
    }
    const Fq c = t.challenge("challenge_c");
    // the evaluations sum_k poly[k] c^k (lib.rs:2640-2655) from the uni-batched proof's L.Z bounds, computed once
    // over the pool: sum_k LZ[k] c^k, LZ[k] = sum_j c^(Rs j) poly[j Rs + k]
    std::vector<const FqV*> all(orig);
    all.insert(all.end(), shifted.begin(), shifted.end());
    const std::vector<FqV> LZs = uni_bounds(all, c);
    size_t rs_max = 0;
    for (auto& v : LZs) rs_max = std::max(rs_max, v.size());
    FqV rc_pow(rs_max);
    {
      Fq nc = fq_one();
      for (size_t i = 0; i < rs_max; i++) {
        rc_pow[i] = nc;
        nc = fq_mul(nc, c);
      }
    }
    FqV ev(2 * n);
    for (size_t p = 0; p < 2 * n; p++) {
      Fq x = fq_zero();
      for (size_t k = 0; k < LZs[p].size(); k++) x = fq_add(x, fq_mul(LZs[p][k], rc_pow[k]));
      ev[p] = x;
    }
    std::vector<CJob> jobs;
    for (auto& x : ev) jobs.push_back(CJob(g.gens_1, {x}, fq_zero()));
    std::vector<Pt> ce = commit_batch(g, jobs);
    if ((rc = prove_uni_batched(ctx, g, all, LZs, c, ev, t, tape, w))) return rc;
    w.pts(std::vector<Pt>(ce.begin(), ce.begin() + n));
    w.pts(std::vector<Pt>(ce.begin() + n, ce.end()));
    w.u64(n);
    for (auto& o : openings) w.pts(o);
  }
  lp.lap("shift");
  // ---- IO_PROOFS (lib.rs:194-272)
  {
    const size_t r_len = lg2(consis * num_ios);
    auto bin = [&](size_t x) {
      FqV v;
      for (size_t k = r_len; k-- > 0;) v.push_back(fq_from_u64((x >> k) & 1));
      return v;
    };
    const std::vector<uint8_t>& live = W->liveness;
    std::vector<size_t> idx;
    for (size_t i = 0; i + 2 < live.size(); i++) idx.push_back(2 + a.input_offset + i);
    if (live.size() > 1 && live[1]) idx.insert(idx.begin(), 5);
    if (live.size() > 0 && live[0]) idx.insert(idx.begin(), 6);
    FqV live_in;
    for (size_t i = 0; i < live.size(); i++)
      if (live[i]) live_in.push_back(W->input[i]);
    idx.resize(live_in.size());
    const size_t oe = a.output_exec_num * num_ios;
    std::vector<size_t> pts = {0, oe, 2, oe + 2 + (niu - 1), oe + 2 + (niu - 1) + a.output_offset - 1};
    pts.insert(pts.end(), idx.begin(), idx.end());
    std::vector<FqV> r_list;
    for (auto x : pts) r_list.push_back(bin(x));
    FqV Zr = {fq_one(), fq_one(), input_block_num, output_block_num, W->output};
    Zr.insert(Zr.end(), live_in.begin(), live_in.end());
    FqV Z = pad_pow2(flatten(W->exec));
    if ((rc = prove_batched_points(ctx, g, Z, r_list, Zr, t, tape, w))) return rc;
  }
  lp.lap("io");
  lp.print();
  if (getenv("SPG_TRACE") && atoi(getenv("SPG_TRACE")) >= 2) {
    fprintf(stderr, "[spg] sigma-protocol commitments: %zu calls, %zu commitments, %.0f us on the host\n",
                    g_commit_stats.calls, g_commit_stats.points, g_commit_stats.us);
    g_commit_stats = CommitStats();
    static uint64_t bursts0 = 0, keccak0 = 0;
    fprintf(stderr, "[spg] host pool bursts: %llu, keccak-f permutations on this thread: %llu\n",
            (unsigned long long)(pool().bursts() - bursts0), (unsigned long long)(keccak_count() - keccak0));
    bursts0 = pool().bursts();
    keccak0 = keccak_count();
  }
  if (getenv("SPG_COPY_TRACE") && atoi(getenv("SPG_COPY_TRACE"))) print_copy_counts();
  *proof_len = w.out.size();
  if (!proof || w.out.size() > proof_cap) return set_err(ctx, SPG_E_ARG, "proof buffer too small");
  memcpy(proof, w.out.data(), w.out.size());
  return SPG_OK;
}

extern "C" int spg_snark_prove(spg_ctx* ctx, spg_snark_comp* block, spg_snark_comp* pairwise, spg_snark_comp* perm_root,
                               const spg_snark_wit* W, spg_r1cs_gens* vars_gens, spg_transcript* transcript,
                               spg_random_tape* tape_h, uint8_t* proof, size_t proof_cap, size_t* proof_len) {
  if (!ctx || !transcript) return SPG_E_ARG;
  // SPG_TRACE: the whole call's wall time (the laps end at the io proofs; this adds the proof copy-out and the
  // release of the prove's host state)
  static const bool tr = getenv("SPG_TRACE") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  int rc;
  {
    spg::HostPin pin;
    rc = spg::tr_status(ctx, transcript->t, spg_snark_prove_impl(ctx, block, pairwise, perm_root, W, vars_gens, transcript, tape_h, proof, proof_cap, proof_len));
  }
  if (tr)
    fprintf(stderr, "[spg] spg_snark_prove call: %.0f us\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  return rc;
}
