// ORACLE — test infrastructure only. Never linked into the product.
// CPU restatement of SNARK::prove and the pieces it adds on top of R1CSProof and SPARK:
//   src/r1csinstance.rs:34-79,645-780   R1CSCommitmentGens, R1CSCommitment, next_power_of_eight, multi_commit,
//                                       commit, R1CSEvalProof
//   src/lib.rs:148-185                  SNARKGens::new (the gens_r1cs_eval part)
//   src/lib.rs:187-300                  IOProofs::prove
//   src/lib.rs:302-446                  ShiftProofs::prove
//   src/lib.rs:701-756                  SNARK (field order = bincode order)
//   src/lib.rs:793-829                  SNARK::multi_encode / encode
//   src/lib.rs:831-968                  SNARK::mem_gen
//   src/lib.rs:971-2746                 SNARK::prove
// plus a verifier of the pieces that carry the argument's soundness (the three R1CSProofs with their
// R1CSEvalProofs and the permutation-product identity), replaying SNARK::prove's transcript.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <map>
#include <vector>

#include "spark.hpp"

namespace orc {

static const size_t INIT_PHY_MEM_WIDTH = 4, INIT_VIR_MEM_WIDTH = 4, PHY_MEM_WIDTH = 4, VIR_MEM_WIDTH = 8,
                    W3_WIDTH = 8;

// ---------------------------------------------------------------- R1CS commitments (r1csinstance.rs)
struct R1CSCommGens {  // R1CSCommitmentGens::new (r1csinstance.rs:39-56)
  SparkGens gens;
  size_t nvx = 0, nvy = 0;
  static R1CSCommGens create(const char* label, size_t num_instances, size_t num_cons, size_t num_vars, size_t nnz) {
    R1CSCommGens g;
    g.nvx = log_2(num_instances) + log_2(num_cons);
    g.nvy = log_2(num_vars);
    g.gens = SparkGens::create(label, g.nvx, g.nvy, num_instances * nnz, 3);
    return g;
  }
};
// SNARKGens::new(num_cons, num_vars, num_instances, nnz).gens_r1cs_eval (lib.rs:164-185)
static inline R1CSCommGens snark_eval_gens(size_t num_cons, size_t num_vars, size_t num_instances, size_t nnz) {
  return R1CSCommGens::create("gens_r1cs_eval", next_pow2(num_instances), num_cons, next_pow2(num_vars), nnz);
}

struct R1CSComm {  // R1CSCommitment (r1csinstance.rs:58-69)
  size_t num_cons = 0, num_vars = 0;
  SparkCommitment comm;
  void ser(Ser& s) const {
    s.u64(num_cons);
    s.u64(num_vars);
    comm.ser(s);
  }
  void append(Transcript& t) const {
    t.append_u64("num_cons", num_cons);
    t.append_u64("num_vars", num_vars);
    comm.append(t);
  }
};

static inline size_t next_power_of_eight(size_t v) {  // r1csinstance.rs:646-652
  size_t b = 1;
  while (b < v) b *= 8;
  return b;
}

// R1CSInstance::multi_commit (r1csinstance.rs:654-715): matrices grouped by next_power_of_eight(nnz)
static inline void r1cs_multi_commit(const R1CSInstance& inst, const R1CSCommGens& g,
                                     std::vector<std::vector<size_t>>* label_map, std::vector<R1CSComm>* comms,
                                     std::vector<MultiSparseDense>* dense) {
  std::vector<std::pair<size_t, size_t>> nnz_size;  // (rounded nnz, label)
  std::vector<std::vector<const SparseMat*>> groups;
  label_map->clear();
  for (size_t i = 0; i < inst.num_instances; i++) {
    const SparseMat* m3[3] = {&inst.A[i], &inst.B[i], &inst.C[i]};
    for (size_t k = 0; k < 3; k++) {
      size_t len = next_power_of_eight(m3[k]->num_nz_entries());
      size_t idx = nnz_size.size();
      for (auto& kv : nnz_size)
        if (kv.first == len) idx = kv.second;
      if (idx == nnz_size.size()) {
        nnz_size.push_back({len, idx});
        label_map->push_back({});
        groups.push_back({});
      }
      (*label_map)[idx].push_back(3 * i + k);
      groups[idx].push_back(m3[k]);
    }
  }
  comms->clear();
  dense->clear();
  for (auto& grp : groups) {
    MultiSparseDense d;
    R1CSComm c;
    c.comm = spark_multi_commit(grp, g.gens, &d);
    c.num_cons = inst.num_instances * inst.max_num_cons;
    c.num_vars = inst.num_vars;
    comms->push_back(c);
    dense->push_back(std::move(d));
  }
}
// R1CSInstance::commit (r1csinstance.rs:717-737)
static inline R1CSComm r1cs_commit(const R1CSInstance& inst, const R1CSCommGens& g, MultiSparseDense* dense) {
  std::vector<const SparseMat*> polys;
  for (size_t i = 0; i < inst.num_instances; i++) {
    polys.push_back(&inst.A[i]);
    polys.push_back(&inst.B[i]);
    polys.push_back(&inst.C[i]);
  }
  R1CSComm c;
  c.comm = spark_multi_commit(polys, g.gens, dense);
  c.num_cons = inst.num_instances * inst.max_num_cons;
  c.num_vars = inst.num_vars;
  return c;
}

// ---------------------------------------------------------------- sub-proofs of SNARK (lib.rs)
struct IOProofs {
  std::vector<PolyEvalProof> proofs;
  void ser(Ser& s) const { ser_proofs(s, proofs); }
};
struct ShiftProofs {
  PolyEvalProof proof;
  std::vector<CPt> C_orig_evals, C_shifted_evals;
  std::vector<std::vector<CPt>> openings;
  void ser(Ser& s) const {
    proof.ser(s);
    s.pts(C_orig_evals);
    s.pts(C_shifted_evals);
    s.u64(openings.size());
    for (auto& o : openings) s.pts(o);
  }
};

static inline FqVec to_bin_array(size_t x, size_t r_len) {  // lib.rs:212-218
  FqVec v;
  for (size_t n = r_len; n-- > 0;) v.push_back(fq_from_u64((x >> n) & 1));
  return v;
}

// IOProofs::prove (lib.rs:194-272)
static inline IOProofs io_proofs_prove(const DensePoly& exec_poly_inputs, size_t num_ios, size_t niu,
                                       size_t num_proofs, const Fq& input_block_num, const Fq& output_block_num,
                                       const std::vector<bool>& liveness, size_t input_offset, size_t output_offset,
                                       const FqVec& input, const Fq& output, size_t output_exec_num,
                                       const DotGens& gens_pc, Transcript& t, RandomTape& tape) {
  size_t r_len = log_2(num_proofs * num_ios);
  std::vector<size_t> idx;
  for (size_t i = 0; i + 2 < liveness.size(); i++) idx.push_back(2 + input_offset + i);
  if (liveness[1]) idx.insert(idx.begin(), 5);
  if (liveness[0]) idx.insert(idx.begin(), 6);
  FqVec live;
  for (size_t i = 0; i < liveness.size(); i++)
    if (liveness[i]) live.push_back(input[i]);
  idx.resize(live.size());
  std::vector<size_t> pts = {0, output_exec_num * num_ios, 2, output_exec_num * num_ios + 2 + (niu - 1),
                             output_exec_num * num_ios + 2 + (niu - 1) + output_offset - 1};
  pts.insert(pts.end(), idx.begin(), idx.end());
  std::vector<FqVec> r_list;
  for (size_t p : pts) r_list.push_back(to_bin_array(p, r_len));
  FqVec Zr = {fq_one(), fq_one(), input_block_num, output_block_num, output};
  Zr.insert(Zr.end(), live.begin(), live.end());
  IOProofs o;
  o.proofs = PolyEvalProof::prove_batched_points(exec_poly_inputs, r_list, Zr, gens_pc, t, tape);
  return o;
}

// ShiftProofs::prove (lib.rs:310-446)
static inline ShiftProofs shift_proofs_prove(const std::vector<const DensePoly*>& orig,
                                             const std::vector<const DensePoly*>& shifted,
                                             const std::vector<size_t>& header_len, const DotGens& gens_pc,
                                             Transcript& t, RandomTape& tape) {
  size_t n = orig.size();
  size_t max_size = 0;
  for (auto p : orig) max_size = std::max(max_size, p->len);
  for (auto p : shifted) max_size = std::max(max_size, p->len);
  ShiftProofs sp;
  sp.openings.resize(n);
  for (size_t p = 0; p < n; p++)
    for (size_t i = 0; i < header_len[p]; i++) {
      CPt e = cpt(commit1((*orig[p])[i], fq_zero(), gens_pc.gens_1));
      t.append_point("shift_header_entry", e.v);
      sp.openings[p].push_back(e);
    }
  Fq c = t.challenge_scalar("challenge_c");
  FqVec rc;
  Fq nc = fq_one();
  for (size_t i = 0; i < max_size; i++) {
    rc.push_back(nc);
    nc = fq_mul(nc, c);
  }
  FqVec oe, se;
  for (size_t p = 0; p < n; p++) {
    Fq a = fq_zero(), b = fq_zero();
    for (size_t k = 0; k < orig[p]->len; k++) a = fq_add(a, fq_mul((*orig[p])[k], rc[k]));
    for (size_t k = 0; k < shifted[p]->len; k++) b = fq_add(b, fq_mul((*shifted[p])[k], rc[k]));
    oe.push_back(a);
    se.push_back(b);
    sp.C_orig_evals.push_back(cpt(commit1(a, fq_zero(), gens_pc.gens_1)));
    sp.C_shifted_evals.push_back(cpt(commit1(b, fq_zero(), gens_pc.gens_1)));
  }
  std::vector<const DensePoly*> all(orig);
  all.insert(all.end(), shifted.begin(), shifted.end());
  FqVec ev(oe);
  ev.insert(ev.end(), se.begin(), se.end());
  CPt cz;
  sp.proof = PolyEvalProof::prove_uni_batched_instances(all, c, ev, gens_pc, t, tape, &cz);
  return sp;
}

// ---------------------------------------------------------------- inputs
struct SnarkInst {  // one public R1CS instance with its SNARKGens parameters and encoding
  R1CSInstance inst;
  R1CSCommGens gens;
  bool multi = false;
  std::vector<std::vector<size_t>> label_map;
  std::vector<R1CSComm> comms;
  std::vector<MultiSparseDense> dense;
  void encode() {
    if (multi) {
      r1cs_multi_commit(inst, gens, &label_map, &comms, &dense);
    } else {
      dense.resize(1);
      comms = {r1cs_commit(inst, gens, &dense[0])};
    }
  }
};

struct SnarkIn {  // SNARK::prove arguments (lib.rs:971-1023), scalars already decoded
  size_t input_block_num = 0, output_block_num = 0;
  std::vector<bool> input_liveness;
  size_t func_input_width = 0, input_offset = 0, output_offset = 0;
  FqVec input;
  Fq output;
  size_t output_exec_num = 0;
  size_t num_vars = 0, num_ios = 0, max_block_num_phy_ops = 0, max_block_num_vir_ops = 0;
  std::vector<size_t> block_num_phy_ops, block_num_vir_ops;
  size_t mem_addr_ts_bits_size = 0, num_inputs_unpadded = 0;
  std::vector<size_t> block_num_vars;
  size_t block_num_instances_bound = 0, block_max_num_proofs = 0;
  std::vector<size_t> block_num_proofs;
  size_t consis_num_proofs = 0, total_num_init_phy_mem_accesses = 0, total_num_init_vir_mem_accesses = 0,
         total_num_phy_mem_accesses = 0, total_num_vir_mem_accesses = 0;
  std::vector<std::vector<FqVec>> block_vars_mat;  // [b][q][i]
  std::vector<FqVec> exec_inputs_list, init_phy_mems_list, init_vir_mems_list, addr_phy_mems_list,
      addr_vir_mems_list, addr_ts_bits_list;
};

struct SNARKProof {  // lib.rs:701-756
  std::vector<PolyCommitment> block_comm_vars_list, exec_comm_inputs;
  PolyCommitment addr_comm_phy_mems, addr_comm_phy_mems_shifted, addr_comm_vir_mems, addr_comm_vir_mems_shifted,
      addr_comm_ts_bits;
  PolyCommitment perm_exec_comm_w2_list, perm_exec_comm_w3_list, perm_exec_comm_w3_shifted;
  std::vector<PolyCommitment> block_comm_w2_list, block_comm_w3_list, block_comm_w3_list_shifted;
  PolyCommitment init_phy_mem_comm_w2, init_phy_mem_comm_w3, init_phy_mem_comm_w3_shifted;
  PolyCommitment init_vir_mem_comm_w2, init_vir_mem_comm_w3, init_vir_mem_comm_w3_shifted;
  PolyCommitment phy_mem_addr_comm_w2, phy_mem_addr_comm_w3, phy_mem_addr_comm_w3_shifted;
  PolyCommitment vir_mem_addr_comm_w2, vir_mem_addr_comm_w3, vir_mem_addr_comm_w3_shifted;
  R1CSProof block_r1cs_sat_proof;
  Fq block_inst_evals_bound_rp[3];
  FqVec block_inst_evals_list;
  std::vector<SparkEvalProof> block_r1cs_eval_proof_list;
  R1CSProof pairwise_check_r1cs_sat_proof;
  Fq pairwise_check_inst_evals_bound_rp[3];
  FqVec pairwise_check_inst_evals_list;
  SparkEvalProof pairwise_check_r1cs_eval_proof;
  R1CSProof perm_root_r1cs_sat_proof;
  Fq perm_root_inst_evals[3];
  SparkEvalProof perm_root_r1cs_eval_proof;
  FqVec perm_poly_poly_list;
  std::vector<PolyEvalProof> proof_eval_perm_poly_prod_list;
  ShiftProofs shift_proof;
  IOProofs io_proof;

  void ser(Ser& s) const {
    auto comms = [&](const std::vector<PolyCommitment>& v) {
      s.u64(v.size());
      for (auto& c : v) s.pts(c);
    };
    comms(block_comm_vars_list);
    comms(exec_comm_inputs);
    for (auto* c : {&addr_comm_phy_mems, &addr_comm_phy_mems_shifted, &addr_comm_vir_mems,
                    &addr_comm_vir_mems_shifted, &addr_comm_ts_bits, &perm_exec_comm_w2_list,
                    &perm_exec_comm_w3_list, &perm_exec_comm_w3_shifted})
      s.pts(*c);
    comms(block_comm_w2_list);
    comms(block_comm_w3_list);
    comms(block_comm_w3_list_shifted);
    for (auto* c : {&init_phy_mem_comm_w2, &init_phy_mem_comm_w3, &init_phy_mem_comm_w3_shifted,
                    &init_vir_mem_comm_w2, &init_vir_mem_comm_w3, &init_vir_mem_comm_w3_shifted,
                    &phy_mem_addr_comm_w2, &phy_mem_addr_comm_w3, &phy_mem_addr_comm_w3_shifted,
                    &vir_mem_addr_comm_w2, &vir_mem_addr_comm_w3, &vir_mem_addr_comm_w3_shifted})
      s.pts(*c);
    block_r1cs_sat_proof.ser(s);
    for (int i = 0; i < 3; i++) s.sc(block_inst_evals_bound_rp[i]);
    s.scs(block_inst_evals_list);
    s.u64(block_r1cs_eval_proof_list.size());
    for (auto& p : block_r1cs_eval_proof_list) p.ser(s);
    pairwise_check_r1cs_sat_proof.ser(s);
    for (int i = 0; i < 3; i++) s.sc(pairwise_check_inst_evals_bound_rp[i]);
    s.scs(pairwise_check_inst_evals_list);
    pairwise_check_r1cs_eval_proof.ser(s);
    perm_root_r1cs_sat_proof.ser(s);
    for (int i = 0; i < 3; i++) s.sc(perm_root_inst_evals[i]);
    perm_root_r1cs_eval_proof.ser(s);
    s.scs(perm_poly_poly_list);
    ser_proofs(s, proof_eval_perm_poly_prod_list);
    shift_proof.ser(s);
    io_proof.ser(s);
  }
};

// commit one flattened witness polynomial and append its commitment (the recurring block of lib.rs)
static inline PolyCommitment commit_append(const DensePoly& p, const DotGens& g, Transcript& t) {
  PolyCommitment c = poly_commit(p, g);
  append_polycomm(t, "poly_commitment", c);
  return c;
}
static inline FqVec flatten(const std::vector<FqVec>& m) {
  FqVec v;
  for (auto& r : m) v.insert(v.end(), r.begin(), r.end());
  return v;
}
static inline std::vector<FqVec> shift_rows(const std::vector<FqVec>& m, size_t width) {
  std::vector<FqVec> s(m.begin() + 1, m.end());
  s.push_back(FqVec(width, fq_zero()));
  return s;
}

struct MemSecs {  // the (w2, w3, w3_shifted) triple of one memory list (lib.rs:831-968)
  WitnessSec w2, w3, w3s;
  PolyCommitment c2, c3, c3s;
};
// SNARK::mem_gen (lib.rs:831-968); vir = true gives the VIR_MEM variant of lib.rs:1809-1951
static inline MemSecs mem_gen(size_t width, size_t total, const std::vector<FqVec>& mems, const Fq& r,
                              const Fq& tau, bool vir, const DotGens& g, Transcript& t) {
  MemSecs o;
  if (total == 0) return o;
  std::vector<FqVec> w2(total, FqVec(width, fq_zero())), w3(total, FqVec(W3_WIDTH, fq_zero()));
  Fq r2 = fq_mul(r, r), r3 = fq_mul(r2, r);
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
    if (q != total - 1)
      w3[q][3] = fq_mul(w3[q][1], fq_sub(fq_add(w3[q + 1][2], fq_one()), w3[q + 1][0]));
    else
      w3[q][3] = w3[q][1];
    w3[q][2] = fq_mul(w3[q][0], w3[q][3]);
    w3[q][4] = fq_mul(mems[q][0], fq_add(fq_add(mems[q][0], mems[q][2]), rest));
    w3[q][5] = mems[q][0];
  }
  DensePoly p2(flatten(w2)), p3(flatten(w3));
  std::vector<FqVec> w3s = shift_rows(w3, W3_WIDTH);
  DensePoly p3s(flatten(w3s));
  o.c2 = commit_append(p2, g, t);
  o.c3 = commit_append(p3, g, t);
  o.c3s = commit_append(p3s, g, t);
  o.w2 = WitnessSec::create({w2}, {p2});
  o.w3 = WitnessSec::create({w3}, {p3});
  o.w3s = WitnessSec::create({w3s}, {p3s});
  return o;
}

// R1CSEvalProof::prove = SparseMatPolyEvalProof::prove on the decommitment (r1csinstance.rs:743-765)
static inline SparkEvalProof r1cs_eval_prove(const MultiSparseDense& d, const FqVec& rx, const FqVec& ry,
                                             const FqVec& evals, const R1CSCommGens& g, Transcript& t,
                                             RandomTape& tape) {
  return spark_prove(d, rx, ry, evals, g.gens, t, tape);
}

struct SnarkTrace {  // what the verifier side needs besides the proof (for the oracle's own check)
  std::vector<std::vector<size_t>> block_ws_num_inputs, block_ws_num_proofs;
  std::vector<std::vector<PolyCommitment>> block_ws_comm;
  std::vector<std::vector<size_t>> pw_ws_num_inputs, pw_ws_num_proofs, pr_ws_num_inputs, pr_ws_num_proofs;
  std::vector<std::vector<PolyCommitment>> pw_ws_comm, pr_ws_comm;
  std::vector<size_t> block_num_proofs_sorted, pairwise_num_proofs, perm_root_num_proofs;
  size_t block_num_instances = 0, pairwise_num_instances = 0, perm_root_num_instances = 0;
  size_t pairwise_size = 0, perm_size = 0, block_max_num_proofs = 0;
  R1CSInstance block_sorted, pairwise_sorted;
  std::vector<size_t> perm_inst_map;  // component of each perm-product instance (lib.rs:2540-2556)
};

static inline WitnessSec dummy_sec() { return WitnessSec(); }

// per-phase wall time of the last snark_prove, under the labels of the reference's Timer scopes (src/timer.rs;
// lib.rs:1088-2692: inst_commit, block_sort, witness_gen, input_commit, Block Correctness Extract, Pairwise Check,
// Perm Root, Perm Product, Shift Proofs, IO Proofs); read by orc_snark_last_phases (bench.py config 1)
struct PhaseTimer {
  std::vector<std::pair<std::string, double>> laps;
  std::chrono::steady_clock::time_point t0;
  void start() {
    laps.clear();
    t0 = std::chrono::steady_clock::now();
  }
  void lap(const char* name) {
    const auto t1 = std::chrono::steady_clock::now();
    laps.push_back({name, std::chrono::duration<double, std::micro>(t1 - t0).count()});
    t0 = t1;
  }
};
// per thread: the all-cores baselines run SNARK::prove on several threads at once (a shared lap list raced)
static thread_local PhaseTimer g_snark_phases;

// SNARK::prove (lib.rs:971-2746)
static inline SNARKProof snark_prove(const SnarkIn& in0, SnarkInst& block, SnarkInst& pairwise, SnarkInst& perm_root,
                                     const R1CSGens& vars_gens, Transcript& t, RandomTape& tape,
                                     SnarkTrace* tr = nullptr) {
  SnarkIn in = in0;
  SNARKProof pf;
  g_snark_phases.start();
  t.append_protocol_name("Spartan SNARK proof");
  const bool dbg0 = getenv("SPG_DEBUG_SNARK") != nullptr;
  auto fp = [&](const char* where) {
    if (!dbg0) return;
    Transcript c = t;
    Fq x = c.challenge_scalar("dbg");
    fprintf(stderr, "fp %s %08x\n", where, (uint32_t)x.v[0]);
  };
  const size_t niu = in.num_inputs_unpadded, num_ios = in.num_ios, io_width = 2 * niu;
  const DotGens& gpc = vars_gens.gens_pc;
  Fq input_block_num = fq_from_u64(in.input_block_num), output_block_num = fq_from_u64(in.output_block_num);
  // ---- INSTANCE COMMITMENTS (lib.rs:1086-1153)
  auto app = [&](const char* l, size_t v) { t.append_scalar(l, fq_from_u64(v)); };
  app("func_input_width", in.func_input_width);
  app("input_offset", in.input_offset);
  app("output_offset", in.output_offset);
  app("output_exec_num", in.output_exec_num);
  app("num_ios", num_ios);
  for (auto n : in.block_num_vars) app("block_num_vars", n);
  app("mem_addr_ts_bits_size", in.mem_addr_ts_bits_size);
  app("num_inputs_unpadded", niu);
  app("block_num_instances_bound", in.block_num_instances_bound);
  app("block_max_num_proofs", in.block_max_num_proofs);
  for (auto p : in.block_num_phy_ops) app("block_num_phy_ops", p);
  for (auto v : in.block_num_vir_ops) app("block_num_vir_ops", v);
  app("total_num_init_phy_mem_accesses", in.total_num_init_phy_mem_accesses);
  app("total_num_init_vir_mem_accesses", in.total_num_init_vir_mem_accesses);
  app("total_num_phy_mem_accesses", in.total_num_phy_mem_accesses);
  app("total_num_vir_mem_accesses", in.total_num_vir_mem_accesses);
  app("block_max_num_proofs", in.block_max_num_proofs);
  for (auto n : in.block_num_proofs) app("block_num_proofs", n);
  fp("params");
  for (auto& b : block.label_map)
    for (auto l : b) app("block_comm_map", l);
  fp("map");
  for (auto& c : block.comms) c.append(t);
  fp("block");
  pairwise.comms[0].append(t);
  fp("pairwise");
  perm_root.comms[0].append(t);
  fp("perm_root");
  t.append_scalar("input_block_num", input_block_num);
  t.append_scalar("output_block_num", output_block_num);
  t.append_scalars("input_list", in.input);
  t.append_scalar("output_list", in.output);

  g_snark_phases.lap("inst_commit");
  // ---- BLOCK SORT (lib.rs:1155-1198): stable, by decreasing num_proofs
  size_t block_num_instances = 0;
  for (auto n : in.block_num_proofs)
    if (n > 0) block_num_instances++;
  std::vector<size_t> order(in.block_num_instances_bound);
  for (size_t i = 0; i < order.size(); i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [&](size_t a, size_t b) { return in.block_num_proofs[a] > in.block_num_proofs[b]; });
  order.resize(block_num_instances);
  std::vector<size_t> block_num_proofs, block_num_vars, block_num_phy_ops, block_num_vir_ops;
  std::vector<std::vector<FqVec>> block_vars_mat;
  for (size_t i : order) {
    block_num_proofs.push_back(in.block_num_proofs[i]);
    block_num_vars.push_back(in.block_num_vars[i]);
    block_num_phy_ops.push_back(in.block_num_phy_ops[i]);
    block_num_vir_ops.push_back(in.block_num_vir_ops[i]);
  }
  // block_vars_mat is indexed by the sorted position in the reference only through block_inst.sort; the
  // witness list itself is supplied sorted by the caller in the reference interface when counts differ. The
  // restatement keeps the reference's behaviour: block_vars_mat[i] pairs with sorted instance i.
  block_vars_mat = in.block_vars_mat;
  R1CSInstance block_sorted = block.inst;
  block_sorted.sort(block_num_instances, order);
  // ---- PADDING (lib.rs:1200-1273)
  size_t block_max_num_proofs = next_pow2(in.block_max_num_proofs);
  for (size_t i = 0; i < block_num_instances; i++) {
    size_t w = block_vars_mat[i][0].size();
    size_t gap = next_pow2(block_num_proofs[i]) - block_num_proofs[i];
    for (size_t k = 0; k < gap; k++) block_vars_mat[i].push_back(FqVec(w, fq_zero()));
    block_num_proofs[i] = next_pow2(block_num_proofs[i]);
  }
  auto pad_list = [&](std::vector<FqVec>& l, size_t& total, size_t width) {
    if (total > 0) {
      size_t np = next_pow2(total);
      for (size_t k = total; k < np; k++) l.push_back(FqVec(width, fq_zero()));
      total = np;
    }
  };
  for (size_t k = in.consis_num_proofs; k < next_pow2(in.consis_num_proofs); k++)
    in.exec_inputs_list.push_back(FqVec(num_ios, fq_zero()));
  size_t consis_num_proofs = next_pow2(in.consis_num_proofs);
  size_t t_iphy = in.total_num_init_phy_mem_accesses, t_ivir = in.total_num_init_vir_mem_accesses,
         t_phy = in.total_num_phy_mem_accesses, t_vir = in.total_num_vir_mem_accesses;
  pad_list(in.init_phy_mems_list, t_iphy, INIT_PHY_MEM_WIDTH);
  pad_list(in.init_vir_mems_list, t_ivir, INIT_VIR_MEM_WIDTH);
  pad_list(in.addr_phy_mems_list, t_phy, PHY_MEM_WIDTH);
  if (t_vir > 0) {
    size_t np = next_pow2(t_vir);
    for (size_t k = t_vir; k < np; k++) {
      in.addr_vir_mems_list.push_back(FqVec(VIR_MEM_WIDTH, fq_zero()));
      in.addr_ts_bits_list.push_back(FqVec(in.mem_addr_ts_bits_size, fq_zero()));
    }
    t_vir = np;
  }
  // ---- PAIRWISE SORT (lib.rs:1275-1296)
  std::vector<std::pair<size_t, size_t>> ps = {{consis_num_proofs, 0}, {t_phy, 1}, {t_vir, 2}};
  std::stable_sort(ps.begin(), ps.end(), [](const std::pair<size_t, size_t>& a, const std::pair<size_t, size_t>& b) {
    return a.first > b.first;
  });
  size_t pairwise_num_instances = 1 + (t_phy > 0 ? 1 : 0) + (t_vir > 0 ? 1 : 0);
  std::vector<size_t> pw_index;
  for (size_t i = 0; i < pairwise_num_instances; i++) pw_index.push_back(ps[i].second);
  R1CSInstance pairwise_sorted = pairwise.inst;
  pairwise_sorted.sort(pairwise_num_instances, pw_index);

  g_snark_phases.lap("block_sort");
  // ---- WITNESS GEN: block (lib.rs:1299-1741)
  Fq comb_tau = t.challenge_scalar("challenge_tau");
  Fq comb_r = t.challenge_scalar("challenge_r");
  const bool dbg = getenv("SPG_DEBUG_SNARK") != nullptr;
  if (dbg) fprintf(stderr, "snark tau %08x %08x r %08x\n", (uint32_t)comb_tau.v[0], (uint32_t)(comb_tau.v[0] >> 32), (uint32_t)comb_r.v[0]);
  FqVec perm_w0 = {comb_tau};
  {
    Fq rt = comb_r;
    for (size_t i = 1; i < 2 * niu; i++) {
      perm_w0.push_back(rt);
      rt = fq_mul(rt, comb_r);
    }
    perm_w0.resize(num_ios, fq_zero());
  }
  DensePoly perm_poly_w0(perm_w0);
  commit_append(perm_poly_w0, gpc, t);
  std::vector<FqVec>& exec = in.exec_inputs_list;
  std::vector<FqVec> perm_exec_w2(consis_num_proofs), perm_exec_w3(consis_num_proofs);
  for (size_t q = 0; q < consis_num_proofs; q++) {
    // [0; 3] ++ (1..2niu-2).map(perm_w0[j] * input[j+2]) ++ [0; num_ios - 2niu]
    FqVec v(3, fq_zero());
    for (size_t j = 1; j < 2 * niu - 2; j++) v.push_back(fq_mul(perm_w0[j], exec[q][j + 2]));
    v.resize(num_ios, fq_zero());
    v[0] = exec[q][0];
    v[1] = exec[q][0];
    for (size_t i = 0; i + 1 < niu; i++) {
      Fq perm = i == 0 ? fq_one() : perm_w0[i];
      v[0] = fq_add(v[0], fq_mul(perm, exec[q][2 + i]));
      v[2] = fq_add(v[2], fq_mul(perm, exec[q][2 + (niu - 1) + i]));
    }
    v[0] = fq_mul(v[0], exec[q][0]);
    v[1] = fq_mul(fq_add(v[1], v[2]), exec[q][0]);
    perm_exec_w2[q] = v;
  }
  for (size_t q = consis_num_proofs; q-- > 0;) {
    FqVec w(8, fq_zero());
    w[0] = exec[q][0];
    Fq s = fq_zero();
    for (size_t k = 3; k < perm_exec_w2[q].size(); k++) s = fq_add(s, perm_exec_w2[q][k]);
    w[1] = fq_mul(w[0], fq_sub(fq_sub(comb_tau, s), exec[q][2]));
    w[4] = perm_exec_w2[q][0];
    w[5] = perm_exec_w2[q][1];
    if (q != consis_num_proofs - 1)
      w[3] = fq_mul(w[1], fq_sub(fq_add(perm_exec_w3[q + 1][2], fq_one()), perm_exec_w3[q + 1][0]));
    else
      w[3] = w[1];
    w[2] = fq_mul(w[0], w[3]);
    perm_exec_w3[q] = w;
  }
  if (dbg)
    for (size_t q = 0; q < 2; q++)
      for (size_t i = 0; i < num_ios; i++) fprintf(stderr, "pe_w2[%zu][%zu] %08x\n", q, i, (uint32_t)perm_exec_w2[q][i].v[0]);
  DensePoly perm_exec_poly_w2(flatten(perm_exec_w2)), perm_exec_poly_w3(flatten(perm_exec_w3));
  std::vector<FqVec> perm_exec_w3s = shift_rows(perm_exec_w3, 8);
  DensePoly perm_exec_poly_w3s(flatten(perm_exec_w3s));
  pf.perm_exec_comm_w2_list = commit_append(perm_exec_poly_w2, gpc, t);
  pf.perm_exec_comm_w3_list = commit_append(perm_exec_poly_w3, gpc, t);
  pf.perm_exec_comm_w3_shifted = commit_append(perm_exec_poly_w3s, gpc, t);

  std::vector<std::vector<FqVec>> block_w2(block_num_instances), block_w3(block_num_instances);
  for (size_t p = 0; p < block_num_instances; p++) {
    const size_t np_ = block_num_phy_ops[p], nv_ = block_num_vir_ops[p];
    const size_t w2_size = next_pow2(2 * niu + 2 * np_ + 4 * nv_);
    auto V_PA = [&](size_t i) { return 2 * i; };
    auto V_PD = [&](size_t i) { return 2 * i + 1; };
    auto V_PMR = [&](size_t i) { return 2 * niu + 2 * i; };
    auto V_PMC = [&](size_t i) { return 2 * niu + 2 * i + 1; };
    auto V_VA = [&](size_t i) { return 2 * np_ + 4 * i; };
    auto V_VD = [&](size_t i) { return 2 * np_ + 4 * i + 1; };
    auto V_VL = [&](size_t i) { return 2 * np_ + 4 * i + 2; };
    auto V_VT = [&](size_t i) { return 2 * np_ + 4 * i + 3; };
    auto V_VMR1 = [&](size_t i) { return 2 * niu + 2 * np_ + 4 * i; };
    auto V_VMR2 = [&](size_t i) { return 2 * niu + 2 * np_ + 4 * i + 1; };
    auto V_VMR3 = [&](size_t i) { return 2 * niu + 2 * np_ + 4 * i + 2; };
    auto V_VMC = [&](size_t i) { return 2 * niu + 2 * np_ + 4 * i + 3; };
    const size_t Q = block_num_proofs[p];
    block_w2[p].assign(Q, FqVec());
    block_w3[p].assign(Q, FqVec());
    for (size_t q = Q; q-- > 0;) {
      const FqVec& bv = block_vars_mat[p][q];
      const Fq V_CNST = bv[0];
      FqVec w2(w2_size, fq_zero());
      w2[0] = bv[0];
      w2[1] = bv[0];
      for (size_t i = 1; i < 2 * (niu - 1); i++) w2[2 + i] = fq_add(w2[2 + i], fq_mul(perm_w0[i], bv[i + 2]));
      for (size_t i = 0; i + 1 < niu; i++) {
        Fq perm = i == 0 ? fq_one() : perm_w0[i];
        w2[0] = fq_add(w2[0], fq_mul(perm, bv[2 + i]));
        w2[2] = fq_add(w2[2], fq_mul(perm, bv[2 + (niu - 1) + i]));
      }
      w2[0] = fq_mul(w2[0], bv[0]);
      w2[1] = fq_mul(fq_add(w2[1], w2[2]), bv[0]);
      FqVec w3(8, fq_zero());
      w3[0] = bv[0];
      Fq s = fq_zero();
      for (size_t k = 3; k < w2.size(); k++) s = fq_add(s, w2[k]);
      // note: w2[3..] at this point holds only the INPUT part; the memory parts are filled below
      w3[1] = fq_mul(w3[0], fq_sub(fq_sub(comb_tau, s), bv[2]));
      if (q != Q - 1)
        w3[3] = fq_mul(w3[1], fq_sub(fq_add(block_w3[p][q + 1][2], fq_one()), block_w3[p][q + 1][0]));
      else
        w3[3] = w3[1];
      w3[2] = fq_mul(w3[0], w3[3]);
      for (size_t i = 0; i < np_; i++) {
        w2[V_PMR(i)] = fq_mul(comb_r, bv[io_width + V_PD(i)]);
        Fq tt = i == 0 ? V_CNST : w2[V_PMC(i - 1)];
        w2[V_PMC(i)] = fq_mul(tt, fq_sub(fq_sub(comb_tau, bv[io_width + V_PA(i)]), w2[V_PMR(i)]));
      }
      Fq px = np_ == 0 ? V_CNST : w2[V_PMC(np_ - 1)];
      if (q != Q - 1)
        w3[5] = fq_mul(px, fq_sub(fq_add(block_w3[p][q + 1][4], fq_one()), block_w3[p][q + 1][0]));
      else
        w3[5] = px;
      w3[4] = fq_mul(V_CNST, w3[5]);
      Fq r2 = fq_mul(comb_r, comb_r), r3 = fq_mul(r2, comb_r);
      for (size_t i = 0; i < nv_; i++) {
        w2[V_VMR1(i)] = fq_mul(comb_r, bv[io_width + V_VD(i)]);
        w2[V_VMR2(i)] = fq_mul(r2, bv[io_width + V_VL(i)]);
        w2[V_VMR3(i)] = fq_mul(r3, bv[io_width + V_VT(i)]);
        Fq tt = i == 0 ? V_CNST : w2[V_VMC(i - 1)];
        Fq d = fq_sub(fq_sub(fq_sub(fq_sub(comb_tau, bv[io_width + V_VA(i)]), w2[V_VMR1(i)]), w2[V_VMR2(i)]),
                      w2[V_VMR3(i)]);
        w2[V_VMC(i)] = fq_mul(tt, d);
      }
      Fq vx = nv_ == 0 ? V_CNST : w2[V_VMC(nv_ - 1)];
      if (q != Q - 1)
        w3[7] = fq_mul(vx, fq_sub(fq_add(block_w3[p][q + 1][6], fq_one()), block_w3[p][q + 1][0]));
      else
        w3[7] = vx;
      w3[6] = fq_mul(V_CNST, w3[7]);
      block_w2[p][q] = w2;
      block_w3[p][q] = w3;
    }
  }
  std::vector<DensePoly> block_poly_w2, block_poly_w3, block_poly_w3s;
  for (size_t p = 0; p < block_num_instances; p++) {
    block_poly_w2.push_back(DensePoly(flatten(block_w2[p])));
    pf.block_comm_w2_list.push_back(commit_append(block_poly_w2.back(), gpc, t));
  }
  std::vector<std::vector<FqVec>> block_w3s(block_num_instances);
  for (size_t p = 0; p < block_num_instances; p++) {
    block_poly_w3.push_back(DensePoly(flatten(block_w3[p])));
    pf.block_comm_w3_list.push_back(commit_append(block_poly_w3.back(), gpc, t));
    block_w3s[p] = shift_rows(block_w3[p], 8);
    block_poly_w3s.push_back(DensePoly(flatten(block_w3s[p])));
    pf.block_comm_w3_list_shifted.push_back(commit_append(block_poly_w3s.back(), gpc, t));
  }
  WitnessSec perm_w0_prover = WitnessSec::create({{perm_w0}}, {perm_poly_w0});
  WitnessSec perm_exec_w2_prover = WitnessSec::create({perm_exec_w2}, {perm_exec_poly_w2});
  WitnessSec perm_exec_w3_prover = WitnessSec::create({perm_exec_w3}, {perm_exec_poly_w3});
  WitnessSec perm_exec_w3s_prover = WitnessSec::create({perm_exec_w3s}, {perm_exec_poly_w3s});
  WitnessSec block_w2_prover = WitnessSec::create(block_w2, block_poly_w2);
  WitnessSec block_w3_prover = WitnessSec::create(block_w3, block_poly_w3);
  WitnessSec block_w3s_prover = WitnessSec::create(block_w3s, block_poly_w3s);

  // ---- memory witnesses (lib.rs:1742-1955)
  MemSecs init_phy = mem_gen(INIT_PHY_MEM_WIDTH, t_iphy, in.init_phy_mems_list, comb_r, comb_tau, false, gpc, t);
  MemSecs init_vir = mem_gen(INIT_VIR_MEM_WIDTH, t_ivir, in.init_vir_mems_list, comb_r, comb_tau, false, gpc, t);
  MemSecs phy_addr = mem_gen(PHY_MEM_WIDTH, t_phy, in.addr_phy_mems_list, comb_r, comb_tau, false, gpc, t);
  MemSecs vir_addr = mem_gen(VIR_MEM_WIDTH, t_vir, in.addr_vir_mems_list, comb_r, comb_tau, true, gpc, t);
  pf.init_phy_mem_comm_w2 = init_phy.c2;
  pf.init_phy_mem_comm_w3 = init_phy.c3;
  pf.init_phy_mem_comm_w3_shifted = init_phy.c3s;
  pf.init_vir_mem_comm_w2 = init_vir.c2;
  pf.init_vir_mem_comm_w3 = init_vir.c3;
  pf.init_vir_mem_comm_w3_shifted = init_vir.c3s;
  pf.phy_mem_addr_comm_w2 = phy_addr.c2;
  pf.phy_mem_addr_comm_w3 = phy_addr.c3;
  pf.phy_mem_addr_comm_w3_shifted = phy_addr.c3s;
  pf.vir_mem_addr_comm_w2 = vir_addr.c2;
  pf.vir_mem_addr_comm_w3 = vir_addr.c3;
  pf.vir_mem_addr_comm_w3_shifted = vir_addr.c3s;

  g_snark_phases.lap("witness_gen");
  // ---- WITNESS COMMITMENTS (lib.rs:1957-2221)
  std::vector<DensePoly> block_poly_vars;
  for (size_t p = 0; p < block_num_instances; p++) {
    block_poly_vars.push_back(DensePoly(flatten(block_vars_mat[p])));
    pf.block_comm_vars_list.push_back(commit_append(block_poly_vars.back(), gpc, t));
  }
  DensePoly exec_poly_inputs(flatten(exec));
  pf.exec_comm_inputs.push_back(commit_append(exec_poly_inputs, gpc, t));
  std::vector<DensePoly> poly_init_phy, poly_init_vir;
  if (t_iphy > 0) {
    poly_init_phy.push_back(DensePoly(flatten(in.init_phy_mems_list)));
    commit_append(poly_init_phy[0], gpc, t);
  }
  if (t_ivir > 0) {
    poly_init_vir.push_back(DensePoly(flatten(in.init_vir_mems_list)));
    commit_append(poly_init_vir[0], gpc, t);
  }
  WitnessSec addr_phy_shifted_prover, addr_vir_shifted_prover, addr_ts_bits_prover;
  std::vector<DensePoly> addr_poly_phy, addr_poly_vir;
  if (t_phy > 0) {
    addr_poly_phy.push_back(DensePoly(flatten(in.addr_phy_mems_list)));
    pf.addr_comm_phy_mems = commit_append(addr_poly_phy[0], gpc, t);
    std::vector<FqVec> sh = shift_rows(in.addr_phy_mems_list, PHY_MEM_WIDTH);
    DensePoly ps(flatten(sh));
    pf.addr_comm_phy_mems_shifted = commit_append(ps, gpc, t);
    addr_phy_shifted_prover = WitnessSec::create({sh}, {ps});
  }
  if (t_vir > 0) {
    addr_poly_vir.push_back(DensePoly(flatten(in.addr_vir_mems_list)));
    pf.addr_comm_vir_mems = commit_append(addr_poly_vir[0], gpc, t);
    std::vector<FqVec> sh = shift_rows(in.addr_vir_mems_list, VIR_MEM_WIDTH);
    DensePoly ps(flatten(sh));
    pf.addr_comm_vir_mems_shifted = commit_append(ps, gpc, t);
    addr_vir_shifted_prover = WitnessSec::create({sh}, {ps});
    DensePoly pb(flatten(in.addr_ts_bits_list));
    pf.addr_comm_ts_bits = commit_append(pb, gpc, t);
    addr_ts_bits_prover = WitnessSec::create({in.addr_ts_bits_list}, {pb});
  }
  WitnessSec block_vars_prover = WitnessSec::create(block_vars_mat, block_poly_vars);
  WitnessSec exec_inputs_prover = WitnessSec::create({exec}, {exec_poly_inputs});
  WitnessSec init_phy_mems_prover = t_iphy > 0 ? WitnessSec::create({in.init_phy_mems_list}, poly_init_phy) : dummy_sec();
  WitnessSec init_vir_mems_prover = t_ivir > 0 ? WitnessSec::create({in.init_vir_mems_list}, poly_init_vir) : dummy_sec();
  WitnessSec addr_phy_mems_prover = t_phy > 0 ? WitnessSec::create({in.addr_phy_mems_list}, addr_poly_phy) : dummy_sec();
  WitnessSec addr_vir_mems_prover = t_vir > 0 ? WitnessSec::create({in.addr_vir_mems_list}, addr_poly_vir) : dummy_sec();

  g_snark_phases.lap("input_commit");
  // ---- BLOCK_CORRECTNESS_EXTRACT (lib.rs:2223-2309)
  std::vector<FqVec> block_ch;
  pf.block_r1cs_sat_proof = R1CSProof::prove(
      block_num_instances, block_max_num_proofs, block_num_proofs, in.num_vars, block_num_vars,
      {&block_vars_prover, &perm_w0_prover, &block_w2_prover, &block_w3_prover, &block_w3s_prover}, block_sorted,
      vars_gens, t, tape, &block_ch);
  {
    const FqVec &rp = block_ch[0], &rx = block_ch[2], &ry = block_ch[3];
    pf.block_inst_evals_list = block.inst.multi_evaluate(rx, ry);
    FqVec lst;
    block_sorted.multi_evaluate_bound_rp(rp, rx, ry, &lst, pf.block_inst_evals_bound_rp);
    for (auto& r : pf.block_inst_evals_list) t.append_scalar("ABCr_claim", r);
    t.challenge_scalar("challenge_c0");
    t.challenge_scalar("challenge_c1");
    t.challenge_scalar("challenge_c2");
    for (size_t i = 0; i < block.comms.size(); i++) {
      FqVec ev;
      for (auto l : block.label_map[i]) ev.push_back(pf.block_inst_evals_list[l]);
      pf.block_r1cs_eval_proof_list.push_back(r1cs_eval_prove(block.dense[i], rx, ry, ev, block.gens, t, tape));
    }
  }

  g_snark_phases.lap("Block Correctness Extract");
  // ---- PAIRWISE_CHECK (lib.rs:2311-2424)
  size_t pairwise_size = std::max(std::max(consis_num_proofs, t_phy), t_vir);
  std::vector<size_t> inst_map, im2;
  WitnessSec pairwise_prover = WitnessSec::merge({&perm_exec_w3_prover, &addr_phy_mems_prover, &addr_vir_mems_prover},
                                                 &inst_map);
  WitnessSec pairwise_shifted_prover =
      WitnessSec::merge({&perm_exec_w3s_prover, &addr_phy_shifted_prover, &addr_vir_shifted_prover}, &im2);
  WitnessSec ts_bits_prover;
  {
    std::vector<const WitnessSec*> comps(inst_map.size(), &perm_w0_prover);
    for (size_t i = 0; i < inst_map.size(); i++)
      if (inst_map[i] == 2) comps[i] = &addr_ts_bits_prover;
    ts_bits_prover = WitnessSec::concat(comps);
  }
  size_t pw_n = pairwise_prover.w_mat.size();
  std::vector<size_t> pw_num_proofs;
  for (auto& m : pairwise_prover.w_mat) pw_num_proofs.push_back(m.size());
  const size_t pw_nv = std::max<size_t>(8, in.mem_addr_ts_bits_size);
  std::vector<FqVec> pw_ch;
  pf.pairwise_check_r1cs_sat_proof = R1CSProof::prove(
      pw_n, pairwise_size, pw_num_proofs, pw_nv, std::vector<size_t>(pw_n, pw_nv),
      {&pairwise_prover, &pairwise_shifted_prover, &ts_bits_prover}, pairwise_sorted, vars_gens, t, tape, &pw_ch);
  {
    const FqVec &rp = pw_ch[0], &rx = pw_ch[2], &ry = pw_ch[3];
    pf.pairwise_check_inst_evals_list = pairwise.inst.multi_evaluate(rx, ry);
    FqVec lst;
    pairwise_sorted.multi_evaluate_bound_rp(rp, rx, ry, &lst, pf.pairwise_check_inst_evals_bound_rp);
    for (auto& r : pf.pairwise_check_inst_evals_list) t.append_scalar("ABCr_claim", r);
    t.challenge_scalar("challenge_c0");
    t.challenge_scalar("challenge_c1");
    t.challenge_scalar("challenge_c2");
    pf.pairwise_check_r1cs_eval_proof =
        r1cs_eval_prove(pairwise.dense[0], rx, ry, pf.pairwise_check_inst_evals_list, pairwise.gens, t, tape);
  }

  g_snark_phases.lap("Pairwise Check");
  // ---- PERM_ROOT (lib.rs:2426-2532)
  size_t perm_size = std::max({consis_num_proofs, t_iphy, t_ivir, t_phy, t_vir});
  std::vector<size_t> m1, m2, m3, m4;
  WitnessSec pr_w1 = WitnessSec::merge({&exec_inputs_prover, &init_phy_mems_prover, &init_vir_mems_prover,
                                        &addr_phy_mems_prover, &addr_vir_mems_prover}, &m1);
  WitnessSec pr_w2 = WitnessSec::merge({&perm_exec_w2_prover, &init_phy.w2, &init_vir.w2, &phy_addr.w2, &vir_addr.w2}, &m2);
  WitnessSec pr_w3 = WitnessSec::merge({&perm_exec_w3_prover, &init_phy.w3, &init_vir.w3, &phy_addr.w3, &vir_addr.w3}, &m3);
  WitnessSec pr_w3s =
      WitnessSec::merge({&perm_exec_w3s_prover, &init_phy.w3s, &init_vir.w3s, &phy_addr.w3s, &vir_addr.w3s}, &m4);
  size_t pr_n = pr_w1.w_mat.size();
  std::vector<size_t> pr_num_proofs;
  for (auto& m : pr_w1.w_mat) pr_num_proofs.push_back(m.size());
  std::vector<FqVec> pr_ch;
  pf.perm_root_r1cs_sat_proof =
      R1CSProof::prove(pr_n, perm_size, pr_num_proofs, num_ios, std::vector<size_t>(pr_n, num_ios),
                       {&perm_w0_prover, &pr_w1, &pr_w2, &pr_w3, &pr_w3s}, perm_root.inst, vars_gens, t, tape, &pr_ch);
  {
    const FqVec &rx = pr_ch[2], &ry = pr_ch[3];
    FqVec e = perm_root.inst.multi_evaluate(rx, ry);  // R1CSInstance::evaluate on the one instance
    for (int k = 0; k < 3; k++) pf.perm_root_inst_evals[k] = e[k];
    t.append_scalar("Ar_claim", e[0]);
    t.append_scalar("Br_claim", e[1]);
    t.append_scalar("Cr_claim", e[2]);
    pf.perm_root_r1cs_eval_proof = r1cs_eval_prove(perm_root.dense[0], rx, ry, e, perm_root.gens, t, tape);
  }

  g_snark_phases.lap("Perm Root");
  // ---- PERM_PRODUCT_PROOF (lib.rs:2534-2609)
  {
    std::vector<const WitnessSec*> comps = {&perm_exec_w3_prover, &init_phy.w3, &init_vir.w3, &phy_addr.w3,
                                            &vir_addr.w3, &block_w3_prover};
    if (in.max_block_num_phy_ops > 0) comps.push_back(&block_w3_prover);
    if (in.max_block_num_vir_ops > 0) comps.push_back(&block_w3_prover);
    std::vector<size_t> im;
    WitnessSec pw3 = WitnessSec::merge(comps, &im);
    const size_t pm_bl_id = 6, vm_bl_id = in.max_block_num_phy_ops > 0 ? 7 : 6;
    std::vector<FqVec> r_list;
    std::vector<const DensePoly*> polys;
    for (size_t i = 0; i < im.size(); i++) {
      const DensePoly& p = pw3.poly_w[i];
      polys.push_back(&pw3.poly_w[i]);
      if (im[i] == vm_bl_id) {
        pf.perm_poly_poly_list.push_back(p[6]);
        r_list.push_back({fq_one(), fq_one(), fq_zero()});
      } else if (im[i] == pm_bl_id) {
        pf.perm_poly_poly_list.push_back(p[4]);
        r_list.push_back({fq_one(), fq_zero(), fq_zero()});
      } else {
        pf.perm_poly_poly_list.push_back(p[2]);
        r_list.push_back({fq_one(), fq_zero()});
      }
    }
    pf.proof_eval_perm_poly_prod_list =
        PolyEvalProof::prove_batched_instances(polys, r_list, pf.perm_poly_poly_list, gpc, t, tape);
    if (tr) tr->perm_inst_map = im;
  }

  g_snark_phases.lap("Perm Product");
  // ---- SHIFT_PROOFS (lib.rs:2611-2668)
  {
    std::vector<const DensePoly*> orig = {&perm_exec_w3_prover.poly_w[0]}, shifted = {&perm_exec_w3s_prover.poly_w[0]};
    std::vector<size_t> hl = {6};
    for (auto& p : block_w3_prover.poly_w) orig.push_back(&p);
    for (auto& p : block_w3s_prover.poly_w) shifted.push_back(&p);
    for (size_t i = 0; i < block_num_instances; i++) hl.push_back(8);
    if (t_iphy > 0) {
      orig.push_back(&init_phy.w3.poly_w[0]);
      shifted.push_back(&init_phy.w3s.poly_w[0]);
      hl.push_back(6);
    }
    if (t_ivir > 0) {
      orig.push_back(&init_vir.w3.poly_w[0]);
      shifted.push_back(&init_vir.w3s.poly_w[0]);
      hl.push_back(6);
    }
    if (t_phy > 0) {
      orig.push_back(&addr_phy_mems_prover.poly_w[0]);
      shifted.push_back(&addr_phy_shifted_prover.poly_w[0]);
      hl.push_back(4);
      orig.push_back(&phy_addr.w3.poly_w[0]);
      shifted.push_back(&phy_addr.w3s.poly_w[0]);
      hl.push_back(6);
    }
    if (t_vir > 0) {
      orig.push_back(&addr_vir_mems_prover.poly_w[0]);
      shifted.push_back(&addr_vir_shifted_prover.poly_w[0]);
      hl.push_back(6);
      orig.push_back(&vir_addr.w3.poly_w[0]);
      shifted.push_back(&vir_addr.w3s.poly_w[0]);
      hl.push_back(6);
    }
    pf.shift_proof = shift_proofs_prove(orig, shifted, hl, gpc, t, tape);
  }

  g_snark_phases.lap("Shift Proofs");
  // ---- IO_PROOFS (lib.rs:2670-2693)
  pf.io_proof = io_proofs_prove(exec_inputs_prover.poly_w[0], num_ios, niu, consis_num_proofs, input_block_num,
                                output_block_num, in.input_liveness, in.input_offset, in.output_offset, in.input,
                                in.output, in.output_exec_num, gpc, t, tape);

  g_snark_phases.lap("IO Proofs");
  if (tr) {
    auto secs = [](const std::vector<const WitnessSec*>& ws, const std::vector<std::vector<PolyCommitment>>& comm,
                   std::vector<std::vector<size_t>>* ni, std::vector<std::vector<size_t>>* np,
                   std::vector<std::vector<PolyCommitment>>* cm) {
      ni->clear();
      np->clear();
      for (auto w : ws) {
        ni->push_back(w->num_inputs);
        std::vector<size_t> n;
        for (auto& m : w->w_mat) n.push_back(m.size());
        np->push_back(n);
      }
      *cm = comm;
    };
    // commitments of the witness sections, recomputed (the verifier reads them from the proof)
    auto comms_of = [&](const WitnessSec& w) {
      std::vector<PolyCommitment> c;
      for (auto& p : w.poly_w) c.push_back(poly_commit(p, gpc));
      return c;
    };
    secs({&block_vars_prover, &perm_w0_prover, &block_w2_prover, &block_w3_prover, &block_w3s_prover},
         {comms_of(block_vars_prover), comms_of(perm_w0_prover), comms_of(block_w2_prover), comms_of(block_w3_prover),
          comms_of(block_w3s_prover)},
         &tr->block_ws_num_inputs, &tr->block_ws_num_proofs, &tr->block_ws_comm);
    secs({&pairwise_prover, &pairwise_shifted_prover, &ts_bits_prover},
         {comms_of(pairwise_prover), comms_of(pairwise_shifted_prover), comms_of(ts_bits_prover)},
         &tr->pw_ws_num_inputs, &tr->pw_ws_num_proofs, &tr->pw_ws_comm);
    secs({&perm_w0_prover, &pr_w1, &pr_w2, &pr_w3, &pr_w3s},
         {comms_of(perm_w0_prover), comms_of(pr_w1), comms_of(pr_w2), comms_of(pr_w3), comms_of(pr_w3s)},
         &tr->pr_ws_num_inputs, &tr->pr_ws_num_proofs, &tr->pr_ws_comm);
    tr->block_num_proofs_sorted = block_num_proofs;
    tr->pairwise_num_proofs = pw_num_proofs;
    tr->perm_root_num_proofs = pr_num_proofs;
    tr->block_num_instances = block_num_instances;
    tr->pairwise_num_instances = pw_n;
    tr->perm_root_num_instances = pr_n;
    tr->pairwise_size = pairwise_size;
    tr->perm_size = perm_size;
    tr->block_max_num_proofs = block_max_num_proofs;
    tr->block_sorted = block_sorted;
    tr->pairwise_sorted = pairwise_sorted;
  }
  return pf;
}


// ---------------------------------------------------------------- verifier (oracle self-check)
struct VSec {  // VerifierWitnessSecInfo (lib.rs:606-698)
  std::vector<size_t> num_inputs, num_proofs;
  std::vector<PolyCommitment> comm_w;
  static VSec merge(const std::vector<const VSec*>& comps, std::vector<size_t>* inst_map) {
    std::vector<size_t> ptr(comps.size(), 0);
    size_t total = 0;
    for (auto c : comps) total += c->num_inputs.size();
    VSec s;
    inst_map->clear();
    while (inst_map->size() < total) {
      size_t best = 0, nc = 0;
      for (size_t i = 0; i < comps.size(); i++)
        if (ptr[i] < comps[i]->num_proofs.size() && comps[i]->num_proofs[ptr[i]] > best) {
          best = comps[i]->num_proofs[ptr[i]];
          nc = i;
        }
      inst_map->push_back(nc);
      s.num_inputs.push_back(comps[nc]->num_inputs[ptr[nc]]);
      s.num_proofs.push_back(comps[nc]->num_proofs[ptr[nc]]);
      s.comm_w.push_back(comps[nc]->comm_w[ptr[nc]]);
      ptr[nc]++;
    }
    return s;
  }
  static VSec concat(const std::vector<const VSec*>& comps) {
    VSec s;
    for (auto c : comps) {
      s.num_inputs.insert(s.num_inputs.end(), c->num_inputs.begin(), c->num_inputs.end());
      s.num_proofs.insert(s.num_proofs.end(), c->num_proofs.begin(), c->num_proofs.end());
      s.comm_w.insert(s.comm_w.end(), c->comm_w.begin(), c->comm_w.end());
    }
    return s;
  }
};
static inline VSec vsec(std::vector<size_t> ni, std::vector<size_t> np, std::vector<PolyCommitment> c) {
  VSec v;
  v.num_inputs = ni;
  v.num_proofs = np;
  v.comm_w = c;
  return v;
}
static inline bool r1cs_verify(const R1CSProof& pf, size_t n, size_t max_np, const std::vector<size_t>& num_proofs,
                               size_t max_ni, const std::vector<const VSec*>& ws, size_t num_cons,
                               const R1CSGens& g, const Fq ev[3], Transcript& t, std::vector<FqVec>* ch) {
  std::vector<std::vector<size_t>> ni, np;
  std::vector<std::vector<PolyCommitment>> cm;
  for (auto w : ws) {
    ni.push_back(w->num_inputs);
    np.push_back(w->num_proofs);
    cm.push_back(w->comm_w);
  }
  return pf.verify(n, max_np, num_proofs, max_ni, ni, np, cm, num_cons, g, ev, t, ch);
}
// verifier side of the per-instance evaluations (lib.rs:3426-3470): rp-bound claims must match the list
static inline bool check_bound_rp(const FqVec& list, const FqVec& rp, const Fq bound[3], const std::vector<size_t>& index) {
  FqVec a, b, c;
  for (size_t i : index) {
    a.push_back(list[3 * i]);
    b.push_back(list[3 * i + 1]);
    c.push_back(list[3 * i + 2]);
  }
  return DensePoly(a).evaluate(rp) == bound[0] && DensePoly(b).evaluate(rp) == bound[1] &&
         DensePoly(c).evaluate(rp) == bound[2];
}

// Replays SNARK::prove's transcript with the verifier's knowledge (public inputs, instance commitments, the
// proof) and checks the three R1CSProofs, their R1CSEvalProofs, the permutation-product openings and identities,
// the shift proofs and the IO proofs (lib.rs:2750-3881). Returns 0 when all checks pass, else the failing stage.
static inline int snark_verify(const SNARKProof& pf, const SnarkIn& in, const SnarkInst& block,
                               const SnarkInst& pairwise, const SnarkInst& perm_root, const R1CSGens& vars_gens,
                               Transcript& t) {
  const size_t niu = in.num_inputs_unpadded, num_ios = in.num_ios;
  const DotGens& gpc = vars_gens.gens_pc;
  t.append_protocol_name("Spartan SNARK proof");
  auto app = [&](const char* l, size_t v) { t.append_scalar(l, fq_from_u64(v)); };
  app("func_input_width", in.func_input_width);
  app("input_offset", in.input_offset);
  app("output_offset", in.output_offset);
  app("output_exec_num", in.output_exec_num);
  app("num_ios", num_ios);
  for (auto n : in.block_num_vars) app("block_num_vars", n);
  app("mem_addr_ts_bits_size", in.mem_addr_ts_bits_size);
  app("num_inputs_unpadded", niu);
  app("block_num_instances_bound", in.block_num_instances_bound);
  app("block_max_num_proofs", in.block_max_num_proofs);
  for (auto p : in.block_num_phy_ops) app("block_num_phy_ops", p);
  for (auto v : in.block_num_vir_ops) app("block_num_vir_ops", v);
  app("total_num_init_phy_mem_accesses", in.total_num_init_phy_mem_accesses);
  app("total_num_init_vir_mem_accesses", in.total_num_init_vir_mem_accesses);
  app("total_num_phy_mem_accesses", in.total_num_phy_mem_accesses);
  app("total_num_vir_mem_accesses", in.total_num_vir_mem_accesses);
  app("block_max_num_proofs", in.block_max_num_proofs);
  for (auto n : in.block_num_proofs) app("block_num_proofs", n);
  for (auto& b : block.label_map)
    for (auto l : b) app("block_comm_map", l);
  for (auto& c : block.comms) c.append(t);
  pairwise.comms[0].append(t);
  perm_root.comms[0].append(t);
  t.append_scalar("input_block_num", fq_from_u64(in.input_block_num));
  t.append_scalar("output_block_num", fq_from_u64(in.output_block_num));
  t.append_scalars("input_list", in.input);
  t.append_scalar("output_list", in.output);
  // sort + pad (sizes only)
  size_t P = 0;
  for (auto n : in.block_num_proofs)
    if (n > 0) P++;
  std::vector<size_t> order(in.block_num_instances_bound);
  for (size_t i = 0; i < order.size(); i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [&](size_t a, size_t b) { return in.block_num_proofs[a] > in.block_num_proofs[b]; });
  order.resize(P);
  std::vector<size_t> bnp, bnv;
  for (size_t i : order) {
    bnp.push_back(next_pow2(in.block_num_proofs[i]));
    bnv.push_back(in.block_num_vars[i]);
  }
  R1CSInstance block_sorted = block.inst;
  block_sorted.sort(P, order);
  const size_t bmax = next_pow2(in.block_max_num_proofs), consis = next_pow2(in.consis_num_proofs);
  // padded memory sizes and the pairwise sort (lib.rs:2951-3009)
  auto pad0 = [](size_t v) { return v == 0 ? size_t(0) : next_pow2(v); };
  const size_t t_iphy = pad0(in.total_num_init_phy_mem_accesses), t_ivir = pad0(in.total_num_init_vir_mem_accesses),
               t_phy = pad0(in.total_num_phy_mem_accesses), t_vir = pad0(in.total_num_vir_mem_accesses);
  std::vector<std::pair<size_t, size_t>> ps = {{consis, 0}, {t_phy, 1}, {t_vir, 2}};
  std::stable_sort(ps.begin(), ps.end(), [](const std::pair<size_t, size_t>& a, const std::pair<size_t, size_t>& b) {
    return a.first > b.first;
  });
  std::vector<size_t> pw_index;
  for (size_t i = 0; i < 1 + (t_phy > 0) + (t_vir > 0); i++) pw_index.push_back(ps[i].second);
  R1CSInstance pairwise_sorted = pairwise.inst;
  pairwise_sorted.sort(pw_index.size(), pw_index);
  // commitments, in the prover's order
  Fq tau = t.challenge_scalar("challenge_tau"), r = t.challenge_scalar("challenge_r");
  FqVec perm_w0 = {tau};
  {
    Fq rt = r;
    for (size_t i = 1; i < 2 * niu; i++) {
      perm_w0.push_back(rt);
      rt = fq_mul(rt, r);
    }
    perm_w0.resize(num_ios, fq_zero());
  }
  PolyCommitment c_w0 = poly_commit(DensePoly(perm_w0), gpc);
  append_polycomm(t, "poly_commitment", c_w0);
  append_polycomm(t, "poly_commitment", pf.perm_exec_comm_w2_list);
  append_polycomm(t, "poly_commitment", pf.perm_exec_comm_w3_list);
  append_polycomm(t, "poly_commitment", pf.perm_exec_comm_w3_shifted);
  if (pf.block_comm_w2_list.size() != P || pf.block_comm_w3_list.size() != P || pf.block_comm_vars_list.size() != P)
    return 1;
  for (auto& c : pf.block_comm_w2_list) append_polycomm(t, "poly_commitment", c);
  for (size_t p = 0; p < P; p++) {
    append_polycomm(t, "poly_commitment", pf.block_comm_w3_list[p]);
    append_polycomm(t, "poly_commitment", pf.block_comm_w3_list_shifted[p]);
  }
  // memory (w2, w3, w3_shifted) triples (lib.rs:3100-3240)
  auto mem_vsecs = [&](size_t total, size_t width, const PolyCommitment& c2, const PolyCommitment& c3,
                       const PolyCommitment& c3s, VSec* w2, VSec* w3, VSec* w3s) {
    if (total == 0) return;
    append_polycomm(t, "poly_commitment", c2);
    append_polycomm(t, "poly_commitment", c3);
    append_polycomm(t, "poly_commitment", c3s);
    *w2 = vsec({width}, {total}, {c2});
    *w3 = vsec({8}, {total}, {c3});
    *w3s = vsec({8}, {total}, {c3s});
  };
  VSec ip2, ip3, ip3s, iv2, iv3, iv3s, pa2, pa3, pa3s, va2, va3, va3s;
  mem_vsecs(t_iphy, INIT_PHY_MEM_WIDTH, pf.init_phy_mem_comm_w2, pf.init_phy_mem_comm_w3,
            pf.init_phy_mem_comm_w3_shifted, &ip2, &ip3, &ip3s);
  mem_vsecs(t_ivir, INIT_VIR_MEM_WIDTH, pf.init_vir_mem_comm_w2, pf.init_vir_mem_comm_w3,
            pf.init_vir_mem_comm_w3_shifted, &iv2, &iv3, &iv3s);
  mem_vsecs(t_phy, PHY_MEM_WIDTH, pf.phy_mem_addr_comm_w2, pf.phy_mem_addr_comm_w3, pf.phy_mem_addr_comm_w3_shifted,
            &pa2, &pa3, &pa3s);
  mem_vsecs(t_vir, VIR_MEM_WIDTH, pf.vir_mem_addr_comm_w2, pf.vir_mem_addr_comm_w3, pf.vir_mem_addr_comm_w3_shifted,
            &va2, &va3, &va3s);
  for (auto& c : pf.block_comm_vars_list) append_polycomm(t, "poly_commitment", c);
  append_polycomm(t, "poly_commitment", pf.exec_comm_inputs[0]);
  // the verifier rebuilds the init lists from the public input stack / input memory (lib.rs:3274-3333):
  // entry i = (1, 0, i, value_i), zero-padded to the power of two
  auto init_vsec = [&](size_t total, size_t n, const std::vector<FqVec>& lst, size_t width) {
    VSec v;
    if (n == 0) return v;
    FqVec flat(total * width, fq_zero());
    for (size_t i = 0; i < n; i++) {
      flat[i * width] = fq_one();
      flat[i * width + 2] = fq_from_u64(i);
      flat[i * width + 3] = lst[i][3];
    }
    PolyCommitment c = poly_commit(DensePoly(flat), gpc);
    append_polycomm(t, "poly_commitment", c);
    return vsec({width}, {total}, {c});
  };
  VSec init_phy_v = init_vsec(t_iphy, in.total_num_init_phy_mem_accesses, in.init_phy_mems_list, INIT_PHY_MEM_WIDTH);
  VSec init_vir_v = init_vsec(t_ivir, in.total_num_init_vir_mem_accesses, in.init_vir_mems_list, INIT_VIR_MEM_WIDTH);
  VSec addr_phy_v, addr_phy_sv, addr_vir_v, addr_vir_sv, ts_bits_v;
  if (t_phy > 0) {
    append_polycomm(t, "poly_commitment", pf.addr_comm_phy_mems);
    append_polycomm(t, "poly_commitment", pf.addr_comm_phy_mems_shifted);
    addr_phy_v = vsec({PHY_MEM_WIDTH}, {t_phy}, {pf.addr_comm_phy_mems});
    addr_phy_sv = vsec({PHY_MEM_WIDTH}, {t_phy}, {pf.addr_comm_phy_mems_shifted});
  }
  if (t_vir > 0) {
    append_polycomm(t, "poly_commitment", pf.addr_comm_vir_mems);
    append_polycomm(t, "poly_commitment", pf.addr_comm_vir_mems_shifted);
    append_polycomm(t, "poly_commitment", pf.addr_comm_ts_bits);
    addr_vir_v = vsec({VIR_MEM_WIDTH}, {t_vir}, {pf.addr_comm_vir_mems});
    addr_vir_sv = vsec({VIR_MEM_WIDTH}, {t_vir}, {pf.addr_comm_vir_mems_shifted});
    ts_bits_v = vsec({in.mem_addr_ts_bits_size}, {t_vir}, {pf.addr_comm_ts_bits});
  }
  // BLOCK_CORRECTNESS_EXTRACT
  std::vector<size_t> w2sz;
  for (size_t p = 0; p < P; p++)
    w2sz.push_back(next_pow2(2 * niu + 2 * in.block_num_phy_ops[order[p]] + 4 * in.block_num_vir_ops[order[p]]));
  VSec bv = vsec(bnv, bnp, pf.block_comm_vars_list), w0 = vsec({num_ios}, {1}, {c_w0}),
       bw2 = vsec(w2sz, bnp, pf.block_comm_w2_list), bw3 = vsec(std::vector<size_t>(P, 8), bnp, pf.block_comm_w3_list),
       bw3s = vsec(std::vector<size_t>(P, 8), bnp, pf.block_comm_w3_list_shifted);
  std::vector<FqVec> ch;
  if (!r1cs_verify(pf.block_r1cs_sat_proof, P, bmax, bnp, in.num_vars, {&bv, &w0, &bw2, &bw3, &bw3s},
                   block_sorted.max_num_cons, vars_gens, pf.block_inst_evals_bound_rp, t, &ch))
    return 2;
  {
    const FqVec &rp = ch[0], &rx = ch[2], &ry = ch[3];
    if (pf.block_inst_evals_list.size() != 3 * block.inst.num_instances) return 3;
    if (!check_bound_rp(pf.block_inst_evals_list, rp, pf.block_inst_evals_bound_rp, order)) return 3;
    for (auto& e : pf.block_inst_evals_list) t.append_scalar("ABCr_claim", e);
    t.challenge_scalar("challenge_c0");
    t.challenge_scalar("challenge_c1");
    t.challenge_scalar("challenge_c2");
    if (pf.block_r1cs_eval_proof_list.size() != block.comms.size()) return 4;
    for (size_t i = 0; i < block.comms.size(); i++) {
      FqVec ev;
      for (auto l : block.label_map[i]) ev.push_back(pf.block_inst_evals_list[l]);
      if (!spark_verify(pf.block_r1cs_eval_proof_list[i], block.comms[i].comm, rx, ry, ev, block.gens.gens, t))
        return 4;
    }
  }
  // PAIRWISE_CHECK (lib.rs:3474-3568): CONSIS_CHECK, PHY_MEM_COHERE, VIR_MEM_COHERE
  VSec pe3 = vsec({8}, {consis}, {pf.perm_exec_comm_w3_list}), pe3s = vsec({8}, {consis}, {pf.perm_exec_comm_w3_shifted});
  const size_t pw_nv = std::max<size_t>(8, in.mem_addr_ts_bits_size);
  std::vector<size_t> pw_map, pw_map2;
  VSec pw = VSec::merge({&pe3, &addr_phy_v, &addr_vir_v}, &pw_map);
  VSec pws = VSec::merge({&pe3s, &addr_phy_sv, &addr_vir_sv}, &pw_map2);
  VSec pwb;
  {
    std::vector<const VSec*> comps(pw_map.size(), &w0);
    for (size_t i = 0; i < pw_map.size(); i++)
      if (pw_map[i] == 2) comps[i] = &ts_bits_v;
    pwb = VSec::concat(comps);
  }
  const size_t pairwise_size = std::max({consis, t_phy, t_vir});
  if (!r1cs_verify(pf.pairwise_check_r1cs_sat_proof, pw.num_proofs.size(), pairwise_size, pw.num_proofs, pw_nv,
                   {&pw, &pws, &pwb}, pairwise_sorted.max_num_cons, vars_gens, pf.pairwise_check_inst_evals_bound_rp,
                   t, &ch))
    return 5;
  {
    const FqVec &rp = ch[0], &rx = ch[2], &ry = ch[3];
    if (!check_bound_rp(pf.pairwise_check_inst_evals_list, rp, pf.pairwise_check_inst_evals_bound_rp, pw_index))
      return 6;
    for (auto& e : pf.pairwise_check_inst_evals_list) t.append_scalar("ABCr_claim", e);
    t.challenge_scalar("challenge_c0");
    t.challenge_scalar("challenge_c1");
    t.challenge_scalar("challenge_c2");
    if (!spark_verify(pf.pairwise_check_r1cs_eval_proof, pairwise.comms[0].comm, rx, ry,
                      pf.pairwise_check_inst_evals_list, pairwise.gens.gens, t))
      return 7;
  }
  // PERM_EXEC_ROOT, MEM_ADDR_ROOT (lib.rs:3569-3650)
  VSec ex1 = vsec({num_ios}, {consis}, {pf.exec_comm_inputs[0]}), pw2 = vsec({num_ios}, {consis}, {pf.perm_exec_comm_w2_list});
  std::vector<size_t> mm;
  VSec r1 = VSec::merge({&ex1, &init_phy_v, &init_vir_v, &addr_phy_v, &addr_vir_v}, &mm);
  VSec r2 = VSec::merge({&pw2, &ip2, &iv2, &pa2, &va2}, &mm);
  VSec r3 = VSec::merge({&pe3, &ip3, &iv3, &pa3, &va3}, &mm);
  VSec r3s = VSec::merge({&pe3s, &ip3s, &iv3s, &pa3s, &va3s}, &mm);
  const size_t perm_size = std::max({consis, t_iphy, t_ivir, t_phy, t_vir});
  if (!r1cs_verify(pf.perm_root_r1cs_sat_proof, r1.num_proofs.size(), perm_size, r1.num_proofs, num_ios,
                   {&w0, &r1, &r2, &r3, &r3s}, perm_root.inst.max_num_cons, vars_gens, pf.perm_root_inst_evals, t, &ch))
    return 8;
  {
    const FqVec &rx = ch[2], &ry = ch[3];
    t.append_scalar("Ar_claim", pf.perm_root_inst_evals[0]);
    t.append_scalar("Br_claim", pf.perm_root_inst_evals[1]);
    t.append_scalar("Cr_claim", pf.perm_root_inst_evals[2]);
    FqVec e(pf.perm_root_inst_evals, pf.perm_root_inst_evals + 3);
    if (!spark_verify(pf.perm_root_r1cs_eval_proof, perm_root.comms[0].comm, rx, ry, e, perm_root.gens.gens, t))
      return 9;
  }
  // PERM_PRODUCT identities (lib.rs:3652-3772): exec == block, phy block == phy addr, vir block == vir addr
  {
    std::vector<const VSec*> comps = {&pe3, &ip3, &iv3, &pa3, &va3, &bw3};
    if (in.max_block_num_phy_ops > 0) comps.push_back(&bw3);
    if (in.max_block_num_vir_ops > 0) comps.push_back(&bw3);
    std::vector<size_t> im;
    VSec m = VSec::merge(comps, &im);
    if (pf.perm_poly_poly_list.size() != m.num_proofs.size()) return 10;
    // the openings of every w3 instance at (1, 0), (1, 0, 0) or (1, 1, 0) (lib.rs:3679-3713)
    const size_t pm_bl_id = 6, vm_bl_id = in.max_block_num_phy_ops > 0 ? 7 : 6;
    std::vector<FqVec> r_list;
    std::vector<size_t> nv_list;
    for (size_t i = 0; i < im.size(); i++) {
      if (im[i] == vm_bl_id) r_list.push_back({fq_one(), fq_one(), fq_zero()});
      else if (im[i] == pm_bl_id) r_list.push_back({fq_one(), fq_zero(), fq_zero()});
      else r_list.push_back({fq_one(), fq_zero()});
      nv_list.push_back(log_2(m.num_proofs[i] * 8));
    }
    if (!verify_plain_batched_instances(pf.proof_eval_perm_poly_prod_list, gpc, t, r_list, pf.perm_poly_poly_list,
                                        m.comm_w, nv_list))
      return 14;
    Fq pe = fq_one(), pb = fq_one(), pmb = fq_one(), pma = fq_one(), vmb = fq_one(), vma = fq_one();
    for (size_t i = 0; i < im.size(); i++) {
      const Fq& v = pf.perm_poly_poly_list[i];
      switch (im[i]) {
        case 0: pe = fq_mul(pe, v); break;
        case 1: pmb = fq_mul(pmb, v); break;
        case 2: vmb = fq_mul(vmb, v); break;
        case 3: pma = fq_mul(pma, v); break;
        case 4: vma = fq_mul(vma, v); break;
        case 5: pb = fq_mul(pb, v); break;
        case 6:
          if (in.max_block_num_phy_ops > 0) pmb = fq_mul(pmb, v);
          else vmb = fq_mul(vmb, v);
          break;
        case 7: vmb = fq_mul(vmb, v); break;
      }
    }
    if (!(pe == pb)) return 11;
    if (!(pmb == pma)) return 12;
    if (!(vmb == vma)) return 13;
  }
  // SHIFT_PROOFS (lib.rs:3772-3853 -> ShiftProofs::verify, :449-506)
  {
    std::vector<const PolyCommitment*> orig = {&pf.perm_exec_comm_w3_list}, shifted = {&pf.perm_exec_comm_w3_shifted};
    std::vector<size_t> sizes = {8 * consis}, hl = {6};
    for (size_t p = 0; p < P; p++) {
      orig.push_back(&pf.block_comm_w3_list[p]);
      shifted.push_back(&pf.block_comm_w3_list_shifted[p]);
      sizes.push_back(8 * bnp[p]);
      hl.push_back(8);
    }
    auto add = [&](const PolyCommitment& o, const PolyCommitment& sh, size_t size, size_t h) {
      orig.push_back(&o);
      shifted.push_back(&sh);
      sizes.push_back(size);
      hl.push_back(h);
    };
    if (t_iphy > 0) add(pf.init_phy_mem_comm_w3, pf.init_phy_mem_comm_w3_shifted, 8 * t_iphy, 6);
    if (t_ivir > 0) add(pf.init_vir_mem_comm_w3, pf.init_vir_mem_comm_w3_shifted, 8 * t_ivir, 6);
    if (t_phy > 0) {
      add(pf.addr_comm_phy_mems, pf.addr_comm_phy_mems_shifted, 4 * t_phy, 4);
      add(pf.phy_mem_addr_comm_w3, pf.phy_mem_addr_comm_w3_shifted, 8 * t_phy, 6);
    }
    if (t_vir > 0) {
      add(pf.addr_comm_vir_mems, pf.addr_comm_vir_mems_shifted, 8 * t_vir, 6);
      add(pf.vir_mem_addr_comm_w3, pf.vir_mem_addr_comm_w3_shifted, 8 * t_vir, 6);
    }
    const ShiftProofs& sp = pf.shift_proof;
    if (sp.openings.size() != orig.size() || sp.C_orig_evals.size() != orig.size() ||
        sp.C_shifted_evals.size() != orig.size())
      return 15;
    for (size_t p = 0; p < hl.size(); p++) {
      if (sp.openings[p].size() < hl[p]) return 15;
      for (size_t i = 0; i < hl[p]; i++) t.append_point("shift_header_entry", sp.openings[p][i].v);
    }
    const Fq c = t.challenge_scalar("challenge_c");
    std::vector<Ge> evals;
    for (auto& e : sp.C_orig_evals) evals.push_back(unpack(e));
    for (auto& e : sp.C_shifted_evals) evals.push_back(unpack(e));
    std::vector<const PolyCommitment*> comms(orig);
    comms.insert(comms.end(), shifted.begin(), shifted.end());
    std::vector<size_t> sz2(sizes);
    sz2.insert(sz2.end(), sizes.begin(), sizes.end());
    if (!verify_uni_batched_instances(sp.proof, gpc, t, c, evals, comms, sz2)) return 15;
  }
  // IO_PROOFS (lib.rs:3855-3873 -> IOProofs::verify, :283-359)
  {
    const size_t r_len = log_2(consis * num_ios);
    std::vector<size_t> idx;
    for (size_t i = 0; i + 2 < in.input_liveness.size(); i++) idx.push_back(2 + in.input_offset + i);
    if (in.input_liveness[1]) idx.insert(idx.begin(), 5);
    if (in.input_liveness[0]) idx.insert(idx.begin(), 6);
    FqVec live;
    for (size_t i = 0; i < in.input_liveness.size(); i++)
      if (in.input_liveness[i]) live.push_back(in.input[i]);
    idx.resize(live.size());
    const size_t oe = in.output_exec_num * num_ios;
    std::vector<size_t> pts = {0, oe, 2, oe + 2 + (niu - 1), oe + 2 + (niu - 1) + in.output_offset - 1};
    pts.insert(pts.end(), idx.begin(), idx.end());
    std::vector<FqVec> r_list;
    for (size_t p : pts) r_list.push_back(to_bin_array(p, r_len));
    FqVec Zr = {fq_one(), fq_one(), fq_from_u64(in.input_block_num), fq_from_u64(in.output_block_num), in.output};
    Zr.insert(Zr.end(), live.begin(), live.end());
    if (pf.exec_comm_inputs.empty() ||
        !verify_plain_batched_points(pf.io_proof.proofs, gpc, t, r_list, Zr, pf.exec_comm_inputs[0]))
      return 16;
  }
  return 0;
}
}  // namespace orc
