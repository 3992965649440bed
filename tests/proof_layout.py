"""Field map of bincode(R1CSProof) (src/r1csproof.rs:24-43, serde derive order) used to name the first
differing field when a parity test fails."""
import struct


class _R:
    def __init__(self, b):
        self.b, self.o, self.fields = b, 0, []

    def take(self, name, n):
        self.fields.append((name, self.o, self.o + n))
        self.o += n

    def u64(self, name):
        v = struct.unpack_from("<Q", self.b, self.o)[0]
        self.take(name, 8)
        return v

    def pts(self, name):
        n = self.u64(name + ".len")
        for i in range(n):
            self.take(f"{name}[{i}]", 32)

    def scs(self, name):
        n = self.u64(name + ".len")
        for i in range(n):
            self.take(f"{name}[{i}]", 32)


def _zk_sumcheck(r, name):
    r.pts(name + ".comm_polys")
    r.pts(name + ".comm_evals")
    n = r.u64(name + ".proofs.len")
    for i in range(n):
        p = f"{name}.proofs[{i}]"
        r.take(p + ".delta", 32)
        r.take(p + ".beta", 32)
        r.scs(p + ".z")
        r.take(p + ".z_delta", 32)
        r.take(p + ".z_beta", 32)


def r1cs_proof_fields(b):
    r = _R(b)
    _r1cs(r, "")
    assert r.o == len(b), (r.o, len(b))
    return r.fields


def _r1cs(r, pfx):
    _zk_sumcheck(r, pfx + "sc_proof_phase1")
    for i in range(4):
        r.take(pfx + f"claims_phase2[{i}]", 32)
    for f in ("alpha", "z1", "z2"):
        r.take(pfx + "pok_Cz_claim." + f, 32)
    for f in ("alpha", "beta", "delta", "z0", "z1", "z2", "z3", "z4"):
        r.take(pfx + "proof_prod." + f, 32)
    r.take(pfx + "proof_eq_sc_phase1.alpha", 32)
    r.take(pfx + "proof_eq_sc_phase1.z", 32)
    _zk_sumcheck(r, pfx + "sc_proof_phase2")
    n = r.u64(pfx + "comm_vars_at_ry_list.len")
    for i in range(n):
        r.pts(pfx + f"comm_vars_at_ry_list[{i}]")
    r.take(pfx + "comm_vars_at_ry", 32)
    n = r.u64(pfx + "proof_eval_vars_at_ry_list.len")
    for i in range(n):
        p = pfx + f"proof_eval_vars_at_ry_list[{i}]"
        r.pts(p + ".L")
        r.pts(p + ".R")
        for f in ("delta", "beta", "z1", "z2"):
            r.take(p + "." + f, 32)
    r.take(pfx + "proof_eq_sc_phase2.alpha", 32)
    r.take(pfx + "proof_eq_sc_phase2.z", 32)


def first_diff(a, b):
    """name of the first field whose bytes differ (a, b same length)"""
    for name, s, e in r1cs_proof_fields(a):
        if a[s:e] != b[s:e]:
            return name
    return None


def _batched(r, name):  # ProductCircuitEvalProofBatched (src/product_tree.rs:262-269)
    nl = r.u64(name + ".proof.len")
    for i in range(nl):
        p = f"{name}.proof[{i}]"
        npol = r.u64(p + ".polys.len")
        for j in range(npol):
            r.scs(f"{p}.polys[{j}]")
        r.scs(p + ".claims_prod_left")
        r.scs(p + ".claims_prod_right")
    for k in ("left", "right", "weight"):
        r.scs(f"{name}.claims_dotp.{k}")


def _dotlog(r, name):
    r.pts(name + ".L")
    r.pts(name + ".R")
    for f in ("delta", "beta", "z1", "z2"):
        r.take(name + "." + f, 32)


def spark_proof_fields(b):
    """bincode(SparseMatPolyEvalProof) (src/sparse_mlpoly.rs:1469-1475)"""
    r = _R(b)
    _spark(r, "")
    assert r.o == len(b), (r.o, len(b))
    return r.fields


def _spark(r, pfx):
    r.pts(pfx + "comm_derefs")
    for side in ("row", "col"):
        r.take(pfx + f"{side}_init", 32)
        r.scs(pfx + f"{side}_read")
        r.scs(pfx + f"{side}_write")
        r.take(pfx + f"{side}_audit", 32)
    r.scs(pfx + "dotp_left")
    r.scs(pfx + "dotp_right")
    _batched(r, pfx + "proof_mem")
    _batched(r, pfx + "proof_ops")
    for side in ("row", "col"):
        r.scs(pfx + f"eval_{side}_addr")
        r.scs(pfx + f"eval_{side}_read_ts")
        r.take(pfx + f"eval_{side}_audit_ts", 32)
    r.scs(pfx + "eval_val")
    r.scs(pfx + "eval_row_ops_val")
    r.scs(pfx + "eval_col_ops_val")
    _dotlog(r, pfx + "proof_ops")
    _dotlog(r, pfx + "proof_mem")
    _dotlog(r, pfx + "proof_derefs")


def first_diff_spark(a, b):
    for name, s, e in spark_proof_fields(a):
        if a[s:e] != b[s:e]:
            return name
    return None


def snark_proof_fields(b):
    """bincode(SNARK) (src/lib.rs:701-756)"""
    r = _R(b)

    def comms(name):
        n = r.u64(name + ".len")
        for i in range(n):
            r.pts(f"{name}[{i}]")

    def evalproofs(name):
        n = r.u64(name + ".len")
        for i in range(n):
            _dotlog(r, f"{name}[{i}]")

    comms("block_comm_vars_list")
    comms("exec_comm_inputs")
    for n in ("addr_comm_phy_mems", "addr_comm_phy_mems_shifted", "addr_comm_vir_mems", "addr_comm_vir_mems_shifted",
              "addr_comm_ts_bits", "perm_exec_comm_w2_list", "perm_exec_comm_w3_list", "perm_exec_comm_w3_shifted"):
        r.pts(n)
    for n in ("block_comm_w2_list", "block_comm_w3_list", "block_comm_w3_list_shifted"):
        comms(n)
    for m in ("init_phy_mem", "init_vir_mem", "phy_mem_addr", "vir_mem_addr"):
        for k in ("w2", "w3", "w3_shifted"):
            r.pts(f"{m}_comm_{k}")
    _r1cs(r, "block_r1cs_sat_proof.")
    for i in range(3):
        r.take(f"block_inst_evals_bound_rp[{i}]", 32)
    r.scs("block_inst_evals_list")
    n = r.u64("block_r1cs_eval_proof_list.len")
    for i in range(n):
        _spark(r, f"block_r1cs_eval_proof_list[{i}].")
    _r1cs(r, "pairwise_check_r1cs_sat_proof.")
    for i in range(3):
        r.take(f"pairwise_check_inst_evals_bound_rp[{i}]", 32)
    r.scs("pairwise_check_inst_evals_list")
    _spark(r, "pairwise_check_r1cs_eval_proof.")
    _r1cs(r, "perm_root_r1cs_sat_proof.")
    for i in range(3):
        r.take(f"perm_root_inst_evals[{i}]", 32)
    _spark(r, "perm_root_r1cs_eval_proof.")
    r.scs("perm_poly_poly_list")
    evalproofs("proof_eval_perm_poly_prod_list")
    _dotlog(r, "shift_proof.proof")
    r.pts("shift_proof.C_orig_evals")
    r.pts("shift_proof.C_shifted_evals")
    n = r.u64("shift_proof.openings.len")
    for i in range(n):
        r.pts(f"shift_proof.openings[{i}]")
    evalproofs("io_proof.proofs")
    assert r.o == len(b), (r.o, len(b))
    return r.fields


def first_diff_snark(a, b):
    for name, s, e in snark_proof_fields(a):
        if a[s:e] != b[s:e]:
            return name
    return None
