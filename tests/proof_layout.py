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
    _zk_sumcheck(r, "sc_proof_phase1")
    for i in range(4):
        r.take(f"claims_phase2[{i}]", 32)
    for f in ("alpha", "z1", "z2"):
        r.take("pok_Cz_claim." + f, 32)
    for f in ("alpha", "beta", "delta", "z0", "z1", "z2", "z3", "z4"):
        r.take("proof_prod." + f, 32)
    r.take("proof_eq_sc_phase1.alpha", 32)
    r.take("proof_eq_sc_phase1.z", 32)
    _zk_sumcheck(r, "sc_proof_phase2")
    n = r.u64("comm_vars_at_ry_list.len")
    for i in range(n):
        r.pts(f"comm_vars_at_ry_list[{i}]")
    r.take("comm_vars_at_ry", 32)
    n = r.u64("proof_eval_vars_at_ry_list.len")
    for i in range(n):
        p = f"proof_eval_vars_at_ry_list[{i}]"
        r.pts(p + ".L")
        r.pts(p + ".R")
        for f in ("delta", "beta", "z1", "z2"):
            r.take(p + "." + f, 32)
    r.take("proof_eq_sc_phase2.alpha", 32)
    r.take("proof_eq_sc_phase2.z", 32)
    assert r.o == len(b), (r.o, len(b))
    return r.fields


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
    r.pts("comm_derefs")
    for side in ("row", "col"):
        r.take(f"{side}_init", 32)
        r.scs(f"{side}_read")
        r.scs(f"{side}_write")
        r.take(f"{side}_audit", 32)
    r.scs("dotp_left")
    r.scs("dotp_right")
    _batched(r, "proof_mem")
    _batched(r, "proof_ops")
    for side in ("row", "col"):
        r.scs(f"eval_{side}_addr")
        r.scs(f"eval_{side}_read_ts")
        r.take(f"eval_{side}_audit_ts", 32)
    r.scs("eval_val")
    r.scs("eval_row_ops_val")
    r.scs("eval_col_ops_val")
    _dotlog(r, "proof_ops")
    _dotlog(r, "proof_mem")
    _dotlog(r, "proof_derefs")
    assert r.o == len(b), (r.o, len(b))
    return r.fields


def first_diff_spark(a, b):
    for name, s, e in spark_proof_fields(a):
        if a[s:e] != b[s:e]:
            return name
    return None
