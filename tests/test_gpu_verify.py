"""SNARK::verify on the product path (spg_snark_verify, verify.hip; src/lib.rs:2750-3881): every proof the GPU
prover emits for the SNARK cases verifies (those bytes equal the CPU oracle's, whose own verifier accepts them,
tests/test_gpu_snark.py), and the verifier rejects a proof with any field altered, a different transcript label
or different public inputs. Parity of the verdicts with the reference is pinned by construction: the accepted
bytes are the oracle's, and each rejection names the reference check that failed."""
import os

import pytest

from r1cs_cases import GPU_SNARK_CASES, SNARK_CASES

pytestmark = pytest.mark.gpu
CASES = dict(SNARK_CASES, **GPU_SNARK_CASES)


@pytest.fixture(scope="module")
def vars_gens(ctx):
    import spg

    return spg.R1CSGens(ctx, b"gens_r1cs_sat", 1 << 24)


class Program:
    def __init__(self, ctx, vars_gens, case):
        import spg
        import workload

        self.ctx, self.gens = ctx, vars_gens
        self.wl = workload.SnarkWorkload(**CASES[case])
        self.v = workload.SnarkViews(self.wl)
        self.block = spg.SnarkComp(ctx, self.v.block, multi=True)
        self.pairwise = spg.SnarkComp(ctx, self.v.pairwise)
        self.perm_root = spg.SnarkComp(ctx, self.v.perm_root)
        wit = spg.SnarkWitness(ctx, self.v.inputs)
        self.proof = spg.snark_prove(ctx, self.block, self.pairwise, self.perm_root, wit, vars_gens,
                                     spg.Transcript(b"snark_test"), spg.RandomTape(b"proof", workload.tape_seed()))

    def verify(self, proof=None, label=b"snark_test", inputs=None):
        import spg

        return spg.snark_verify(self.ctx, self.block, self.pairwise, self.perm_root, inputs or self.v.inputs,
                                self.gens, spg.Transcript(label), self.proof if proof is None else proof)


@pytest.mark.parametrize("case", sorted(CASES))
def test_verify_accepts(ctx, vars_gens, case):
    ok, why = Program(ctx, vars_gens, case).verify()
    assert ok, why


def test_verify_rejects_altered_fields(ctx, vars_gens):
    """one bit flipped in each of a spread of fields (points, scalars, vector lengths) of every proof part"""
    from proof_layout import snark_proof_fields

    prog = Program(ctx, vars_gens, "mem_both_b3_x64_q2")
    fields = snark_proof_fields(prog.proof)
    step = max(1, len(fields) // 48)
    picked = fields[::step] + [f for f in fields if f[0].endswith(".len")][:8]
    for name, s, e in picked:
        bad = bytearray(prog.proof)
        bad[s + (e - s) // 2] ^= 0x04
        ok, why = prog.verify(bytes(bad))
        assert not ok, f"accepted with {name} altered"
    ok, why = prog.verify(prog.proof[:-1])
    assert not ok and "malformed" in why
    ok, why = prog.verify(prog.proof + b"\x00")
    assert not ok and "malformed" in why


def test_verify_rejects_other_transcript_or_inputs(ctx, vars_gens):
    import ctypes

    import numpy as np

    import workload

    prog = Program(ctx, vars_gens, "b2_x32_q2")
    ok, why = prog.verify(label=b"snark_other")
    assert not ok
    # a different claimed output of the program (the IO proof opens the real one)
    out = np.ascontiguousarray(workload.to_mont_limbs([prog.wl.output + 1])[0])
    prog.v.inputs.output = out.ctypes.data_as(ctypes.c_void_p).value
    ok, why = prog.verify()
    assert not ok, "accepted a wrong output"


@pytest.mark.parametrize("a,b", [("io_proof.proofs[0]", "io_proof.proofs[1]"),
                                 ("shift_proof.C_orig_evals[0]", "shift_proof.C_orig_evals[1]"),
                                 ("block_r1cs_eval_proof_list[0].dotp_left[0]", "block_r1cs_eval_proof_list[0].dotp_right[0]")])
def test_verify_rejects_swapped_parts(ctx, vars_gens, a, b):
    """well-formed proofs with two parts exchanged (the oracle's ORC_TAMPER cases io_proof / shift_eval, whose
    verifier rejects them at IOProofs / ShiftProofs, tests/test_oracle_snark.py): the product verifier rejects too"""
    from proof_layout import snark_proof_fields

    prog = Program(ctx, vars_gens, "b2_x32_q2")
    spans = {}
    for name, s, e in snark_proof_fields(prog.proof):
        for want in (a, b):
            if name == want or name.startswith(want + "."):
                lo, hi = spans.get(want, (s, e))
                spans[want] = (min(lo, s), max(hi, e))
    (sa, ea), (sb, eb) = spans[a], spans[b]
    assert ea - sa == eb - sb and ea <= sb
    p = prog.proof
    swapped = p[:sa] + p[sb:eb] + p[ea:sb] + p[sa:ea] + p[eb:]
    assert swapped != p
    ok, why = prog.verify(swapped)
    assert not ok, f"accepted with {a} and {b} exchanged"


def test_verify_rejects_noncanonical_scalar_limbs(ctx, vars_gens):
    """A proof scalar whose four limbs are >= q (here m + q for the prover's m, the same residue mod q). The
    reference deserialises `Scalar([u64; 4])` without a range check (src/scalar/ristretto255.rs:198) and then runs
    its Montgomery arithmetic on an out-of-range input, whose result is not defined by the field; libspg's reader
    rejects such limbs as malformed. This is a deliberate, stricter deviation, pinned here."""
    from proof_layout import snark_proof_fields

    Q = 2**252 + 27742317777372353535851937790883648493
    prog = Program(ctx, vars_gens, "b2_x32_q2")
    fields = [f for f in snark_proof_fields(prog.proof) if f[0].endswith(".z1")]
    assert fields
    name, s, e = fields[0]
    m = int.from_bytes(prog.proof[s:e], "little")
    assert m < Q
    bad = bytearray(prog.proof)
    bad[s:e] = (m + Q).to_bytes(32, "little")
    ok, why = prog.verify(bytes(bad))
    assert not ok and "malformed" in why, (name, why)


# ---- the verifier's side of the boundary: commitment bytes + public arguments (spg_snark_verify_public) ----------
PUBLIC_CASES = {
    "b2_x32_q2": dict(num_blocks=2, log_cons=5, log_proofs=1, num_vars=32),
    # input stack / memory of power-of-two lengths: SNARK::verify asserts total_num_init_*_mem_accesses ==
    # input_{stack,mem}.len().next_power_of_two() (src/lib.rs:3276-3281)
    "mem_pow2_b3_x64_q2": dict(num_blocks=3, log_cons=6, log_proofs=1, num_vars=64, phy_ops=1, vir_ops=2, init_phy=4,
                               init_vir=8, niu=5),
}
PRE = [(b"app-domain", b"verifier session"), (b"app-nonce", bytes(range(24)))]


def _pre_transcript(oracle, label, pre):
    t = oracle.OracleTranscript(label)
    for lbl, msg in pre:
        t.append_message(lbl, msg)
    return t


@pytest.mark.parametrize("case", sorted(PUBLIC_CASES))
def test_verify_from_commitment_bytes_on_caller_transcript(ctx, oracle, vars_gens, case):
    """The verifier holds only what SNARK::verify is given (src/lib.rs:2750-2798): the ComputationCommitment bytes the
    prover's encoder exported, block_comm_map, the SNARKGens arguments, the public values as [u8; 32] (input stack
    and memory, not their init lists) and its own `&mut Transcript` after application pre-appends (behind
    spg_transcript_new_callbacks). Its verdicts must agree with the CPU oracle's verifier on the same transcripts:
    accept with the prover's pre-appends (and leave the caller transcript in the oracle verifier's state), reject with
    other pre-appends, and reject when one commitment row is swapped for another."""
    import spg
    import workload

    wl = workload.SnarkWorkload(**PUBLIC_CASES[case])
    v = workload.SnarkViews(wl)
    pub = workload.SnarkPublic(wl)
    seed = workload.tape_seed()
    # prover side: encode, export the commitments, prove on the caller's pre-appended transcript
    block = spg.SnarkComp(ctx, v.block, multi=True)
    pairwise = spg.SnarkComp(ctx, v.pairwise)
    perm_root = spg.SnarkComp(ctx, v.perm_root)
    cb, cmap = block.comm_bytes(True), block.comm_map()
    cp, cr = pairwise.comm_bytes(False), perm_root.comm_bytes(False)
    tp = _pre_transcript(oracle, b"snark_pub", PRE)
    proof = spg.snark_prove(ctx, block, pairwise, perm_root, spg.SnarkWitness(ctx, v.inputs), vars_gens,
                            spg.Transcript.from_callbacks(tp.append_message, tp.challenge_bytes),
                            spg.RandomTape(b"proof", seed))
    del block, pairwise, perm_root
    # the oracle: the same proof on the same pre-appends, and its verdict on a verifier transcript with them
    ovt = _pre_transcript(oracle, b"snark_pub", PRE)
    ref, verdict = oracle.snark_prove_verify_on(wl, seed, _pre_transcript(oracle, b"snark_pub", PRE), ovt)
    assert proof == ref and verdict == 0
    # verifier side, from bytes alone
    c = pub.c
    vb = spg.SnarkComp.load(ctx, cb, True, cmap, c.block_num_cons, pub.block_gens)
    vp = spg.SnarkComp.load(ctx, cp, False, None, c.pairwise_check_num_cons, pub.pairwise_gens)
    vr = spg.SnarkComp.load(ctx, cr, False, None, c.perm_root_num_cons, pub.perm_root_gens)

    def verify(pre, comms=(vb, vp, vr)):
        t = _pre_transcript(oracle, b"snark_pub", pre)
        ok, why = spg.snark_verify_public(ctx, *comms, c, vars_gens,
                                          spg.Transcript.from_callbacks(t.append_message, t.challenge_bytes), proof)
        return ok, why, t

    ok, why, t = verify(PRE)
    assert ok, why
    assert t.challenge_bytes(b"after", 32) == ovt.challenge_bytes(b"after", 32), "verifier transcripts diverge"
    other = PRE[:1] + [(b"app-nonce", bytes(range(1, 25)))]
    ok, _, _ = verify(other)
    _, overdict = oracle.snark_prove_verify_on(wl, seed, _pre_transcript(oracle, b"snark_pub", PRE),
                                               _pre_transcript(oracle, b"snark_pub", other))
    assert not ok and overdict != 0, "verdicts on other pre-appends: product accepted or oracle accepted"
    # a verifier holding a wrong commitment: the first two row commitments of the perm-root comb_ops swapped
    bad = bytearray(cr)
    o = 8 * 5 + 8  # num_cons, num_vars, batch_size, num_ops, num_mem_cells, then comm_comb_ops' length
    if len(bad) >= o + 64:
        bad[o:o + 32], bad[o + 32:o + 64] = cr[o + 32:o + 64], cr[o:o + 32]
        if bytes(bad) != cr:
            vr_bad = spg.SnarkComp.load(ctx, bytes(bad), False, None, c.perm_root_num_cons, pub.perm_root_gens)
            ok, _, _ = verify(PRE, (vb, vp, vr_bad))
            assert not ok, "a swapped commitment row was accepted"


def test_comm_load_rejects_malformed_bytes(ctx, vars_gens):
    """truncated or trailing commitment bytes, a wrong num_cons and a map that does not cover the batch are argument
    errors, not a verifier that silently checks against something else"""
    import spg
    import workload

    wl = workload.SnarkWorkload(**PUBLIC_CASES["b2_x32_q2"])
    v = workload.SnarkViews(wl)
    pub = workload.SnarkPublic(wl)
    block = spg.SnarkComp(ctx, v.block, multi=True)
    cb, cmap = block.comm_bytes(True), block.comm_map()
    n = pub.c.block_num_cons
    for bad, m, nc in ((cb[:-1], cmap, n), (cb + b"\0", cmap, n), (cb, cmap, 3 * n), (cb, [l[:-1] for l in cmap], n)):
        with pytest.raises(spg.SpgError, match="SPG_E_ARG"):
            spg.SnarkComp.load(ctx, bad, True, m, nc, pub.block_gens)
