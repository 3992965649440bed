"""The drop-in transcript seam on the GPU: SNARK::prove / R1CSProof::prove / SparseMatPolyEvalProof::prove take the
caller's `&mut merlin::Transcript` (src/lib.rs:1022, src/r1csproof.rs:210-222, src/sparse_mlpoly.rs:1497-1505). libspg
runs them on a transcript whose every append_message / challenge_bytes is forwarded to the caller's own
(spg_transcript_new_callbacks); here that caller-side transcript is the oracle's merlin restatement. The caller appends
messages before the call and draws a challenge after it: the proof bytes must equal the oracle's proof on its own
transcript under the same appends, and both transcripts must end in the same state."""
import numpy as np
import pytest

from r1cs_cases import CASES, SNARK_CASES
from test_gpu_snark import GENS_LABEL, GENS_NV
from test_oracle_spark import spark_inputs

pytestmark = pytest.mark.gpu
PRE = [(b"app-domain", b"caller session 7"), (b"app-nonce", bytes(range(40)))]


def caller_transcript(oracle, label):
    """(the caller's own transcript after its pre-appends, an spg transcript forwarding to it)"""
    import spg

    t = oracle.OracleTranscript(label)
    for lbl, msg in PRE:
        t.append_message(lbl, msg)
    return t, spg.Transcript.from_callbacks(t.append_message, t.challenge_bytes)


def _ref_transcript(oracle, label):
    t = oracle.OracleTranscript(label)
    for lbl, msg in PRE:
        t.append_message(lbl, msg)
    return t


@pytest.fixture(scope="module")
def vars_gens(ctx):
    import spg

    return spg.R1CSGens(ctx, GENS_LABEL, GENS_NV)


@pytest.mark.parametrize("case", ["b2_x32_q2", "mem_both_b3_x64_q2"])
def test_snark_prove_on_caller_transcript(ctx, oracle, vars_gens, case):
    import spg
    import workload

    wl = workload.SnarkWorkload(**SNARK_CASES[case])
    seed = workload.tape_seed()
    v = workload.SnarkViews(wl)
    block, pairwise = spg.SnarkComp(ctx, v.block, multi=True), spg.SnarkComp(ctx, v.pairwise)
    perm_root, wit = spg.SnarkComp(ctx, v.perm_root), spg.SnarkWitness(ctx, v.inputs)
    back, cb = caller_transcript(oracle, b"snark_example")
    got = spg.snark_prove(ctx, block, pairwise, perm_root, wit, vars_gens, cb, spg.RandomTape(b"proof", seed))
    ref_t = _ref_transcript(oracle, b"snark_example")
    ref = oracle.snark_prove_on(wl, seed, ref_t)
    assert got == ref
    assert back.challenge_bytes(b"after", 32) == ref_t.challenge_bytes(b"after", 32)
    # the proof differs from one on a fresh transcript: the pre-appends reached the prover's challenges
    fresh = spg.snark_prove(ctx, block, pairwise, perm_root, wit, vars_gens, spg.Transcript(b"snark_example"),
                            spg.RandomTape(b"proof", seed))
    assert fresh != got


@pytest.mark.parametrize("case", ["p3_ragged_3secs", "p2_x256_2secs"])
def test_r1cs_prove_on_caller_transcript(ctx, oracle, vars_gens, case):
    import spg
    import workload

    nc, npf, nws, shared = CASES[case]
    wl = workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared)
    seed = workload.tape_seed()
    v = workload.CViews(wl)
    inst, wit = spg.R1CSInst(ctx, v.inst), spg.R1CSWitness(ctx, v.secs, wl.nws)
    back, cb = caller_transcript(oracle, b"r1cs_example")
    got, ch = spg.r1cs_prove(ctx, vars_gens, inst, wit, wl.P, wl.max_num_proofs, wl.num_proofs, wl.max_num_inputs,
                             wl.num_inputs, cb, spg.RandomTape(b"proof", seed))
    ref_t = _ref_transcript(oracle, b"r1cs_example")
    ref, ref_ch = oracle.r1cs_prove(wl, seed, transcript=ref_t)
    assert got == ref
    assert all(np.array_equal(a, b) for a, b in zip(ch, ref_ch))
    assert back.challenge_bytes(b"after", 32) == ref_t.challenge_bytes(b"after", 32)


def test_spark_prove_on_caller_transcript(ctx, oracle):
    import spg
    import workload

    wl, rx, ry = spark_inputs(oracle, "p2_x64_2secs")
    seed = workload.tape_seed()
    v = workload.CViews(wl)
    gens_nnz = len(wl.entries) * max(max(int(m.shape[0]) for m in mats) for mats in wl.entries)
    comm = spg.SparkCommitment(ctx, v.inst, b"gens_r1cs_eval", gens_nnz, 3)
    evals = spg.r1cs_multi_evaluate(ctx, spg.R1CSInst(ctx, v.inst), len(wl.entries), rx, ry)
    back, cb = caller_transcript(oracle, b"spark_example")
    got = comm.prove(rx, ry, evals, cb, spg.RandomTape(b"proof", seed))
    ref_t = _ref_transcript(oracle, b"spark_example")
    _, ref, _ = oracle.spark_prove(wl, rx, ry, seed, transcript=ref_t)
    assert got == ref
    assert back.challenge_bytes(b"after", 32) == ref_t.challenge_bytes(b"after", 32)


def test_failing_caller_transcript_fails_the_proof(ctx, oracle, vars_gens):
    """a caller transcript that refuses an operation mid-proof: spg_r1cs_prove returns SPG_E_CALLBACK"""
    import spg
    import workload

    nc, npf, nws, shared = CASES["p2_x4_q2"]
    wl = workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared)
    v = workload.CViews(wl)
    t = oracle.OracleTranscript(b"r1cs_example")
    n = [0]

    def app(label, msg):
        n[0] += 1
        if n[0] == 25:
            raise RuntimeError("refused")
        t.append_message(label, msg)

    cb = spg.Transcript.from_callbacks(app, t.challenge_bytes)
    with pytest.raises(spg.SpgError, match="SPG_E_CALLBACK"):
        spg.r1cs_prove(ctx, vars_gens, spg.R1CSInst(ctx, v.inst), spg.R1CSWitness(ctx, v.secs, wl.nws), wl.P,
                       wl.max_num_proofs, wl.num_proofs, wl.max_num_inputs, wl.num_inputs, cb,
                       spg.RandomTape(b"proof", workload.tape_seed()))
