"""SPARK on the GPU (libspg.so: spg_spark_commit / spg_spark_prove) vs the CPU oracle: identical
bincode(SparseMatPolyCommitment) and bincode(SparseMatPolyEvalProof) under the same transcript label and
RandomTape seed. The small cases are pinned by tests/golden/spark_proofs.json (oracle round trips that
verify), the larger one against the oracle run live."""
import hashlib
import json
import os

import pytest

from r1cs_cases import GPU_SPARK_CASES, SPARK_CASES
from test_oracle_spark import spark_inputs

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
GENS_LABEL = b"gens_r1cs_eval"


def gpu_spark(ctx, wl, rx, ry, seed, label=b"spark_test"):
    import spg
    import workload

    v = workload.CViews(wl)
    gens_nnz = len(wl.entries) * max(max(int(m.shape[0]) for m in mats) for mats in wl.entries)
    comm = spg.SparkCommitment(ctx, v.inst, GENS_LABEL, gens_nnz, 3)
    inst = spg.R1CSInst(ctx, v.inst)
    evals = spg.r1cs_multi_evaluate(ctx, inst, len(wl.entries), rx, ry)
    t = spg.Transcript(label)
    tape = spg.RandomTape(b"proof", seed)
    return comm.bytes, comm.prove(rx, ry, evals, t, tape)


def _check(got, ref):
    if got != ref:
        from proof_layout import first_diff_spark

        where = first_diff_spark(got, ref) if len(got) == len(ref) else f"length {len(got)} vs {len(ref)}"
        pytest.fail(f"SPARK proof bytes differ first at {where}")


@pytest.mark.parametrize("case", sorted(SPARK_CASES))
def test_spark_matches_golden(ctx, oracle, case):
    import workload

    wl, rx, ry = spark_inputs(oracle, case)
    comm, proof = gpu_spark(ctx, wl, rx, ry, workload.tape_seed())
    golden = json.load(open(os.path.join(G, "spark_proofs.json")))[case]
    assert hashlib.sha256(comm).hexdigest() == golden["comm_sha256"]
    if hashlib.sha256(proof).hexdigest() != golden["proof_sha256"]:
        _, ref, ok = oracle.spark_prove(wl, rx, ry, workload.tape_seed())
        assert ok
        _check(proof, ref)


@pytest.mark.parametrize("case", sorted(GPU_SPARK_CASES))
def test_spark_matches_oracle_large(ctx, oracle, case):
    import workload

    wl, rx, ry = spark_inputs(oracle, case, GPU_SPARK_CASES)
    comm, proof = gpu_spark(ctx, wl, rx, ry, workload.tape_seed())
    rcomm, ref, ok = oracle.spark_prove(wl, rx, ry, workload.tape_seed())
    assert ok
    assert comm == rcomm
    _check(proof, ref)


def test_spark_repeatable(ctx, oracle):
    import workload

    wl, rx, ry = spark_inputs(oracle, "p2_x64_2secs")
    a = gpu_spark(ctx, wl, rx, ry, workload.tape_seed())
    b = gpu_spark(ctx, wl, rx, ry, workload.tape_seed())
    assert a == b


@pytest.mark.parametrize("env", [{"SPG_WIDE_MIN": "1"}, {"SPG_LAYER_QUAD": "0", "SPG_WIDE_MIN": "1000000000000"},
                                 {"SPG_LAYER_DESC_COPY": "1"}, {"SPG_LAYER_TRIPLE": "0"},
                                 {"SPG_TRIPLE_MAX": "1536", "SPG_WIDE_MIN": "1000000000000", "SPG_STEP_COSTS": "18,25,1"},
                                 {"SPG_STEP_COSTS": "18,10,12"}])
def test_spark_round_kernel_forms(oracle, env):
    """every layer round through the throughput form (k_layer_round_wide, normally only for rounds that fill the
    chip) or through the one-lane form, or the layer descriptors uploaded by a copy instead of riding in the
    eq-table launch; the small rounds paired only (no k_layer_triple), tripled wherever they fit, or paired before
    the triples: same proof bytes as the oracle (a fresh process reads the switches)"""
    import subprocess
    import sys

    import workload

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys, hashlib; sys.path[:0] = [%r, %r, %r]\n"
        "import spg, workload\n"
        "from test_oracle_spark import spark_inputs\n"
        "from test_gpu_spark import gpu_spark\n"
        "import pyoracle\n"
        "wl, rx, ry = spark_inputs(pyoracle, 'p2_x64_2secs')\n"
        "ctx = spg.Context(0)\n"
        "c, p = gpu_spark(ctx, wl, rx, ry, workload.tape_seed())\n"
        "print(hashlib.sha256(p).hexdigest())\n"
    ) % (os.path.join(root, "spartan-parallel_amd"), os.path.join(root, "tests"), os.path.join(root, "oracle"))
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    wl, rx, ry = spark_inputs(oracle, "p2_x64_2secs")
    _, ref, ok = oracle.spark_prove(wl, rx, ry, workload.tape_seed())
    assert ok and out.stdout.split()[-1] == hashlib.sha256(ref).hexdigest()


@pytest.mark.parametrize("case", sorted(SPARK_CASES))
def test_spark_verify(ctx, oracle, case):
    """spg_spark_verify (SparseMatPolyEvalProof::verify) accepts the GPU proof (the oracle's bytes) and rejects it
    with a field altered, other evaluations or another transcript label"""
    import spg
    import workload
    from proof_layout import spark_proof_fields

    wl, rx, ry = spark_inputs(oracle, case)
    v = workload.CViews(wl)
    gens_nnz = len(wl.entries) * max(max(int(m.shape[0]) for m in mats) for mats in wl.entries)
    comm = spg.SparkCommitment(ctx, v.inst, GENS_LABEL, gens_nnz, 3)
    evals = spg.r1cs_multi_evaluate(ctx, spg.R1CSInst(ctx, v.inst), len(wl.entries), rx, ry)
    proof = comm.prove(rx, ry, evals, spg.Transcript(b"spark_test"), spg.RandomTape(b"proof", workload.tape_seed()))
    ok, why = comm.verify(rx, ry, evals, spg.Transcript(b"spark_test"), proof)
    assert ok, why
    ok, _ = comm.verify(rx, ry, evals, spg.Transcript(b"spark_other"), proof)
    assert not ok
    bad_evals = evals.copy()
    bad_evals[0] = workload.to_mont_limbs([1])[0]
    if (bad_evals == evals).all():
        bad_evals[0] = workload.to_mont_limbs([2])[0]
    ok, _ = comm.verify(rx, ry, bad_evals, spg.Transcript(b"spark_test"), proof)
    assert not ok
    fields = spark_proof_fields(proof)
    for name, s, e in fields[:: max(1, len(fields) // 24)]:
        bad = bytearray(proof)
        bad[s + (e - s) // 2] ^= 0x04
        ok, _ = comm.verify(rx, ry, evals, spg.Transcript(b"spark_test"), bytes(bad))
        assert not ok, f"accepted with {name} altered"
