"""CPU oracle for SNARK::prove (src/lib.rs:971-2746) on the synthetic program workload: prove -> the oracle's
verifier (three R1CSProofs with their R1CSEvalProofs, rp-bound evaluation claims, permutation-product identity)
accepts, and the proof bytes are frozen in tests/golden/snark_proofs.json."""
import hashlib
import json
import os

import pytest

from r1cs_cases import SNARK_CASES

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("case", sorted(SNARK_CASES))
def test_snark_roundtrip(oracle, case):
    import workload

    wl = workload.SnarkWorkload(**SNARK_CASES[case])
    proof, rc = oracle.snark_prove(wl, workload.tape_seed())
    assert rc == 0, f"oracle verifier rejected at stage {rc}"
    golden = json.load(open(os.path.join(G, "snark_proofs.json")))[case]
    assert golden["proof_len"] == len(proof)
    assert golden["proof_sha256"] == hashlib.sha256(proof).hexdigest()


def test_snark_workload_is_satisfied():
    """the synthetic trace chains outputs to inputs and every block row holds (A z) * (B z) = (C z)"""
    import numpy as np

    import workload

    wl = workload.SnarkWorkload(num_blocks=2, log_cons=5, log_proofs=1, num_vars=32)
    Q = workload.Q
    ex = wl.exec_inputs
    assert ex.shape == (4, wl.num_ios, 4)
    assert wl.output_exec_num == 3 and wl.output_block_num == 2
    mats = wl.block_inst[0]
    # rows of the user part only reference the VAR section; evaluate them on block 0's first execution
    Rinv = pow(workload.R, -1, Q)
    z = [int.from_bytes(np.ascontiguousarray(wl.block_vars[0][0][i]).tobytes(), "little") * Rinv % Q
         for i in range(wl.num_vars)]
    A, B, C = mats[0]
    val = lambda e: int.from_bytes(np.ascontiguousarray(e[2:]).tobytes(), "little") * Rinv % Q
    for row in range(wl.chain + 3):
        s = []
        for M in (A, B, C):
            acc = 0
            for e in M[M[:, 0] == row]:
                acc += val(e) * z[int(e[1])]
            s.append(acc % Q)
        assert s[0] * s[1] % Q == s[2], row


@pytest.mark.parametrize("what", ["phy_data", "vir_data", "ts_bits"])
def test_snark_memory_trace_is_checked(oracle, what):
    """the oracle verifier rejects a memory trace whose address-sorted list disagrees with the block accesses
    (permutation identities, lib.rs:3652-3772) or breaks the coherence rows (PHY/VIR_MEM_COHERE)"""
    import workload

    wl = workload.SnarkWorkload(num_blocks=2, log_cons=6, log_proofs=1, num_vars=64, phy_ops=1, vir_ops=2,
                                init_phy=2, init_vir=2, niu=5)
    if what == "phy_data":
        wl.addr_phy_mems[-1][3] += 1
    elif what == "vir_data":
        wl.addr_vir_mems[-1][3] += 1
    else:
        wl.addr_ts_bits[0][2] ^= 1
    _, rc = oracle.snark_prove(wl, workload.tape_seed())
    assert rc != 0


@pytest.mark.parametrize("tamper,stage", [("io_proof", 16), ("shift_eval", 15), ("perm_opening", 14)])
def test_snark_verifier_checks_openings(oracle, tamper, stage, monkeypatch):
    """the oracle verifier re-checks the perm-product openings (PolyEvalProof::verify_plain_batched_instances),
    the shift proofs (ShiftProofs::verify) and the IO proofs (IOProofs::verify): a verifier that sees swapped IO
    opening proofs, swapped shift evaluations or misplaced perm-product opening proofs rejects at that stage"""
    import workload

    wl = workload.SnarkWorkload(num_blocks=2, log_cons=5, log_proofs=1, num_vars=32)
    monkeypatch.setenv("ORC_TAMPER", tamper)
    _, rc = oracle.snark_prove(wl, workload.tape_seed())
    assert rc == stage
