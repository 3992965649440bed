"""CPU oracle for SPARK (SparseMatPolyEvalProof, src/sparse_mlpoly.rs:1469-1610, with the product-circuit
argument of src/product_tree.rs): multi_commit -> prove -> verify round trips on the synthetic R1CS
matrices, proof bytes frozen in tests/golden/spark_proofs.json."""
import hashlib
import json
import os

import numpy as np
import pytest

from r1cs_cases import SPARK_CASES

G = os.path.join(os.path.dirname(__file__), "golden")


def spark_inputs(oracle, case, cases=SPARK_CASES):
    import workload

    nc, npf, nws, shared = cases[case]
    wl = workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared)
    nx = (wl.max_num_cons - 1).bit_length()
    ny = (wl.num_vars - 1).bit_length()
    rng = np.random.default_rng(3)
    r = oracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * (nx + ny), dtype=np.uint8).tobytes())
    return wl, r[:nx], r[nx:]


@pytest.mark.parametrize("case", sorted(SPARK_CASES))
def test_spark_roundtrip(oracle, case):
    import workload

    wl, rx, ry = spark_inputs(oracle, case)
    comm, proof, ok = oracle.spark_prove(wl, rx, ry, workload.tape_seed())
    assert ok
    golden = json.load(open(os.path.join(G, "spark_proofs.json")))[case]
    assert golden["comm_sha256"] == hashlib.sha256(comm).hexdigest()
    assert golden["proof_sha256"] == hashlib.sha256(proof).hexdigest()
    assert golden["proof_len"] == len(proof)
