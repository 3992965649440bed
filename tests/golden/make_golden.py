"""Generate the committed golden fixtures under tests/golden/.

Sources, in order of authority:
  1. Known-answer vectors the reference's own tests hold (src/scalar/ristretto255.rs:772-1202,
     src/unipoly.rs:127-181, src/dense_mlpoly.rs:1234-1252) -> fq_kat.json (transcribed values).
  2. libsodium 1.0.18 in this container (/opt/conda/lib/libsodium.so), an independent ristretto255
     implementation -> ristretto_sodium.json.
  3. The CPU oracle (oracle/), after it has been checked against 1 and 2 -> gens_*.json, msm_*.json.
     MSM fixtures are additionally cross-checked against libsodium (sum of scalar multiplications).

Run:  python tests/golden/make_golden.py
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as O  # noqa: E402

Q = 2**252 + 27742317777372353535851937790883648493
P = 2**255 - 19


def le(x, n=32):
    return int(x).to_bytes(n, "little").hex()


def limbs(x):
    return [int((x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF) for i in range(4)]


def fq_kat():
    # values transcribed from the reference's Fq tests (src/scalar/ristretto255.rs)
    largest = [0x5812631A5CF5D3EC, 0x14DEF9DEA2F79CD6, 0x0000000000000000, 0x1000000000000000]
    return {
        "source": "src/scalar/ristretto255.rs:772-1202",
        "MODULUS": [0x5812631A5CF5D3ED, 0x14DEF9DEA2F79CD6, 0, 0x1000000000000000],
        "INV": 0xD2B51DA312547E1B,
        "R": [0xD6EC31748D98951D, 0xC6EF5BF4737DCF70, 0xFFFFFFFFFFFFFFFE, 0x0FFFFFFFFFFFFFFF],
        "R2": [0xA40611E3449C0F01, 0xD00E1BA768859347, 0xCEEC73D217F5BE65, 0x0399411B7C309A3D],
        "R3": [0x2A9E49687B83A2DB, 0x278324E6AEF7F3EC, 0x8065DC6C04EC5B65, 0x0E530B773599CEC7],
        "LARGEST": largest,
        "to_bytes": {
            "zero": [0] * 32,
            "one": [1] + [0] * 31,
            "R2": [29, 149, 152, 141, 116, 49, 236, 214, 112, 207, 125, 115, 244, 91, 239, 198, 254, 255, 255, 255,
                   255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 15],
            "neg_one": [236, 211, 245, 92, 26, 99, 18, 88, 214, 156, 247, 162, 222, 249, 222, 20, 0, 0, 0, 0, 0, 0,
                        0, 0, 0, 0, 0, 0, 0, 0, 0, 16],
        },
        "from_bytes_invalid": [
            [1, 0, 0, 0, 255, 255, 255, 255, 254, 91, 254, 255, 2, 164, 189, 83, 5, 216, 161, 9, 8, 216, 57, 51, 72,
             125, 157, 41, 83, 167, 237, 115],
            [2, 0, 0, 0, 255, 255, 255, 255, 254, 91, 254, 255, 2, 164, 189, 83, 5, 216, 161, 9, 8, 216, 57, 51, 72,
             125, 157, 41, 83, 167, 237, 115],
            [1, 0, 0, 0, 255, 255, 255, 255, 254, 91, 254, 255, 2, 164, 189, 83, 5, 216, 161, 9, 8, 216, 58, 51, 72,
             125, 157, 41, 83, 167, 237, 115],
            [1, 0, 0, 0, 255, 255, 255, 255, 254, 91, 254, 255, 2, 164, 189, 83, 5, 216, 161, 9, 8, 216, 57, 51, 72,
             125, 157, 41, 83, 167, 237, 116],
        ],
        "from_bytes_wide_max": [0xA40611E3449C0F00, 0xD00E1BA768859347, 0xCEEC73D217F5BE65, 0x0399411B7C309A3D],
        "addition_largest_plus_largest": [0x5812631A5CF5D3EB, 0x14DEF9DEA2F79CD6, 0, 0x1000000000000000],
        "from_raw_all_ff_equals": [0xD6EC31748D98951C, 0xC6EF5BF4737DCF70, 0xFFFFFFFFFFFFFFFE, 0x0FFFFFFFFFFFFFFF],
        "double_input_raw": [0x1FFF3231233FFFFD, 0x4884B7FA00034802, 0x998C4FEFECBC4FF3, 0x1824B159ACC50562],
        "q_minus_2": [0x5812631A5CF5D3EB, 0x14DEF9DEA2F79CD6, 0, 0x1000000000000000],
        # src/unipoly.rs:127-181 : 2x^2+3x+1 from evals (1,6,15); x^3+2x^2+3x+1 from evals (1,7,23,55)
        "unipoly_quad_evals": [1, 6, 15],
        "unipoly_quad_coeffs": [1, 3, 2],
        "unipoly_quad_eval_at_4": 45,
        "unipoly_cubic_evals": [1, 7, 23, 55],
        "unipoly_cubic_coeffs": [1, 3, 2, 1],
        "unipoly_cubic_eval_at_4": 109,
        # src/dense_mlpoly.rs:1234-1252 : Z = [1,2,1,4], r = [4,3] -> 28
        "mle_Z": [1, 2, 1, 4],
        "mle_r": [4, 3],
        "mle_eval": 28,
    }


def sodium():
    lib = ctypes.CDLL("/opt/conda/lib/libsodium.so")
    assert lib.sodium_init() >= 0
    return lib


def ristretto_sodium(lib, rng):
    out = {"source": "libsodium 1.0.18 crypto_core_ristretto255_* / crypto_scalarmult_ristretto255", "from_hash": [],
           "scalarmult": [], "add": []}
    for _ in range(32):
        h = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
        o = ctypes.create_string_buffer(32)
        lib.crypto_core_ristretto255_from_hash(o, h)
        out["from_hash"].append([h.hex(), o.raw.hex()])
    pts = [bytes.fromhex(x[1]) for x in out["from_hash"]]
    for i in range(16):
        k = int.from_bytes(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), "little") % Q
        o = ctypes.create_string_buffer(32)
        assert lib.crypto_scalarmult_ristretto255(o, le(k) and bytes.fromhex(le(k)), pts[i]) == 0
        out["scalarmult"].append([pts[i].hex(), le(k), o.raw.hex()])
        o2 = ctypes.create_string_buffer(32)
        lib.crypto_core_ristretto255_add(o2, pts[i], pts[i + 1])
        out["add"].append([pts[i].hex(), pts[i + 1].hex(), o2.raw.hex()])
    return out


def gens_fixture(lib, label, count):
    pts = O.gens_stream(label, count)
    # cross-check against libsodium's one-way map over the same SHAKE256 stream
    basepoint = bytes.fromhex("e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76")
    stream = hashlib.shake_256(label + basepoint).digest(64 * count)
    for i in range(count):
        o = ctypes.create_string_buffer(32)
        lib.crypto_core_ristretto255_from_hash(o, stream[64 * i:64 * i + 64])
        assert o.raw == pts[i].tobytes(), (label, i)
    return {"label": label.decode(), "count": count, "points": [p.tobytes().hex() for p in pts]}


def random_mont_scalars(rng, n):
    raw = rng.integers(0, 256, 64 * n, dtype=np.uint8).tobytes()
    return O.fq_from_bytes_wide(raw)


def edge_scalars():
    # 0, 1, q-1, 2^252, 2, small, (q-1)/2, 2^128 as Montgomery values
    vals = [0, 1, Q - 1, 2**252, 2, 7, (Q - 1) // 2, 2**128]
    return np.stack([O.fq_from_raw(limbs(v)) for v in vals])


def sodium_msm(lib, pts, scalars_mont):
    canon = O.fq_to_bytes(scalars_mont)
    acc = None
    for i in range(len(pts)):
        k = canon[i].tobytes()
        if int.from_bytes(k, "little") == 0:
            continue
        o = ctypes.create_string_buffer(32)
        if lib.crypto_scalarmult_ristretto255(o, k, bytes(pts[i])) != 0:
            continue  # identity result (libsodium returns -1); contributes nothing
        if acc is None:
            acc = o.raw
        else:
            o2 = ctypes.create_string_buffer(32)
            lib.crypto_core_ristretto255_add(o2, acc, o.raw)
            acc = o2.raw
    return acc if acc is not None else bytes(32)


def msm_fixture(lib, rng, label, n, with_edges=True):
    pts = O.gens_stream(label, n + 1)
    s = random_mont_scalars(rng, n)
    if with_edges:
        e = edge_scalars()
        s[: len(e)] = e
    res = O.msm(pts[:n], s)
    assert res == sodium_msm(lib, pts[:n], s), "oracle MSM disagrees with libsodium"
    return {"label": label.decode(), "n": n, "scalars_mont": [[int(x) for x in row] for row in s], "out": res.hex()}


def r1cs_fixture():
    """sha256 of bincode(R1CSProof) from the oracle for tests/r1cs_cases.py, each after prove -> verify."""
    sys.path.insert(0, os.path.join(ROOT, "spartan-parallel_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import workload
    from r1cs_cases import CASES

    out = {}
    for name, (nc, npf, nws, shared) in sorted(CASES.items()):
        wl = workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared)
        pf, _ = O.r1cs_prove(wl, workload.tape_seed())
        assert O.r1cs_verify(wl, pf, workload.tape_seed()) == 1, name
        out[name] = {"len": len(pf), "sha256": hashlib.sha256(pf).hexdigest()}
    return out


def spark_fixture():
    """sha256 of bincode(SparseMatPolyCommitment) and bincode(SparseMatPolyEvalProof) from the oracle, each
    after its verifier accepted (tests/r1cs_cases.py SPARK_CASES)."""
    sys.path.insert(0, os.path.join(ROOT, "spartan-parallel_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import workload
    from r1cs_cases import SPARK_CASES
    from test_oracle_spark import spark_inputs

    out = {}
    for name in sorted(SPARK_CASES):
        wl, rx, ry = spark_inputs(O, name)
        comm, proof, ok = O.spark_prove(wl, rx, ry, workload.tape_seed())
        assert ok, name
        out[name] = {"comm_sha256": hashlib.sha256(comm).hexdigest(), "proof_sha256": hashlib.sha256(proof).hexdigest(),
                     "proof_len": len(proof)}
    return out


def snark_fixture():
    """sha256 of bincode(SNARK) from the oracle's SNARK::prove, each after the oracle's verifier (three
    R1CSProofs, three R1CSEvalProofs, permutation-product identity) accepted (tests/r1cs_cases.py SNARK_CASES)."""
    sys.path.insert(0, os.path.join(ROOT, "spartan-parallel_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import workload
    from r1cs_cases import SNARK_CASES

    out = {}
    for name in sorted(SNARK_CASES):
        wl = workload.SnarkWorkload(**SNARK_CASES[name])
        proof, rc = O.snark_prove(wl, workload.tape_seed())
        assert rc == 0, (name, rc)
        out[name] = {"proof_sha256": hashlib.sha256(proof).hexdigest(), "proof_len": len(proof)}
    return out


def main():
    O.build()
    if sys.argv[1:] == ["snark"]:
        json.dump(snark_fixture(), open(os.path.join(HERE, "snark_proofs.json"), "w"), indent=1)
        return
    if sys.argv[1:] == ["r1cs"]:
        json.dump(r1cs_fixture(), open(os.path.join(HERE, "r1cs_proofs.json"), "w"), indent=1)
        return
    if sys.argv[1:] == ["spark"]:
        json.dump(spark_fixture(), open(os.path.join(HERE, "spark_proofs.json"), "w"), indent=1)
        return
    rng = np.random.default_rng(0x5350415254414E31)
    lib = sodium()
    w = lambda name, obj: json.dump(obj, open(os.path.join(HERE, name), "w"), indent=1)
    w("fq_kat.json", fq_kat())
    w("ristretto_sodium.json", ristretto_sodium(lib, rng))
    w("gens_r1cs_sat_first16.json", gens_fixture(lib, b"gens_r1cs_sat", 16))
    w("gens_spg_bench_msm_first16.json", gens_fixture(lib, b"spg_bench_msm", 16))
    w("msm_64.json", msm_fixture(lib, rng, b"gens_r1cs_sat", 64))
    w("msm_256.json", msm_fixture(lib, rng, b"spg_bench_msm", 256))
    w("r1cs_proofs.json", r1cs_fixture())
    w("spark_proofs.json", spark_fixture())
    w("snark_proofs.json", snark_fixture())
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
