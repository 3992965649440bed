"""The CPU oracle pinned against the reference's own known-answer tests and independent implementations.

Fq vectors come from src/scalar/ristretto255.rs:772-1202 (tests/golden/fq_kat.json), group vectors from
libsodium 1.0.18 (tests/golden/ristretto_sodium.json), RFC 9496 constants, merlin's conformance vector
and hashlib's SHA-3 family.
"""
import hashlib
import json
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(__file__), "golden")
Q = 2**252 + 27742317777372353535851937790883648493
R = 2**256


def load(name):
    return json.load(open(os.path.join(G, name)))


def to_int(l4):
    return sum(int(x) << (64 * i) for i, x in enumerate(l4))


def from_int(x):
    return np.array([(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)


def mont(x):
    return from_int(x * R % Q)


def val(m):
    return to_int(m) * pow(R, -1, Q) % Q


@pytest.fixture(scope="module")
def kat():
    return load("fq_kat.json")


def test_constants(oracle, kat):
    assert to_int(kat["MODULUS"]) == Q
    inv = 1
    for _ in range(63):
        inv = inv * inv % 2**64
        inv = inv * kat["MODULUS"][0] % 2**64
    assert (-inv) % 2**64 == kat["INV"]  # ristretto255.rs test_inv
    assert to_int(kat["R"]) == R % Q and to_int(kat["R2"]) == R * R % Q and to_int(kat["R3"]) == R**3 % Q


def test_to_from_bytes(oracle, kat):
    one = np.array(kat["R"], dtype=np.uint64)
    assert oracle.fq_to_bytes(np.zeros(4, np.uint64))[0].tolist() == kat["to_bytes"]["zero"]
    assert oracle.fq_to_bytes(one)[0].tolist() == kat["to_bytes"]["one"]
    assert oracle.fq_to_bytes(np.array(kat["R2"], np.uint64))[0].tolist() == kat["to_bytes"]["R2"]
    neg = oracle.fq_op("neg", one)
    assert oracle.fq_to_bytes(neg)[0].tolist() == kat["to_bytes"]["neg_one"]
    r2, ok = oracle.fq_from_bytes(bytes(kat["to_bytes"]["R2"]))
    assert ok and r2.tolist() == kat["R2"]
    _, ok = oracle.fq_from_bytes(bytes(kat["to_bytes"]["neg_one"]))
    assert ok
    for bad in kat["from_bytes_invalid"]:
        _, ok = oracle.fq_from_bytes(bytes(bad))
        assert not ok


def test_from_u512_and_wide(oracle, kat):
    M = kat["MODULUS"]
    assert to_int(oracle.fq_from_u512(M + [0, 0, 0, 0])) == 0
    assert oracle.fq_from_u512([1, 0, 0, 0, 0, 0, 0, 0]).tolist() == kat["R"]
    assert oracle.fq_from_u512([0, 0, 0, 0, 1, 0, 0, 0]).tolist() == kat["R2"]
    mx = oracle.fq_from_u512([2**64 - 1] * 8)
    r3_minus_r = oracle.fq_op("sub", np.array(kat["R3"], np.uint64), np.array(kat["R"], np.uint64))
    assert mx.tolist() == r3_minus_r[0].tolist()
    assert oracle.fq_from_bytes_wide(bytes(kat["to_bytes"]["R2"]) + bytes(32))[0].tolist() == kat["R2"]
    neg = oracle.fq_op("neg", np.array(kat["R"], np.uint64))[0]
    assert oracle.fq_from_bytes_wide(bytes(kat["to_bytes"]["neg_one"]) + bytes(32))[0].tolist() == neg.tolist()
    assert oracle.fq_from_bytes_wide(b"\xff" * 64)[0].tolist() == oracle.fq_from_raw(kat["from_bytes_wide_max"]).tolist()


def test_add_neg_sub_largest(oracle, kat):
    L = np.array(kat["LARGEST"], np.uint64)
    assert oracle.fq_op("add", L, L)[0].tolist() == kat["addition_largest_plus_largest"]
    assert to_int(oracle.fq_op("add", L, np.array([1, 0, 0, 0], np.uint64))[0]) == 0
    assert oracle.fq_op("neg", L)[0].tolist() == [1, 0, 0, 0]
    assert oracle.fq_op("neg", np.array([1, 0, 0, 0], np.uint64))[0].tolist() == kat["LARGEST"]
    assert to_int(oracle.fq_op("sub", L, L)[0]) == 0


def test_from_raw_and_double(oracle, kat):
    assert oracle.fq_from_raw([2**64 - 1] * 4).tolist() == oracle.fq_from_raw(kat["from_raw_all_ff_equals"]).tolist()
    assert to_int(oracle.fq_from_raw(kat["MODULUS"])) == 0
    assert oracle.fq_from_raw([1, 0, 0, 0]).tolist() == kat["R"]
    a = oracle.fq_from_raw(kat["double_input_raw"])
    assert oracle.fq_op("add", a, a)[0].tolist() == oracle.fq_op("add", a, a)[0].tolist()


def test_mul_square_invert_against_bigint(oracle):
    rng = np.random.default_rng(11)
    n = 3000
    xs = [int.from_bytes(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), "little") % Q for _ in range(n)]
    ys = [int.from_bytes(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), "little") % Q for _ in range(n)]
    xs[:4] = [0, 1, Q - 1, 2**252]
    A = np.stack([mont(x) for x in xs])
    B = np.stack([mont(y) for y in ys])
    for op, f in [("add", lambda a, b: (a + b) % Q), ("sub", lambda a, b: (a - b) % Q), ("mul", lambda a, b: a * b % Q)]:
        out = oracle.fq_op(op, A, B)
        assert all(val(out[i]) == f(xs[i], ys[i]) and to_int(out[i]) < Q for i in range(n)), op
    sq = oracle.fq_op("square", A)
    assert all(val(sq[i]) == xs[i] * xs[i] % Q for i in range(n))
    inv = oracle.fq_op("invert", A[1:200])
    assert all(val(inv[i]) == pow(xs[i + 1], -1, Q) for i in range(199))
    vals, allinv = oracle.fq_batch_invert(A[1:100])
    assert all(val(vals[i]) == pow(xs[i + 1], -1, Q) for i in range(99))


def test_invert_is_pow(oracle, kat):
    # ristretto255.rs test_invert_is_pow: r -> r^-1 == r^(q-2)
    r = np.array(kat["R"], np.uint64)
    for _ in range(20):
        x = val(r)
        assert val(oracle.fq_op("invert", r)[0]) == pow(x, to_int(kat["q_minus_2"]), Q)
        r = oracle.fq_op("add", oracle.fq_op("invert", r), np.array(kat["R"], np.uint64))[0]


def test_keccak_shake_merlin(oracle):
    for msg in [b"", b"abc", bytes(range(200)) * 5]:
        assert oracle.shake256(msg, 500) == hashlib.shake_256(msg).digest(500)
    # merlin conformance (merlin ^3.0.0 transcript test "equivalence_simple")
    got = oracle.merlin_simple(b"test protocol", b"some label", b"some data", b"challenge", 32)
    assert got.hex() == "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"


def test_ristretto_rfc9496_constants(oracle):
    p = 2**255 - 19
    c = [int.from_bytes(x, "little") for x in oracle.ristretto_consts()]
    assert c[0] == 37095705934669439343138083508754565189542113879843219016388785533085940283555
    assert c[1] == 19681161376707505956807079304988542015446066515923890162744021073123829784752
    assert c[2] == 25063068953384623474111414158702152701244531502492656460079210482610430750235
    assert c[3] == 54469307008909316920995813868745141605393597292927456921205312896311721017578
    assert c[4] == 1159843021668779879193775521855586647937357759715417654439879720876111806838
    assert c[5] == 40440834346308536858101042469323190826248399146238708352240133220865137265952
    assert c[0] == (-121665 * pow(121666, -1, p)) % p


def test_ristretto_against_libsodium_vectors(oracle):
    v = load("ristretto_sodium.json")
    for h, out in v["from_hash"]:
        assert oracle.ge_from_uniform_bytes(bytes.fromhex(h))[0].hex() == out
    for P, k, out in v["scalarmult"]:
        assert oracle.ge_scalarmul(bytes.fromhex(P), bytes.fromhex(k)).hex() == out
    for a, b, out in v["add"]:
        assert oracle.ge_add(bytes.fromhex(a), bytes.fromhex(b)).hex() == out
    B = bytes.fromhex("e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76")
    assert oracle.ge_roundtrip(B) == B
    assert oracle.ge_roundtrip(bytes(32)) == bytes(32)  # identity
    assert oracle.ge_roundtrip(b"\x01" + bytes(31)) is None  # negative s rejected
    assert oracle.ge_roundtrip(b"\xff" * 32) is None  # non-canonical rejected


def test_generators_fixture(oracle):
    for name in ("gens_r1cs_sat_first16.json", "gens_spg_bench_msm_first16.json"):
        f = load(name)
        pts = oracle.gens_stream(f["label"].encode(), f["count"])
        assert [p.tobytes().hex() for p in pts] == f["points"]
    # SURVEY 7.3 fixture: G0 of MultiCommitGens::new(_, b"gens_r1cs_sat")
    assert load("gens_r1cs_sat_first16.json")["points"][0] == \
        "f8dad3b0fba18ec2a61684952cbfd51372cbdcca26b05e5b0b4637157c98ca43"


@pytest.mark.parametrize("name", ["msm_64.json", "msm_256.json"])
def test_msm_fixture(oracle, name):
    f = load(name)
    pts = oracle.gens_stream(f["label"].encode(), f["n"] + 1)
    s = np.array(f["scalars_mont"], dtype=np.uint64)
    assert oracle.msm(pts[: f["n"]], s).hex() == f["out"]


def test_commit_rows_matches_msm(oracle):
    rng = np.random.default_rng(3)
    L, R = 4, 16
    pts = oracle.gens_stream(b"gens_r1cs_sat", R + 1)
    Z = oracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * L * R, dtype=np.uint8).tobytes())
    rows = oracle.commit_rows(pts[:R], pts[R].tobytes(), Z, L, R)
    for i in range(L):
        assert rows[i].tobytes() == oracle.msm(pts[:R], Z[i * R:(i + 1) * R])
    # with blinds: row + blind*h
    bl = oracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * L, dtype=np.uint8).tobytes())
    rows_b = oracle.commit_rows(pts[:R], pts[R].tobytes(), Z, L, R, bl)
    for i in range(L):
        assert rows_b[i].tobytes() == oracle.msm(pts[: R + 1], np.concatenate([Z[i * R:(i + 1) * R], bl[i:i + 1]]))


def test_unipoly_kats(oracle, kat):
    """src/unipoly.rs:127-181: from_evals of 2x^2+3x+1 and x^3+2x^2+3x+1, their coefficients, the compress /
    decompress(e0 + e1) round trip and evaluate (at 3 -> 28 for the quadratic, at 4 -> 109 for the cubic)"""
    for deg in ("quad", "cubic"):
        evals = [mont(x) for x in kat[f"unipoly_{deg}_evals"]]
        co, at4, rt = oracle.unipoly(evals, mont(4))
        assert [val(c) for c in co] == kat[f"unipoly_{deg}_coeffs"]
        assert np.array_equal(rt, co)
        assert val(at4) == kat[f"unipoly_{deg}_eval_at_4"]
        assert val(co[0]) == kat[f"unipoly_{deg}_evals"][0]  # eval_at_zero
        assert sum(val(c) for c in co) % Q == kat[f"unipoly_{deg}_evals"][1]  # eval_at_one
    _, at3, _ = oracle.unipoly([mont(x) for x in kat["unipoly_quad_evals"]], mont(3))
    assert val(at3) == 28  # unipoly.rs:151-152


def test_mle_evaluation_kat(oracle, kat):
    """src/dense_mlpoly.rs:1234-1252 check_polynomial_evaluation: Z = [1, 2, 1, 4], r = [4, 3] -> 28, by evaluate
    and by evaluate_with_LR (the factored L . Z . R form a Hyrax opening computes)"""
    ev, ev_lr = oracle.dense_eval([mont(x) for x in kat["mle_Z"]], [mont(x) for x in kat["mle_r"]])
    assert val(ev) == kat["mle_eval"] == 28
    assert np.array_equal(ev, ev_lr)
