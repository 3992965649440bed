"""The product's field / curve / transcript headers (spartan-parallel_amd/csrc/*.hpp) compiled for the
host (lib/libspg_hostcheck.so) and compared bit-for-bit with the CPU oracle. These are the same
sources the HIP kernels compile, so a disagreement here is a kernel bug caught without a GPU."""
import ctypes
import hashlib
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HC = os.environ.get("SPG_HOSTCHECK_LIB") or os.path.join(ROOT, "spartan-parallel_amd", "lib", "libspg_hostcheck.so")
Q = 2**252 + 27742317777372353535851937790883648493
P = 2**255 - 19


@pytest.fixture(scope="module")
def hc():
    if not os.path.exists(HC):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "spartan-parallel_amd"), "lib/libspg_hostcheck.so"])
    return ctypes.CDLL(HC)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def rand_fq(oracle, rng, n):
    return oracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * n, dtype=np.uint8).tobytes())


@pytest.mark.parametrize("op,code", [("add", 0), ("sub", 1), ("mul", 2), ("neg", 3), ("square", 4), ("invert", 5),
                                     ("mul", 8), ("mul", 9)])  # 8, 9: the device's product-scanning and CIOS forms
def test_fq_ops(oracle, hc, op, code):
    rng = np.random.default_rng(code)
    n = 4000 if code != 5 else 2000
    a, b = rand_fq(oracle, rng, n), rand_fq(oracle, rng, n)
    a[0] = 0
    a[1] = oracle.fq_from_u64(1)
    b[2] = oracle.fq_op("neg", oracle.fq_from_u64(1))[0]
    a[3] = b[3] = oracle.fq_op("neg", oracle.fq_from_u64(1))[0]  # (q-1)^2
    if code == 5:
        a[0] = oracle.fq_from_u64(3)
        for i, x in enumerate([2, 4, 1 << 40, 12345678901234567]):  # long runs of trailing zeros
            a[4 + i] = oracle.fq_from_u64(x)
        a[8] = oracle.fq_op("neg", oracle.fq_from_u64(2))[0]
    out = np.zeros_like(a)
    hc.spgh_fq_op(code, _p(a), _p(b), _p(out), ctypes.c_size_t(n))
    ref = oracle.fq_op(op, a, b) if op in ("add", "sub", "mul") else oracle.fq_op(op, a)
    assert np.array_equal(out, ref)


def test_fq_mont_conversion(oracle, hc):
    rng = np.random.default_rng(5)
    a = rand_fq(oracle, rng, 1000)
    out = np.zeros_like(a)
    hc.spgh_fq_op(6, _p(a), None, _p(out), ctypes.c_size_t(1000))
    ref = oracle.fq_to_bytes(a).view(np.uint64).reshape(-1, 4)
    assert np.array_equal(out, ref)


def test_fp_ops_against_bigint(hc):
    rng = np.random.default_rng(9)
    n = 2000
    # loose inputs anywhere in [0, 2^256), including values >= p and near 2^256
    A = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    B = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    A[0] = 0xFFFFFFFF
    B[1] = 0xFFFFFFFF
    A[2] = np.array([0xFFFFFFED] + [0xFFFFFFFF] * 6 + [0x7FFFFFFF], dtype=np.uint32)  # p
    B[3] = 0
    toint = lambda r: sum(int(x) << (32 * i) for i, x in enumerate(r))
    for code, f in [(0, lambda a, b: (a + b) % P), (1, lambda a, b: (a - b) % P), (2, lambda a, b: a * b % P),
                    (3, lambda a, b: a * a % P), (5, lambda a, b: a % P)]:
        out = np.zeros_like(A)
        hc.spgh_fp_op(code, _p(A), _p(B), _p(out), ctypes.c_size_t(n))
        for i in range(n):
            assert toint(out[i]) == f(toint(A[i]), toint(B[i])), (code, i)
    out = np.zeros_like(A)
    hc.spgh_fp_op(4, _p(A[4:104]), None, _p(out), ctypes.c_size_t(100))
    for i in range(100):
        a = toint(A[4 + i]) % P
        assert toint(out[i]) == pow(a, P - 2, P)


def test_fp_device_forms_boundary(hc):
    """the device's product-scanning Fp multiply and squaring (field.hpp mul_8x8 / sqr_8) on the host, on
    random and boundary inputs (all-ones limbs, p, 2^256 - 1, 0) against Python big-int"""
    rng = np.random.default_rng(19)
    n = 3000
    A = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    B = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    edge = [np.full(8, 0xFFFFFFFF, np.uint32), np.zeros(8, np.uint32),
            np.array([0xFFFFFFED] + [0xFFFFFFFF] * 6 + [0x7FFFFFFF], dtype=np.uint32),
            np.array([0xFFFFFFEC] + [0xFFFFFFFF] * 6 + [0x7FFFFFFF], dtype=np.uint32),
            np.array([1, 0, 0, 0, 0, 0, 0, 0], dtype=np.uint32),
            np.array([0xFFFFFFFF] * 4 + [0] * 4, dtype=np.uint32), np.array([0] * 4 + [0xFFFFFFFF] * 4, np.uint32)]
    for i, e in enumerate(edge):
        for j, f in enumerate(edge):
            A[i * len(edge) + j] = e
            B[i * len(edge) + j] = f
    toint = lambda r: sum(int(x) << (32 * i) for i, x in enumerate(r))
    for code, f in [(6, lambda a, b: a * b % P), (7, lambda a, b: a * a % P)]:
        out = np.zeros_like(A)
        hc.spgh_fp_op(code, _p(A), _p(B), _p(out), ctypes.c_size_t(n))
        for i in range(n):
            assert toint(out[i]) == f(toint(A[i]), toint(B[i])), (code, i)


def test_fp_add_sub_double_wrap(hc):
    """fp_add / fp_sub fold a second wrap by 2^256 into limb 0 alone (field.hpp): inputs whose sums or
    differences wrap twice (limbs near 2^32 - 1, values near 2^256 and 0) against Python big-int"""
    vals = [0, 1, 37, 38, 75, 2**255 - 19, 2**255 - 20, 2**256 - 1, 2**256 - 38, 2**256 - 39, 2**256 - 75, 2**128 - 1]
    pairs = [(a, b) for a in vals for b in vals]
    A = np.array([[(a >> (32 * i)) & 0xFFFFFFFF for i in range(8)] for a, _ in pairs], dtype=np.uint32)
    B = np.array([[(b >> (32 * i)) & 0xFFFFFFFF for i in range(8)] for _, b in pairs], dtype=np.uint32)
    toint = lambda r: sum(int(x) << (32 * i) for i, x in enumerate(r))
    for code, f in [(0, lambda a, b: (a + b) % P), (1, lambda a, b: (a - b) % P)]:
        out = np.zeros_like(A)
        hc.spgh_fp_op(code, _p(A), _p(B), _p(out), ctypes.c_size_t(len(pairs)))
        for i, (a, b) in enumerate(pairs):
            assert toint(out[i]) % P == f(a, b), (code, a, b)


def test_fp_addsub_and_mul_k(hc):
    """fp_addsub (one carry pass for lane-dependent add / sub in the quad point arithmetic) returns the same
    representative as fp_add / fp_sub; fp_mul_k (small constants of the scaled quad addition) against big-int"""
    rng = np.random.default_rng(23)
    vals = [0, 1, 37, 38, 75, 2**255 - 19, 2**256 - 1, 2**256 - 38, 2**256 - 39, 2**256 - 75, 2**256 - 76]
    pairs = [(a, b) for a in vals for b in vals]
    n = len(pairs) + 2000
    A = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    B = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    for i, (a, b) in enumerate(pairs):
        A[i] = [(a >> (32 * k)) & 0xFFFFFFFF for k in range(8)]
        B[i] = [(b >> (32 * k)) & 0xFFFFFFFF for k in range(8)]
    toint = lambda r: sum(int(x) << (32 * i) for i, x in enumerate(r))
    raw = {}
    for code in (8, 9, 10, 11):
        raw[code] = np.zeros_like(A)
        hc.spgh_fp_op(code, _p(A), _p(B), _p(raw[code]), ctypes.c_size_t(n))
    assert np.array_equal(raw[8], raw[10]) and np.array_equal(raw[9], raw[11])
    for i in range(n):
        a, b = toint(A[i]), toint(B[i])
        assert toint(raw[8][i]) % P == (a + b) % P and toint(raw[9][i]) % P == (a - b) % P
    B[:, 0] = rng.integers(0, 2**18, size=n, dtype=np.uint64).astype(np.uint32)
    B[:4, 0] = [0, 1, 243330, 2**18 - 1]
    out = np.zeros_like(A)
    hc.spgh_fp_op(12, _p(A), _p(B), _p(out), ctypes.c_size_t(n))
    for i in range(n):
        assert toint(out[i]) == toint(A[i]) * int(B[i, 0]) % P, i


@pytest.mark.parametrize("workers,delay_us", [(7, 0), (7, 50), (3, 200)])
def test_pool_bursts(hc, workers, delay_us):
    """hpool.hpp: bursts of growing / varying size with workers delayed inside their lock-free snapshot;
    every task must run exactly once and be finished when parallel_for returns (stale-snapshot
    race)"""
    hc.spgh_pool_stress.restype = ctypes.c_long
    bad = hc.spgh_pool_stress(workers, 3000 if delay_us == 0 else 400, 64, delay_us, 1234 + delay_us)
    assert bad == 0


def test_curve_ops(oracle, hc):
    rng = np.random.default_rng(12)
    u = rng.integers(0, 256, 64 * 64, dtype=np.uint8)
    out = np.zeros(32 * 64, np.uint8)
    hc.spgh_from_uniform(_p(u), _p(out), ctypes.c_size_t(64))
    ref = oracle.ge_from_uniform_bytes(u.tobytes())
    assert [out[32 * i:32 * i + 32].tobytes() for i in range(64)] == ref
    l_minus_1 = (Q - 1).to_bytes(32, "little")
    for i in range(32):
        A = np.frombuffer(ref[i], np.uint8).copy()
        B = np.frombuffer(ref[i + 1], np.uint8).copy()
        o = np.zeros(32, np.uint8)
        for op in range(4):
            assert hc.spgh_point_op(op, _p(A), _p(B), _p(o)) == 1
            if op in (0, 2):
                exp = oracle.ge_add(ref[i], ref[i + 1])
            elif op == 1:
                exp = oracle.ge_add(ref[i], ref[i])
            else:
                exp = oracle.ge_add(ref[i], oracle.ge_scalarmul(ref[i + 1], l_minus_1))
            assert o.tobytes() == exp
        assert hc.spgh_niels_roundtrip(_p(A), _p(o)) == 1 and o.tobytes() == ref[i]
        assert hc.spgh_roundtrip(_p(A), _p(o)) == 1 and o.tobytes() == ref[i]
    bad = np.frombuffer(b"\x01" + bytes(31), np.uint8).copy()
    assert hc.spgh_roundtrip(_p(bad), _p(o)) == 0


def test_shake_and_merlin(hc):
    for msg in [b"", b"abc", bytes(range(256)) * 3]:
        o = np.zeros(400, np.uint8)
        m = np.frombuffer(msg or b"\0", np.uint8).copy()
        hc.spgh_shake256(_p(m), ctypes.c_size_t(len(msg)), _p(o), ctypes.c_size_t(400))
        assert o.tobytes() == hashlib.shake_256(msg).digest(400)
    o = np.zeros(32, np.uint8)
    m1 = np.frombuffer(b"some data", np.uint8).copy()
    hc.spgh_merlin_simple(b"test protocol", b"some label", _p(m1), ctypes.c_size_t(9), b"challenge", _p(o),
                          ctypes.c_size_t(32))
    assert o.tobytes().hex() == "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"


def test_host_radix51_curve_matches_device_form(hc):
    """hcurve.hpp (host prover arithmetic, radix 2^51) against the device-form curve (8 x u32 limbs):
    compress, decompress, add, mixed add through batch-normalised Niels, dbl, scalar mul."""
    lib = hc
    rng = np.random.default_rng(7)
    n = 64
    uni = rng.integers(0, 256, 64 * n, dtype=np.uint8)
    k = rng.integers(0, 256, 32 * n, dtype=np.uint8)
    k[31::32] &= 0x0F
    bad = lib.spgh_hcurve_check(uni.ctypes.data_as(ctypes.c_void_p), k.ctypes.data_as(ctypes.c_void_p),
                                ctypes.c_size_t(n))
    assert bad == 0


def test_host_ifma_sums_match_scalar(hc):
    """hvec.hpp's 8-lane AVX-512 IFMA sums (mixed additions of Niels entries, full additions of extended points) give
    the scalar additions' points for every length 0 .. 70 (lane padding, one partial group, several groups); skipped
    on a CPU without IFMA, where the prover takes the scalar additions"""
    rng = np.random.default_rng(11)
    n = 70
    uni = rng.integers(0, 256, 64 * n, dtype=np.uint8)
    bad = hc.spgh_vec_check(uni.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n))
    if bad == -1:
        pytest.skip("no AVX-512 IFMA on this CPU")
    assert bad == 0


def test_host_double_and_compress_batch(hc):
    """hcurve.hpp's batched encoding of doubles (one inversion for the batch) gives the bytes of the lone RFC 9496
    encoding of 2 Q for 200 hash-to-group points, each also moved by the 2- and 4-torsion points (same Ristretto
    element, other representatives), and for the identity and the torsion points (zero e g f h: the lone path)"""
    rng = np.random.default_rng(12)
    n = 200
    uni = rng.integers(0, 256, 64 * n, dtype=np.uint8)
    assert hc.spgh_dbl_compress_check(uni.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(n)) == 0


def _mont(x):
    R = 2**256
    v = x * R % Q
    return np.array([(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)


def _val(m):
    return sum(int(x) << (64 * i) for i, x in enumerate(m)) * pow(2**256, -1, Q) % Q


def test_product_unipoly_kat(hc):
    """the prover's round polynomial (hostmath.hpp uni_from_evals3 / uni_eval, the code every ZK and SPARK
    sumcheck round runs) on the reference's cubic KAT, src/unipoly.rs:156-181: evals (1, 7, 23, 55) ->
    x^3 + 2x^2 + 3x + 1, value 109 at 4; and a random cubic against Lagrange interpolation"""
    ev = np.stack([_mont(x) for x in (1, 7, 23, 55)])
    co, at = np.zeros((4, 4), np.uint64), np.zeros(4, np.uint64)
    hc.spgh_uni_from_evals3(_p(ev), _p(_mont(4)), _p(co), _p(at))
    assert [_val(c) for c in co] == [1, 3, 2, 1] and _val(at) == 109
    rng = np.random.default_rng(7)
    cs = [int(x) for x in rng.integers(0, 2**62, 4)]
    f = lambda x: sum(c * x**i for i, c in enumerate(cs)) % Q  # noqa: E731
    ev = np.stack([_mont(f(x)) for x in range(4)])
    hc.spgh_uni_from_evals3(_p(ev), _p(_mont(11)), _p(co), _p(at))
    assert [_val(c) for c in co] == cs and _val(at) == f(11)


def test_product_mle_kat(hc):
    """hostmath.hpp dense_eval_host / eq_evals_host on src/dense_mlpoly.rs:1234-1252: Z = [1, 2, 1, 4] at r = [4, 3]
    is 28; the eq table is big-endian in r (r[0] the most significant index bit, dense_mlpoly.rs:76-92)"""
    Z = np.stack([_mont(x) for x in (1, 2, 1, 4)])
    r = np.stack([_mont(4), _mont(3)])
    out, chis = np.zeros(4, np.uint64), np.zeros((4, 4), np.uint64)
    hc.spgh_dense_eval(_p(Z), ctypes.c_size_t(4), _p(r), ctypes.c_size_t(2), _p(out), _p(chis))
    assert _val(out) == 28
    r0, r1 = 4, 3
    assert [_val(c) for c in chis] == [(1 - r0) * (1 - r1) % Q, (1 - r0) * r1 % Q, r0 * (1 - r1) % Q, r0 * r1 % Q]
