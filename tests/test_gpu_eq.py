"""EqPolynomial::evals (src/dense_mlpoly.rs:76-92) on the GPU (spg_eq_evals -> dev_eq_table) vs the oracle's
field arithmetic running the reference's doubling loop, bit-exact. The sizes cover every launch form of the
device table: one partial block (ell <= 8), whole blocks with a high-bit product (9..16), and the factored
hi (x) lo form (> 16). The restatement itself is pinned against
plain Python integers on the CPU."""
import numpy as np
import pytest

Q = 2**252 + 27742317777372353535851937790883648493
R = 2**256


def eq_ref(oracle, r):
    """src/dense_mlpoly.rs:79-90: evals[2k+1] = evals[k] * r_j, evals[2k] = evals[k] - evals[2k+1]"""
    t = oracle.fq_from_u64(1).reshape(1, 4)
    for x in r:
        hi = oracle.fq_op("mul", t, np.repeat(x.reshape(1, 4), t.shape[0], axis=0))
        lo = oracle.fq_op("sub", t, hi)
        t = np.stack([lo, hi], axis=1).reshape(-1, 4)
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("ell", [0, 1, 2, 3, 4, 7, 8, 9, 11, 12, 13, 16, 17, 20])
def test_eq_evals_match_oracle(ctx, oracle, ell):
    import spg

    rng = np.random.default_rng(100 + ell)
    r = oracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * ell, dtype=np.uint8).tobytes()) if ell else \
        np.zeros((0, 4), dtype=np.uint64)
    got = spg.Buf.eq_evals(ctx, r).download()
    assert got.shape == (1 << ell, 4)
    assert np.array_equal(got, eq_ref(oracle, r))


@pytest.mark.gpu
def test_eq_evals_edge_challenges(ctx, oracle):
    """r_j in {0, 1, q - 1}: the table has exact zeros, ones and signed ones"""
    import spg

    zero, one = oracle.fq_from_u64(0), oracle.fq_from_u64(1)
    minus_one = oracle.fq_op("neg", one).reshape(4)
    r = np.stack([zero, one, minus_one, one, zero, minus_one, minus_one, one, zero, one])
    got = spg.Buf.eq_evals(ctx, r).download()
    assert np.array_equal(got, eq_ref(oracle, r))


def test_eq_ref_matches_python_integers(oracle):
    """CPU: the oracle-arithmetic restatement equals the reference loop run on Python integers"""
    rng = np.random.default_rng(7)
    r = oracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * 6, dtype=np.uint8).tobytes())
    to_int = lambda m: sum(int(m[i]) << (64 * i) for i in range(4)) * pow(R, -1, Q) % Q
    ri = [to_int(x) for x in r]
    ev = [1] * (1 << len(ri))
    size = 1
    for j in range(len(ri)):
        size *= 2
        for i in range(size - 1, 0, -2):
            s = ev[i // 2]
            ev[i] = s * ri[j] % Q
            ev[i - 1] = (s - ev[i]) % Q
    assert [to_int(x) for x in eq_ref(oracle, r)] == ev


@pytest.mark.gpu
def test_mle_kat_on_device_eq_table(ctx, oracle):
    """src/dense_mlpoly.rs:1234-1252: Z = [1, 2, 1, 4] evaluated at r = [4, 3] through the device chi table is 28"""
    import spg

    def m(x):
        v = x * R % Q
        return np.array([(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)

    chi = spg.Buf.eq_evals(ctx, np.stack([m(4), m(3)])).download()
    Z = np.stack([m(x) for x in (1, 2, 1, 4)])
    acc = np.zeros(4, np.uint64)
    for z, c in zip(Z, chi):
        acc = oracle.fq_op("add", acc, oracle.fq_op("mul", z, c))[0]
    assert np.array_equal(acc, m(28))
