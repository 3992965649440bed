"""The per-operation seams (csrc/seams.hip, include/spg.h "per-operation seams") against the oracle, bit-exact:
DensePolynomial::bound_poly_var_top / _bot / evaluate (src/dense_mlpoly.rs:267-275, 350-358, 361-367) and
SumcheckInstanceProof::prove_cubic with the product-circuit comb A B C (src/sumcheck.rs:193-262,
src/product_tree.rs:185-189), its transcript included. The CPU tests pin the restatement used as the checker: the
oracle's field ops (fq_op, pinned by the reference's Fq KATs in test_oracle_core.py), its UniPoly (pinned by the
reference's UniPoly KATs) and its merlin transcript (pinned by the merlin conformance vector)."""
import numpy as np
import pytest

Q = 2**252 + 27742317777372353535851937790883648493
R = 2**256


def mont(x):
    v = x % Q * R % Q
    return np.array([(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)


def rand_fq(oracle, rng, n):
    return oracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * n, dtype=np.uint8).tobytes()).reshape(n, 4)


def bound_top_ref(oracle, Z, r):
    """src/dense_mlpoly.rs:267-275"""
    n = Z.shape[0] // 2
    lo, hi = Z[:n], Z[n:]
    rr = np.repeat(r.reshape(1, 4), n, axis=0)
    return oracle.fq_op("add", lo, oracle.fq_op("mul", rr, oracle.fq_op("sub", hi, lo)))


def bound_bot_ref(oracle, Z, r):
    """src/dense_mlpoly.rs:350-358"""
    lo, hi = Z[0::2].copy(), Z[1::2].copy()
    rr = np.repeat(r.reshape(1, 4), lo.shape[0], axis=0)
    return oracle.fq_op("add", lo, oracle.fq_op("mul", rr, oracle.fq_op("sub", hi, lo)))


def cubic_evals_ref(oracle, A, B, C):
    """src/sumcheck.rs:207-236 with comb_func = A B C (src/product_tree.rs:185-189)"""
    n = A.shape[0] // 2

    def fsum(v):  # field sum, pairwise
        v = v.reshape(-1, 4)
        while v.shape[0] > 1:
            if v.shape[0] & 1:
                v = np.concatenate([v, np.zeros((1, 4), np.uint64)])
            h = v.shape[0] // 2
            v = oracle.fq_op("add", v[:h], v[h:])
        return v[0]

    def prod(a, b, c):
        return oracle.fq_op("mul", oracle.fq_op("mul", a, b), c)

    def pt2(X):
        return oracle.fq_op("sub", oracle.fq_op("add", X[n:], X[n:]), X[:n])

    def pt3(X, X2):
        return oracle.fq_op("sub", oracle.fq_op("add", X2, X[n:]), X[:n])

    A2, B2, C2 = pt2(A), pt2(B), pt2(C)
    e0 = fsum(prod(A[:n], B[:n], C[:n]))
    e2 = fsum(prod(A2, B2, C2))
    e3 = fsum(prod(pt3(A, A2), pt3(B, B2), pt3(C, C2)))
    return np.stack([e0, e2, e3])


def prove_cubic_ref(oracle, claim, num_rounds, A, B, C, tr):
    """src/sumcheck.rs:193-262 on the oracle's field ops, UniPoly and merlin transcript (tr: OracleTranscript)"""
    e = claim
    polys, rs = [], []
    for _ in range(num_rounds):
        e0, e2, e3 = cubic_evals_ref(oracle, A, B, C)
        evals = np.stack([e0, oracle.fq_op("sub", e, e0)[0], e2, e3])
        coeffs, _, _ = oracle.unipoly(evals, np.zeros(4, np.uint64))
        tr.append_message(b"poly", b"UniPoly_begin")  # src/unipoly.rs:112-120
        for c in coeffs:
            tr.append_message(b"coeff", oracle.fq_to_bytes(c.reshape(1, 4)).tobytes())
        tr.append_message(b"poly", b"UniPoly_end")
        r = oracle.fq_from_bytes_wide(tr.challenge_bytes(b"challenge_nextround", 64)).reshape(4)  # transcript.rs:26-30
        rs.append(r)
        A, B, C = bound_top_ref(oracle, A, r), bound_top_ref(oracle, B, r), bound_top_ref(oracle, C, r)
        _, e, _ = oracle.unipoly(evals, r)
        polys.append(np.stack([coeffs[0], coeffs[2], coeffs[3]]))  # CompressedUniPoly (src/unipoly.rs:82-87)
    return polys, rs, np.stack([A[0], B[0], C[0]])


def test_prove_cubic_ref_is_a_valid_sumcheck(oracle):
    """CPU: the checker's restatement satisfies the sumcheck relations the reference verifier checks
    (src/sumcheck.rs:31-78: poly(0) + poly(1) = e each round; the last e = A(r) B(r) C(r) = claims' product)"""
    rng = np.random.default_rng(5)
    ell = 4
    A, B, C = (rand_fq(oracle, rng, 1 << ell) for _ in range(3))
    claim = cubic_evals_ref(oracle, np.concatenate([A, np.zeros_like(A)]), np.concatenate([B, np.zeros_like(B)]),
                            np.concatenate([C, np.zeros_like(C)]))[0]  # sum_i A_i B_i C_i
    tr = oracle.OracleTranscript(b"cubic")
    polys, rs, claims = prove_cubic_ref(oracle, claim, ell, A, B, C, tr)
    e = claim
    for p, r in zip(polys, rs):
        c0, c2, c3 = p
        # decompress with hint e: c1 = e - 2 c0 - c2 - c3 (src/unipoly.rs:95-108)
        c1 = oracle.fq_op("sub", oracle.fq_op("sub", oracle.fq_op("sub", e, oracle.fq_op("add", c0, c0)), c2), c3)[0]
        at = [c0, c1, c2, c3]
        ev, pw = c0, r
        for c in at[1:]:
            ev = oracle.fq_op("add", ev, oracle.fq_op("mul", c, pw))[0]
            pw = oracle.fq_op("mul", pw, r)[0]
        e = ev
    fin = oracle.fq_op("mul", oracle.fq_op("mul", claims[0], claims[1]), claims[2])[0]
    assert np.array_equal(e, fin)
    # and each claim is the MLE of its table at r (DensePolynomial::evaluate)
    for T, c in zip((A, B, C), claims):
        assert np.array_equal(oracle.dense_eval(T, np.stack(rs))[0], c)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4, 6, 256, 1000, 1 << 16])
def test_bound_top_and_bot_match_oracle(ctx, oracle, n):
    import spg

    rng = np.random.default_rng(n)
    Z, r = rand_fq(oracle, rng, n), rand_fq(oracle, rng, 1)[0]
    for name, ref in (("bound_top", bound_top_ref), ("bound_bot", bound_bot_ref)):
        b = spg.Buf(ctx, Z)
        getattr(b, name)(r)
        assert b.n == n // 2 and spg.lib().spg_buf_len(b.handle) == n // 2
        assert np.array_equal(b.download(), ref(oracle, Z, r)), name


@pytest.mark.gpu
def test_bound_chain_and_edge_challenges(ctx, oracle):
    """r in {0, 1, q - 1} and a chain of folds down to one entry: top then bot alternately, as a caller binding
    variables from both ends would"""
    import spg

    rng = np.random.default_rng(3)
    Z = rand_fq(oracle, rng, 64)
    b = spg.Buf(ctx, Z)
    ref = Z
    rs = [mont(0), mont(1), mont(-1), rand_fq(oracle, rng, 1)[0], mont(2), mont(-1)]
    for k, r in enumerate(rs):
        if k % 2:
            b.bound_bot(r)
            ref = bound_bot_ref(oracle, ref, r)
        else:
            b.bound_top(r)
            ref = bound_top_ref(oracle, ref, r)
        assert np.array_equal(b.download(), ref)
    assert b.n == 1


@pytest.mark.gpu
def test_bound_rejects_odd_or_short(ctx, oracle):
    import spg

    for n in (1, 3):
        b = spg.Buf(ctx, rand_fq(oracle, np.random.default_rng(n), n))
        with pytest.raises(spg.SpgError):
            b.bound_top(mont(5))
        with pytest.raises(spg.SpgError):
            b.bound_bot(mont(5))
        assert b.n == n


@pytest.mark.gpu
@pytest.mark.parametrize("ell", [0, 1, 2, 5, 10, 16])
def test_evaluate_matches_oracle(ctx, oracle, ell):
    import spg

    rng = np.random.default_rng(40 + ell)
    Z = rand_fq(oracle, rng, 1 << ell)
    r = rand_fq(oracle, rng, ell) if ell else np.zeros((0, 4), np.uint64)
    b = spg.Buf(ctx, Z)
    got = b.evaluate(r)
    want = oracle.dense_eval(Z, r)[0] if ell else Z[0]
    assert np.array_equal(got, want)
    assert np.array_equal(b.download(), Z)  # left unchanged


@pytest.mark.gpu
def test_evaluate_mle_kat(ctx):
    """src/dense_mlpoly.rs:1234-1252: Z = [1, 2, 1, 4] at r = [4, 3] is 28"""
    import spg

    b = spg.Buf(ctx, np.stack([mont(x) for x in (1, 2, 1, 4)]))
    assert np.array_equal(b.evaluate(np.stack([mont(4), mont(3)])), mont(28))
    with pytest.raises(spg.SpgError):
        b.evaluate(np.stack([mont(4)]))  # the reference asserts r.len() == num_vars


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8, 1 << 12])
def test_cubic_round_evals_match_oracle(ctx, oracle, n):
    import spg

    rng = np.random.default_rng(70 + n)
    A, B, C = (rand_fq(oracle, rng, n) for _ in range(3))
    got = spg.Buf.cubic_round_evals(spg.Buf(ctx, A), spg.Buf(ctx, B), spg.Buf(ctx, C))
    assert np.array_equal(got, cubic_evals_ref(oracle, A, B, C))


@pytest.mark.gpu
@pytest.mark.parametrize("ell,rounds", [(1, 1), (3, 3), (6, 6), (6, 2), (10, 10)])
def test_prove_cubic_matches_oracle(ctx, oracle, ell, rounds):
    """bytes of the proof (compressed polys), the challenges, the final claims and the transcript state after the
    call (the next challenge) all equal the oracle's; the spg transcript runs over the caller's merlin through the
    drop-in callbacks, so the same transcript object is what both sides advance"""
    import spg

    rng = np.random.default_rng(90 + 7 * ell + rounds)
    A, B, C = (rand_fq(oracle, rng, 1 << ell) for _ in range(3))
    claim = rand_fq(oracle, rng, 1)[0]
    want_polys, want_r, want_claims = prove_cubic_ref(oracle, claim, rounds, A, B, C,
                                                      ref_tr := oracle.OracleTranscript(b"product_tree"))
    caller = oracle.OracleTranscript(b"product_tree")
    t = spg.Transcript.from_callbacks(caller.append_message, caller.challenge_bytes)
    bA, bB, bC = spg.Buf(ctx, A), spg.Buf(ctx, B), spg.Buf(ctx, C)
    polys, r, claims = spg.Buf.prove_cubic(claim, rounds, bA, bB, bC, t)
    assert np.array_equal(polys, np.stack(want_polys))
    assert np.array_equal(r, np.stack(want_r))
    if rounds == ell:
        assert np.array_equal(claims, want_claims)
    else:  # the tables stay partly bound: claims are their first entries, the rest must match too
        assert np.array_equal(bA.download(), bound_chain(oracle, A, want_r))
        assert np.array_equal(claims[0], bound_chain(oracle, A, want_r)[0])
    assert bA.n == 1 << (ell - rounds)
    assert caller.challenge_bytes(b"after", 32) == ref_tr.challenge_bytes(b"after", 32)


def bound_chain(oracle, T, rs):
    for r in rs:
        T = bound_top_ref(oracle, T, r)
    return T


@pytest.mark.gpu
def test_prove_cubic_native_transcript_and_bad_shapes(ctx, oracle):
    """spg's own transcript gives the same proof as the callback one; non-power-of-two or too-short tables and
    mismatched lengths are SPG_E_ARG before any round"""
    import spg

    rng = np.random.default_rng(11)
    A, B, C = (rand_fq(oracle, rng, 16) for _ in range(3))
    claim = mont(12345)
    p1 = spg.Buf.prove_cubic(claim, 4, spg.Buf(ctx, A), spg.Buf(ctx, B), spg.Buf(ctx, C), spg.Transcript(b"pt"))
    want = prove_cubic_ref(oracle, claim, 4, A, B, C, oracle.OracleTranscript(b"pt"))
    assert np.array_equal(p1[0], np.stack(want[0])) and np.array_equal(p1[2], want[2])
    with pytest.raises(spg.SpgError):
        spg.Buf.prove_cubic(claim, 5, spg.Buf(ctx, A), spg.Buf(ctx, B), spg.Buf(ctx, C), spg.Transcript(b"pt"))
    with pytest.raises(spg.SpgError):
        spg.Buf.prove_cubic(claim, 1, spg.Buf(ctx, A), spg.Buf(ctx, B[:8]), spg.Buf(ctx, C), spg.Transcript(b"pt"))
    with pytest.raises(spg.SpgError):
        spg.Buf.prove_cubic(claim, 1, spg.Buf(ctx, A[:12]), spg.Buf(ctx, B[:12]), spg.Buf(ctx, C[:12]),
                            spg.Transcript(b"pt"))


# ---- DensePolynomialPqx (src/custom_dense_mlpoly.rs:22-359) ----

def pqx_py(z, num_proofs, max_np, nws, num_inputs, max_ni, steps):
    """pure-Python restatement of new + bound_poly (custom_dense_mlpoly.rs:45-64, 205-289) on integers mod q, small
    sizes only: pins the oracle's C++ (orc_pqx_bind) on the CPU"""
    P = len(num_proofs)
    Z, k = [], 0
    for p in range(P):
        Z.append([[[z[k + (q * nws + w) * num_inputs[p] + x] for x in range(num_inputs[p])] for w in range(nws)]
                  for q in range(num_proofs[p])])
        k += num_proofs[p] * nws * num_inputs[p]
    ninst, nw2 = 1 << (P - 1).bit_length(), 1 << (nws - 1).bit_length()
    npf, nin = list(num_proofs), list(num_inputs)
    for mode, r in steps:
        if mode == 1:
            if max_np != 1 or max_ni != 1:
                return None
            ninst //= 2
            for p in range(ninst):
                for w in range(min(nw2, len(Z[p][0]))):
                    hi = Z[p + ninst][0][w][0] if p + ninst < P else 0
                    Z[p][0][w][0] = (Z[p][0][w][0] + r * (hi - Z[p][0][w][0])) % Q
        elif mode == 2:
            max_np //= 2
            for p in range(min(ninst, P)):
                if npf[p] == 1:
                    for w in range(min(nw2, len(Z[p][0]))):
                        for x in range(nin[p]):
                            Z[p][0][w][x] = (1 - r) * Z[p][0][w][x] % Q
                else:
                    npf[p] //= 2
                    for q in range(npf[p]):
                        for w in range(min(nw2, len(Z[p][q]))):
                            for x in range(nin[p]):
                                Z[p][q][w][x] = (Z[p][q][w][x] + r * (Z[p][q + npf[p]][w][x] - Z[p][q][w][x])) % Q
        elif mode == 3:
            nw2 //= 2
            for p in range(min(ninst, P)):
                for q in range(npf[p]):
                    for w in range(nw2):
                        for x in range(nin[p]):
                            hi = Z[p][q][w + nw2][x] if w + nw2 < len(Z[p][q]) else 0
                            Z[p][q][w][x] = (Z[p][q][w][x] + r * (hi - Z[p][q][w][x])) % Q
        else:
            max_ni //= 2
            for p in range(min(ninst, P)):
                if nin[p] == 1:
                    for q in range(npf[p]):
                        for w in range(min(nw2, len(Z[p][q]))):
                            Z[p][q][w][0] = (1 - r) * Z[p][q][w][0] % Q
                else:
                    nin[p] //= 2
                    for q in range(npf[p]):
                        for w in range(min(nw2, len(Z[p][q]))):
                            for x in range(nin[p]):
                                Z[p][q][w][x] = (Z[p][q][w][x] + r * (Z[p][q][w][x + nin[p]] - Z[p][q][w][x])) % Q
    flat = [v for p in Z for q in p for w in q for v in w]
    return flat, (ninst, max_np, nw2, max_ni), npf, nin


def to_int(m):
    return sum(int(m[i]) << (64 * i) for i in range(4)) * pow(R, -1, Q) % Q


# (num_proofs, max_num_proofs, num_witness_secs, num_inputs, max_num_inputs): ragged q and x, a w count that is not a
# power of two (zero hi sections), single-proof / single-input instances, and > 32 instances (descriptors in HBM)
PQX_SHAPES = [
    ([4, 1, 2], 4, 3, [8, 2, 1], 8),
    ([2, 2], 2, 4, [4, 4], 4),
    ([1], 1, 1, [1], 1),
    ([8, 4, 4, 2, 1], 8, 2, [16, 16, 4, 8, 2], 16),
    ([2] * 20 + [1] * 20, 2, 3, [4] * 40, 4),
]


def pqx_plan(shape, order):
    """a full set of binds: every x, w, q variable, then p (the R1CS proof's order is x first, then w, q, p), or
    q / w / x interleaved"""
    npf, max_np, nws, nin, max_ni = shape
    lx, lq = (max_ni - 1).bit_length(), (max_np - 1).bit_length()
    lw, lp = (nws - 1).bit_length(), (len(npf) - 1).bit_length()
    if order == "xwqp":
        modes = [4] * lx + [3] * lw + [2] * lq
    else:
        modes = [2] * lq + [4] * lx + [3] * lw
        modes = modes[::2] + modes[1::2]
    return modes + [1] * lp


def test_pqx_oracle_matches_python_loops(oracle):
    """CPU: orc_pqx_bind equals the reference loops restated on Python integers, after every bind, including the
    panic case (p bound first)"""
    rng = np.random.default_rng(17)
    for shape in PQX_SHAPES[:4]:
        npf, max_np, nws, nin, max_ni = shape
        n = sum(a * nws * b for a, b in zip(npf, nin))
        z = rand_fq(oracle, rng, n)
        for order in ("xwqp", "mixed"):
            modes = pqx_plan(shape, order)
            rs = rand_fq(oracle, rng, len(modes)) if modes else np.zeros((0, 4), np.uint64)
            for k in range(len(modes) + 1):
                got = oracle.pqx_bind(z, npf, max_np, nws, nin, max_ni, modes[:k], rs[:k])
                want = pqx_py([to_int(v) for v in z], npf, max_np, nws, nin, max_ni,
                              [(m, to_int(r)) for m, r in zip(modes[:k], rs[:k])])
                assert [to_int(v) for v in got[0]] == want[0] and list(got[1:]) == list(want[1:])
        if max_np > 1 or max_ni > 1:
            assert oracle.pqx_bind(z, npf, max_np, nws, nin, max_ni, [1], rand_fq(oracle, rng, 1)) is None
            assert pqx_py([0] * n, npf, max_np, nws, nin, max_ni, [(1, 5)]) is None


@pytest.mark.gpu
@pytest.mark.parametrize("si", range(len(PQX_SHAPES)))
@pytest.mark.parametrize("order", ["xwqp", "mixed"])
def test_pqx_bound_matches_oracle(ctx, oracle, si, order):
    """every allocated entry and every size field after each bind equal the oracle's"""
    import spg

    shape = PQX_SHAPES[si]
    npf, max_np, nws, nin, max_ni = shape
    rng = np.random.default_rng(200 + si)
    z = rand_fq(oracle, rng, sum(a * nws * b for a, b in zip(npf, nin)))
    modes = pqx_plan(shape, order)
    rs = rand_fq(oracle, rng, max(len(modes), 1))
    T = spg.Pqx(ctx, z, npf, max_np, nws, nin, max_ni)
    assert np.array_equal(T.download(), z)
    for k, m in enumerate(modes):
        T.bound(rs[k], m)
        want = oracle.pqx_bind(z, npf, max_np, nws, nin, max_ni, modes[:k + 1], rs[:k + 1])
        assert np.array_equal(T.download(), want[0]), (k, m)
        dims, gp, gi = T.shape()
        assert (dims, gp, gi) == (want[1], want[2], want[3])


@pytest.mark.gpu
@pytest.mark.parametrize("si", range(len(PQX_SHAPES)))
def test_pqx_evaluate_matches_oracle(ctx, oracle, si):
    """evaluate(r_p, r_q, r_w, r_x) = the oracle's x, w, q, p binds then index(0, 0, 0, 0); the table is unchanged;
    a p bind before q and x are bound is SPG_E_ARG (the reference's assert)"""
    import spg

    npf, max_np, nws, nin, max_ni = PQX_SHAPES[si]
    rng = np.random.default_rng(300 + si)
    z = rand_fq(oracle, rng, sum(a * nws * b for a, b in zip(npf, nin)))
    lx, lq = (max_ni - 1).bit_length(), (max_np - 1).bit_length()
    lw, lp = (nws - 1).bit_length(), (len(npf) - 1).bit_length()
    rp, rq, rw, rx = (rand_fq(oracle, rng, n) if n else np.zeros((0, 4), np.uint64) for n in (lp, lq, lw, lx))
    T = spg.Pqx(ctx, z, npf, max_np, nws, nin, max_ni)
    got = T.evaluate(rp, rq, rw, rx)
    want = oracle.pqx_bind(z, npf, max_np, nws, nin, max_ni, [4] * lx + [3] * lw + [2] * lq + [1] * lp,
                           np.concatenate([rx, rw, rq, rp]))
    assert np.array_equal(got, want[0][0])
    assert np.array_equal(T.download(), z)
    if max_np > 1 or max_ni > 1:
        with pytest.raises(spg.SpgError):
            T.bound(mont(3), 1)
        with pytest.raises(spg.SpgError):
            T.evaluate(rp if lp else np.stack([mont(2)]), [], rw, rx)


@pytest.mark.gpu
def test_pqx_rejects_bad_shapes(ctx, oracle):
    import spg

    z = rand_fq(oracle, np.random.default_rng(1), 64)
    for npf, max_np, nin, max_ni in (([3], 4, [4], 4), ([4], 2, [4], 4), ([2], 2, [4], 3)):
        with pytest.raises(spg.SpgError):
            spg.Pqx(ctx, z, npf, max_np, 1, nin, max_ni)
    T = spg.Pqx(ctx, z[:8], [2], 2, 1, [4], 4)
    with pytest.raises(spg.SpgError):
        T.bound(mont(1), 5)


# ---- R1CSInstance::multiply_vec_block (src/r1csinstance.rs:363-436) ----
# (num_cons, num_proofs, witness sections, one shared instance): ragged q, several sections, a shared matrix, and
# > 32 instances (k_spmv's descriptors in HBM)
SPMV_CASES = {
    "ragged3": ([16, 8, 4], [4, 1, 2], 3, False),
    "shared": ([8, 8], [2, 4], 2, True),
    "one": ([32], [8], 1, False),
    "many": ([4] * 36, [2] * 18 + [1] * 18, 2, False),
}


def spmv_workload(oracle, case):
    import workload

    nc, npf, nws, shared = SPMV_CASES[case]
    wl = workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared)
    rng = np.random.default_rng(len(case))
    for mats in wl.entries:  # random matrix values instead of the synthetic circuit's ones
        for m in mats:
            m[:, 2:] = rand_fq(oracle, rng, m.shape[0])
    z = np.concatenate([np.stack([wl.sections[w][p][q] for w in range(wl.nws)]).reshape(-1, 4)
                        for p in range(wl.P) for q in range(wl.num_proofs[p])])
    return wl, z


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(SPMV_CASES))
def test_multiply_vec_block_matches_oracle(ctx, oracle, case):
    """Az, Bz, Cz entry by entry in new_rev order and their sizes; then Az bound through the Pqx seam as the R1CS
    proof binds it (x rounds first) equals the oracle's"""
    import spg
    import workload

    wl, z = spmv_workload(oracle, case)
    v = workload.CViews(wl)
    inst = spg.R1CSInst(ctx, v.inst)
    got = spg.r1cs_multiply_vec_block(ctx, inst, wl.num_proofs, wl.max_num_proofs, wl.num_inputs, wl.max_num_inputs,
                                      wl.nws, z)
    want = oracle.r1cs_multiply_vec_block(wl, z, wl.num_inputs)
    nc = [wl.num_cons[0 if wl.shared else p] for p in range(wl.P)]
    for T, W in zip(got, want):
        assert np.array_equal(T.download(), W)
        dims, gp, gi = T.shape()
        assert dims == (1 << (wl.P - 1).bit_length(), wl.max_num_proofs, 1, wl.max_num_cons)
        assert gp == list(wl.num_proofs) and gi == nc
    lx, lq = (wl.max_num_cons - 1).bit_length(), (wl.max_num_proofs - 1).bit_length()
    modes = [4] * lx + [2] * lq
    rs = rand_fq(oracle, np.random.default_rng(9), max(len(modes), 1))
    for k, m in enumerate(modes):
        got[0].bound(rs[k], m)
    ref = oracle.pqx_bind(want[0], wl.num_proofs, wl.max_num_proofs, 1, nc, wl.max_num_cons, modes, rs[:len(modes)])
    assert np.array_equal(got[0].download(), ref[0])


@pytest.mark.gpu
def test_multiply_vec_block_rejects_bad_shapes(ctx, oracle):
    import spg
    import workload

    wl, z = spmv_workload(oracle, "ragged3")
    inst = spg.R1CSInst(ctx, workload.CViews(wl).inst)
    with pytest.raises(spg.SpgError):  # 2 instances against a 3-instance matrix list
        spg.r1cs_multiply_vec_block(ctx, inst, wl.num_proofs[:2], wl.max_num_proofs, wl.num_inputs[:2],
                                    wl.max_num_inputs, wl.nws, z)
    with pytest.raises(spg.SpgError):  # num_proofs not a power of two
        spg.r1cs_multiply_vec_block(ctx, inst, [3, 1, 2], 4, wl.num_inputs, wl.max_num_inputs, wl.nws, z)
    with pytest.raises(spg.SpgError):  # 9 sections
        spg.r1cs_multiply_vec_block(ctx, inst, wl.num_proofs, wl.max_num_proofs, wl.num_inputs, wl.max_num_inputs, 9,
                                    np.zeros((4096, 4), np.uint64))


# ---- one phase-1 round (src/sumcheck.rs:1173-1245) ----

def phase1_round_py(Ap, Aq, Ax, tabs, shape, mode):
    """the reference's round loop on Python integers: tabs = (B, C, D) as integer lists in the Pqx allocation layout,
    shape = (anp, ani, num_proofs, num_inputs) -- current sizes before the round's halving"""
    anp, ani, npf, nin = shape
    P = len(npf)
    off = [sum(anp[k] * ani[k] for k in range(p)) for p in range(P)]
    instance_len, proof_len = len(Ap), len(Aq) // 2 if mode == 2 else len(Aq)
    cons_len = len(Ax) // 2 if mode == 4 else len(Ax)

    def idx(T, p, q, x):
        return T[off[p] + q * ani[p] + x] if (p < P and q < anp[p] and x < ani[p]) else 0

    def idx_hi(T, p, q, x):
        if mode == 4:
            return 0 if nin[p] == 1 else T[off[p] + q * ani[p] + x + nin[p] // 2]
        return 0 if npf[p] == 1 else T[off[p] + (q + npf[p] // 2) * ani[p] + x]

    e = [0, 0, 0]
    comb = lambda a, b, c, d: a * (b * c - d)  # noqa: E731 (r1csproof.rs comb_func)
    for p in range(min(instance_len, P)):
        lnc = nin[p] // 2 if (mode == 4 and nin[p] > 1) else nin[p]
        lnp = npf[p] // 2 if (mode == 2 and npf[p] > 1) else npf[p]
        for q in range(lnp):
            sq, sx = proof_len // lnp, cons_len // lnc
            for x in range(lnc):
                a = Ap[p] * Aq[q * sq] * Ax[x * sx]
                ah = Ap[p] * (Aq[q * sq + proof_len] * Ax[x * sx] if mode == 2 else Aq[q * sq] * Ax[x * sx + cons_len])
                lo = [idx(T, p, q, x) for T in tabs]
                hi = [idx_hi(T, p, q, x) for T in tabs]
                e[0] += comb(a, *lo)
                b2 = [2 * h - l for h, l in zip(hi, lo)]
                a2 = 2 * ah - a
                e[1] += comb(a2, *b2)
                b3 = [v + h - l for v, h, l in zip(b2, hi, lo)]
                e[2] += comb(a2 + ah - a, *b3)
    return [v % Q for v in e]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["ragged3", "shared", "many"])
def test_phase1_rounds_match_python_loop(ctx, oracle, case):
    """every x round then every q round of phase 1 on Az, Bz, Cz from the SpMV seam: (e0, e2, e3) against the
    reference loop restated on Python integers, the tables bound between rounds through the seams"""
    import spg
    import workload

    wl, z = spmv_workload(oracle, case)
    inst = spg.R1CSInst(ctx, workload.CViews(wl).inst)
    tabs = spg.r1cs_multiply_vec_block(ctx, inst, wl.num_proofs, wl.max_num_proofs, wl.num_inputs, wl.max_num_inputs,
                                       wl.nws, z)
    rng = np.random.default_rng(77)
    lp = (wl.P - 1).bit_length()
    eq = [spg.Buf(ctx, rand_fq(oracle, rng, n)) for n in (1 << lp, wl.max_num_proofs, wl.max_num_cons)]
    Ap, Aq, Ax = eq
    lx, lq = (wl.max_num_cons - 1).bit_length(), (wl.max_num_proofs - 1).bit_length()
    anp, ani = list(wl.num_proofs), [wl.num_cons[0 if wl.shared else p] for p in range(wl.P)]
    for j, mode in enumerate([4] * lx + [2] * lq):
        got = spg.phase1_round_evals(Ap, Aq, Ax, *tabs, mode)
        _, npf, nin = tabs[0].shape()
        want = phase1_round_py([to_int(v) for v in Ap.download()], [to_int(v) for v in Aq.download()],
                               [to_int(v) for v in Ax.download()],
                               [[to_int(v) for v in T.download()] for T in tabs], (anp, ani, npf, nin), mode)
        assert [to_int(v) for v in got] == want, (j, mode)
        r = rand_fq(oracle, rng, 1)[0]
        (Ax if mode == 4 else Aq).bound_top(r)
        for T in tabs:
            T.bound(r, mode)
    with pytest.raises(spg.SpgError):  # every x and q variable bound: no x / q round left
        spg.phase1_round_evals(Ap, Aq, Ax, *tabs, 4)


# ---- one phase-2 round (src/sumcheck.rs:881-941) ----

class PyPqx:
    """a Pqx table's allocation (integers) and current sizes, with the reference's index / index_high
    (custom_dense_mlpoly.rs:118-173)"""

    def __init__(self, vals, anp, anw, ani, shape):
        self.v, self.anp, self.anw, self.ani = vals, anp, anw, ani
        (self.ninst, _, self.nws, _), self.npf, self.nin = shape
        self.off = [sum(anp[k] * anw * ani[k] for k in range(p)) for p in range(len(anp))]

    def at(self, p, q, w, x):
        return self.v[self.off[p] + (q * self.anw + w) * self.ani[p] + x]

    def index(self, p, q, w, x):
        ok = p < len(self.anp) and q < self.anp[p] and w < self.anw and x < self.ani[p]
        return self.at(p, q, w, x) if ok else 0

    def index_high(self, p, q, w, x, mode):
        if mode == 1:
            ph = p + self.ninst // 2
            return self.at(ph, q, w, x) if ph < len(self.anp) else 0
        if mode == 3:
            wh = w + self.nws // 2
            return self.at(p, q, wh, x) if wh < self.anw else 0
        return 0 if self.nin[p] == 1 else self.at(p, q, w, x + self.nin[p] // 2)


def phase2_round_py(A, B, C, mode, single, nws_arg):
    instance_len = len(A) // 2 if mode == 1 else len(A)
    ws_len = C.nws // 2 if mode == 3 else C.nws
    e = [0, 0, 0]
    for p in range(min(instance_len, len(C.nin))):
        pi = 0 if single else p
        ni = C.nin[p] // 2 if (mode == 4 and C.nin[p] > 1) else C.nin[p]
        for w in range(min(ws_len, nws_arg)):
            for y in range(ni):
                a, ah = A[p], (A[p + instance_len] if mode == 1 else A[p])
                bl, bh = B.index(pi, 0, w, y), B.index_high(pi, 0, w, y, mode)
                cl, ch = C.index(p, 0, w, y), C.index_high(p, 0, w, y, mode)
                e[0] += a * bl * cl
                a2, b2, c2 = 2 * ah - a, 2 * bh - bl, 2 * ch - cl
                e[1] += a2 * b2 * c2
                e[2] += (a2 + ah - a) * (b2 + bh - bl) * (c2 + ch - cl)
    return [v % Q for v in e]


@pytest.mark.gpu
@pytest.mark.parametrize("single", [False, True])
@pytest.mark.parametrize("nws", [1, 3, 4])
def test_phase2_rounds_match_python_loop(ctx, oracle, single, nws):
    """every y, w and p round of phase 2 on random ABC / Z tables (ragged widths, a section count that is not a
    power of two, one shared ABC or one per instance): (e0, e2, e3) against the reference loop on Python integers,
    the tables bound between rounds through the seams as sumcheck.rs:961-967 binds them"""
    import spg

    rng = np.random.default_rng(500 + nws + 10 * single)
    ni = [8, 4, 8] if not single else [8, 8, 8]
    P, max_ni = len(ni), 8
    z = rand_fq(oracle, rng, sum(nws * x for x in ni))
    abc_ni = ni[:1] if single else ni
    abc = rand_fq(oracle, rng, sum(nws * x for x in abc_ni))
    Z = spg.Pqx(ctx, z, [1] * P, 1, nws, ni, max_ni)
    B = spg.Pqx(ctx, abc, [1] * len(abc_ni), 1, nws, abc_ni, max_ni)
    A = spg.Buf(ctx, rand_fq(oracle, rng, 4))
    ly, lw, lp = 3, (nws - 1).bit_length(), 2
    for j, mode in enumerate([4] * ly + [3] * lw + [1] * lp):
        got = spg.phase2_round_evals(A, B, Z, mode, single, nws)
        Bp = PyPqx([to_int(v) for v in B.download()], [1] * len(abc_ni), nws, abc_ni, B.shape())
        Zp = PyPqx([to_int(v) for v in Z.download()], [1] * P, nws, ni, Z.shape())
        want = phase2_round_py([to_int(v) for v in A.download()], Bp, Zp, mode, single, nws)
        assert [to_int(v) for v in got] == want, (j, mode)
        r = rand_fq(oracle, rng, 1)[0]
        if mode == 1:
            A.bound_top(r)
        if mode != 1 or not single:
            B.bound(r, mode)
        Z.bound(r, mode)
