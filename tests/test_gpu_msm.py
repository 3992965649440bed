"""MSM / generator parity on the GPU: libspg.so vs the CPU oracle, bit-exact compressed bytes.
Covers MultiCommitGens::new (src/commitments.rs:15-33), vartime_multiscalar_mul (src/group.rs:98-116)
with edge scalars, Commitments::commit with blinds (src/commitments.rs:87-92) and Hyrax rows
(src/dense_mlpoly.rs:184-212)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
Q = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def gens64(ctx):
    import spg

    return spg.Gens(ctx, 1024, b"gens_r1cs_sat")


def rand_fq(oracle, rng, n):
    return oracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * n, dtype=np.uint8).tobytes())


def test_gens_derive_matches_oracle(ctx, oracle, gens64):
    comp = gens64.compressed()
    ref = oracle.gens_stream(b"gens_r1cs_sat", 1025)
    assert np.array_equal(comp, ref)
    f = json.load(open(os.path.join(G, "gens_r1cs_sat_first16.json")))
    assert [c.tobytes().hex() for c in comp[:16]] == f["points"]


def test_gens_upload_roundtrip(ctx, oracle):
    import spg

    ref = oracle.gens_stream(b"upload", 33)
    g = spg.Gens(ctx, 32, compressed=ref)
    assert np.array_equal(g.compressed(), ref)
    rng = np.random.default_rng(2)
    s = rand_fq(oracle, rng, 32)
    assert g.msm(s) == oracle.msm(ref[:32], s)
    bad = ref.copy()
    bad[3, 0] ^= 1  # odd s -> invalid encoding
    with pytest.raises(spg.SpgError):
        spg.Gens(ctx, 32, compressed=bad)


@pytest.mark.parametrize("name", ["msm_64.json", "msm_256.json"])
def test_msm_golden(ctx, name):
    import spg

    f = json.load(open(os.path.join(G, name)))
    g = spg.Gens(ctx, f["n"], f["label"].encode())
    s = np.array(f["scalars_mont"], dtype=np.uint64)
    assert g.msm(s).hex() == f["out"]


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 100, 1000, 1024])
def test_msm_random_sizes(ctx, oracle, gens64, n):
    rng = np.random.default_rng(n)
    s = rand_fq(oracle, rng, n)
    pts = gens64.compressed()
    assert gens64.msm(s) == oracle.msm(pts[:n], s)


def test_msm_edge_scalars(ctx, oracle, gens64):
    pts = gens64.compressed()
    n = 256
    one = oracle.fq_from_u64(1)
    zero = np.zeros(4, np.uint64)
    neg1 = oracle.fq_op("neg", one)[0]
    cases = {
        "zeros": np.tile(zero, (n, 1)),
        "ones": np.tile(one, (n, 1)),
        "neg_ones": np.tile(neg1, (n, 1)),
        "mixed01": np.stack([one if i % 3 else zero for i in range(n)]),
        "same_random": np.tile(rand_fq(oracle, np.random.default_rng(1), 1)[0], (n, 1)),
        "pow2_252": np.tile(oracle.fq_from_raw([0, 0, 0, 1 << 60]), (n, 1)),
    }
    for name, s in cases.items():
        assert gens64.msm(s) == oracle.msm(pts[:n], s), name
    assert gens64.msm(np.tile(zero, (n, 1))) == bytes(32)  # identity


def test_msm_blind_and_offset(ctx, oracle, gens64):
    pts = gens64.compressed()
    rng = np.random.default_rng(4)
    s = rand_fq(oracle, rng, 50)
    bl = rand_fq(oracle, rng, 1)
    exp = oracle.msm(np.concatenate([pts[:50], pts[1024:1025]]), np.concatenate([s, bl]))
    assert gens64.msm(s, blind=bl) == exp
    assert gens64.msm(s, gen_offset=10) == oracle.msm(pts[10:60], s)


# (128, 512) and (64, 1024): >= 64 rows wider than the latency path take the LDS row sort (k_digits_rows)
@pytest.mark.parametrize("L,R", [(1, 1), (4, 2), (8, 32), (64, 128), (16, 1024), (128, 512), (64, 1024)])
def test_commit_rows(ctx, oracle, gens64, L, R):
    rng = np.random.default_rng(L * 1000 + R)
    pts = gens64.compressed()
    Z = rand_fq(oracle, rng, L * R)
    Z[: min(L * R, 5)] = 0
    if L >= 64:
        Z[3 * R: 4 * R] = 0  # an all-zero row: empty histogram
    assert np.array_equal(gens64.commit_rows(Z, L, R), oracle.commit_rows(pts[:R], pts[1024].tobytes(), Z, L, R))
    bl = rand_fq(oracle, rng, L)
    assert np.array_equal(gens64.commit_rows(Z, L, R, bl),
                          oracle.commit_rows(pts[:R], pts[1024].tobytes(), Z, L, R, bl))


def test_large_msm_2e16_property(ctx, oracle):
    """Config-2 size: a 2^16-point MSM (spg_msm) equals the oracle's vartime Pippenger MSM of the same 2^16 pairs."""
    import spg

    n = 1 << 16
    g = spg.Gens(ctx, n, b"spg_bench_msm")
    pts = g.compressed()
    rng = np.random.default_rng(1)
    s = rand_fq(oracle, rng, n)
    got = g.msm(s)
    assert got == oracle.msm(pts[:n], s)


@pytest.mark.parametrize("n,world", [(1000, 3), (4099, 8), (1 << 16, 8), (20000, 1)])
def test_msm_partial_shards(ctx, oracle, n, world):
    """per-rank uncompressed partials (spg_msm_partial, both the latency path and the batch
    pipeline) add on the host (spg_points_sum_compress) to the unsharded MSM, and each partial equals the
    oracle's partial point"""
    import shard
    import spg

    g = spg.Gens(ctx, n, b"spg_bench_msm")
    pts = g.compressed()
    s = rand_fq(oracle, np.random.default_rng(n), n)
    parts = [g.msm_partial(s[lo:hi], gen_offset=lo) for lo, hi in (shard.chunk(n, r, world) for r in range(world))]
    assert spg.points_sum_compress(parts) == g.msm(s) == oracle.msm(pts[:n], s)
    lo, hi = shard.chunk(n, world - 1, world)
    ref = oracle.msm_partial(pts[lo:hi], s[lo:hi])
    # same point, possibly different projective representative: compare encodings
    assert spg.points_sum_compress([parts[-1]]) == spg.points_sum_compress([ref])


# (512, 64): latency-path rows through the comb with 4 window groups, encoded on the device (> 384 points);
# (100, 100): below 2^14 scalars, latency-path buckets, encoded on the host pool
@pytest.mark.parametrize("L,R", [(64, 256), (100, 300), (72, 1000), (512, 64), (100, 100)])
def test_commit_rows_comb(ctx, oracle, gens64, L, R):
    """>= 64 rows of <= 1024 scalars (>= 2^14 in all) take the comb tables (comb.hip): one table entry per nonzero
    signed 12-bit digit, no buckets. Edge scalars (0, 1, -1, 2^252, q - 2^252) put digits of every magnitude class,
    the top window's carry and all-zero windows into the rows; with and without blinds, against the oracle"""
    rng = np.random.default_rng(L * 7 + R)
    pts = gens64.compressed()
    Z = rand_fq(oracle, rng, L * R)
    one = oracle.fq_from_u64(1)
    minus1 = oracle.fq_op("neg", one)[0]
    p252 = oracle.fq_from_raw([0, 0, 0, 1 << 60])
    Z[0:R] = minus1
    Z[R:2 * R] = p252
    Z[2 * R:3 * R] = oracle.fq_op("neg", p252)[0]
    Z[3 * R:4 * R] = 0
    Z[4 * R:5 * R] = one
    Z[5 * R::7] = minus1
    assert np.array_equal(gens64.commit_rows(Z, L, R), oracle.commit_rows(pts[:R], pts[1024].tobytes(), Z, L, R))
    bl = rand_fq(oracle, rng, L)
    bl[0] = minus1
    assert np.array_equal(gens64.commit_rows(Z, L, R, bl),
                          oracle.commit_rows(pts[:R], pts[1024].tobytes(), Z, L, R, bl))


def test_commit_rows_wide(ctx, oracle):
    """Hyrax rows of 2^14 scalars (window c = 14, 2^13 bucket counters) in batches of >= 64 rows take the LDS row
    sort too (the SPARK derefs / comb_ops commitments at 2^24 nonzeros have such rows)"""
    import spg

    L, R = 64, 1 << 14
    g = spg.Gens(ctx, R, b"spg_wide_rows")
    pts = g.compressed()
    Z = rand_fq(oracle, np.random.default_rng(14), L * R)
    Z[5 * R: 6 * R] = 0
    assert np.array_equal(g.commit_rows(Z, L, R), oracle.commit_rows(pts[:R], pts[R].tobytes(), Z, L, R))


@pytest.fixture(scope="module")
def gens_big(ctx):
    import spg

    return spg.Gens(ctx, 20000, b"spg_big_msm")


def test_msm_big_edge_and_skew(ctx, oracle, gens_big):
    """one MSM larger than the latency path (the default: comb.hip msm_single_comb, c = 9 windows over the 20001-slot
    comb table, two window groups per scalar): edge scalars, an all-zero stretch, one scalar repeated (a skewed
    distribution), a blind, and a generator offset, against the oracle"""
    edge_and_skew_checks(oracle, gens_big)


@pytest.mark.parametrize("env", [{"SPG_BIG_COMB": "0"}, {"SPG_BIG_COMB_G": "4"}, {"SPG_BIG_COMB_G": "1"}])
def test_msm_single_comb_edge_and_skew(env):
    """the same checks through msm_big.hip's bucket pipeline (SPG_BIG_COMB=0: a bucket holding most entries splits
    into many chunks) and through the comb with 4 or 1 window groups per scalar, in a fresh process that reads the
    switch"""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys; sys.path[:0] = [%r, %r, %r]\n"
        "import spg, pyoracle\n"
        "from test_gpu_msm import edge_and_skew_checks\n"
        "ctx = spg.Context(0)\n"
        "edge_and_skew_checks(pyoracle, spg.Gens(ctx, 20000, b'spg_big_msm'))\n"
        "print('ok')\n"
    ) % (os.path.join(root, "spartan-parallel_amd"), os.path.join(root, "oracle"), os.path.join(root, "tests"))
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split()[-1] == "ok"


def edge_and_skew_checks(oracle, gens_big):
    n = 20000
    pts = gens_big.compressed()
    rng = np.random.default_rng(20000)
    s = rand_fq(oracle, rng, n)
    one = oracle.fq_from_u64(1)
    edge = [np.zeros(4, np.uint64), one[0], oracle.fq_from_u64(2)[0], oracle.fq_op("neg", one)[0],
            oracle.fq_from_raw([0, 0, 0, 1 << 60]), oracle.fq_from_raw([2**64 - 1, 2**64 - 1, 2**64 - 1, (1 << 60) - 1])]
    for i, e in enumerate(edge):
        s[i] = e
    s[100:400] = 0
    assert gens_big.msm(s) == oracle.msm(pts[:n], s), "edge"
    skew = np.tile(s[9], (n, 1))
    skew[::7] = s[::7]
    assert gens_big.msm(skew) == oracle.msm(pts[:n], skew), "skewed"
    bl = rand_fq(oracle, rng, 1)
    exp = oracle.msm(np.concatenate([pts[:n], pts[n:n + 1]]), np.concatenate([s, bl]))
    assert gens_big.msm(s, blind=bl) == exp, "blind"
    m = n - 1500
    assert gens_big.msm(s[:m], gen_offset=1500) == oracle.msm(pts[1500:n], s[:m]), "offset"
    zeros = np.zeros((n, 4), np.uint64)
    assert gens_big.msm(zeros) == bytes(32), "identity"


@pytest.mark.parametrize("c", ["8", "10", "13", "14"])
def test_msm_big_windows(oracle, c):
    """every window width of the large-MSM bucket path (SPG_BIG_C with SPG_BIG_COMB=0, a fresh process reads them)
    gives the oracle's 2^16 MSM"""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = 1 << 16
    code = (
        "import sys, numpy as np; sys.path[:0] = [%r, %r]\n"
        "import spg, pyoracle\n"
        "ctx = spg.Context(0)\n"
        "g = spg.Gens(ctx, %d, b'spg_bench_msm')\n"
        "rng = np.random.default_rng(%s)\n"
        "s = pyoracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * %d, dtype=np.uint8).tobytes())\n"
        "print(g.msm(s).hex())\n"
    ) % (os.path.join(root, "spartan-parallel_amd"), os.path.join(root, "oracle"), n, c, n)
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SPG_BIG_C=c, SPG_BIG_COMB="0"),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    rng = np.random.default_rng(int(c))
    s = rand_fq(oracle, rng, n)
    pts = oracle.gens_stream(b"spg_bench_msm", n + 1)
    assert out.stdout.split()[-1] == oracle.msm(pts[:n], s).hex()


def test_msm_resident_scalars(ctx, oracle):
    """spg_msm_buf / spg_msm_partial_buf over scalars uploaded once (the config-2 bench's entry points) give the
    oracle's MSM: whole vector (large path), shards that add up, a small range (latency path), empty and bad ranges"""
    import spg

    n = 1 << 16
    g = spg.Gens(ctx, n, b"spg_bench_msm")
    rng = np.random.default_rng(11)
    s = rand_fq(oracle, rng, n)
    buf = spg.Buf(ctx, s)
    pts = oracle.gens_stream(b"spg_bench_msm", n + 1)
    ref = oracle.msm(pts[:n], s)
    assert g.msm_buf(buf) == ref
    cuts = [0, 1000, 1001, 40000, n]
    parts = [g.msm_partial_buf(buf, offset=lo, n=hi - lo, gen_offset=lo) for lo, hi in zip(cuts, cuts[1:])]
    assert spg.points_sum_compress(parts) == ref
    assert g.msm_buf(buf, offset=7, n=300, gen_offset=7) == oracle.msm(pts[7:307], s[7:307])
    assert g.msm_buf(buf, offset=5, n=0) == bytes(32)
    with pytest.raises(spg.SpgError):
        g.msm_buf(buf, offset=n - 10, n=11)


@pytest.mark.parametrize("form", ["0", "1"])
def test_msm_big_accumulation_forms(oracle, form):
    """both accumulation forms of the large-MSM path (SPG_BIG_ITEMS: 0 quad chunks, 1 lane-then-quad buckets)
    give the oracle's 2^16 MSM, skewed scalars included"""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = 1 << 16
    code = (
        "import sys, numpy as np; sys.path[:0] = [%r, %r]\n"
        "import spg, pyoracle\n"
        "ctx = spg.Context(0)\n"
        "g = spg.Gens(ctx, %d, b'spg_bench_msm')\n"
        "rng = np.random.default_rng(5)\n"
        "s = pyoracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * %d, dtype=np.uint8).tobytes())\n"
        "s[: %d // 2] = s[0]\n"  # half the scalars equal: every window's digit repeats (one bucket per window)
        "print(g.msm(s).hex())\n"
    ) % (os.path.join(root, "spartan-parallel_amd"), os.path.join(root, "oracle"), n, n, n)
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SPG_BIG_ITEMS=form, SPG_BIG_COMB="0"),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    rng = np.random.default_rng(5)
    s = rand_fq(oracle, rng, n)
    s[: n // 2] = s[0]
    pts = oracle.gens_stream(b"spg_bench_msm", n + 1)
    assert out.stdout.split()[-1] == oracle.msm(pts[:n], s).hex()
