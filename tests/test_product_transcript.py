"""Host-side Fiat-Shamir objects of libspg (no device needed): merlin transcript and RandomTape
against the oracle and merlin's published conformance vector (src/transcript.rs, src/random.rs)."""
import numpy as np


def test_merlin_conformance():
    import spg

    t = spg.Transcript(b"test protocol")
    t.append_message(b"some label", b"some data")
    assert t.challenge_bytes(b"challenge", 32).hex() == \
        "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"


def test_transcript_matches_oracle(oracle):
    import spg

    for n in (1, 32, 64, 200):
        t = spg.Transcript(b"proto")
        t.append_message(b"lbl", b"x" * n)
        assert t.challenge_bytes(b"ch", n) == oracle.merlin_simple(b"proto", b"lbl", b"x" * n, b"ch", n)


def test_challenge_scalar_is_wide_reduction(oracle):
    import spg

    t1 = spg.Transcript(b"proto")
    t2 = spg.Transcript(b"proto")
    s = t1.challenge_scalar(b"c")
    wide = t2.challenge_bytes(b"c", 64)
    ref = oracle.fq_from_bytes_wide(wide)
    assert np.array_equal(np.asarray(ref).reshape(-1)[:4], s)


def test_random_tape_deterministic():
    import spg
    import workload

    a = spg.RandomTape(b"proof", workload.tape_seed())
    b = spg.RandomTape(b"proof", workload.tape_seed())
    c = spg.RandomTape(b"proof", workload.tape_seed(b"other"))
    x, y, z = a.random_scalar(b"t1"), b.random_scalar(b"t1"), c.random_scalar(b"t1")
    assert np.array_equal(x, y) and not np.array_equal(x, z)
