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


def _oracle_backed(oracle, label, pre=()):
    """an spg transcript whose state is the caller's (oracle) merlin transcript, after the caller's own appends"""
    import spg

    t = oracle.OracleTranscript(label)
    for lbl, msg in pre:
        t.append_message(lbl, msg)
    return t, spg.Transcript.from_callbacks(t.append_message, t.challenge_bytes)


def test_callback_transcript_continues_caller_state(oracle):
    """spg_transcript_new_callbacks (SNARK::prove's `&mut Transcript`, src/lib.rs:1022): operations through the
    handle land in the caller's transcript, interleaved with the caller's own, exactly as one merlin transcript"""
    import spg

    pre = [(b"caller", b"appended before the call")]
    back, cb = _oracle_backed(oracle, b"drop-in", pre)
    ref = spg.Transcript(b"drop-in")
    for lbl, msg in pre:
        ref.append_message(lbl, msg)
    for t in (cb, ref):
        t.append_message(b"protocol-name", b"Spartan SNARK proof")
        t.append_scalar(b"num_ios", np.array([1, 2, 3, 4], dtype=np.uint64))
    assert np.array_equal(cb.challenge_scalar(b"tau"), ref.challenge_scalar(b"tau"))
    assert cb.challenge_bytes(b"c", 17) == ref.challenge_bytes(b"c", 17)
    back.append_message(b"caller-after", b"x")  # the caller keeps using its transcript directly
    ref.append_message(b"caller-after", b"x")
    assert back.challenge_bytes(b"final", 32) == ref.challenge_bytes(b"final", 32)


def test_callback_transcript_failure_is_latched():
    """a failing callback: that operation and every later one report SPG_E_CALLBACK (challenges read as zero)"""
    import pytest
    import spg

    calls = []

    def app(label, msg):
        calls.append(label)
        if label == b"bad":
            raise RuntimeError("caller transcript refused")

    t = spg.Transcript.from_callbacks(app, lambda label, n: b"\x01" * n)
    t.append_message(b"ok", b"1")
    with pytest.raises(spg.SpgError, match="SPG_E_CALLBACK"):
        t.append_message(b"bad", b"2")
    with pytest.raises(spg.SpgError, match="SPG_E_CALLBACK"):
        t.challenge_bytes(b"after", 4)
    assert calls == [b"ok", b"bad"]


def test_native_merlin_callbacks_match_library_transcript():
    """Transcript.from_native_merlin: the drop-in mode bench.py times (C callbacks over a caller-owned merlin in
    libspg_hostcheck, no Python on the transcript path) ends in the same state as the library's own transcript"""
    import spg

    cb = spg.Transcript.from_native_merlin(b"drop-in")
    ref = spg.Transcript(b"drop-in")
    for t in (cb, ref):
        t.append_message(b"protocol-name", b"Spartan SNARK proof")
        t.append_scalar(b"num_ios", np.array([5, 6, 7, 8], dtype=np.uint64))
    assert np.array_equal(cb.challenge_scalar(b"tau"), ref.challenge_scalar(b"tau"))
    assert cb.challenge_bytes(b"c", 200) == ref.challenge_bytes(b"c", 200)
    # the caller's own transcript object holds the state: reading it directly continues the same stream
    assert cb.caller_challenge(b"final", 32) == ref.challenge_bytes(b"final", 32)
