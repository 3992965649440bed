"""ORACLE loader — test infrastructure only.

ctypes bindings over oracle/build/liboracle.so, the CPU restatement of the reference's algorithms
(see the headers in oracle/*.hpp for the reference file:line each function follows). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the product
(spartan-parallel_amd/) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def u64s(x):
    return np.ascontiguousarray(x, dtype=np.uint64)


# ---------------- Fq ----------------
_OPS = {"add": 0, "sub": 1, "mul": 2, "neg": 3, "square": 4, "invert": 5}


def fq_op(op, a, b=None):
    a = u64s(a).reshape(-1, 4)
    n = a.shape[0]
    out = np.zeros_like(a)
    bb = None if b is None else u64s(b).reshape(-1, 4)
    lib().orc_fq_binop(ctypes.c_int(_OPS[op]), _p(a), None if bb is None else _p(bb), _p(out), ctypes.c_size_t(n))
    return out


def fq_to_bytes(a):
    a = u64s(a).reshape(-1, 4)
    out = np.zeros((a.shape[0], 32), dtype=np.uint8)
    lib().orc_fq_to_bytes(_p(a), _p(out), ctypes.c_size_t(a.shape[0]))
    return out


def fq_from_bytes(b32):
    b = np.frombuffer(bytes(b32), dtype=np.uint8).copy()
    out = np.zeros(4, dtype=np.uint64)
    ok = lib().orc_fq_from_bytes(_p(b), _p(out))
    return out, bool(ok)


def fq_from_bytes_wide(b):
    b = np.frombuffer(bytes(b), dtype=np.uint8).copy().reshape(-1, 64)
    out = np.zeros((b.shape[0], 4), dtype=np.uint64)
    lib().orc_fq_from_bytes_wide(_p(b), _p(out), ctypes.c_size_t(b.shape[0]))
    return out


def fq_from_u512(limbs):
    l8 = u64s(limbs)
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_fq_from_u512(_p(l8), _p(out))
    return out


def fq_from_raw(limbs):
    l4 = u64s(limbs)
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_fq_from_raw(_p(l4), _p(out))
    return out


def fq_from_u64(x):
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_fq_from_u64(ctypes.c_uint64(x), _p(out))
    return out


def fq_batch_invert(a):
    a = u64s(a).reshape(-1, 4).copy()
    allinv = np.zeros(4, dtype=np.uint64)
    lib().orc_fq_batch_invert(_p(a), ctypes.c_size_t(a.shape[0]), _p(allinv))
    return a, allinv


# ---------------- UniPoly / MLE evaluation ----------------
def unipoly(evals, r):
    """UniPoly::from_evals (src/unipoly.rs:23-54) -> (coeffs, evaluate(r), decompress(compress(), e0 + e1).coeffs)"""
    e = u64s(evals).reshape(-1, 4)
    n = e.shape[0]
    co, rt = np.zeros((n, 4), np.uint64), np.zeros((n, 4), np.uint64)
    at = np.zeros(4, np.uint64)
    lib().orc_unipoly(_p(e), ctypes.c_size_t(n), _p(u64s(r)), _p(co), _p(at), _p(rt))
    return co, at, rt


def dense_eval(Z, r):
    """DensePolynomial::new(Z).evaluate(r) and evaluate_with_LR (src/dense_mlpoly.rs:361-367, 1212-1231)"""
    z, rr = u64s(Z).reshape(-1, 4), u64s(r).reshape(-1, 4)
    out = np.zeros((2, 4), np.uint64)
    lib().orc_dense_eval(_p(z), ctypes.c_size_t(z.shape[0]), _p(rr), ctypes.c_size_t(rr.shape[0]), _p(out))
    return out[0], out[1]


def pqx_bind(z, num_proofs, max_num_proofs, nws, num_inputs, max_num_inputs, modes, rs):
    """DensePolynomialPqx::new then bound_poly(r, mode) per step (src/custom_dense_mlpoly.rs:45-64, 180-289) ->
    (Z afterwards in z's layout, (num_instances, max_num_proofs, num_witness_secs, max_num_inputs), num_proofs,
    num_inputs); None where the reference would panic (bound_poly_p before q and x are bound)"""
    P = len(num_proofs)
    zz = u64s(z).reshape(-1, 4)
    out = np.zeros_like(zz)
    sizes = np.zeros(4 + 2 * P, dtype=np.uint64)
    np_ = np.asarray(num_proofs, dtype=np.uint64)
    ni_ = np.asarray(num_inputs, dtype=np.uint64)
    md = np.asarray(list(modes) or [0], dtype=np.int32)
    rr = u64s(rs).reshape(-1, 4) if len(modes) else np.zeros((1, 4), np.uint64)
    rc = lib().orc_pqx_bind(_p(zz), ctypes.c_size_t(P), _p(np_), ctypes.c_size_t(max_num_proofs), ctypes.c_size_t(nws),
                            _p(ni_), ctypes.c_size_t(max_num_inputs), _p(md), _p(rr), ctypes.c_size_t(len(modes)),
                            _p(out), _p(sizes))
    if rc != 0:
        return None
    s = [int(x) for x in sizes]
    return out, tuple(s[:4]), s[4:4 + P], s[4 + P:]


# ---------------- hashing ----------------
def keccak_f1600(state200):
    s = np.frombuffer(bytes(state200), dtype=np.uint8).copy()
    lib().orc_keccak_f1600(_p(s))
    return s.tobytes()


def shake256(data, n):
    d = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8).copy()
    out = np.zeros(n, dtype=np.uint8)
    lib().orc_shake256(_p(d), ctypes.c_size_t(len(data)), _p(out), ctypes.c_size_t(n))
    return out.tobytes()


def merlin_simple(label, l1, m1, l2, n):
    out = np.zeros(n, dtype=np.uint8)
    m = np.frombuffer(bytes(m1) or b"\0", dtype=np.uint8).copy()
    lib().orc_merlin_simple(ctypes.c_char_p(label), ctypes.c_char_p(l1), _p(m), ctypes.c_size_t(len(m1)),
                            ctypes.c_char_p(l2), _p(out), ctypes.c_size_t(n))
    return out.tobytes()


class OracleTranscript:
    """merlin Transcript of the oracle as a handle: the caller-side state behind spg_transcript_new_callbacks in the
    drop-in tests (append_message / challenge_bytes, src/transcript.rs:5-63)"""

    def __init__(self, label):
        f = lib().orc_transcript_new
        f.restype = ctypes.c_void_p
        self.h = ctypes.c_void_p(f(ctypes.c_char_p(bytes(label))))

    def append_message(self, label, msg):
        m = np.frombuffer(bytes(msg) or b"\0", dtype=np.uint8).copy()
        lib().orc_transcript_append(self.h, ctypes.c_char_p(bytes(label)), _p(m), ctypes.c_size_t(len(msg)))

    def append_raw(self, label_ptr, msg_ptr, n):  # from a ctypes callback (pointers as given by libspg)
        lib().orc_transcript_append(self.h, ctypes.c_char_p(label_ptr), ctypes.c_void_p(msg_ptr), ctypes.c_size_t(n))

    def challenge_raw(self, label_ptr, out_ptr, n):
        lib().orc_transcript_challenge(self.h, ctypes.c_char_p(label_ptr), ctypes.c_void_p(out_ptr), ctypes.c_size_t(n))

    def challenge_bytes(self, label, n):
        out = np.zeros(max(n, 1), dtype=np.uint8)
        lib().orc_transcript_challenge(self.h, ctypes.c_char_p(bytes(label)), _p(out), ctypes.c_size_t(n))
        return out[:n].tobytes()

    def __del__(self):
        try:
            lib().orc_transcript_free(self.h)
        except Exception:
            pass


# ---------------- ristretto ----------------
def ristretto_consts():
    out = np.zeros(6 * 32, dtype=np.uint8)
    lib().orc_ristretto_consts(_p(out))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(6)]


def ge_roundtrip(b32):
    i = np.frombuffer(bytes(b32), dtype=np.uint8).copy()
    out = np.zeros(32, dtype=np.uint8)
    ok = lib().orc_ge_decompress_compress(_p(i), _p(out))
    return out.tobytes() if ok else None


def ge_from_uniform_bytes(b64):
    b = np.frombuffer(bytes(b64), dtype=np.uint8).copy()
    n = len(b) // 64
    out = np.zeros(32 * n, dtype=np.uint8)
    lib().orc_ge_from_uniform_bytes(_p(b), _p(out), ctypes.c_size_t(n))
    return [out[32 * k:32 * k + 32].tobytes() for k in range(n)]


def ge_add(a, b):
    x = np.frombuffer(bytes(a), dtype=np.uint8).copy()
    y = np.frombuffer(bytes(b), dtype=np.uint8).copy()
    out = np.zeros(32, dtype=np.uint8)
    ok = lib().orc_ge_add(_p(x), _p(y), _p(out))
    return out.tobytes() if ok else None


def ge_scalarmul(P, k32):
    x = np.frombuffer(bytes(P), dtype=np.uint8).copy()
    k = np.frombuffer(bytes(k32), dtype=np.uint8).copy()
    out = np.zeros(32, dtype=np.uint8)
    ok = lib().orc_ge_scalarmul(_p(x), _p(k), _p(out))
    return out.tobytes() if ok else None


def gens_stream(label, count):
    out = np.zeros(32 * count, dtype=np.uint8)
    lb = np.frombuffer(bytes(label), dtype=np.uint8).copy()
    lib().orc_gens_stream(_p(lb), ctypes.c_size_t(len(label)), ctypes.c_size_t(count), _p(out))
    return out.reshape(count, 32)


def msm(bases, scalars):
    bases = np.ascontiguousarray(bases, dtype=np.uint8).reshape(-1, 32)
    s = u64s(scalars).reshape(-1, 4)
    assert bases.shape[0] == s.shape[0]
    out = np.zeros(32, dtype=np.uint8)
    ok = lib().orc_msm(_p(bases), _p(s), ctypes.c_size_t(s.shape[0]), _p(out))
    assert ok
    return out.tobytes()


def msm_partial(bases, scalars):
    """uncompressed MSM result (X, Y, Z, T as 4 x 32 LE bytes) of one shard"""
    bases = np.ascontiguousarray(bases, dtype=np.uint8).reshape(-1, 32)
    s = u64s(scalars).reshape(-1, 4)
    assert bases.shape[0] == s.shape[0]
    out = np.zeros(128, dtype=np.uint8)
    assert lib().orc_msm_partial(_p(bases), _p(s), ctypes.c_size_t(s.shape[0]), _p(out))
    return out.tobytes()


def commit_rows(bases, h, Z, L, R, blinds=None):
    bases = np.ascontiguousarray(bases, dtype=np.uint8).reshape(-1, 32)
    hh = np.frombuffer(bytes(h), dtype=np.uint8).copy()
    Z = u64s(Z).reshape(-1, 4)
    assert Z.shape[0] == L * R
    out = np.zeros((L, 32), dtype=np.uint8)
    bl = None if blinds is None else u64s(blinds).reshape(-1, 4)
    ok = lib().orc_commit_rows(_p(bases), ctypes.c_size_t(bases.shape[0]), _p(hh), _p(Z), ctypes.c_size_t(L),
                               ctypes.c_size_t(R), None if bl is None else _p(bl), _p(out))
    assert ok
    return out


# ---------------------------------------------------------------- R1CSProof
def r1cs_prove(wl, tape_seed, gens_label=b"gens_r1cs_sat", gens_num_vars=1 << 24, label=b"r1cs_test",
               transcript=None):
    """bincode(R1CSProof) and the challenge vectors [rp, rq_rev, rx, rw||ry] for an R1CSWorkload (on a fresh
    Transcript(label), or on the caller's OracleTranscript `transcript`, which keeps its state)."""
    import workload

    v = workload.CViews(wl)
    cap = 1 << 22
    buf = np.zeros(cap, dtype=np.uint8)
    ln = ctypes.c_size_t(0)
    ch = np.zeros((4096, 4), dtype=np.uint64)
    chl = (ctypes.c_size_t * 4)()
    seed = u64s(tape_seed)
    common = (ctypes.byref(v.inst), ctypes.c_size_t(wl.P), ctypes.c_size_t(wl.max_num_proofs), v.num_proofs,
              ctypes.c_size_t(wl.max_num_inputs), v.num_inputs, v.secs, ctypes.c_size_t(wl.nws),
              ctypes.c_char_p(gens_label), ctypes.c_size_t(gens_num_vars))
    tail = (_p(seed), _p(buf), ctypes.c_size_t(cap), ctypes.byref(ln), _p(ch), chl)
    if transcript is None:
        rc = lib().orc_r1cs_prove(*common, ctypes.c_char_p(label), *tail)
    else:
        rc = lib().orc_r1cs_prove_tr(*common, transcript.h, *tail)
    assert rc == 0, rc
    lens = list(chl)
    out, o = [], 0
    for L in lens:
        out.append(ch[o:o + L].copy())
        o += L
    return buf[: ln.value].tobytes(), out


def r1cs_verify(wl, proof, tape_seed, gens_label=b"gens_r1cs_sat", gens_num_vars=1 << 24, label=b"r1cs_test"):
    import workload

    v = workload.CViews(wl)
    pb = np.frombuffer(proof, dtype=np.uint8).copy()
    seed = u64s(tape_seed)
    return lib().orc_r1cs_verify(ctypes.byref(v.inst), ctypes.c_size_t(wl.P), ctypes.c_size_t(wl.max_num_proofs),
                                 v.num_proofs, ctypes.c_size_t(wl.max_num_inputs), v.secs, ctypes.c_size_t(wl.nws),
                                 ctypes.c_char_p(gens_label), ctypes.c_size_t(gens_num_vars), ctypes.c_char_p(label),
                                 _p(pb), ctypes.c_size_t(len(proof)), _p(seed))


def r1cs_multi_evaluate(wl, rx, ry):
    """R1CSInstance::multi_evaluate (src/r1csinstance.rs:583-596) -> (3 * num_instances, 4) limbs"""
    import workload

    v = workload.CViews(wl)
    rx = u64s(rx).reshape(-1, 4)
    ry = u64s(ry).reshape(-1, 4)
    out = np.zeros((3 * len(wl.entries), 4), dtype=np.uint64)
    rc = lib().orc_r1cs_multi_evaluate(ctypes.byref(v.inst), _p(rx), ctypes.c_size_t(rx.shape[0]), _p(ry),
                                       ctypes.c_size_t(ry.shape[0]), _p(out))
    assert rc == 0
    return out


def r1cs_multiply_vec_block(wl, z, num_inputs):
    """R1CSInstance::multiply_vec_block (src/r1csinstance.rs:363-436) -> (Az, Bz, Cz) flattened in Pqx order"""
    import workload

    v = workload.CViews(wl)
    zz = u64s(z).reshape(-1, 4)
    npf = np.asarray(wl.num_proofs, dtype=np.uint64)
    nin = np.asarray(num_inputs, dtype=np.uint64)
    nc = [wl.num_cons[0 if wl.shared else p] for p in range(wl.P)]
    n = sum(a * b for a, b in zip(wl.num_proofs, nc))
    outs = [np.zeros((n, 4), np.uint64) for _ in range(3)]
    rc = lib().orc_multiply_vec_block(ctypes.byref(v.inst), ctypes.c_size_t(wl.P), _p(npf), ctypes.c_size_t(wl.max_num_proofs),
                                      _p(nin), ctypes.c_size_t(wl.max_num_inputs), ctypes.c_size_t(wl.nws), _p(zz),
                                      *[_p(o) for o in outs])
    assert rc == 0
    return outs


def spark_prove(wl, rx, ry, tape_seed, gens_label=b"gens_r1cs_eval", gens_nnz=None, gens_batch=3,
                label=b"spark_test", transcript=None):
    """SparseMatPolyEvalProof over [A_0, B_0, C_0, ...] of the workload's instance at (rx, ry):
    (bincode(commitment), bincode(proof), verified); with an OracleTranscript `transcript` the proof runs on it
    (no verification)"""
    import workload

    v = workload.CViews(wl)
    rx = u64s(rx).reshape(-1, 4)
    ry = u64s(ry).reshape(-1, 4)
    if gens_nnz is None:  # R1CSCommitmentGens::new: num_instances * num_nz_entries (src/r1csinstance.rs:39-56)
        gens_nnz = len(wl.entries) * max(max(int(m.shape[0]) for m in mats) for mats in wl.entries)
    cb = np.zeros(1 << 20, dtype=np.uint8)
    pb = np.zeros(1 << 22, dtype=np.uint8)
    cl, pl = ctypes.c_size_t(0), ctypes.c_size_t(0)
    seed = u64s(tape_seed)
    rc = lib().orc_spark_prove_tr(ctypes.byref(v.inst), ctypes.c_char_p(gens_label), ctypes.c_size_t(gens_nnz),
                               ctypes.c_size_t(gens_batch), _p(rx), ctypes.c_size_t(rx.shape[0]), _p(ry),
                               ctypes.c_size_t(ry.shape[0]), ctypes.c_char_p(label),
                               None if transcript is None else transcript.h, _p(seed), _p(cb),
                               ctypes.c_size_t(len(cb)), ctypes.byref(cl), _p(pb), ctypes.c_size_t(len(pb)),
                               ctypes.byref(pl))
    assert rc >= 0, rc
    return cb[: cl.value].tobytes(), pb[: pl.value].tobytes(), rc == 1


def concurrent_proves(fn, k):
    """fn() on k threads at once in the oracle's baseline mode (the ctypes calls release the GIL): every copy does its
    setup (commitments, generator derivation, instance encoding), all meet at a barrier, then all prove at once with
    the verification skipped. Returns the wall seconds from the first prove's start to the last one's end."""
    import threading

    bar = threading.Barrier(k)
    cb = ctypes.CFUNCTYPE(None)(lambda: bar.wait())
    f = lib().orc_baseline_mode
    f(cb, ctypes.c_int(1))
    wins, errs = [], []

    def body():
        try:
            fn()
            t0, t1 = ctypes.c_double(0), ctypes.c_double(0)
            lib().orc_last_prove_window(ctypes.byref(t0), ctypes.byref(t1))
            wins.append((t0.value, t1.value))
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            bar.abort()

    try:
        ts = [threading.Thread(target=body) for _ in range(k)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        f(None, ctypes.c_int(0))
    if errs:
        raise errs[0]
    return (max(w[1] for w in wins) - min(w[0] for w in wins)) * 1e-6


def last_prove_seconds():
    """the calling thread's last prove window (orc_r1cs_prove / orc_snark_prove / orc_spark_prove): the prove alone,
    without setup or verification"""
    t0, t1 = ctypes.c_double(0), ctypes.c_double(0)
    lib().orc_last_prove_window(ctypes.byref(t0), ctypes.byref(t1))
    return (t1.value - t0.value) * 1e-6


def spark_concurrent_prove(wl, rx, ry, tape_seed, k, gens_nnz=None):
    """k concurrent oracle SPARK proves (multi_evaluate + SparseMatPolyEvalProof::prove) of the same workload"""
    return concurrent_proves(lambda: spark_prove(wl, rx, ry, tape_seed, gens_nnz=gens_nnz), k)


def snark_concurrent_prove(wl, tape_seed, k, **kw):
    """k concurrent oracle SNARK::prove calls of the same workload, timed prove-only (SNARK::encode, the R1CSGens
    derivation and the verification outside the window)"""
    return concurrent_proves(lambda: snark_prove(wl, tape_seed, **kw), k)


def r1cs_concurrent_prove(wl, tape_seed, k, **kw):
    """k concurrent oracle R1CSProof::prove calls of the same workload, timed prove-only (R1CSGens derivation outside)"""
    return concurrent_proves(lambda: r1cs_prove(wl, tape_seed, **kw), k)


def spark_last_prove_us():
    """wall time (us) of the last spark_prove's multi_evaluate + SparseMatPolyEvalProof::prove on the host"""
    f = lib().orc_spark_last_prove_us
    f.restype = ctypes.c_double
    return f()


def snark_prove(wl, tape_seed, gens_label=b"gens_r1cs_sat", gens_num_vars=1 << 24, label=b"snark_test", cap=1 << 24):
    """SNARK::prove on a workload.SnarkWorkload -> (bincode(SNARK), verifier status: 0 = accepted)"""
    import workload

    v = workload.SnarkViews(wl)
    out = np.zeros(cap, dtype=np.uint8)
    ln = ctypes.c_size_t(0)
    seed = u64s(tape_seed)
    rc = lib().orc_snark_prove(ctypes.byref(v.inputs), ctypes.byref(v.block), ctypes.byref(v.pairwise),
                               ctypes.byref(v.perm_root), ctypes.c_char_p(gens_label), ctypes.c_size_t(gens_num_vars),
                               ctypes.c_char_p(label), _p(seed), _p(out), ctypes.c_size_t(cap), ctypes.byref(ln))
    assert rc >= 0, rc
    return out[: ln.value].tobytes(), rc


def snark_prove_on(wl, tape_seed, transcript, gens_label=b"gens_r1cs_sat", gens_num_vars=1 << 24, cap=1 << 24):
    """SNARK::prove on the caller's OracleTranscript (which keeps its state, as `&mut Transcript`) -> bincode(SNARK)"""
    import workload

    v = workload.SnarkViews(wl)
    out = np.zeros(cap, dtype=np.uint8)
    ln = ctypes.c_size_t(0)
    seed = u64s(tape_seed)
    rc = lib().orc_snark_prove_tr(ctypes.byref(v.inputs), ctypes.byref(v.block), ctypes.byref(v.pairwise),
                                  ctypes.byref(v.perm_root), ctypes.c_char_p(gens_label), ctypes.c_size_t(gens_num_vars),
                                  transcript.h, _p(seed), _p(out), ctypes.c_size_t(cap), ctypes.byref(ln))
    assert rc == 0, rc
    return out[: ln.value].tobytes()


def snark_prove_verify_on(wl, tape_seed, prover_transcript, verifier_transcript, gens_label=b"gens_r1cs_sat",
                          gens_num_vars=1 << 24, cap=1 << 24):
    """SNARK::prove on the caller's prover OracleTranscript, then the oracle's SNARK::verify on the caller's verifier
    OracleTranscript (both keep their state) -> (bincode(SNARK), verdict: 0 = accepted, >0 = failing stage)"""
    import workload

    v = workload.SnarkViews(wl)
    out = np.zeros(cap, dtype=np.uint8)
    ln = ctypes.c_size_t(0)
    seed = u64s(tape_seed)
    rc = lib().orc_snark_prove_verify_tr(ctypes.byref(v.inputs), ctypes.byref(v.block), ctypes.byref(v.pairwise),
                                         ctypes.byref(v.perm_root), ctypes.c_char_p(gens_label),
                                         ctypes.c_size_t(gens_num_vars), prover_transcript.h, verifier_transcript.h,
                                         _p(seed), _p(out), ctypes.c_size_t(cap), ctypes.byref(ln))
    assert rc >= 0, rc
    return out[: ln.value].tobytes(), rc


def snark_last_phases():
    """[(phase, microseconds)] of the last snark_prove, under the reference's Timer labels (src/lib.rs:1088-2692)"""
    f = lib().orc_snark_last_phases
    f.restype = ctypes.c_int
    names = ctypes.create_string_buffer(32 * 32)
    us = (ctypes.c_double * 32)()
    k = f(names, us, 32)
    return [(names.raw[32 * i:32 * i + 32].split(b"\0")[0].decode(), us[i]) for i in range(k)]


def snark_last_prove_us():
    f = lib().orc_snark_last_prove_us
    f.restype = ctypes.c_double
    return f()


def snark_last_verify_us():
    f = lib().orc_snark_last_verify_us
    f.restype = ctypes.c_double
    return f()
