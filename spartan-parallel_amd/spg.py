"""ctypes binding of libspg.so — the MI355X-native Spartan prover hot path (C-ABI in include/spg.h).

Mirrors the reference crate's seams with the same argument meaning:
  * Gens(n, label)            ~ MultiCommitGens::new(n, label)          (src/commitments.rs:15-33)
  * Gens.msm(scalars, blind)  ~ GroupElement::vartime_multiscalar_mul   (src/group.rs:98-116)
                                + blind * h                              (src/commitments.rs:87-92)
  * Gens.commit_rows(Z, L, R) ~ DensePolynomial::commit_inner           (src/dense_mlpoly.rs:184-212)
Scalars are numpy uint64 arrays of shape (..., 4): the reference's Montgomery limbs.
There is no CPU fallback: constructing a Context without a gfx950 device raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPG_LIB") or os.path.join(_HERE, "lib", "libspg.so")

SPG_ERRORS = {-1: "SPG_E_ARG", -2: "SPG_E_NOMEM", -3: "SPG_E_HIP", -4: "SPG_E_POINT", -5: "SPG_E_NODEVICE",
              -6: "SPG_E_VERIFY", -7: "SPG_E_CALLBACK"}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libspg.so not built at {LIB_PATH}; run __graft_entry__.build()")
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.spg_last_error.restype = ctypes.c_char_p
        _lib.spg_last_kernel_us.restype = ctypes.c_double
        _lib.spg_gens_n.restype = ctypes.c_size_t
    return _lib


def comb_stats():
    """spg_comb_stats: (HBM bytes of this process's comb tables now allocated, comb tables built so far, their summed
    build seconds, HBM bytes of the live generator sets' 2^k G_i tables) -- the fixed-base precomputation behind the MSM
    paths"""
    b = ctypes.c_uint64()
    k = ctypes.c_int()
    s = ctypes.c_double()
    g = ctypes.c_uint64()
    rc = lib().spg_comb_stats(ctypes.byref(b), ctypes.byref(k), ctypes.byref(s), ctypes.byref(g))
    if rc != 0:
        raise SpgError(f"spg_comb_stats: {SPG_ERRORS.get(rc, rc)}")
    return int(b.value), int(k.value), float(s.value), int(g.value)


_hc = None


def hostcheck():
    """lib/libspg_hostcheck.so: the host build of the product's field / curve / transcript code (tests, and the
    caller-side merlin of Transcript.from_native_merlin)"""
    global _hc
    if _hc is None:
        path = os.environ.get("SPG_HOSTCHECK_LIB") or os.path.join(_HERE, "lib", "libspg_hostcheck.so")
        _hc = ctypes.CDLL(path)
        _hc.spgh_merlin_new.restype = ctypes.c_void_p
        _hc.spgh_merlin_new.argtypes = [ctypes.c_char_p]
        _hc.spgh_merlin_free.argtypes = [ctypes.c_void_p]
        _hc.spgh_merlin_challenge_cb.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t]
    return _hc


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class SpgError(RuntimeError):
    pass


# int (*spg_allgather_fn)(void* user, const void* send, size_t bytes, void* recv)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


def torch_allgather(dist, group=None, device="cpu"):
    """An spg_allgather_fn over torch.distributed (gloo: device='cpu'; nccl = RCCL: device='cuda:<local>'):
    the `bytes` of rank k land at recv + k * bytes on every rank."""
    import torch

    def cb(user, send, nbytes, recv):
        try:
            world = dist.get_world_size(group)
            buf = bytearray(ctypes.string_at(send, nbytes)) if nbytes else bytearray(1)
            src = torch.frombuffer(buf, dtype=torch.uint8).to(device)
            outs = [torch.empty_like(src) for _ in range(world)]
            dist.all_gather(outs, src, group=group)
            flat = torch.cat(outs).cpu().numpy() if nbytes else None
            if nbytes:
                for k in range(world):
                    ctypes.memmove(recv + k * nbytes, flat[k * len(buf):].ctypes.data, nbytes)
            return 0
        except Exception as e:  # noqa: BLE001 - reported through the return code
            import sys

            print(f"spg allgather callback failed: {e!r}", file=sys.stderr)
            return 1

    return ALLGATHER_FN(cb)


class Context:
    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        rc = lib().spg_init(ctypes.c_int(device), ctypes.byref(self._h))
        if rc != 0:
            raise SpgError(f"spg_init({device}) failed: {SPG_ERRORS.get(rc, rc)} (no gfx950 device?)")

    def check(self, rc, what):
        if rc != 0:
            msg = lib().spg_last_error(self._h).decode(errors="replace")
            raise SpgError(f"{what}: {SPG_ERRORS.get(rc, rc)}: {msg}")

    def out_buf(self, cap):
        """the proof output buffer of this context's calls, kept between calls (a context runs one call at a time;
        each wrapper copies its bytes out): a fresh 16 MB np.zeros per prove cost ~0.3 ms of mmap / munmap and page
        faults beside the pool's spinning threads"""
        b = getattr(self, "_out", None)
        if b is None or b.shape[0] < cap:
            b = self._out = np.empty(cap, dtype=np.uint8)
        return b

    @property
    def handle(self):
        return self._h

    def set_comm(self, rank, nranks, allgather_fn=None):
        """spg_set_comm: shard R1CSProof::prove by instance over nranks processes (one GPU each)."""
        self._comm = allgather_fn  # keep the ctypes thunk alive
        fn = allgather_fn if allgather_fn is not None else ctypes.cast(None, ALLGATHER_FN)
        self.check(lib().spg_set_comm(self._h, ctypes.c_int(rank), ctypes.c_int(nranks), fn, None), "spg_set_comm")

    def set_comm_rccl(self, rank, nranks, dist=None, unique_id=None):
        """spg_set_comm_rccl: libspg's own RCCL transport on the context stream. Rank 0's 128-byte id
        (spg_rccl_unique_id) reaches every rank through `dist` (torch.distributed broadcast_object_list over the
        default group) unless unique_id is given."""
        if unique_id is None:
            buf = (ctypes.c_uint8 * 128)()
            if rank == 0:
                rc = lib().spg_rccl_unique_id(buf)
                if rc != 0:
                    raise SpgError(f"spg_rccl_unique_id: {SPG_ERRORS.get(rc, rc)}")
            if nranks > 1:
                obj = [bytes(buf) if rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                unique_id = obj[0]
            else:
                unique_id = bytes(buf)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        self._comm = None
        self.check(lib().spg_set_comm_rccl(self._h, uid, ctypes.c_int(rank), ctypes.c_int(nranks)), "spg_set_comm_rccl")

    def comm_allgather(self, data, nranks):
        """spg_comm_allgather over the context's transport: every rank's `data` (equal lengths), rank-ordered"""
        n = len(data)
        src = (ctypes.c_uint8 * max(n, 1)).from_buffer_copy(bytes(data) or b"\0")
        dst = (ctypes.c_uint8 * max(n * nranks, 1))()
        self.check(lib().spg_comm_allgather(self._h, src, ctypes.c_size_t(n), dst), "spg_comm_allgather")
        raw = bytes(dst)
        return [raw[k * n:(k + 1) * n] for k in range(nranks)]

    def set_comb(self, on=True):
        """spg_set_comb: off -> this context's MSMs skip the comb tables (bucket Pippenger pipelines only)"""
        self.check(lib().spg_set_comb(self._h, ctypes.c_int(1 if on else 0)), "spg_set_comb")

    def last_kernel_us(self):
        return lib().spg_last_kernel_us(self._h)

    def prof_enable(self, on=True):
        self.check(lib().spg_prof_enable(self._h, ctypes.c_int(1 if on else 0)), "spg_prof_enable")

    def prof_read(self, reset=True, ops=False):
        """{kernel_name: (launches, total_us, algorithmic_bytes)} of the kernels timed since the last reset;
        ops=True appends the modelled VALU work of those launches to each tuple: curve mixed additions, then Fq
        products."""
        mx = 128
        names = ctypes.create_string_buffer(32 * mx)
        launches = np.zeros(mx, dtype=np.int64)
        tot = np.zeros(mx, dtype=np.float64)
        nbytes = np.zeros(mx, dtype=np.float64)
        nops = np.zeros(mx, dtype=np.float64)
        nfqm = np.zeros(mx, dtype=np.float64)
        k = lib().spg_prof_read3(self._h, names, _p(launches), _p(tot), _p(nbytes), _p(nops), _p(nfqm),
                                 ctypes.c_int(mx), ctypes.c_int(1 if reset else 0))
        if k < 0:
            self.check(k, "spg_prof_read3")
        raw = names.raw
        out = {}
        for i in range(k):
            nm = raw[32 * i:32 * i + 32].split(b"\0", 1)[0].decode()
            rec = (int(launches[i]), float(tot[i]), float(nbytes[i]))
            out[nm] = rec + (float(nops[i]), float(nfqm[i])) if ops else rec
        return out

    def close(self):
        if self._h:
            lib().spg_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _scalars(x):
    a = np.ascontiguousarray(x, dtype=np.uint64)
    if a.shape[-1] != 4:
        a = a.reshape(-1, 4)
    return a


class Buf:
    """Device-resident vector of Montgomery scalars (spg_buf)."""

    def __init__(self, ctx, scalars):
        self.ctx = ctx
        a = _scalars(scalars)
        self.n = a.shape[0]
        self._h = ctypes.c_void_p()
        ctx.check(lib().spg_buf_upload(ctx.handle, _p(a), ctypes.c_size_t(self.n), ctypes.byref(self._h)),
                  "spg_buf_upload")

    @property
    def handle(self):
        return self._h

    def download(self):
        out = np.zeros((self.n, 4), dtype=np.uint64)
        self.ctx.check(lib().spg_buf_download(self.ctx.handle, self._h, _p(out)), "spg_buf_download")
        return out

    @classmethod
    def eq_evals(cls, ctx, r):
        """EqPolynomial::new(r).evals() (src/dense_mlpoly.rs:76-92) built on the device (spg_eq_evals)."""
        a = _scalars(r) if len(r) else np.zeros((0, 4), dtype=np.uint64)
        b = cls.__new__(cls)
        b.ctx = ctx
        b.n = 1 << a.shape[0]
        b._h = ctypes.c_void_p()
        ctx.check(lib().spg_eq_evals(ctx.handle, _p(a), ctypes.c_size_t(a.shape[0]), ctypes.byref(b._h)),
                  "spg_eq_evals")
        return b

    # per-operation seams (csrc/seams.hip)
    def bound_top(self, r):
        """DensePolynomial::bound_poly_var_top (src/dense_mlpoly.rs:267-275), in place; the length halves."""
        self.ctx.check(lib().spg_buf_bound_top(self.ctx.handle, self._h, _p(_scalars(r))), "spg_buf_bound_top")
        self.n //= 2

    def bound_bot(self, r):
        """DensePolynomial::bound_poly_var_bot (src/dense_mlpoly.rs:350-358), in place; the length halves."""
        self.ctx.check(lib().spg_buf_bound_bot(self.ctx.handle, self._h, _p(_scalars(r))), "spg_buf_bound_bot")
        self.n //= 2

    def evaluate(self, r):
        """DensePolynomial::evaluate (src/dense_mlpoly.rs:361-367) at r (len(r) = log2 of the length)."""
        a = _scalars(r) if len(r) else np.zeros((1, 4), dtype=np.uint64)
        out = np.zeros(4, dtype=np.uint64)
        self.ctx.check(lib().spg_buf_evaluate(self.ctx.handle, self._h, _p(a), ctypes.c_size_t(len(r)), _p(out)),
                       "spg_buf_evaluate")
        return out

    @staticmethod
    def cubic_round_evals(A, B, C):
        """One prove_cubic round's (e0, e2, e3) with comb A B C (src/sumcheck.rs:207-236)."""
        out = np.zeros((3, 4), dtype=np.uint64)
        A.ctx.check(lib().spg_cubic_round_evals(A.ctx.handle, A._h, B._h, C._h, _p(out)), "spg_cubic_round_evals")
        return out

    @staticmethod
    def prove_cubic(claim, num_rounds, A, B, C, transcript):
        """SumcheckInstanceProof::prove_cubic with comb A B C (src/sumcheck.rs:193-262): A, B, C bound in place.
        Returns (compressed polys [num_rounds, 3, 4], r [num_rounds, 4], claims [3, 4])."""
        polys = np.zeros((max(num_rounds, 1), 3, 4), dtype=np.uint64)
        r = np.zeros((max(num_rounds, 1), 4), dtype=np.uint64)
        claims = np.zeros((3, 4), dtype=np.uint64)
        A.ctx.check(lib().spg_prove_cubic(A.ctx.handle, _p(_scalars(claim)), ctypes.c_size_t(num_rounds), A._h, B._h,
                                          C._h, transcript.handle, _p(polys), _p(r), _p(claims)), "spg_prove_cubic")
        for b in (A, B, C):
            b.n >>= num_rounds
        return polys[:num_rounds], r[:num_rounds], claims

    def free(self):
        if self._h:
            lib().spg_buf_free(self.ctx.handle, self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Pqx:
    """DensePolynomialPqx (src/custom_dense_mlpoly.rs:22-359) resident in HBM (spg_pqx_*): z holds instance p's
    num_proofs[p] x num_witness_secs x num_inputs[p] scalars in (q_rev, w, x_rev) order, instances concatenated."""

    def __init__(self, ctx, z, num_proofs, max_num_proofs, num_witness_secs, num_inputs, max_num_inputs):
        self.ctx = ctx
        a = _scalars(z)
        self.P = len(num_proofs)
        self.n = a.shape[0]
        np_ = np.asarray(num_proofs, dtype=np.uint64)
        ni_ = np.asarray(num_inputs, dtype=np.uint64)
        self._h = ctypes.c_void_p()
        ctx.check(lib().spg_pqx_new(ctx.handle, _p(a), ctypes.c_size_t(self.P), _p(np_), ctypes.c_size_t(max_num_proofs),
                                    ctypes.c_size_t(num_witness_secs), _p(ni_), ctypes.c_size_t(max_num_inputs),
                                    ctypes.byref(self._h)), "spg_pqx_new")

    def bound(self, r, mode):
        """bound_poly(r, mode): 1 = p, 2 = q, 3 = w, 4 = x (src/custom_dense_mlpoly.rs:180-199)"""
        self.ctx.check(lib().spg_pqx_bound(self.ctx.handle, self._h, _p(_scalars(r)), ctypes.c_int(mode)),
                       "spg_pqx_bound")

    def evaluate(self, rp, rq, rw, rx):
        """evaluate(r_p, r_q, r_w, r_x) (src/custom_dense_mlpoly.rs:320-333); the table is left unchanged"""
        arrs = [_scalars(r) if len(r) else np.zeros((1, 4), dtype=np.uint64) for r in (rp, rq, rw, rx)]
        args = []
        for a, r in zip(arrs, (rp, rq, rw, rx)):
            args += [_p(a), ctypes.c_size_t(len(r))]
        out = np.zeros(4, dtype=np.uint64)
        self.ctx.check(lib().spg_pqx_evaluate(self.ctx.handle, self._h, *args, _p(out)), "spg_pqx_evaluate")
        return out

    def shape(self):
        dims = np.zeros(4, dtype=np.uint64)
        npf = np.zeros(self.P, dtype=np.uint64)
        nin = np.zeros(self.P, dtype=np.uint64)
        assert lib().spg_pqx_shape(self._h, _p(dims), _p(npf), _p(nin)) == 0
        return tuple(int(x) for x in dims), [int(x) for x in npf], [int(x) for x in nin]

    def download(self):
        out = np.zeros((self.n, 4), dtype=np.uint64)
        self.ctx.check(lib().spg_pqx_download(self.ctx.handle, self._h, _p(out)), "spg_pqx_download")
        return out

    def __del__(self):
        try:
            if self._h:
                lib().spg_pqx_free(self.ctx.handle, self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


class Gens:
    """Device-resident MultiCommitGens (G_0..G_{n-1}, h) with fixed-base window tables."""

    def __init__(self, ctx, n, label=None, compressed=None):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        if compressed is not None:
            comp = np.ascontiguousarray(compressed, dtype=np.uint8).reshape(-1, 32)
            assert comp.shape[0] == n + 1
            rc = lib().spg_gens_upload(ctx.handle, _p(comp), ctypes.c_size_t(n), ctypes.byref(self._h))
            ctx.check(rc, "spg_gens_upload")
        else:
            lb = np.frombuffer(bytes(label), dtype=np.uint8).copy() if label else np.zeros(1, np.uint8)
            rc = lib().spg_gens_derive(ctx.handle, _p(lb), ctypes.c_size_t(len(label or b"")), ctypes.c_size_t(n),
                                       ctypes.byref(self._h))
            ctx.check(rc, "spg_gens_derive")
        self.n = n

    def compressed(self):
        out = np.zeros((self.n + 1, 32), dtype=np.uint8)
        self.ctx.check(lib().spg_gens_download(self.ctx.handle, self._h, _p(out)), "spg_gens_download")
        return out

    def msm(self, scalars, blind=None, gen_offset=0):
        s = _scalars(scalars)
        out = np.zeros(32, dtype=np.uint8)
        bl = None if blind is None else _scalars(blind)
        rc = lib().spg_msm(self.ctx.handle, self._h, ctypes.c_size_t(gen_offset), _p(s), ctypes.c_size_t(s.shape[0]),
                           None if bl is None else _p(bl), _p(out))
        self.ctx.check(rc, "spg_msm")
        return out.tobytes()

    def msm_partial(self, scalars, gen_offset=0):
        """spg_msm_partial: uncompressed (X, Y, Z, T) partial sum of one shard, 128 bytes"""
        s = _scalars(scalars)
        out = np.zeros(128, dtype=np.uint8)
        rc = lib().spg_msm_partial(self.ctx.handle, self._h, ctypes.c_size_t(gen_offset), _p(s),
                                   ctypes.c_size_t(s.shape[0]), _p(out))
        self.ctx.check(rc, "spg_msm_partial")
        return out.tobytes()

    def msm_partial_buf(self, buf, offset=0, n=None, gen_offset=0):
        """spg_msm_partial_buf: the partial sum of scalars already resident in HBM (a Buf), 128 bytes"""
        n = buf.n - offset if n is None else n
        out = np.zeros(128, dtype=np.uint8)
        rc = lib().spg_msm_partial_buf(self.ctx.handle, self._h, ctypes.c_size_t(gen_offset), buf._h,
                                       ctypes.c_size_t(offset), ctypes.c_size_t(n), _p(out))
        self.ctx.check(rc, "spg_msm_partial_buf")
        return out.tobytes()

    def msm_buf(self, buf, offset=0, n=None, gen_offset=0):
        """spg_msm_buf: vartime_multiscalar_mul of resident scalars, 32-byte compression"""
        n = buf.n - offset if n is None else n
        out = np.zeros(32, dtype=np.uint8)
        rc = lib().spg_msm_buf(self.ctx.handle, self._h, ctypes.c_size_t(gen_offset), buf._h, ctypes.c_size_t(offset),
                               ctypes.c_size_t(n), _p(out))
        self.ctx.check(rc, "spg_msm_buf")
        return out.tobytes()

    def commit_rows(self, Z, L, R, blinds=None):
        z = _scalars(Z)
        assert z.shape[0] == L * R
        out = np.zeros((L, 32), dtype=np.uint8)
        bl = None if blinds is None else _scalars(blinds)
        rc = lib().spg_commit_rows(self.ctx.handle, self._h, _p(z), ctypes.c_size_t(L), ctypes.c_size_t(R),
                                   None if bl is None else _p(bl), _p(out))
        self.ctx.check(rc, "spg_commit_rows")
        return out

    def commit_rows_buf(self, zbuf, L, R, offset=0, blinds_buf=None):
        out = np.zeros((L, 32), dtype=np.uint8)
        rc = lib().spg_commit_rows_buf(self.ctx.handle, self._h, zbuf.handle, ctypes.c_size_t(offset), ctypes.c_size_t(L),
                                       ctypes.c_size_t(R), None if blinds_buf is None else blinds_buf.handle, _p(out))
        self.ctx.check(rc, "spg_commit_rows_buf")
        return out

    def free(self):
        if self._h:
            lib().spg_gens_free(self.ctx.handle, self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---------------------------------------------------------------- Fiat-Shamir objects
# int (*spg_transcript_append_fn)(void* user, const char* label, const uint8_t* msg, size_t len)
# int (*spg_transcript_challenge_fn)(void* user, const char* label, uint8_t* out, size_t len)
TRANSCRIPT_APPEND_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t)
TRANSCRIPT_CHALLENGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p,
                                           ctypes.c_size_t)


class Transcript:
    """ProofTranscript over merlin (src/transcript.rs:5-63), host object in libspg; or, with from_callbacks, a view
    of the caller's own transcript (every append_message / challenge_bytes is forwarded to it)."""

    def __init__(self, label):
        self._h = ctypes.c_void_p()
        rc = lib().spg_transcript_new(ctypes.c_char_p(bytes(label)), ctypes.byref(self._h))
        if rc != 0:
            raise SpgError(f"spg_transcript_new: {SPG_ERRORS.get(rc, rc)}")

    @classmethod
    def from_callbacks(cls, append, challenge):
        """spg_transcript_new_callbacks: append(label: bytes, msg: bytes) and challenge(label: bytes, n) -> n bytes
        are the caller's merlin append_message / challenge_bytes; an exception in either is a failed callback
        (the running call returns SPG_E_CALLBACK)."""

        def app(user, label, msg, n):
            try:
                append(label, ctypes.string_at(msg, n) if n else b"")
                return 0
            except Exception:  # noqa: BLE001 - reported through the return code
                return 1

        def chal(user, label, out, n):
            try:
                b = challenge(label, n)
                assert len(b) == n
                if n:
                    ctypes.memmove(out, b, n)
                return 0
            except Exception:  # noqa: BLE001
                return 1

        t = cls.__new__(cls)
        t._cbs = (TRANSCRIPT_APPEND_FN(app), TRANSCRIPT_CHALLENGE_FN(chal))  # keep the thunks alive
        t._h = ctypes.c_void_p()
        rc = lib().spg_transcript_new_callbacks(t._cbs[0], t._cbs[1], None, ctypes.byref(t._h))
        if rc != 0:
            raise SpgError(f"spg_transcript_new_callbacks: {SPG_ERRORS.get(rc, rc)}")
        return t

    @classmethod
    def from_native_merlin(cls, label):
        """spg_transcript_new_callbacks over a caller-owned merlin::Transcript in native code (libspg_hostcheck's
        spgh_merlin_*: C callbacks, no Python per append / challenge) -- the drop-in mode a Rust caller gets with
        extern "C" trampolines over its &mut Transcript. The returned object also holds
        the caller's transcript: caller_challenge(label, n) reads challenge bytes from it after a prove."""
        hc = hostcheck()
        t = cls.__new__(cls)
        t._merlin = ctypes.c_void_p(hc.spgh_merlin_new(ctypes.c_char_p(bytes(label))))
        t._free_merlin = hc.spgh_merlin_free
        t._h = ctypes.c_void_p()
        rc = lib().spg_transcript_new_callbacks(ctypes.cast(hc.spgh_merlin_append_cb, ctypes.c_void_p),
                                                ctypes.cast(hc.spgh_merlin_challenge_cb, ctypes.c_void_p),
                                                t._merlin, ctypes.byref(t._h))
        if rc != 0:
            hc.spgh_merlin_free(t._merlin)
            raise SpgError(f"spg_transcript_new_callbacks: {SPG_ERRORS.get(rc, rc)}")
        return t

    def caller_challenge(self, label, n):
        out = (ctypes.c_uint8 * max(n, 1))()
        hostcheck().spgh_merlin_challenge_cb(self._merlin, ctypes.c_char_p(bytes(label)), out, ctypes.c_size_t(n))
        return bytes(out)[:n]

    @property
    def handle(self):
        return self._h

    def append_message(self, label, msg):
        m = np.frombuffer(bytes(msg), dtype=np.uint8).copy() if msg else np.zeros(1, np.uint8)
        rc = lib().spg_transcript_append_message(self._h, ctypes.c_char_p(bytes(label)), _p(m), ctypes.c_size_t(len(msg)))
        if rc != 0:
            raise SpgError(f"spg_transcript_append_message: {SPG_ERRORS.get(rc, rc)}")

    def append_scalar(self, label, s):
        a = _scalars(s)
        assert lib().spg_transcript_append_scalar(self._h, ctypes.c_char_p(bytes(label)), _p(a)) == 0

    def challenge_scalar(self, label):
        out = np.zeros(4, dtype=np.uint64)
        assert lib().spg_transcript_challenge_scalar(self._h, ctypes.c_char_p(bytes(label)), _p(out)) == 0
        return out

    def challenge_bytes(self, label, n):
        out = np.zeros(max(n, 1), dtype=np.uint8)
        rc = lib().spg_transcript_challenge_bytes(self._h, ctypes.c_char_p(bytes(label)), _p(out), ctypes.c_size_t(n))
        if rc != 0:
            raise SpgError(f"spg_transcript_challenge_bytes: {SPG_ERRORS.get(rc, rc)}")
        return out[:n].tobytes()

    def __del__(self):
        try:
            if self._h:
                lib().spg_transcript_free(self._h)
                self._h = ctypes.c_void_p()
            m = getattr(self, "_merlin", None)
            if m:
                self._free_merlin(m)
                self._merlin = None
        except Exception:
            pass


class RandomTape:
    """RandomTape (src/random.rs:7-29) with a caller-supplied init scalar (Montgomery limbs)."""

    def __init__(self, name, init_scalar):
        self._h = ctypes.c_void_p()
        a = _scalars(init_scalar)
        rc = lib().spg_random_tape_new(ctypes.c_char_p(bytes(name)), _p(a), ctypes.byref(self._h))
        if rc != 0:
            raise SpgError(f"spg_random_tape_new: {SPG_ERRORS.get(rc, rc)}")

    @property
    def handle(self):
        return self._h

    def random_scalar(self, label):
        out = np.zeros(4, dtype=np.uint64)
        assert lib().spg_random_tape_scalar(self._h, ctypes.c_char_p(bytes(label)), _p(out)) == 0
        return out

    def __del__(self):
        try:
            if self._h:
                lib().spg_random_tape_free(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


# ---------------------------------------------------------------- R1CSProof
class R1CSGens:
    """R1CSGens::new(label, _, num_vars) (src/r1csproof.rs:71-79), resident in HBM."""

    def __init__(self, ctx, label, num_vars):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        lb = np.frombuffer(bytes(label), dtype=np.uint8).copy()
        ctx.check(lib().spg_r1cs_gens_new(ctx.handle, _p(lb), ctypes.c_size_t(len(label)), ctypes.c_size_t(num_vars),
                                          ctypes.byref(self._h)), "spg_r1cs_gens_new")

    @property
    def handle(self):
        return self._h

    def compressed(self):
        cnt = ctypes.c_size_t(0)
        self.ctx.check(lib().spg_r1cs_gens_download(self.ctx.handle, self._h, None, ctypes.byref(cnt)), "download")
        out = np.zeros((cnt.value, 32), dtype=np.uint8)
        self.ctx.check(lib().spg_r1cs_gens_download(self.ctx.handle, self._h, _p(out), ctypes.byref(cnt)), "download")
        return out

    def __del__(self):
        try:
            if self._h:
                lib().spg_r1cs_gens_free(self.ctx.handle, self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


class R1CSInst:
    """R1CSInstance uploaded once (CSR + merged CSC in HBM). `cinst` is a workload.CViews().inst."""

    def __init__(self, ctx, cinst):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        ctx.check(lib().spg_r1cs_inst_new(ctx.handle, ctypes.byref(cinst), ctypes.byref(self._h)), "spg_r1cs_inst_new")

    @property
    def handle(self):
        return self._h

    def __del__(self):
        try:
            if self._h:
                lib().spg_r1cs_inst_free(self.ctx.handle, self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


def phase1_round_evals(Ap, Aq, Ax, B, C, D, mode):
    """one x (mode 4) or q (mode 2) round of the phase-1 sumcheck (src/sumcheck.rs:1173-1245): (e0, e2, e3)"""
    out = np.zeros((3, 4), dtype=np.uint64)
    Ap.ctx.check(lib().spg_phase1_round_evals(Ap.ctx.handle, Ap.handle, Aq.handle, Ax.handle, B._h, C._h, D._h,
                                              ctypes.c_int(mode), _p(out)), "spg_phase1_round_evals")
    return out


def phase2_round_evals(A, ABC, Z, mode, single_inst, num_witness_secs):
    """one y (4), w (3) or p (1) round of the phase-2 sumcheck (src/sumcheck.rs:881-941): (e0, e2, e3)"""
    out = np.zeros((3, 4), dtype=np.uint64)
    A.ctx.check(lib().spg_phase2_round_evals(A.ctx.handle, A.handle, ABC._h, Z._h, ctypes.c_int(mode),
                                             ctypes.c_int(1 if single_inst else 0), ctypes.c_size_t(num_witness_secs),
                                             _p(out)), "spg_phase2_round_evals")
    return out


def r1cs_multiply_vec_block(ctx, inst, num_proofs, max_num_proofs, num_inputs, max_num_inputs, num_witness_secs, z):
    """R1CSInstance::multiply_vec_block (src/r1csinstance.rs:363-436) -> (Az, Bz, Cz) as resident Pqx tables; z holds
    instance p's num_proofs[p] x num_witness_secs x num_inputs[p] scalars, instances concatenated"""
    P = len(num_proofs)
    a = _scalars(z)
    np_ = np.asarray(num_proofs, dtype=np.uint64)
    ni_ = np.asarray(num_inputs, dtype=np.uint64)
    hs = [ctypes.c_void_p() for _ in range(3)]
    ctx.check(lib().spg_r1cs_multiply_vec_block(ctx.handle, inst.handle, ctypes.c_size_t(P), _p(np_),
                                                ctypes.c_size_t(max_num_proofs), _p(ni_), ctypes.c_size_t(max_num_inputs),
                                                ctypes.c_size_t(num_witness_secs), _p(a), *[ctypes.byref(h) for h in hs]),
              "spg_r1cs_multiply_vec_block")
    out = []
    for h in hs:
        t = Pqx.__new__(Pqx)
        t.ctx, t._h, t.P = ctx, h, P
        dims = np.zeros(4, dtype=np.uint64)
        npf = np.zeros(P, dtype=np.uint64)
        nin = np.zeros(P, dtype=np.uint64)
        assert lib().spg_pqx_shape(h, _p(dims), _p(npf), _p(nin)) == 0
        t.n = int(sum(int(x) * int(y) for x, y in zip(npf, nin)))
        out.append(t)
    return tuple(out)


def r1cs_multi_evaluate(ctx, inst, num_instances, rx, ry):
    """R1CSInstance::multi_evaluate -> (3 * num_instances, 4) limbs [A_0, B_0, C_0, A_1, ...]"""
    rx = _scalars(rx)
    ry = _scalars(ry)
    out = np.zeros((3 * num_instances, 4), dtype=np.uint64)
    ctx.check(lib().spg_r1cs_multi_evaluate(ctx.handle, inst.handle, _p(rx), ctypes.c_size_t(rx.shape[0]), _p(ry),
                                            ctypes.c_size_t(ry.shape[0]), _p(out)), "spg_r1cs_multi_evaluate")
    return out


class R1CSWitness:
    """Witness sections (Vec<&ProverWitnessSecInfo>) resident in HBM. `secs` is workload.CViews().secs.
    shard=(p0, p1): upload only instances [p0, p1) of the per-instance sections (sharded proving)."""

    def __init__(self, ctx, secs, nws, shard=None):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        if shard is None:
            ctx.check(lib().spg_r1cs_witness_new(ctx.handle, secs, ctypes.c_size_t(nws), ctypes.byref(self._h)),
                      "spg_r1cs_witness_new")
        else:
            ctx.check(lib().spg_r1cs_witness_new_shard(ctx.handle, secs, ctypes.c_size_t(nws), ctypes.c_size_t(shard[0]),
                                                       ctypes.c_size_t(shard[1]), ctypes.byref(self._h)),
                      "spg_r1cs_witness_new_shard")

    @property
    def handle(self):
        return self._h

    def __del__(self):
        try:
            if self._h:
                lib().spg_r1cs_witness_free(self.ctx.handle, self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


def r1cs_prove(ctx, gens, inst, witness, num_instances, max_num_proofs, num_proofs, max_num_inputs, num_inputs,
               transcript, tape, cap=1 << 22):
    """R1CSProof::prove -> (bincode bytes, [rp, rq_rev, rx, rw||ry] as (k, 4) uint64 arrays)."""
    buf = ctx.out_buf(cap)
    ln = ctypes.c_size_t(0)
    ch = np.zeros((4096, 4), dtype=np.uint64)
    chl = (ctypes.c_size_t * 4)()
    npf = (ctypes.c_size_t * num_instances)(*num_proofs)
    nin = (ctypes.c_size_t * num_instances)(*num_inputs)
    rc = lib().spg_r1cs_prove(ctx.handle, gens.handle, inst.handle, ctypes.c_size_t(num_instances),
                              ctypes.c_size_t(max_num_proofs), npf, ctypes.c_size_t(max_num_inputs), nin,
                              witness.handle, transcript.handle, tape.handle, _p(buf), ctypes.c_size_t(cap),
                              ctypes.byref(ln), _p(ch), chl)
    ctx.check(rc, "spg_r1cs_prove")
    out, o = [], 0
    for L in list(chl):
        out.append(ch[o:o + L].copy())
        o += L
    return buf[: ln.value].tobytes(), out


class CWitnessComm(ctypes.Structure):
    _fields_ = [("num_instances", ctypes.c_size_t), ("num_proofs", ctypes.POINTER(ctypes.c_size_t)),
                ("num_inputs", ctypes.POINTER(ctypes.c_size_t)), ("comm_len", ctypes.POINTER(ctypes.c_size_t)),
                ("comms", ctypes.c_void_p)]


def r1cs_gens_commit(ctx, gens, Z):
    """DensePolynomial::commit (no blinds) with gens.gens_pc -> list of 32-byte Hyrax row commitments"""
    z = _scalars(Z)
    out = np.zeros(32 * 4096, dtype=np.uint8)
    L = ctypes.c_size_t(0)
    ctx.check(lib().spg_r1cs_gens_commit(ctx.handle, gens.handle, _p(z), ctypes.c_size_t(z.shape[0]), _p(out),
                                         ctypes.c_size_t(out.shape[0]), ctypes.byref(L)), "spg_r1cs_gens_commit")
    return [out[32 * i: 32 * i + 32].tobytes() for i in range(L.value)]


def r1cs_verify(ctx, gens, num_instances, max_num_proofs, num_proofs, max_num_inputs, sections, num_cons, evals,
                transcript, proof):
    """R1CSProof::verify (src/r1csproof.rs:687-954). sections: per witness section (num_proofs, num_inputs, comms)
    with one entry per instance (comms: lists of 32-byte row commitments). Returns (ok, reason, challenges)."""
    keep = []
    secs = (CWitnessComm * len(sections))()
    for i, (npf, nin, comms) in enumerate(sections):
        a, b = (ctypes.c_size_t * len(npf))(*npf), (ctypes.c_size_t * len(nin))(*nin)
        cl = (ctypes.c_size_t * len(comms))(*[len(c) for c in comms])
        blob = np.frombuffer(b"".join(b"".join(c) for c in comms) or b"\0", dtype=np.uint8).copy()
        keep += [a, b, cl, blob]
        secs[i] = CWitnessComm(len(npf), a, b, cl, blob.ctypes.data)
    ev = _scalars(evals)
    buf = np.frombuffer(bytes(proof), dtype=np.uint8).copy() if len(proof) else np.zeros(1, np.uint8)
    ch = np.zeros((4096, 4), dtype=np.uint64)
    chl = (ctypes.c_size_t * 4)()
    npf = (ctypes.c_size_t * num_instances)(*num_proofs)
    rc = lib().spg_r1cs_verify(ctx.handle, gens.handle, ctypes.c_size_t(num_instances), ctypes.c_size_t(max_num_proofs),
                               npf, ctypes.c_size_t(max_num_inputs), secs, ctypes.c_size_t(len(sections)),
                               ctypes.c_size_t(num_cons), _p(ev), transcript.handle, _p(buf), ctypes.c_size_t(len(proof)),
                               _p(ch), chl)
    if rc == SPG_E_VERIFY:
        return False, lib().spg_last_error(ctx.handle).decode(errors="replace"), None
    ctx.check(rc, "spg_r1cs_verify")
    out, o = [], 0
    for L in list(chl):
        out.append(ch[o:o + L].copy())
        o += L
    return True, "", out


def shard_range(num_instances, rank, nranks):
    """instances [p0, p1) held by `rank` in a sharded R1CSProof (include/spg.h, spg_set_comm): balanced split,
    the first num_instances % nranks ranks hold one instance more (same rule as r1cs.hip Prover::shard_begin)"""
    def begin(r):
        return r * (num_instances // nranks) + min(r, num_instances % nranks)
    return begin(rank), begin(rank + 1)


class SparkCommitment:
    """SparseMatPolynomial::multi_commit over the 3P matrices of an R1CS instance (src/sparse_mlpoly.rs:566-587)
    with SparseMatPolyCommitmentGens::new(label, nvx, nvy, gens_nnz, gens_batch). The dense representation
    stays in HBM for SparkCommitment.prove. `cinst` is a workload.CViews().inst."""

    def __init__(self, ctx, cinst, label, gens_nnz, gens_batch=3, cap=1 << 22):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        if isinstance(label, str):
            label = label.encode()
        buf = np.zeros(cap, dtype=np.uint8)
        ln = ctypes.c_size_t(0)
        lb = (ctypes.c_uint8 * len(label)).from_buffer_copy(label)
        ctx.check(lib().spg_spark_commit(ctx.handle, ctypes.byref(cinst), lb, ctypes.c_size_t(len(label)),
                                         ctypes.c_size_t(gens_nnz), ctypes.c_size_t(gens_batch), ctypes.byref(self._h),
                                         _p(buf), ctypes.c_size_t(cap), ctypes.byref(ln)), "spg_spark_commit")
        self.bytes = buf[: ln.value].tobytes()

    @property
    def handle(self):
        return self._h

    def prove(self, rx, ry, evals, transcript, tape, cap=1 << 24):
        """SparseMatPolyEvalProof::prove (src/sparse_mlpoly.rs:1497-1564) -> bincode bytes"""
        rx = _scalars(rx)
        ry = _scalars(ry)
        ev = _scalars(evals)
        buf = self.ctx.out_buf(cap)
        ln = ctypes.c_size_t(0)
        self.ctx.check(lib().spg_spark_prove(self.ctx.handle, self._h, _p(rx), ctypes.c_size_t(rx.shape[0]), _p(ry),
                                             ctypes.c_size_t(ry.shape[0]), _p(ev), ctypes.c_size_t(ev.shape[0]),
                                             transcript.handle, tape.handle, _p(buf), ctypes.c_size_t(cap),
                                             ctypes.byref(ln)), "spg_spark_prove")
        return buf[: ln.value].tobytes()

    def verify(self, rx, ry, evals, transcript, proof):
        """SparseMatPolyEvalProof::verify (src/sparse_mlpoly.rs:1566-1610) -> (ok, reason)"""
        rx, ry, ev = _scalars(rx), _scalars(ry), _scalars(evals)
        buf = np.frombuffer(bytes(proof), dtype=np.uint8).copy() if len(proof) else np.zeros(1, np.uint8)
        rc = lib().spg_spark_verify(self.ctx.handle, self._h, _p(rx), ctypes.c_size_t(rx.shape[0]), _p(ry),
                                    ctypes.c_size_t(ry.shape[0]), _p(ev), ctypes.c_size_t(ev.shape[0]),
                                    transcript.handle, _p(buf), ctypes.c_size_t(len(proof)))
        if rc == SPG_E_VERIFY:
            return False, lib().spg_last_error(self.ctx.handle).decode(errors="replace")
        self.ctx.check(rc, "spg_spark_verify")
        return True, ""

    def __del__(self):
        try:
            if self._h:
                lib().spg_spark_free(self.ctx.handle, self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


class SnarkComp:
    """SNARK::multi_encode (multi=True) / SNARK::encode of one R1CS instance (src/lib.rs:793-829); `cinst` is a
    workload.SnarkViews().block / .pairwise / .perm_root (spg_snark_instance)."""

    def __init__(self, ctx, cinst, multi=False):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        ctx.check(lib().spg_snark_encode(ctx.handle, ctypes.byref(cinst), ctypes.c_int(1 if multi else 0),
                                         ctypes.byref(self._h)), "spg_snark_encode")

    @property
    def handle(self):
        return self._h

    def comm_bytes(self, as_list):
        """bincode(Vec<ComputationCommitment>) (as_list) or bincode(ComputationCommitment) (spg_snark_comm_bytes)"""
        ln = ctypes.c_size_t(0)
        lib().spg_snark_comm_bytes(self.ctx.handle, self._h, ctypes.c_int(1 if as_list else 0), None,
                                   ctypes.c_size_t(0), ctypes.byref(ln))
        buf = np.zeros(max(ln.value, 1), dtype=np.uint8)
        self.ctx.check(lib().spg_snark_comm_bytes(self.ctx.handle, self._h, ctypes.c_int(1 if as_list else 0),
                                                  _p(buf), ctypes.c_size_t(ln.value), ctypes.byref(ln)),
                       "spg_snark_comm_bytes")
        return buf[: ln.value].tobytes()

    def comm_map(self):
        """block_comm_map: one list of matrix indices 3p + m per commitment (spg_snark_comm_map)"""
        idx = np.zeros(1 << 16, dtype=np.uintp)
        lens = np.zeros(1 << 12, dtype=np.uintp)
        n = ctypes.c_size_t(0)
        self.ctx.check(lib().spg_snark_comm_map(self.ctx.handle, self._h, _p(idx), ctypes.c_size_t(len(idx)), _p(lens),
                                                ctypes.c_size_t(len(lens)), ctypes.byref(n)), "spg_snark_comm_map")
        out, o = [], 0
        for g in range(n.value):
            out.append([int(x) for x in idx[o:o + int(lens[g])]])
            o += int(lens[g])
        return out

    @classmethod
    def load(cls, ctx, comm, as_list, comm_map, num_cons, gens):
        """a verifier-side instance from ComputationCommitment bytes (spg_snark_comm_load): comm_map = block_comm_map
        for a list, num_cons = block_num_cons / pairwise_check_num_cons / perm_root_num_cons, gens = the
        SNARKGens::new(num_cons, num_vars, num_instances, num_nz_entries) arguments"""
        c = cls.__new__(cls)
        c.ctx = ctx
        c._h = ctypes.c_void_p()
        buf = np.frombuffer(bytes(comm), dtype=np.uint8).copy() if len(comm) else np.zeros(1, np.uint8)
        flat = np.array([k for l in (comm_map or []) for k in l] or [0], dtype=np.uintp)
        lens = np.array([len(l) for l in (comm_map or [])] or [0], dtype=np.uintp)
        ctx.check(lib().spg_snark_comm_load(ctx.handle, _p(buf), ctypes.c_size_t(len(comm)),
                                            ctypes.c_int(1 if as_list else 0), _p(flat), _p(lens),
                                            ctypes.c_size_t(len(comm_map or [])), ctypes.c_size_t(num_cons),
                                            *[ctypes.c_size_t(x) for x in gens], ctypes.byref(c._h)),
                  "spg_snark_comm_load")
        return c

    def __del__(self):
        try:
            if self._h:
                lib().spg_snark_comp_free(self.ctx.handle, self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


class SnarkWitness:
    """SNARK::prove's run-time inputs with block_vars / exec inputs resident in HBM (workload.SnarkViews().inputs)"""

    def __init__(self, ctx, cinputs):
        self.ctx = ctx
        self._h = ctypes.c_void_p()
        ctx.check(lib().spg_snark_witness_new(ctx.handle, ctypes.byref(cinputs), ctypes.byref(self._h)),
                  "spg_snark_witness_new")

    @property
    def handle(self):
        return self._h

    def __del__(self):
        try:
            if self._h:
                lib().spg_snark_witness_free(self.ctx.handle, self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass


def snark_prove(ctx, block, pairwise, perm_root, witness, vars_gens, transcript, tape, cap=1 << 24):
    """SNARK::prove (src/lib.rs:971-2746) -> bincode(SNARK)"""
    buf = ctx.out_buf(cap)
    ln = ctypes.c_size_t(0)
    ctx.check(lib().spg_snark_prove(ctx.handle, block.handle, pairwise.handle, perm_root.handle, witness.handle,
                                    vars_gens.handle, transcript.handle, tape.handle, _p(buf), ctypes.c_size_t(cap),
                                    ctypes.byref(ln)), "spg_snark_prove")
    return buf[: ln.value].tobytes()


SPG_E_VERIFY = -6


def snark_verify(ctx, block, pairwise, perm_root, inputs, vars_gens, transcript, proof):
    """SNARK::verify (src/lib.rs:2750-3881) of bincode(SNARK) bytes against the encoded instances and the public
    inputs (`inputs`: workload.SnarkViews().inputs; only its sizes, input / output and init memory lists are read).
    Returns (True, "") when the proof verifies, (False, reason) when it does not; raises on bad arguments."""
    buf = np.frombuffer(bytes(proof), dtype=np.uint8).copy() if len(proof) else np.zeros(1, np.uint8)
    rc = lib().spg_snark_verify(ctx.handle, block.handle, pairwise.handle, perm_root.handle, ctypes.byref(inputs),
                                vars_gens.handle, transcript.handle, _p(buf), ctypes.c_size_t(len(proof)))
    if rc == SPG_E_VERIFY:
        return False, lib().spg_last_error(ctx.handle).decode(errors="replace")
    ctx.check(rc, "spg_snark_verify")
    return True, ""


def snark_verify_public(ctx, block, pairwise, perm_root, public, vars_gens, transcript, proof):
    """SNARK::verify from what the reference verifier is given (spg_snark_verify_public): SnarkComp.load'ed
    commitments and `public` (a workload.CSnarkPublic). Returns (True, "") / (False, reason); raises on bad arguments."""
    buf = np.frombuffer(bytes(proof), dtype=np.uint8).copy() if len(proof) else np.zeros(1, np.uint8)
    rc = lib().spg_snark_verify_public(ctx.handle, block.handle, pairwise.handle, perm_root.handle,
                                       ctypes.byref(public), vars_gens.handle, transcript.handle, _p(buf),
                                       ctypes.c_size_t(len(proof)))
    if rc == SPG_E_VERIFY:
        return False, lib().spg_last_error(ctx.handle).decode(errors="replace")
    ctx.check(rc, "spg_snark_verify_public")
    return True, ""


def points_sum_compress(parts):
    """spg_points_sum_compress (host only): encoding of the sum of 128-byte partial points"""
    buf = np.frombuffer(b"".join(parts), dtype=np.uint8).copy() if parts else np.zeros(1, np.uint8)
    out = np.zeros(32, dtype=np.uint8)
    rc = lib().spg_points_sum_compress(_p(buf), ctypes.c_size_t(len(parts)), _p(out))
    assert rc == 0, rc
    return out.tobytes()
