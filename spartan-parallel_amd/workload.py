"""Synthetic data-parallel R1CS workloads (host-side input preparation; no proving here).

The reference ships no benchmark and its synthetic generator is commented out
(src/r1csinstance.rs:224-320, src/instance.rs:1517-1532), so the shape is fixed here:
P instances ("blocks"), instance p has X_p constraints and Q_p executions; section 0 of every
execution is a chain of squarings  z = [1, s, s^2, s^4, ...]  with constraint k:
    z[1+k] * z[1+k] = z[2+k]                      (A, B, C each one entry per row)
for the first half of the rows; the second half are copy constraints z_w[k] * 1 = z_w[k] that reach
into the other witness sections w >= 1 (random data), so the SpMV touches every section. Execution
seeds come from xoshiro-like splitmix64 streams seeded with 0x5350415254414E31 ("SPARTAN1").
All scalars are emitted as the reference's Montgomery limbs (uint64 x 4).
"""
import numpy as np

Q = 2**252 + 27742317777372353535851937790883648493
R = 2**256 % Q
MASK64 = (1 << 64) - 1


def splitmix64(state, n):
    out = np.empty(n, dtype=object)
    s = state
    for i in range(n):
        s = (s + 0x9E3779B97F4A7C15) & MASK64
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        out[i] = z ^ (z >> 31)
    return out, s


def to_mont_limbs(vals):
    """python ints (canonical, < q) -> (n, 4) uint64 Montgomery limbs"""
    v = np.asarray(vals, dtype=object).reshape(-1)
    m = (v * R) % Q
    out = np.empty((len(m), 4), dtype=np.uint64)
    for i in range(4):
        out[:, i] = ((m >> (64 * i)) & MASK64).astype(np.uint64)
    return out


def random_fq(n, state):
    a, s = splitmix64(state, 4 * n)
    a = a.reshape(n, 4)
    vals = (a[:, 0] | (a[:, 1] << 64) | (a[:, 2] << 128) | (a[:, 3] << 192)) % Q
    return vals, s


class R1CSWorkload:
    """Inputs of R1CSProof::prove (src/r1csproof.rs:210-230) for the synthetic circuit."""

    def __init__(self, num_cons, num_proofs, num_sections=1, max_num_inputs=None, seed=0x5350415254414E31,
                 shared_instance=False, instances=None):
        """instances: generate witness data only for these instance indices (sharded proving); every
        instance then draws from its own stream seed ^ (p+1)*0x9E3779B97F4A7C15, so any rank can build its
        shard alone. None: all instances from one sequential stream (the layout the fixtures pin)."""
        self.P = len(num_cons)
        assert len(num_proofs) == self.P
        for x in list(num_cons) + list(num_proofs):
            assert x & (x - 1) == 0, "powers of two"
        self.num_cons = list(num_cons)
        self.num_proofs = list(num_proofs)
        self.max_num_cons = max(num_cons)
        self.max_num_proofs = max(num_proofs)
        self.nws = num_sections
        self.max_num_inputs = max_num_inputs or max(4, 2 * self.max_num_cons)
        self.num_inputs = [min(max(4, 2 * x), self.max_num_inputs) if not shared_instance else self.max_num_inputs
                           for x in num_cons]
        if shared_instance:
            assert len(set(num_cons)) == 1
        self.num_vars = (1 << (num_sections - 1).bit_length()) * self.max_num_inputs
        self.shared = shared_instance
        state = seed
        # ---- matrices
        self.entries = []  # per instance: [A, B, C] as (n, 6) uint64 rows (row, col, val0..3)
        one = to_mont_limbs([1])[0]
        n_inst = 1 if shared_instance else self.P
        for p in range(n_inst):
            X, Y = self.num_cons[p], self.num_inputs[p]
            half = X // 2 if (num_sections > 1 and X >= 2) else X
            A, B, C = [], [], []
            for k in range(half):
                A.append((k, 1 + k)); B.append((k, 1 + k)); C.append((k, 2 + k))
            for k in range(half, X):
                w = 1 + (k % (num_sections - 1)) if num_sections > 1 else 0
                col = w * self.max_num_inputs + (k % Y)
                A.append((k, col)); B.append((k, 0)); C.append((k, col))
            mats = []
            for m in (A, B, C):
                arr = np.zeros((len(m), 6), dtype=np.uint64)
                arr[:, 0] = [r for r, _ in m]
                arr[:, 1] = [c for _, c in m]
                arr[:, 2:] = one
                mats.append(arr)
            self.entries.append(mats)
        # ---- witness sections: w_mat[p] = (num_proofs[p], num_inputs[p]) scalars
        self.sections = []
        inst_state = {}
        for w in range(num_sections):
            mats = []
            for p in range(self.P):
                X, Y, Qp = self.num_cons[p], self.num_inputs[p], self.num_proofs[p]
                if instances is not None:
                    if p not in instances:
                        mats.append(None)
                        continue
                    state = inst_state.get(p, (seed ^ ((p + 1) * 0x9E3779B97F4A7C15)) & MASK64)
                if w == 0:
                    half = X // 2 if (num_sections > 1 and X >= 2) else X
                    seeds, state = random_fq(Qp, state)
                    z = np.zeros((Qp, Y), dtype=object)
                    z[:, :] = 0
                    z[:, 0] = 1
                    z[:, 1] = seeds
                    cur = seeds.copy()
                    for k in range(half):
                        cur = (cur * cur) % Q
                        z[:, 2 + k] = cur
                    mats.append(to_mont_limbs(z.reshape(-1)).reshape(Qp, Y, 4))
                else:
                    vals, state = random_fq(Qp * Y, state)
                    mats.append(to_mont_limbs(vals).reshape(Qp, Y, 4))
                if instances is not None:
                    inst_state[p] = state
            self.sections.append(mats)

    @property
    def total_constraints(self):
        return sum(x * q for x, q in zip(self.num_cons, self.num_proofs))


# ---------------------------------------------------------------- C views (include/spg.h)
import ctypes  # noqa: E402


class SparseEntry(ctypes.Structure):
    _fields_ = [("row", ctypes.c_uint64), ("col", ctypes.c_uint64), ("val", ctypes.c_uint64 * 4)]


class CInstance(ctypes.Structure):
    _fields_ = [("num_instances", ctypes.c_size_t), ("max_num_cons", ctypes.c_size_t),
                ("num_vars", ctypes.c_size_t), ("num_cons", ctypes.POINTER(ctypes.c_size_t)),
                ("nnz", ctypes.POINTER(ctypes.c_size_t)), ("entries", ctypes.POINTER(ctypes.c_void_p))]


class CWitnessSec(ctypes.Structure):
    _fields_ = [("num_instances", ctypes.c_size_t), ("num_proofs", ctypes.POINTER(ctypes.c_size_t)),
                ("num_inputs", ctypes.POINTER(ctypes.c_size_t)), ("w", ctypes.POINTER(ctypes.c_void_p))]


def _sz(a):
    arr = (ctypes.c_size_t * len(a))(*a)
    return arr


class CViews:
    """Keeps numpy buffers alive and exposes the spg_r1cs_instance / spg_witness_sec views."""

    def __init__(self, wl):
        self.keep = []
        n_inst = len(wl.entries)
        ptrs = (ctypes.c_void_p * (3 * n_inst))()
        nnz = []
        for p, mats in enumerate(wl.entries):
            for m in range(3):
                arr = np.ascontiguousarray(mats[m])
                self.keep.append(arr)
                ptrs[3 * p + m] = arr.ctypes.data
                nnz.append(arr.shape[0])
        self.nc = _sz(wl.num_cons[:n_inst])
        self.nnz = _sz(nnz)
        self.ptrs = ptrs
        self.inst = CInstance(n_inst, wl.max_num_cons, wl.num_vars, self.nc, self.nnz, ptrs)
        secs = (CWitnessSec * wl.nws)()
        self.sec_keep = []
        for w in range(wl.nws):
            mats = wl.sections[w]
            wp = (ctypes.c_void_p * len(mats))()
            for p, m in enumerate(mats):
                if m is None:  # held by another rank
                    wp[p] = None
                    continue
                arr = np.ascontiguousarray(m)
                self.keep.append(arr)
                wp[p] = arr.ctypes.data
            npf = _sz([wl.num_proofs[p] if m is None else m.shape[0] for p, m in enumerate(mats)])
            nin = _sz([wl.num_inputs[p] if m is None else m.shape[1] for p, m in enumerate(mats)])
            self.sec_keep.append((wp, npf, nin))
            secs[w] = CWitnessSec(len(mats), npf, nin, wp)
        self.secs = secs
        self.num_proofs = _sz(wl.num_proofs)
        self.num_inputs = _sz(wl.num_inputs)


def tape_seed(label=b"spg-tape-seed-0"):
    """RandomTape init scalar = Scalar::from_bytes_wide(SHAKE256(label)[0..64]) as Montgomery limbs."""
    import hashlib

    b = hashlib.shake_256(label).digest(64)
    return to_mont_limbs([int.from_bytes(b, "little") % Q])[0]


class SparkWorkload:
    """one SparseMatPolynomial per A, B and C with num_vars_x = num_vars_y = k and
    2^k entries each: entry i has row = i, col = (i * 0x9E3779B1) mod 2^k, val = a random scalar (seed 5;
    uniform 252-bit limbs taken as Montgomery representations). Exposed as a one-instance R1CS so the
    same C views (CViews) carry it to spg_spark_commit / spg_r1cs_multi_evaluate."""

    def __init__(self, log_nnz, seed=5):
        n = 1 << log_nnz
        rng = np.random.default_rng(seed)
        i = np.arange(n, dtype=np.uint64)
        mats = []
        for _ in range(3):
            arr = np.empty((n, 6), dtype=np.uint64)
            arr[:, 0] = i
            arr[:, 1] = (i * np.uint64(0x9E3779B1)) & np.uint64(n - 1)
            arr[:, 2:] = rng.integers(0, 1 << 63, size=(n, 4), dtype=np.uint64, endpoint=False) * np.uint64(2) \
                + rng.integers(0, 2, size=(n, 4), dtype=np.uint64)
            arr[:, 5] &= np.uint64((1 << 60) - 1)
            mats.append(arr)
        self.entries = [mats]
        self.P = 1
        self.num_cons = [n]
        self.max_num_cons = n
        self.num_vars = n
        self.nws = 0
        self.sections = []
        self.num_proofs = [1]
        self.num_inputs = [n]
        self.nnz = n
