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
                 shared_instance=False, instances=None, num_inputs=None):
        """instances: generate witness data only for these instance indices (sharded proving); every
        instance then draws from its own stream seed ^ (p+1)*0x9E3779B97F4A7C15, so any rank can build its
        shard alone. None: all instances from one sequential stream (the layout the fixtures pin).
        num_inputs: per-instance witness widths (powers of two <= max_num_inputs) instead of the derived ones, e.g.
        one shared matrix serving instances of different widths (check_prove_args accepts it; ADVICE r4 case)."""
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
        if num_inputs is not None:
            assert len(num_inputs) == self.P
            assert all(y & (y - 1) == 0 and 4 <= y <= self.max_num_inputs for y in num_inputs)
            self.num_inputs = list(num_inputs)
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


# ---------------------------------------------------------------- SNARK::prove workload
def _instance_new(num_instances, max_num_cons, num_cons, num_vars, A, B, C):
    """Instance::new (src/instance.rs:19-146): pads num_cons / max_num_cons / num_vars to powers of two
    (at least 2 constraints) and turns (row, col, int) triples into (n, 6) uint64 entry arrays."""
    npow = lambda x: 1 << max(0, (x - 1).bit_length())
    nvp = npow(num_vars)
    mnc = max_num_cons if max_num_cons >= 2 else 2
    if npow(max_num_cons) != max_num_cons:
        mnc = npow(max_num_cons)
    ncp = [2 if c <= 1 else npow(c) for c in num_cons]
    mats = []
    for b in range(num_instances):
        one = []
        for L in (A[b], B[b], C[b]):
            arr = np.zeros((len(L), 6), dtype=np.uint64)
            if L:
                vals = to_mont_limbs([v % Q for _, _, v in L])
                for k, (r, c, _) in enumerate(L):
                    assert r < num_cons[b] and c < num_vars
                    arr[k, 0] = r
                    arr[k, 1] = c
                arr[:, 2:] = vals
            one.append(arr)
        mats.append(one)
    return mats, mnc, ncp, nvp


class _Constr:
    """Instance::gen_constr (src/instance.rs:156-192): appends one row of (col, int) terms to A, B, C"""

    def __init__(self):
        self.A, self.B, self.C = [], [], []

    def add(self, row, a, b, c):
        self.A += [(row, col, v) for col, v in a]
        self.B += [(row, col, v) for col, v in b]
        self.C += [(row, col, v) for col, v in c]


def gen_block_inst(num_vars, args, niu, num_phy_ops, num_vir_ops):
    """Instance::gen_block_inst (src/instance.rs:253-737) -> (block_num_vars, block_max_num_cons,
    block_num_non_zero_entries, (mats, max_num_cons, num_cons, num_vars))"""
    io_width = 2 * niu
    V_valid = V_cnst = 0
    V_input = lambda i: 2 + i
    V_output = lambda i: 2 + (niu - 1) + i
    V_PA = lambda i: io_width + 2 * i
    V_PD = lambda i: io_width + 2 * i + 1
    V_VA = lambda b, i: io_width + 2 * num_phy_ops[b] + 4 * i
    V_VD = lambda b, i: io_width + 2 * num_phy_ops[b] + 4 * i + 1
    V_VL = lambda b, i: io_width + 2 * num_phy_ops[b] + 4 * i + 2
    V_VT = lambda b, i: io_width + 2 * num_phy_ops[b] + 4 * i + 3
    V_tau = num_vars
    V_r = lambda i: num_vars + i
    V_in_dp = lambda i: V_input(0) if i == 0 else 2 * num_vars + 2 + i
    V_out_dp = lambda i: 2 * num_vars + 2 + (niu - 1) + i
    V_PMR = lambda i: 2 * num_vars + 2 * niu + 2 * i
    V_PMC = lambda i: 2 * num_vars + 2 * niu + 2 * i + 1
    V_VMR1 = lambda b, i: 2 * num_vars + 2 * niu + 2 * num_phy_ops[b] + 4 * i
    V_VMR2 = lambda b, i: 2 * num_vars + 2 * niu + 2 * num_phy_ops[b] + 4 * i + 1
    V_VMR3 = lambda b, i: 2 * num_vars + 2 * niu + 2 * num_phy_ops[b] + 4 * i + 2
    V_VMC = lambda b, i: 2 * num_vars + 2 * niu + 2 * num_phy_ops[b] + 4 * i + 3
    V_v, V_x, V_pi, V_d = 3 * num_vars, 3 * num_vars + 1, 3 * num_vars + 2, 3 * num_vars + 3
    V_Pp, V_Pd, V_Vp, V_Vd = 3 * num_vars + 4, 3 * num_vars + 5, 3 * num_vars + 6, 3 * num_vars + 7
    V_sv, V_spi, V_Psp, V_Vsp = 4 * num_vars, 4 * num_vars + 2, 4 * num_vars + 4, 4 * num_vars + 6
    A_l, B_l, C_l, ncons = [], [], [], []
    max_nc, nnz = 0, 0
    for b, arg in enumerate(args):
        k = _Constr()
        nA = nB = nC = 0
        for i, (a, bb, c) in enumerate(arg):
            nA += len(a); nB += len(bb); nC += len(c)
            k.add(i, a, bb, c)
        cnt = len(arg)
        for i in range(1, niu - 1):
            k.add(cnt, [(V_input(i), 1)], [(V_r(i), 1)], [(V_in_dp(i), 1)]); cnt += 1
        for i in range(niu - 1):
            k.add(cnt, [(V_output(i), 1)], [(V_r(i + niu - 1), 1)], [(V_out_dp(i), 1)]); cnt += 1
        k.add(cnt, [], [], [(V_valid, 1), (V_v, -1)]); cnt += 1
        k.add(cnt, [(V_tau, 1)] + [(V_in_dp(i), -1) for i in range(2 * niu - 2)], [(V_cnst, 1)], [(V_x, 1)]); cnt += 1
        k.add(cnt, [(V_x, 1)], [(V_spi, 1), (V_cnst, 1), (V_sv, -1)], [(V_d, 1)]); cnt += 1
        k.add(cnt, [(V_v, 1)], [(V_d, 1)], [(V_pi, 1)]); cnt += 1
        nA += 4 * niu - 2; nB += 2 * niu + 2; nC += 2 * niu + 2
        for i in range(num_phy_ops[b]):
            k.add(cnt, [(V_r(1), 1)], [(V_PD(i), 1)], [(V_PMR(i), 1)]); cnt += 1
            k.add(cnt, [(V_cnst, 1) if i == 0 else (V_PMC(i - 1), 1)], [(V_tau, 1), (V_PA(i), -1), (V_PMR(i), -1)],
                  [(V_PMC(i), 1)]); cnt += 1
        cnt += 1
        k.add(cnt, [(V_cnst, 1) if num_phy_ops[b] == 0 else (V_PMC(num_phy_ops[b] - 1), 1)],
              [(V_Psp, 1), (V_cnst, 1), (V_sv, -1)], [(V_Pd, 1)]); cnt += 1
        k.add(cnt, [(V_v, 1)], [(V_Pd, 1)], [(V_Pp, 1)]); cnt += 1
        nA += 3 * num_phy_ops[b] + 2; nB += 7 * num_phy_ops[b] + 4; nC += 3 * num_phy_ops[b] + 2
        for i in range(num_vir_ops[b]):
            k.add(cnt, [(V_r(1), 1)], [(V_VD(b, i), 1)], [(V_VMR1(b, i), 1)]); cnt += 1
            k.add(cnt, [(V_r(2), 1)], [(V_VL(b, i), 1)], [(V_VMR2(b, i), 1)]); cnt += 1
            k.add(cnt, [(V_r(3), 1)], [(V_VT(b, i), 1)], [(V_VMR3(b, i), 1)]); cnt += 1
            k.add(cnt, [(V_cnst, 1) if i == 0 else (V_VMC(b, i - 1), 1)],
                  [(V_tau, 1), (V_VA(b, i), -1), (V_VMR1(b, i), -1), (V_VMR2(b, i), -1), (V_VMR3(b, i), -1)],
                  [(V_VMC(b, i), 1)]); cnt += 1
        cnt += 1
        k.add(cnt, [(V_cnst, 1) if num_vir_ops[b] == 0 else (V_VMC(b, num_vir_ops[b] - 1), 1)],
              [(V_Vsp, 1), (V_cnst, 1), (V_sv, -1)], [(V_Vd, 1)]); cnt += 1
        k.add(cnt, [(V_v, 1)], [(V_Vd, 1)], [(V_Vp, 1)]); cnt += 1
        nA += 5 * num_vir_ops[b] + 2; nB += 13 * num_vir_ops[b] + 4; nC += 5 * num_vir_ops[b] + 2
        max_nc = max(max_nc, cnt)
        ncons.append(cnt)
        nnz = max(nnz, nA, nB, nC)
        A_l.append(k.A); B_l.append(k.B); C_l.append(k.C)
    block_num_vars = 8 * num_vars
    inst = _instance_new(len(args), max_nc, ncons, block_num_vars, A_l, B_l, C_l)
    return block_num_vars, max_nc, nnz, inst


def gen_pairwise_check_inst(max_ts_width, mem_addr_ts_bits_size):
    """Instance::gen_pairwise_check_inst (src/instance.rs:740-1073) -> (num_vars, max_num_cons, nnz, inst)"""
    width = max(8, mem_addr_ts_bits_size)
    max_nc = 8 + max_ts_width
    ncons = [2, 4, 8 + max_ts_width]
    nnz = max(13 + max_ts_width, 5 + 2 * max_ts_width)
    c0 = _Constr()  # CONSIS_CHECK
    c0.add(0, [(5, 1), (width + 4, -1)], [(width + 4, 1)], [])
    c1 = _Constr()  # PHY_MEM_COHERE
    c1.add(0, [(0, 1), (0, -1)], [(width, 1)], [])
    c1.add(1, [(width, 1)], [(0, 1), (width + 2, -1), (2, 1)], [(1, 1)])
    c1.add(2, [(1, 1)], [(width + 2, 1), (2, -1)], [])
    c1.add(3, [(1, 1)], [(width + 3, 1), (3, -1)], [])
    c2 = _Constr()  # VIR_MEM_COHERE
    V_D2, V_EQ = 2 * width, 2 * width + 1
    V_B = lambda i: 2 * width + 2 + i
    n = 0
    c2.add(n, [(0, 1), (0, -1)], [(width, 1)], []); n += 1
    c2.add(n, [(width, 1)], [(0, 1), (width + 2, -1), (2, 1)], [(1, 1)]); n += 1
    c2.add(n, [(1, 1)], [(width + 2, 1), (2, -1)], []); n += 1
    c2.add(n, [(V_EQ, 1)], [(V_EQ, 1)], [(V_EQ, 1)]); n += 1
    for i in range(max_ts_width):
        c2.add(n, [(V_B(i), 1)], [(V_B(i), 1)], [(V_B(i), 1)]); n += 1
    c2.add(n, [(1, 1)], [(width + 5, 1), (5, -1)], [(V_EQ, 1)] + [(V_B(i), 1 << i) for i in range(max_ts_width)]); n += 1
    c2.add(n, [(1, 1)], [(width + 4, 1)], [(V_D2, 1)]); n += 1
    c2.add(n, [(V_D2, 1)], [(width + 3, 1), (3, -1)], []); n += 1
    c2.add(n, [(0, 1), (1, -1)], [(width + 4, 1)], []); n += 1
    inst = _instance_new(3, max_nc, ncons, 4 * width, [c0.A, c1.A, c2.A], [c0.B, c1.B, c2.B], [c0.C, c1.C, c2.C])
    return width, max_nc, nnz, inst


def gen_perm_root_inst(niu, num_vars):
    """Instance::gen_perm_root_inst (src/instance.rs:1088-1327) -> (num_cons, nnz, inst)"""
    V_tau = 0
    V_r = lambda i: i
    V_valid = V_cnst = num_vars
    V_input = lambda i: num_vars + 2 + i
    V_output = lambda i: num_vars + 2 + (niu - 1) + i
    V_ZO = 2 * num_vars + 2
    V_in_dp = lambda i: V_input(0) if i == 0 else 2 * num_vars + 2 + i
    V_out_dp = lambda i: 2 * num_vars + 2 + (niu - 1) + i
    V_v, V_x, V_pi, V_d, V_I, V_O = (3 * num_vars + k for k in range(6))
    V_sv, V_spi = 4 * num_vars, 4 * num_vars + 2
    k = _Constr()
    n = 0
    for i in range(1, niu - 1):
        k.add(n, [(V_input(i), 1)], [(V_r(i), 1)], [(V_in_dp(i), 1)]); n += 1
    for i in range(niu - 1):
        k.add(n, [(V_output(i), 1)], [(V_r(i + niu - 1), 1)], [(V_out_dp(i), 1)]); n += 1
    k.add(n, [(V_ZO, 1)], [(V_r(niu - 1), 1)], [(V_out_dp(i), 1) for i in range(niu - 1)]); n += 1
    k.add(n, [(V_valid, 1)], [(V_cnst, 1)] + [(V_in_dp(i), 1) for i in range(niu - 1)], [(V_I, 1)]); n += 1
    k.add(n, [(V_valid, 1)], [(V_valid, 1), (V_ZO, 1)], [(V_O, 1)]); n += 1
    k.add(n, [], [], [(V_valid, 1), (V_v, -1)]); n += 1
    k.add(n, [(V_tau, 1)] + [(V_in_dp(i), -1) for i in range(2 * niu - 2)], [(num_vars, 1)], [(V_x, 1)]); n += 1
    k.add(n, [(V_x, 1)], [(V_spi, 1), (V_cnst, 1), (V_sv, -1)], [(V_d, 1)]); n += 1
    k.add(n, [(V_v, 1)], [(V_d, 1)], [(V_pi, 1)]); n += 1
    num_cons = 2 * niu + 4
    nnz = 4 * niu + 5
    inst = _instance_new(1, num_cons, [num_cons], 8 * num_vars, [k.A], [k.B], [k.C])
    return num_cons, nnz, inst


class SnarkWorkload:
    """Inputs of SNARK::prove (src/lib.rs:971-1026) for a synthetic straight-line program (SURVEY.md 8d
    configs 1 and 3): `num_blocks` block types executed round-robin, 2^log_proofs executions each, no memory
    operations. Every execution k of block b = k mod num_blocks reads inputs (i0 = b, i1 = x_k, i2 = y_k) and
    writes outputs (o0 = next block, o1 = x_k^(2^m), o2 = y_k) through a chain of m squarings in its private
    variables, so the block, consistency and permutation instances are all satisfied. The instances are
    built by restatements of Instance::gen_block_inst / gen_pairwise_check_inst / gen_perm_root_inst, and the
    block constraints fill 2^log_cons rows after the permutation rows are added."""

    NIU = 4  # default num_inputs_unpadded: (v, _, i0, i1, i2 | o0, o1, o2) -> num_ios = 8

    def __init__(self, num_blocks=2, log_cons=10, log_proofs=9, num_vars=1024, max_ts_width=2, seed=0x5350415254414E31,
                 phy_ops=0, vir_ops=0, init_phy=0, init_vir=0, niu=None, schedule=None, vars_width=None):
        # schedule: the block of every execution (default round robin, num_blocks << log_proofs executions); uneven
        # schedules give unsorted block_num_proofs and blocks that never run. vars_width: per-block witness widths
        # (num_vars_per_block, powers of two <= num_vars; default num_vars): block b's rows keep their first
        # vars_width[b] entries, which must hold the whole chain
        # niu >= 5 is needed for virtual memory: a VIR entry's timestamp (column 5) must fall on an input slot of
        # the perm-root instance, whose output slots must be zero for memory entries (ZO = 0)
        niu = niu or self.NIU
        self.num_blocks = num_blocks
        self.num_vars = num_vars
        self.num_inputs_unpadded = niu
        self.num_ios = 1 << (2 * niu - 1).bit_length()
        io_width = 2 * niu
        assert vir_ops in (0, 2), "virtual memory: each execution stores then loads one cell (2 ops)"
        # memory-op variables (PA, PD)*phy_ops then (VA, VD, VL, VT)*vir_ops follow the io block
        # (Instance::gen_block_inst layout, src/instance.rs:268-283); the squaring chain follows them
        base = io_width + 2 * phy_ops + 4 * vir_ops
        extra = (niu - 2) + (niu - 1) + 4 + 3 + 3 + 2 * phy_ops + 4 * vir_ops
        m = (1 << log_cons) - extra - 3
        assert m >= 1 and base + m + 1 <= num_vars, "num_vars too small for the chain"
        self.chain = m
        self._vars_width = list(vars_width) if vars_width else [num_vars] * num_blocks
        assert len(self._vars_width) == num_blocks and all(
            base + m + 1 <= w <= num_vars and not w & (w - 1) for w in self._vars_width), "vars_width"
        self.chain_base = base
        # user constraints of every block (A, B, C lists of (col, int) per row)
        V_in, V_out = (lambda i: 2 + i), (lambda i: 2 + (niu - 1) + i)
        rows = [([(V_in(1), 1)], [(0, 1)], [(base, 1)])]
        rows += [([(base + j - 1, 1)], [(base + j - 1, 1)], [(base + j, 1)]) for j in range(1, m + 1)]
        rows += [([(base + m, 1)], [(0, 1)], [(V_out(1), 1)]), ([(V_in(2), 1)], [(0, 1)], [(V_out(2), 1)])]
        args = [rows for _ in range(num_blocks)]
        self.args = args  # CompileTimeKnowledge.args (examples/interface.rs:47-71), as (col, int) terms
        self.block_num_phy_ops = [phy_ops] * num_blocks
        self.block_num_vir_ops = [vir_ops] * num_blocks
        self.block_num_vars, self.block_max_num_cons, self.block_nnz, self.block_inst = gen_block_inst(
            num_vars, args, niu, self.block_num_phy_ops, self.block_num_vir_ops)
        self.max_ts_width = max_ts_width
        self.mem_addr_ts_bits_size = 1 << (2 + max_ts_width - 1).bit_length()
        (self.pairwise_num_vars, self.pairwise_max_num_cons, self.pairwise_nnz,
         self.pairwise_inst) = gen_pairwise_check_inst(max_ts_width, self.mem_addr_ts_bits_size)
        self.perm_root_num_cons, self.perm_root_nnz, self.perm_root_inst = gen_perm_root_inst(niu, self.num_ios)
        # ---- execution trace
        if schedule is None:
            schedule = [k % num_blocks for k in range(num_blocks << log_proofs)]
        assert schedule and all(0 <= b < num_blocks for b in schedule)
        E = len(schedule)
        seeds, st = random_fq(2, seed)
        x, y = int(seeds[0]), int(seeds[1])
        self.x0 = x
        # Memory trace, consistent with the verifier's memory checks (src/lib.rs:3275-3330 init lists,
        # :3474-3568 PHY/VIR_MEM_COHERE, :3652-3772 permutation products):
        #  * physical: the input stack init_phy_mems = (1, 0, a, stack[a]) for a < init_phy; execution k, op i
        #    reads cell (k * phy_ops + i) mod init_phy;
        #  * virtual: input memory init_vir_mems = (1, 0, a, mem[a]) for a < init_vir (ls = ts = 0); execution
        #    k stores a fresh value into cell k mod init_vir and loads it back, both at timestamp k // init_vir + 1.
        #  The address-sorted lists hold the init entries and every block access.
        assert not phy_ops or init_phy > 0, "physical ops read the input stack"
        assert not vir_ops or init_vir > 0, "virtual ops need an input memory"
        stack, st = random_fq(max(init_phy, 1), st)
        imem, st = random_fq(max(init_vir, 1), st)
        vir_data, st = random_fq(max(E, 1), st)
        self.input_stack = [int(v) for v in stack[:init_phy]]
        self.input_mem = [int(v) for v in imem[:init_vir]]
        phy_acc = [(a, self.input_stack[a]) for a in range(init_phy)]
        vir_acc = [(a, self.input_mem[a], 0, 0) for a in range(init_vir)]
        per_block = [[] for _ in range(num_blocks)]
        exec_rows = []
        for k in range(E):
            b = schedule[k]
            nb = schedule[k + 1] if k + 1 < E else num_blocks
            chain = [x]
            for _ in range(m):
                chain.append(chain[-1] * chain[-1] % Q)
            xo = chain[-1]
            io = [1, 0, b, x, y] + [0] * (niu - 4) + [nb, xo, y] + [0] * (niu - 4)
            exec_rows.append(io + [0] * (self.num_ios - len(io)))
            memv = []
            for i in range(phy_ops):
                a = (k * phy_ops + i) % init_phy
                memv += [a, self.input_stack[a]]
                phy_acc.append((a, self.input_stack[a]))
            if vir_ops:
                a, d, ts = k % init_vir, int(vir_data[k]), k // init_vir + 1
                memv += [a, d, 0, ts, a, d, 1, ts]
                vir_acc += [(a, d, 0, ts), (a, d, 1, ts)]
            row = io + memv + chain + [0] * (num_vars - base - len(chain))
            per_block[b].append(row)
            x = xo
        self.output = x
        self.block_num_proofs = [len(r) for r in per_block]
        self.block_max_num_proofs = max(self.block_num_proofs)
        self.block_vars = [to_mont_limbs(np.array([row[:w] for row in r], dtype=object).reshape(-1)).reshape(len(r), w, 4)
                           for r, w in zip(per_block, self._vars_width)]
        self.consis_num_proofs = E
        self.exec_inputs = to_mont_limbs(np.array(exec_rows, dtype=object).reshape(-1)).reshape(E, self.num_ios, 4)

        # D = v_next * (v + addr - addr_next) (gen_pairwise_check_inst, src/instance.rs:815-1060)
        def mems(acc, width):
            out = []
            for j, e in enumerate(acc):
                D = 0 if j + 1 == len(acc) else (1 + e[0] - acc[j + 1][0]) % Q
                out.append([1, D] + list(e) + [0] * (width - 2 - len(e)))
            return out
        phy_acc.sort(key=lambda e: e[0])  # stable: the init entry of a cell precedes its reads
        vir_acc.sort(key=lambda e: (e[0], e[3], e[2]))
        self.init_phy_mems = [[1, 0, a, v] for a, v in enumerate(self.input_stack)]
        self.init_vir_mems = [[1, 0, a, v] for a, v in enumerate(self.input_mem)]
        self.addr_phy_mems = mems(phy_acc, 4) if phy_ops else []
        self.addr_vir_mems = mems(vir_acc, 8) if vir_ops else []
        # timestamp aux row (D2, EQ, B_0..): D2 = D1 * ls_next, D1 * (ts_next - ts) = EQ + sum 2^i B_i
        self.addr_ts_bits = []
        for j, e in enumerate(self.addr_vir_mems):
            nxt = self.addr_vir_mems[j + 1] if j + 1 < len(self.addr_vir_mems) else [0] * 8
            diff = (nxt[5] - e[5]) % Q if e[1] else 0
            assert diff < (1 << max_ts_width)
            bits = [(diff >> i) & 1 for i in range(max_ts_width)]
            row = [e[1] * nxt[4] % Q, 0] + bits
            self.addr_ts_bits.append(row + [0] * (self.mem_addr_ts_bits_size - len(row)))
        self.input_block_num = schedule[0]
        self.output_block_num = num_blocks
        self.input_liveness = [False, False, True]
        self.func_input_width = 1
        self.input_offset = 1
        self.output_offset = 2
        self.input = to_mont_limbs([0, 0, self.x0])
        self.output_mont = to_mont_limbs([self.output])[0]
        self.output_exec_num = E - 1

    @property
    def num_vars_per_block(self):
        return list(self._vars_width)

    @property
    def block_vars_sorted(self):
        """block_vars in the prover's instance order (num_proofs descending, stable): the reference pairs
        block_vars_mat[i] with sorted instance i (src/lib.rs:1155-1178)"""
        order = sorted(range(self.num_blocks), key=lambda b: -self.block_num_proofs[b])
        return [self.block_vars[b] for b in order]

    @property
    def total_constraints(self):
        """N = sum_p Q_p * X_p after padding"""
        npow = lambda v: 1 << max(0, (v - 1).bit_length())
        return sum(npow(q) * c for q, c in zip(self.block_num_proofs, self.block_inst[2]))


class CSnarkInstance(ctypes.Structure):
    _fields_ = [("inst", CInstance), ("gens_num_cons", ctypes.c_size_t), ("gens_num_vars", ctypes.c_size_t),
                ("gens_num_instances", ctypes.c_size_t), ("gens_num_nz_entries", ctypes.c_size_t)]


class CSnarkInputs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_size_t) for n in ("input_block_num", "output_block_num")] + [
        ("input_liveness", ctypes.c_void_p), ("input_len", ctypes.c_size_t)] + [
        (n, ctypes.c_size_t) for n in ("func_input_width", "input_offset", "output_offset")] + [
        ("input", ctypes.c_void_p), ("output", ctypes.c_void_p), ("output_exec_num", ctypes.c_size_t),
        ("num_vars", ctypes.c_size_t), ("num_ios", ctypes.c_size_t), ("max_block_num_phy_ops", ctypes.c_size_t),
        ("block_num_phy_ops", ctypes.POINTER(ctypes.c_size_t)), ("max_block_num_vir_ops", ctypes.c_size_t),
        ("block_num_vir_ops", ctypes.POINTER(ctypes.c_size_t)), ("mem_addr_ts_bits_size", ctypes.c_size_t),
        ("num_inputs_unpadded", ctypes.c_size_t), ("block_num_vars", ctypes.POINTER(ctypes.c_size_t)),
        ("block_num_instances_bound", ctypes.c_size_t), ("block_max_num_proofs", ctypes.c_size_t),
        ("block_num_proofs", ctypes.POINTER(ctypes.c_size_t))] + [
        (n, ctypes.c_size_t) for n in ("consis_num_proofs", "total_num_init_phy_mem_accesses",
                                       "total_num_init_vir_mem_accesses", "total_num_phy_mem_accesses",
                                       "total_num_vir_mem_accesses")] + [
        ("block_vars", ctypes.POINTER(ctypes.c_void_p))] + [
        (n, ctypes.c_void_p) for n in ("exec_inputs", "init_phy_mems", "init_vir_mems", "addr_phy_mems",
                                       "addr_vir_mems", "addr_ts_bits")]


class CSnarkPublic(ctypes.Structure):
    """include/spg.h spg_snark_public: SNARK::verify's public arguments (src/lib.rs:2750-2798)"""
    _fields_ = [(n, ctypes.c_size_t) for n in ("input_block_num", "output_block_num")] + [
        ("input_liveness", ctypes.c_void_p), ("input_len", ctypes.c_size_t)] + [
        (n, ctypes.c_size_t) for n in ("func_input_width", "input_offset", "output_offset")] + [
        ("input", ctypes.c_void_p), ("input_stack", ctypes.c_void_p), ("input_stack_len", ctypes.c_size_t),
        ("input_mem", ctypes.c_void_p), ("input_mem_len", ctypes.c_size_t), ("output", ctypes.c_void_p),
        ("output_exec_num", ctypes.c_size_t), ("num_vars", ctypes.c_size_t), ("num_ios", ctypes.c_size_t),
        ("max_block_num_phy_ops", ctypes.c_size_t), ("block_num_phy_ops", ctypes.POINTER(ctypes.c_size_t)),
        ("max_block_num_vir_ops", ctypes.c_size_t), ("block_num_vir_ops", ctypes.POINTER(ctypes.c_size_t)),
        ("mem_addr_ts_bits_size", ctypes.c_size_t), ("num_inputs_unpadded", ctypes.c_size_t),
        ("block_num_vars", ctypes.POINTER(ctypes.c_size_t)), ("block_num_instances_bound", ctypes.c_size_t),
        ("block_max_num_proofs", ctypes.c_size_t), ("block_num_proofs", ctypes.POINTER(ctypes.c_size_t)),
        ("block_num_cons", ctypes.c_size_t)] + [
        (n, ctypes.c_size_t) for n in ("consis_num_proofs", "total_num_init_phy_mem_accesses",
                                       "total_num_init_vir_mem_accesses", "total_num_phy_mem_accesses",
                                       "total_num_vir_mem_accesses", "pairwise_check_num_cons", "perm_root_num_cons")]


def scalar_bytes(vals):
    """canonical scalars (python ints < q) -> (n, 32) little-endian bytes, the reference's [u8; 32]"""
    out = np.zeros((len(vals), 32), dtype=np.uint8)
    for i, v in enumerate(vals):
        out[i] = np.frombuffer(int(v).to_bytes(32, "little"), dtype=np.uint8)
    return out


class SnarkPublic:
    """What the reference verifier of a SnarkWorkload is given (spg_snark_public): the public values as [u8; 32]
    bytes, the input stack / memory (not their init lists) and the sizes, plus the verifier-side commitment
    arguments: num_cons and SNARKGens::new arguments of each instance (as SnarkViews encodes them)."""

    def __init__(self, wl):
        self.keep = []

        def arr(a):
            a = np.ascontiguousarray(a)
            self.keep.append(a)
            return a.ctypes.data

        def sz(v):
            a = _sz(v)
            self.keep.append(a)
            return a

        npow = lambda v: 0 if v == 0 else 1 << (v - 1).bit_length()
        stack, mem = list(getattr(wl, "input_stack", [])), list(getattr(wl, "input_mem", []))
        c = CSnarkPublic()
        c.input_block_num, c.output_block_num = wl.input_block_num, wl.output_block_num
        c.input_liveness = arr(np.array(wl.input_liveness, dtype=np.uint8))
        c.input_len = len(wl.input_liveness)
        c.func_input_width, c.input_offset, c.output_offset = wl.func_input_width, wl.input_offset, wl.output_offset
        c.input = arr(scalar_bytes([0, 0, wl.x0]))
        c.input_stack = arr(scalar_bytes(stack)) if stack else None
        c.input_stack_len = len(stack)
        c.input_mem = arr(scalar_bytes(mem)) if mem else None
        c.input_mem_len = len(mem)
        c.output = arr(scalar_bytes([wl.output]))
        c.output_exec_num = wl.output_exec_num
        c.num_vars, c.num_ios = wl.num_vars, wl.num_ios
        c.max_block_num_phy_ops = max(wl.block_num_phy_ops)
        c.block_num_phy_ops = sz(wl.block_num_phy_ops)
        c.max_block_num_vir_ops = max(wl.block_num_vir_ops)
        c.block_num_vir_ops = sz(wl.block_num_vir_ops)
        c.mem_addr_ts_bits_size = wl.mem_addr_ts_bits_size
        c.num_inputs_unpadded = wl.num_inputs_unpadded
        c.block_num_vars = sz(wl.num_vars_per_block)
        c.block_num_instances_bound = wl.num_blocks
        c.block_max_num_proofs = wl.block_max_num_proofs
        c.block_num_proofs = sz(wl.block_num_proofs)
        c.block_num_cons = wl.block_inst[1]
        c.consis_num_proofs = wl.consis_num_proofs
        c.total_num_init_phy_mem_accesses = npow(len(stack))
        c.total_num_init_vir_mem_accesses = npow(len(mem))
        c.total_num_phy_mem_accesses = len(getattr(wl, "addr_phy_mems", []))
        c.total_num_vir_mem_accesses = len(getattr(wl, "addr_vir_mems", []))
        c.pairwise_check_num_cons = wl.pairwise_inst[1]
        c.perm_root_num_cons = wl.perm_root_inst[1]
        self.c = c
        B = wl.num_blocks
        # (num_cons, SNARKGens::new arguments) per instance, as SnarkViews passes them to the encoder
        self.block_gens = (wl.block_max_num_cons, wl.block_num_vars, B, wl.block_nnz)
        self.pairwise_gens = (wl.pairwise_max_num_cons, 4 * wl.pairwise_num_vars, 3, wl.pairwise_nnz)
        self.perm_root_gens = (wl.perm_root_num_cons, 8 * wl.num_ios, 1, wl.perm_root_nnz)


class SnarkViews:
    """C views (include/spg.h spg_snark_inputs / spg_snark_instance) of a SnarkWorkload; keeps buffers alive."""

    def __init__(self, wl):
        self.keep = []

        def arr(a, dt=np.uint64):
            a = np.ascontiguousarray(a, dtype=dt)
            self.keep.append(a)
            return a.ctypes.data

        def sz(v):
            a = _sz(v)
            self.keep.append(a)
            return a

        def inst(mats_tuple, gens):
            mats, mnc, ncp, nvp = mats_tuple
            n = len(mats)
            ptrs = (ctypes.c_void_p * (3 * n))()
            nnz = []
            for p, m3 in enumerate(mats):
                for k in range(3):
                    ptrs[3 * p + k] = arr(m3[k]) if m3[k].shape[0] else None
                    nnz.append(m3[k].shape[0])
            self.keep.append(ptrs)
            ci = CInstance(n, mnc, nvp, sz(ncp), sz(nnz), ptrs)
            return CSnarkInstance(ci, *gens)

        B = wl.num_blocks
        self.block = inst(wl.block_inst, (wl.block_max_num_cons, wl.block_num_vars, B, wl.block_nnz))
        self.pairwise = inst(wl.pairwise_inst, (wl.pairwise_max_num_cons, 4 * wl.pairwise_num_vars, 3, wl.pairwise_nnz))
        self.perm_root = inst(wl.perm_root_inst, (wl.perm_root_num_cons, 8 * wl.num_ios, 1, wl.perm_root_nnz))
        bv = (ctypes.c_void_p * B)(*[arr(v) if len(v) else None for v in wl.block_vars_sorted])
        self.keep.append(bv)
        c = CSnarkInputs()
        c.input_block_num, c.output_block_num = wl.input_block_num, wl.output_block_num
        c.input_liveness = arr(np.array(wl.input_liveness, dtype=np.uint8), np.uint8)
        c.input_len = len(wl.input_liveness)
        c.func_input_width, c.input_offset, c.output_offset = wl.func_input_width, wl.input_offset, wl.output_offset
        c.input = arr(wl.input)
        c.output = arr(wl.output_mont)
        c.output_exec_num = wl.output_exec_num
        c.num_vars, c.num_ios = wl.num_vars, wl.num_ios
        c.max_block_num_phy_ops = max(wl.block_num_phy_ops)
        c.block_num_phy_ops = sz(wl.block_num_phy_ops)
        c.max_block_num_vir_ops = max(wl.block_num_vir_ops)
        c.block_num_vir_ops = sz(wl.block_num_vir_ops)
        c.mem_addr_ts_bits_size = wl.mem_addr_ts_bits_size
        c.num_inputs_unpadded = wl.num_inputs_unpadded
        c.block_num_vars = sz(wl.num_vars_per_block)
        c.block_num_instances_bound = B
        c.block_max_num_proofs = wl.block_max_num_proofs
        c.block_num_proofs = sz(wl.block_num_proofs)
        c.consis_num_proofs = wl.consis_num_proofs
        c.block_vars = bv
        c.exec_inputs = arr(wl.exec_inputs)

        def mem_list(rows):  # int rows, or an (n, width, 4) uint64 array already in Montgomery limbs
            if len(rows) == 0:
                return 0, None
            if isinstance(rows, np.ndarray) and rows.dtype == np.uint64:
                return rows.shape[0], arr(rows)
            return len(rows), arr(to_mont_limbs(np.array(rows, dtype=object).reshape(-1)))
        c.total_num_init_phy_mem_accesses, c.init_phy_mems = mem_list(getattr(wl, "init_phy_mems", []))
        c.total_num_init_vir_mem_accesses, c.init_vir_mems = mem_list(getattr(wl, "init_vir_mems", []))
        c.total_num_phy_mem_accesses, c.addr_phy_mems = mem_list(getattr(wl, "addr_phy_mems", []))
        c.total_num_vir_mem_accesses, c.addr_vir_mems = mem_list(getattr(wl, "addr_vir_mems", []))
        _, c.addr_ts_bits = mem_list(getattr(wl, "addr_ts_bits", []))
        self.inputs = c
