"""The fused fold + evaluation of the R1CSProof sumcheck rounds (sumcheck.hip, k_phase1_eval<true> /
k_phase2_eval<true>) restated in Python over small integers: for ragged instance shapes, every entry the
next round reads equals the separately folded table's (pqx_prepare + pqx_fold_at semantics), and no entry written by
one point is read by another within the launch (in-place folding is race-free; one ABC shared by every instance goes
to its ping-pong buffer). Index algebra only -- the kernels themselves are checked on the GPU by the golden-proof
tests and test_round_forms."""
import random
MOD = 1000003
def run(l_proofs, l_cons, fused, seed):
    rnd = random.Random(seed)
    P = len(l_proofs)
    off = []; tot = 0
    for p in range(P):
        off.append(tot); tot += l_proofs[p] * l_cons[p]
    T = [rnd.randrange(MOD) for _ in range(tot)]
    anw = [1]*P; ani = list(l_cons)
    num_proofs = list(l_proofs); num_inputs = list(l_cons)
    sc_np = list(l_proofs); sc_nc = list(l_cons)
    nx = max(l_cons).bit_length() - 1; nq = max(l_proofs).bit_length() - 1
    rng = random.Random(seed + 1)
    reads = []
    pending = None  # (mode, r, strides)
    for j in range(nx + nq):
        mode = 'X' if j < nx else 'Q'
        for p in range(P):
            if mode == 'X' and sc_nc[p] > 1: sc_nc[p] //= 2
            if mode == 'Q' and sc_np[p] > 1: sc_np[p] //= 2
        rr = []
        for p in range(P):
            for q in range(sc_np[p]):
                for x in range(sc_nc[p]):
                    base = off[p] + q * anw[p] * ani[p] + x
                    if mode == 'X':
                        zero_hi = num_inputs[p] == 1; hi = base + num_inputs[p] // 2
                    else:
                        zero_hi = num_proofs[p] == 1; hi = base + (num_proofs[p] // 2) * anw[p] * ani[p]
                    def get(s):
                        if pending is None: return T[s]
                        fm, r, st = pending
                        lo = T[s]
                        v = (lo + r * (T[s + st[p]] - lo)) % MOD if st[p] else ((1 - r) * lo) % MOD
                        return v
                    lo = get(base)
                    hv = 0 if zero_hi else get(hi)
                    if pending is not None:
                        st_ = pending[2][p]
                        rs = {base, base + st_} | (set() if zero_hi else {hi, hi + st_})
                        ws_ = {base} | (set() if zero_hi else {hi})
                        pid = (p, q, x)
                        for s in rs: readers.setdefault(s, set()).add(pid)
                        for s in ws_: writers.setdefault(s, set()).add(pid)
                    rr.append((lo, hv))
                    if pending is not None:
                        # write back (simulate: collect writes, apply after reading all? each entry read once)
                        writes.append((base, lo))
                        if not zero_hi: writes.append((hi, hv))
        if pending is not None:
            for s, v in writes: T[s] = v
            for s, wp in writers.items():
                assert len(wp) == 1 and readers.get(s, set()) <= wp, ("race", s, wp, readers.get(s))
        readers.clear(); writers.clear()
        writes = []
        reads.append(rr)
        r = rng.randrange(MOD)
        # fold of round j
        if fused:
            st = []
            for p in range(P):
                n = num_inputs[p] if mode == 'X' else num_proofs[p]
                row = 1 if mode == 'X' else anw[p] * ani[p]
                st.append(0 if n == 1 else (n // 2) * row)
            for p in range(P):
                if mode == 'X':
                    if num_inputs[p] != 1: num_inputs[p] //= 2
                else:
                    if num_proofs[p] != 1: num_proofs[p] //= 2
            pending = (mode, r, st)
        else:
            # pqx_prepare + pqx_fold_at
            for p in range(P):
                if mode == 'Q':
                    rows = 1 if num_proofs[p] == 1 else num_proofs[p] // 2; cols = num_inputs[p]
                else:
                    rows = num_proofs[p]; cols = 1 if num_inputs[p] == 1 else num_inputs[p] // 2
                for q in range(rows):
                    for x in range(cols):
                        base = off[p] + q * anw[p] * ani[p] + x
                        if mode == 'X':
                            scale = num_inputs[p] == 1; hi = base + num_inputs[p] // 2
                        else:
                            scale = num_proofs[p] == 1; hi = base + (num_proofs[p] // 2) * anw[p] * ani[p]
                        lo = T[base]
                        T[base] = ((1 - r) * lo) % MOD if scale else (lo + r * (T[hi] - lo)) % MOD
            for p in range(P):
                if mode == 'X':
                    if num_inputs[p] != 1: num_inputs[p] //= 2
                else:
                    if num_proofs[p] != 1: num_proofs[p] //= 2
    return reads
writes = []
readers = {}
writers = {}
import itertools
def test_phase1_fused_fold_matches_separate():
    cases = [([4, 4], [8, 8]), ([8, 2, 1], [16, 4, 2]), ([1], [1]), ([2, 1], [1, 8]), ([16, 4], [2, 32]), ([1, 1, 1, 1], [4, 4, 4, 4])]
    for lp, lc in cases:
        for seed in range(3):
            a = run(lp, lc, False, seed)
            b = run(lp, lc, True, seed)
            assert a == b, (lp, lc, seed)



def npow2(n):
    k = 1
    while k < n: k *= 2
    return k
class Tab:
    def __init__(s, rnd, zlen, anw, ani, num_instances, num_inputs, nws_pad):
        s.zlen = zlen; s.anw = anw; s.ani = ani; s.off = []; t = 0
        for p in range(zlen): s.off.append(t); t += anw[p] * ani[p]
        s.d = [rnd.randrange(MOD) for _ in range(t)]
        s.num_instances = num_instances; s.num_inputs = list(num_inputs); s.nws = nws_pad
def pq_lo(T, p, w, y):
    if p >= T.zlen: return -1
    if w >= T.anw[p] or y >= T.ani[p]: return -1
    return T.off[p] + w * T.ani[p] + y
def pq_hi(T, p, w, y, mode):
    if mode == 'X':
        return (-1, w) if T.num_inputs[p] == 1 else (T.off[p] + w * T.ani[p] + y + T.num_inputs[p] // 2, w)
    wh = w + T.nws // 2
    return (T.off[p] + wh * T.ani[p] + y if wh < T.anw[p] else -1, wh)
def fold_sep(T, mode, r):
    P = min(T.num_instances, T.zlen)
    if mode == 'W': T.nws //= 2
    new_ni = list(T.num_inputs)
    for p in range(P):
        if mode == 'W':
            nw = T.nws; cols = T.num_inputs[p]
        else:
            nw = min(T.nws, T.anw[p])
            if T.num_inputs[p] == 1: cols = 1
            else: cols = T.num_inputs[p] // 2; new_ni[p] = cols
        for w in range(nw):
            for x in range(cols):
                base = T.off[p] + w * T.ani[p] + x
                lo = T.d[base]
                if mode == 'X':
                    if T.num_inputs[p] == 1: T.d[base] = ((1 - r) * lo) % MOD; continue
                    h = T.d[base + T.num_inputs[p] // 2]
                else:
                    wh = w + T.nws
                    h = 0 if wh >= T.anw[p] else T.d[T.off[p] + wh * T.ani[p] + x]
                T.d[base] = (lo + r * (h - lo)) % MOD
    T.num_inputs = new_ni
def plan(T, mode):
    P = min(T.num_instances, T.zlen)
    st = [0] * T.zlen; fw = 0
    if mode == 'W':
        fw = T.nws // 2
        for p in range(P): st[p] = fw * T.ani[p]
        T.nws = fw
        return st, fw
    for p in range(P):
        n = T.num_inputs[p]
        st[p] = 0 if n == 1 else n // 2
    for p in range(P):
        if T.num_inputs[p] != 1: T.num_inputs[p] //= 2
    return st, fw
def run2(l_inputs, nws, single, fused, seed):
    rnd = random.Random(seed)
    P = len(l_inputs)
    pad = npow2(nws)
    Z = Tab(rnd, P, [nws] * P, list(l_inputs), npow2(P), l_inputs, pad)
    if single:
        A = Tab(rnd, 1, [nws], [l_inputs[0]], 1, l_inputs, pad)
    else:
        A = Tab(rnd, P, [nws] * P, list(l_inputs), npow2(P), l_inputs, pad)
    ny = max(l_inputs).bit_length() - 1; nw = pad.bit_length() - 1
    inputs_len, ws_len = 1 << ny, 1 << nw
    sc_ni = list(l_inputs)
    rng = random.Random(seed + 7)
    reads = []; pending = None
    for j in range(ny + nw):
        mode = 'X' if j < ny else 'W'
        if inputs_len > 1: inputs_len //= 2
        elif ws_len > 1: ws_len //= 2
        if mode == 'X':
            sc_ni = [n // 2 if n > 1 else n for n in sc_ni]
        W = min(ws_len, nws)
        rr = []; writesA = []; writesZ = []; readers = {}; writers = {}
        Bold = list(A.d)
        for p in range(P):
            for w in range(W):
                for y in range(sc_ni[p]):
                    pi = 0 if single else p
                    vals = []
                    for tname, T, pp in (('A', A, pi), ('Z', Z, p)):
                        sl = pq_lo(T, pp, w, y); sh, wc = pq_hi(T, pp, w, y, mode)
                        out = []
                        for s, wcc in ((sl, w), (sh, wc)):
                            if s < 0: out.append(0); continue
                            if pending is None: out.append(T.d[s]); continue
                            r, fm, fw, sA, sZ = pending
                            st = (sA if tname == 'A' else sZ)[pp]
                            pair = st and (fm != 'W' or wcc + fw < T.anw[pp])
                            lo = T.d[s]
                            v = (lo + r * (T.d[s + st] - lo)) % MOD if pair else ((1 - r) * lo) % MOD
                            out.append(v)
                            key = (tname, s)
                            readers.setdefault(key, set()).add((p, w, y))
                            if pair: readers.setdefault((tname, s + st), set()).add((p, w, y))
                            if tname == 'Z' or not single or p == 0:
                                writers.setdefault(key, set()).add((p, w, y))
                                (writesA if tname == 'A' else writesZ).append((s, v))
                        vals.extend(out)
                    rr.append(tuple(vals))
        if pending is not None:
            for key, wp in writers.items():
                assert len(wp) == 1, ("multiple writers", key, wp)
                if not (single and key[0] == 'A'):
                    assert readers.get(key, set()) <= wp, ("race", key, wp, readers.get(key))
            if single:  # ping-pong: new buffer = old buffer overwritten by writes (entries not written are stale)
                newA = [None] * len(A.d)
                for s, v in writesA: newA[s] = v
                A.d = newA
            else:
                for s, v in writesA: A.d[s] = v
            for s, v in writesZ: Z.d[s] = v
        reads.append(rr)
        r = rng.randrange(MOD)
        if fused and j + 1 < ny + nw:
            sA, fw = plan(A, mode); sZ, _ = plan(Z, mode)
            pending = (r, mode, fw, sA, sZ)
        else:
            fold_sep(A, mode, r); fold_sep(Z, mode, r)
            pending = None
    return reads
def test_phase2_fused_fold_matches_separate():
    cases = [([8, 8], 5), ([8, 4, 2], 3), ([4], 1), ([16, 16, 16, 16], 8), ([2, 8], 6), ([32], 5), ([4, 4], 2)]
    for li, nws in cases:
        for single in (False, True):
            if single and li[0] != max(li):
                continue
            for seed in range(2):
                a = run2(li, nws, single, False, seed)
                b = run2(li, nws, single, True, seed)
                assert a == b, (li, nws, single, seed)

