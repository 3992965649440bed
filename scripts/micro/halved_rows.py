"""Microbenchmark: 128 Hyrax rows of 256 scalars (the shape of the SPARK derefs commits) through spg_commit_rows_buf,
dense (uniform) against small (< 2^32) scalars; run once per SPG_HALVED_ENC setting (the switch is read once)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd")]
import spg  # noqa: E402

L_ORD = 2**252 + 27742317777372353535851937790883648493


def mont(vals):
    out = np.zeros((len(vals), 4), np.uint64)
    for i, v in enumerate(vals):
        m = (int(v) << 256) % L_ORD
        for k in range(4):
            out[i, k] = (m >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    return out


rng = np.random.default_rng(5)
L, R = 128, 256
n = L * R
dense = mont([int.from_bytes(rng.bytes(32), "little") % L_ORD for _ in range(n)])
small = mont([int(x) for x in rng.integers(0, 2**32, n)])
ctx = spg.Context(0)
g = spg.Gens(ctx, R, b"spg_halved_rows")
for name, z in (("dense", dense), ("small", small)):
    buf = spg.Buf(ctx, z)
    for _ in range(3):
        g.commit_rows_buf(buf, L, R)
    t = time.perf_counter()
    for _ in range(50):
        g.commit_rows_buf(buf, L, R)
    print("SPG_HALVED_ENC=%s %s: %.1f us per 128 x 256 commit" % (os.environ.get("SPG_HALVED_ENC", "1"), name,
                                                                (time.perf_counter() - t) / 50 * 1e6))
