"""Latency of the small-MSM path (Bullet-round sizes) for each window width; GPU only."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spartan-parallel_amd"))
import spg  # noqa: E402

ctx = spg.Context(0)
g = spg.Gens(ctx, 4100, b"gens_r1cs_sat")
rng = np.random.default_rng(1)
for n in (130, 1028, 4098):
    s = rng.integers(0, 2**63, (n, 4), dtype=np.uint64)
    s[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    ref = None
    for c in (4, 5, 6, 7, 8, 9):
        os.environ["SPG_SMSM_C"] = str(c)
        out = g.msm(s)
        ref = ref or out
        assert out == ref
        ctx.prof_enable(True)
        ctx.prof_read(reset=True)
        t = time.perf_counter()
        for _ in range(20):
            g.msm(s)
        dt = (time.perf_counter() - t) / 20
        pr = ctx.prof_read(reset=True)
        ctx.prof_enable(False)
        parts = " ".join(f"{k}={v[1] / v[0]:.1f}us" for k, v in sorted(pr.items()))
        print(f"n={n} c={c} wall={dt * 1e6:.1f}us {parts}", flush=True)
