"""MSM timing probe (development aid): device time of spg_commit_rows_buf / spg_msm at the config-2 shapes
with per-kernel event timing, plus the oracle CPU Pippenger on a bounded sample."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd"), os.path.join(ROOT, "oracle")]
import pyoracle  # noqa: E402
import spg  # noqa: E402

ctx = spg.Context(0)
rng = np.random.default_rng(1)


def rand(n):
    return pyoracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * n, dtype=np.uint8).tobytes())


for (label, n, L, R) in [(b"spg_bench_msm", 1 << 16, 1, 1 << 16), (b"gens_r1cs_sat", 4096, 1024, 1024),
                         (b"gens_r1cs_sat", 4096, 512, 1024), (b"gens_r1cs_sat", 4096, 64, 128)]:
    g = spg.Gens(ctx, n, label)
    Z = rand(L * R)
    zb = spg.Buf(ctx, Z)
    for _ in range(2):
        g.commit_rows_buf(zb, L, R)
    ctx.prof_enable(True)
    ctx.prof_read(reset=True)
    reps = 5
    t0 = time.perf_counter()
    us = []
    for _ in range(reps):
        g.commit_rows_buf(zb, L, R)
        us.append(ctx.last_kernel_us())
    wall = (time.perf_counter() - t0) / reps
    prof = ctx.prof_read(reset=True)
    ctx.prof_enable(False)
    print(f"L={L} R={R}: device {np.median(us):.1f} us/call, wall {wall*1e6:.1f} us; points/s {L*R/(np.median(us)*1e-6):.3e}")
    for k, (c, t, _b) in sorted(prof.items(), key=lambda x: -x[1][1]):
        print(f"    {k:20s} {t/c:10.1f} us x{c}")
    g.free()
    zb.free()

# CPU oracle sample
pts = pyoracle.gens_stream(b"gens_r1cs_sat", 1025)
Z = rand(8 * 1024)
t0 = time.perf_counter()
pyoracle.commit_rows(pts[:1024], pts[1024].tobytes(), Z, 8, 1024)
dt = time.perf_counter() - t0
print(f"oracle CPU 1 core: 8 rows x 1024: {dt:.3f}s -> {8*1024/dt:.3e} points/s")
