"""Witness-upload probe (config 4's 2^22-constraint witness, 134 MB): spg_r1cs_witness_new timed alone, 5 times, the
previous witness freed first. Run under different SPG_H2D / SPG_H2D_THREADS / SPG_H2D_CHUNK_KB settings (read once per
process); SPG_H2D_TRACE=1 prints every streamed call."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "spartan-parallel_amd")]
import spg  # noqa: E402
import workload  # noqa: E402

ctx = spg.Context(0)
wl = workload.R1CSWorkload([1024] * 8, [512] * 8, num_sections=1, instances=range(8))
v = workload.CViews(wl)
w = None
ts = []
for _ in range(5):
    w = None
    t0 = time.perf_counter()
    w = spg.R1CSWitness(ctx, v.secs, wl.nws)
    ts.append((time.perf_counter() - t0) * 1e3)
print(os.environ.get("SPG_H2D", "1"), os.environ.get("SPG_H2D_THREADS", "8"), os.environ.get("SPG_H2D_CHUNK_KB", "auto"),
      " ".join(f"{t:.2f}" for t in ts))
